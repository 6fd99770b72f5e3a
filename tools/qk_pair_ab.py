"""A/B of the paired Q/K prompt GEMM (vsim_gemm_set_qk_pair) on long GPT-J-architecture prompts:
the same model and prompt, alternating the switch between repetitions, ms per prompt eval.
Usage: AB_MODES=0,1,2 python tools/qk_pair_ab.py [config ...]   (default codegen-16B gpt-j-6B; N = 2048;
modes: 0 separate launches, 1 pair with the hybrid split, 2 pair of whole tiles)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

N = int(os.environ.get("AB_N", "2048"))
REPS = int(os.environ.get("AB_REPS", "4"))
L = hip.lib()
for cfg in sys.argv[1:] or ["codegen-16B", "gpt-j-6B"]:
    arch_s, hp = mg.CONFIGS[cfg]
    model = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                                 n_layer=hp.n_layer, n_rot=hp.n_rot,
                                                 use_parallel_residual=hp.use_parallel_residual),
                             n_ctx=N + 8, device=0)
    model.randomize(seed=1234, std=0.02)
    model.set_mode(hip.MODE_FAST)
    ids = [(7919 * i + 11) % hp.n_vocab for i in range(N)]
    modes = [int(v) for v in os.environ.get("AB_MODES", "0,1").split(",")]
    times = {m: [] for m in modes}
    logits = {}
    for r in range(len(modes) * (REPS + 1)):
        on = modes[r % len(modes)]
        if os.environ.get("AB_KNOB") == "streamk":  # (the same A/B over vsim_gemm_set_streamk modes)
            L.vsim_gemm_set_streamk(on)
        else:
            L.vsim_gemm_set_qk_pair(on)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lg = model.eval(0, ids)
        torch.cuda.synchronize()
        if r >= len(modes):
            times[on].append((time.perf_counter() - t0) * 1e3)
        logits.setdefault(on, lg)
    L.vsim_gemm_set_qk_pair(1)
    L.vsim_gemm_set_streamk(1)
    knob = os.environ.get("AB_KNOB", "qk_pair")
    out = {"config": cfg, "N": N, "knob": knob,
           "modes": "stream-K off / on" if knob == "streamk" else
                    "0 separate launches, 1 pair + hybrid split, 2 pair, whole tiles"}
    for m in modes:
        out[f"mode{m}_ms"] = [round(t, 2) for t in times[m]]
        out[f"mode{m}_median"] = round(sorted(times[m])[len(times[m]) // 2], 2)
        out[f"mode{m}_logits_max_abs_diff_vs_mode{modes[0]}"] = float(abs(logits[m] - logits[modes[0]]).max())
    print(json.dumps(out), flush=True)
    model.close()
