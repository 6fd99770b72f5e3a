"""In-process A/B of the long-prompt GEMM tile order (vsim_gemm_set_tile_order) on the
codegen-16B N = 2048 fast prompt (bench.py --prefill's model and tokens), alternating orders
over rounds so drift and clock changes hit every arm alike.
usage: python tools/prefill_order_ab.py [ORDERS=4,0] [ROUNDS=3] [REPS=3]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

orders = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4,0").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
arch_s, hp = mg.CONFIGS["codegen-16B"]
N = 2048
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual),
                     n_ctx=N + 8)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_FAST)
m.reserve(N)
ids = [(7919 * i + 11) % hp.n_vocab for i in range(N)]
m.eval(0, ids)
torch.cuda.synchronize()
res = {o: [] for o in orders}
for r in range(rounds):
    for o in orders:
        hip.lib().vsim_gemm_set_tile_order(o)
        m.eval(0, ids)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            m.eval(0, ids)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        res[o].append(ms)
        print(f"round {r} tile order {o}: {ms:.2f} ms per prompt", flush=True)
for o in orders:
    print(f"tile order {o}: min {min(res[o]):.2f} median {sorted(res[o])[len(res[o]) // 2]:.2f} ms", flush=True)
