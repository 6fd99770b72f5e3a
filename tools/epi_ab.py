"""A/B of two library builds on the fast prompt path: the same random-init models, the same
prompts, logits compared bit for bit.  Used to show that moving work into the long-prompt
GEMM's epilogue (RoPE + KV write, residual join) leaves every logit bit unchanged.

  python3 tools/epi_ab.py BASE.so     (the default build is the other arm)
"""
import dataclasses
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [  # (name, config, overrides)
    ("small-gptj", "small-gptj", {}),
    ("small-neox", "small-neox", {}),
    ("small-neox-serial", "small-neox", {"use_parallel_residual": 0}),
    ("codegen-width-1L", "codegen-16B", {"n_layer": 1, "n_vocab": 4096}),
]


def child(out):
    from vsim_amd import hip
    from vsim_amd import modelgen as mg
    res = {}
    for name, cfg, ov in CASES:
        arch_s, hp = mg.CONFIGS[cfg]
        hp = dataclasses.replace(hp, **ov)
        arch = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX}[arch_s]
        m = hip.Model.create(arch, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                        n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual),
                             n_ctx=1024, device=0)
        m.randomize(seed=77, std=0.05)
        m.set_mode(hip.MODE_FAST)
        rng = np.random.default_rng(3)
        a = [int(v) for v in rng.integers(0, hp.n_vocab, 290)]
        b = [int(v) for v in rng.integers(0, hp.n_vocab, 300)]
        l1 = m.eval(0, a)
        l2 = m.eval(290, b)  # a second long prompt on top of the cache (n_past not a multiple of 8)
        l3 = m.eval(590, [int(np.argmax(l2))])
        res[name] = np.concatenate([l1, l2, l3]).astype(np.float32)
        m.close()
    np.savez(out, **res)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    base = sys.argv[1]
    outs = {}
    for arm, lib in (("base", base), ("new", None)):
        env = dict(os.environ)
        if lib:
            env["VSIM_LIB"] = lib
        else:
            env.pop("VSIM_LIB", None)
        out = f"/tmp/epi_ab_{arm}.npz"
        subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True, timeout=300)
        outs[arm] = np.load(out)
    rep = {}
    for name, _, _ in CASES:
        x, y = outs["base"][name], outs["new"][name]
        rep[name] = {"bit_identical": bool(np.array_equal(x.view(np.uint32), y.view(np.uint32))),
                     "max_abs_diff": float(np.max(np.abs(x - y)))}
    print(json.dumps(rep))
    sys.exit(0 if all(r["bit_identical"] for r in rep.values()) else 1)


if __name__ == "__main__":
    main()
