#!/usr/bin/env python3
"""Phase timing of the exact decode attention (run with VSIM_TAIL=0 VSIM_ATT_DBG=1; GPU
diagnostic): s_memtime stamps of head 0 in the last layer's k_attn_decode, at several
context lengths of an eager GPT-J decode step."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=2,
                                         n_rot=hp.n_rot, use_parallel_residual=1), n_ctx=512)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
m.set_graph(False)
names = ["q/k load, rope, kv write", "KQ (certified)", "max/exp/sum", "KQV + quantize"]
rng = np.random.default_rng(0)
lg = m.eval(0, [int(t) for t in rng.integers(0, hp.n_vocab, 500)])
for P in (16, 64, 128, 256, 384, 496):
    acc = np.zeros(4)
    for r in range(3):
        m.eval(P, [7])
        buf = (ctypes.c_ulonglong * 8)()
        hip.lib().vsim_debug_attn_prof(buf)
        acc += np.diff(np.array(buf[:5], dtype=np.float64))
    acc /= 3
    print(f"P={P:4d} " + "  ".join(f"{nm}: {v / 2.4e3:6.2f} us" for nm, v in zip(names, acc)) +
          f"  total {acc.sum() / 2.4e3:6.2f} us", flush=True)
