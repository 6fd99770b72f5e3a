#!/usr/bin/env python3
"""Phase timing of the decode LayerNorm kernel (run with VSIM_LN_DBG=1; GPU diagnostic):
s_memtime stamps of the last LayerNorm launch of an eager GPT-J decode step."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual), n_ctx=256)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
m.set_graph(False)
lg = m.eval(0, [50278, 12092, 2])
names = ["loads+sum terms", "reduce mean", "var pass+reduce", "scale", "normalize", "quantize"]
acc = np.zeros(6)
n = 10
for i in range(n):
    lg = m.eval(3 + i, [int(np.argmax(lg))])
    buf = (ctypes.c_ulonglong * 8)()
    hip.lib().vsim_debug_ln_prof(buf)
    acc += np.diff(np.array(buf[:7], dtype=np.float64))
print("LayerNorm phases (s_memtime ticks, 2.4 GHz, mean over the final norm of %d steps):" % n)
for nm, v in zip(names, acc / n):
    print(f"  {nm:18s} {v:8.0f}  ({v / 2.4e3:.2f} us)")
print(f"  total              {acc.sum() / n:8.0f}  ({acc.sum() / n / 2.4e3:.2f} us)")
