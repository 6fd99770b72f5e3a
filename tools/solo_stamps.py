"""Where the k_gemv_solo batch (fc_in, Q, K, V: 448 groups of 64 rows) spends its chunk steps (r06
diagnostic): GPT-J-6B exact decode on the VSIM_NB_STAMPS build, then per producer wave the shader
cycles summed over its steps -- waiting at the step's lgkmcnt(0) (the scalar-loaded activation
factors, and the previous step's LDS stores), computing the pair terms (and issuing their LDS
stores), waiting at the chunk barrier (s_memtime, summed over the steps) -- and the consumer's
cycles at its barriers, per chunk step;
split by whether the group's CU holds one group or two (HW_ID stamps of the same build).
Usage: VSIM_LIB=vsim_amd/_build/var/nbstamps.so python tools/solo_stamps.py [STEPS]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual),
                     n_ctx=512, device=0)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
m.set_graph(True)
tok = int(np.argmax(m.eval(0, [50278, 12092, 2, 0, 50281])))
m.generate(5, tok, steps)
buf = np.zeros((2048, 32), np.uint64)
f = hip.lib().vsim_debug_nb_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert f(buf.ctypes.data, buf.nbytes) == 0
m.close()

G = 448
rows = buf[512:512 + G]
hw = rows[:, 0].astype(np.int64)
cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | ((hw >> 32) << 8)  # CU, SH, SE, XCC (solo_placement.py)
uniq, cnt = np.unique(cu, return_counts=True)
per_cu = dict(zip(uniq.tolist(), cnt.tolist()))
two = np.array([per_cu[c] >= 2 for c in cu.tolist()])
nit = np.maximum(rows[:, 31].astype(float), 1)
prod = rows[:, 12:30].astype(float).reshape(G, 6, 3) / nit[:, None, None]
cons_bar = rows[:, 30].astype(float) / nit
cdur = (rows[:, 9] - rows[:, 8]).astype(float) / nit  # consumer s_memtime per step (start..end)
print(f"last k_gemv_solo batch of a {steps}-step GPT-J-6B decode: {G} groups, {int(np.median(nit))} steps each; "
      f"{two.sum()} groups on CUs holding two, {(~two).sum()} alone")
for name, sel in (("two per CU", two), ("alone", ~two)):
    if sel.sum() == 0:
        continue
    p = prod[sel]
    print(f"{name:10s} per step (shader cycles, medians): producer factor/LDS wait {np.median(p[:, :, 0]):6.0f}"
          f"  compute {np.median(p[:, :, 1]):6.0f}  barrier {np.median(p[:, :, 2]):6.0f}"
          f"  | consumer barrier {np.median(cons_bar[sel]):6.0f}  consumer step {np.median(cdur[sel]):6.0f}")
    print(f"{'':10s} compute by producer index (median): " + " ".join(f"{np.median(p[:, i, 1]):5.0f}" for i in range(6)))
