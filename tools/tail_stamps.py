"""Reads the per-chunk s_memtime stamps of k_layer_tail's fc_out tiles from the diagnostic
variant (tools/variants/mk_tail_stamps.py; VSIM_LIB=vsim_amd/_build/var/stamps.so) after a GPT-J-6B
exact decode, and prints where a chunk step's cycles go: the consumer's adds and barrier wait,
the producers' compute, DMA wait and barrier wait (p = 0 on SIMD1, p = 3 beside the consumer).
The stamps are the last tail launched (layer 27 of the last token)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual), n_ctx=512)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
m.eval(0, [1, 2, 3, 4, 5])
toks = m.generate(5, 6, int(os.environ.get("STAMP_STEPS", "40")))
ST_K, ST_N = 72, 12
buf = np.zeros((128, ST_K, ST_N), np.uint64)
L = hip.lib()
L.vsim_debug_tail_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.vsim_debug_tail_stamps(buf.ctypes.data, buf.nbytes) == 0
s = buf.astype(np.float64)
NCH = int(os.environ.get("STAMP_CHUNKS", "64"))
CP = int(os.environ.get("STAMP_CP", "128"))
ks = np.arange(4, NCH)  # steady steps


def med(a):
    return float(np.median(a))


cons_add = s[:, ks, 1] - s[:, ks, 0]
cons_bar = s[:, ks, 2] - s[:, ks, 1]
stepc = s[:, ks + 1, 0] - s[:, ks, 0]
out = [f"tiles 128, steps {ks[0]}..{ks[-1]} (chunk = {CP} pair terms per row), medians over tiles x steps, cycles:",
       f"  consumer step {med(stepc):.0f}: adds {med(cons_add):.0f} ({med(cons_add) / CP:.2f} per add), "
       f"barrier wait {med(cons_bar):.0f}"]
for name, b in (("producer p=0 (SIMD1)", 3), ("producer p=2 (wave 3)", 7)):
    comp = s[:, ks, b + 1] - s[:, ks, b]
    vmw = s[:, ks, b + 2] - s[:, ks, b + 1]
    bar = s[:, ks, b + 3] - s[:, ks, b + 2]
    out.append(f"  {name}: compute+stores {med(comp):.0f}, DMA wait {med(vmw):.0f} (p90 {np.percentile(vmw, 90):.0f}), "
               f"barrier wait {med(bar):.0f}")
rt = s[:, :, 11]
clk = (s[:, NCH, 0] - s[:, 2, 0]) / ((rt[:, NCH] - rt[:, 2]) / 1e8) / 1e9
span = (rt[:, NCH + 1] - rt[:, 0]) / 1e2  # us
t0 = (rt[:, 0] - rt[:, 0].min()) / 1e2
out.append(f"  shader clock {med(clk):.2f} GHz; tile span step 0..{NCH + 1} median {med(span):.1f} us "
           f"(min {span.min():.1f}, max {span.max():.1f}); tile start skew max {t0.max():.1f} us")
per_k = np.median(s[:, 1:NCH + 2, 0] - s[:, 0:NCH + 1, 0], axis=0)
out.append("  median step cycles by step: " + " ".join(f"{v:.0f}" for v in per_k))
print("\n".join(out))
