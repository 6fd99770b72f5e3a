"""Where k_gemv_solo's waves run (r05 diagnostic): GPT-J-6B exact decode on the VSIM_NB_STAMPS build
(VSIM_LIB=vsim_amd/_build/var/nbstamps.so); each wave of the last fc_in + QKV batch (448 groups of
eight waves) stamps HW_ID | XCC_ID << 32 into row 512 + group.  The kernel assumes waves 0 and 4
(the consumer and the filler that only joins the barriers) share one SIMD and that the two groups
of a CU put their consumers on the same SIMD; this counts how often that holds."""
import collections
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual),
                     n_ctx=512, device=0)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
m.set_graph(True)
tok = int(np.argmax(m.eval(0, [50278, 12092, 2, 0, 50281])))
m.generate(5, tok, 8)
buf = np.zeros((2048, 32), np.uint64)
f = hip.lib().vsim_debug_nb_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert f(buf.ctypes.data, buf.nbytes) == 0
m.close()

G, W = 448, 8
hw = buf[512:512 + G, :W].astype(np.int64)
assert (hw != 0).all(), "missing stamps"
simd = (hw >> 4) & 3
cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | ((hw >> 32) << 8)  # CU, SH, SE, XCC
print(f"k_gemv_solo: {G} groups of {W} waves")
print(f"  waves 0 and 4 on one SIMD: {(simd[:, 0] == simd[:, 4]).sum()} of {G}")
print(f"  consumer (wave 0) SIMD counts: {collections.Counter(simd[:, 0].tolist())}")
pat = collections.Counter(tuple(r) for r in simd.tolist())
print("  SIMD of waves 0..7, most common patterns:")
for p_, c_ in pat.most_common(6):
    print(f"    {p_}: {c_}")
bycu = collections.defaultdict(list)
for g in range(G):
    bycu[int(cu[g, 0])].append(g)
two = [v for v in bycu.values() if len(v) == 2]
same = sum(1 for a, b in two if simd[a, 0] == simd[b, 0])
print(f"  CUs with two groups: {len(two)}, with one: {sum(1 for v in bycu.values() if len(v) == 1)}, "
      f"more: {sum(1 for v in bycu.values() if len(v) > 2)}")
print(f"  two-group CUs whose consumers share one SIMD: {same} of {len(two)}")
# producers on a consumer's SIMD (from either group of the CU)
shared = 0
for a, b in two:
    for c, o in ((a, b), (b, a)):
        s0 = simd[c, 0]
        shared += int(sum(1 for w in range(W) if w % 4 and simd[c, w] == s0) + sum(1 for w in range(W) if w % 4 and simd[o, w] == s0))
print(f"  producer waves on a consumer's SIMD, summed over the two-group CUs' consumers: {shared}")
# the consumer SIMDs of a two-group CU: (lower group's, higher group's)
pairs = collections.Counter((int(simd[a, 0]), int(simd[b, 0])) for a, b in (sorted(v) for v in two))
print(f"  consumer SIMD pairs (lower, higher group index): {dict(pairs)}")
print(f"  group index gap of the two groups of a CU: {collections.Counter(b - a for a, b in (sorted(v) for v in two)).most_common(5)}")
# the consumers' clocks over their loops (s_memtime cycles / s_memrealtime at 100 MHz)
cl = buf[512:512 + G, 8:12].astype(np.int64)
dm, dr = cl[:, 1] - cl[:, 0], cl[:, 3] - cl[:, 2]
ghz = dm / (dr / 100.0) / 1e3
print(f"  consumer loop: median {np.median(dr) / 100:.2f} us, shader clock median {np.median(ghz):.3f} GHz "
      f"(p10 {np.percentile(ghz, 10):.3f}, p90 {np.percentile(ghz, 90):.3f})")
t0 = cl[:, 2].min()
st, en = (cl[:, 2] - t0) / 100.0, (cl[:, 3] - t0) / 100.0
for name, sel in (("groups 0..255", slice(0, 256)), ("groups 256..447", slice(256, G))):
    print(f"  {name}: consumer loop start med {np.median(st[sel]):.2f} max {st[sel].max():.2f} us, "
          f"end med {np.median(en[sel]):.2f} max {en[sel].max():.2f} us")
