"""Where the in-tail LayerNorm (r06, TailLn) spends the end of the layer tail: GPT-J-6B exact
decode on the VSIM_NB_STAMPS build (tools/build_variant.sh nbstamps Makefile
's/-fno-slp-vectorize$/& -DVSIM_NB_STAMPS/'), then the s_memrealtime stamps (100 MHz) of the
last tail of the run: per fc_out tile (the LN owner) the chain's end, the out-projection's
granules seen, the partial sums published, every tile's partials seen, the block quantized;
per out-projection tile the time its granules were stored.  Usage: VSIM_LIB=...nbstamps.so
python tools/lnt_stamps.py [STEPS [CONFIG]]  (CONFIG: gpt-j-6B, pythia-12b, gpt-neoxt-20b; 4 layers of
the wider two, so the run stays short)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cfg = sys.argv[2] if len(sys.argv) > 2 else "gpt-j-6B"
arch_s, hp = mg.CONFIGS[cfg]
ARCH = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX}
m = hip.Model.create(ARCH[arch_s], dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                        n_layer=hp.n_layer if cfg == "gpt-j-6B" else 4,
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

d = hp.n_embd // hp.n_head
nsplit = 2 if d % 2 == 0 and (d // 2) % 32 == 0 else 1  # (model.cpp ATT_SPLIT)
nf, na, no = hp.n_embd // 32, hp.n_head * nsplit, hp.n_embd // 32
tl = buf[1536:1536 + nf + na + no, :16].astype(np.int64)
spn = buf[1536:1536 + nf, 13:15].astype(np.int64)  # the owners' re-polls: granule, partials
t0 = tl[:, 0].min()
us = lambda v: (v - t0) / 100.0  # noqa: E731
fo = tl[:nf]


def q(name, v):
    v = us(v)
    print(f"  {name:34s} min {v.min():6.2f}  med {np.median(v):6.2f}  max {v.max():6.2f} us")


print(f"last tail of a {steps}-step {cfg} decode (position {5 + steps}), us from the first workgroup's start")
wk = tl[nf + na:]
print(f"out-projection tiles ({len(wk)}):")
q("start", wk[:, 0])
q("granules stored", wk[:, 8])
hd = tl[nf:nf + na]
print(f"heads ({na} workgroups):")
q("flag stored (end)", hd[:, 2])
print("fc_out tiles (LN owners):")
q("start", fo[:, 0])
q("chain end (LN entry)", fo[:, 8])
q("out-proj granules seen", fo[:, 9])
q("partials published", fo[:, 10])
q("all partials seen", fo[:, 11])
q("block quantized", fo[:, 12])
q("end", fo[:, 2])
last = int(np.argmax(fo[:, 8]))
print(f"the last chain (tile {last}): entry {us(fo[last, 8]):.2f}, granules {us(fo[last, 9]):.2f}, "
      f"published {us(fo[last, 10]):.2f}, seen by all {us(fo[:, 11]).max():.2f} (first to see {us(fo[:, 11]).min():.2f}), "
      f"last block {us(fo[:, 12]).max():.2f}")
ends = us(fo[:, 8])
print("fc_out chain end by XCD (tile % 8), median / max:",
      " ".join(f"{x}:{np.median(ends[x::8]):.2f}/{ends[x::8].max():.2f}" for x in range(8)))
order = np.argsort(-ends)
print("slowest fc_out tiles (index: chain end):", " ".join(f"{i}:{ends[i]:.2f}" for i in order[:10]))
print("owners' re-polls (count: tiles) -- granule:", dict(zip(*np.unique(spn[:, 0], return_counts=True))),
      " partials: median", int(np.median(spn[:, 1])), "max", int(spn[:, 1].max()))
