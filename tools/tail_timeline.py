"""Reads the per-workgroup s_memrealtime timeline of k_layer_tail from the diagnostic variant
(tools/variants/mk_tail_timeline.py; VSIM_LIB=vsim_amd/_build/var/timeline.so) after a GPT-J-6B
exact decode to positions P (argv, default 40 250) and prints, in us from the tail's first fc_out
start: fc_out tiles' ends, the heads' phases (KQ, softmax, KQV, quantize+count), the
out-projection tiles' wait end and end."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

arch_s, hp = mg.CONFIGS["gpt-j-6B"]
L = hip.lib()
L.vsim_debug_tail_timeline.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
nf, H, no = 128, hp.n_head, 128
for P in [int(v) for v in sys.argv[1:]] or [40, 250]:
    m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                             n_layer=hp.n_layer, n_rot=hp.n_rot,
                                             use_parallel_residual=hp.use_parallel_residual), n_ctx=512)
    m.randomize(seed=1234, std=0.02)
    m.eval(0, [1, 2, 3, 4, 5])
    m.generate(5, 6, P - 5)
    tl = np.zeros((512, 8), np.uint64)
    assert L.vsim_debug_tail_timeline(tl.ctypes.data, tl.nbytes) == 0
    t = tl.astype(np.float64) / 100.0  # us
    t0 = t[:nf, 0].min()
    f, hd, op = t[:nf] - t0, t[nf:nf + H] - t0, t[nf + H:nf + H + no] - t0
    q = lambda a: f"{np.median(a):6.2f} med / {a.min():6.2f}..{a.max():6.2f}"
    print(f"P = {P} (n_past of the last step), us from the first fc_out start:")
    print(f"  fc_out start {q(f[:, 0])}   end {q(f[:, 1])}")
    print(f"  heads  start {q(hd[:, 0])}  KQ done {q(hd[:, 1])}  softmax {q(hd[:, 2])}  KQV {q(hd[:, 3])}  counted {q(hd[:, 4])}")
    print(f"  o-proj start {q(op[:, 0])}  wait over {q(op[:, 1])}  end {q(op[:, 2])}")
    print(f"  tail end (max of all) {max(f[:, 1].max(), op[:, 2].max()):.2f}", flush=True)
    m.close()
