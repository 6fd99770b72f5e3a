#!/usr/bin/env python3
"""LayerNorm timing and fallback counts on the GPT-J decode residual (GPU diagnostic)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

L = hip.lib()
E = 4096
for name, x in [("randn", torch.randn(E, device="cuda")), ("randn*30", torch.randn(E, device="cuda") * 30),
                ("uniform", torch.rand(E, device="cuda"))]:
    y = torch.empty_like(x)
    w = torch.ones(E, device="cuda")
    b = torch.zeros(E, device="cuda")
    f0 = hip.norm_fallbacks()
    for _ in range(3):
        hip.check(L.vsim_op_norm(x.data_ptr(), y.data_ptr(), E, 1, w.data_ptr(), b.data_ptr(), None))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        hip.check(L.vsim_op_norm(x.data_ptr(), y.data_ptr(), E, 1, w.data_ptr(), b.data_ptr(), None))
    e1.record()
    torch.cuda.synchronize()
    f1 = hip.norm_fallbacks()
    print(f"{name:10s} norm {e0.elapsed_time(e1) * 1e3 / 50:8.2f} us  fallbacks(mean,var) {f1[0]-f0[0]},{f1[1]-f0[1]} of 53")
arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual), n_ctx=256)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
f0 = hip.norm_fallbacks()
lg = m.eval(0, [50278, 12092, 2, 0, 50281])
for i in range(8):
    lg = m.eval(5 + i, [int(np.argmax(lg))])
f1 = hip.norm_fallbacks()
print(f"gpt-j decode: fallbacks (mean, var) {f1[0]-f0[0]}, {f1[1]-f0[1]} over {8 * 29 + 29} norms (prompt incl.)")
