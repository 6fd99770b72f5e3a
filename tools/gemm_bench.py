"""Long-prompt GEMM timing (k_gemm_f16_256 via vsim_op_gemm_f16) at the codegen-16B shapes
(N = 2048): TFLOP/s per shape, HIP events over repeated launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402

N = 2048
shapes = [(6144, 6144), (24576, 6144), (6144, 24576)]
for M, K in shapes:
    w = torch.empty(M * K, dtype=torch.float16, device="cuda").normal_(0, 0.05)
    x = torch.empty(N * K, dtype=torch.float16, device="cuda").normal_(0, 0.5)
    y = torch.empty(N * M, dtype=torch.float32, device="cuda")
    f = lambda: hip.check(hip.lib().vsim_op_gemm_f16(w.data_ptr(), M, K, x.data_ptr(), N, None, y.data_ptr(), None), "g")
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"M={M} K={K} N={N}: {ms * 1e3:.1f} us  {2.0 * M * K * N / ms / 1e9:.0f} TFLOP/s", flush=True)
