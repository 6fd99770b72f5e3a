"""Long-prompt GEMM timing at the codegen-16B shapes (N = 2048): TFLOP/s per shape, HIP events
over repeated launches, for the model's kernel (vsim_op_gemm_q4_256: the W4T32 weight
dequantized in LDS) and the fp16-image kernel it replaced (vsim_op_gemm_f16 on k_w4_expand_f16's
image), on the same weights."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

N = int(os.environ.get("GEMM_N", "2048"))
shapes = [(6144, 6144), (24576, 6144), (6144, 24576)]
if os.environ.get("GEMM_SHAPES"):  # "M1xK1,M2xK2,..."
    shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["GEMM_SHAPES"].split(",")]
IMG = os.environ.get("GEMM_IMG", "1") != "0"
# GEMM_ORDERS="4,0": time the model kernel under each tile order (vsim_gemm_set_tile_order), alternating
ORDERS = [int(v) for v in os.environ["GEMM_ORDERS"].split(",")] if os.environ.get("GEMM_ORDERS") else None
# GEMM_COPIES=C: the model kernel also timed rotating over C copies of the weights (C x the bytes
# past the 256 MB MALL: every launch reads weights no recent launch touched, as in a prompt)
COPIES = int(os.environ.get("GEMM_COPIES", "0"))
L = hip.lib()


def timeit(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


rng = np.random.default_rng(0)
for M, K in shapes:
    aos = torch.from_numpy(mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.02))).cuda()
    w = torch.empty(hip.q4_bytes(M, K), dtype=torch.uint8, device="cuda")
    hip.check(L.vsim_op_q4_repack(aos.data_ptr(), w.data_ptr(), M, K, None), "repack")
    img = torch.empty(M * K if IMG else 8, dtype=torch.float16, device="cuda")
    if IMG:
        hip.check(L.vsim_op_q4_expand_f16(w.data_ptr(), M, K, img.data_ptr(), None), "expand")
    x = torch.empty(N * K, dtype=torch.float16, device="cuda").normal_(0, 0.5)
    y = torch.empty(N * M, dtype=torch.float32, device="cuda")
    fq = lambda: hip.check(L.vsim_op_gemm_q4_256(w.data_ptr(), M, K, x.data_ptr(), N, None, y.data_ptr(), None, None,
                                                 0, 0, 0, 0, None, None), "q4")
    fi = lambda: hip.check(L.vsim_op_gemm_f16(img.data_ptr(), M, K, x.data_ptr(), N, None, y.data_ptr(), None), "img")
    if ORDERS:
        for rnd in range(2):
            for o in ORDERS:
                L.vsim_gemm_set_tile_order(o)
                ms = timeit(fq)
                print(f"M={M} K={K} N={N} tile order {o}: {ms * 1e3:.1f} us  {2.0 * M * K * N / ms / 1e9:.0f} TFLOP/s",
                      flush=True)
        L.vsim_gemm_set_tile_order(ORDERS[0])
    if COPIES > 1:
        wc = [w] + [w.clone() for _ in range(COPIES - 1)]
        it = [0]

        def fc():
            it[0] += 1
            hip.check(L.vsim_op_gemm_q4_256(wc[it[0] % COPIES].data_ptr(), M, K, x.data_ptr(), N, None, y.data_ptr(),
                                            None, None, 0, 0, 0, 0, None, None), "q4")
        for rnd in range(2):
            for name, f in (("q4 one weight copy", fq), (f"q4 {COPIES} weight copies", fc)):
                ms = timeit(f)
                print(f"M={M} K={K} N={N} {name}: {ms * 1e3:.1f} us  {2.0 * M * K * N / ms / 1e9:.0f} TFLOP/s", flush=True)
        del wc
    for name, f in (("q4 (model kernel)", fq), ("fp16 image", fi))[:2 if IMG else 1]:
        ms = timeit(f)
        print(f"M={M} K={K} N={N} {name:18s}: {ms * 1e3:.1f} us  {2.0 * M * K * N / ms / 1e9:.0f} TFLOP/s", flush=True)
    del aos, w, img, x, y
