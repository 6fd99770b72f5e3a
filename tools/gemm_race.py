"""Race screen of the long-prompt GEMM (k_gemm_f16_256, LDS-DMA staged across raw barriers; the
model's in-LDS-dequant variant on the W4T32 weight as well as the fp16-image one):
every variant (plain, RoPE, residual join, GELU-quantize epilogue) at several shapes, REPS
launches on the same inputs, each output compared bit for bit with the first.  A staging
hazard shows up as an occasional different tile (cdna_hip_programming.md: screen a sync
structure over many runs at several sizes)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

REPS = int(os.environ.get("REPS", "40"))


def main():
    L = hip.lib()
    g = torch.Generator(device="cuda").manual_seed(7)
    bad = 0
    shapes = [(6144, 6144, 2048), (24576, 1024, 2048), (1056, 128, 257), (512, 4096, 300), (6144, 24576, 2048),
              (6144, 4096, 1800), (4096, 4096, 2048), (4096, 16384, 2048)]
    if os.environ.get("RACE_SHAPES"):  # "MxKxN,..."
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["RACE_SHAPES"].split(",")]
    for M, K, N in shapes:
        aos = torch.from_numpy(mg.quantize_q4_0(np.random.default_rng(M + K).standard_normal(M * K).astype(
            np.float32) * np.float32(0.05))).cuda()
        wq = torch.empty(hip.q4_bytes(M, K), dtype=torch.uint8, device="cuda")
        hip.check(L.vsim_op_q4_repack(aos.data_ptr(), wq.data_ptr(), M, K, None), "repack")
        w = torch.empty(M * K, dtype=torch.float16, device="cuda")
        hip.check(L.vsim_op_q4_expand_f16(wq.data_ptr(), M, K, w.data_ptr(), None), "expand")
        x = (torch.randn(N * K, device="cuda", generator=g) * 0.5).half()
        b = torch.randn(M, device="cuda", generator=g) * 0.1
        y = torch.empty(N * M, device="cuda")
        y2 = torch.empty(N * M, device="cuda")
        q = torch.empty(N * M, dtype=torch.float16, device="cuda")
        half = 32
        pos = torch.arange(N + 3, dtype=torch.float64, device="cuda")[:, None]
        th = pos * 10000.0 ** (-2.0 * torch.arange(half, dtype=torch.float64, device="cuda") / 64)[None, :]
        cs = torch.stack([torch.cos(th), torch.sin(th)], -1).contiguous()
        r0 = torch.randn(N * M, device="cuda", generator=g)
        ra = torch.randn(N * M, device="cuda", generator=g)
        runs = {
            "plain": lambda: L.vsim_op_gemm_f16(w.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), y.data_ptr(), None),
            "rope": lambda: L.vsim_op_gemm_f16_rope(w.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), y.data_ptr(),
                                                    cs.data_ptr(), 128, 64, 3, None),
            "gelu_q": lambda: L.vsim_op_gemm_f16_gelu_q(w.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), q.data_ptr(),
                                                        None),
            "q4": lambda: L.vsim_op_gemm_q4_256(wq.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), y.data_ptr(), None,
                                                None, 0, 0, 0, 0, None, None),
            "q4_rope": lambda: L.vsim_op_gemm_q4_256(wq.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), y.data_ptr(),
                                                     None, cs.data_ptr(), 128, 64, 3, 0, None, None),
            "q4_gelu": lambda: L.vsim_op_gemm_q4_256(wq.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), None,
                                                     q.data_ptr(), None, 0, 0, 0, 0, None, None),
        }
        if M % 256 == 0 and K % 128 == 0:
            def pair():  # the paired Q/K launch; the second output folded into the compared one
                rc = L.vsim_op_gemm_q4_256_pair(wq.data_ptr(), wq.data_ptr(), M, K, x.data_ptr(), N, y.data_ptr(),
                                                y2.data_ptr(), cs.data_ptr(), 128, 64, 3, None)
                y.view(torch.int32).bitwise_xor_(y2.view(torch.int32))
                return rc
            runs["q4_pair"] = pair
        for name, f in runs.items():
            out = q if name.endswith("gelu_q") or name == "q4_gelu" else y
            hip.check(f(), name)
            ref = out.clone()
            diff = 0
            for _ in range(REPS):
                hip.check(f(), name)
                h = out.dtype == torch.float16
                diff += int(not torch.equal(out.view(torch.int16) if h else out.view(torch.int32),
                                            ref.view(torch.int16) if h else ref.view(torch.int32)))
            bad += diff
            print(f"{name:7s} M={M} K={K} N={N}: {diff} of {REPS} differ", flush=True)
        # residual join in place: the same start each time
        res = r0.clone()
        hip.check(L.vsim_op_gemm_f16_join(w.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), res.data_ptr(),
                                          ra.data_ptr(), None), "join")
        ref = res.clone()
        diff = 0
        for _ in range(REPS):
            res.copy_(r0)
            hip.check(L.vsim_op_gemm_f16_join(w.data_ptr(), M, K, x.data_ptr(), N, b.data_ptr(), res.data_ptr(),
                                              ra.data_ptr(), None), "join")
            diff += int(not torch.equal(res.view(torch.int32), ref.view(torch.int32)))
        bad += diff
        print(f"join    M={M} K={K} N={N}: {diff} of {REPS} differ", flush=True)
    torch.cuda.synchronize()
    print("race screen:", "clean" if bad == 0 else f"{bad} differing outputs")
    sys.exit(0 if bad == 0 else 1)


if __name__ == "__main__":
    main()
