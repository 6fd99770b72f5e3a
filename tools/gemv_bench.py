#!/usr/bin/env python3
"""Per-shape GEMV timing (GPT-J decode shapes) for the exact and fast kernels.
usage: python tools/gemv_bench.py [--iters 50]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from vsim_amd import hip  # noqa: E402

SHAPES = [("qkvo", 4096, 4096), ("fc_in", 16384, 4096), ("fc_out", 4096, 16384), ("lm_head", 50400, 4096),
          ("qkv+fc_in rows", 28672, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--modes", default="exact,fast")
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    modes = [{"exact": hip.MODE_EXACT, "fast": hip.MODE_FAST}[m] for m in args.modes.split(",")]
    L = hip.lib()
    for name, M, K in SHAPES:
        w = torch.empty(hip.q4_bytes(M, K), dtype=torch.uint8, device="cuda")
        # random W4T32 weights via the randomizer of a throwaway 1-layer model is overkill:
        # fill bytes directly (scales must be finite)
        nblk = (M + 31) // 32 * 32 * (K // 32)
        w[: nblk * 16].random_(0, 256)
        d = w[nblk * 16:].view(torch.float32)
        d.copy_(torch.rand(nblk, device="cuda") * 0.01)
        x = torch.randn(K, device="cuda")
        xq = torch.empty(hip.q4_bytes(1, K), dtype=torch.uint8, device="cuda")
        xd = torch.empty(K, device="cuda")
        y = torch.empty(M, device="cuda")
        hip.check(L.vsim_op_q4_quantize(x.data_ptr(), K, 1, xq.data_ptr(), xd.data_ptr(), None))
        # bit-exactness of the decode kernel vs the row-per-lane kernel (n = 2 path)
        x2 = torch.cat([x, x])
        xq2 = torch.empty(hip.q4_bytes(2, K), dtype=torch.uint8, device="cuda")
        xd2 = torch.empty(2 * K, device="cuda")
        y2 = torch.empty(2 * M, device="cuda")
        hip.check(L.vsim_op_q4_quantize(x2.data_ptr(), K, 2, xq2.data_ptr(), xd2.data_ptr(), None))
        hip.check(L.vsim_op_q4_gemv(w.data_ptr(), M, K, xq2.data_ptr(), xd2.data_ptr(), 2, None, y2.data_ptr(),
                                    hip.MODE_EXACT, None))
        hip.check(L.vsim_op_q4_gemv(w.data_ptr(), M, K, xq.data_ptr(), xd.data_ptr(), 1, None, y.data_ptr(),
                                    hip.MODE_EXACT, None))
        torch.cuda.synchronize()
        if not args.no_check:
            same = torch.equal(y.view(torch.int32), y2[:M].view(torch.int32))
            print(f"{name:16s} exact decode kernel bit-identical to row kernel: {same}", flush=True)
            if not same:
                bad = (y.view(torch.int32) != y2[:M].view(torch.int32)).nonzero().flatten().cpu()
                rel = ((y - y2[:M]).abs() / y2[:M].abs().clamp_min(1e-30)).max().item()
                print(f"    {bad.numel()} rows differ (first {bad[:8].tolist()}, row%32 set "
                      f"{sorted(set((bad % 32).tolist()))[:12]}), max rel {rel:.3g}", flush=True)
        for mode in modes:
            for _ in range(3):
                hip.check(L.vsim_op_q4_gemv(w.data_ptr(), M, K, xq.data_ptr(), xd.data_ptr(), 1, None, y.data_ptr(),
                                            mode, None))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                hip.check(L.vsim_op_q4_gemv(w.data_ptr(), M, K, xq.data_ptr(), xd.data_ptr(), 1, None, y.data_ptr(),
                                            mode, None))
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            gbs = M * K * 0.625 / (us * 1e-6) / 1e9
            chain = K / 2 * 7.8 / 2.4e3  # us at 7.8 cycles per dependent add (measured), 2.4 GHz
            print(f"{name:16s} M={M:6d} K={K:6d} {'exact' if mode == 0 else 'fast ':5s} {us:9.2f} us "
                  f"{gbs:8.1f} GB/s  (chain floor {chain:.1f} us)", flush=True)

if __name__ == "__main__":
    main()
