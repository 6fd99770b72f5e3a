#!/usr/bin/env python3
"""Cross-process determinism of the fast prompt GEMM (vsim_op_q4_gemv, fast mode, n >= 8):
python3 tools/gemm_det.py --n 16 --out a.npz; ... --compare a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--m", type=int, default=2048)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        a, b = (np.load(f)["y"] for f in args.compare)
        same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
        print(f"gemm n bit-identical: {same}  max|diff| {np.abs(a - b).max():.3g}  rows differing "
              f"{int((a != b).any(axis=1).sum())} of {a.shape[0]}")
        sys.exit(0)
    import torch
    from vsim_amd import hip
    L = hip.lib()
    g = torch.Generator(device="cpu").manual_seed(7)
    M, K, N = args.m, args.k, args.n
    nblk = (M + 31) // 32 * 32 * (K // 32)
    w = torch.empty(hip.q4_bytes(M, K), dtype=torch.uint8)
    w[: nblk * 16] = torch.randint(0, 256, (nblk * 16,), generator=g, dtype=torch.uint8)
    w[nblk * 16:].view(torch.float32)[:nblk] = torch.rand(nblk, generator=g) * 0.01
    w = w.cuda()
    x = torch.randn(N * K, generator=g).cuda()
    xq = torch.empty(hip.q4_bytes(N, K), dtype=torch.uint8, device="cuda")
    xd = torch.empty(N * K, device="cuda")
    y = torch.full((N * M,), float("nan"), device="cuda")
    hip.check(L.vsim_op_q4_quantize(x.data_ptr(), K, N, xq.data_ptr(), xd.data_ptr(), None))
    hip.check(L.vsim_op_q4_gemv(w.data_ptr(), M, K, xq.data_ptr(), xd.data_ptr(), N, None, y.data_ptr(),
                                hip.MODE_FAST, None))
    torch.cuda.synchronize()
    np.savez(args.out, y=y.view(N, M).cpu().numpy())
    print("saved", args.out, "nan:", int(torch.isnan(y).sum()))


if __name__ == "__main__":
    main()
