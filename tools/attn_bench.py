"""Microbench of the fast prompt attention (vsim_op_attn_prefill: k_kv_f16 + k_attn_prefill_f16)
at the codegen-16B shape (N = 2048, d = 256, H = 24); prints the mean time and a hash of the
output bits (A/B builds via VSIM_LIB must agree on it when they only reschedule)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402


def main(N=2048, d=256, H=24, reps=20):
    E = d * H
    g = torch.Generator(device="cuda").manual_seed(1)
    q = torch.randn(N * E, device="cuda", generator=g) * 0.5
    k = torch.randn(N * E, device="cuda", generator=g) * 0.5
    v = torch.randn(N * E, device="cuda", generator=g)
    out = torch.empty(N * E, device="cuda")
    L = hip.lib()
    scale = 1.0 / d ** 0.5

    def go():
        hip.check(L.vsim_op_attn_prefill(q.data_ptr(), k.data_ptr(), v.data_ptr(), d, H, N, 0, scale, out.data_ptr(),
                                         None), "attn")
    for _ in range(3):
        go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
    print(f"attn N={N} d={d} H={H}: {1e3 * e0.elapsed_time(e1) / reps:.1f} us per call, out {h}")


if __name__ == "__main__":
    main()
