import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip, modelgen as mg
DEV = "cuda:0"
L = hip.lib()
for (M, K, N) in [(1056, 128, 600), (3072, 1024, 512), (6144, 6144, 2048), (24576, 64, 2048)]:
    rng = np.random.default_rng(5 * M + K + N)
    w_aos = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.05))
    aos = torch.from_numpy(w_aos).to(DEV)
    w = torch.empty(hip.q4_bytes(M, K), dtype=torch.uint8, device=DEV)
    hip.check(L.vsim_op_q4_repack(aos.data_ptr(), w.data_ptr(), M, K, None), "repack")
    img = torch.empty(M * K, dtype=torch.float16, device=DEV)
    hip.check(L.vsim_op_q4_expand_f16(w.data_ptr(), M, K, img.data_ptr(), None), "expand")
    x = torch.from_numpy((rng.standard_normal((N, K)) * 0.5).astype(np.float16)).to(DEV)
    bd = torch.from_numpy((rng.standard_normal(M) * 0.1).astype(np.float32)).to(DEV)
    a = torch.empty(N * M, dtype=torch.float16, device=DEV); b = torch.empty_like(a); c = torch.empty_like(a)
    hip.check(L.vsim_op_gemm_f16_gelu_q(img.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), a.data_ptr(), None), "img")
    hip.check(L.vsim_op_gemm_q4_256(w.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), None, b.data_ptr(), None, 0, 0, 0, 0, None, None), "q4")
    hip.check(L.vsim_op_gemm_q4_256(w.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), None, c.data_ptr(), None, 0, 0, 0, 0, None, None), "q4")
    torch.cuda.synchronize()
    ai, bi, ci = (t.view(torch.int16).cpu().numpy() for t in (a, b, c))
    bad = np.nonzero(ai != bi)[0]
    print(f"M={M} K={K} N={N}: img vs q4 {len(bad)} differ, q4 rerun {int((bi != ci).sum())} differ", flush=True)
    if len(bad):
        n_, m_ = bad // M, bad % M
        print("  rows m", np.unique(m_)[:12], " cols n", np.unique(n_)[:12], "count rows", len(np.unique(m_)))
        i = bad[0]; print("  img", a.view(-1)[i].item(), "q4", b.view(-1)[i].item())
