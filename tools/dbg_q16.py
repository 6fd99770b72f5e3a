import numpy as np, torch, sys
sys.path.insert(0, '.')
from vsim_amd import hip
DEV = 'cuda:0'
for (H, N, n_past) in [(2, 200, 0), (3, 300, 37), (1, 64, 130), (2, 300, 0), (3, 200, 0), (2, 200, 37)]:
    d = 256
    rng = np.random.default_rng(7 * N + n_past)
    E, nk = d * H, n_past + N
    q_, k_, v_ = (torch.from_numpy(rng.standard_normal((n, E)).astype(np.float32)).to(DEV) for n in (N, nk, nk))
    scale = float(np.float32(1.0 / np.sqrt(d)))
    L = hip.lib()
    out = torch.empty(N * E, dtype=torch.float32, device=DEV)
    hip.check(L.vsim_op_attn_prefill(q_.data_ptr(), k_.data_ptr(), v_.data_ptr(), d, H, N, n_past, scale, out.data_ptr(), None), "attn")
    ref16 = torch.empty(N * E, dtype=torch.float16, device=DEV)
    hip.check(L.vsim_op_act_quant_f16(out.data_ptr(), E, N, None, 0, ref16.data_ptr(), None), "aq")
    got16 = torch.full((N * E,), float("nan"), dtype=torch.float16, device=DEV)
    hip.check(L.vsim_op_attn_prefill_q16(q_.data_ptr(), k_.data_ptr(), v_.data_ptr(), d, H, N, n_past, scale, got16.data_ptr(), None), "q16")
    torch.cuda.synchronize()
    g = got16.view(torch.int16).cpu().numpy(); r = ref16.view(torch.int16).cpu().numpy()
    bad = np.nonzero(g != r)[0]
    print(H, N, n_past, "mismatches", len(bad), "nan", int(np.isnan(got16.float().cpu().numpy()).sum()))
    if len(bad):
        rows = np.unique(bad // E); cols = np.unique(bad % E)
        print(" rows", rows[:20], len(rows), " cols", cols[:20], len(cols))
        i = bad[0]; b0 = (i // 32) * 32
        o = out.cpu().numpy()[b0:b0 + 32]
        print(" block f32", o)
        print(" got", got16.cpu().numpy()[b0:b0 + 32]); print(" ref", ref16.cpu().numpy()[b0:b0 + 32])
