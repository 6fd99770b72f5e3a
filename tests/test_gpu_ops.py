"""Per-op parity of the HIP kernels (through the C-ABI) against the reference's own
outputs (tests/golden/ops_*.npz, produced by the reference ggml ops at --threads 1).

Exact mode must be bit-identical.  The fast GEMV is checked against an fp64 evaluation
of the same Q4_0 x Q4_0 product with an error bound (tolerance written below).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from golden_util import cases, ops  # noqa: E402
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def repack(aos_np, rows, k):
    src = dev(aos_np)
    dst = torch.empty(hip.q4_bytes(rows, k), dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_q4_repack(src.data_ptr(), dst.data_ptr(), rows, k, None), "repack")
    return dst


def quantize(x_np, k, n):
    x = dev(x_np.astype(np.float32))
    xq = torch.empty(hip.q4_bytes(n, k), dtype=torch.uint8, device=DEV)
    xd = torch.empty(n * k, dtype=torch.float32, device=DEV)
    hip.check(hip.lib().vsim_op_q4_quantize(x.data_ptr(), k, n, xq.data_ptr(), xd.data_ptr(), None), "quantize")
    return xq, xd


def gemv(w, M, K, xq, xd, n, mode, bias=None):
    y = torch.empty(n * M, dtype=torch.float32, device=DEV)
    hip.check(hip.lib().vsim_op_q4_gemv(w.data_ptr(), M, K, xq.data_ptr(), xd.data_ptr(), n,
                                        None if bias is None else bias.data_ptr(), y.data_ptr(), mode, None), "gemv")
    return host(y)


def test_repack_roundtrip():
    rng = np.random.default_rng(0)
    aos = mg.quantize_q4_0(rng.standard_normal(96 * 256).astype(np.float32))
    soa = repack(aos, 96, 256)
    back = torch.empty(aos.size, dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_q4_unpack(soa.data_ptr(), back.data_ptr(), 96, 256, None), "unpack")
    assert np.array_equal(host(back), aos)
    # rows not a multiple of the 32-row tile (pythia's 50288-row head)
    aos2 = mg.quantize_q4_0(rng.standard_normal(50 * 64).astype(np.float32))
    w2 = repack(aos2, 50, 64)
    back2 = torch.empty(aos2.size, dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_q4_unpack(w2.data_ptr(), back2.data_ptr(), 50, 64, None), "unpack")
    assert np.array_equal(host(back2), aos2)


def test_quantize_bit_exact():
    z = ops("qrow")
    x = z["x"]
    xq, _ = quantize(x, x.size, 1)
    aos = torch.empty(x.size // 32 * 20, dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_act_unpack(xq.data_ptr(), aos.data_ptr(), 1, x.size, None), "unpack")
    assert np.array_equal(host(aos), z["y"])


@pytest.mark.parametrize("c", cases(ops("mulmat")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_gemv_exact_bit_exact(c):
    M, K, N = (int(v) for v in c["shape"])
    w = repack(c["w"], M, K)
    xq, xd = quantize(c["x"], K, N)
    y = gemv(w, M, K, xq, xd, N, hip.MODE_EXACT)
    assert np.array_equal(bits(y), bits(c["y"]))


@pytest.mark.parametrize("M,K,N", [(33, 64, 2), (130, 96, 129), (1000, 128, 300), (257, 4096, 5),
                                   (4096, 64, 1030), (6144, 256, 256), (96, 24576, 17)])
def test_gemm_exact_ragged_vs_oracle(M, K, N):
    """The exact prompt GEMM (gemm_exact.hip: 128 x 128 tiles of (row, token) chains) against
    the oracle's mul_mat (ggml.c:4891-5165 with its INIT quantization): bit-identical at ragged
    M, N (partial tiles in both directions), one-block K, and with a bias epilogue."""
    import oracle_py as O
    rng = np.random.default_rng(M * 7 + K * 3 + N)
    w_aos = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.02))
    x = (rng.standard_normal(N * K) * 1.5).astype(np.float32)
    w = repack(w_aos, M, K)
    xq, xd = quantize(x, K, N)
    y = gemv(w, M, K, xq, xd, N, hip.MODE_EXACT).reshape(N, M)
    y_or = O.mul_mat(w_aos, M, K, x, N, nthreads=8).reshape(N, M)
    assert np.array_equal(bits(y), bits(y_or))
    b = rng.standard_normal(M).astype(np.float32)
    yb = gemv(w, M, K, xq, xd, N, hip.MODE_EXACT, bias=dev(b)).reshape(N, M)
    assert np.array_equal(bits(yb), bits(y_or + b[None, :]))


def _fp64_product(w_aos, M, K, xq_aos, N):
    W = mg.dequantize_q4_0(w_aos, K).astype(np.float64)       # [M, K]
    X = mg.dequantize_q4_0(xq_aos, K).astype(np.float64)      # [N, K]
    return (X @ W.T), (np.abs(X) @ np.abs(W).T)


@pytest.mark.parametrize("c", cases(ops("mulmat")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_gemv_fast_within_bound(c):
    M, K, N = (int(v) for v in c["shape"])
    w = repack(c["w"], M, K)
    xq, xd = quantize(c["x"], K, N)
    y = gemv(w, M, K, xq, xd, N, hip.MODE_FAST).reshape(N, M)
    xq_aos = torch.empty(N * K // 32 * 20, dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_act_unpack(xq.data_ptr(), xq_aos.data_ptr(), N, K, None), "unpack")
    exact, absum = _fp64_product(c["w"], M, K, host(xq_aos), N)
    # tolerance: |y - y64| <= 4*K*2^-24 * sum|w_i x_i| (fp32 accumulation bound, well above
    # the observed error); the reference's own chain meets the same bound
    tol = 4.0 * K * 2.0 ** -24 * absum + 1e-30
    assert np.all(np.abs(y - exact) <= tol)
    assert np.all(np.abs(c["y"].reshape(N, M) - exact) <= tol)


def test_gemv_bias_epilogue():
    rng = np.random.default_rng(3)
    M, K = 256, 512
    aos = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.02))
    b = rng.standard_normal(M).astype(np.float32)
    w = repack(aos, M, K)
    xq, xd = quantize(rng.standard_normal(K).astype(np.float32), K, 1)
    y0 = gemv(w, M, K, xq, xd, 1, hip.MODE_EXACT)
    y1 = gemv(w, M, K, xq, xd, 1, hip.MODE_EXACT, bias=dev(b))
    assert np.array_equal(bits(y1), bits((y0 + b).astype(np.float32)))


@pytest.mark.parametrize("c", cases(ops("norm")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_norm_bit_exact(c):
    n, r = (int(v) for v in c["shape"])
    x = dev(c["x"])
    y = torch.empty_like(x)
    hip.check(hip.lib().vsim_op_norm(x.data_ptr(), y.data_ptr(), n, r, None, None, None), "norm")
    assert np.array_equal(bits(host(y)), bits(c["y"]))


def test_norm_fallback_paths():
    """Rows built to defeat both fast-path certificates must still match the oracle."""
    import oracle_py as O
    rng = np.random.default_rng(11)
    n = 4096
    rows = []
    r0 = rng.standard_normal(n).astype(np.float32) * 100
    r0[::7] = np.float32(1e-30)  # tiny values: mean sum not provably exact
    rows.append(r0)
    r1 = np.full(n, 3.0, np.float32) + rng.standard_normal(n).astype(np.float32) * np.float32(1e-6)
    rows.append(r1)  # near-constant row: variance tiny
    x = np.concatenate(rows).astype(np.float32)
    ref = O.norm(x, n, len(rows))
    xt = dev(x)
    y = torch.empty_like(xt)
    hip.check(hip.lib().vsim_op_norm(xt.data_ptr(), y.data_ptr(), n, len(rows), None, None, None), "norm")
    assert np.array_equal(bits(host(y)), bits(ref))


@pytest.mark.parametrize("n", [4096, 4160, 1024])
def test_norm_sequential_mean_sum_cases(n):
    """The LayerNorm's fallback for rows whose mean sum is not provably order-independent
    (kern.hpp seq_sum_exact: per-256 chunk certificates, exact prefix sums, speculation from
    the running sum checked by TwoSum, lane-0 order where a chunk fails): rows with one or a
    few tiny elements (the common case: no restart), many tiny elements in one chunk (more
    roundings than the restart cap), a huge dynamic range inside a chunk (its certificate
    fails), denormals, zeros, a large running sum that rounds as it grows, exact cancellations,
    a partial last chunk (n = 4160).  Every row against the oracle's sequential sum, bit for bit."""
    import oracle_py as O
    rng = np.random.default_rng(n)
    rows = []
    for k in range(48):
        r = (rng.standard_normal(n) * rng.choice([0.05, 1.0, 40.0])).astype(np.float32)
        kind = k % 8
        if kind == 0:
            r[rng.integers(0, n)] = np.float32(3e-7) * np.float32(rng.standard_normal())
        elif kind == 1:
            r[rng.integers(0, n, 5)] = (rng.standard_normal(5) * 1e-9).astype(np.float32)
        elif kind == 2:
            c = rng.integers(0, n // 256) * 256
            r[c:c + 200] = (rng.standard_normal(200) * 1e-12).astype(np.float32)  # > the cap in one chunk
        elif kind == 3:
            r[rng.integers(0, n, 3)] = np.float32(1e30)
            r[rng.integers(0, n, 3)] = np.float32(1e-30)
        elif kind == 4:
            r[rng.integers(0, n, 7)] = np.float32(1e-41)  # denormals
            r[rng.integers(0, n, 50)] = np.float32(0.0)
        elif kind == 5:
            r = (np.abs(r) * 1000 + 1e-4 * rng.standard_normal(n)).astype(np.float32)  # growing running sum
        elif kind == 6:
            r[1::2] = -r[0::2]  # exact cancellation pairs ...
            r[rng.integers(0, n)] = np.float32(1e-8)  # ... and one tiny element
        else:
            r[rng.integers(0, n, 40)] *= np.float32(1e-7)
        rows.append(r)
    x = np.concatenate(rows).astype(np.float32)
    ref = O.norm(x, n, len(rows))
    xt = dev(x)
    y = torch.empty_like(xt)
    g = torch.zeros(64, device=DEV)  # (an op that fetches the device tables also sets up the fallback counters)
    hip.check(hip.lib().vsim_op_gelu(g.data_ptr(), g.data_ptr(), g.numel(), None), "gelu")
    torch.cuda.synchronize()
    before = hip.norm_fallbacks()[0]
    hip.check(hip.lib().vsim_op_norm(xt.data_ptr(), y.data_ptr(), n, len(rows), None, None, None), "norm")
    got = host(y).reshape(len(rows), n)
    bad = [i for i in range(len(rows)) if not np.array_equal(bits(got[i]), bits(ref.reshape(len(rows), n)[i]))]
    assert not bad, f"rows {bad} differ"
    assert hip.norm_fallbacks()[0] > before  # the fallback path ran


def _argmax_rows(n, rng):
    base = rng.standard_normal(n).astype(np.float32)
    rows = {"random": base}
    t = base.copy()  # the maximum at three indices: the first one wins
    if n >= 3:
        m = t.max() + 1
        for i in sorted(rng.choice(n, 3, replace=False)):
            t[i] = m
    rows["ties"] = t
    t = base.copy()
    if n >= 2:
        i, j = sorted(rng.choice(n, 2, replace=False))
        t[j], t[i] = np.nan, np.nan  # the first NaN wins over every number
    rows["nan"] = t
    z = np.zeros(n, np.float32)
    z[: (n + 1) // 2] = -0.0  # -0.0 equals +0.0: index 0
    rows["zeros"] = z
    rows["neg_inf"] = np.full(n, -np.inf, np.float32)
    t = np.full(n, -np.inf, np.float32)
    t[-1] = np.float32(-3.4e38)
    rows["last"] = t
    return rows


@pytest.mark.parametrize("n", [1, 7, 1029, 50400, 250880, 262147])
def test_argmax_numpy_conventions(n):
    """vsim_op_argmax (the kernel of the model's greedy step) returns numpy.argmax: first of
    equal maxima, -0.0 == +0.0, first NaN; rows from 1 value to BLOOM's vocabulary and past it,
    on 16-byte-aligned and misaligned rows (the float4 path and the scalar path).  The tie rule
    is numpy's, not the reference's: its greedy pick (sample_top_k, utils.cpp:339-371) orders
    equal logits by std::partial_sort, which leaves their order unspecified; rows without ties
    give the same index either way."""
    rng = np.random.default_rng(n)
    out = torch.zeros(1, dtype=torch.int32, device=DEV)
    for name, row in _argmax_rows(n, rng).items():
        for off in (0, 1):
            buf = np.concatenate([np.zeros(off, np.float32), row])
            xt = dev(buf)
            hip.check(hip.lib().vsim_op_argmax(xt.data_ptr() + 4 * off, n, out.data_ptr(), None), "argmax")
            assert int(out.item()) == int(np.argmax(row)), (name, off)


def test_gelu_bit_exact():
    z = ops("gelu")
    x = dev(z["x"])
    y = torch.empty_like(x)
    hip.check(hip.lib().vsim_op_gelu(x.data_ptr(), y.data_ptr(), x.numel(), None), "gelu")
    assert np.array_equal(bits(host(y)), bits(z["y"]))


@pytest.mark.parametrize("c", cases(ops("attnsm")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_scale_mask_softmax_bit_exact(c):
    nc, nr, nz, n_past = (int(v) for v in c["shape"])
    p = dev(c["x"])
    hip.check(hip.lib().vsim_op_attn_softmax(p.data_ptr(), nc, nr, nz, n_past, float(c["scale"][0]), None), "sm")
    assert np.array_equal(bits(host(p)), bits(c["y"]))


@pytest.mark.parametrize("style", [0, 1], ids=["neox", "gptj"])
def test_rope_bit_exact(style):
    for c in cases(ops("rope_neox" if style == 0 else "rope_gptj")):
        d, H, T, n_past, n_dims, mode = (int(v) for v in c["shape"])
        x = dev(c["x"])
        hip.check(hip.lib().vsim_op_rope(style, x.data_ptr(), d, H, T, n_past, n_dims, mode, None), "rope")
        assert np.array_equal(bits(host(x)), bits(c["y"])), c["shape"]


def test_kq_bit_exact():
    for c in cases(ops("kq")):
        d, H, nk, N = (int(v) for v in c["shape"])
        K, Q = dev(c["a"]), dev(c["b"])
        out = torch.empty(H * N * nk, dtype=torch.float32, device=DEV)
        hip.check(hip.lib().vsim_op_kq(K.data_ptr(), d * H, Q.data_ptr(), d * H, d, H, nk, N, out.data_ptr(), None),
                  "kq")
        assert np.array_equal(bits(host(out)), bits(c["y"])), c["shape"]


def test_kqv_bit_exact():
    for c in cases(ops("kqv")):
        d, H, nk, N = (int(v) for v in c["shape"])
        V, S = dev(c["a"]), dev(c["b"])
        out = torch.empty(H * N * d, dtype=torch.float32, device=DEV)
        hip.check(hip.lib().vsim_op_kqv(V.data_ptr(), d * H, S.data_ptr(), d, H, nk, N, out.data_ptr(), None), "kqv")
        assert np.array_equal(bits(host(out)), bits(c["y"])), c["shape"]


@pytest.mark.parametrize("d,H,nk,N", [(64, 3, 130, 70), (96, 2, 97, 33), (256, 2, 300, 257), (4, 1, 5, 3),
                                      (128, 2, 64, 64)])
def test_kq_kqv_tiled_vs_oracle(d, H, nk, N):
    """The prompt attention products (attn_exact.hip, 64 x 64 register tiles) against the
    oracle's KQ (double sum of float products, ggml.c:399-434) and KQV (float chain over the keys,
    ggml.c:610-639) at ragged shapes: partial tiles in every direction, d not a multiple of the
    32-element staging chunk, softmax-like rows with exact zeros."""
    import oracle_py as O
    rng = np.random.default_rng(d * 1000 + nk + N)
    K = rng.standard_normal((nk, d * H)).astype(np.float32)
    Q = rng.standard_normal((N, d * H)).astype(np.float32)
    out = torch.empty(H * N * nk, dtype=torch.float32, device=DEV)
    Kd, Qd = dev(K), dev(Q)  # (held: a temporary's memory would be reused by the next allocation)
    hip.check(hip.lib().vsim_op_kq(Kd.data_ptr(), d * H, Qd.data_ptr(), d * H, d, H, nk, N, out.data_ptr(), None), "kq")
    assert np.array_equal(bits(host(out)), bits(O.kq(K, Q, d, H, nk, N)))
    V = rng.standard_normal((nk, d * H)).astype(np.float32)
    S = rng.random((H, N, nk)).astype(np.float32)
    S[S < 0.3] = 0.0
    out = torch.empty(H * N * d, dtype=torch.float32, device=DEV)
    Vd, Sd = dev(V), dev(S)
    hip.check(hip.lib().vsim_op_kqv(Vd.data_ptr(), d * H, Sd.data_ptr(), d, H, nk, N, out.data_ptr(), None), "kqv")
    assert np.array_equal(bits(host(out)), bits(O.kqv(V, S, d, H, nk, N)))


@pytest.mark.parametrize("d,H,N,n_past", [(64, 3, 130, 70), (256, 2, 200, 3), (96, 2, 65, 64), (128, 1, 64, 0)])
def test_kq_kqv_causal_vs_oracle(d, H, N, n_past):
    """The causal skipping of the exact prompt products (attn_exact.hip: fully masked KQ tiles left
    unwritten, KQV chains stopped at the tile's last unmasked key) with multi-tile query batches on
    top of a cache (n_past > 0) and ragged edges: every unmasked score bit for bit the oracle's,
    masked ones untouched where a whole tile is masked, and KQV over probabilities that are +0
    past each query's last key bit for bit the oracle's full chain."""
    import oracle_py as O
    nk = n_past + N
    rng = np.random.default_rng(7 * d + 31 * N + n_past)
    K = rng.standard_normal((nk, d * H)).astype(np.float32)
    Q = rng.standard_normal((N, d * H)).astype(np.float32)
    out = torch.full((H * N * nk,), 12345.0, dtype=torch.float32, device=DEV)
    Kd, Qd = dev(K), dev(Q)
    hip.check(hip.lib().vsim_op_kq_causal(Kd.data_ptr(), d * H, Qd.data_ptr(), d * H, d, H, nk, N, n_past,
                                          out.data_ptr(), None), "kq_causal")
    got = host(out).reshape(H, N, nk)
    ref = O.kq(K, Q, d, H, nk, N).reshape(H, N, nk)
    seen = np.arange(nk)[None, :] <= (n_past + np.arange(N))[:, None]  # query j sees keys <= n_past + j
    assert np.array_equal(bits(got[:, seen]), bits(ref[:, seen]))
    # a 64 x 64 tile (query block, key block) whose keys are all past every query's last key
    for q0 in range(0, N, 64):
        for k0 in range(0, nk, 64):
            if k0 > n_past + min(q0 + 64, N) - 1:
                assert np.all(got[:, q0:q0 + 64, k0:k0 + 64] == 12345.0), (q0, k0)
    V = rng.standard_normal((nk, d * H)).astype(np.float32)
    S = rng.random((H, N, nk)).astype(np.float32)
    S[S < 0.3] = 0.0
    S[:, ~seen] = 0.0  # what softmax leaves past the mask
    out = torch.empty(H * N * d, dtype=torch.float32, device=DEV)
    Vd, Sd = dev(V), dev(S)
    hip.check(hip.lib().vsim_op_kqv_causal(Vd.data_ptr(), d * H, Sd.data_ptr(), d, H, nk, N, n_past,
                                           out.data_ptr(), None), "kqv_causal")
    assert np.array_equal(bits(host(out)), bits(O.kqv(V, S, d, H, nk, N)))


def test_get_rows_bit_exact():
    z = ops("getrows")
    K, V = (int(v) for v in z["shape"])
    w = repack(z["w"], V, K)
    idx = dev(z["idx"])
    y = torch.empty(idx.numel() * K, dtype=torch.float32, device=DEV)
    hip.check(hip.lib().vsim_op_get_rows(w.data_ptr(), K, V, idx.data_ptr(), idx.numel(), y.data_ptr(), None), "rows")
    assert np.array_equal(bits(host(y)), bits(z["y"]))


def rand_q4_aos(rng, M, K, std=0.02):
    """Random Q4_0 rows straight as AoS blocks (uniform nibbles, scales |N(0, 1)| * std / 3):
    the shape of a quantized weight without quantizing hundreds of millions of floats."""
    nblk = M * K // 32
    out = np.empty((nblk, 20), np.uint8)
    out[:, :4] = (np.abs(rng.standard_normal(nblk, dtype=np.float32)) * np.float32(std / 3)).view(np.uint8).reshape(-1, 4)
    out[:, 4:] = rng.integers(0, 256, (nblk, 16), dtype=np.uint8)
    return out.reshape(-1)


# Shapes and the kernel launch_gemv_chain_batch picks for them (gemv_chain.hip): >= 192
# 128-row groups -> k_gemv_solo with two consumers (the bench's Q/K/V + fc_in batch, 28672 x
# 4096; 24600 x 4096: a ragged last group and a partial last tile; the heads), else >= 192
# 64-row groups -> k_gemv_solo with one (fc_in alone, 16384 x 4096), fewer -> k_gemv_chain32
# (fc_out, out-projection).
@pytest.mark.parametrize("M,K", [(4096, 4096), (1024, 16384), (50400, 256), (16384, 4096), (28672, 4096),
                                 (24600, 4096), (50400, 4096), (50432, 6144), (250880, 1024), (6144, 24576),
                                 (4064, 4096)])
def test_gemv_exact_full_width_vs_oracle(M, K):
    """GPT-J / 20B / BLOOM widths (K = n_embd and 4*n_embd, V rows) against the CPU restatement."""
    import oracle_py as O
    rng = np.random.default_rng(M + K)
    aos = rand_q4_aos(rng, M, K)
    x = rng.standard_normal(K).astype(np.float32)
    ref = O.mul_mat(aos, M, K, x, 1, nthreads=16)
    w = repack(aos, M, K)
    xq, xd = quantize(x, K, 1)
    assert np.array_equal(bits(gemv(w, M, K, xq, xd, 1, hip.MODE_EXACT)), bits(ref))



def w16_of(w_aos, K):
    """The fp16 weight operand of the prompt GEMMs: each Q4_0 value d*(q-8) rounded ONCE to
    fp16 from its exact value (gemm_f16.hip deq_word_f16: one v_fma_mix; the product d*(q-8)
    is exact in fp64 and numpy's fp64 -> fp16 conversion rounds to nearest even directly)."""
    blk = np.asarray(w_aos, dtype=np.uint8).reshape(-1, mg.QBYTES)
    d = blk[:, :4].copy().view(np.float32).reshape(-1).astype(np.float64)
    q = np.empty((blk.shape[0], 32), dtype=np.float64)
    q[:, 0::2] = (blk[:, 4:] & 0xF).astype(np.float64) - 8
    q[:, 1::2] = (blk[:, 4:] >> 4).astype(np.float64) - 8
    return (q * d[:, None]).astype(np.float16).reshape(-1, K)

@pytest.mark.parametrize("M,K,N", [(520, 512, 300), (256, 4096, 8), (1000, 1024, 129), (96, 96, 40)])
def test_prefill_gemm_f16(M, K, N):
    """Fast-mode prompt GEMM (gemm_f16.hip: fp16 MFMA after in-LDS dequant).  Operands are
    d*(q-8) rounded to fp16 (the weight once from its exact value, w16_of; the activation via
    its f32 value), products exact, fp32 accumulation: the result must be
    within 4*K*2^-24*sum|w16*x16| of the fp64 product of the fp16-rounded operands, and
    within 2^-10*sum|w*x| (operand rounding) of the unrounded Q4_0 x Q4_0 product.
    Ragged M and N (not multiples of the 128 x 128 tile) and K = 96 (odd block count)."""
    rng = np.random.default_rng(M + K + N)
    w_aos = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.05))
    b = rng.standard_normal(M).astype(np.float32)
    w = repack(w_aos, M, K)
    xq, xd = quantize(rng.standard_normal(N * K).astype(np.float32), K, N)
    y = gemv(w, M, K, xq, xd, N, hip.MODE_FAST, bias=dev(b)).reshape(N, M)
    xq_aos = torch.empty(N * K // 32 * 20, dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_act_unpack(xq.data_ptr(), xq_aos.data_ptr(), N, K, None), "unpack")
    W = mg.dequantize_q4_0(w_aos, K)
    X = mg.dequantize_q4_0(host(xq_aos), K)
    W16 = w16_of(w_aos, K).astype(np.float64)
    X16 = X.astype(np.float16).astype(np.float64)
    ref16 = X16 @ W16.T + b
    abs16 = np.abs(X16) @ np.abs(W16).T
    assert np.all(np.abs(y - ref16) <= 4.0 * K * 2.0 ** -24 * abs16 + 1e-6 * np.abs(b))
    ref = X.astype(np.float64) @ W.astype(np.float64).T + b
    absum = np.abs(X.astype(np.float64)) @ np.abs(W.astype(np.float64)).T
    assert np.all(np.abs(y - ref) <= 2.0 ** -10 * absum + 1e-5 * (np.abs(b) + 1))


@pytest.mark.parametrize("c", cases(ops("mulmat_prompt")), ids=lambda c: "x".join(map(str, c["shape"][:3])))
def test_prompt_gemm_vs_reference_mul_mat(c):
    """Both prompt GEMM paths against the REFERENCE's Q4_0 mul_mat output at prompt shapes
    (tests/golden/ops_mulmat_prompt.npz: ggml.c:4891-5165 at N >= 256, K = 4096 / 6144 / 24576):
      * exact mode (the chain GEMV over N rows, k_gemv_exact_rows): bit-identical;
      * the long-prompt fast path the model runs for N >= 256 (vsim_op_act_quant_f16, then
        vsim_op_gemm_q4_256: the W4T32 weight dequantized to fp16 in LDS, fp16 MFMA, fp32
        accumulation, gemm_f16.hip): per element
          |y - y_ref| <= (2^-10 + 1.5 K 2^-24) * sum_k |w_k x_k|
        (w, x the Q4_0 values d*(q-8)): each fp16 operand carries <= 2^-11 relative rounding,
        the reference's K/2-add fp32 chain and our fp32 accumulation <= (K/2 + K) 2^-24 each.
        This bound is derived, not fitted; the measured maximum is printed."""
    import golden_util as gu
    M, K, N, seed = (int(v) for v in c["shape"])
    w_aos, x = gu.prompt_mulmat_inputs(M, K, N, seed)
    assert gu.inputs_sha(w_aos, x) == str(c["sha"])
    y_ref = c["y"].reshape(N, M)
    w = repack(w_aos, M, K)
    xq, xd = quantize(x, K, N)
    y = gemv(w, M, K, xq, xd, N, hip.MODE_EXACT).reshape(N, M)
    assert np.array_equal(bits(y), bits(y_ref)), "exact prompt GEMV"
    # the fast path, as the model's long-prompt layer calls it (the GEMM on the W4T32 weight)
    x16 = torch.empty(N * K, dtype=torch.float16, device=DEV)
    xt = dev(x)
    hip.check(hip.lib().vsim_op_act_quant_f16(xt.data_ptr(), K, N, None, 0, x16.data_ptr(), None), "act_quant")
    yf = torch.empty(N * M, dtype=torch.float32, device=DEV)
    hip.check(hip.lib().vsim_op_gemm_q4_256(w.data_ptr(), M, K, x16.data_ptr(), N, None, yf.data_ptr(), None, None,
                                            0, 0, 0, 0, None, None), "gemm")
    yf = host(yf).reshape(N, M)
    xq_aos = torch.empty(N * K // 32 * 20, dtype=torch.uint8, device=DEV)
    hip.check(hip.lib().vsim_op_act_unpack(xq.data_ptr(), xq_aos.data_ptr(), N, K, None), "unpack")
    W = np.abs(mg.dequantize_q4_0(w_aos, K).astype(np.float64))
    X = np.abs(mg.dequantize_q4_0(host(xq_aos), K).astype(np.float64))
    absum = X @ W.T
    bound = (2.0 ** -10 + 1.5 * K * 2.0 ** -24) * absum
    err = np.abs(yf.astype(np.float64) - y_ref)
    ratio = float(np.max(err / np.maximum(absum, 1e-30)))
    print(f"{M}x{K}x{N}: max |y - y_ref| / sum|w x| = {ratio:.3g} (bound {2.0 ** -10 + 1.5 * K * 2.0 ** -24:.3g})")
    bad = err > bound
    assert not bad.any(), f"{bad.sum()} elements outside the bound, worst ratio {ratio:.3g}"


@pytest.mark.parametrize("M,K,N", [(520, 512, 300), (256, 64, 256), (1000, 128, 600), (3072, 1024, 512),
                                   (300, 4096, 257), (24576, 64, 2048)])
def test_prefill_gemm_f16_256(M, K, N):
    """Long-prompt GEMM (gemm_f16.hip k_gemm_f16_256 on the fp16 weight image of
    k_w4_expand_f16): the image holds exactly the fp16 roundings of d*(q-8) (w16_of); the product is
    within 4*K*2^-24*sum|w16*x16| of the fp64 product of the same fp16 operands.  Ragged M
    and N (not multiples of the tile), K = 64 and 128 (one and two K-tiles: the prologue's and
    loop's clamped stages), K = 4096; 192-row tiles everywhere but (24576, 64, 2048), whose
    shape takes the 256-row tiles (launch_gemm_f16_256's choice)."""
    rng = np.random.default_rng(3 * M + K + N)
    w_aos = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.05))
    b = rng.standard_normal(M).astype(np.float32)
    w = repack(w_aos, M, K)
    W16 = w16_of(w_aos, K)
    img = torch.empty(M * K, dtype=torch.float16, device=DEV)
    hip.check(hip.lib().vsim_op_q4_expand_f16(w.data_ptr(), M, K, img.data_ptr(), None), "expand")
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy().view(np.uint16), W16.reshape(-1).view(np.uint16))
    X16 = (rng.standard_normal((N, K)) * 0.5).astype(np.float16)
    x16 = torch.from_numpy(X16).to(DEV)
    y = torch.empty(N * M, dtype=torch.float32, device=DEV)
    bt = dev(b)
    hip.check(hip.lib().vsim_op_gemm_f16(img.data_ptr(), M, K, x16.data_ptr(), N, bt.data_ptr(), y.data_ptr(),
                                         None), "gemm")
    torch.cuda.synchronize()
    y = y.cpu().numpy().reshape(N, M)
    Wd, Xd = W16.astype(np.float64).reshape(M, K), X16.astype(np.float64)
    ref = Xd @ Wd.T + b
    tol = 4.0 * K * 2.0 ** -24 * (np.abs(Xd) @ np.abs(Wd).T) + 1e-6 * np.abs(b)
    bad = np.abs(y - ref) > tol
    assert not bad.any(), f"{bad.sum()} of {bad.size} outside the bound, first {np.argwhere(bad)[:4].tolist()}"


@pytest.mark.parametrize("M,K,N,d,n_rot,p0", [(512, 256, 300, 128, 64, 0), (1024, 128, 257, 256, 64, 37),
                                              (6144, 512, 520, 256, 64, 5)])
def test_prefill_gemm_rope_join_epilogues_bit_identical(M, K, N, d, n_rot, p0):
    """The long-prompt GEMM with RoPE (Q and K of a GPT-J prompt, written straight to their
    cache rows) or the residual join (fc_out) in its epilogue: bit-identical to the plain GEMM
    followed by the step's own arithmetic -- k_rope_kv_write's double products rounded to
    float (vsim.cpp:553-580), k_add_residual's inpL + (attn + ff) and ff + inpL orders
    (vsim.cpp:694-695, 657) -- restated here in numpy (ragged N, n_past > 0)."""
    rng = np.random.default_rng(M + K + N + p0)
    W16 = (rng.standard_normal((M, K)) * 0.05).astype(np.float16)
    X16 = (rng.standard_normal((N, K)) * 0.5).astype(np.float16)
    b = (rng.standard_normal(M) * 0.1).astype(np.float32)
    w, x, bd = torch.from_numpy(W16).to(DEV), torch.from_numpy(X16).to(DEV), dev(b)
    L = hip.lib()
    y = torch.empty(N * M, dtype=torch.float32, device=DEV)
    hip.check(L.vsim_op_gemm_f16(w.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), y.data_ptr(), None), "gemm")
    y0 = y.cpu().numpy().reshape(N, M)
    # RoPE: the table as the model builds it ([pos][n_rot/2] of (cos, sin) in double)
    half = n_rot // 2
    pos = np.arange(p0 + N, dtype=np.float64)[:, None]
    theta = pos * 10000.0 ** (-2.0 * np.arange(half, dtype=np.float64) / n_rot)[None, :]
    cs = np.stack([np.cos(theta), np.sin(theta)], axis=-1)  # [pos][half][2]
    yr = torch.empty(N * M, dtype=torch.float32, device=DEV)
    csd = torch.from_numpy(np.ascontiguousarray(cs)).to(DEV)
    hip.check(L.vsim_op_gemm_f16_rope(w.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), yr.data_ptr(),
                                      csd.data_ptr(), d, n_rot, p0, None), "rope")
    ref = y0.copy()
    hd = ref.reshape(N, M // d, d)
    x0, x1 = hd[:, :, 0:n_rot:2].astype(np.float64), hd[:, :, 1:n_rot:2].astype(np.float64)
    c = cs[p0:p0 + N, :, 0][:, None, :]
    s = cs[p0:p0 + N, :, 1][:, None, :]
    r0, r1 = (x0 * c - x1 * s).astype(np.float32), (x0 * s + x1 * c).astype(np.float32)
    hd[:, :, 0:n_rot:2], hd[:, :, 1:n_rot:2] = r0, r1
    assert np.array_equal(yr.cpu().numpy().reshape(N, M).view(np.uint32), ref.view(np.uint32))
    # residual join, parallel (res + (res_a + y)) and serial (y + res) orders, in place
    R = rng.standard_normal((N, M)).astype(np.float32)
    A = rng.standard_normal((N, M)).astype(np.float32)
    for a in (A, None):
        res = torch.from_numpy(R.copy()).to(DEV)
        ad = torch.from_numpy(a).to(DEV) if a is not None else None
        hip.check(L.vsim_op_gemm_f16_join(w.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), res.data_ptr(),
                                          ad.data_ptr() if ad is not None else None, None), "join")
        want = R + (a + y0) if a is not None else y0 + R
        assert np.array_equal(res.cpu().numpy().view(np.uint32), want.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("M,K,N", [(512, 256, 300), (1056, 128, 257), (4096, 1024, 512)])
def test_prefill_gemm_gelu_epilogue_bit_identical(M, K, N):
    """fc_in of a long prompt with bias + GELU + Q4_0 quantize in the GEMM epilogue gives the
    same fp16 operand bits as the GEMM's f32 output through k_act_quant_f16 (ragged M, N)."""
    rng = np.random.default_rng(M + 7 * K + N)
    W16 = (rng.standard_normal((M, K)) * 0.05).astype(np.float16)
    X16 = (rng.standard_normal((N, K)) * 0.5).astype(np.float16)
    b = (rng.standard_normal(M) * 0.1).astype(np.float32)
    w, x, bd = torch.from_numpy(W16).to(DEV), torch.from_numpy(X16).to(DEV), dev(b)
    y = torch.empty(N * M, dtype=torch.float32, device=DEV)
    ref = torch.empty(N * M, dtype=torch.float16, device=DEV)
    got = torch.empty(N * M, dtype=torch.float16, device=DEV)
    L = hip.lib()
    hip.check(L.vsim_op_gemm_f16(w.data_ptr(), M, K, x.data_ptr(), N, None, y.data_ptr(), None), "gemm")
    hip.check(L.vsim_op_act_quant_f16(y.data_ptr(), M, N, bd.data_ptr(), 1, ref.data_ptr(), None), "act")
    hip.check(L.vsim_op_gemm_f16_gelu_q(w.data_ptr(), M, K, x.data_ptr(), N, bd.data_ptr(), got.data_ptr(), None), "gq")
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize("M,K,N", [(520, 512, 300), (256, 64, 256), (1056, 128, 600), (3072, 1024, 512),
                                   (300, 4096, 257), (24576, 64, 2048), (6144, 6144, 2048)])
def test_prefill_gemm_q4_in_lds_dequant_bit_identical(M, K, N):
    """The long-prompt GEMM the model runs (vsim_op_gemm_q4_256: the W4T32 weight's raw blocks
    loaded two K-tiles ahead and dequantized in LDS, no fp16 image) gives the bits of the image
    GEMM (k_w4_expand_f16 + vsim_op_gemm_f16*) for every epilogue: plain (+bias), GELU-quantize,
    GPT-J RoPE, residual join.  Ragged M / N, one and two K-tiles, both tile heights (AP 3 / 4,
    launch_gemm_f16_256's choice), the codegen-16B square shape."""
    rng = np.random.default_rng(5 * M + K + N)
    w_aos = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.05))
    w = repack(w_aos, M, K)
    img = torch.empty(M * K, dtype=torch.float16, device=DEV)
    L = hip.lib()
    hip.check(L.vsim_op_q4_expand_f16(w.data_ptr(), M, K, img.data_ptr(), None), "expand")
    # one pass per tile (a stream-K split sums in another order: test_prefill_gemm_streamk_bound)
    was = L.vsim_gemm_set_streamk(0)
    try:
        _q4_vs_image(L, M, K, N, rng, w, img)
    finally:
        L.vsim_gemm_set_streamk(was)


def _q4_vs_image(L, M, K, N, rng, w, img):
    x = torch.from_numpy((rng.standard_normal((N, K)) * 0.5).astype(np.float16)).to(DEV)
    bd = dev((rng.standard_normal(M) * 0.1).astype(np.float32))

    def both(fn_img, fn_q4, out_dtype=torch.float32, init=None):
        a = torch.empty(N * M, dtype=out_dtype, device=DEV) if init is None else init.clone()
        b = torch.empty(N * M, dtype=out_dtype, device=DEV) if init is None else init.clone()
        hip.check(fn_img(a), "image path")
        hip.check(fn_q4(b), "q4 path")
        torch.cuda.synchronize()
        assert torch.equal(a.view(torch.int32 if out_dtype == torch.float32 else torch.int16),
                           b.view(torch.int32 if out_dtype == torch.float32 else torch.int16))

    xp, wp, ip, bp = x.data_ptr(), w.data_ptr(), img.data_ptr(), bd.data_ptr()
    both(lambda y: L.vsim_op_gemm_f16(ip, M, K, xp, N, bp, y.data_ptr(), None),
         lambda y: L.vsim_op_gemm_q4_256(wp, M, K, xp, N, bp, y.data_ptr(), None, None, 0, 0, 0, 0, None, None))
    if M % 32 == 0:
        both(lambda q: L.vsim_op_gemm_f16_gelu_q(ip, M, K, xp, N, bp, q.data_ptr(), None),
             lambda q: L.vsim_op_gemm_q4_256(wp, M, K, xp, N, bp, None, q.data_ptr(), None, 0, 0, 0, 0, None, None),
             out_dtype=torch.float16)
    if M % 256 == 0:
        d, n_rot, p0 = 256, 64, 3
        half = n_rot // 2
        theta = np.arange(p0 + N, dtype=np.float64)[:, None] * 10000.0 ** (-2.0 * np.arange(half) / n_rot)[None, :]
        cs = dev(np.ascontiguousarray(np.stack([np.cos(theta), np.sin(theta)], axis=-1)))
        both(lambda y: L.vsim_op_gemm_f16_rope(ip, M, K, xp, N, bp, y.data_ptr(), cs.data_ptr(), d, n_rot, p0, None),
             lambda y: L.vsim_op_gemm_q4_256(wp, M, K, xp, N, bp, y.data_ptr(), None, cs.data_ptr(), d, n_rot, p0, 0,
                                             None, None))
    if M % 4 == 0:
        R = dev(rng.standard_normal(N * M).astype(np.float32))
        A = dev(rng.standard_normal(N * M).astype(np.float32))
        both(lambda r: L.vsim_op_gemm_f16_join(ip, M, K, xp, N, bp, r.data_ptr(), A.data_ptr(), None),
             lambda r: L.vsim_op_gemm_q4_256(wp, M, K, xp, N, bp, r.data_ptr(), None, None, 0, 0, 0, 1, A.data_ptr(),
                                             None), init=R)


@pytest.mark.parametrize("M,K,N", [(6144, 6144, 2048), (6144, 4096, 1800), (6144, 24576, 2048), (4096, 4096, 2048),
                                   (4096, 16384, 2048)])
def test_prefill_gemm_streamk_bound(M, K, N):
    """Grids of at least half and fewer than all the CUs (every 6144-row codegen-16B GEMM, GPT-J-6B's
    128 tiles at N = 2048) split each tile's K range
    between two workgroups and add the partial sums once.  Against one pass per tile: the same
    products in another order, so per element |y_sk - y_1| <= 2 K 2^-24 sum_k |w_k x_k| (the
    bound both orders obey); plain and residual-join epilogues, repeated runs bit-identical."""
    rng = np.random.default_rng(M + K + N)
    w = repack(mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.05)), M, K)
    img = torch.empty(M * K, dtype=torch.float16, device=DEV)
    L = hip.lib()
    hip.check(L.vsim_op_q4_expand_f16(w.data_ptr(), M, K, img.data_ptr(), None), "expand")
    x = torch.from_numpy((rng.standard_normal((N, K)) * 0.5).astype(np.float16)).to(DEV)
    bd = dev((rng.standard_normal(M) * 0.1).astype(np.float32))
    res = dev((rng.standard_normal(N * M)).astype(np.float32))
    wp, xp, bp = w.data_ptr(), x.data_ptr(), bd.data_ptr()

    def plain(y):
        return L.vsim_op_gemm_q4_256(wp, M, K, xp, N, bp, y.data_ptr(), None, None, 0, 0, 0, 0, None, None)

    def join(y):
        return L.vsim_op_gemm_q4_256(wp, M, K, xp, N, bp, y.data_ptr(), None, None, 0, 0, 0, 1, None, None)  # y = res

    absprod = (x.float().abs() @ img.view(M, K).float().abs().t()).reshape(-1)
    tol = 2.0 * K * 2.0 ** -24 * absprod
    was = L.vsim_gemm_set_streamk(1)
    try:
        for fn, init in ((plain, None), (join, res)):
            outs = {}
            for sk in (0, 1, 1):
                L.vsim_gemm_set_streamk(sk)
                y = torch.empty(N * M, device=DEV) if init is None else init.clone()
                hip.check(fn(y), "gemm")
                outs.setdefault(sk, []).append(y)
            torch.cuda.synchronize()
            a, b, b2 = outs[0][0], outs[1][0], outs[1][1]
            assert torch.equal(b.view(torch.int32), b2.view(torch.int32)), "stream-K not deterministic"
            err = (a - b).abs()
            assert bool((err <= tol + 1e-30).all()), float((err / (tol + 1e-30)).max())
            assert int((err > 0).sum()) > 0 or K <= 128  # (the split really ran)
    finally:
        L.vsim_gemm_set_streamk(was)


@pytest.mark.parametrize("M,K,N,p0", [(512, 256, 300, 0), (4096, 4096, 2048, 5), (6144, 6144, 2048, 3)])
def test_prefill_gemm_qk_pair(M, K, N, p0):
    """A long GPT-J prompt's Q and K projections as one launch (vsim_op_gemm_q4_256_pair, both
    RoPE epilogues) against two single launches of one pass per tile.  Without the split the
    pair is bit-identical (every shape).  With it, the tiles past whole rounds of the CUs (the
    codegen-16B pair: 384 tiles, the last 128 halved over 256 workgroups, all in the second
    weight) add two partial sums: per element within the split bound 2 K 2^-24 sum_k |w_k x_k|
    of the element and of its RoPE partner, plus one ulp of the rotation; the first weight's
    tiles stay bit-identical; repeated runs are bit-identical."""
    rng = np.random.default_rng(M + K + N + p0)
    ws = [repack(mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.05)), M, K)
          for _ in range(2)]
    x = torch.from_numpy((rng.standard_normal((N, K)) * 0.5).astype(np.float16)).to(DEV)
    d, n_rot = 256, 64
    half = n_rot // 2
    theta = np.arange(p0 + N, dtype=np.float64)[:, None] * 10000.0 ** (-2.0 * np.arange(half) / n_rot)[None, :]
    cs = dev(np.ascontiguousarray(np.stack([np.cos(theta), np.sin(theta)], axis=-1)))
    L = hip.lib()
    xp, cp = x.data_ptr(), cs.data_ptr()

    def single(w):
        y = torch.empty(N * M, device=DEV)
        hip.check(L.vsim_op_gemm_q4_256(w.data_ptr(), M, K, xp, N, None, y.data_ptr(), None, cp, d, n_rot, p0, 0,
                                        None, None), "single")
        return y

    def pair():
        y0, y1 = torch.empty(N * M, device=DEV), torch.empty(N * M, device=DEV)
        hip.check(L.vsim_op_gemm_q4_256_pair(ws[0].data_ptr(), ws[1].data_ptr(), M, K, xp, N, y0.data_ptr(),
                                             y1.data_ptr(), cp, d, n_rot, p0, None), "pair")
        return y0, y1

    was = L.vsim_gemm_set_streamk(0)
    try:
        ref = [single(w) for w in ws]
        p0_, p1_ = pair()
        torch.cuda.synchronize()
        assert torch.equal(p0_.view(torch.int32), ref[0].view(torch.int32))
        assert torch.equal(p1_.view(torch.int32), ref[1].view(torch.int32))
        L.vsim_gemm_set_streamk(1)
        mode = L.vsim_gemm_set_qk_pair(2)  # (paired, whole tiles only: bit-identical with the split allowed)
        try:
            c0, c1 = pair()
        finally:
            L.vsim_gemm_set_qk_pair(mode)
        (a0, a1), (b0, b1) = pair(), pair()
        torch.cuda.synchronize()
        assert torch.equal(c0.view(torch.int32), ref[0].view(torch.int32))
        assert torch.equal(c1.view(torch.int32), ref[1].view(torch.int32))
    finally:
        L.vsim_gemm_set_streamk(was)
    assert torch.equal(a0.view(torch.int32), b0.view(torch.int32)) and torch.equal(a1.view(torch.int32),
                                                                                      b1.view(torch.int32))
    assert torch.equal(a0.view(torch.int32), ref[0].view(torch.int32))
    img = torch.empty(M * K, dtype=torch.float16, device=DEV)
    hip.check(L.vsim_op_q4_expand_f16(ws[1].data_ptr(), M, K, img.data_ptr(), None), "expand")
    torch.cuda.synchronize()
    absprod = (x.float().abs() @ img.view(M, K).float().abs().t())  # [N][M]
    tol = 2.0 * K * 2.0 ** -24 * absprod
    col = torch.arange(M, device=DEV)
    partner = torch.where(col % d < n_rot, col ^ 1, col)  # GPT-J RoPE rotates adjacent pairs
    tol = (tol + tol[:, partner]).reshape(-1) + 2.0 ** -23 * ref[1].abs()
    err = (a1 - ref[1]).abs()
    assert bool((err <= tol + 1e-30).all()), float((err / (tol + 1e-30)).max())
    if M * 2 // 256 * ((N + 255) // 256) > 256:
        assert int((err > 0).sum()) > 0  # (the split really ran)


def _q4_f16_ref(y):
    """quantize_row_q4_0 (ggml.c:209-251) per 32-block of the f32 rows y, the values d*(q-8)
    rounded once to fp16 (the prompt GEMMs' operand)."""
    b = y.reshape(-1, 32).astype(np.float32)
    amax = np.abs(b).max(axis=1).astype(np.float32)
    d = (amax / np.float32(7.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    t = (b * idv[:, None]).astype(np.float32)
    q = np.where(t >= 0, np.floor(t + 0.5), -np.floor(-t + 0.5))  # round half away from zero
    return (d[:, None].astype(np.float64) * q).astype(np.float16).reshape(y.shape)


@pytest.mark.parametrize("k,rows", [(6144, 300), (4096, 257), (1024, 64), (5120, 33), (2080, 20)])
def test_prompt_norm_f16q(k, rows):
    """The fast-mode prompt LayerNorm + affine straight to the fp16 GEMM operand (one wave per row
    for k % 256 == 0, the workgroup kernel otherwise) against numpy: the norm in double with the
    reference's float steps, then quantize_row_q4_0 per block.  The double sums run in another
    order, so a value may move by one quantization step where a rounding lands on a boundary:
    nearly all values bit-equal, none off by more than a step."""
    rng = np.random.default_rng(k + rows)
    x = (rng.standard_normal((rows, k)) * 2.0 + 0.3).astype(np.float32)
    w = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float32)
    b = (0.1 * rng.standard_normal(k)).astype(np.float32)
    out = torch.empty(rows * k, dtype=torch.float16, device=DEV)
    xg, wg, bg = dev(x), dev(w), dev(b)  # (held: a temporary's memory could be reused before the launch)
    hip.check(hip.lib().vsim_op_norm_f16q(xg.data_ptr(), k, rows, wg.data_ptr(), bg.data_ptr(), out.data_ptr(), None),
              "norm_f16q")
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(rows, k)
    xd = x.astype(np.float64)
    mean = xd.sum(axis=1, keepdims=True) / k
    var = ((xd - mean) ** 2).sum(axis=1, keepdims=True) / k
    scale = (1.0 / np.sqrt(var + np.float64(np.float32(1e-5)))).astype(np.float32)
    y = ((xd - mean).astype(np.float32) * scale).astype(np.float32)
    y = (w[None, :] * y).astype(np.float32) + b[None, :]
    want = _q4_f16_ref(y.astype(np.float32))
    step = (np.abs(y.reshape(-1, 32)).max(axis=1) / 7.0).repeat(32).reshape(rows, k)
    diff = np.abs(got.astype(np.float64) - want.astype(np.float64))
    assert float((diff > 0).mean()) < 1e-3
    assert bool((diff <= step * 1.001 + 1e-6).all())


@pytest.mark.parametrize("H,N,n_past", [(2, 200, 0), (3, 300, 37), (1, 64, 130)])
def test_attn_prefill_quantized_output_bit_identical(H, N, n_past):
    """d = 256: the attention writing the out-projection's fp16 operand itself
    (vsim_op_attn_prefill_q16) gives the bits vsim_op_act_quant_f16 makes of its f32 output."""
    d = 256
    rng = np.random.default_rng(7 * N + n_past)
    E, nk = d * H, n_past + N
    q_, k_, v_ = (dev(rng.standard_normal((n, E)).astype(np.float32)) for n in (N, nk, nk))
    scale = float(np.float32(1.0 / np.sqrt(d)))
    L = hip.lib()
    out = torch.empty(N * E, dtype=torch.float32, device=DEV)
    hip.check(L.vsim_op_attn_prefill(q_.data_ptr(), k_.data_ptr(), v_.data_ptr(), d, H, N, n_past, scale,
                                     out.data_ptr(), None), "attn")
    ref16 = torch.empty(N * E, dtype=torch.float16, device=DEV)
    hip.check(L.vsim_op_act_quant_f16(out.data_ptr(), E, N, None, 0, ref16.data_ptr(), None), "act_quant")
    got16 = torch.full((N * E,), float("nan"), dtype=torch.float16, device=DEV)
    hip.check(L.vsim_op_attn_prefill_q16(q_.data_ptr(), k_.data_ptr(), v_.data_ptr(), d, H, N, n_past, scale,
                                         got16.data_ptr(), None), "attn_q16")
    torch.cuda.synchronize()
    assert torch.equal(got16.view(torch.int16), ref16.view(torch.int16))


@pytest.mark.parametrize("d,H,N,n_past", [(256, 2, 200, 0), (256, 3, 300, 37), (256, 1, 64, 130), (256, 2, 1100, 40),
                                           (128, 3, 130, 17), (96, 2, 64, 5), (64, 4, 9, 40)])
def test_attn_prefill_f16(d, H, N, n_past):
    """Fast-mode prompt attention (attn_prefill.hip; d = 256 on the two-waves-per-group kernel)
    against fp64 causal attention: scores and probabilities pass through fp16, so the tolerance
    is 2e-2 of max|V| (the observed error is ~1e-3).  Ragged N, a cache before the prompt."""
    rng = np.random.default_rng(d + N + n_past)
    E, nk = d * H, n_past + N
    Q = rng.standard_normal((N, E)).astype(np.float32)
    K = rng.standard_normal((nk, E)).astype(np.float32)
    V = rng.standard_normal((nk, E)).astype(np.float32)
    scale = float(np.float32(1.0 / np.sqrt(d)))
    out = torch.empty(N * E, dtype=torch.float32, device=DEV)
    q_, k_, v_ = dev(Q), dev(K), dev(V)
    hip.check(hip.lib().vsim_op_attn_prefill(q_.data_ptr(), k_.data_ptr(), v_.data_ptr(), d, H, N, n_past, scale,
                                             out.data_ptr(), None), "attn_prefill")
    y = host(out).reshape(N, E)
    ref = np.empty((N, E))
    for h in range(H):
        sl = slice(h * d, (h + 1) * d)
        s = (Q[:, sl].astype(np.float64) @ K[:, sl].astype(np.float64).T) * scale
        mask = np.arange(nk)[None, :] > (n_past + np.arange(N))[:, None]
        s[mask] = -np.inf
        p = np.exp(s - s.max(axis=1, keepdims=True))
        p /= p.sum(axis=1, keepdims=True)
        ref[:, sl] = p @ V[:, sl].astype(np.float64)
    assert np.max(np.abs(y - ref)) <= 2e-2 * np.max(np.abs(V))
