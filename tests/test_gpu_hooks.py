"""The vsim_ggml_* hooks (include/vsim_hip.h): host ggml_tensors in, host ggml_tensors out,
called the way the reference's thread pool would call them - every thread, every phase.
Checked bit-for-bit against the reference's own op outputs (tests/golden/ops_*.npz from
oracle/ref_harness at --threads 1) and, for the KQV product at nth > 1, against the
reference's thread grouping restated in numpy (ggml.c:4535-4581 partials summed in thread
order by FINALIZE, ggml.c:4469-4493).
"""
import ctypes

import numpy as np
import pytest

from golden_util import cases, ops
from vsim_amd import hip

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def params(ith=0, nth=1, typ=hip.GGML_TASK_COMPUTE):
    p = hip.GgmlComputeParams()
    p.type, p.ith, p.nth = typ, ith, nth
    return p


def call_all_threads(fn, nth, *tensors):
    """Every phase on every thread, as ggml_graph_compute does: all return codes."""
    rcs = []
    for typ in (hip.GGML_TASK_INIT, hip.GGML_TASK_COMPUTE, hip.GGML_TASK_FINALIZE):
        for ith in range(nth):
            rcs.append(fn(ctypes.byref(params(ith, nth, typ)), *[ctypes.byref(t) for t in tensors]))
    return rcs


@pytest.mark.parametrize("style", [0, 1], ids=["neox", "gptj"])
def test_rope_hook_bit_exact(style):
    L = hip.lib()
    fn = L.vsim_ggml_gptneox_rope_f32 if style == 0 else L.vsim_ggml_rope_f32
    for c in cases(ops("rope_neox" if style == 0 else "rope_gptj")):
        d, H, T, n_past, n_dims, mode = (int(v) for v in c["shape"])
        x = np.array(c["x"], np.float32)
        pr = np.array([n_past, n_dims, mode], np.int32)
        t = hip.ggml_f32(x, [d, H, T])
        tp = hip.ggml_f32(pr, [3], typ=hip.GGML_TYPE_I32)
        assert call_all_threads(fn, 3, t, tp, t) == [0] * 9
        assert np.array_equal(bits(x), bits(c["y"])), c["shape"]


def test_softmax_hook_bit_exact():
    """scale and diag_mask_inf are nodes of their own before soft_max (vsim.cpp:586-594):
    applied here in float32 as the reference does, then the hook's soft_max."""
    fn = hip.lib().vsim_ggml_soft_max_f32
    for c in cases(ops("attnsm")):
        nc, nr, nz, n_past = (int(v) for v in c["shape"])
        x = (np.array(c["x"], np.float32) * np.float32(c["scale"][0])).reshape(nz, nr, nc)
        for j in range(nr):
            for i in range(n_past, nc):
                if i > n_past + j:
                    x[:, j, i] = -np.inf
        x = np.ascontiguousarray(x.reshape(-1))
        t = hip.ggml_f32(x, [nc, nr, nz])
        assert call_all_threads(fn, 2, t, t) == [0] * 6
        assert np.array_equal(bits(x), bits(c["y"])), c["shape"]


def kq_tensors(c):
    d, H, nk, N = (int(v) for v in c["shape"])
    E = d * H
    K, Q = np.array(c["a"], np.float32), np.array(c["b"], np.float32)
    out = np.zeros(nk * N * H, np.float32)
    # the permuted views of vsim.cpp:562-583: K [d, nk, H] and Q [d, N, H] over [pos][E] rows
    tk = hip.ggml_f32(K, [d, nk, H], [4, 4 * E, 4 * d])
    tq = hip.ggml_f32(Q, [d, N, H], [4, 4 * E, 4 * d])
    to = hip.ggml_f32(out, [nk, N, H])
    return (K, Q, out), (tk, tq, to)


def kqv_tensors(c):
    d, H, nk, N = (int(v) for v in c["shape"])
    E = d * H
    V, S = np.array(c["a"], np.float32), np.array(c["b"], np.float32)
    out = np.zeros(d * N * H, np.float32)
    # V_trans = permute(reshape(view(memory_v)), 1, 2, 0, 3) (vsim.cpp:596-603): [nk, d, H]
    tv = hip.ggml_f32(V, [nk, d, H], [4 * E, 4, 4 * d])
    ts = hip.ggml_f32(S, [nk, N, H])
    to = hip.ggml_f32(out, [d, N, H])
    return (V, S, out), (tv, ts, to)


def test_mul_mat_f32_hook_kq_bit_exact():
    fn = hip.lib().vsim_ggml_mul_mat_f32
    for c in cases(ops("kq")):
        arrays, ts = kq_tensors(c)  # `arrays` keeps the host buffers the tensors point at alive
        out = arrays[2]
        assert call_all_threads(fn, 4, *ts) == [0] * 12
        assert np.array_equal(bits(out), bits(c["y"])), c["shape"]


def kqv_reference(V, S, d, H, nk, N, nth):
    """ggml.c:4535-4581 + 4469-4493 restated: thread t mads columns [t*dc, min(t*dc+dc, nk))
    sequentially in float32 from 0; FINALIZE adds the partials in thread order."""
    E = d * H
    Vr = V.reshape(-1, E)[:nk]                   # [k][E]
    Sr = S.reshape(H, N, nk)                     # [h][q][k]
    out = np.zeros((H, N, d), np.float32)
    dc = (nk + nth - 1) // nth
    for t in range(nth):
        part = np.zeros((H, N, d), np.float32)
        for ic in range(dc * t, min(dc * t + dc, nk)):
            v = Vr[ic].reshape(H, 1, d)
            s = Sr[:, :, ic].reshape(H, N, 1)
            part = (part + (v * s).astype(np.float32)).astype(np.float32)
        out = part if t == 0 else (out + part).astype(np.float32)
    return out.reshape(-1)


@pytest.mark.parametrize("nth", [1, 3, 4, 7])
def test_mul_mat_f32_hook_kqv_thread_grouping(nth):
    fn = hip.lib().vsim_ggml_mul_mat_f32
    for c in cases(ops("kqv")):
        d, H, nk, N = (int(v) for v in c["shape"])
        (V, S, out), ts = kqv_tensors(c)
        assert call_all_threads(fn, nth, *ts) == [0] * (3 * nth)
        if nth == 1:
            assert np.array_equal(bits(out), bits(c["y"])), c["shape"]
        assert np.array_equal(bits(out), bits(kqv_reference(V, S, d, H, nk, N, nth))), (c["shape"], nth)


def test_hooks_refuse_consistently():
    """A layout the hook cannot take: every thread and phase gets VSIM_EINVAL (so every thread
    falls back to its own CPU slice) and the tensor is untouched."""
    L = hip.lib()
    x = np.arange(64, dtype=np.float32)
    before = x.copy()
    t = hip.ggml_f32(x, [8, 4], [4, 64])  # rows 64 bytes apart over 8 floats: not contiguous
    rcs = call_all_threads(L.vsim_ggml_soft_max_f32, 4, t, t)
    assert rcs == [-1] * 12
    assert np.array_equal(x, before)
