"""ctypes view of oracle/_build/libvsim_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB_PATH = os.path.join(ROOT, "oracle", "_build", "libvsim_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "port"], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB_PATH)
        vp, ci, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.vo_model_load.restype = vp
        L.vo_model_load.argtypes = [ctypes.c_char_p, ci, ci]
        L.vo_model_eval.argtypes = [vp, ci, vp, ci, vp, ci]
        L.vo_model_synthetic.restype = vp
        L.vo_model_synthetic.argtypes = [ci, ci, ci, ci, ci, ci, ci, ctypes.c_uint64, cf]
        L.vo_model_create.restype = vp
        L.vo_model_create.argtypes = [ci, ci, ci, ci, ci, ci, ci, ci]
        L.vo_model_set_tensor.argtypes = [vp, ctypes.c_char_p, vp, ctypes.c_size_t]
        L.vo_model_hparams.argtypes = [vp, vp]
        L.vo_model_free.argtypes = [vp]
        L.vo_generate.argtypes = [vp, vp, ci, ci, ci, ci, cf, cf, ci, cf, ci, vp, ci, ci]
        L.vo_quantize_row_q4_0.argtypes = [vp, vp, ci]
        L.vo_mul_mat_q4_0_f32.argtypes = [vp, ci, ci, vp, ci, vp, ci]
        L.vo_mul_mat_q4_0_q.argtypes = [vp, ci, ci, vp, ci, vp, ci]
        L.vo_norm_f32.argtypes = [vp, vp, ci, ci]
        L.vo_gelu_f32.argtypes = [vp, vp, ci]
        L.vo_soft_max_f32.argtypes = [vp, ci, ci]
        L.vo_scale_f32.argtypes = [vp, ci, cf]
        L.vo_diag_mask_inf_f32.argtypes = [vp, ci, ci, ci, ci]
        L.vo_alibi_f32.argtypes = [vp, ci, ci, ci, ci]
        L.vo_rope_neox.argtypes = [vp, ci, ci, ci, ci, ci, ci]
        L.vo_rope_gptj.argtypes = [vp, ci, ci, ci, ci, ci, ci]
        L.vo_kq.argtypes = [vp, ci, vp, ci, ci, ci, ci, ci, vp]
        L.vo_kqv.argtypes = [vp, ci, vp, ci, ci, ci, ci, vp]
        L.vo_get_rows_q4_0.argtypes = [vp, ci, vp, ci, vp]
        L.vo_tables.argtypes = [vp, vp]
        L.vo_init_tables()
        _lib = L
    return _lib


def p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def quantize(x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros(x.size // 32 * 20, np.uint8)
    lib().vo_quantize_row_q4_0(p(x), p(y), x.size)
    return y


def mul_mat(w, M, K, x, N, nthreads=1):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros(M * N, np.float32)
    lib().vo_mul_mat_q4_0_f32(p(w), M, K, p(x), N, p(y), nthreads)
    return y


def mul_mat_q(w, M, K, xq, N, nthreads=1):
    y = np.zeros(M * N, np.float32)
    lib().vo_mul_mat_q4_0_q(p(w), M, K, p(xq), N, p(y), nthreads)
    return y


def norm(x, n, rows):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().vo_norm_f32(p(x), p(y), n, rows)
    return y


def gelu(x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().vo_gelu_f32(p(x), p(y), x.size)
    return y


def attn_softmax(x, nc, nr, nz, n_past, scale):
    y = np.array(x, np.float32, copy=True)
    lib().vo_scale_f32(p(y), y.size, ctypes.c_float(scale))
    lib().vo_diag_mask_inf_f32(p(y), nc, nr, nz, n_past)
    lib().vo_soft_max_f32(p(y), nc, nr * nz)
    return y


def attn_softmax_alibi(x, nc, nr, nz, n_past, n_head, scale):
    """scale -> ggml_alibi -> diag_mask_inf -> soft_max (the BLOOM score path)."""
    y = np.ascontiguousarray(x, np.float32).copy()
    L = lib()
    L.vo_scale_f32(p(y), y.size, scale)
    L.vo_alibi_f32(p(y), nc, nr, nz, n_head)
    L.vo_diag_mask_inf_f32(p(y), nc, nr, nz, n_past)
    L.vo_soft_max_f32(p(y), nc, nr * nz)
    return y


def rope(style, x, d, H, T, n_past, n_dims, mode):
    y = np.array(x, np.float32, copy=True)
    fn = lib().vo_rope_neox if style == "neox" else lib().vo_rope_gptj
    fn(p(y), d, H, T, n_past, n_dims, mode)
    return y


def kq(K, Q, d, H, nk, N):
    out = np.zeros(H * N * nk, np.float32)
    lib().vo_kq(p(np.ascontiguousarray(K, np.float32)), d * H, p(np.ascontiguousarray(Q, np.float32)), d * H,
                d, H, nk, N, p(out))
    return out


def kqv(V, S, d, H, nk, N):
    out = np.zeros(H * N * d, np.float32)
    lib().vo_kqv(p(np.ascontiguousarray(V, np.float32)), d * H, p(np.ascontiguousarray(S, np.float32)),
                 d, H, nk, N, p(out))
    return out


def get_rows(w, K, idx):
    idx = np.ascontiguousarray(idx, np.int32)
    y = np.zeros(idx.size * K, np.float32)
    lib().vo_get_rows_q4_0(p(w), K, p(idx), idx.size, p(y))
    return y


def tables():
    e = np.zeros(65536, np.uint16)
    g = np.zeros(65536, np.uint16)
    lib().vo_tables(p(e), p(g))
    return e, g


class Model:
    def __init__(self, path, arch: int, n_ctx: int = 512, synthetic=None):
        if synthetic is not None:  # (n_vocab, n_embd, n_head, n_layer, n_rot, seed, std)
            nv, ne, nh, nl, nr, seed, std = synthetic
            self.h = lib().vo_model_synthetic(arch, nv, ne, nh, nl, nr, n_ctx, seed, std)
        else:
            self.h = lib().vo_model_load(path.encode(), arch, n_ctx)
        if not self.h:
            raise RuntimeError(f"oracle could not load {path}")
        hp = np.zeros(8, np.int32)
        lib().vo_model_hparams(self.h, p(hp))
        self.n_vocab, self.n_embd, self.n_head, self.n_layer, self.n_rot = (int(v) for v in hp[:5])

    @classmethod
    def from_device(cls, dm, arch_s: str, n_ctx: int = 512):
        """An oracle model holding exactly the weights of the device model `dm` (read back
        through vsim_model_get_tensor, i.e. unpacked from the device layout)."""
        import sys
        sys.path.insert(0, ROOT)
        from vsim_amd import modelgen as mg
        hp = dm.hp
        self = cls.__new__(cls)
        arch = {"gptneox": 0, "gptj": 1, "bloom": 2}[arch_s]
        self.h = lib().vo_model_create(arch, hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot,
                                       hp.use_parallel_residual, n_ctx)
        mhp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, hp.use_parallel_residual)
        for name, ne, kind in mg.tensor_specs(arch_s, mhp):
            n = int(np.prod(ne))
            nbytes = n // 32 * 20 if kind == "q" else 4 * n
            buf = dm.get_tensor(name, nbytes)
            if lib().vo_model_set_tensor(self.h, name.encode(), p(buf), nbytes) != 0:
                raise RuntimeError(f"oracle set_tensor {name}")
        self.n_vocab, self.n_embd, self.n_head, self.n_layer, self.n_rot = (
            hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot)
        return self

    def eval(self, n_past, tokens, nthreads=1):
        t = np.ascontiguousarray(tokens, np.int32)
        lg = np.zeros(self.n_vocab, np.float32)
        rc = lib().vo_model_eval(self.h, n_past, p(t), t.size, p(lg), nthreads)
        if rc != 0:
            raise RuntimeError("oracle eval failed")
        return lg

    def generate(self, prompt, n_predict, seed=42, top_k=40, top_p=0.95, temp=0.8, repeat_last_n=64,
                 repeat_penalty=1.3, n_batch=8, nthreads=1):
        pr = np.ascontiguousarray(prompt, np.int32)
        out = np.zeros(4096, np.int32)
        n = lib().vo_generate(self.h, p(pr), pr.size, n_predict, seed, top_k, top_p, temp, repeat_last_n,
                              repeat_penalty, n_batch, p(out), out.size, nthreads)
        return [int(v) for v in out[:n]]

    def __del__(self):
        if getattr(self, "h", None):
            lib().vo_model_free(self.h)
            self.h = None
