"""ctypes binding of libvsim_hip.so (include/vsim_hip.h).

The HIP library is the product; this module only marshals arguments.  There is no
CPU fallback: if the library is missing or a call fails, an exception is raised.
Device buffers are torch tensors on a ROCm device (torch is plumbing here: memory and
streams), passed to the C-ABI as raw pointers.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VSIM_LIB") or os.path.join(HERE, "_build", "libvsim_hip.so")  # VSIM_LIB: A/B builds

MODE_EXACT = 0
MODE_FAST = 1
ARCH_GPTNEOX = 0
ARCH_GPTJ = 1
ARCH_BLOOM = 2

# symbols declared in include/vsim_hip.h (checked by tests/test_capi.py)
EXPORTS = [
    "vsim_last_error", "vsim_device_count", "vsim_q4_bytes",
    "init_xmax", "imax_ggml_compute_forward_mul_mat_q4_0_f32",
    "vsim_ggml_gptneox_rope_f32", "vsim_ggml_rope_f32", "vsim_ggml_soft_max_f32", "vsim_ggml_mul_mat_f32",
    "vsim_dropin_stats", "vsim_dropin_reset", "vsim_norm_fallbacks", "vsim_spin_timeouts",
    "vsim_op_q4_repack", "vsim_op_q4_unpack", "vsim_op_act_repack", "vsim_op_act_unpack",
    "vsim_op_q4_quantize", "vsim_op_q4_gemv", "vsim_op_q4_expand_f16", "vsim_op_gemm_f16",
    "vsim_op_act_quant_f16", "vsim_op_gemm_f16_gelu_q", "vsim_op_gemm_f16_rope", "vsim_op_gemm_f16_join",
    "vsim_op_gemm_q4_256", "vsim_op_get_rows",
    "vsim_op_norm", "vsim_op_gelu", "vsim_op_argmax", "vsim_op_attn_softmax", "vsim_op_rope", "vsim_op_kq", "vsim_op_kqv", "vsim_op_kq_causal", "vsim_op_kqv_causal",
    "vsim_op_attn_prefill", "vsim_op_attn_prefill_q16", "vsim_gemm_set_streamk", "vsim_gemm_set_qk_pair", "vsim_gemm_set_tile_order", "vsim_op_gemm_q4_256_pair", "vsim_op_norm_f16q",
    "vsim_op_tables",
    "vsim_model_create", "vsim_model_load_file", "vsim_model_set_tensor", "vsim_model_get_tensor",
    "vsim_model_randomize",
    "vsim_model_set_mode", "vsim_model_reserve", "vsim_model_hparams", "vsim_model_eval", "vsim_model_eval_argmax", "vsim_model_generate",
    "vsim_model_stream",
    "vsim_model_logits_dev", "vsim_model_info", "vsim_model_set_graph", "vsim_model_set_profile",
    "vsim_model_profile_kernel", "vsim_model_profile_stats", "vsim_model_free",
    "vsim_graph_compute", "vsim_graph_compute_rc", "vsim_graph_sync_tensor", "vsim_graph_reset", "vsim_graph_stats",
    "vsim_graph_set_profile", "vsim_graph_profile_report", "vsim_graph_match", "vsim_graph_fast_stats",
    "vsim_model_stage_bind", "vsim_model_stage_begin", "vsim_model_stage_step", "vsim_model_sync",
    "vsim_model_debug_poison",
]

_lib = None


class VsimError(RuntimeError):
    pass


# ggml ABI mirrors (include/ggml_abi.h; offsets checked against the reference's ggml.h by
# tests/test_capi.py): for callers that hand host tensors to the drop-in hooks.
GGML_TYPE_Q4_0, GGML_TYPE_I32, GGML_TYPE_F32 = 0, 4, 6
GGML_TASK_INIT, GGML_TASK_COMPUTE, GGML_TASK_FINALIZE = 0, 1, 2


class GgmlTensor(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("n_dims", ctypes.c_int), ("ne", ctypes.c_int * 4),
                ("nb", ctypes.c_size_t * 4), ("op", ctypes.c_int), ("is_param", ctypes.c_bool),
                ("grad", ctypes.c_void_p), ("src0", ctypes.c_void_p), ("src1", ctypes.c_void_p),
                ("opt", ctypes.c_void_p * 4), ("n_tasks", ctypes.c_int), ("perf_runs", ctypes.c_int),
                ("perf_cycles", ctypes.c_int64), ("perf_time_us", ctypes.c_int64), ("data", ctypes.c_void_p),
                ("padding", ctypes.c_char * 8)]


class GgmlComputeParams(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("ith", ctypes.c_int), ("nth", ctypes.c_int), ("wsize", ctypes.c_size_t),
                ("wdata", ctypes.c_void_p)]


def ggml_f32(buf, ne, nb=None, typ=GGML_TYPE_F32):
    """A host ggml_tensor over numpy array `buf` (kept alive by the caller) with shape ne and
    byte strides nb (contiguous when None)."""
    ne = list(ne) + [1] * (4 - len(ne))
    nb = [4] if nb is None else list(nb)
    while len(nb) < 4:  # the missing outer strides as ggml sets them: nb[i] = nb[i-1] * ne[i-1]
        nb.append(nb[-1] * ne[len(nb) - 1])
    t = GgmlTensor()
    t.type = typ
    t.n_dims = 4
    for i in range(4):
        t.ne[i] = ne[i]
        t.nb[i] = nb[i]
    t.data = buf.ctypes.data
    return t


class HParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("n_vocab", "n_embd", "n_head", "n_layer", "n_rot", "use_parallel_residual")]


def lib():
    """Load libvsim_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VsimError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, ci, cf, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    L.vsim_last_error.restype = ctypes.c_char_p
    L.vsim_q4_bytes.restype = sz
    L.vsim_q4_bytes.argtypes = [ci, ci]
    L.vsim_op_q4_repack.argtypes = [vp, vp, ci, ci, vp]
    L.vsim_op_q4_unpack.argtypes = [vp, vp, ci, ci, vp]
    L.vsim_op_act_repack.argtypes = [vp, vp, ci, ci, vp]
    L.vsim_op_act_unpack.argtypes = [vp, vp, ci, ci, vp]
    L.vsim_op_q4_quantize.argtypes = [vp, ci, ci, vp, vp, vp]
    L.vsim_op_q4_gemv.argtypes = [vp, ci, ci, vp, vp, ci, vp, vp, ci, vp]
    L.vsim_op_get_rows.argtypes = [vp, ci, ci, vp, ci, vp, vp]
    L.vsim_op_q4_expand_f16.argtypes = [vp, ci, ci, vp, vp]
    L.vsim_op_gemm_f16.argtypes = [vp, ci, ci, vp, ci, vp, vp, vp]
    L.vsim_op_act_quant_f16.argtypes = [vp, ci, ci, vp, ci, vp, vp]
    L.vsim_op_gemm_f16_gelu_q.argtypes = [vp, ci, ci, vp, ci, vp, vp, vp]
    L.vsim_op_gemm_f16_rope.argtypes = [vp, ci, ci, vp, ci, vp, vp, vp, ci, ci, ci, vp]
    L.vsim_op_gemm_f16_join.argtypes = [vp, ci, ci, vp, ci, vp, vp, vp, vp]
    L.vsim_op_gemm_q4_256.argtypes = [vp, ci, ci, vp, ci, vp, vp, vp, vp, ci, ci, ci, ci, vp, vp]
    L.vsim_op_norm.argtypes = [vp, vp, ci, ci, vp, vp, vp]
    L.vsim_op_gelu.argtypes = [vp, vp, ci, vp]
    L.vsim_op_argmax.argtypes = [vp, ci, vp, vp]
    L.vsim_op_attn_softmax.argtypes = [vp, ci, ci, ci, ci, cf, vp]
    L.vsim_op_rope.argtypes = [ci, vp, ci, ci, ci, ci, ci, ci, vp]
    L.vsim_op_kq.argtypes = [vp, ci, vp, ci, ci, ci, ci, ci, vp, vp]
    L.vsim_op_kqv.argtypes = [vp, ci, vp, ci, ci, ci, ci, vp, vp]
    L.vsim_op_kq_causal.argtypes = [vp, ci, vp, ci, ci, ci, ci, ci, ci, vp, vp]
    L.vsim_op_kqv_causal.argtypes = [vp, ci, vp, ci, ci, ci, ci, ci, vp, vp]
    L.vsim_op_attn_prefill.argtypes = [vp, vp, vp, ci, ci, ci, ci, cf, vp, vp]
    L.vsim_op_attn_prefill_q16.argtypes = [vp, vp, vp, ci, ci, ci, ci, cf, vp, vp]
    L.vsim_gemm_set_streamk.argtypes = [ci]
    L.vsim_gemm_set_qk_pair.argtypes = [ci]
    L.vsim_gemm_set_tile_order.argtypes = [ci]
    L.vsim_op_gemm_q4_256_pair.argtypes = [vp, vp, ci, ci, vp, ci, vp, vp, vp, ci, ci, ci, vp]
    L.vsim_op_norm_f16q.argtypes = [vp, ci, ci, vp, vp, vp, vp]
    L.vsim_op_tables.argtypes = [vp, vp]
    L.vsim_model_create.argtypes = [ci, ctypes.POINTER(HParams), ci, ci, ci, ci, ctypes.POINTER(vp)]
    L.vsim_model_load_file.argtypes = [ctypes.c_char_p, ci, ci, ci, ci, ci, ctypes.POINTER(vp)]
    L.vsim_model_set_tensor.argtypes = [vp, ctypes.c_char_p, vp, sz]
    L.vsim_model_get_tensor.argtypes = [vp, ctypes.c_char_p, vp, sz]
    L.vsim_model_randomize.argtypes = [vp, ctypes.c_uint64, cf]
    L.vsim_model_set_mode.argtypes = [vp, ci]
    L.vsim_model_reserve.argtypes = [vp, ci]
    L.vsim_model_set_graph.argtypes = [vp, ci]
    L.vsim_model_hparams.argtypes = [vp, ctypes.POINTER(HParams), ctypes.POINTER(ci), ctypes.POINTER(ci),
                                     ctypes.POINTER(ci)]
    L.vsim_model_eval.argtypes = [vp, ci, vp, ci, vp, vp, vp]
    L.vsim_model_eval_argmax.argtypes = [vp, ci, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
    L.vsim_model_generate.argtypes = [vp, ci, ctypes.c_int32, ci, ctypes.POINTER(ctypes.c_int32)]
    L.vsim_model_stream.restype = vp
    L.vsim_model_stream.argtypes = [vp]
    L.vsim_model_logits_dev.restype = vp
    L.vsim_model_logits_dev.argtypes = [vp]
    L.vsim_model_info.argtypes = [vp, ctypes.POINTER(ci), ctypes.POINTER(ci), ctypes.POINTER(sz)]
    L.vsim_model_free.argtypes = [vp]
    L.vsim_model_set_profile.argtypes = [vp, ci]
    L.vsim_model_profile_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long),
                                           ctypes.POINTER(ctypes.c_double)]
    L.vsim_model_profile_kernel.argtypes = [vp, ci, ctypes.c_char_p, ci, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_double)]
    L.vsim_dropin_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
    tp, pp = ctypes.POINTER(GgmlTensor), ctypes.POINTER(GgmlComputeParams)
    L.vsim_ggml_gptneox_rope_f32.argtypes = [pp, tp, tp, tp]
    L.vsim_ggml_rope_f32.argtypes = [pp, tp, tp, tp]
    L.vsim_ggml_soft_max_f32.argtypes = [pp, tp, tp]
    L.vsim_ggml_mul_mat_f32.argtypes = [pp, tp, tp, tp]
    L.vsim_graph_compute_rc.argtypes = [vp, vp]
    L.vsim_model_stage_bind.argtypes = [vp, vp, vp, vp, vp]
    L.vsim_model_stage_begin.argtypes = [vp, ci]
    L.vsim_model_stage_step.argtypes = [vp]
    L.vsim_model_sync.argtypes = [vp]
    L.vsim_model_debug_poison.argtypes = [vp, ci]
    L.vsim_graph_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
    L.vsim_graph_set_profile.argtypes = [ci]
    L.vsim_graph_profile_report.argtypes = [ctypes.c_char_p, sz]
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().vsim_last_error().decode(errors="replace")
        raise VsimError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int:
    """Raw pointer of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def q4_bytes(rows: int, k: int) -> int:
    return int(lib().vsim_q4_bytes(rows, k))


class Model:
    """Device-resident model executor (vsim_model_* in include/vsim_hip.h)."""

    def __init__(self, handle, arch):
        self.h = handle
        self.arch = arch
        hp = HParams()
        n_ctx, lb, le = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().vsim_model_hparams(self.h, ctypes.byref(hp), ctypes.byref(n_ctx), ctypes.byref(lb),
                                       ctypes.byref(le)), "hparams")
        self.hp = hp
        self.n_ctx = n_ctx.value
        self.layer_begin, self.layer_end = lb.value, le.value
        self.n_vocab, self.n_embd = hp.n_vocab, hp.n_embd
        self.first = self.layer_begin == 0
        self.last = self.layer_end == hp.n_layer

    @classmethod
    def load(cls, path, arch, n_ctx=512, device=0, layer_begin=0, layer_end=-1):
        h = ctypes.c_void_p()
        check(lib().vsim_model_load_file(path.encode(), arch, n_ctx, device, layer_begin, layer_end,
                                         ctypes.byref(h)), f"load {path}")
        return cls(h, arch)

    @classmethod
    def create(cls, arch, hp: dict, n_ctx=512, device=0, layer_begin=0, layer_end=-1):
        h = ctypes.c_void_p()
        c = HParams(**hp)
        check(lib().vsim_model_create(arch, ctypes.byref(c), n_ctx, device, layer_begin, layer_end,
                                      ctypes.byref(h)), "create")
        return cls(h, arch)

    def randomize(self, seed=0, std=0.02):
        check(lib().vsim_model_randomize(self.h, seed, std), "randomize")

    def get_tensor(self, name: str, nbytes: int) -> np.ndarray:
        """One tensor in the ggml file's format (Q4_0 AoS blocks / F32), as raw bytes."""
        buf = np.zeros(nbytes, np.uint8)
        check(lib().vsim_model_get_tensor(self.h, name.encode(), ptr(buf), nbytes), f"get_tensor {name}")
        return buf

    def set_mode(self, mode):
        check(lib().vsim_model_set_mode(self.h, mode), "set_mode")

    def reserve(self, n_tokens):
        """Allocates a prompt of up to n_tokens' buffers and loads its kernels ahead of the first eval."""
        check(lib().vsim_model_reserve(self.h, n_tokens), "reserve")

    def set_graph(self, enable: bool):
        check(lib().vsim_model_set_graph(self.h, 1 if enable else 0), "set_graph")

    def eval(self, n_past, tokens=None, resid_in=None, resid_out=None, want_logits=True):
        N = len(tokens) if tokens is not None else int(resid_in.shape[0])
        tok = np.ascontiguousarray(tokens, np.int32) if tokens is not None else None
        lg = np.zeros(self.n_vocab, np.float32) if (want_logits and self.last) else None
        check(lib().vsim_model_eval(self.h, n_past, ptr(tok), N, ptr(resid_in), ptr(resid_out), ptr(lg)), "eval")
        return lg

    def eval_argmax(self, n_past, token) -> int:
        """Greedy decode step: the next token (argmax of the logits, taken on the device)."""
        nxt = ctypes.c_int32()
        check(lib().vsim_model_eval_argmax(self.h, n_past, int(token), ctypes.byref(nxt)), "eval_argmax")
        return nxt.value

    def generate(self, n_past, token, n_steps) -> list:
        """n_steps greedy decode steps kept on the device; returns the generated tokens."""
        out = (ctypes.c_int32 * max(n_steps, 1))()
        check(lib().vsim_model_generate(self.h, n_past, int(token), n_steps, out), "generate")
        return list(out[:n_steps])

    def info(self):
        k, g, w = ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
        check(lib().vsim_model_info(self.h, ctypes.byref(k), ctypes.byref(g), ctypes.byref(w)), "info")
        return {"kernels_per_eval": k.value, "graph": bool(g.value), "weight_bytes": w.value}

    def set_profile(self, enable: bool):
        check(lib().vsim_model_set_profile(self.h, 1 if enable else 0), "set_profile")

    def profile_stats(self):
        ms, n, b = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
        check(lib().vsim_model_profile_stats(self.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b)), "prof")
        return {"gemv_ms": ms.value, "gemv_launches": n.value, "gemv_bytes": b.value}

    def profile_kernels(self) -> list:
        """Per-kernel totals since set_profile(True): [{name, ms, launches, bytes}]."""
        out, i = [], 0
        name = ctypes.create_string_buffer(96)
        ms, n, b = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
        while lib().vsim_model_profile_kernel(self.h, i, name, 96, ctypes.byref(ms), ctypes.byref(n),
                                              ctypes.byref(b)) == 0:
            out.append({"name": name.value.decode(), "ms": ms.value, "launches": n.value, "bytes": b.value})
            i += 1
        return out

    def stream(self) -> int:
        return lib().vsim_model_stream(self.h)

    def stage_bind(self, tok_in=0, resid_in=0, resid_out=0, tok_out=0):
        """Bind the pipeline-stage buffers (device addresses, e.g. torch tensors' data_ptr())."""
        check(lib().vsim_model_stage_bind(self.h, tok_in or None, resid_in or None, resid_out or None,
                                          tok_out or None), "stage_bind")

    def stage_begin(self, n_past: int):
        check(lib().vsim_model_stage_begin(self.h, n_past), "stage_begin")

    def stage_step(self):
        """Enqueue one stage step on the model's stream (no wait)."""
        check(lib().vsim_model_stage_step(self.h), "stage_step")

    def sync(self):
        check(lib().vsim_model_sync(self.h), "sync")

    def debug_poison(self, n_tokens: int):
        """Fill the scratch and the KV cache with NaN (test support, include/vsim_hip.h)."""
        check(lib().vsim_model_debug_poison(self.h, n_tokens), "debug_poison")

    def close(self):
        if getattr(self, "h", None):
            lib().vsim_model_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def norm_fallbacks():
    """Exact-LayerNorm rows that took the sequential fallback so far: (mean, variance)."""
    out = (ctypes.c_uint * 2)()
    check(lib().vsim_norm_fallbacks(out), "norm_fallbacks")
    return int(out[0]), int(out[1])


def spin_timeouts():
    """Bounded cross-workgroup waits that gave up so far (0 in a healthy run)."""
    out = ctypes.c_uint()
    check(lib().vsim_spin_timeouts(ctypes.byref(out)), "spin_timeouts")
    return int(out.value)


def dropin_stats():
    v = [ctypes.c_uint64() for _ in range(4)]
    lib().vsim_dropin_stats(*[ctypes.byref(x) for x in v])
    return {"calls": v[0].value, "h2d": v[1].value, "d2h": v[2].value, "cached": v[3].value}
