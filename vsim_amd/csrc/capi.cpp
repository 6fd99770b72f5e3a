// vsim_amd/csrc/capi.cpp — the C-ABI entry points of libvsim_hip.so:
//   * drop-in replacements for the reference offload layer (imax.c:52-142, 1133-2292),
//   * vsim_ggml_* hooks for the ops the reference computes in static ggml.c kernels,
//   * op-level device API (vsim_op_*).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {
int tables_host(uint16_t *exp_f16, uint16_t *gelu_f16);
}  // namespace vsim

using namespace vsim;

#define RC(x)                \
  do {                       \
    int rc_ = (x);           \
    if (rc_) return rc_;     \
  } while (0)

extern "C" {

// ---------------------------------------------------------------- op-level API
int vsim_op_q4_repack(const void *aos, void *soa, int rows, int k, void *stream) {
  return launch_q4_repack(aos, soa, rows, k, (hipStream_t)stream);
}
int vsim_op_q4_unpack(const void *soa, void *aos, int rows, int k, void *stream) {
  return launch_q4_unpack(soa, aos, rows, k, (hipStream_t)stream);
}
int vsim_op_act_repack(const void *aos, void *xq, int n, int k, void *stream) {
  return launch_act_repack(aos, xq, n, k, (hipStream_t)stream);
}
int vsim_op_act_unpack(const void *xq, void *aos, int n, int k, void *stream) {
  return launch_act_unpack(xq, aos, n, k, (hipStream_t)stream);
}
int vsim_op_q4_quantize(const float *x, int k, int n, void *xq, float *xd, void *stream) {
  return launch_q4_quantize(x, k, n, xq, xd, (hipStream_t)stream);
}
int vsim_op_q4_gemv(const void *w, int M, int K, const void *xq, const float *xd, int n, const float *bias, float *y,
                    int mode, void *stream) {
  return launch_q4_gemv(w, M, K, xq, xd, n, bias, y, mode, (hipStream_t)stream);
}
int vsim_op_get_rows(const void *w, int K, int V, const int32_t *rows, int n, float *y, void *stream) {
  return launch_get_rows(w, K, V, rows, n, y, (hipStream_t)stream);
}
int vsim_norm_fallbacks(unsigned out[2]) { return vsim::norm_stats(out); }

int vsim_op_norm(const float *x, float *y, int k, int rows, const float *w, const float *b, void *stream) {
  return launch_norm(x, y, k, rows, w, b, (hipStream_t)stream);
}
int vsim_op_gelu(const float *x, float *y, int n, void *stream) {
  return launch_gelu(x, y, n, nullptr, 1, (hipStream_t)stream);
}
int vsim_op_attn_softmax(float *p, int nc, int nr, int nz, int n_past, float scale, void *stream) {
  return launch_attn_softmax(p, nc, nr, nz, n_past, scale, (hipStream_t)stream);
}
int vsim_op_rope(int style, float *x, int d, int H, int T, int n_past, int n_dims, int mode, void *stream) {
  if (n_dims <= 0 || n_dims % 2 || n_dims > d) { set_error("rope: bad n_dims"); return VSIM_EINVAL; }
  const int n_pos = (mode == 0 ? n_past + T : T);
  std::vector<double2> cs((size_t)n_pos * (n_dims / 2));
  rope_table_host(cs.data(), n_pos, n_dims);
  double2 *dcs = nullptr;
  VSIM_HIP(hipMalloc(&dcs, cs.size() * sizeof(double2)));
  hipStream_t s = (hipStream_t)stream;
  int rc = hipMemcpyAsync(dcs, cs.data(), cs.size() * sizeof(double2), hipMemcpyHostToDevice, s) == hipSuccess
               ? launch_rope(style, x, d, H, T, n_past, n_dims, mode, dcs, s)
               : VSIM_EHIP;
  if (hipStreamSynchronize(s) != hipSuccess && rc == 0) rc = VSIM_EHIP;
  (void)hipFree(dcs);
  return rc;
}
int vsim_op_kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int n, float *kq, void *stream) {
  return launch_kq(K, ldk, Q, ldq, d, H, nk, n, kq, (hipStream_t)stream);
}
int vsim_op_kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int n, float *out, void *stream) {
  return launch_kqv(V, ldv, S, d, H, nk, n, out, 0, (hipStream_t)stream);
}
int vsim_op_attn_prefill(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                         float scale, float *out, void *stream) {
  return launch_attn_prefill_f16(Q, kc, vc, d, H, N, n_past, scale, out, (hipStream_t)stream);
}
int vsim_op_tables(uint16_t *exp_f16_host, uint16_t *gelu_f16_host) { return tables_host(exp_f16_host, gelu_f16_host); }

}  // extern "C"

// ---------------------------------------------------------------- drop-in state
namespace {

struct WEntry {
  void *dev;
  int rows, k;
};

struct DropIn {
  std::mutex mu;
  bool ready = false;
  int device = 0;
  int mode = VSIM_MODE_EXACT;
  hipStream_t stream = nullptr;
  std::unordered_map<const void *, WEntry> wcache;
  uint8_t *act_aos = nullptr, *act_soa = nullptr;
  float *xd = nullptr, *y = nullptr, *tmp = nullptr;
  size_t act_cap = 0, xd_cap = 0, y_cap = 0, tmp_cap = 0;
  uint64_t calls = 0, h2d = 0, d2h = 0, cached = 0;
} g;

int grow(void **p, size_t *cap, size_t want) {
  if (want <= *cap) return VSIM_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  const size_t n = want + want / 2;
  VSIM_HIP(hipMalloc(p, n));
  *cap = n;
  return VSIM_OK;
}

int ensure_init() {
  if (g.ready) return VSIM_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("init_xmax: no HIP device");
    return VSIM_ENODEV;
  }
  const char *e = getenv("VSIM_DEVICE");
  g.device = e ? atoi(e) : 0;
  if (g.device < 0 || g.device >= ndev) g.device = 0;
  const char *md = getenv("VSIM_MODE");
  g.mode = (md && !strcmp(md, "fast")) ? VSIM_MODE_FAST : VSIM_MODE_EXACT;
  VSIM_HIP(hipSetDevice(g.device));
  VSIM_HIP(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));
  DevTables t;
  RC(tables_get(&t));
  g.ready = true;
  return VSIM_OK;
}

[[noreturn]] void die(const char *where) {
  // the reference exits on offload errors (imax.c:64-69, 2042-2049)
  printf("%s: %s\n", where, vsim_last_error());
  fflush(stdout);
  exit(1);
}

int upload_tensor(const ggml_tensor *t, void **dev, size_t *cap) {
  size_t nb = (size_t)t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3] * sizeof(float);
  RC(grow(dev, cap, nb));
  VSIM_HIP(hipMemcpyAsync(*dev, t->data, nb, hipMemcpyHostToDevice, g.stream));
  g.h2d += nb;
  return VSIM_OK;
}

bool contiguous_f32(const ggml_tensor *t) {
  return t->type == GGML_TYPE_F32 && t->nb[0] == 4 && t->nb[1] == t->nb[0] * t->ne[0] &&
         t->nb[2] == t->nb[1] * t->ne[1] && t->nb[3] == t->nb[2] * t->ne[2];
}

}  // namespace

extern "C" {

// imax.c:52-142: device init.  Same symbol, called once by vsim.cpp:788 after the model
// load; selects the GPU (VSIM_DEVICE), builds the fp16 tables, creates the stream.
void init_xmax(void) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (ensure_init()) die("init_xmax");
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, g.device) == hipSuccess)
    printf("vsim-hip: device %d %s (%s), %d CUs, mode=%s\n", g.device, p.name, p.gcnArchName, p.multiProcessorCount,
           g.mode == VSIM_MODE_EXACT ? "exact" : "fast");
}

// imax.c:1133-1139 signature, called from ggml.c:5115 in the COMPUTE phase of every
// Q4_0 x F32 mul_mat with params->wdata = the Q4_0-quantized src1 rows (INIT phase,
// ggml.c:5024-5041).  Thread 0 runs the whole product on the GPU; other threads of the
// reference's pool return at once and meet thread 0 at ggml's barrier.
void imax_ggml_compute_forward_mul_mat_q4_0_f32(int THREAD, int LANE, const struct ggml_compute_params *params,
                                                const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                                                struct ggml_tensor *dst) {
  (void)THREAD;
  (void)LANE;
  if (params->type != GGML_TASK_COMPUTE || params->ith != 0) return;
  std::lock_guard<std::mutex> lk(g.mu);
  if (ensure_init()) die("imax_ggml_compute_forward_mul_mat_q4_0_f32");
  const int K = src0->ne[0], M = src0->ne[1], N = src1->ne[1];
  if (src0->type != GGML_TYPE_Q4_0 || src0->ne[2] != 1 || src0->ne[3] != 1 || src1->ne[2] != 1 ||
      src1->ne[3] != 1 || K % QK || src0->nb[1] != (size_t)K / QK * QBYTES || dst->nb[0] != 4 ||
      dst->nb[1] != (size_t)M * 4) {
    printf("imax_ggml_compute_forward_mul_mat_q4_0_f32: unsupported shape ne00=%d ne01=%d ne02=%d ne11=%d\n", K, M,
           src0->ne[2], N);
    exit(1);
  }
  hipStream_t s = g.stream;
  if (hipSetDevice(g.device) != hipSuccess) die("hipSetDevice");
  // device weight cache, keyed by the host tensor (model weights live for the run)
  auto it = g.wcache.find(src0->data);
  if (it == g.wcache.end() || it->second.rows != M || it->second.k != K) {
    const size_t wb = (size_t)M * K / QK * QBYTES;
    void *dev = nullptr, *stage = nullptr;
    if (hipMalloc(&dev, w4_bytes(M, K)) != hipSuccess || hipMalloc(&stage, wb) != hipSuccess) die("weight cache alloc");
    if (hipMemcpyAsync(stage, src0->data, wb, hipMemcpyHostToDevice, s) != hipSuccess) die("weight upload");
    if (launch_q4_repack(stage, dev, M, K, s)) die("weight repack");
    if (hipStreamSynchronize(s) != hipSuccess) die("weight upload sync");
    (void)hipFree(stage);
    if (it != g.wcache.end()) (void)hipFree(it->second.dev);
    g.wcache[src0->data] = WEntry{dev, M, K};
    g.h2d += wb;
    g.cached += wb;
    it = g.wcache.find(src0->data);
  }
  const size_t ab = (size_t)N * K / QK * QBYTES;
  if (grow((void **)&g.act_aos, &g.act_cap, ab) || grow((void **)&g.act_soa, &g.tmp_cap, ab) ||
      grow((void **)&g.xd, &g.xd_cap, (size_t)N * K * 4) || grow((void **)&g.y, &g.y_cap, (size_t)N * M * 4))
    die("activation alloc");
  if (hipMemcpyAsync(g.act_aos, params->wdata, ab, hipMemcpyHostToDevice, s) != hipSuccess) die("activation upload");
  if (launch_act_repack(g.act_aos, g.act_soa, N, K, s)) die("activation repack");
  if (launch_q4_dequant(g.act_soa, N, K, g.xd, s)) die("activation dequant");
  if (launch_q4_gemv(it->second.dev, M, K, g.act_soa, g.xd, N, nullptr, g.y, g.mode, s)) die("gemv");
  if (hipMemcpyAsync(dst->data, g.y, (size_t)N * M * 4, hipMemcpyDeviceToHost, s) != hipSuccess) die("result copy");
  if (hipStreamSynchronize(s) != hipSuccess) die("gemv sync");
  g.calls++;
  g.h2d += ab;
  g.d2h += (size_t)N * M * 4;
}

void vsim_dropin_stats(uint64_t *calls, uint64_t *h2d, uint64_t *d2h, uint64_t *cached) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (calls) *calls = g.calls;
  if (h2d) *h2d = g.h2d;
  if (d2h) *d2h = g.d2h;
  if (cached) *cached = g.cached;
}

void vsim_dropin_reset(void) {
  std::lock_guard<std::mutex> lk(g.mu);
  for (auto &kv : g.wcache) (void)hipFree(kv.second.dev);
  g.wcache.clear();
  g.calls = g.h2d = g.d2h = g.cached = 0;
}

// ---- hooks for the reference's static ggml.c kernels (host tensors in/out, exact) ----
// ggml_compute_forward_gptneox_rope_f32 (ggml.c:6086) / ggml_compute_forward_rope_f32
// (ggml.c:5919): src0 [d, H, T] contiguous F32, src1 I32 {n_past, n_dims, mode}, in place.
static int rope_hook(int style, const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                     const struct ggml_tensor *src1, struct ggml_tensor *dst) {
  if (params->type != GGML_TASK_COMPUTE) return 0;
  if (params->ith != 0) return 0;
  std::lock_guard<std::mutex> lk(g.mu);
  RC(ensure_init());
  if (!contiguous_f32(src0) || src0->ne[3] != 1 || dst->data != src0->data) {
    set_error("rope hook: needs a contiguous in-place F32 [d,H,T] tensor");
    return VSIM_EINVAL;
  }
  const int32_t *pr = (const int32_t *)src1->data;
  const int d = src0->ne[0], H = src0->ne[1], T = src0->ne[2];
  RC(upload_tensor(src0, (void **)&g.tmp, &g.tmp_cap));
  RC(vsim_op_rope(style, g.tmp, d, H, T, pr[0], pr[1], pr[2], g.stream));
  VSIM_HIP(hipMemcpy(dst->data, g.tmp, (size_t)d * H * T * 4, hipMemcpyDeviceToHost));
  g.d2h += (size_t)d * H * T * 4;
  return 0;
}

int vsim_ggml_gptneox_rope_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                               const struct ggml_tensor *src1, struct ggml_tensor *dst) {
  return rope_hook(0, params, src0, src1, dst);
}

int vsim_ggml_rope_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                       const struct ggml_tensor *src1, struct ggml_tensor *dst) {
  return rope_hook(1, params, src0, src1, dst);
}

// ggml_compute_forward_soft_max_f32 (ggml.c:5825): rows of ne0, in place (scale = 1,
// no mask: the reference applies scale and diag_mask_inf as separate nodes before).
int vsim_ggml_soft_max_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                           struct ggml_tensor *dst) {
  if (params->type != GGML_TASK_COMPUTE || params->ith != 0) return 0;
  std::lock_guard<std::mutex> lk(g.mu);
  RC(ensure_init());
  if (!contiguous_f32(src0) || dst->data != src0->data) {
    set_error("soft_max hook: needs a contiguous in-place F32 tensor");
    return VSIM_EINVAL;
  }
  const int nc = src0->ne[0], nr = src0->ne[1] * src0->ne[2] * src0->ne[3];
  RC(upload_tensor(src0, (void **)&g.tmp, &g.tmp_cap));
  RC(launch_attn_softmax(g.tmp, nc, nr, 1, nc, 1.0f, g.stream));
  VSIM_HIP(hipMemcpy(dst->data, g.tmp, (size_t)nc * nr * 4, hipMemcpyDeviceToHost));
  g.d2h += (size_t)nc * nr * 4;
  return 0;
}

// ggml_compute_forward_mul_mat_f32 (ggml.c:4355): the two attention products of
// vsim.cpp:583 (K permuted view x Q) and vsim.cpp:607 (V_trans view x softmax).
int vsim_ggml_mul_mat_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                          const struct ggml_tensor *src1, struct ggml_tensor *dst) {
  if (params->type != GGML_TASK_COMPUTE || params->ith != 0) return 0;
  std::lock_guard<std::mutex> lk(g.mu);
  RC(ensure_init());
  hipStream_t s = g.stream;
  const int H = src0->ne[2];
  if (src0->nb[1] >= src0->nb[0]) {
    // KQ: src0 [d, nk, H] nb {4, ldk*4, d*4}; src1 [d, N, H] nb {4, ldq*4, d*4}
    const int d = src0->ne[0], nk = src0->ne[1], N = src1->ne[1];
    const int ldk = (int)(src0->nb[1] / 4), ldq = (int)(src1->nb[1] / 4);
    if (src0->nb[0] != 4 || src0->nb[2] != (size_t)d * 4 || src1->nb[0] != 4 || src1->nb[2] != (size_t)d * 4) {
      set_error("mul_mat_f32 hook: unsupported KQ view");
      return VSIM_EINVAL;
    }
    const size_t kb = ((size_t)(nk - 1) * ldk + (size_t)H * d) * 4, qb = ((size_t)(N - 1) * ldq + (size_t)H * d) * 4;
    float *dk = nullptr, *dq = nullptr, *dy = nullptr;
    VSIM_HIP(hipMalloc(&dk, kb));
    VSIM_HIP(hipMalloc(&dq, qb));
    VSIM_HIP(hipMalloc(&dy, (size_t)H * N * nk * 4));
    (void)hipMemcpyAsync(dk, src0->data, kb, hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(dq, src1->data, qb, hipMemcpyHostToDevice, s);
    int rc = launch_kq(dk, ldk, dq, ldq, d, H, nk, N, dy, s);
    (void)hipMemcpyAsync(dst->data, dy, (size_t)H * N * nk * 4, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(dk); (void)hipFree(dq); (void)hipFree(dy);
    g.h2d += kb + qb;
    g.d2h += (size_t)H * N * nk * 4;
    return rc;
  }
  // KQV: src0 = V_trans [nk, d, H] nb {ldv*4, 4, d*4}; src1 = S [nk, N, H] contiguous
  const int nk = src0->ne[0], d = src0->ne[1], N = src1->ne[1];
  const int ldv = (int)(src0->nb[0] / 4);
  if (src0->nb[1] != 4 || src0->nb[2] != (size_t)d * 4 || !contiguous_f32(src1)) {
    set_error("mul_mat_f32 hook: unsupported KQV view");
    return VSIM_EINVAL;
  }
  const size_t vb = ((size_t)(nk - 1) * ldv + (size_t)H * d) * 4, sb = (size_t)nk * N * H * 4;
  float *dv = nullptr, *ds = nullptr, *dy = nullptr;
  VSIM_HIP(hipMalloc(&dv, vb));
  VSIM_HIP(hipMalloc(&ds, sb));
  VSIM_HIP(hipMalloc(&dy, (size_t)H * N * d * 4));
  (void)hipMemcpyAsync(dv, src0->data, vb, hipMemcpyHostToDevice, s);
  (void)hipMemcpyAsync(ds, src1->data, sb, hipMemcpyHostToDevice, s);
  int rc = launch_kqv(dv, ldv, ds, d, H, nk, N, dy, 0, s);
  (void)hipMemcpyAsync(dst->data, dy, (size_t)H * N * d * 4, hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  (void)hipFree(dv); (void)hipFree(ds); (void)hipFree(dy);
  g.h2d += vb + sb;
  g.d2h += (size_t)H * N * d * 4;
  return rc;
}

}  // extern "C"
