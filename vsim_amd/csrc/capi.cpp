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
#include <map>
#include <vector>

#include "common.hpp"
#include "graph.hpp"
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
int vsim_op_q4_expand_f16(const void *w, int M, int K, void *w16, void *stream) {
  if (!w || !w16 || M <= 0 || K <= 0 || K % QK) { set_error("q4_expand_f16: bad argument"); return VSIM_EINVAL; }
  return launch_w4_expand_f16(w4_view(w, M, K), w16, (hipStream_t)stream);
}
int vsim_op_gemm_f16(const void *w16, int M, int K, const void *x16, int n, const float *bias, float *y,
                     void *stream) {
  if (!w16 || !x16 || !y) { set_error("gemm_f16: null argument"); return VSIM_EINVAL; }
  return launch_gemm_f16_256(w16, M, K, x16, n, bias, y, (hipStream_t)stream);
}
int vsim_op_act_quant_f16(const float *x, int K, int n, const float *bias, int gelu, void *x16, void *stream) {
  if (!x || !x16) { set_error("act_quant_f16: null argument"); return VSIM_EINVAL; }
  return launch_act_quant_f16(x, K, n, bias, gelu != 0, x16, (hipStream_t)stream);
}
int vsim_op_gemm_f16_gelu_q(const void *w16, int M, int K, const void *x16, int n, const float *bias, void *q16,
                            void *stream) {
  if (!w16 || !x16 || !q16) { set_error("gemm_f16_gelu_q: null argument"); return VSIM_EINVAL; }
  return launch_gemm_f16_256(w16, M, K, x16, n, bias, nullptr, (hipStream_t)stream, q16);
}
int vsim_op_gemm_f16_rope(const void *w16, int M, int K, const void *x16, int n, const float *bias, float *y,
                          const double *cs, int d, int n_rot, int p0, void *stream) {
  if (!w16 || !x16 || !y || !cs || p0 < 0) { set_error("gemm_f16_rope: bad argument"); return VSIM_EINVAL; }
  G2Epi e;
  e.cs = (const double2 *)cs;
  e.d = d;
  e.n_rot = n_rot;
  e.p0 = p0;
  return launch_gemm_f16_256(w16, M, K, x16, n, bias, y, (hipStream_t)stream, nullptr, &e);
}
int vsim_op_gemm_f16_join(const void *w16, int M, int K, const void *x16, int n, const float *bias, float *res,
                          const float *res_a, void *stream) {
  if (!w16 || !x16 || !res) { set_error("gemm_f16_join: null argument"); return VSIM_EINVAL; }
  G2Epi e;
  e.res = res;
  e.res_a = res_a;
  return launch_gemm_f16_256(w16, M, K, x16, n, bias, res, (hipStream_t)stream, nullptr, &e);
}
int vsim_op_gemm_q4_256(const void *w, int M, int K, const void *x16, int n, const float *bias, float *y, void *q16,
                        const double *cs, int d, int n_rot, int p0, int join, const float *res_a, void *stream) {
  if (!w || !x16 || (!q16 && !y) || M <= 0 || K <= 0 || K % QK || p0 < 0) {
    set_error("gemm_q4_256: bad argument");
    return VSIM_EINVAL;
  }
  if ((q16 != nullptr) + (cs != nullptr) + (join != 0) > 1) {
    set_error("gemm_q4_256: one epilogue at a time (q16, cs or join)");
    return VSIM_EINVAL;
  }
  G2Epi e;
  if (cs) {
    e.cs = (const double2 *)cs;
    e.d = d;
    e.n_rot = n_rot;
    e.p0 = p0;
  } else if (join) {
    e.res = y;
    e.res_a = res_a;
  }
  return launch_gemm_q4_256(w4_view(w, M, K), x16, n, bias, q16 ? nullptr : y, (hipStream_t)stream, q16,
                            cs || join ? &e : nullptr);
}
int vsim_op_get_rows(const void *w, int K, int V, const int32_t *rows, int n, float *y, void *stream) {
  return launch_get_rows(w, K, V, rows, n, y, (hipStream_t)stream);
}
int vsim_norm_fallbacks(unsigned out[2]) { return vsim::norm_stats(out); }
int vsim_spin_timeouts(unsigned *out) { return vsim::spin_timeouts(out); }

int vsim_op_norm(const float *x, float *y, int k, int rows, const float *w, const float *b, void *stream) {
  return launch_norm(x, y, k, rows, w, b, (hipStream_t)stream);
}
int vsim_op_gelu(const float *x, float *y, int n, void *stream) {
  return launch_gelu(x, y, n, nullptr, 1, (hipStream_t)stream);
}
int vsim_op_argmax(const float *x, int n, int32_t *out, void *stream) {
  // one zeroed 16-byte workspace per (device, stream), kept: the kernel leaves it zeroed, so the
  // call is a single launch (no allocation, no synchronization, capturable) like the model's
  static std::mutex mu;
  static std::map<std::pair<int, void *>, unsigned long long *> wss;
  int dev = 0;
  VSIM_HIP(hipGetDevice(&dev));
  unsigned long long *ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu);
    unsigned long long *&w = wss[{dev, stream}];
    if (!w) {
      VSIM_HIP(hipMalloc((void **)&w, 2 * sizeof(unsigned long long)));
      VSIM_HIP(hipMemset(w, 0, 2 * sizeof(unsigned long long)));
    }
    ws = w;
  }
  return launch_argmax(x, n, (int *)out, ws, (hipStream_t)stream);
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
int vsim_op_kq_causal(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int n, int n_past,
                      float *kq, void *stream) {
  if (n_past < 0) { set_error("kq_causal: n_past must be >= 0"); return VSIM_EINVAL; }
  return launch_kq(K, ldk, Q, ldq, d, H, nk, n, kq, (hipStream_t)stream, n_past);
}
int vsim_op_kqv_causal(const float *V, int ldv, const float *S, int d, int H, int nk, int n, int n_past, float *out,
                       void *stream) {
  if (n_past < 0) { set_error("kqv_causal: n_past must be >= 0"); return VSIM_EINVAL; }
  return launch_kqv(V, ldv, S, d, H, nk, n, out, 0, (hipStream_t)stream, n_past);
}
int vsim_op_attn_prefill(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                         float scale, float *out, void *stream) {
  return launch_attn_prefill_f16(Q, kc, vc, d, H, N, n_past, scale, out, (hipStream_t)stream);
}
int vsim_op_attn_prefill_q16(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                             float scale, void *out16, void *stream) {
  return launch_attn_prefill_f16(Q, kc, vc, d, H, N, n_past, scale, nullptr, (hipStream_t)stream, nullptr, 0, false,
                                 out16);
}
int vsim_op_tables(uint16_t *exp_f16_host, uint16_t *gelu_f16_host) { return tables_host(exp_f16_host, gelu_f16_host); }
int vsim_gemm_set_streamk(int enable) { return gemm_set_streamk(enable); }
int vsim_gemm_set_qk_pair(int mode) { return gemm_set_qk_pair(mode); }
int vsim_gemm_set_tile_order(int cols) { return gemm_set_tile_order(cols); }
int vsim_op_gemm_q4_256_pair(const void *w0, const void *w1, int M, int K, const void *x16, int n, float *y0, float *y1,
                             const double *cs, int d, int n_rot, int p0, void *stream) {
  if (!w0 || !w1 || !x16 || !y0 || !y1 || !cs || M <= 0 || K <= 0 || K % QK || p0 < 0 || n <= 0) {
    set_error("gemm_q4_256_pair: bad argument");
    return VSIM_EINVAL;
  }
  G2Epi e;
  e.cs = (const double2 *)cs;
  e.d = d;
  e.n_rot = n_rot;
  e.p0 = p0;
  return launch_gemm_q4_256_pair(w4_view(w0, M, K), w4_view(w1, M, K), x16, n, y0, y1, e, e, (hipStream_t)stream);
}
int vsim_op_norm_f16q(const float *x, int k, int rows, const float *w, const float *b, void *x16, void *stream) {
  return launch_norm_f16q(x, x16, k, rows, w, b, (hipStream_t)stream);
}

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
// Contract (include/vsim_hip.h): a hook is called by every thread of the reference's pool in
// every phase of the node.  Its checks read tensor metadata only, so all threads reach the
// same verdict: either every thread gets VSIM_EINVAL and runs its own CPU slice, or thread 0
// runs the whole op in its COMPUTE phase and every other call returns 0 ("handled": the INIT
// and FINALIZE phases then have nothing left to do).  A device failure after the checks exits,
// as the reference's offload layer does (imax.c:2042-2049).
namespace {

size_t f32_span(const ggml_tensor *t) {
  size_t s = 4;
  for (int i = 0; i < 4; ++i)
    if (t->ne[i] > 1) s += (size_t)(t->ne[i] - 1) * t->nb[i];
  return s;
}

GT gt_dev(const ggml_tensor *t, const void *dev) {
  GT g;
  g.p = (const char *)dev;
  for (int i = 0; i < 4; ++i) {
    g.ne[i] = t->ne[i];
    g.nb[i] = (long long)t->nb[i];
  }
  return g;
}

// cached device buffers of the hooks (grown, never freed per call)
void *hb[4] = {nullptr, nullptr, nullptr, nullptr};
size_t hcap[4] = {0, 0, 0, 0};
double2 *hcs = nullptr;
size_t hcs_cap = 0;

void *hbuf(int i, size_t bytes, const char *what) {
  if (grow(&hb[i], &hcap[i], bytes)) die(what);
  return hb[i];
}

void to_dev(void *dev, const void *host, size_t bytes) {
  if (hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, g.stream) != hipSuccess) die("hook upload");
  g.h2d += bytes;
}

void to_host(void *host, const void *dev, size_t bytes) {
  if (hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, g.stream) != hipSuccess ||
      hipStreamSynchronize(g.stream) != hipSuccess)
    die("hook download");
  g.d2h += bytes;
}

bool handled_elsewhere(const ggml_compute_params *params) {
  return params->type != GGML_TASK_COMPUTE || params->ith != 0;
}

void lock_and_init(const char *who) {
  if (ensure_init()) die(who);
  if (hipSetDevice(g.device) != hipSuccess) die(who);
}

}  // namespace

// ggml_compute_forward_gptneox_rope_f32 (ggml.c:6086) / ggml_compute_forward_rope_f32
// (ggml.c:5919): src0 [d, H, T] contiguous F32, src1 I32 {n_past, n_dims, mode}, in place.
static int rope_hook(int style, const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                     const struct ggml_tensor *src1, struct ggml_tensor *dst) {
  const int32_t *pr = src1 && src1->type == GGML_TYPE_I32 ? (const int32_t *)src1->data : nullptr;
  if (!contiguous_f32(src0) || src0->ne[3] != 1 || dst->data != src0->data || !pr || pr[1] <= 0 || pr[1] % 2 ||
      pr[1] > src0->ne[0] || (pr[2] != 0 && pr[2] != 1)) {
    set_error("rope hook: needs a contiguous in-place F32 [d,H,T] tensor and {n_past, n_dims, mode}");
    return VSIM_EINVAL;
  }
  if (handled_elsewhere(params)) return 0;
  std::lock_guard<std::mutex> lk(g.mu);
  lock_and_init("rope hook");
  const int d = src0->ne[0], H = src0->ne[1], T = src0->ne[2], n_past = pr[0], n_dims = pr[1], mode = pr[2];
  const size_t nb = (size_t)d * H * T * 4;
  const int n_pos = mode == 0 ? n_past + T : T;
  std::vector<double2> cs((size_t)n_pos * (n_dims / 2));
  rope_table_host(cs.data(), n_pos, n_dims);
  float *x = (float *)hbuf(0, nb, "rope hook alloc");
  if (grow((void **)&hcs, &hcs_cap, cs.size() * sizeof(double2))) die("rope hook alloc");
  to_dev(x, src0->data, nb);
  to_dev(hcs, cs.data(), cs.size() * sizeof(double2));
  if (launch_rope(style, x, d, H, T, n_past, n_dims, mode, hcs, g.stream)) die("rope hook");
  to_host(dst->data, x, nb);
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
  if (!contiguous_f32(src0) || dst->data != src0->data) {
    set_error("soft_max hook: needs a contiguous in-place F32 tensor");
    return VSIM_EINVAL;
  }
  if (handled_elsewhere(params)) return 0;
  std::lock_guard<std::mutex> lk(g.mu);
  lock_and_init("soft_max hook");
  const int nc = src0->ne[0], nr = src0->ne[1] * src0->ne[2] * src0->ne[3];
  const size_t nb = (size_t)nc * nr * 4;
  float *x = (float *)hbuf(0, nb, "soft_max hook alloc");
  to_dev(x, src0->data, nb);
  if (launch_attn_softmax(x, nc, nr, 1, nc, 1.0f, g.stream)) die("soft_max hook");
  to_host(dst->data, x, nb);
  return 0;
}

// ggml_compute_forward_mul_mat_f32 (ggml.c:4355-4595) for any strided F32 views: src0 rows
// contiguous -> double-accumulated dots (the KQ product, vsim.cpp:583); src0 transposed ->
// sequential mads in params->nth column partials, summed in thread order (the KQV product,
// vsim.cpp:607), the grouping the reference's pool uses at that thread count.
int vsim_ggml_mul_mat_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                          const struct ggml_tensor *src1, struct ggml_tensor *dst) {
  const bool types = src0->type == GGML_TYPE_F32 && src1->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_F32;
  const bool shapes = src0->ne[0] == src1->ne[0] && src0->ne[2] == src1->ne[2] && src0->ne[3] == src1->ne[3] &&
                      dst->ne[0] == src0->ne[1] && dst->ne[1] == src1->ne[1] && dst->ne[2] == src0->ne[2] &&
                      dst->ne[3] == src1->ne[3];
  const bool dot = src0->nb[1] >= src0->nb[0];
  const bool layout = dot ? (src0->nb[0] == 4 && src1->nb[0] == 4 && dst->nb[0] == 4)
                          : (src0->nb[1] == 4 && contiguous_f32(dst));
  if (!types || !shapes || !layout || params->nth <= 0) {
    set_error("mul_mat_f32 hook: unsupported F32 operands");
    return VSIM_EINVAL;
  }
  if (handled_elsewhere(params)) return 0;
  std::lock_guard<std::mutex> lk(g.mu);
  lock_and_init("mul_mat_f32 hook");
  const size_t sa = f32_span(src0), sb = f32_span(src1), sd = f32_span(dst);
  char *da = (char *)hbuf(1, sa, "mul_mat_f32 hook alloc");
  char *db = (char *)hbuf(2, sb, "mul_mat_f32 hook alloc");
  char *dd = (char *)hbuf(3, sd, "mul_mat_f32 hook alloc");
  to_dev(da, src0->data, sa);
  to_dev(db, src1->data, sb);
  int rc;
  if (dot) {
    to_dev(dd, dst->data, sd);  // strided dst: the bytes between its elements stay as they were
    rc = launch_g_mm_dot(gt_dev(dst, dd), gt_dev(src0, da), gt_dev(src1, db), src0->ne[0], g.stream);
  } else {
    rc = launch_g_mm_mad((float *)dd, gt_dev(src0, da), gt_dev(src1, db), src1->ne[0], params->nth, dst->ne[0],
                         dst->ne[1], dst->ne[2], dst->ne[3], g.stream);
  }
  if (rc) die("mul_mat_f32 hook");
  to_host(dst->data, dd, sd);
  return 0;
}

}  // extern "C"
