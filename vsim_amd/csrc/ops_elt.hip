// vsim_amd/csrc/ops_elt.hip — LayerNorm, GELU, bias and residual adds.
//
//   ggml_compute_forward_norm_f32  ggml.c:4246-4304 (double mean/variance, eps 1e-5f)
//   ggml_vec_gelu_f32 (fp16 LUT)   ggml.c:795-803, table ggml.c:1240-1251
//   add / mul / repeat             ggml.c:3344-3418, 3474-3522, 3809-3847
#include <cmath>
#include <cstring>
#include <atomic>
#include <mutex>
#include <vector>

#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

// ------------------------------------------------------------------ LayerNorm (exact)
// The reference sums the row sequentially in double.  We sum in parallel and prove the
// sum equal to the sequential one, falling back to the sequential loop otherwise:
//  * mean: every partial sum of floats that are multiples of 2^umin is exact in double
//    while sum|x| < 2^(53+umin), so then any order gives the sequential value;
//  * variance: sequential and tree sums of w_i = v_i^2 >= 0 differ by at most
//    (2n+64)*2^-53*sum(w); if both ends of that interval give the same float scale
//    (the map S -> (float)(1/sqrt(S/n+eps)) is monotone) the scale is the reference's.
// `stats` (optional) counts fallbacks: [0] mean, [1] variance.
__global__ void __launch_bounds__(NORM_THREADS) k_norm_exact(const float *__restrict__ X, float *__restrict__ Y, int n,
                                                              const float *__restrict__ gw,
                                                              const float *__restrict__ gb, unsigned *stats) {
  extern __shared__ __attribute__((aligned(16))) float xrow[];
  ln_exact_lds(X + (size_t)blockIdx.x * n, xrow, n, gw, gb, stats);
  float *y = Y + (size_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < n; i += NORM_THREADS) y[i] = xrow[i];
}

// Fast-mode prompt LayerNorm straight to the next GEMM's fp16 operand: the norm + affine of
// one row in LDS (double tree sums, without the exact path's certificate and sequential
// fallbacks: ~3 % of rows, each ~25-50 us of one lane, set this kernel's time), then
// quantize_row_q4_0 per 32-block and the values d*(q-8) as fp16.
// 512 threads: rows up to 8192 take the norm's all-loads-at-once path (4 float4 per thread)
constexpr int NORMQ_THREADS = 512;
__global__ void __launch_bounds__(NORMQ_THREADS) k_norm_f16q(const float *__restrict__ X, _Float16 *__restrict__ Q16,
                                                             int n, const float *__restrict__ gw,
                                                             const float *__restrict__ gb, unsigned *stats) {
  extern __shared__ __attribute__((aligned(16))) float xrow[];
  ln_exact_lds_t<NORMQ_THREADS, false>(X + (size_t)blockIdx.x * n, xrow, n, gw, gb, stats);
  const int lane = threadIdx.x & 63, nb = n / QK;
  _Float16 *q = Q16 + (size_t)blockIdx.x * n;
  for (int b2 = threadIdx.x >> 6; 2 * b2 < nb; b2 += NORMQ_THREADS / 64) {
    const int b = 2 * b2 + (lane >> 5);
    const bool ok = b < nb;  // (uniform per half-wave)
    const float v = ok ? xrow[b * QK + (lane & 31)] : 0.0f;
    float d;
    const int qv = q4_half(v, d);
    if (ok) q[b * QK + (lane & 31)] = f16_of_product(d, (float)(qv - 8));
  }
}

// Per-device health counters, allocated with the device's tables (tables_get): [0] LayerNorm
// mean fallbacks, [1] variance fallbacks (ln_exact_lds), [2] bounded cross-workgroup waits that
// gave up (k_layer_tail, the stream-K finisher, the barrier-free chain GEMV).  A kernel gets the
// counters of the device it runs on.
static unsigned *g_dev_stats[64];
static int current_device() {
  int dev = 0;
  return hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 ? dev : 0;
}
unsigned *dev_stats() { return g_dev_stats[current_device()]; }

int launch_norm(const float *x, float *y, int k, int rows, const float *w, const float *b, hipStream_t s) {
  if (k <= 0 || rows <= 0) { set_error("norm: bad shape"); return VSIM_EINVAL; }
  if ((w == nullptr) != (b == nullptr)) { set_error("norm: affine needs both w and b"); return VSIM_EINVAL; }
  if ((size_t)k * 4 > 64 * 1024) { set_error("norm: row longer than 16384"); return VSIM_EINVAL; }
  hipLaunchKernelGGL(k_norm_exact, dim3(rows), dim3(NORM_THREADS), (size_t)k * 4, s, x, y, k, w, b, dev_stats());
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_norm_f16q(const float *x, void *x16, int k, int rows, const float *w, const float *b, hipStream_t s) {
  if (k <= 0 || rows <= 0 || k % QK || !w || !b) { set_error("norm_f16q: bad shape"); return VSIM_EINVAL; }
  if ((size_t)k * 4 > 64 * 1024) { set_error("norm: row longer than 16384"); return VSIM_EINVAL; }
  hipLaunchKernelGGL(k_norm_f16q, dim3(rows), dim3(NORMQ_THREADS), (size_t)k * 4, s, x, (_Float16 *)x16, k, w, b,
                     dev_stats());
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ GELU via fp16 LUT
// y = fp16->fp32(table_gelu_f16[fp32->fp16(x + bias)])  (bias add fused: ggml_add then
// ggml_gelu, vsim.cpp:680-683)
__global__ void k_gelu(const float *__restrict__ x, float *__restrict__ y, int n, const float *__restrict__ bias,
                       int bias_len, const uint16_t *__restrict__ tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = x[i];
  if (bias) v = v + bias[i % bias_len];
  y[i] = h2f(tab[f2h(v)]);
}

int launch_gelu(const float *x, float *y, int n, const float *bias, int bias_len, hipStream_t s) {
  DevTables t;
  if (int rc = tables_get(&t)) return rc;
  hipLaunchKernelGGL(k_gelu, dim3((n + 255) / 256), dim3(256), 0, s, x, y, n, bias, bias_len, t.gelu_f16);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ adds
// GPT-NeoX parallel residual (vsim.cpp:694-695): inpL = inpL + (attn + ff)
// non-parallel (vsim.cpp:631-657): inpL = ff + inpL — the reference adds only the FF
// output back (the attention output reaches inpL only through the FF LayerNorm input).
__global__ void k_add_residual(float *__restrict__ inpL, const float *__restrict__ attn, const float *__restrict__ ff,
                               int n, int serial) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  inpL[i] = serial ? ff[i] + inpL[i] : inpL[i] + (attn[i] + ff[i]);
}

int launch_add_residual(float *inpL, const float *attn, const float *ff, int n, int serial, hipStream_t s) {
  hipLaunchKernelGGL(k_add_residual, dim3((n + 255) / 256), dim3(256), 0, s, inpL, attn, ff, n, serial);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

__global__ void k_add_bias(float *x, const float *b, int k, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k * n) return;
  x[i] = x[i] + b[i % k];
}

int launch_add_bias(float *x, const float *b, int k, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_add_bias, dim3((k * n + 255) / 256), dim3(256), 0, s, x, b, k, n);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ fp16 tables
// Host-built exactly as ggml_init does (ggml.c:1240-1251: glibc exp/tanh in double,
// then fp32 -> fp16 by the bit-exact converter), uploaded once per device.
static float host_h2f(uint16_t h) {
  const uint32_t w = (uint32_t)h << 16;
  const uint32_t sign = w & 0x80000000u;
  const uint32_t two_w = w + w;
  uint32_t a = (two_w >> 4) + (0xE0u << 23), b = (two_w >> 17) | (126u << 23);
  float fa, fb;
  memcpy(&fa, &a, 4);
  memcpy(&fb, &b, 4);
  const float normalized = fa * 0x1.0p-112f;
  const float denormalized = fb - 0.5f;
  uint32_t rn, rd;
  memcpy(&rn, &normalized, 4);
  memcpy(&rd, &denormalized, 4);
  const uint32_t r = sign | (two_w < (1u << 27) ? rd : rn);
  float f;
  memcpy(&f, &r, 4);
  return f;
}

static uint16_t host_f2h(float f) {
  volatile float base = (fabsf(f) * 0x1.0p+112f);
  base = base * 0x1.0p-110f;
  uint32_t w;
  memcpy(&w, &f, 4);
  const uint32_t shl1_w = w + w;
  const uint32_t sign = w & 0x80000000u;
  uint32_t bias = shl1_w & 0xFF000000u;
  if (bias < 0x71000000u) bias = 0x71000000u;
  const uint32_t bb = (bias >> 1) + 0x07800000u;
  float fb;
  memcpy(&fb, &bb, 4);
  const float sum = fb + base;
  uint32_t bits;
  memcpy(&bits, &sum, 4);
  const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
  const uint32_t mantissa_bits = bits & 0x00000FFFu;
  const uint32_t nonsign = exp_bits + mantissa_bits;
  return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

static float host_gelu(float x) {
  const double A = 0.044715, S = 0.79788456;
  return 0.5 * x * (1.0 + tanh(S * x * (1.0 + A * x * x)));
}

static std::mutex g_tab_mu;
static std::vector<uint16_t> g_exp_host, g_gelu_host;
static DevTables g_dev_tab[64];
static bool g_dev_tab_ok[64];

static void build_host_tables() {
  if (!g_exp_host.empty()) return;
  g_exp_host.resize(65536);
  g_gelu_host.resize(65536);
  for (int i = 0; i < 65536; ++i) {
    const float f = host_h2f((uint16_t)i);
    g_gelu_host[i] = host_f2h(host_gelu(f));
    g_exp_host[i] = host_f2h((float)exp((double)f));
  }
}

int tables_get(DevTables *t) {
  int dev = 0;
  VSIM_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tab_mu);
  if (dev < 0 || dev >= 64) { set_error("tables: device id out of range"); return VSIM_EINVAL; }
  if (!g_dev_tab_ok[dev]) {
    build_host_tables();
    uint16_t *p = nullptr;
    VSIM_HIP(hipMalloc(&p, 2 * 65536 * sizeof(uint16_t)));
    VSIM_HIP(hipMemcpy(p, g_exp_host.data(), 65536 * 2, hipMemcpyHostToDevice));
    VSIM_HIP(hipMemcpy(p + 65536, g_gelu_host.data(), 65536 * 2, hipMemcpyHostToDevice));
    g_dev_tab[dev].exp_f16 = p;
    g_dev_tab[dev].gelu_f16 = p + 65536;
    g_dev_tab_ok[dev] = true;
    if (!g_dev_stats[dev]) {
      VSIM_HIP(hipMalloc(&g_dev_stats[dev], 4 * sizeof(unsigned)));
      VSIM_HIP(hipMemset(g_dev_stats[dev], 0, 4 * sizeof(unsigned)));
    }
  }
  *t = g_dev_tab[dev];
  return VSIM_OK;
}

int tables_host(uint16_t *exp_f16, uint16_t *gelu_f16) {
  std::lock_guard<std::mutex> lk(g_tab_mu);
  build_host_tables();
  memcpy(exp_f16, g_exp_host.data(), 65536 * 2);
  memcpy(gelu_f16, g_gelu_host.data(), 65536 * 2);
  return VSIM_OK;
}

static thread_local unsigned *t_err_target = nullptr;
static std::atomic<unsigned> g_model_spins{0};
unsigned *set_spin_error_target(unsigned *p) {
  unsigned *o = t_err_target;
  t_err_target = p;
  return o;
}
void add_model_spin_timeouts(unsigned n) { g_model_spins += n; }
unsigned *spin_error_counter() {
  if (t_err_target) return t_err_target;
  unsigned *st = dev_stats();
  return st ? st + 2 : nullptr;
}

// counter k summed over every device that has one (hipMemcpy of a device word: a full sync of
// that device's null stream, so call after the work to be checked has been synchronized)
static int stats_sum(int k, unsigned *out) {
  *out = 0;
  int cur = 0;
  VSIM_HIP(hipGetDevice(&cur));
  for (int dev = 0; dev < 64; ++dev) {
    if (!g_dev_stats[dev]) continue;
    unsigned v = 0;
    VSIM_HIP(hipSetDevice(dev));
    VSIM_HIP(hipMemcpy(&v, g_dev_stats[dev] + k, sizeof(unsigned), hipMemcpyDeviceToHost));
    *out += v;
  }
  VSIM_HIP(hipSetDevice(cur));
  return VSIM_OK;
}
int spin_timeouts(unsigned *out) {  // the devices' counters and every model's (spin_check)
  const int rc = stats_sum(2, out);
  *out += g_model_spins.load();
  return rc;
}

int norm_stats(unsigned *out2) {
  const int rc = stats_sum(0, &out2[0]);
  if (rc != VSIM_OK) return rc;
  return stats_sum(1, &out2[1]);
}

// ------------------------------------------------------------------ greedy argmax
// Index of the largest logit with numpy.argmax's conventions: the first index among equal
// maxima (-0.0 equal to +0.0), and the first NaN if there is one.  Each value and its index
// become one 64-bit key whose unsigned order is that order: the value's bits mapped to an
// unsigned order (NaN -> all ones, -0.0 -> +0.0) above ~index.  The workgroups reduce their
// keys, fold them into ws[0] with one 64-bit atomic max each, then count themselves in ws[1];
// the last to count reads the result and zeroes ws for the next launch.  r05: the single
// 1024-thread workgroup this replaced pulled the whole 50k-logit row through one CU, 14.45 us
// per token (profiles/r05_exact_kernel_stats.csv).
__device__ __forceinline__ unsigned long long am_key(float v, int i) {
  uint32_t u = __float_as_uint(v);
  if (v != v) u = 0xFFFFFFFFu;
  else if (v == 0.0f) u = 0x80000000u;
  else u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (0xFFFFFFFFu - (uint32_t)i);
}
constexpr int AM_T = 256, AM_MAX_WG = 64;
static int am_grid(const float *x, int n) {
  const int n4 = ((uintptr_t)x & 15) ? 0 : n / 4;
  const int per = n4 > n - 4 * n4 ? n4 : n - 4 * n4;  // float4 items or scalar items, whichever the grid walks more
  const int g = (per + AM_T - 1) / AM_T;
  return g < 1 ? 1 : g > AM_MAX_WG ? AM_MAX_WG : g;
}
// GEN: the device-resident greedy loop's epilogue -- the token also becomes the next step's
// input (tok), is recorded at hist[n_past] and n_past advances (k_argmax is the last kernel
// of the step, so every reader of n_past has run).
template <bool GEN>
__global__ void __launch_bounds__(AM_T) k_argmax(const float *__restrict__ x, int n, int *__restrict__ out,
                                                 unsigned long long *ws, int *tok, int *npast, int *hist) {
  __shared__ unsigned long long sk[AM_T / 64];
  unsigned long long best = 0;
  const int n4 = ((uintptr_t)x & 15) ? 0 : n / 4;
  const int gt = blockIdx.x * AM_T + threadIdx.x, nt = gridDim.x * AM_T;
  const float4 *x4 = (const float4 *)x;
  for (int i = gt; i < n4; i += nt) {
    const float4 v = x4[i];
    best = max(best, am_key(v.x, 4 * i));
    best = max(best, am_key(v.y, 4 * i + 1));
    best = max(best, am_key(v.z, 4 * i + 2));
    best = max(best, am_key(v.w, 4 * i + 3));
  }
  for (int i = 4 * n4 + gt; i < n; i += nt) best = max(best, am_key(x[i], i));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) best = max(best, (unsigned long long)__shfl_xor(best, o, 64));
  if ((threadIdx.x & 63) == 0) sk[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int w = 1; w < AM_T / 64; ++w) best = max(best, sk[w]);
  unsigned *cnt = (unsigned *)(ws + 1);
  // The hand-off is the first row of MI355X_MICROARCH.md's sc1 hand-off table, with the atomic max
  // as the payload store: one lane per workgroup performs its max (an agent-scope atomic, performed
  // at the device-coherent level like an sc1 store) and drains it (vmcnt(0)) before its one add to
  // the unsharded counter; the workgroup whose add returns gridDim.x - 1 reads ws with an sc1 load
  // only after that add returned.  No fence: relaxed atomics are not ordered by the memory model,
  // so this relies on the measured gfx950 behaviour the table records (a drained device-scope
  // atomic is visible to a later sc1 load from any XCD), as k_layer_tail's hand-offs do.
  __hip_atomic_fetch_max(ws, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the max is performed before this workgroup counts
  if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gridDim.x - 1) return;
  const unsigned long long k = __hip_atomic_load(ws, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int bi = (int)(0xFFFFFFFFu - (uint32_t)k);
  *out = bi;
  if (GEN) {
    const int np = *npast;
    *tok = bi;
    hist[np] = bi;
    *npast = np + 1;
  }
  __hip_atomic_store(ws, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int launch_argmax(const float *x, int n, int *out, unsigned long long *ws, hipStream_t s) {
  if (n <= 0) { set_error("argmax: empty row"); return VSIM_EINVAL; }
  hipLaunchKernelGGL(k_argmax<false>, dim3(am_grid(x, n)), dim3(AM_T), 0, s, x, n, out, ws, nullptr, nullptr, nullptr);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_argmax_gen(const float *x, int n, int *out, unsigned long long *ws, int *tok, int *npast, int *hist,
                      hipStream_t s) {
  if (n <= 0) { set_error("argmax: empty row"); return VSIM_EINVAL; }
  hipLaunchKernelGGL(k_argmax<true>, dim3(am_grid(x, n)), dim3(AM_T), 0, s, x, n, out, ws, tok, npast, hist);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
