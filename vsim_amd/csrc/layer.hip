// vsim_amd/csrc/layer.hip — fused kernels of the single-token decode step.
//
// One decoder layer = 4 launches (vsim.cpp:521-696 for GPT-NeoX with parallel residual,
// the same ops for GPT-J):
//   1. k_ln_quant      LayerNorm(s) + affine + activation quantization (ggml.c:4246,
//                      5024-5041): inpL -> Q4_0 activation row(s) and their xd factors
//   2. GEMV batch      {Q, K, V, fc_in} in one launch; fc_in's epilogue adds the bias, looks
//                      up GELU and quantizes each 32-row tile into the fc_out activation
//   3. k_attn_decode   per head: RoPE on q and the new k, KV-cache write, KQ (double
//                      accumulator), scale/softmax (fp16 exp table), KQV (sequential float
//                      mad), quantize the head's output for the out-projection
//   4. dual GEMV       out-projection and fc_out for the same 32 rows in one workgroup,
//                      epilogue inpL += (attn + ff)  (vsim.cpp:694-695)
// Every value is computed with the reference's operation order and rounding (exact mode);
// the fast mode swaps in the integer-dot GEMV bodies.  n_past is read from device memory so
// the whole step can be captured once in a hipGraph and replayed per token.
#include <cstdlib>

#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

extern unsigned *g_norm_stats;

// ------------------------------------------------------------------ 1. LN + quantize
// One 1024-thread workgroup per LayerNorm (two for GPT-NeoX's parallel-residual pair); the
// normalized row is quantized by whole waves, two 32-blocks per wave step.
constexpr int LNQ_THREADS = 1024;
__device__ unsigned long long g_ln_prof[8];  // timing experiment output (VSIM_LN_DBG)

template <bool PROF>
__global__ void __launch_bounds__(LNQ_THREADS) k_ln_quant(LnQuantJob j0, LnQuantJob j1, int n, unsigned *stats) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  const LnQuantJob &J = blockIdx.x == 0 ? j0 : j1;
  unsigned long long *prof = PROF && blockIdx.x == 0 ? g_ln_prof : nullptr;
  ln_exact_lds_t<LNQ_THREADS>(J.x, row, n, J.w, J.b, stats, J.ja, J.jab, J.jf, J.jfb, J.jout, prof);
  const int nb = n / QK, lane = threadIdx.x & 63;
  for (int b2 = threadIdx.x >> 6; 2 * b2 < nb; b2 += LNQ_THREADS / 64) {
    const int b = 2 * b2 + (lane >> 5);
    const bool ok = b < nb;
    const float v = ok ? row[b * QK + (lane & 31)] : 0.0f;
    quantize_half(v, lane, ok, J.qs + (size_t)b * 16, J.d + b, J.xd + (size_t)b * QK);
  }
  if (PROF && blockIdx.x == 0 && threadIdx.x == 0) g_ln_prof[6] = __builtin_amdgcn_s_memtime();
}

int launch_ln_quant(const LnQuantJob &j0, const LnQuantJob *j1, int n, hipStream_t s) {
  static const bool prof = getenv("VSIM_LN_DBG") != nullptr;
  if (prof)
    hipLaunchKernelGGL(k_ln_quant<true>, dim3(j1 ? 2 : 1), dim3(LNQ_THREADS), (size_t)n * 4, s, j0, j1 ? *j1 : j0,
                       n, g_norm_stats);
  else
    hipLaunchKernelGGL(k_ln_quant<false>, dim3(j1 ? 2 : 1), dim3(LNQ_THREADS), (size_t)n * 4, s, j0,
                       j1 ? *j1 : j0, n, g_norm_stats);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

__global__ void k_residual_join(const float *x, const float *a, const float *ab, const float *f, const float *fb,
                                float *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float attn = ab ? a[i] + ab[i] : a[i];
  out[i] = x[i] + (attn + (f[i] + fb[i]));
}

int launch_residual_join(const float *x, const float *a, const float *ab, const float *f, const float *fb, float *out,
                         int n, hipStream_t s) {
  hipLaunchKernelGGL(k_residual_join, dim3((n + 255) / 256), dim3(256), 0, s, x, a, ab, f, fb, out, n);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ GEMV epilogues
// Called by all 64 lanes of wave 0 with the row sums in lanes 0..31.
__device__ __forceinline__ void gemv_epilogue(const GemvJob &J, int t, float s, int lane) {
  const int row = t * T32 + lane;
  if (J.epi == EPI_GELU_Q) {
    float g = 0.0f;
    if (lane < T32) {
      const float v = s + J.bias[row];
      g = h2f(J.gelu_tab[f2h(v)]);
      if (J.y) J.y[row] = g;
    }
    quantize_block_lanes(g, lane, J.oq_qs + (size_t)t * 16, J.oq_d + t, J.oxd + (size_t)t * QK);
  } else if (lane < T32 && row < J.w.rows) {
    J.y[row] = J.bias ? s + J.bias[row] : s;
  }
}

// ------------------------------------------------------------------ fast GEMV + epilogues
constexpr int FW = 8;  // waves per workgroup of the fast kernels
__global__ void __launch_bounds__(64 * FW) k_gemv_fast_epi(GemvBatch B) {
  __shared__ float part[FW * 2][T32];
  int t = blockIdx.x, ji = 0;
  while (ji + 1 < B.nj && t >= B.j[ji].w.tiles) { t -= B.j[ji].w.tiles; ++ji; }
  const GemvJob &J = B.j[ji];
  const int nb = J.w.nb();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & (T32 - 1), h = lane >> 5;
  const uint8_t *qs = J.w.qs + (size_t)t * nb * T32 * 16;
  const float *dd = J.w.d + (size_t)t * nb * T32;
  float acc = 0.0f;
  for (int b = 2 * wave + h; b < nb; b += 2 * FW) {
    const size_t o = (size_t)b * T32 + r;
    const uint4 q = *(const uint4 *)(qs + o * 16);
    const float d0 = dd[o];
    const uint4 xv = *(const uint4 *)(J.xqs + (size_t)b * 16);
    int sd = __builtin_amdgcn_sdot8((int)(q.x ^ 0x88888888u), (int)(xv.x ^ 0x88888888u), 0, false);
    sd = __builtin_amdgcn_sdot8((int)(q.y ^ 0x88888888u), (int)(xv.y ^ 0x88888888u), sd, false);
    sd = __builtin_amdgcn_sdot8((int)(q.z ^ 0x88888888u), (int)(xv.z ^ 0x88888888u), sd, false);
    sd = __builtin_amdgcn_sdot8((int)(q.w ^ 0x88888888u), (int)(xv.w ^ 0x88888888u), sd, false);
    acc = __builtin_fmaf(d0 * J.xdd[b], (float)sd, acc);
  }
  part[2 * wave + h][r] = acc;
  __syncthreads();
  if (wave == 0) {
    float sum = 0.0f;
    if (lane < T32) {
#pragma unroll
      for (int i = 0; i < 2 * FW; ++i) sum += part[i][lane];
    }
    gemv_epilogue(J, t, sum, lane);
  }
}

int launch_gemv_epi(const GemvBatch &B, int mode, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < B.nj; ++i) tiles += B.j[i].w.tiles;
  if (mode == VSIM_MODE_EXACT) return launch_gemv_chain_batch(B, s);  // gemv_chain.hip
  hipLaunchKernelGGL(k_gemv_fast_epi, dim3(tiles), dim3(64 * FW), 0, s, B);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ 3. attention (N = 1)
// One 1024-thread workgroup per head.  KQ: one wave per key, products over the head
// dimension summed as a tree in double; the reference's sequential double sum lies within
// 2*d*2^-53*sum|p| of it, so when both ends of that interval round to the same float the
// score is the reference's, otherwise lane 0 redoes the key sequentially (ggml.c:4760-4800
// for the f32 dot with a double accumulator).  KQV keeps the reference's sequential float
// chain over the keys, one chain per output element.
constexpr int ATT_THREADS = 1024;
constexpr int ATT_WAVES = ATT_THREADS / 64;
constexpr int ATT_KB = 4;   // keys per wave per load group
constexpr int ATT_DPL = 4;  // max head-dim elements per lane (d <= 256)

__global__ void __launch_bounds__(ATT_THREADS) k_attn_decode(AttnJob A) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int h = blockIdx.x, d = A.d, E = A.d * A.H;
  const int n_past = *A.npast;
  const int nk = n_past + 1;
  float *qh = sm;           // [d]
  float *kh = sm + d;       // [d]
  float *pr = sm + 2 * d;   // [nk] scores / probabilities
  __shared__ float shf[ATT_WAVES];
  __shared__ double shd[ATT_WAVES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < d; i += ATT_THREADS) {
    qh[i] = A.q[h * d + i];
    kh[i] = A.k[h * d + i];
    A.vc[(size_t)n_past * E + h * d + i] = A.v[h * d + i];
  }
  __syncthreads();
  // RoPE (ggml.c:6117-6152 / 5952-5973), position p = n_past for both q (mode 0) and k
  const int half = A.n_rot / 2;
  for (int j = tid; j < half; j += ATT_THREADS) {
    const double2 c = A.cs[(size_t)n_past * half + j];
    const int i0 = A.style == 0 ? j : 2 * j, i1 = A.style == 0 ? j + half : 2 * j + 1;
    const double q0 = qh[i0], q1 = qh[i1], k0 = kh[i0], k1 = kh[i1];
    if (A.style == 0) {
      qh[i0] = (float)(c.x * q0 - c.y * q1);
      qh[i1] = (float)(c.x * q1 + c.y * q0);
      kh[i0] = (float)(c.x * k0 - c.y * k1);
      kh[i1] = (float)(c.x * k1 + c.y * k0);
    } else {
      qh[i0] = (float)(q0 * c.x - q1 * c.y);
      qh[i1] = (float)(q0 * c.y + q1 * c.x);
      kh[i0] = (float)(k0 * c.x - k1 * c.y);
      kh[i1] = (float)(k0 * c.y + k1 * c.x);
    }
  }
  __syncthreads();
  for (int i = tid; i < d; i += ATT_THREADS) A.kc[(size_t)n_past * E + h * d + i] = kh[i];
  // KQ[k] = (float) sum_i (double)(K[k][i] * q[i]) in order i = 0..d-1; then * scale.
  // Each wave takes keys in groups of ATT_KB and loads the whole group before reducing, so
  // the cache reads of a group overlap (one wave per key would pay the latency per key).
  float mx = -INFINITY;
  for (int k0 = wid * ATT_KB; k0 < nk; k0 += ATT_WAVES * ATT_KB) {
    float kv[ATT_KB][ATT_DPL];
#pragma unroll
    for (int j = 0; j < ATT_KB; ++j) {
      const int k = min(k0 + j, nk - 1);
      const float *kr = k == n_past ? kh : A.kc + (size_t)k * E + h * d;
#pragma unroll
      for (int e = 0; e < ATT_DPL; ++e) {
        const int i = lane + 64 * e;
        kv[j][e] = i < d ? kr[i] : 0.0f;
      }
    }
#pragma unroll
    for (int j = 0; j < ATT_KB; ++j) {
      const int k = k0 + j;
      if (k >= nk) break;  // wave-uniform
      double t = 0.0, ta = 0.0;
#pragma unroll
      for (int e = 0; e < ATT_DPL; ++e) {
        const int i = lane + 64 * e;
        if (i < d) {
          const double p = (double)(kv[j][e] * qh[i]);
          t += p;
          ta += fabs(p);
        }
      }
      t = wave_sum_d(t);
      ta = wave_sum_d(ta);
      const double bnd = 2.0 * d * 0x1.0p-53 * ta;
      float sc = (float)(t - bnd);
      if (sc != (float)(t + bnd)) {  // wave-uniform: redo this key in the reference order
        const float *kr = k == n_past ? kh : A.kc + (size_t)k * E + h * d;
        double acc = 0.0;
        if (lane == 0)
          for (int i = 0; i < d; ++i) acc += (double)(kr[i] * qh[i]);
        sc = (float)__shfl(acc, 0, 64);
      }
      sc = sc * A.scale;
      if (lane == 0) pr[k] = sc;
      mx = mx > sc ? mx : sc;
    }
  }
  // max, exp via table, exact double sum (fp16 values: any order), 1/sum
  mx = wave_max_f(mx);
  if (lane == 0) shf[wid] = mx;
  __syncthreads();
  mx = shf[0];
  for (int w = 1; w < ATT_WAVES; ++w) mx = mx > shf[w] ? mx : shf[w];
  double sum = 0.0;
  for (int k = tid; k < nk; k += ATT_THREADS) {
    const float val = h2f(A.etab[f2h(pr[k] - mx)]);
    pr[k] = val;
    sum += (double)val;
  }
  sum = wave_sum_d(sum);
  if (lane == 0) shd[wid] = sum;
  __syncthreads();
  sum = 0.0;
  for (int w = 0; w < ATT_WAVES; ++w) sum += shd[w];
  const float inv = (float)(1.0 / sum);
  for (int k = tid; k < nk; k += ATT_THREADS) pr[k] = pr[k] * inv;
  __syncthreads();
  // KQV: y[dd] = sum_k V[k][dd] * p[k], sequential float chain from 0.0f; V rows loaded
  // 16 keys ahead of the chain
  for (int dd0 = 0; dd0 < d; dd0 += ATT_THREADS) {
    const int dd = dd0 + tid;
    float y = 0.0f;
    if (dd < d) {
      const float *vcol = A.vc + h * d + dd;
      int k = 0;
      for (; k + 16 <= nk; k += 16) {
        float vv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) vv[j] = vcol[(size_t)(k + j) * E];
#pragma unroll
        for (int j = 0; j < 16; ++j) y = y + vv[j] * pr[k + j];
      }
      for (; k < nk; ++k) y = y + vcol[(size_t)k * E] * pr[k];
      if (A.out) A.out[h * d + dd] = y;
    }
    // quantize the head's outputs, two 32-blocks per wave
    if (dd0 + wid * 64 < d) {
      const int blk = (h * d + dd0 + wid * 64) / QK + (lane >> 5);
      const bool ok = dd0 + wid * 64 + (lane & ~31) < d;
      quantize_half(y, lane, ok, A.oq_qs + (size_t)blk * 16, A.oq_d + blk, A.oxd + (size_t)blk * QK);
    }
  }
}

int launch_attn_decode(const AttnJob &A, int n_ctx, hipStream_t s) {
  if (A.d % 32 != 0 || A.d > 64 * ATT_DPL) {
    set_error("attention: head dim must be a multiple of 32, at most 256");
    return VSIM_EINVAL;
  }
  const size_t smem = (size_t)(2 * A.d + n_ctx) * sizeof(float);
  hipLaunchKernelGGL(k_attn_decode, dim3(A.H), dim3(ATT_THREADS), smem, s, A);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim

extern "C" int vsim_debug_ln_prof(unsigned long long *out8) {
  return hipMemcpyFromSymbol(out8, HIP_SYMBOL(vsim::g_ln_prof), sizeof(vsim::g_ln_prof)) == hipSuccess ? 0 : -1;
}
