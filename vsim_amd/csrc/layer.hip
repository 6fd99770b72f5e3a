// vsim_amd/csrc/layer.hip — fused kernels of the single-token decode step.
//
// One decoder layer (vsim.cpp:521-696 for GPT-NeoX with parallel residual, the same ops for
// GPT-J) = 2 launches in exact mode since r06 (3 for layer 0 and the serial fallback):
//   1. k_ln_quant      (the previous layer's residual join +) LayerNorm(s) + affine +
//                      activation quantization (ggml.c:4246, 5024-5041): inpL -> Q4_0
//                      activation row(s) and their xd factors; layer 0 only when the tail
//                      runs the next LayerNorm itself (gemv_chain.hip, TailLn)
//   2. GEMV batch      {fc_in, Q, K, V} in one launch; fc_in's epilogue adds the bias, looks
//                      up GELU and quantizes each 32-row tile into the fc_out activation
//   3. k_layer_tail    (gemv_chain.hip) fc_out beside the attention heads (attn.hpp: RoPE,
//                      KV-cache write, KQ with a double accumulator, scale/softmax with the
//                      fp16 exp table, KQV as a sequential float chain, quantization) and the
//                      out-projection; k_attn_decode below is the same head as its own launch
//                      for contexts whose scores do not fit the tail's LDS
// Every value is computed with the reference's operation order and rounding (exact mode);
// the fast mode swaps in the integer-dot GEMV bodies.  n_past is read from device memory so
// the whole step can be captured once in a hipGraph and replayed per token.
#include <cstdlib>

#include "attn.hpp"
#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

// ------------------------------------------------------------------ 1. LN + quantize
// One 1024-thread workgroup per LayerNorm (two for GPT-NeoX's parallel-residual pair); the
// normalized row is quantized by whole waves, two 32-blocks per wave step.
constexpr int LNQ_THREADS = 512;

// LNQ_SPLIT workgroups per LayerNorm: each computes the whole row's statistics (the row is
// 16 KB, read from L2) and normalizes, writes and quantizes one slice of LNQ_SPLIT, so the
// latency-bound per-element phases run on LNQ_SPLIT CUs.
constexpr int LNQ_SPLIT = 8;
__global__ void __launch_bounds__(LNQ_THREADS) k_ln_quant(LnQuantJob j0, LnQuantJob j1, int n, unsigned *stats) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  const int part = blockIdx.x % LNQ_SPLIT;
  const LnQuantJob &J = blockIdx.x < LNQ_SPLIT ? j0 : j1;
  if (blockIdx.x == 0 && threadIdx.x == 0 && J.ep) *J.ep += 1u;
  const int nb = n / QK;
  const int b0 = part * nb / LNQ_SPLIT, b1 = (part + 1) * nb / LNQ_SPLIT;  // this slice's blocks
  ln_quant_job<LNQ_THREADS>(J, row, n, part == 0 ? stats : nullptr, b0, b1);
}

int launch_ln_quant(const LnQuantJob &j0, const LnQuantJob *j1, int n, hipStream_t s) {
  const dim3 grid((j1 ? 2 : 1) * LNQ_SPLIT);
  hipLaunchKernelGGL(k_ln_quant, grid, dim3(LNQ_THREADS), (size_t)n * 4, s, j0, j1 ? *j1 : j0, n, dev_stats());
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

__global__ void k_residual_join(const float *x, const float *a, const float *ab, const float *f, const float *fb,
                                float *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float ff = f[i] + fb[i];
  if (!a) {  // serial residual: x + (ff + b)
    out[i] = x[i] + ff;
    return;
  }
  const float attn = ab ? a[i] + ab[i] : a[i];
  out[i] = x[i] + (attn + ff);
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
// attn.hpp; one 1024-thread workgroup per head
constexpr int ATT_THREADS = 1024;
__global__ void __launch_bounds__(ATT_THREADS) k_attn_decode(AttnJob A) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  attn_body<ATT_THREADS>(A, blockIdx.x, sm);
}

int launch_attn_decode(const AttnJob &A, int n_ctx, hipStream_t s) {
  const int S = A.nsplit > 1 ? A.nsplit : 1;
  if (A.d % 32 != 0 || A.d > 256 || A.n_ctx != n_ctx || A.d % S != 0 || (A.d / S) % QK != 0) {
    set_error("attention: head dim must be a multiple of 32, at most 256");
    return VSIM_EINVAL;
  }
  const size_t smem = (size_t)attn_lds_floats(A.d, n_ctx) * sizeof(float);
  hipLaunchKernelGGL(k_attn_decode, dim3(A.H * S), dim3(ATT_THREADS), smem, s, A);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
