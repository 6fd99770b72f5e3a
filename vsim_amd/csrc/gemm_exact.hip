// vsim_amd/csrc/gemm_exact.hip — exact-mode Q4_0 GEMM for prompt batches (N > 1 tokens).
//
// The reference computes every (row, token) of a prompt mul_mat as its own sequential fp32
// chain (imax.c:1182-1230, ggml_vec_dot_q4_0 ggml.c:472-511, over the INIT-phase Q4_0 rows of
// ggml.c:5024-5041):
//     sumf = 0;  for each byte pair p in order:  sumf = sumf + (f0*f2 + f1*f3)
// with f0/f1 = d_w*(n-8) of the weight's two nibbles and f2/f3 = d_x*(m-8) of the activation's,
// every product and sum rounded on its own (no FMA).  The chains cannot be re-associated, but
// there are M x N of them, so a prompt batch is a plain register-tiled SIMT GEMM whose K loop
// runs in the reference's order: each lane owns an 8 x 8 block of (row, token) chains and adds
// one pair term to each of its 64 accumulators per step.  The bound is VALU issue (2 fp32 ops
// per weight-token: two products, their sum and the chain add per pair), not HBM or LDS.
//
// Per K-chunk of one Q4_0 block (16 pairs) a workgroup stages in LDS:
//   w[p][row] = (f0, f1)  -- the weight dequantized once per chunk (d*(n-8), one rounding,
//                            as dequantize_row_q4_0 / the reference dot form it)
//   x[p][tok] = (f2, f3)  -- the activation factors xd (pair-interleaved in HBM, kern.hpp)
// The next chunk's raw weight nibbles, scales and factors are loaded into registers while the
// current one is computed (one LDS stage, two barriers per chunk of ~16 x 256 VALU ops).
#include "kern.hpp"

namespace vsim {

template <int BM, int BN>
struct GxShape {
  static constexpr int TX = BM / 8, TY = BN / 8, THREADS = TX * TY;
  static constexpr int PAIRS = QK / 2;
  static constexpr int WT = 2 * BM / THREADS;  // weight (row, half-block) tasks per thread
  static constexpr int XT = 2 * BN / THREADS;  // activation (token, half-block) tasks per thread
  static_assert(2 * BM % THREADS == 0 && 2 * BN % THREADS == 0, "loader tasks");
  static_assert(THREADS % 64 == 0, "whole waves");
};

template <int BM, int BN>
__global__ void __launch_bounds__(BM * BN / 64)
    k_gemm_exact(W4 W, const float *__restrict__ xd, int N, const float *__restrict__ bias, float *__restrict__ y) {
  using S = GxShape<BM, BN>;
  __shared__ __attribute__((aligned(16))) float2 Lw[S::PAIRS][BM];
  __shared__ __attribute__((aligned(16))) float2 Lx[S::PAIRS][BN];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int M = W.rows, K = W.k, nb = W.nb();
  const int rows_alloc = W.tiles * T32;

  // ---- loaders: task t -> (row or token t % B, half t / B of the block: pairs 8h .. 8h+7)
  const uint8_t *wq[S::WT];
  const float *wd[S::WT];
  const float *xp[S::XT];
#pragma unroll
  for (int u = 0; u < S::WT; ++u) {
    const int t = tid + u * S::THREADS, r = min(m0 + t % BM, rows_alloc - 1), h = t / BM;
    const size_t o = W.off(r, 0);  // block b of row r: o + b * T32
    wq[u] = W.qs + o * 16 + 8 * h;
    wd[u] = W.d + o;
  }
#pragma unroll
  for (int u = 0; u < S::XT; ++u) {
    const int t = tid + u * S::THREADS, n = min(n0 + t % BN, N - 1), h = t / BN;
    xp[u] = xd + (size_t)n * K + 16 * h;
  }
  uint2 rq[S::WT];
  float rd[S::WT];
  f32x4 rx[S::XT][4];
  auto fetch = [&](int b) {
#pragma unroll
    for (int u = 0; u < S::WT; ++u) {
      rq[u] = *(const uint2 *)(wq[u] + (size_t)b * (T32 * 16));
      rd[u] = wd[u][(size_t)b * T32];
    }
#pragma unroll
    for (int u = 0; u < S::XT; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) rx[u][g] = *(const f32x4 *)(xp[u] + (size_t)b * QK + 4 * g);
  };
  auto stage = [&]() {
#pragma unroll
    for (int u = 0; u < S::WT; ++u) {
      const int t = tid + u * S::THREADS, i = t % BM, h = t / BM;
      const uint32_t qw[2] = {rq[u].x, rq[u].y};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t byte = (qw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        // d0*(float)(n-8): one rounding (imax.c:1219-1222)
        Lw[8 * h + j][i] = make_float2(rd[u] * (float)((int)(byte & 0xF) - 8), rd[u] * (float)((int)(byte >> 4) - 8));
      }
    }
#pragma unroll
    for (int u = 0; u < S::XT; ++u) {
      const int t = tid + u * S::THREADS, i = t % BN, h = t / BN;
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // (x0, x2, x1, x3) of 4 elements -> pairs (x0, x1), (x2, x3)
        Lx[8 * h + 2 * g][i] = make_float2(rx[u][g].x, rx[u][g].z);
        Lx[8 * h + 2 * g + 1][i] = make_float2(rx[u][g].y, rx[u][g].w);
      }
    }
  };

  // ---- compute: rows tx*4 + {0..3} and BM/2 + tx*4 + {0..3}, tokens likewise with ty
  const int tx = tid % S::TX, ty = tid / S::TX;
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;

  if (nb > 0) fetch(0);
  for (int b = 0; b < nb; ++b) {
    __syncthreads();  // the previous chunk's reads are done
    stage();
    __syncthreads();
    if (b + 1 < nb) fetch(b + 1);
#pragma unroll 2
    for (int p = 0; p < S::PAIRS; ++p) {
      f32x4 wv[4], xv[4];  // (f0, f1) of 2 rows per vector; (f2, f3) of 2 tokens per vector
      const f32x4 *w4 = (const f32x4 *)&Lw[p][0];
      const f32x4 *x4 = (const f32x4 *)&Lx[p][0];
      wv[0] = w4[2 * tx];
      wv[1] = w4[2 * tx + 1];
      wv[2] = w4[BM / 4 + 2 * tx];
      wv[3] = w4[BM / 4 + 2 * tx + 1];
      xv[0] = x4[2 * ty];
      xv[1] = x4[2 * ty + 1];
      xv[2] = x4[BN / 4 + 2 * ty];
      xv[3] = x4[BN / 4 + 2 * ty + 1];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float f0 = (i & 1) ? wv[i >> 1].z : wv[i >> 1].x;
        const float f1 = (i & 1) ? wv[i >> 1].w : wv[i >> 1].y;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f2 = (j & 1) ? xv[j >> 1].z : xv[j >> 1].x;
          const float f3 = (j & 1) ? xv[j >> 1].w : xv[j >> 1].y;
          acc[i][j] = acc[i][j] + (f0 * f2 + f1 * f3);  // sumf += f0*f2 + f1*f3
        }
      }
    }
  }

  // ---- epilogue: y[n][m] (+ bias[m]), four consecutive rows per store
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = n0 + (j < 4 ? 4 * ty + j : BN / 2 + 4 * ty + j - 4);
    if (n >= N) continue;
    float *yr = y + (size_t)n * M;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int r = m0 + hh * (BM / 2) + 4 * tx;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = bias && r + i < M ? acc[4 * hh + i][j] + bias[r + i] : acc[4 * hh + i][j];
      if (r + 3 < M && (M & 3) == 0) {
        *(f32x4 *)(yr + r) = f32x4{v[0], v[1], v[2], v[3]};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r + i < M) yr[r + i] = v[i];
      }
    }
  }
}

// y[n][m] = exact Q4_0 dot of weight row m and activation row n (+ bias[m]) for n < N, every
// (m, n) the reference's chain; xd: [N][K] activation factors (pair-interleaved, kern.hpp)
int launch_gemm_exact(const W4 &W, const float *xd, int n, const float *bias, float *y, hipStream_t s) {
  if (W.k % QK || W.rows <= 0 || n <= 0 || !xd) {
    set_error("gemm_exact: bad shape or missing activation factors");
    return VSIM_EINVAL;
  }
  constexpr int BM = 128, BN = 128;
  hipLaunchKernelGGL((k_gemm_exact<BM, BN>), dim3((W.rows + BM - 1) / BM, (n + BN - 1) / BN),
                     dim3(GxShape<BM, BN>::THREADS), 0, s, W, xd, n, bias, y);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
