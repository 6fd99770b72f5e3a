// vsim_amd/csrc/attn_prefill.hip — prompt (prefill) attention on fp16 MFMA, fast mode.
//
// For N > 1 tokens at n_past, the reference computes KQ = K·Q (ggml.c:4495-4534), scale,
// causal mask (key > n_past + query -> -inf), softmax over the keys (5825-5893) and
// KQV = V·softmax (4535-4581) per head.  This kernel does the same in one pass with an
// online softmax (flash attention): no [H][N][n_past+N] score tensor, K and V read once
// per 128 queries.  It is the throughput path for long prompts (codegen-16B, N = 2048),
// in the fast mode with the fp16 MFMA GEMM (gemm_f16.hip); exact mode keeps the
// reference-order kernels of ops_attn.hip.
//
// One workgroup = one head x 128 queries, 4 waves of 32 queries; keys in blocks of 64.
//  * S^T = K·Q^T on v_mfma_f32_32x32x16_f16: keys are the tile's rows (in registers),
//    queries its columns (one per lane), so each query's softmax statistics are a
//    reduction over the lane's own registers plus one exchange with lane ^ 32.  Q comes
//    pre-scaled by scale * log2(e) (fp16 fragments in registers for the whole loop), so
//    p = exp2(s - max).
//  * O^T += V^T·P^T: P^T is the S^T accumulator itself, converted to fp16 in place -- the
//    MFMA operand that sums over the accumulator's row index needs no lane movement
//    (cdna_hip_programming.md §3); V is staged transposed in LDS with the matching k
//    order.  O^T (head dim x 32 queries) lives in the accumulator registers.
#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

typedef _Float16 ahalf8 __attribute__((ext_vector_type(8)));
typedef _Float16 ahalf4 __attribute__((ext_vector_type(4)));
typedef float af32x16 __attribute__((ext_vector_type(16)));

constexpr int AP_BQ = 128, AP_BK = 64, AP_THREADS = 256;

template <int D>
__global__ void __launch_bounds__(AP_THREADS) k_attn_prefill_f16(const float *__restrict__ Q,
                                                                  const float *__restrict__ kc,
                                                                  const float *__restrict__ vc, int E, int N,
                                                                  int n_past, float qscale, float *__restrict__ out) {
  constexpr int KLD = D + 8;      // K tile [key][dim], halves
  constexpr int VLD = AP_BK + 8;  // V^T tile [dim][key], halves
  constexpr int NT = D / 32;      // O^T tiles (32 dims each)
  __shared__ __attribute__((aligned(16))) _Float16 Ks[AP_BK * KLD];
  __shared__ __attribute__((aligned(16))) _Float16 Vt[D * VLD];
  const int h = blockIdx.y, q0 = blockIdx.x * AP_BQ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hl = lane >> 5;
  const int qw = q0 + wave * 32;  // this wave's first query
  const int myq = qw + r;         // this lane's query (column of S^T / O^T)
  const float *kbase = kc + (size_t)h * D, *vbase = vc + (size_t)h * D;

  // Q^T fragments: lane (query r, half hl) holds Q[q][16s + 8hl + j], j < 8, for every s
  ahalf8 qf[D / 16];
  {
    const float *qr = Q + (size_t)min(myq, N - 1) * E + h * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const float4 a = *(const float4 *)(qr + 16 * s + 8 * hl), b = *(const float4 *)(qr + 16 * s + 8 * hl + 4);
      ahalf8 f;
      f[0] = (_Float16)(a.x * qscale);
      f[1] = (_Float16)(a.y * qscale);
      f[2] = (_Float16)(a.z * qscale);
      f[3] = (_Float16)(a.w * qscale);
      f[4] = (_Float16)(b.x * qscale);
      f[5] = (_Float16)(b.y * qscale);
      f[6] = (_Float16)(b.z * qscale);
      f[7] = (_Float16)(b.w * qscale);
      qf[s] = f;
    }
  }
  af32x16 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = (af32x16){};
  float mrow = -INFINITY, lrow = 0.0f;

  const int klast = n_past + min(q0 + AP_BQ, N) - 1;  // last key any query of the block sees
  const int nkb = klast / AP_BK + 1;
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * AP_BK;
    // stage K (row-major) and V^T as fp16; keys past klast read as zero (masked below)
    for (int e = tid; e < AP_BK * D / 4; e += AP_THREADS) {
      const int key = e / (D / 4), c4 = (e % (D / 4)) * 4;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k0 + key <= klast) kv = *(const float4 *)(kbase + (size_t)(k0 + key) * E + c4);
      ahalf4 hk = {(_Float16)kv.x, (_Float16)kv.y, (_Float16)kv.z, (_Float16)kv.w};
      *(ahalf4 *)&Ks[key * KLD + c4] = hk;
    }
    for (int e = tid; e < AP_BK * D / 4; e += AP_THREADS) {
      // consecutive threads take consecutive keys of one 4-dim group (conflict-light
      // transposed stores)
      const int key = e % AP_BK, c4 = (e / AP_BK) * 4;
      float4 vv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k0 + key <= klast) vv = *(const float4 *)(vbase + (size_t)(k0 + key) * E + c4);
      Vt[(c4 + 0) * VLD + key] = (_Float16)vv.x;
      Vt[(c4 + 1) * VLD + key] = (_Float16)vv.y;
      Vt[(c4 + 2) * VLD + key] = (_Float16)vv.z;
      Vt[(c4 + 3) * VLD + key] = (_Float16)vv.w;
    }
    __syncthreads();
    if (k0 <= n_past + min(qw + 31, N - 1)) {  // wave-uniform: some key of the block is visible
      // S^T tiles t = 0, 1 (keys k0 + 32t + row)
      af32x16 st[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        st[t] = (af32x16){};
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          const ahalf8 kf = *(const ahalf8 *)&Ks[(32 * t + r) * KLD + 16 * s + 8 * hl];
          st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[s], st[t], 0, 0, 0);
        }
      }
      // causal mask and the block maximum of this lane's query
      float bm = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int key = k0 + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * hl;
          if (key > n_past + myq) st[t][g] = -INFINITY;
          bm = fmaxf(bm, st[t][g]);
        }
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mnew = fmaxf(mrow, bm);
      const float alpha = mnew == -INFINITY ? 1.0f : exp2f(mrow - mnew);
      float ls = 0.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float p = st[t][g] == -INFINITY ? 0.0f : exp2f(st[t][g] - mnew);
          st[t][g] = p;
          ls += p;
        }
      ls += __shfl_xor(ls, 32, 64);
      lrow = lrow * alpha + ls;
      mrow = mnew;
#pragma unroll
      for (int i = 0; i < NT; ++i) o[i] = o[i] * alpha;
      // O^T += V^T · P^T: k-step s2 of tile t covers keys 32t + 16s2 + 8(j>>2) + 4hl + (j&3)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          ahalf8 pf;
#pragma unroll
          for (int j = 0; j < 8; ++j) pf[j] = (_Float16)st[t][8 * s2 + j];
          const int kbase2 = 32 * t + 16 * s2 + 4 * hl;
#pragma unroll
          for (int i = 0; i < NT; ++i) {
            const _Float16 *vr = &Vt[(32 * i + r) * VLD + kbase2];
            const ahalf4 v0 = *(const ahalf4 *)vr, v1 = *(const ahalf4 *)(vr + 8);
            const ahalf8 vf = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
            o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf, o[i], 0, 0, 0);
          }
        }
    }
    __syncthreads();
  }
  // O^T / l: lane = query, rows = dims (reg & 3) + 8 (reg >> 2) + 4 hl of tile i
  if (myq < N) {
    const float inv = 1.0f / lrow;
    float *orow = out + (size_t)myq * E + h * D;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * i + 8 * g + 4 * hl;
        *(float4 *)(orow + dd) = make_float4(o[i][4 * g] * inv, o[i][4 * g + 1] * inv, o[i][4 * g + 2] * inv,
                                             o[i][4 * g + 3] * inv);
      }
  }
}

bool attn_prefill_supported(int d) { return d == 64 || d == 96 || d == 128 || d == 256; }

int launch_attn_prefill_f16(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                            float scale, float *out, hipStream_t s) {
  const int E = d * H;
  const float qscale = scale * 1.4426950408889634f;  // exp(x) = exp2(x * log2 e)
  const dim3 grid((N + AP_BQ - 1) / AP_BQ, H);
  switch (d) {
    case 64: hipLaunchKernelGGL(k_attn_prefill_f16<64>, grid, dim3(AP_THREADS), 0, s, Q, kc, vc, E, N, n_past, qscale, out); break;
    case 96: hipLaunchKernelGGL(k_attn_prefill_f16<96>, grid, dim3(AP_THREADS), 0, s, Q, kc, vc, E, N, n_past, qscale, out); break;
    case 128: hipLaunchKernelGGL(k_attn_prefill_f16<128>, grid, dim3(AP_THREADS), 0, s, Q, kc, vc, E, N, n_past, qscale, out); break;
    case 256: hipLaunchKernelGGL(k_attn_prefill_f16<256>, grid, dim3(AP_THREADS), 0, s, Q, kc, vc, E, N, n_past, qscale, out); break;
    default: set_error("attention prefill: head dim must be 64, 96, 128 or 256"); return VSIM_EINVAL;
  }
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
