// vsim_amd/csrc/ops_q4.hip — Q4_0 kernels for gfx950: layout repack, activation
// quantization, the decode GEMV (exact and fast), embedding get_rows.
//
// Reference behaviour restated (not translated):
//   quantize_row_q4_0        ggml.c:209-251
//   dequantize_row_q4_0      ggml.c:301-334 (get_rows, ggml.c:5603-5628)
//   Q4_0 x Q4_0 dot          imax.c:1182-1230 (== ggml_vec_dot_q4_0, ggml.c:472-511)
#include "common.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

// ------------------------------------------------------------------ repack AoS <-> SoA
__global__ void k_q4_aos2soa(const uint8_t *__restrict__ aos, uint8_t *__restrict__ qs, float *__restrict__ d,
                             size_t nblocks) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const uint32_t *src = (const uint32_t *)(aos + b * QBYTES);  // blocks are 4-byte aligned
  d[b] = __uint_as_float(src[0]);
  uint4 q;
  q.x = src[1]; q.y = src[2]; q.z = src[3]; q.w = src[4];
  *(uint4 *)(qs + b * 16) = q;
}

__global__ void k_q4_soa2aos(const uint8_t *__restrict__ qs, const float *__restrict__ d, uint8_t *__restrict__ aos,
                             size_t nblocks) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  uint32_t *dst = (uint32_t *)(aos + b * QBYTES);
  const uint4 q = *(const uint4 *)(qs + b * 16);
  dst[0] = __float_as_uint(d[b]);
  dst[1] = q.x; dst[2] = q.y; dst[3] = q.z; dst[4] = q.w;
}

int launch_q4_repack(const void *aos, void *soa, int rows, int k, hipStream_t s) {
  if (k % QK || rows <= 0) { set_error("q4_repack: k must be a multiple of 32"); return VSIM_EINVAL; }
  const size_t nbk = (size_t)rows * (k / QK);
  uint8_t *qs = (uint8_t *)soa;
  float *d = (float *)(qs + nbk * 16);
  hipLaunchKernelGGL(k_q4_aos2soa, dim3((unsigned)((nbk + 255) / 256)), dim3(256), 0, s, (const uint8_t *)aos, qs, d,
                     nbk);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_q4_unpack(const void *soa, void *aos, int rows, int k, hipStream_t s) {
  if (k % QK || rows <= 0) { set_error("q4_unpack: k must be a multiple of 32"); return VSIM_EINVAL; }
  const size_t nbk = (size_t)rows * (k / QK);
  const uint8_t *qs = (const uint8_t *)soa;
  const float *d = (const float *)(qs + nbk * 16);
  hipLaunchKernelGGL(k_q4_soa2aos, dim3((unsigned)((nbk + 255) / 256)), dim3(256), 0, s, qs, d, (uint8_t *)aos, nbk);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ activation quantize
// One thread per 32-block.  Bit-identical to quantize_row_q4_0: fp32 amax, d = amax/7
// (correctly rounded division), id = 1/d, q = (int8)round(x*id) + 8 with round-half-
// away-from-zero, nibble pairs (q[2l], q[2l+1]).  Also emits xd = d*(q-8) per element,
// the activation factor f2/f3 of the reference dot (ggml.c:497-498).
__global__ void k_q4_quantize(const float *__restrict__ x, int k, int n, uint8_t *__restrict__ qs,
                              float *__restrict__ dd, float *__restrict__ xd) {
  const int nb = k / QK;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb * n) return;
  const float4 *src = (const float4 *)(x + (size_t)b * QK);
  float v[QK];
#pragma unroll
  for (int i = 0; i < QK / 4; ++i) {
    const float4 t = src[i];
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
  float amax = 0.0f;
#pragma unroll
  for (int l = 0; l < QK; ++l) amax = amax > fabsf(v[l]) ? amax : fabsf(v[l]);
  const float d = amax / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  uint32_t w[4] = {0, 0, 0, 0};
  float out[QK];
#pragma unroll
  for (int l = 0; l < QK; l += 2) {
    const int q0 = (int)(int8_t)roundf(v[l] * id) + 8;
    const int q1 = (int)(int8_t)roundf(v[l + 1] * id) + 8;
    w[l / 8] |= (uint32_t)((q0 & 0xF) | ((q1 & 0xF) << 4)) << (8 * ((l / 2) & 3));
    out[l] = d * (float)(q0 - 8);
    out[l + 1] = d * (float)(q1 - 8);
  }
  *(uint4 *)(qs + (size_t)b * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  dd[b] = d;
  if (xd) {
    float4 *o = (float4 *)(xd + (size_t)b * QK);
#pragma unroll
    for (int i = 0; i < QK / 4; ++i) o[i] = make_float4(out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]);
  }
}

int launch_q4_quantize(const float *x, int k, int n, void *xq, float *xd, hipStream_t s) {
  if (k % QK || n <= 0) { set_error("q4_quantize: k must be a multiple of 32"); return VSIM_EINVAL; }
  const int nbk = n * (k / QK);
  uint8_t *qs = (uint8_t *)xq;
  float *d = (float *)(qs + (size_t)nbk * 16);
  hipLaunchKernelGGL(k_q4_quantize, dim3((nbk + 127) / 128), dim3(128), 0, s, x, k, n, qs, d, xd);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ exact GEMV
// y[ic][r] = the reference's sequential float chain (imax.c:1191-1229):
//   for blocks i, bytes j: f0 = d0*(lo-8), f1 = d0*(hi-8), f2/f3 = xd; s += f0*f2 + f1*f3
// One lane owns one (row, token) chain; the chain order is the reference's.
template <int NT>
__global__ void __launch_bounds__(256) k_gemv_exact(Q4View W, const float *__restrict__ xd, int n,
                                                     const float *__restrict__ bias, float *__restrict__ y) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= W.rows) return;
  const int nb = W.nb();
  const int K = W.k;
  const uint4 *qrow = (const uint4 *)(W.qs + (size_t)r * nb * 16);
  const float *drow = W.d + (size_t)r * nb;
  for (int ic0 = 0; ic0 < n; ic0 += NT) {
    float acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0.0f;
    for (int i = 0; i < nb; ++i) {
      const float d0 = drow[i];
      const uint4 q = qrow[i];
      const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int wv = 0; wv < 4; ++wv) {
#pragma unroll
        for (int bj = 0; bj < 4; ++bj) {
          const uint32_t byte = (qw[wv] >> (8 * bj)) & 0xFF;
          const float f0 = d0 * (float)((int)(byte & 0xF) - 8);
          const float f1 = d0 * (float)((int)(byte >> 4) - 8);
          const int e = i * QK + 2 * (wv * 4 + bj);
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            if (ic0 + t < n) {
              const float2 a = *(const float2 *)(xd + (size_t)(ic0 + t) * K + e);
              acc[t] = acc[t] + (f0 * a.x + f1 * a.y);
            }
          }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (ic0 + t < n) y[(size_t)(ic0 + t) * W.rows + r] = bias ? acc[t] + bias[r] : acc[t];
  }
}

// ------------------------------------------------------------------ fast GEMV
// Same operands, HBM-streaming form: one wave per row, lanes stride over 16-byte nibble
// blocks (1 KiB coalesced per wave-instruction), integer block dot with v_dot8_i32_i4 on
// (nibble ^ 8) == signed (q - 8), then d0*d1*isum accumulated in fp32 and reduced across
// the wave.  Different rounding from the reference chain (not bit-exact).
template <int NT>
__global__ void __launch_bounds__(256) k_gemv_fast(Q4View W, const uint8_t *__restrict__ xqs,
                                                    const float *__restrict__ xdd, int n,
                                                    const float *__restrict__ bias, float *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= W.rows) return;
  const int nb = W.nb();
  const uint4 *qrow = (const uint4 *)(W.qs + (size_t)r * nb * 16);
  const float *drow = W.d + (size_t)r * nb;
  for (int ic0 = 0; ic0 < n; ic0 += NT) {
    float acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0.0f;
    for (int i = lane; i < nb; i += 64) {
      const uint4 q = qrow[i];
      const float d0 = drow[i];
      const int a0 = (int)(q.x ^ 0x88888888u), a1 = (int)(q.y ^ 0x88888888u);
      const int a2 = (int)(q.z ^ 0x88888888u), a3 = (int)(q.w ^ 0x88888888u);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (ic0 + t < n) {
          const size_t xb = (size_t)(ic0 + t) * nb + i;
          const uint4 xv = *(const uint4 *)(xqs + xb * 16);
          int s = __builtin_amdgcn_sdot8(a0, (int)(xv.x ^ 0x88888888u), 0, false);
          s = __builtin_amdgcn_sdot8(a1, (int)(xv.y ^ 0x88888888u), s, false);
          s = __builtin_amdgcn_sdot8(a2, (int)(xv.z ^ 0x88888888u), s, false);
          s = __builtin_amdgcn_sdot8(a3, (int)(xv.w ^ 0x88888888u), s, false);
          acc[t] = __builtin_fmaf(d0 * xdd[xb], (float)s, acc[t]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float v = wave_sum_f(acc[t]);
      if (lane == 0 && ic0 + t < n) y[(size_t)(ic0 + t) * W.rows + r] = bias ? v + bias[r] : v;
    }
  }
}

int launch_q4_gemv(const void *w, int M, int K, const void *xq, const float *xd, int n, const float *bias, float *y,
                   int mode, hipStream_t s) {
  if (K % QK || M <= 0 || n <= 0) { set_error("q4_gemv: bad shape"); return VSIM_EINVAL; }
  const Q4View W = q4_view(w, M, K);
  if (mode == VSIM_MODE_EXACT) {
    if (!xd) { set_error("q4_gemv: exact mode needs xd"); return VSIM_EINVAL; }
    hipLaunchKernelGGL(k_gemv_exact<1>, dim3((M + 255) / 256), dim3(256), 0, s, W, xd, n, bias, y);
  } else {
    const size_t nbk = (size_t)n * (K / QK);
    const uint8_t *xqs = (const uint8_t *)xq;
    const float *xdd = (const float *)(xqs + nbk * 16);
    if (n == 1)
      hipLaunchKernelGGL(k_gemv_fast<1>, dim3((M + 3) / 4), dim3(256), 0, s, W, xqs, xdd, n, bias, y);
    else
      hipLaunchKernelGGL(k_gemv_fast<4>, dim3((M + 3) / 4), dim3(256), 0, s, W, xqs, xdd, n, bias, y);
  }
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ get_rows
__global__ void k_get_rows(Q4View W, const int32_t *__restrict__ rows, int n, float *__restrict__ y) {
  const int nb = W.nb();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb * n) return;
  const int t = b / nb, i = b % nb;
  const int r = rows[t];
  if (r < 0 || r >= W.rows) {  // the reference would read out of bounds; we emit NaN
    for (int l = 0; l < QK; ++l) y[(size_t)t * W.k + i * QK + l] = __builtin_nanf("");
    return;
  }
  const float d = W.d[(size_t)r * nb + i];
  const uint4 q = *(const uint4 *)(W.qs + ((size_t)r * nb + i) * 16);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
  float *o = y + (size_t)t * W.k + i * QK;
#pragma unroll
  for (int wv = 0; wv < 4; ++wv)
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) {
      const uint32_t byte = (qw[wv] >> (8 * bj)) & 0xFF;
      o[2 * (wv * 4 + bj)] = (float)((int)(byte & 0xF) - 8) * d;
      o[2 * (wv * 4 + bj) + 1] = (float)((int)(byte >> 4) - 8) * d;
    }
}

int launch_get_rows(const void *w, int K, int V, const int32_t *rows, int n, float *y, hipStream_t s) {
  if (K % QK || n <= 0) { set_error("get_rows: bad shape"); return VSIM_EINVAL; }
  const Q4View W = q4_view(w, V, K);
  const int nbk = n * (K / QK);
  hipLaunchKernelGGL(k_get_rows, dim3((nbk + 127) / 128), dim3(128), 0, s, W, rows, n, y);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ dequantize (SoA)
// xd[r][e] = d*(q-8) for every element: the activation factors of the exact dot when the
// quantized rows arrive from the host already quantized (the drop-in path).
__global__ void k_q4_dequant(Q4View X, float *__restrict__ y) {
  const int nb = X.nb();
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (size_t)nb * X.rows) return;
  const float d = X.d[b];
  const uint4 q = *(const uint4 *)(X.qs + b * 16);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
  float *o = y + b * QK;
#pragma unroll
  for (int wv = 0; wv < 4; ++wv)
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) {
      const uint32_t byte = (qw[wv] >> (8 * bj)) & 0xFF;
      o[2 * (wv * 4 + bj)] = d * (float)((int)(byte & 0xF) - 8);
      o[2 * (wv * 4 + bj) + 1] = d * (float)((int)(byte >> 4) - 8);
    }
}

int launch_q4_dequant(const void *soa, int rows, int k, float *y, hipStream_t s) {
  const Q4View X = q4_view(soa, rows, k);
  const size_t nbk = (size_t)rows * (k / QK);
  hipLaunchKernelGGL(k_q4_dequant, dim3((unsigned)((nbk + 127) / 128)), dim3(128), 0, s, X, y);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ synthetic weights
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float randn(uint64_t seed, uint64_t i) {
  const uint64_t h = mix64(seed ^ mix64(i));
  const float u1 = ((uint32_t)(h >> 40) + 1) * (1.0f / 16777217.0f);
  const float u2 = ((uint32_t)(h & 0xFFFFFF)) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

__global__ void k_randn_q4(uint8_t *__restrict__ qs, float *__restrict__ dd, size_t nblocks, uint64_t seed, float sd) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  float v[QK];
  float amax = 0.0f;
#pragma unroll
  for (int l = 0; l < QK; ++l) {
    v[l] = randn(seed, b * QK + l) * sd;
    amax = amax > fabsf(v[l]) ? amax : fabsf(v[l]);
  }
  const float d = amax / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int l = 0; l < QK; l += 2) {
    const int q0 = (int)(int8_t)roundf(v[l] * id) + 8;
    const int q1 = (int)(int8_t)roundf(v[l + 1] * id) + 8;
    w[l / 8] |= (uint32_t)((q0 & 0xF) | ((q1 & 0xF) << 4)) << (8 * ((l / 2) & 3));
  }
  *(uint4 *)(qs + b * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  dd[b] = d;
}

__global__ void k_randn_f32(float *x, int n, uint64_t seed, float sd, float mean) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = mean + randn(seed, (uint64_t)i) * sd;
}

int launch_randn_q4(void *soa, int rows, int k, uint64_t seed, float stddev, hipStream_t s) {
  const size_t nbk = (size_t)rows * (k / QK);
  uint8_t *qs = (uint8_t *)soa;
  float *d = (float *)(qs + nbk * 16);
  hipLaunchKernelGGL(k_randn_q4, dim3((unsigned)((nbk + 255) / 256)), dim3(256), 0, s, qs, d, nbk, seed, stddev);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_randn_f32(float *x, int n, uint64_t seed, float stddev, float mean, hipStream_t s) {
  hipLaunchKernelGGL(k_randn_f32, dim3((n + 255) / 256), dim3(256), 0, s, x, n, seed, stddev, mean);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
