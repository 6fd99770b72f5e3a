// vsim_amd/csrc/ops_q4.hip — Q4_0 kernels for gfx950: weight tiling, activation
// quantization, the decode GEMV (exact and fast), embedding get_rows.
//
// Reference behaviour restated (not translated):
//   quantize_row_q4_0        ggml.c:209-251
//   dequantize_row_q4_0      ggml.c:301-334 (get_rows, ggml.c:5603-5628)
//   Q4_0 x Q4_0 dot          imax.c:1182-1230 (== ggml_vec_dot_q4_0, ggml.c:472-511)
//
// Weight layout "W4T32" (see W4 in common.hpp): rows are grouped in tiles of 32; inside a
// tile the 16-byte nibble blocks are stored block-major, so the 32 rows' block b sit in
// 512 contiguous bytes and the 32 scales of block b in 128 contiguous bytes.  A wave whose
// lanes own rows reads whole cache lines; bytes per weight stay 0.625.
#include <algorithm>

#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

// ------------------------------------------------------------------ W4T32 pack / unpack
__global__ void k_w4_pack(const uint8_t *__restrict__ aos, W4 W) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = W.nb();
  const size_t total = (size_t)W.tiles * T32 * nb;
  if (i >= total) return;
  // i enumerates (row, block) in row-major order over the padded rows
  const int r = (int)(i / nb), b = (int)(i % nb);
  const size_t o = W.off(r, b);
  if (r >= W.rows) {  // padding rows of the last tile: d = 0, q = 8 (value 0)
    ((float *)W.d)[o] = 0.0f;
    *(uint4 *)(W.qs + o * 16) = make_uint4(0x88888888u, 0x88888888u, 0x88888888u, 0x88888888u);
    return;
  }
  const uint32_t *src = (const uint32_t *)(aos + i * QBYTES);  // AoS blocks are 4-byte aligned
  ((float *)W.d)[o] = __uint_as_float(src[0]);
  *(uint4 *)(W.qs + o * 16) = make_uint4(src[1], src[2], src[3], src[4]);
}

__global__ void k_w4_unpack(W4 W, uint8_t *__restrict__ aos) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = W.nb();
  if (i >= (size_t)W.rows * nb) return;
  const int r = (int)(i / nb), b = (int)(i % nb);
  const size_t o = W.off(r, b);
  uint32_t *dst = (uint32_t *)(aos + i * QBYTES);
  const uint4 q = *(const uint4 *)(W.qs + o * 16);
  dst[0] = __float_as_uint(W.d[o]);
  dst[1] = q.x; dst[2] = q.y; dst[3] = q.z; dst[4] = q.w;
}

int launch_q4_repack(const void *aos, void *w, int rows, int k, hipStream_t s) {
  if (k % QK || rows <= 0) { set_error("q4_repack: k must be a multiple of 32"); return VSIM_EINVAL; }
  const W4 W = w4_view(w, rows, k);
  const size_t tot = (size_t)W.tiles * T32 * W.nb();
  hipLaunchKernelGGL(k_w4_pack, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, (const uint8_t *)aos, W);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_q4_unpack(const void *w, void *aos, int rows, int k, hipStream_t s) {
  if (k % QK || rows <= 0) { set_error("q4_unpack: k must be a multiple of 32"); return VSIM_EINVAL; }
  const W4 W = w4_view(w, rows, k);
  const size_t tot = (size_t)rows * W.nb();
  hipLaunchKernelGGL(k_w4_unpack, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, W, (uint8_t *)aos);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// activation rows (AoS, as the reference's INIT phase writes them) -> row-major SoA
__global__ void k_act_aos2soa(const uint8_t *__restrict__ aos, uint8_t *__restrict__ qs, float *__restrict__ d,
                              size_t nblocks) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const uint32_t *src = (const uint32_t *)(aos + b * QBYTES);
  d[b] = __uint_as_float(src[0]);
  *(uint4 *)(qs + b * 16) = make_uint4(src[1], src[2], src[3], src[4]);
}

__global__ void k_act_soa2aos(const uint8_t *__restrict__ qs, const float *__restrict__ d, uint8_t *__restrict__ aos,
                              size_t nblocks) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  uint32_t *dst = (uint32_t *)(aos + b * QBYTES);
  const uint4 q = *(const uint4 *)(qs + b * 16);
  dst[0] = __float_as_uint(d[b]);
  dst[1] = q.x; dst[2] = q.y; dst[3] = q.z; dst[4] = q.w;
}

int launch_act_repack(const void *aos, void *xq, int n, int k, hipStream_t s) {
  const size_t nbk = (size_t)n * (k / QK);
  uint8_t *qs = (uint8_t *)xq;
  float *d = (float *)(qs + nbk * 16);
  hipLaunchKernelGGL(k_act_aos2soa, dim3((unsigned)((nbk + 255) / 256)), dim3(256), 0, s, (const uint8_t *)aos, qs,
                     d, nbk);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_act_unpack(const void *xq, void *aos, int n, int k, hipStream_t s) {
  const size_t nbk = (size_t)n * (k / QK);
  const uint8_t *qs = (const uint8_t *)xq;
  const float *d = (const float *)(qs + nbk * 16);
  hipLaunchKernelGGL(k_act_soa2aos, dim3((unsigned)((nbk + 255) / 256)), dim3(256), 0, s, qs, d, (uint8_t *)aos,
                     nbk);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

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
  quantize_block(v, qs + (size_t)b * 16, dd + b, xd ? xd + (size_t)b * QK : nullptr);
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

// xd[r][e] = d*(q-8): activation factors of rows that arrive already quantized (drop-in)
__global__ void k_q4_dequant(const uint8_t *__restrict__ qs, const float *__restrict__ dd, size_t nblocks,
                             float *__restrict__ y) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const float d = dd[b];
  const uint4 q = *(const uint4 *)(qs + b * 16);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
  float *o = y + b * QK;
#pragma unroll
  for (int wv = 0; wv < 4; ++wv)
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) {
      const uint32_t byte = (qw[wv] >> (8 * bj)) & 0xFF;
      o[xd_slot(2 * (wv * 4 + bj))] = d * (float)((int)(byte & 0xF) - 8);
      o[xd_slot(2 * (wv * 4 + bj) + 1)] = d * (float)((int)(byte >> 4) - 8);
    }
}

int launch_q4_dequant(const void *xq, int rows, int k, float *y, hipStream_t s) {
  const size_t nbk = (size_t)rows * (k / QK);
  const uint8_t *qs = (const uint8_t *)xq;
  const float *d = (const float *)(qs + nbk * 16);
  hipLaunchKernelGGL(k_q4_dequant, dim3((unsigned)((nbk + 127) / 128)), dim3(128), 0, s, qs, d, nbk, y);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ------------------------------------------------------------------ activation quantize
// (quantize_block: kern.hpp)

// ------------------------------------------------------------------ fast GEMV
// HBM-streaming form of the same product: one 512-thread workgroup per 32-row tile, lane
// (r, h) = (lane & 31, lane >> 5) of wave w streams blocks b = 2w + h, +16, ... (each
// wave-instruction reads 1 KiB contiguous), integer block dot with v_dot8_i32_i4 on
// (nibble ^ 8) == signed (q - 8), d0*d1*isum accumulated in fp32; 16 partials per row
// summed through LDS in a fixed order (deterministic).  Not bit-exact to the reference.
constexpr int FAST_WAVES = 8;
__global__ void __launch_bounds__(64 * FAST_WAVES) k_gemv_fast(GemvBatch B) {
  __shared__ float part[FAST_WAVES * 2][T32];
  int t = blockIdx.x, ji = 0;
  while (ji + 1 < B.nj && t >= B.j[ji].w.tiles) { t -= B.j[ji].w.tiles; ++ji; }
  const GemvJob J = B.j[ji];
  const int nb = J.w.nb();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & (T32 - 1), h = lane >> 5;
  const uint8_t *qs = J.w.qs + (size_t)t * nb * T32 * 16;
  const float *dd = J.w.d + (size_t)t * nb * T32;
  float acc = 0.0f;
  for (int b = 2 * wave + h; b < nb; b += 2 * FAST_WAVES) {
    const size_t o = (size_t)b * T32 + r;
    const uint4 q = *(const uint4 *)(qs + o * 16);
    const float d0 = dd[o];
    const uint4 xv = *(const uint4 *)(J.xqs + (size_t)b * 16);
    int sdot = __builtin_amdgcn_sdot8((int)(q.x ^ 0x88888888u), (int)(xv.x ^ 0x88888888u), 0, false);
    sdot = __builtin_amdgcn_sdot8((int)(q.y ^ 0x88888888u), (int)(xv.y ^ 0x88888888u), sdot, false);
    sdot = __builtin_amdgcn_sdot8((int)(q.z ^ 0x88888888u), (int)(xv.z ^ 0x88888888u), sdot, false);
    sdot = __builtin_amdgcn_sdot8((int)(q.w ^ 0x88888888u), (int)(xv.w ^ 0x88888888u), sdot, false);
    acc = __builtin_fmaf(d0 * J.xdd[b], (float)sdot, acc);
  }
  part[2 * wave + h][r] = acc;
  __syncthreads();
  if (threadIdx.x < T32) {
    float sum = 0.0f;
#pragma unroll
    for (int i = 0; i < 2 * FAST_WAVES; ++i) sum += part[i][threadIdx.x];
    const int row = t * T32 + threadIdx.x;
    if (row < J.w.rows) J.y[row] = J.bias ? sum + J.bias[row] : sum;
  }
}

int launch_gemv_batch(const GemvBatch &B, int mode, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < B.nj; ++i) tiles += B.j[i].w.tiles;
  if (tiles == 0) return VSIM_OK;
  if (mode == VSIM_MODE_EXACT) {
    return launch_gemv_chain_batch(B, s);  // gemv_chain.hip
  } else {
    hipLaunchKernelGGL(k_gemv_fast, dim3(tiles), dim3(64 * FAST_WAVES), 0, s, B);
  }
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// (GEMM_MIN_N, common.hpp: fast mode, from this many tokens on, the MFMA GEMM)

int launch_q4_gemv(const void *w, int M, int K, const void *xq, const float *xd, int n, const float *bias, float *y,
                   int mode, hipStream_t s) {
  if (K % QK || M <= 0 || n <= 0) { set_error("q4_gemv: bad shape"); return VSIM_EINVAL; }
  const W4 W = w4_view(w, M, K);
  if (mode == VSIM_MODE_EXACT && !xd) { set_error("q4_gemv: exact mode needs xd"); return VSIM_EINVAL; }
  // fast mode, prompt batches: fp16 MFMA GEMM after in-LDS dequant (gemm_f16.hip)
  if (mode == VSIM_MODE_FAST && n >= GEMM_MIN_N) return launch_gemm_q4_f16(W, xq, n, bias, y, s);
  // exact mode, prompt batches: the register-tiled chain GEMM (gemm_exact.hip).  Its 128-token
  // tiles cost the same for 5 tokens as for 128 (r04 rocprof: 1.09 ms per GPT-J GEMM for a
  // 5-token prompt), so short batches take the decode GEMV, up to 4 tokens per launch (one job
  // each: the same chains, bit for bit)
  if (mode == VSIM_MODE_EXACT && n > EXACT_GEMV_MAX_N) return launch_gemm_exact(W, xd, n, bias, y, s);
  const size_t nbk = (size_t)n * (K / QK);
  const uint8_t *xqs = (const uint8_t *)xq;
  const float *xdd = (const float *)(xqs + nbk * 16);
  const int per = mode == VSIM_MODE_EXACT ? 4 : 1;
  for (int i0 = 0; i0 < n; i0 += per) {
    GemvBatch B{};
    B.nj = std::min(per, n - i0);
    for (int u = 0; u < B.nj; ++u) {
      const int ic = i0 + u;
      B.j[u].w = W;
      B.j[u].xd = xd ? xd + (size_t)ic * K : nullptr;
      B.j[u].xqs = xqs + (size_t)ic * (K / QK) * 16;
      B.j[u].xdd = xdd + (size_t)ic * (K / QK);
      B.j[u].bias = bias;
      B.j[u].y = y + (size_t)ic * M;
    }
    if (int rc = launch_gemv_batch(B, mode, s)) return rc;
  }
  return VSIM_OK;
}

// ------------------------------------------------------------------ get_rows
__global__ void k_get_rows(W4 W, const int32_t *__restrict__ rows, int n, float *__restrict__ y) {
  const int nb = W.nb();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb * n) return;
  const int t = b / nb, i = b % nb;
  const int r = rows[t];
  float *o = y + (size_t)t * W.k + i * QK;
  if (r < 0 || r >= W.rows) {  // the reference would read out of bounds; we emit NaN
    for (int l = 0; l < QK; ++l) o[l] = __builtin_nanf("");
    return;
  }
  const size_t off = W.off(r, i);
  const float d = W.d[off];
  const uint4 q = *(const uint4 *)(W.qs + off * 16);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
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
  const W4 W = w4_view(w, V, K);
  const int nbk = n * (K / QK);
  hipLaunchKernelGGL(k_get_rows, dim3((nbk + 127) / 128), dim3(128), 0, s, W, rows, n, y);
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

__global__ void k_randn_w4(W4 W, uint64_t seed, float sd) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = W.nb();
  if (i >= (size_t)W.tiles * T32 * nb) return;
  const int r = (int)(i / nb), b = (int)(i % nb);
  const size_t o = W.off(r, b);
  if (r >= W.rows) {
    ((float *)W.d)[o] = 0.0f;
    *(uint4 *)(W.qs + o * 16) = make_uint4(0x88888888u, 0x88888888u, 0x88888888u, 0x88888888u);
    return;
  }
  float v[QK];
#pragma unroll
  for (int l = 0; l < QK; ++l) v[l] = randn(seed, i * QK + l) * sd;
  quantize_block(v, (uint8_t *)W.qs + o * 16, (float *)W.d + o, nullptr);
}

__global__ void k_randn_f32(float *x, int n, uint64_t seed, float sd, float mean) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = mean + randn(seed, (uint64_t)i) * sd;
}

int launch_randn_q4(void *w, int rows, int k, uint64_t seed, float stddev, hipStream_t s) {
  const W4 W = w4_view(w, rows, k);
  const size_t tot = (size_t)W.tiles * T32 * W.nb();
  hipLaunchKernelGGL(k_randn_w4, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, W, seed, stddev);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_randn_f32(float *x, int n, uint64_t seed, float stddev, float mean, hipStream_t s) {
  hipLaunchKernelGGL(k_randn_f32, dim3((n + 255) / 256), dim3(256), 0, s, x, n, seed, stddev, mean);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
