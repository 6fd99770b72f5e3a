// vsim_amd/csrc/graph.hip — strided F32 kernels for the ggml graph executor (graph.cpp).
//
// The decode path's fused kernels assume the layouts of the builder's own executor; a ggml
// graph reaches the device as nodes over views (permute, reshape, view_1d of the KV cache), so
// these kernels take each operand as a base pointer plus the tensor's ne / nb (bytes), and do
// exactly what the reference's CPU kernel does element by element:
//   dup / cpy          ggml.c:3213-3315  (destination contiguous, source in logical order)
//   add / mul          ggml.c:3344-3395, 3474-3499 (rows j*nb1, columns of 4 bytes; src1 may
//                      be strided in dim 0)
//   repeat             ggml.c:3809-3847  (2-D)
//   scale              ggml.c:5492-5525  (in place: ggml_scale returns a view)
//   diag_mask_inf      ggml.c:5764-5798  (in place)
//   mul_mat f32        ggml.c:4355-4595: rows of src0 contiguous (nb01 >= nb00) -> one double
//                      accumulator of float products per output (ggml_vec_dot_f32 399-434);
//                      src0 transposed -> per-thread partial sums of sequential float mads
//                      (ggml_vec_mad_f32 610-639) over column ranges of size ceil(ne10/nth),
//                      added in thread order in FINALIZE (4469-4493).  nth = the graph's
//                      n_threads, so the result equals the reference at any --threads.
#include "common.hpp"
#include "graph.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

__device__ __forceinline__ const float *at(const GT &t, int i0, int i1, int i2, int i3) {
  return (const float *)(t.p + i0 * t.nb[0] + i1 * t.nb[1] + i2 * t.nb[2] + i3 * t.nb[3]);
}

__global__ void k_g_dup(float *__restrict__ dst, GT s, long long n) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  long long r = i;
  const int i0 = (int)(r % s.ne[0]);
  r /= s.ne[0];
  const int i1 = (int)(r % s.ne[1]);
  r /= s.ne[1];
  const int i2 = (int)(r % s.ne[2]);
  const int i3 = (int)(r / s.ne[2]);
  dst[i] = *at(s, i0, i1, i2, i3);
}

// op 0: add, 1: mul.  nr rows of nc; row j of each operand at base + j*nb1.
__global__ void k_g_binop(int op, char *__restrict__ d, long long dnb1, const char *__restrict__ a, long long anb1,
                          const char *__restrict__ b, long long bnb0, long long bnb1, int nc, long long nr) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= nr * nc) return;
  const long long j = i / nc;
  const int c = (int)(i % nc);
  const float x = ((const float *)(a + j * anb1))[c];
  const float y = *(const float *)(b + j * bnb1 + c * bnb0);
  ((float *)(d + j * dnb1))[c] = op == 0 ? x + y : x * y;
}

__global__ void k_g_repeat(char *__restrict__ d, long long dnb1, const char *__restrict__ s, long long snb1, int nc,
                           int nr, int nc0, int nr0) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)nr * nc) return;
  const int r = (int)(i / nc), c = (int)(i % nc);
  ((float *)(d + r * dnb1))[c] = ((const float *)(s + (r % nr0) * snb1))[c % nc0];
}

__global__ void k_g_scale(char *__restrict__ x, long long nb1, int nc, long long nr, float v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= nr * nc) return;
  float *p = (float *)(x + (i / nc) * nb1) + i % nc;
  *p = *p * v;
}

__global__ void k_g_diag_mask(char *__restrict__ x, long long nb0, long long nb1, long long nb2, int nc, int nr, int nz,
                              int n_past) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)nz * nr * nc) return;
  const int c = (int)(i % nc), j = (int)((i / nc) % nr), k = (int)(i / ((long long)nc * nr));
  if (c >= n_past && c > n_past + j) *(float *)(x + k * nb2 + j * nb1 + c * nb0) = -INFINITY;
}

// dst[i0, i1, i2, i3] = sum_k (double)(src0[k, i0, i2, i3] * src1[k, i1, i2, i3]) in k order
__global__ void k_g_mm_dot(GT d, GT a, GT b, int K) {
  const long long n = (long long)d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  long long r = i;
  const int i0 = (int)(r % d.ne[0]);
  r /= d.ne[0];
  const int i1 = (int)(r % d.ne[1]);
  r /= d.ne[1];
  const int i2 = (int)(r % d.ne[2]);
  const int i3 = (int)(r / d.ne[2]);
  const float *x = at(a, 0, i0, i2, i3), *y = at(b, 0, i1, i2, i3);
  double s = 0.0;
  for (int k = 0; k < K; ++k) s += (double)(x[k] * y[k]);
  *(float *)at(d, i0, i1, i2, i3) = (float)s;
}

// dst contiguous [ne01, ne11, ne12, ne13]; src0 transposed (its dim-1 stride is 4 bytes)
__global__ void k_g_mm_mad(float *__restrict__ dst, GT a, GT b, int nc, int nth, int ne0, int ne1, int ne2,
                           long long n) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  long long r = i;
  const int j = (int)(r % ne0);
  r /= ne0;
  const int i1 = (int)(r % ne1);
  r /= ne1;
  const int i2 = (int)(r % ne2);
  const int i3 = (int)(r / ne2);
  const int dc = (nc + nth - 1) / nth;
  float out = 0.0f;
  for (int t = 0; t < nth; ++t) {
    const int ic0 = dc * t, ic1 = min(ic0 + dc, nc);
    float part = 0.0f;
    for (int ic = ic0; ic < ic1; ++ic) part = part + *at(a, ic, j, i2, i3) * *at(b, ic, i1, i2, i3);
    out = t == 0 ? part : out + part;
  }
  dst[i] = out;
}

static dim3 grid1(long long n) { return dim3((unsigned)((n + 255) / 256)); }

int launch_g_dup(float *dst, const GT &s, long long n, hipStream_t st) {
  if (n <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_dup, grid1(n), dim3(256), 0, st, dst, s, n);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_g_binop(int op, char *d, long long dnb1, const char *a, long long anb1, const char *b, long long bnb0,
                   long long bnb1, int nc, long long nr, hipStream_t st) {
  if (nr * nc <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_binop, grid1(nr * nc), dim3(256), 0, st, op, d, dnb1, a, anb1, b, bnb0, bnb1, nc, nr);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_g_repeat(char *d, long long dnb1, const char *s, long long snb1, int nc, int nr, int nc0, int nr0,
                    hipStream_t st) {
  if (nc <= 0 || nr <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_repeat, grid1((long long)nr * nc), dim3(256), 0, st, d, dnb1, s, snb1, nc, nr, nc0, nr0);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_g_scale(char *x, long long nb1, int nc, long long nr, float v, hipStream_t st) {
  if (nr * nc <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_scale, grid1(nr * nc), dim3(256), 0, st, x, nb1, nc, nr, v);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_g_diag_mask(char *x, long long nb0, long long nb1, long long nb2, int nc, int nr, int nz, int n_past,
                       hipStream_t st) {
  const long long n = (long long)nz * nr * nc;
  if (n <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_diag_mask, grid1(n), dim3(256), 0, st, x, nb0, nb1, nb2, nc, nr, nz, n_past);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_g_mm_dot(const GT &d, const GT &a, const GT &b, int K, hipStream_t st) {
  const long long n = (long long)d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
  if (n <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_mm_dot, grid1(n), dim3(256), 0, st, d, a, b, K);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_g_mm_mad(float *dst, const GT &a, const GT &b, int nc, int nth, int ne0, int ne1, int ne2, int ne3,
                    hipStream_t st) {
  const long long n = (long long)ne0 * ne1 * ne2 * ne3;
  if (n <= 0) return VSIM_OK;
  hipLaunchKernelGGL(k_g_mm_mad, grid1(n), dim3(256), 0, st, dst, a, b, nc, nth, ne0, ne1, ne2, n);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
