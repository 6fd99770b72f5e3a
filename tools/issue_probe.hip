// tools/issue_probe.hip — VALU issue cost per instruction form on gfx950 (cycles per
// wave-instruction, independent instructions), at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void k_issue(float *out, long long *cyc, int n) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  unsigned u0 = threadIdx.x, u1 = u0 * 3, u2 = u0 * 5, u3 = u0 * 7;
  const f2 m = {1.0001f, 0.9999f};
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) {  // v_mul_f32
        asm volatile("v_mul_f32 %0, %0, %0\n v_mul_f32 %1, %1, %1\n v_mul_f32 %2, %2, %2\n v_mul_f32 %3, %3, %3"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        asm volatile("v_mul_f32 %0, %0, %0\n v_mul_f32 %1, %1, %1\n v_mul_f32 %2, %2, %2\n v_mul_f32 %3, %3, %3"
                     : "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      } else if (OP == 1) {  // v_pk_mul_f32
        asm volatile("v_pk_mul_f32 %0, %0, %0\n v_pk_mul_f32 %1, %1, %1\n v_pk_mul_f32 %2, %2, %2\n v_pk_mul_f32 %3, %3, %3"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
        asm volatile("v_pk_mul_f32 %0, %0, %0\n v_pk_mul_f32 %1, %1, %1\n v_pk_mul_f32 %2, %2, %2\n v_pk_mul_f32 %3, %3, %3"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
      } else if (OP == 2) {  // v_perm_b32
        asm volatile("v_perm_b32 %0, %0, %1, %2\n v_perm_b32 %1, %1, %2, %3\n v_perm_b32 %2, %2, %3, %0\n v_perm_b32 %3, %3, %0, %1"
                     : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
        asm volatile("v_perm_b32 %0, %0, %1, %2\n v_perm_b32 %1, %1, %2, %3\n v_perm_b32 %2, %2, %3, %0\n v_perm_b32 %3, %3, %0, %1"
                     : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
      } else if (OP == 3) {  // v_pk_fma_f32
        asm volatile("v_pk_fma_f32 %0, %0, %4, %0\n v_pk_fma_f32 %1, %1, %4, %1\n v_pk_fma_f32 %2, %2, %4, %2\n v_pk_fma_f32 %3, %3, %4, %3"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(m));
        asm volatile("v_pk_fma_f32 %0, %0, %4, %0\n v_pk_fma_f32 %1, %1, %4, %1\n v_pk_fma_f32 %2, %2, %4, %2\n v_pk_fma_f32 %3, %3, %4, %3"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(m));
      } else if (OP == 4) {  // v_cvt_f32_ubyte0
        asm volatile("v_cvt_f32_ubyte0 %0, %4\n v_cvt_f32_ubyte1 %1, %4\n v_cvt_f32_ubyte2 %2, %4\n v_cvt_f32_ubyte3 %3, %4"
                     : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3) : "v"(u0));
        asm volatile("v_cvt_f32_ubyte0 %0, %4\n v_cvt_f32_ubyte1 %1, %4\n v_cvt_f32_ubyte2 %2, %4\n v_cvt_f32_ubyte3 %3, %4"
                     : "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) : "v"(u1));
      } else if (OP == 5) {  // v_fma_f32 (VOP3)
        asm volatile("v_fma_f32 %0, %0, %0, %0\n v_fma_f32 %1, %1, %1, %1\n v_fma_f32 %2, %2, %2, %2\n v_fma_f32 %3, %3, %3, %3"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        asm volatile("v_fma_f32 %0, %0, %0, %0\n v_fma_f32 %1, %1, %1, %1\n v_fma_f32 %2, %2, %2, %2\n v_fma_f32 %3, %3, %3, %3"
                     : "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      }
    }
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y +
                                               (float)(u0 + u1 + u2 + u3);
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char *name, float *out, long long *cyc) {
  const int n = 256;
  for (int wps : {1, 2, 3}) {
    const int threads = 64 * 4 * wps;  // wps waves per SIMD
    hipLaunchKernelGGL(k_issue<OP>, 256, threads, 0, 0, out, cyc, n);
    hipLaunchKernelGGL(k_issue<OP>, 256, threads, 0, 0, out, cyc, n);
    hipDeviceSynchronize();
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-18s waves/SIMD=%d: %.2f cycles per wave-instruction (per wave), %.2f per SIMD\n", name, wps,
           (double)c / (n * 64.0), (double)c / (n * 64.0) / wps);
  }
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 1 << 22);
  (void)hipMalloc(&cyc, 1 << 16);
  run<0>("v_mul_f32", out, cyc);
  run<5>("v_fma_f32", out, cyc);
  run<1>("v_pk_mul_f32", out, cyc);
  run<3>("v_pk_fma_f32", out, cyc);
  run<2>("v_perm_b32", out, cyc);
  run<4>("v_cvt_f32_ubyteN", out, cyc);
  return 0;
}
