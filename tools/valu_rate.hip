// tools/valu_rate.hip — issue cost per wave64 VALU instruction on gfx950 for the ops the exact
// GEMV's producers use (packed f32, fp8 conversion, integer), with 1, 2 and 3 waves per SIMD
// and independent operands (throughput, not latency).  Cycles from s_memtime per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

template <int OP>
__global__ void k_rate(float *out, unsigned long long *cyc, int n) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7, a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11, a12 = a0 + 12, a13 = a0 + 13,
        a14 = a0 + 14, a15 = a0 + 15;
  const float c = 1.0001f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (OP == 0) {  // v_pk_fma_f32 x8 (16 floats)
      asm volatile(
          "v_pk_fma_f32 v[10:11], v[10:11], v[12:13], v[12:13]\n v_pk_fma_f32 v[14:15], v[14:15], v[12:13], v[12:13]\n"
          "v_pk_fma_f32 v[16:17], v[16:17], v[12:13], v[12:13]\n v_pk_fma_f32 v[18:19], v[18:19], v[12:13], v[12:13]\n"
          "v_pk_fma_f32 v[20:21], v[20:21], v[12:13], v[12:13]\n v_pk_fma_f32 v[22:23], v[22:23], v[12:13], v[12:13]\n"
          "v_pk_fma_f32 v[24:25], v[24:25], v[12:13], v[12:13]\n v_pk_fma_f32 v[26:27], v[26:27], v[12:13], v[12:13]\n" ::
              : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23",
                "v24", "v25", "v26", "v27");
    }
    if (OP == 1) {  // v_pk_mul_f32 x8
      asm volatile(
          "v_pk_mul_f32 v[10:11], v[10:11], v[12:13]\n v_pk_mul_f32 v[14:15], v[14:15], v[12:13]\n"
          "v_pk_mul_f32 v[16:17], v[16:17], v[12:13]\n v_pk_mul_f32 v[18:19], v[18:19], v[12:13]\n"
          "v_pk_mul_f32 v[20:21], v[20:21], v[12:13]\n v_pk_mul_f32 v[22:23], v[22:23], v[12:13]\n"
          "v_pk_mul_f32 v[24:25], v[24:25], v[12:13]\n v_pk_mul_f32 v[26:27], v[26:27], v[12:13]\n" ::
              : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23",
                "v24", "v25", "v26", "v27");
    }
    if (OP == 2) {  // v_cvt_pk_f32_fp8 x8
      asm volatile(
          "v_cvt_pk_f32_fp8 v[10:11], v30\n v_cvt_pk_f32_fp8 v[14:15], v31\n v_cvt_pk_f32_fp8 v[16:17], v32\n"
          "v_cvt_pk_f32_fp8 v[18:19], v33\n v_cvt_pk_f32_fp8 v[20:21], v34\n v_cvt_pk_f32_fp8 v[22:23], v35\n"
          "v_cvt_pk_f32_fp8 v[24:25], v36\n v_cvt_pk_f32_fp8 v[26:27], v37\n" ::
              : "v10", "v11", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25",
                "v26", "v27");
    }
    if (OP == 3) {  // v_mul_f32 x8
      asm volatile(
          "v_mul_f32 v10, v10, v12\n v_mul_f32 v14, v14, v12\n v_mul_f32 v16, v16, v12\n v_mul_f32 v18, v18, v12\n"
          "v_mul_f32 v20, v20, v12\n v_mul_f32 v22, v22, v12\n v_mul_f32 v24, v24, v12\n v_mul_f32 v26, v26, v12\n" ::
              : "v10", "v12", "v14", "v16", "v18", "v20", "v22", "v24", "v26");
    }
    if (OP == 4) {  // v_fma_f32 x8
      asm volatile(
          "v_fma_f32 v10, v10, v12, v13\n v_fma_f32 v14, v14, v12, v13\n v_fma_f32 v16, v16, v12, v13\n"
          "v_fma_f32 v18, v18, v12, v13\n v_fma_f32 v20, v20, v12, v13\n v_fma_f32 v22, v22, v12, v13\n"
          "v_fma_f32 v24, v24, v12, v13\n v_fma_f32 v26, v26, v12, v13\n" ::
              : "v10", "v12", "v13", "v14", "v16", "v18", "v20", "v22", "v24", "v26");
    }
    if (OP == 5) {  // v_and_b32 x8
      asm volatile(
          "v_and_b32 v10, v10, v12\n v_and_b32 v14, v14, v12\n v_and_b32 v16, v16, v12\n v_and_b32 v18, v18, v12\n"
          "v_and_b32 v20, v20, v12\n v_and_b32 v22, v22, v12\n v_and_b32 v24, v24, v12\n v_and_b32 v26, v26, v12\n" ::
              : "v10", "v12", "v14", "v16", "v18", "v20", "v22", "v24", "v26");
    }
    if (OP == 6) {  // v_add_f32 x8
      asm volatile(
          "v_add_f32 v10, v10, v12\n v_add_f32 v14, v14, v12\n v_add_f32 v16, v16, v12\n v_add_f32 v18, v18, v12\n"
          "v_add_f32 v20, v20, v12\n v_add_f32 v22, v22, v12\n v_add_f32 v24, v24, v12\n v_add_f32 v26, v26, v12\n" ::
              : "v10", "v12", "v14", "v16", "v18", "v20", "v22", "v24", "v26");
    }
    if (OP == 7) {  // v_pk_add_f32 x8
      asm volatile(
          "v_pk_add_f32 v[10:11], v[10:11], v[12:13]\n v_pk_add_f32 v[14:15], v[14:15], v[12:13]\n"
          "v_pk_add_f32 v[16:17], v[16:17], v[12:13]\n v_pk_add_f32 v[18:19], v[18:19], v[12:13]\n"
          "v_pk_add_f32 v[20:21], v[20:21], v[12:13]\n v_pk_add_f32 v[22:23], v[22:23], v[12:13]\n"
          "v_pk_add_f32 v[24:25], v[24:25], v[12:13]\n v_pk_add_f32 v[26:27], v[26:27], v[12:13]\n" ::
              : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23",
                "v24", "v25", "v26", "v27");
    }
    if (OP == 8) {  // v_cvt_f32_ubyte0 x8
      asm volatile(
          "v_cvt_f32_ubyte0 v10, v30\n v_cvt_f32_ubyte0 v14, v31\n v_cvt_f32_ubyte0 v16, v32\n v_cvt_f32_ubyte0 v18, v33\n"
          "v_cvt_f32_ubyte0 v20, v34\n v_cvt_f32_ubyte0 v22, v35\n v_cvt_f32_ubyte0 v24, v36\n v_cvt_f32_ubyte0 v26, v37\n" ::
              : "v10", "v14", "v16", "v18", "v20", "v22", "v24", "v26");
    }
    if (OP == 9) {  // v_pk_fma_f32 with an SGPR-pair operand (as the producers' factor multiply)
      asm volatile(
          "v_pk_mul_f32 v[10:11], s[0:1], v[10:11]\n v_pk_mul_f32 v[14:15], s[2:3], v[14:15]\n"
          "v_pk_mul_f32 v[16:17], s[4:5], v[16:17]\n v_pk_mul_f32 v[18:19], s[6:7], v[18:19]\n"
          "v_pk_mul_f32 v[20:21], s[0:1], v[20:21]\n v_pk_mul_f32 v[22:23], s[2:3], v[22:23]\n"
          "v_pk_mul_f32 v[24:25], s[4:5], v[24:25]\n v_pk_mul_f32 v[26:27], s[6:7], v[26:27]\n" ::
              : "v10", "v11", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25",
                "v26", "v27");
    }
    if (OP == 10) {  // v_perm_b32 x8
      asm volatile(
          "v_perm_b32 v10, v30, v31, v12\n v_perm_b32 v14, v30, v31, v12\n v_perm_b32 v16, v30, v31, v12\n"
          "v_perm_b32 v18, v30, v31, v12\n v_perm_b32 v20, v30, v31, v12\n v_perm_b32 v22, v30, v31, v12\n"
          "v_perm_b32 v24, v30, v31, v12\n v_perm_b32 v26, v30, v31, v12\n" ::
              : "v10", "v14", "v16", "v18", "v20", "v22", "v24", "v26");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + a9 + a10 + a11 + a12 + a13 + a14 + a15 + c;
  if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <int OP>
void run(const char *name, float *out, unsigned long long *cyc) {
  const int n = 2048;
  printf("%-22s", name);
  for (int w : {4, 8, 12, 16}) {
    hipLaunchKernelGGL(k_rate<OP>, 1, 64 * w, 0, 0, out, cyc, n);
    hipLaunchKernelGGL(k_rate<OP>, 1, 64 * w, 0, 0, out, cyc, n);
    (void)hipDeviceSynchronize();
    unsigned long long c[16];
    (void)hipMemcpy(c, cyc, 8 * w, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    for (int i = 0; i < w; ++i) mx = c[i] > mx ? c[i] : mx;
    // per SIMD: w/4 waves each issued 8n instructions in mx cycles
    printf("  %2d waves/CU: %5.2f cyc/instr/SIMD", w, (double)mx / (8.0 * n * (w / 4)));
  }
  printf("\n");
}

int main() {
  float *out;
  unsigned long long *cyc;
  (void)hipMalloc(&out, 4096 * 4);
  (void)hipMalloc(&cyc, 16 * 8);
  run<0>("v_pk_fma_f32", out, cyc);
  run<1>("v_pk_mul_f32", out, cyc);
  run<7>("v_pk_add_f32", out, cyc);
  run<9>("v_pk_mul_f32 (sgpr)", out, cyc);
  run<2>("v_cvt_pk_f32_fp8", out, cyc);
  run<8>("v_cvt_f32_ubyte0", out, cyc);
  run<3>("v_mul_f32", out, cyc);
  run<4>("v_fma_f32", out, cyc);
  run<6>("v_add_f32", out, cyc);
  run<5>("v_and_b32", out, cyc);
  run<10>("v_perm_b32", out, cyc);
  return 0;
}
