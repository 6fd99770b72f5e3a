// tools/cons_lat4.hip — r05: the exact-decode consumer loop as built in gemv_chain.hip's barrier-free
// GEMVs (batches of BQ ds_read_b128 issued one batch ahead of their 4*BQ dependent v_add_f32 in one
// volatile asm statement), one workgroup per CU on every CU, varying
//   NC : consumer waves per workgroup (waves 0..NC-1: consecutive waves sit on different SIMDs)
//   AL : active lanes per consumer (64, 32 or 16 rows)
//   PB : busy "producer" waves (every wave not a consumer, up to 8) storing ds_write_b128 terms into
//        a second LDS region beside VALU work, as the real producers do; 0 = idle
// and prints cycles per add of one chain (s_memtime, mean over workgroups).  The loads cannot be
// hoisted: a memory clobber separates the batches (tools/cons_lat2.hip's "batch8" row was hoisted).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int CP = 256, LD = CP + 4, NBATCH = CP / 32;

#define A4(i) "v_add_f32 %0, %0, %" #i "\n\t"
#define ADDS8(acc, a)                                                                                        \
  asm volatile(A4(1) A4(2) A4(3) A4(4) A4(5) A4(6) A4(7) A4(8) A4(9) A4(10) A4(11) A4(12) A4(13) A4(14) A4(15) \
                   A4(16) A4(17) A4(18) A4(19) A4(20) A4(21) A4(22) A4(23) A4(24) A4(25) A4(26) A4(27) A4(28)  \
                       A4(29) A4(30) A4(31) A4(32)                                                         \
               : "+v"(acc)                                                                                 \
               : "v"(a[0].x), "v"(a[0].y), "v"(a[0].z), "v"(a[0].w), "v"(a[1].x), "v"(a[1].y), "v"(a[1].z),   \
                 "v"(a[1].w), "v"(a[2].x), "v"(a[2].y), "v"(a[2].z), "v"(a[2].w), "v"(a[3].x), "v"(a[3].y),    \
                 "v"(a[3].z), "v"(a[3].w), "v"(a[4].x), "v"(a[4].y), "v"(a[4].z), "v"(a[4].w), "v"(a[5].x),    \
                 "v"(a[5].y), "v"(a[5].z), "v"(a[5].w), "v"(a[6].x), "v"(a[6].y), "v"(a[6].z), "v"(a[6].w),    \
                 "v"(a[7].x), "v"(a[7].y), "v"(a[7].z), "v"(a[7].w)                                         \
               : "memory")

template <int NC, int AL, int PB>
__global__ void __launch_bounds__(576) k_cons(float *out, unsigned long long *cyc, int nrep) {
  __shared__ __attribute__((aligned(16))) float P[64 * LD];
  __shared__ __attribute__((aligned(16))) float W[8][64 * 20];
  for (int i = threadIdx.x; i < 64 * LD; i += blockDim.x) P[i] = (i & 15) * 1e-3f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= NC) {
    const int p = wave - NC;
    if (p >= PB) return;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 a = {lane * 1e-3f, 1.0f}, b = {0.5f, 0.25f}, c = {1e-3f, 2e-3f};
    for (int k = 0; k < nrep * NBATCH / 8; ++k) {  // ~ the real producers' 68 VALU + 4 stores per 256-term chunk
#pragma unroll
      for (int i = 0; i < 68; ++i) a = __builtin_elementwise_fma(a, b, c);
#pragma unroll
      for (int w = 0; w < 4; ++w) *(float4 *)&W[p][lane * 20 + 4 * w] = make_float4(a.x, a.y, a.x, a.y);
      asm volatile("" ::: "memory");
    }
    if (lane == 0) out[4096 + blockIdx.x * 8 + p] = a.x + a.y;
    return;
  }
  float acc = 0.f;
  const int row = (wave * AL + lane) & 63;
  __builtin_amdgcn_s_setprio(3);
  unsigned long long t0 = 0, t1 = 0;
  if (lane < AL) {
    const f32x4 *pr = (const f32x4 *)&P[row * LD];
    f32x4 cur[8], nxt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cur[j] = pr[j];
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nrep; ++r) {
#pragma unroll
      for (int q = 0; q < NBATCH; ++q) {
        const int qn = (q + 1) % NBATCH;
#pragma unroll
        for (int j = 0; j < 8; ++j) nxt[j] = pr[8 * qn + j];
        ADDS8(acc, cur);
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
      }
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0 && wave == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NC, int AL, int PB>
void run(float *out, unsigned long long *cyc, unsigned long long *h, int grid) {
  const int nrep = 64;
  const int threads = 64 * (NC + (PB > 0 ? PB : 0));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_cons<NC, AL, PB>), grid, threads, 0, 0, out, cyc, nrep);
  (void)hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; ++i) s += h[i];
  printf("consumers %d x %2d lanes, %d busy producers: %5.2f cycles per add\n", NC, AL, PB,
         s / grid / (nrep * (double)CP));
}


// IL: the reads of batch i+2 interleaved with the adds of batch i inside one asm statement
// (one ds_read_b128 after every 4 adds), three register sets, an explicit lgkmcnt(8) at the top
#define IL_ASM(acc, a, c, addr, off)                                                                        \
  asm volatile("s_waitcnt lgkmcnt(8)\n\t"                                                                  \
               A4(10) "ds_read_b128 %1, %42 offset:" #off "+0\n\t" A4(11) A4(12) A4(13) A4(14)               \
               "ds_read_b128 %2, %42 offset:" #off "+16\n\t" A4(15) A4(16) A4(17) A4(18)                     \
               "ds_read_b128 %3, %42 offset:" #off "+32\n\t" A4(19) A4(20) A4(21) A4(22)                     \
               "ds_read_b128 %4, %42 offset:" #off "+48\n\t" A4(23) A4(24) A4(25) A4(26)                     \
               "ds_read_b128 %5, %42 offset:" #off "+64\n\t" A4(27) A4(28) A4(29) A4(30)                     \
               "ds_read_b128 %6, %42 offset:" #off "+80\n\t" A4(31) A4(32) A4(33) A4(34)                     \
               "ds_read_b128 %7, %42 offset:" #off "+96\n\t" A4(35) A4(36) A4(37) A4(38)                     \
               "ds_read_b128 %8, %42 offset:" #off "+112\n\t" A4(39) A4(40) A4(41)                          \
               : "+v"(acc), "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3]), "=&v"(c[4]), "=&v"(c[5]),        \
                 "=&v"(c[6]), "=&v"(c[7])                                                                  \
               : "v"(a[0].x), "v"(a[0].y), "v"(a[0].z), "v"(a[0].w), "v"(a[1].x), "v"(a[1].y), "v"(a[1].z),   \
                 "v"(a[1].w), "v"(a[2].x), "v"(a[2].y), "v"(a[2].z), "v"(a[2].w), "v"(a[3].x), "v"(a[3].y),    \
                 "v"(a[3].z), "v"(a[3].w), "v"(a[4].x), "v"(a[4].y), "v"(a[4].z), "v"(a[4].w), "v"(a[5].x),    \
                 "v"(a[5].y), "v"(a[5].z), "v"(a[5].w), "v"(a[6].x), "v"(a[6].y), "v"(a[6].z), "v"(a[6].w),    \
                 "v"(a[7].x), "v"(a[7].y), "v"(a[7].z), "v"(a[7].w), "v"(addr)                              \
               : "memory")

template <int AL>
__global__ void __launch_bounds__(64) k_il(float *out, unsigned long long *cyc, int nrep) {
  __shared__ __attribute__((aligned(16))) float P[64 * LD];
  for (int i = threadIdx.x; i < 64 * LD; i += blockDim.x) P[i] = (i & 15) * 1e-3f;
  __syncthreads();
  const int lane = threadIdx.x;
  float acc = 0.f;
  unsigned long long t0 = 0, t1 = 0;
  if (lane < AL) {
    const f32x4 *pr = (const f32x4 *)&P[lane * LD];
    const unsigned addr = (unsigned)(uintptr_t)&P[lane * LD];
    f32x4 b0[8], b1[8], b2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      b0[j] = pr[j];
      b1[j] = pr[8 + j];
    }
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nrep; ++r) {  // 8 batches per rep: 0..5 in two rotations, then 6, 7
      IL_ASM(acc, b0, b2, addr, 256);
      IL_ASM(acc, b1, b0, addr, 384);
      IL_ASM(acc, b2, b1, addr, 512);
      IL_ASM(acc, b0, b2, addr, 640);
      IL_ASM(acc, b1, b0, addr, 768);
      IL_ASM(acc, b2, b1, addr, 896);
      IL_ASM(acc, b0, b2, addr, 0);
      IL_ASM(acc, b1, b0, addr, 128);
      // (b2, b0 hold batches 0, 1 of the next rep: rotate names back)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 t = b2[j];
        b2[j] = b1[j];
        b1[j] = b0[j];
        b0[j] = t;
      }
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int AL>
void run_il(float *out, unsigned long long *cyc, unsigned long long *h, int grid) {
  const int nrep = 64;
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_il<AL>), grid, 64, 0, 0, out, cyc, nrep);
  (void)hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; ++i) s += h[i];
  printf("interleaved asm, 1 consumer x %2d lanes:  %5.2f cycles per add\n", AL, s / grid / (nrep * (double)CP));
}

int main() {
  const int grid = 256;
  float *out;
  unsigned long long *cyc, h[256];
  (void)hipMalloc(&out, grid * 64 * 4 + 65536);
  (void)hipMalloc(&cyc, grid * 8);
  run<1, 64, 0>(out, cyc, h, grid);
  run<1, 32, 0>(out, cyc, h, grid);
  run<1, 16, 0>(out, cyc, h, grid);
  run<2, 64, 0>(out, cyc, h, grid);
  run<2, 32, 0>(out, cyc, h, grid);
  run<4, 32, 0>(out, cyc, h, grid);
  run<4, 16, 0>(out, cyc, h, grid);
  run<1, 32, 8>(out, cyc, h, grid);
  run<1, 64, 6>(out, cyc, h, grid);
  run<2, 32, 6>(out, cyc, h, grid);
  run<4, 16, 4>(out, cyc, h, grid);
  run_il<64>(out, cyc, h, grid);
  run_il<32>(out, cyc, h, grid);
  return 0;
}
