// tools/cons_lat5.hip — r05: can a chain take its terms from other lanes of its wave?  The dependent
// v_add_f32 with a DPP quad_perm source (lane 4r adds lane 4r+k's register, k = 0..3, so one
// ds_read_b128 over 64 lanes brings 16 terms for each of 16 rows instead of 4 for each of 64)
// against the plain dependent add, alone and inside a consumer loop of batches (reads one batch
// ahead, as the tail's consumer), one workgroup per CU on every CU.  Prints cycles per add.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int CP = 256, LD = 272;  // terms per chunk and row, row stride (floats)

#define DA(q, r) "v_add_f32_dpp %0, %" #r ", %0 quad_perm:[" q "] row_mask:0xf bank_mask:0xf\n\t"
#define DQ(r) DA("0,0,0,0", r) DA("1,1,1,1", r) DA("2,2,2,2", r) DA("3,3,3,3", r)
#define PA(r) "v_add_f32 %0, %0, %" #r "\n\t"

// 64 dependent adds: plain (operands in 16 registers x 4 components) or DPP (16 registers x 4 lanes)
__global__ void __launch_bounds__(64) k_chain(float *out, unsigned long long *cyc, int nrep, int dpp) {
  f32x4 v[4];
  for (int i = 0; i < 4; ++i) v[i] = f32x4{threadIdx.x * 1e-3f, 1e-4f, 2e-4f, 3e-4f};
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (dpp) {
    for (int r = 0; r < nrep; ++r)
      asm volatile(DQ(1) DQ(2) DQ(3) DQ(4) DQ(5) DQ(6) DQ(7) DQ(8) DQ(9) DQ(10) DQ(11) DQ(12) DQ(13) DQ(14) DQ(15) DQ(16)
                   : "+v"(acc)
                   : "v"(v[0].x), "v"(v[0].y), "v"(v[0].z), "v"(v[0].w), "v"(v[1].x), "v"(v[1].y), "v"(v[1].z),
                     "v"(v[1].w), "v"(v[2].x), "v"(v[2].y), "v"(v[2].z), "v"(v[2].w), "v"(v[3].x), "v"(v[3].y),
                     "v"(v[3].z), "v"(v[3].w));
  } else {
    for (int r = 0; r < nrep; ++r)
      asm volatile(PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15) PA(16)
                   PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15) PA(16)
                   PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15) PA(16)
                   PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15) PA(16)
                   : "+v"(acc)
                   : "v"(v[0].x), "v"(v[0].y), "v"(v[0].z), "v"(v[0].w), "v"(v[1].x), "v"(v[1].y), "v"(v[1].z),
                     "v"(v[1].w), "v"(v[2].x), "v"(v[2].y), "v"(v[2].z), "v"(v[2].w), "v"(v[3].x), "v"(v[3].y),
                     "v"(v[3].z), "v"(v[3].w));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// consumer loop over a 16-row x CP-term slot: DPP (lane 4r+k reads terms 16j+4k..+3 of row r; a
// batch = 8 reads = 128 terms per row, 128 adds) or plain (lane r < 32 reads 4 terms of row r per
// read, duplicated upper half; a batch = 8 reads = 32 adds), reads one batch ahead
#define ADD8D(acc, a)                                                                                          \
  asm volatile(DQ(1) DQ(2) DQ(3) DQ(4) DQ(5) DQ(6) DQ(7) DQ(8) DQ(9) DQ(10) DQ(11) DQ(12) DQ(13) DQ(14) DQ(15) DQ(16)  \
                   DQ(17) DQ(18) DQ(19) DQ(20) DQ(21) DQ(22) DQ(23) DQ(24) DQ(25) DQ(26) DQ(27) DQ(28) DQ(29) DQ(30)  \
                       DQ(31) DQ(32)                                                                         \
               : "+v"(acc)                                                                                   \
               : "v"(a[0].x), "v"(a[0].y), "v"(a[0].z), "v"(a[0].w), "v"(a[1].x), "v"(a[1].y), "v"(a[1].z),     \
                 "v"(a[1].w), "v"(a[2].x), "v"(a[2].y), "v"(a[2].z), "v"(a[2].w), "v"(a[3].x), "v"(a[3].y),      \
                 "v"(a[3].z), "v"(a[3].w), "v"(a[4].x), "v"(a[4].y), "v"(a[4].z), "v"(a[4].w), "v"(a[5].x),      \
                 "v"(a[5].y), "v"(a[5].z), "v"(a[5].w), "v"(a[6].x), "v"(a[6].y), "v"(a[6].z), "v"(a[6].w),      \
                 "v"(a[7].x), "v"(a[7].y), "v"(a[7].z), "v"(a[7].w)                                           \
               : "memory")
#define ADD8P(acc, a)                                                                                          \
  asm volatile(PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15) PA(16)  \
                   PA(17) PA(18) PA(19) PA(20) PA(21) PA(22) PA(23) PA(24) PA(25) PA(26) PA(27) PA(28) PA(29) PA(30)  \
                       PA(31) PA(32)                                                                         \
               : "+v"(acc)                                                                                   \
               : "v"(a[0].x), "v"(a[0].y), "v"(a[0].z), "v"(a[0].w), "v"(a[1].x), "v"(a[1].y), "v"(a[1].z),     \
                 "v"(a[1].w), "v"(a[2].x), "v"(a[2].y), "v"(a[2].z), "v"(a[2].w), "v"(a[3].x), "v"(a[3].y),      \
                 "v"(a[3].z), "v"(a[3].w), "v"(a[4].x), "v"(a[4].y), "v"(a[4].z), "v"(a[4].w), "v"(a[5].x),      \
                 "v"(a[5].y), "v"(a[5].z), "v"(a[5].w), "v"(a[6].x), "v"(a[6].y), "v"(a[6].z), "v"(a[6].w),      \
                 "v"(a[7].x), "v"(a[7].y), "v"(a[7].z), "v"(a[7].w)                                           \
               : "memory")

template <bool DPP, int PB>
__global__ void __launch_bounds__(576) k_loop(float *out, unsigned long long *cyc, int nrep) {
  __shared__ __attribute__((aligned(16))) float P[32 * LD];
  __shared__ __attribute__((aligned(16))) float W[8][64 * 20];
  for (int i = threadIdx.x; i < 32 * LD; i += blockDim.x) P[i] = (i & 15) * 1e-3f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= 1) {  // busy producers, as in tools/cons_lat4.hip
    const int p = wave - 1;
    if (p >= PB) return;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 a = {lane * 1e-3f, 1.0f}, b = {0.5f, 0.25f}, c = {1e-3f, 2e-3f};
    for (int k = 0; k < nrep * 8; ++k) {
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
  // DPP: lane 4r+k, row r (16 rows), 16-term groups; plain: lane l -> row l & 31
  const f32x4 *pr = DPP ? (const f32x4 *)&P[(lane >> 2) * LD] + (lane & 3) : (const f32x4 *)&P[(lane & 31) * LD];
  constexpr int STEP = DPP ? 4 : 1;  // float4 index step between a lane's consecutive reads
  constexpr int NB = DPP ? CP / 128 : CP / 32;  // batches per slot pass
  __builtin_amdgcn_s_setprio(3);
  f32x4 cur[8], nxt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cur[j] = pr[STEP * j];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < nrep; ++r) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int qn = (q + 1) % NB;
#pragma unroll
      for (int j = 0; j < 8; ++j) nxt[j] = pr[STEP * (8 * qn + j)];
      if constexpr (DPP)
        ADD8D(acc, cur);
      else
        ADD8P(acc, cur);
#pragma unroll
      for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int grid = 256, nrep = 64;
  float *out;
  unsigned long long *cyc, h[256];
  (void)hipMalloc(&out, grid * 64 * 4 + 65536);
  (void)hipMalloc(&cyc, grid * 8);
  auto report = [&](const char *what, double adds) {
    (void)hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid; ++i) s += h[i];
    printf("%-52s %5.2f cycles per add\n", what, s / grid / adds);
  };
  for (int d = 0; d < 2; ++d) {
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_chain, grid, 64, 0, 0, out, cyc, nrep, d);
    report(d ? "dependent v_add_f32_dpp quad_perm, alone" : "dependent v_add_f32, alone", nrep * 64.0);
  }
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_loop<false, 0>), grid, 64, 0, 0, out, cyc, nrep);
  report("plain loop (4 terms per read per row), alone", nrep * (double)CP);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_loop<true, 0>), grid, 64, 0, 0, out, cyc, nrep);
  report("DPP loop (16 terms per read per row), alone", nrep * (double)CP);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_loop<false, 8>), grid, 576, 0, 0, out, cyc, nrep);
  report("plain loop, 8 busy producers", nrep * (double)CP);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_loop<true, 8>), grid, 576, 0, 0, out, cyc, nrep);
  report("DPP loop, 8 busy producers", nrep * (double)CP);
  return 0;
}
