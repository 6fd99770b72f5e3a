// tools/cons_lat3.hip — the exact-decode consumer loop (one dependent add chain per lane over
// 16-byte LDS reads of pair terms, chunks of CP terms between barriers, a 3-slot ring written by
// three other waves) with two read schedules, one workgroup per CU on every CU:
//   rolling : one ds_read_b128 after every 4 adds, WIN reads ahead (gemv_chain.hip, r03)
//   burst   : reads in bursts of B ds_read_b128 for the next batch, then the 4B adds of the
//             current batch (two batches of registers)
// Producers idle (barriers only) or busy (packed VALU + ds_write_b128 of the next chunk).
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int RING = 3;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CP, int SCHED, int B, bool BUSY, bool RAW = false>
__global__ void __launch_bounds__(256) k_cons(float *out, unsigned long long *cyc, int nch) {
  constexpr int LD = CP + 4, NV = CP / 4;
  __shared__ __attribute__((aligned(16))) float P[RING][64 * LD];
  for (int i = threadIdx.x; i < RING * 64 * LD; i += 256) (&P[0][0])[i] = (i & 15) * 1e-3f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave > 0) {
    f32x2 a = {lane * 1e-3f, 1.0f}, b = {0.5f, 0.25f}, c = {1e-3f, 2e-3f};
    for (int k = 0; k < nch + 2; ++k) {
      if (BUSY) {
#pragma unroll
        for (int i = 0; i < 68; ++i) a = __builtin_elementwise_fma(a, b, c);
        float *dst = &P[k % RING][lane * LD + ((wave - 1) * 16) % CP];
#pragma unroll
        for (int w = 0; w < 4; ++w) *(float4 *)(dst + 4 * w) = make_float4(a.x, a.y, a.x, a.y);
      }
      __syncthreads();
    }
    if (lane == 0) out[blockIdx.x * 4 + wave] = a.x + a.y;
    return;
  }
  float acc = 0.f;
  __builtin_amdgcn_s_setprio(3);
  unsigned long long t0 = 0;
  auto src = [&](int c) { return (const f32x4 *)&P[c % RING][lane * LD]; };
  if constexpr (SCHED == 0) {
    constexpr int WIN = B;
    f32x4 win[WIN];
    for (int k = 0; k < nch + 2; ++k) {
      const int ch = k - 2;
      if (ch == -1) {
#pragma unroll
        for (int j = 0; j < WIN; ++j) win[j] = src(0)[j];
        t0 = __builtin_amdgcn_s_memtime();
      } else if (ch >= 0 && ch < nch) {
        const f32x4 *pc = src(ch), *pn = src(ch + 1);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const f32x4 v = win[j % WIN];
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
          const int jn = j + WIN;
          win[j % WIN] = jn < NV ? pc[jn] : pn[jn - NV];
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
      if (RAW) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      } else {
        __syncthreads();
      }
    }
  } else {
    // bursts: batch q of chunk ch = vectors [q B, q B + B); NB batches per chunk
    constexpr int NB = NV / B;
    static_assert(NV % B == 0, "batches tile the chunk");
    f32x4 cur[B], nxt[B];
    for (int k = 0; k < nch + 2; ++k) {
      const int ch = k - 2;
      if (ch == -1) {
#pragma unroll
        for (int j = 0; j < B; ++j) cur[j] = src(0)[j];
        t0 = __builtin_amdgcn_s_memtime();
      } else if (ch >= 0 && ch < nch) {
        const f32x4 *pc = src(ch), *pn = src(ch + 1);
#pragma unroll
        for (int q = 0; q < NB; ++q) {
#pragma unroll
          for (int j = 0; j < B; ++j) nxt[j] = q + 1 < NB ? pc[(q + 1) * B + j] : pn[j];
#pragma unroll
          for (int j = 0; j < B; ++j) {
            acc = acc + cur[j].x;
            acc = acc + cur[j].y;
            acc = acc + cur[j].z;
            acc = acc + cur[j].w;
          }
          __builtin_amdgcn_sched_group_barrier(0x100, B, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4 * B, 0);
#pragma unroll
          for (int j = 0; j < B; ++j) cur[j] = nxt[j];
        }
      }
      if (RAW) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      } else {
        __syncthreads();
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 4] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CP, int SCHED, int B, bool BUSY, bool RAW = false>
void run(float *out, unsigned long long *cyc, unsigned long long *h, int grid) {
  const int nch = 8192 / CP;  // fc_out: K/2 = 8192 terms per row
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_cons<CP, SCHED, B, BUSY, RAW>), grid, 256, 0, 0, out, cyc, nch);
  (void)hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; ++i) s += h[i];
  printf("chunk %3d, %-7s %2d, producers %-4s, %s barrier: %5.2f cycles per add\n", CP, SCHED ? "burst" : "rolling", B,
         BUSY ? "busy" : "idle", RAW ? "raw " : "sync", s / grid / (nch * (double)CP));
}

int main() {
  const int grid = 256;
  float *out;
  unsigned long long *cyc, h[256];
  (void)hipMalloc(&out, grid * 16);
  (void)hipMalloc(&cyc, grid * 8);
  run<128, 0, 8, false>(out, cyc, h, grid);
  run<128, 0, 16, false>(out, cyc, h, grid);
  run<128, 1, 4, false>(out, cyc, h, grid);
  run<128, 1, 8, false>(out, cyc, h, grid);
  run<128, 1, 16, false>(out, cyc, h, grid);
  run<128, 0, 16, true>(out, cyc, h, grid);
  run<128, 1, 8, true>(out, cyc, h, grid);
  run<96, 0, 8, true>(out, cyc, h, grid);
  run<96, 1, 8, true>(out, cyc, h, grid);
  run<96, 1, 12, true>(out, cyc, h, grid);
  run<128, 0, 8, false, true>(out, cyc, h, grid);
  run<128, 0, 16, true, true>(out, cyc, h, grid);
  run<128, 1, 8, false, true>(out, cyc, h, grid);
  run<128, 1, 16, false, true>(out, cyc, h, grid);
  run<128, 1, 8, true, true>(out, cyc, h, grid);
  run<128, 1, 16, true, true>(out, cyc, h, grid);
  run<96, 0, 8, true, true>(out, cyc, h, grid);
  run<96, 1, 12, true, true>(out, cyc, h, grid);
  return 0;
}
