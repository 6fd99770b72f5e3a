// tools/cons_lat.hip — cycles per add of the exact-decode consumer loop (gemv_chain.hip's
// rolling window of 16-byte LDS reads feeding one dependent v_add_f32 chain per lane), one
// workgroup per CU on every CU, under four loads on the other SIMDs:
//   idle    : the other three waves only meet the per-chunk barrier
//   stores  : they write the next chunk's pair terms (ds_write_b128, the producers' LDS traffic)
//   valu    : they run the producers' arithmetic (packed f32, ~68 instructions per chunk step)
//   both    : stores + arithmetic (the real producer side)
// and with read windows of 8 and 16.  Cycles from s_memtime over the chunk loop of wave 0.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int CP = 96, LD = CP + 4, RING = 3;  // 96 pair terms per chunk and row (k_gemv_solo)
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int WIN, int MODE>
__global__ void __launch_bounds__(256) k_cons(float *out, unsigned long long *cyc, int nch) {
  __shared__ __attribute__((aligned(16))) float P[RING][64 * LD];
  for (int i = threadIdx.x; i < RING * 64 * LD; i += 256) (&P[0][0])[i] = (i & 15) * 1e-3f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave > 0) {
    f32x2 a = {lane * 1e-3f, 1.0f}, b = {0.5f, 0.25f}, c = {1e-3f, 2e-3f};
    for (int k = 0; k < nch + 2; ++k) {
      if (MODE & 2) {
#pragma unroll
        for (int i = 0; i < 68; ++i) a = __builtin_elementwise_fma(a, b, c);
      }
      if (MODE & 1) {  // 16 pairs x 64 rows of this producer's block per chunk, as 4 float4 per lane
        float *dst = &P[k % RING][lane * LD + (wave - 1) * 16];
#pragma unroll
        for (int w = 0; w < 4; ++w) *(float4 *)(dst + 4 * w) = make_float4(a.x, a.y, a.x, a.y);
      }
      __syncthreads();
    }
    if (lane == 0) out[blockIdx.x * 4 + wave] = a.x + a.y;
    return;
  }
  float acc = 0.f;
  float4 win[WIN];
  __builtin_amdgcn_s_setprio(3);
  unsigned long long t0 = 0;
  for (int k = 0; k < nch + 2; ++k) {
    const int ch = k - 2;
    if (ch == -1) {
      const float *p0 = &P[0][lane * LD];
#pragma unroll
      for (int j = 0; j < WIN; ++j) win[j] = *(const float4 *)(p0 + 4 * j);
      t0 = __builtin_amdgcn_s_memtime();
    } else if (ch >= 0 && ch < nch) {
      const float *pc = &P[ch % RING][lane * LD], *pn = &P[(ch + 1) % RING][lane * LD];
#pragma unroll
      for (int j = 0; j < CP / 4; ++j) {
        const float4 v = win[j % WIN];
        acc = acc + v.x;
        acc = acc + v.y;
        acc = acc + v.z;
        acc = acc + v.w;
        const int jn = j + WIN;
        win[j % WIN] = jn < CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 4] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

static const char *kMode[] = {"idle", "stores", "valu", "both"};

template <int WIN, int MODE>
void run(float *out, unsigned long long *cyc, unsigned long long *h, int grid) {
  const int nch = 86;  // 8256 pairs: fc_out's K/2 = 8192 in chunks of 96
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_cons<WIN, MODE>), grid, 256, 0, 0, out, cyc, nch);
  (void)hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; ++i) s += h[i];
  printf("window %2d, others %-6s: %5.2f cycles per add (mean of %d workgroups)\n", WIN, kMode[MODE],
         s / grid / (nch * (double)CP), grid);
}

int main() {
  const int grid = 256;
  float *out;
  unsigned long long *cyc, h[256];
  (void)hipMalloc(&out, grid * 16);
  (void)hipMalloc(&cyc, grid * 8);
  run<8, 0>(out, cyc, h, grid);
  run<8, 1>(out, cyc, h, grid);
  run<8, 2>(out, cyc, h, grid);
  run<8, 3>(out, cyc, h, grid);
  run<12, 3>(out, cyc, h, grid);
  run<24, 0>(out, cyc, h, grid);
  run<24, 3>(out, cyc, h, grid);
  return 0;
}
