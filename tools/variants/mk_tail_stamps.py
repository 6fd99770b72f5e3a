"""Writes a diagnostic copy of vsim_amd/csrc/gemv_chain.hip whose k_layer_tail fc_out tiles
stamp s_memtime per chunk step into the launch's dynamic LDS pad (no extra global memory ops
inside the loop), copied at the tile's end to a device array read back by
vsim_debug_tail_stamps(host, bytes).  Build: python tools/variants/mk_tail_stamps.py OUT.hip, then
tools/build_variant.sh stamps gemv_chain.hip =OUT.hip.  Stamps per tile and step k (u64):
 [0] consumer at the step's top, [1] consumer after its adds, [2] consumer after the barrier,
 [3..6] producer wave 1 (p = 0): top, after the pair terms and stores, after its vmcnt wait,
 after the barrier; [7..10] the same for p = 2 (wave 3); [11] s_memrealtime
 at the consumer's step top (100 MHz)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

src = open("vsim_amd/csrc/gemv_chain.hip").read()


def rep(old, new, count=1):
    global src
    src = replace_exact(src, old, new, count)


rep("""__device__ __forceinline__ void producer_barrier()""",
    """constexpr int ST_K = 72, ST_N = 12;
__device__ unsigned long long g_tail_stamps[128][ST_K][ST_N];
__device__ __forceinline__ unsigned long long stamp_now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void producer_barrier()""")
rep("""__device__ __forceinline__ void chain32_body(const GemvBatch &B, int t, C2Lds<S> &L) {""",
    """__device__ __forceinline__ void chain32_body(const GemvBatch &B, int t, C2Lds<S> &L,
                                             unsigned long long *st = nullptr) {""")
# producer step stamps
rep("""    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const uint4 &qc, float dqc, uint4 &qn, float &dqn) {
      ldraw(k + 1, qn, dqn, xn);""",
    """    const int sp = p == 0 ? 3 : (p == 2 ? 7 : -1);
    auto stp = [&](int k, int i) {
      if (st && sp >= 0 && lane == 0 && k < ST_K) st[k * ST_N + sp + i] = stamp_now();
    };
    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const uint4 &qc, float dqc, uint4 &qn, float &dqn) {
      stp(k, 0);
      ldraw(k + 1, qn, dqn, xn);""")
rep("""      ps = ps == C2_RING - 1 ? 0 : ps + 1;
      if (xp)  // this wave's DMA of chunk k+2 landed
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM3);
      else
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM2);
      __syncthreads();
    };""",
    """      ps = ps == C2_RING - 1 ? 0 : ps + 1;
      stp(k, 1);
      if (xp)  // this wave's DMA of chunk k+2 landed
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM3);
      else
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM2);
      stp(k, 2);
      __syncthreads();
      stp(k, 3);
    };""")
rep("""  for (int k = 0; k < nit; ++k) {
    const int c = k - 2;
    if (c == -1 && nch > 0) {""",
    """  for (int k = 0; k < nit; ++k) {
    const int c = k - 2;
    if (st && lane == 0 && k < ST_K) {
      st[k * ST_N + 0] = stamp_now();
      st[k * ST_N + 11] = __builtin_amdgcn_s_memrealtime();
    }
    if (c == -1 && nch > 0) {""")
rep("""      }
    }
    __syncthreads();
  }

  // ----------------------------------------------------------------- epilogue""",
    """      }
    }
    if (st && lane == 0 && k < ST_K) st[k * ST_N + 1] = stamp_now();
    __syncthreads();
    if (st && lane == 0 && k < ST_K) st[k * ST_N + 2] = stamp_now();
  }

  // ----------------------------------------------------------------- epilogue""")
rep("""  int b = blockIdx.x;
  if (b < T.nf) {
    chain32_body(T.f, b, L.g);
    return;
  }""",
    """  extern __shared__ unsigned long long st_lds[];
  int b = blockIdx.x;
  if (b < T.nf) {
    for (int i = threadIdx.x; i < ST_K * ST_N; i += blockDim.x) st_lds[i] = 0;
    __syncthreads();
    chain32_body(T.f, b, L.g, b < 128 ? st_lds : nullptr);
    __syncthreads();
    if (b < 128)
      for (int i = threadIdx.x; i < ST_K * ST_N; i += blockDim.x) (&g_tail_stamps[b][0][0])[i] = st_lds[i];
    return;
  }""")
rep("""  hipLaunchKernelGGL(k_layer_tail, dim3(T.nf + a.H * S + no), dim3(C2Tail::THREADS), 8192, s, T);""",
    """  static_assert(ST_K * ST_N * 8 <= 8192, "stamps fit the dynamic pad");
  hipLaunchKernelGGL(k_layer_tail, dim3(T.nf + a.H * S + no), dim3(C2Tail::THREADS), 8192, s, T);""")
src += """
extern "C" int vsim_debug_tail_stamps(void *host, size_t bytes) {
  if (bytes > sizeof(vsim::g_tail_stamps)) bytes = sizeof(vsim::g_tail_stamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(vsim::g_tail_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
"""
open(sys.argv[1], "w").write(src)
