"""Writes a diagnostic copy of vsim_amd/csrc/gemv_chain.hip (and of attn.hpp, as OUTDIR/attn.hpp)
whose k_layer_tail records s_memrealtime (100 MHz, one clock for the chip) per workgroup role:
fc_out tiles [start, end], heads [start, after KQ, after softmax, after KQV, end], out-projection
tiles [start, wait over, end], into g_tail_tl[workgroup][8], read back by
vsim_debug_tail_timeline(host, bytes).  The last tail launched (layer 27 of the last token) is kept.
usage: python tools/variants/mk_tail_timeline.py OUTDIR  (then build_variant.sh NAME
gemv_chain.hip =OUTDIR/gemv_chain.hip attn.hpp =OUTDIR/attn.hpp)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
g = open("vsim_amd/csrc/gemv_chain.hip").read()
a = open("vsim_amd/csrc/attn.hpp").read()


def rep(s, old, new):
    return replace_exact(s, old, new)


a = rep(a, "namespace vsim {\n", """namespace vsim {
__device__ unsigned long long g_tail_tl[512][8];
__device__ __forceinline__ void tl_mark(int wg, int i) {
  if (wg >= 0 && threadIdx.x == 0) g_tail_tl[wg][i] = __builtin_amdgcn_s_memrealtime();
}
""")
a = rep(a, "__device__ __forceinline__ void attn_body(const AttnJob &A, int hs, float *sm) {",
        "__device__ __forceinline__ void attn_body(const AttnJob &A, int hs, float *sm, int tl = -1) {\n  tl_mark(tl, 0);")
a = rep(a, """  // max, exp via table, exact double sum (fp16 values: any order), 1/sum
  mx = wave_max_f(mx);""", """  // max, exp via table, exact double sum (fp16 values: any order), 1/sum
  tl_mark(tl, 1);
  mx = wave_max_f(mx);""")
a = rep(a, """  for (int k = tid; k < nk; k += ATT_THREADS) pr[k] = pr[k] * inv;
  __syncthreads();""", """  for (int k = tid; k < nk; k += ATT_THREADS) pr[k] = pr[k] * inv;
  __syncthreads();
  tl_mark(tl, 2);""")
a = rep(a, """  // quantize the part's outputs: wave w holds columns c0 + 64w .. +63, two 32-blocks""",
        """  tl_mark(tl, 3);
  // quantize the part's outputs: wave w holds columns c0 + 64w .. +63, two 32-blocks""")
g = rep(g, """  int b = blockIdx.x;
  if (b < T.nf) {
    chain32_body(T.f, b, L.g);
    return;
  }""", """  int b = blockIdx.x;
  const int wg = blockIdx.x < 512 ? (int)blockIdx.x : -1;
  if (b < T.nf) {
    tl_mark(wg, 0);
    chain32_body(T.f, b, L.g);
    __syncthreads();
    tl_mark(wg, 1);
    return;
  }""")
g = rep(g, """    attn_body<C2Tail::THREADS, true>(T.a, b, L.a);""", """    attn_body<C2Tail::THREADS, true>(T.a, b, L.a, wg);""")
g = rep(g, """    if (threadIdx.x == 0) __hip_atomic_fetch_add(T.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  b -= na;""", """    if (threadIdx.x == 0) __hip_atomic_fetch_add(T.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tl_mark(wg, 4);
    return;
  }
  b -= na;
  tl_mark(wg, 0);""")
g = rep(g, """  __syncthreads();
  chain32_body(T.o, b, L.g);""", """  __syncthreads();
  tl_mark(wg, 1);
  chain32_body(T.o, b, L.g);
  __syncthreads();
  tl_mark(wg, 2);""")
g += """
extern "C" int vsim_debug_tail_timeline(void *host, size_t bytes) {
  if (bytes > sizeof(vsim::g_tail_tl)) bytes = sizeof(vsim::g_tail_tl);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(vsim::g_tail_tl), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
"""
open(os.path.join(out, "gemv_chain.hip"), "w").write(g)
open(os.path.join(out, "attn.hpp"), "w").write(a)
