"""A/B copy of gemv_chain.hip + kern.hpp: the tail's heads store their out-projection operand
write-through (sc1, CO = true) and count after a vmcnt drain instead of an agent-scope release
fence (an L2 write-back per head); the out-projection tiles fetch the factors by sc1 LDS-DMA and
skip the agent-scope acquire (an L2 invalidate on their XCD, which also drops fc_out's lines).
usage: python tools/variants/mk_tail_coherent.py OUTDIR"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
g = open("vsim_amd/csrc/gemv_chain.hip").read()
k = open("vsim_amd/csrc/kern.hpp").read()


def rep(s, old, new):
    return replace_exact(s, old, new)


k = rep(k, "__device__ __forceinline__ void glds4(const void *g, uint32_t lds) {", """__device__ __forceinline__ void glds16_sc1(const void *g, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\\n\\ts_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %1, off sc1\\n\\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void *g, uint32_t lds) {""")
g = rep(g, "        glds16(x + (size_t)bx * QK + 4 * (lane & 7), lds_addr(&RX[slot][256 * p]));",
        "        glds16_sc1(x + (size_t)bx * QK + 4 * (lane & 7), lds_addr(&RX[slot][256 * p]));")
g = rep(g, """    attn_body<C2Tail::THREADS>(T.a, b, L.a);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every wave's output stores""",
        """    attn_body<C2Tail::THREADS, true>(T.a, b, L.a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-through output stores landed""")
g = rep(g, """  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  chain32_body(T.o, b, L.g);""", """  __syncthreads();
  chain32_body(T.o, b, L.g);""")
open(os.path.join(out, "gemv_chain.hip"), "w").write(g)
open(os.path.join(out, "kern.hpp"), "w").write(k)
