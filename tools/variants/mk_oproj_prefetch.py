"""A/B copy of vsim_amd/csrc/gemv_chain.hip whose k_layer_tail out-projection tiles load their
first NCH chunks of weights (nibbles and scales) once while they wait for the heads, so the LDS-DMA
after the wait hits L2.  usage: python tools/variants/mk_oproj_prefetch.py OUT.hip NCH"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

src = open("vsim_amd/csrc/gemv_chain.hip").read()
nch = int(sys.argv[2])
old = """  b -= na;
  if (threadIdx.x == 0) {
    unsigned spins = 0;"""
new = f"""  b -= na;
  {{  // the tile's first {nch} chunks of weights into L2 while the heads run
    int t = b, ji = 0;
    while (ji < T.o.nj && t >= T.o.j[ji].w.tiles) t -= T.o.j[ji].w.tiles, ++ji;
    if (ji < T.o.nj) {{
      const W4 &w = T.o.j[ji].w;
      const int nb = w.k / QK, nblk = min(nb, {nch} * C2Tail::CB);
      const uint8_t *q = w.qs + (size_t)t * nb * T32 * 16;
      const uint8_t *d = (const uint8_t *)(w.d + (size_t)t * nb * T32);
      for (int i = threadIdx.x; i < nblk * T32 * 16 / 16; i += C2Tail::THREADS) {{
        u32x4 r;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(q + 16 * (size_t)i) : "memory");
      }}
      for (int i = threadIdx.x; i < nblk * T32 * 4 / 16; i += C2Tail::THREADS) {{
        u32x4 r;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(d + 16 * (size_t)i) : "memory");
      }}
    }}
  }}
  if (threadIdx.x == 0) {{
    unsigned spins = 0;"""
src = replace_exact(src, old, new)
old2 = """  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  chain32_body(T.o, b, L.g);"""
new2 = """  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  chain32_body(T.o, b, L.g);"""
src = replace_exact(src, old2, new2)
open(sys.argv[1], "w").write(src)
