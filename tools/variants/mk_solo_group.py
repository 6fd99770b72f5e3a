"""A/B copy of vsim_amd/csrc/gemv_chain.hip whose k_gemv_solo consumer issues its LDS reads in
groups of G (G reads back to back after every 4G adds), as chain32's consumer does since r04.
usage: python tools/variants/mk_solo_group.py OUT.hip G [WIN]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

src = open("vsim_amd/csrc/gemv_chain.hip").read()
g = int(sys.argv[2])
old = """#pragma unroll
      for (int j = 0; j < S::CP / 4; ++j) {
        const float4 v = win[j % S::WIN];
        acc = acc + v.x;
        acc = acc + v.y;
        acc = acc + v.z;
        acc = acc + v.w;
        const int jn = j + S::WIN;
        win[j % S::WIN] = jn < S::CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - S::CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU x4
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read x1
      }"""
new = f"""#pragma unroll
      for (int j0 = 0; j0 < S::CP / 4; j0 += {g}) {{
#pragma unroll
        for (int j = j0; j < j0 + {g}; ++j) {{
          const float4 v = win[j % S::WIN];
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }}
#pragma unroll
        for (int j = j0; j < j0 + {g}; ++j) {{
          const int jn = j + S::WIN;
          win[j % S::WIN] = jn < S::CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - S::CP / 4));
        }}
        __builtin_amdgcn_sched_group_barrier(0x002, {4 * g}, 0);  // VALU x{4 * g}
        __builtin_amdgcn_sched_group_barrier(0x100, {g}, 0);  // DS read x{g}
      }}"""
src = replace_exact(src, old, new)
if len(sys.argv) > 3:
    o = "  static constexpr int WIN = 12;"
    src = replace_exact(src, o, f"  static constexpr int WIN = {sys.argv[3]};")
open(sys.argv[1], "w").write(src)
