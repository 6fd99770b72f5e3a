"""A/B copy of vsim_amd/csrc/gemv_chain.hip whose chain32 consumer issues its LDS reads in
groups of G (G reads back to back after every 4G adds; one lgkmcnt wait per group instead of
one per read), optionally with the tail shape replaced.
usage: python tools/variants/mk_cons_group.py OUT.hip G ["CB, DEPTH, FILL"]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

src = open("vsim_amd/csrc/gemv_chain.hip").read()
g = int(sys.argv[2])
old = """#pragma unroll
      for (int j = 0; j < CP / 4; ++j) {
        const float4 v = win[j % C2_WIN];
        acc = acc + v.x;
        acc = acc + v.y;
        acc = acc + v.z;
        acc = acc + v.w;
        const int jn = j + C2_WIN;
        win[j % C2_WIN] = jn < CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }"""
new = f"""#pragma unroll
      for (int j0 = 0; j0 < CP / 4; j0 += {g}) {{
#pragma unroll
        for (int j = j0; j < j0 + {g}; ++j) {{
          const float4 v = win[j % C2_WIN];
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }}
#pragma unroll
        for (int j = j0; j < j0 + {g}; ++j) {{
          const int jn = j + C2_WIN;
          win[j % C2_WIN] = jn < CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - CP / 4));
        }}
        __builtin_amdgcn_sched_group_barrier(0x002, {4 * g}, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, {g}, 0);
      }}"""
src = replace_exact(src, old, new)
if len(sys.argv) > 3:
    o = "using C2Tail = C2Shape<8, 8, false>;"
    src = replace_exact(src, o, f"using C2Tail = C2Shape<{sys.argv[3]}>;")
open(sys.argv[1], "w").write(src)
