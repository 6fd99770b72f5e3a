"""A/B copy of vsim_amd/csrc/gemv_chain.hip whose chain32 consumer reads 8 pair terms per
ds_read_b128 (lanes 0-31 terms 8i..8i+3 of row lr, lanes 32-63 terms 8i+4..8i+7 of the same row)
and brings the upper half-wave's four down with v_permlane32_swap: half the LDS read
instructions of the consumer, four swaps each (independent of the chain).
usage: python tools/variants/mk_cons_perm.py OUT.hip G   (G reads per group, 8G adds)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import index_or_die  # noqa: E402

src = open("vsim_amd/csrc/gemv_chain.hip").read()
g = int(sys.argv[2])
a = index_or_die(src, "  // --------------------------------------------------------------- consumer (lanes 0-31)")
b = index_or_die(src, "  // ----------------------------------------------------------------- epilogue")
new = f"""  // --------------------------------------------------------------- consumer (lanes 0-31)
  float acc = 0.0f;
  constexpr int W2 = C2_WIN / 2, NR = CP / 8;  // reads in flight, reads per chunk (8 terms each)
  float4 win[W2];
  const int lr = lane & 31, hb = lane >> 5;
  auto src = [&](int c) {{ return &P[c % C2_RING][lr * LD + 4 * hb]; }};
  __builtin_amdgcn_s_setprio(3);
  __syncthreads();
  __syncthreads();
  for (int k = 0; k < nit; ++k) {{
    const int c = k - 2;
    if (c == -1 && nch > 0) {{
      const float *p0 = src(0);
#pragma unroll
      for (int j = 0; j < W2; ++j) win[j] = *(const float4 *)(p0 + 8 * j);
    }} else if (c >= 0 && c < nch) {{
      const float *pc = src(c), *pn = src(c + 1);
#pragma unroll
      for (int j0 = 0; j0 < NR; j0 += {g}) {{
#pragma unroll
        for (int j = j0; j < j0 + {g}; ++j) {{
          const float4 v = win[j % W2];
          const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(v.x), __float_as_uint(v.x), false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(__float_as_uint(v.y), __float_as_uint(v.y), false, false);
          const auto sz = __builtin_amdgcn_permlane32_swap(__float_as_uint(v.z), __float_as_uint(v.z), false, false);
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v.w), __float_as_uint(v.w), false, false);
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
          acc = acc + __uint_as_float(sx[1]);
          acc = acc + __uint_as_float(sy[1]);
          acc = acc + __uint_as_float(sz[1]);
          acc = acc + __uint_as_float(sw[1]);
        }}
#pragma unroll
        for (int j = j0; j < j0 + {g}; ++j) {{
          const int jn = j + W2;
          win[j % W2] = jn < NR ? *(const float4 *)(pc + 8 * jn) : *(const float4 *)(pn + 8 * (jn - NR));
        }}
      }}
    }}
    __syncthreads();
  }}

"""
src = src[:a] + new + src[b:]
open(sys.argv[1], "w").write(src)
