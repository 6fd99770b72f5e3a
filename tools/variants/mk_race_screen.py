"""Race screen (r06): copies of the product sources whose PRODUCING side of
every cross-wave / cross-workgroup hand-off is delayed by s_sleep (~3.4 us per RS_DELAY(1)), so
a consumer that reads before the hand-off's signal -- or a signal that does not order the data
-- reads stale bytes and the bit-exact tests fail.  Each delay sits where the data of the
hand-off is produced, ahead of its signal:
  attn.hpp      the new key row's stores (read back by other waves after the barrier; r05 race);
                the heads' output quantization (the out-projection waits for the head count)
  gemv_chain    a barrier-free GEMV producer's pair terms of every 5th chunk (the consumer waits
                on ready[]); the consumer's slot release every 7th chunk (producers wait on cons);
                the out-projection's granules (the fc_out owner polls their tags); an owner's
                partial-sum granules and its joined-row granules (every owner polls them)
  ops_elt       a third of the argmax workgroups' atomic max (the last counter reads ws)
usage: python tools/variants/mk_race_screen.py OUTDIR [--no-key-barrier]
  --no-key-barrier also removes the barrier between the key-row store and the KQ loads (the r05
  fix), to show the screen catches that race.  Build: tools/build_variant.sh NAME attn.hpp =OUTDIR/attn.hpp
  gemv_chain.hip =OUTDIR/gemv_chain.hip ops_elt.hip =OUTDIR/ops_elt.hip"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import replace_exact  # noqa: E402

out = sys.argv[1]
nobar = "--no-key-barrier" in sys.argv[2:]
os.makedirs(out, exist_ok=True)
DELAY = "#define RS_DELAY(n) do { for (int rs_ = 0; rs_ < (n); ++rs_) __builtin_amdgcn_s_sleep(127); } while (0)\n"

# ---------------------------------------------------------------- attn.hpp
s = open("vsim_amd/csrc/attn.hpp").read()
s = replace_exact(s, "#pragma once\n", "#pragma once\n" + DELAY)
s = replace_exact(s, "  for (int i = tid; i < d; i += ATT_THREADS) A.kc[(size_t)n_past * E + h * d + i] = kh[i];\n",
                  "  if (tid < d) RS_DELAY(3);\n"
                  "  for (int i = tid; i < d; i += ATT_THREADS) A.kc[(size_t)n_past * E + h * d + i] = kh[i];\n")
if nobar:
    s = replace_exact(s, """  // orders them.  r05: until then that read raced the store whenever n_past >= 16.
  __syncthreads();
""", """  // orders them.  r05: until then that read raced the store whenever n_past >= 16.
  // (race screen: barrier removed)
""")
s = replace_exact(s, "    quantize_half<CO>(y, lane, ok, A.oq_qs + (size_t)blk * 16, A.oq_d + blk, A.oxd + (size_t)blk * QK);\n",
                  "    if (CO && h % 3 == 0) RS_DELAY(2);\n"
                  "    quantize_half<CO>(y, lane, ok, A.oq_qs + (size_t)blk * 16, A.oq_d + blk, A.oxd + (size_t)blk * QK);\n")
open(os.path.join(out, "attn.hpp"), "w").write(s)

# ---------------------------------------------------------------- gemv_chain.hip
s = open("vsim_amd/csrc/gemv_chain.hip").read()
s = replace_exact(s, '#include "attn.hpp"\n', '#include "attn.hpp"\n' + DELAY)
# the barrier-free body's producer (the barrier version's line has the same text: 2 matches, the
# second is chain32_nb_body's)
old = """      const float dv = k * CB + o < nb ? dqc : 0.0f;
      const f32x2 d2 = {512.0f * dv, 512.0f * dv}, m2 = {-8.0f * dv, -8.0f * dv};
      float *dst = &L.P[slot][r * LD + o * 16];"""
s = replace_exact(s, old, "      if (p == k % NPW && k % 5 == 0) RS_DELAY(1);\n" + old)
s = replace_exact(s, "        __hip_atomic_store(&L.cons, (unsigned)(c + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n",
                  "      {\n        if (c % 7 == 3) RS_DELAY(1);\n"
                  "        __hip_atomic_store(&L.cons, (unsigned)(c + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n      }\n")
s = replace_exact(s, "  if (lane < 32 && row < rows) st_granule(N.og + row, acc, lnt_tag(N));\n",
                  "  if ((row >> 5) % 5 == 2) RS_DELAY(1);\n"
                  "  if (lane < 32 && row < rows) st_granule(N.og + row, acc, lnt_tag(N));\n")
s = replace_exact(s, "      st16_sc1(N.rec + 2 * t, u32x4{",
                  "      if (t % 7 == 3) RS_DELAY(1);\n      st16_sc1(N.rec + 2 * t, u32x4{")
s = replace_exact(s, "    st_granule(N.jg + i, v, tag);\n",
                  "    if (t % 4 == 1) RS_DELAY(1);\n    st_granule(N.jg + i, v, tag);\n")
open(os.path.join(out, "gemv_chain.hip"), "w").write(s)

# ---------------------------------------------------------------- ops_elt.hip
s = open("vsim_amd/csrc/ops_elt.hip").read()
s = replace_exact(s, '#include "kern.hpp"\n', '#include "kern.hpp"\n' + DELAY)
s = replace_exact(s, "  __hip_atomic_fetch_max(ws, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n",
                  "  if (blockIdx.x % 3 == 1) RS_DELAY(1);\n"
                  "  __hip_atomic_fetch_max(ws, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n")
open(os.path.join(out, "ops_elt.hip"), "w").write(s)
print("wrote", out, "(key barrier removed)" if nobar else "")
