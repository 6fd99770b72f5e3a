"""A/B copy of vsim_amd/csrc/gemv_chain.hip (or of the file given as IN) whose chain32 consumer
reads and adds with lanes 0-31 only (exec-masked upper half: a 32-row tile's lanes 32-63 only
duplicated lanes 0-31, and their LDS reads double the data returned per ds_read_b128).
usage: python tools/variants/mk_cons_lo32.py OUT.hip [IN.hip]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from anchor import count_or_die  # noqa: E402

src = open(sys.argv[2] if len(sys.argv) > 2 else "vsim_amd/csrc/gemv_chain.hip").read()
old = """    if (c == -1 && nch > 0) {
      const float *p0 = src(0);"""
new = """    if (lane >= 32) {
    } else if (c == -1 && nch > 0) {
      const float *p0 = src(0);"""
count_or_die(src, old, 2)  # chain32's consumer first, then k_gemv_solo's
src = src.replace(old, new, 1)
open(sys.argv[1], "w").write(src)
