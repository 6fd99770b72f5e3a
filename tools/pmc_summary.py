"""Per-kernel, per-grid-size means of rocprofv3 --pmc counters (every counter_collection.csv
under the given directories) for kernels whose name contains the filter, plus the ratios
that say what bounds them:
  issue  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES   (both in quad-cycles: share of a wave's life
           spent issuing)
  wait   = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waiting on a dependency, a counter or a barrier)
  mfma   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 4 x CUs)  (MFMA pipe busy share of
           every SIMD's cycles over the dispatch; GRBM_GUI_ACTIVE sums the 8 XCDs)
usage: python tools/pmc_summary.py DIR [DIR...] FILTER [CUS]"""
import collections
import csv
import glob
import os
import sys


def main():
    args = sys.argv[1:]
    cus = 256
    if args and args[-1].isdigit():
        cus = int(args.pop())
    filt = args.pop()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if filt not in name:
                    continue
                key = (name.split("(")[0][:60], r["Grid_Size"])
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in sorted(vals.items()):
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        print(f"{name}  grid {grid}  ({len(next(iter(cs.values())))} dispatches)")
        for k in sorted(m):
            print(f"    {k:28s} {m[k]:16.1f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            if "SQ_ACTIVE_INST_ANY" in m:
                print(f"    issue share {m['SQ_ACTIVE_INST_ANY'] / wc:.3f}")
            if "SQ_WAIT_ANY" in m:
                print(f"    wait share  {m['SQ_WAIT_ANY'] / wc:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            print(f"    MFMA busy share of SIMD cycles {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 4 * cus):.3f}")


if __name__ == "__main__":
    main()
