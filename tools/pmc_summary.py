"""Per-kernel means of rocprofv3 --pmc counters (every counter_collection.csv under the given
directories) for kernels whose name contains FILTER, one block per run of consecutive dispatches
of one kernel and grid (a microbench's shapes run one after the other), plus the ratios that say
what bounds them:
  issue  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES   (share of a wave's life spent issuing)
  wait   = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (parked on s_waitcnt or a barrier)
  stall  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (ready but not issued: the MFMA pipe busy, ...)
  mfma   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 4 x CUs)  (MFMA pipe busy share of
           every SIMD's cycles; GRBM_GUI_ACTIVE sums the 8 XCDs)
  clock  = GRBM_GUI_ACTIVE / 8 / dispatch duration (MI355X_MICROARCH.md, DVFS give-back)
Passes are matched by dispatch order (the same program run once per counter set).
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
    segs = collections.OrderedDict()  # (segment index, name, grid) -> counter -> values
    for d in args:
        for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
            disp = collections.OrderedDict()
            for r in csv.DictReader(open(f)):
                if filt in r["Kernel_Name"]:
                    disp.setdefault(int(r["Dispatch_Id"]), []).append(r)
            seg, last = -1, None
            for _, rs in sorted(disp.items()):
                key = (rs[0]["Kernel_Name"].split("(")[0][:60], rs[0]["Grid_Size"])
                if key != last:
                    seg, last = seg + 1, key
                cs = segs.setdefault((seg,) + key, collections.defaultdict(list))
                for r in rs:
                    cs[r["Counter_Name"]].append(float(r["Counter_Value"]))
                cs["_ns"].append(float(rs[0]["End_Timestamp"]) - float(rs[0]["Start_Timestamp"]))
    for (seg, name, grid), cs in segs.items():
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        print(f"[{seg}] {name}  grid {grid}  ({len(cs['_ns'])} dispatches over the passes, "
              f"mean {m['_ns'] / 1e3:.1f} us)")
        for k in sorted(m):
            if k != "_ns":
                print(f"    {k:28s} {m[k]:16.1f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for lab, k in (("issue", "SQ_ACTIVE_INST_ANY"), ("wait", "SQ_WAIT_ANY"), ("stall", "SQ_WAIT_INST_ANY")):
                if k in m:
                    print(f"    {lab} share {m[k] / wc:.3f}")
        if m.get("GRBM_GUI_ACTIVE"):
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                print(f"    MFMA busy share of SIMD cycles {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 4 * cus):.3f}")
            print(f"    effective clock {m['GRBM_GUI_ACTIVE'] / 8 / m['_ns']:.2f} GHz")


if __name__ == "__main__":
    main()
