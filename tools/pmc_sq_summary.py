"""Per-kernel sums of the SQ counters collected by tools/pmc_sq.sh, with the
derived issue metrics: VALU lane utilisation = THREAD_CYCLES_VALU / (64 x
ACTIVE_INST_VALU... quad-cycle units cancel within SQ_ACTIVE_*), wait shares of
SQ_WAVE_CYCLES, and instructions per wave."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if not k.startswith("wf_"):
            continue
        print(f"== {k}")
        for n in sorted(c):
            print(f"   {n:24s} {c[n]:.4g}")
        w = c.get("SQ_WAVE_CYCLES", 0)
        if w:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                print(f"   {n + ' share':24s} {c.get(n, 0) / w:.3f}")
        if c.get("SQ_ACTIVE_INST_VALU"):
            # THREAD_CYCLES_VALU counts active lanes x cycles; ACTIVE_INST_VALU quad-cycles per wave
            print(f"   {'thread/active_valu':24s} {c.get('SQ_THREAD_CYCLES_VALU', 0) / c['SQ_ACTIVE_INST_VALU']:.2f}")
        if c.get("SQ_INSTS_VALU") and c.get("SQ_WAVES"):
            print(f"   {'valu insts/wave':24s} {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.4g}")


if __name__ == "__main__":
    main()
