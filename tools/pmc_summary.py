"""Per-launch HBM traffic of the bench's kernels from tools/pmc_traffic.sh output.

Counters (MI355X_MICROARCH.md § HBM): FETCH_SIZE / WRITE_SIZE are KiB from the
L2's memory-side request counters (Infinity-Cache hits included).  gfx950
correction: FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads, so
read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B/lane stores.
The untimed renders of bench.py (2 counted passes, no warmup) are dropped.
Writes <dir>/pmc_traffic.json: {kernel: {launches, fetch_bytes, write_bytes, traffic_bytes}} (means per launch).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirname, counter):
    files = glob.glob(os.path.join(dirname, counter, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(float)
    names = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            d = int(r["Dispatch_Id"])
            per[d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    return per, names


def main():
    d = sys.argv[1]
    skip_renders = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    fetch, names = load(d, "FETCH_SIZE")
    write, names_w = load(d, "WRITE_SIZE")
    out = {}
    for per, key, scale in ((fetch, "fetch_bytes", 2 * 1024.0), (write, "write_bytes", 1024.0)):
        nm = names if per is fetch else names_w
        byk = defaultdict(list)
        for disp in sorted(per):
            byk[nm[disp]].append(per[disp] * scale)
        for k, v in byk.items():
            short = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            # bench: renders = 2 counted + timed steps (steps=1, warmup=0); keep the last 1/(skip+1)
            keep = v[len(v) * skip_renders // (skip_renders + 1):] if len(v) % (skip_renders + 1) == 0 else v
            e = out.setdefault(short, {"launches": len(keep)})
            e[key] = sum(keep) / max(1, len(keep))
    for k, e in out.items():
        e["traffic_bytes"] = e.get("fetch_bytes", 0) + e.get("write_bytes", 0)
    json.dump(out, open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1, sort_keys=True)
    for k, e in sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes"]):
        print(f"{k[:40]:40s} launches {e['launches']:4d}  fetch {e.get('fetch_bytes', 0) / 1e9:9.3f} GB  "
              f"write {e.get('write_bytes', 0) / 1e9:9.3f} GB per launch")


if __name__ == "__main__":
    main()
