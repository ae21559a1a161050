"""Per-launch HBM traffic of the bench's kernels from tools/pmc_traffic.sh output.

Counters (MI355X_MICROARCH.md § HBM): FETCH_SIZE / WRITE_SIZE are KiB from the
L2's memory-side request counters (Infinity-Cache hits included).  gfx950
correction: FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads, so
read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B/lane stores.

The profiled command is `bench.py --steps 1 --warmup 0`: two counted passes
precede the timed step.  Kernels are grouped by kind (wf_gen / wf_trace* /
wf_shade / wf_tail / wf_reduce: variants of a kind share the group) and the
LAST n launches of each kind are kept, n = that kind's launches per step in the
bench JSON line of the same run -- exactly the timed step's launches.
Writes <dir>/pmc_traffic.json: {kind: {launches, fetch_bytes, write_bytes,
traffic_bytes, kernels}} (means per launch over the timed step).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KINDS = ("wf_gen", "wf_trace", "wf_step", "wf_shade", "wf_tail", "wf_reduce")
# bench JSON launch key of each kind (wf_step: the fused gen+trace+shade kernel, timed as "trace")
LAUNCH_KEY = {"wf_step": "trace"}


def kind_of(name):
    short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    for k in KINDS:
        if short.startswith(k):
            return k, short
    return None, short


def load(dirname, counter):
    per = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(dirname, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            d = int(r["Dispatch_Id"])
            per[d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    return per, names


def bench_line(dirname, counter):
    for line in open(os.path.join(dirname, f"{counter}.log"), errors="replace"):
        if line.startswith("{"):
            try:
                bl = json.loads(line)
                bl["roofline"]["launches"]
                return bl
            except (ValueError, KeyError):
                pass
    return {}


def bench_launches(dirname, counter):
    return bench_line(dirname, counter).get("roofline", {}).get("launches", {})


def main():
    d = sys.argv[1]
    out = {}
    for counter, key, scale in (("FETCH_SIZE", "fetch_bytes", 2 * 1024.0), ("WRITE_SIZE", "write_bytes", 1024.0)):
        per, names = load(d, counter)
        launches = bench_launches(d, counter)
        byk = defaultdict(list)
        for disp in sorted(per):
            k, short = kind_of(names[disp])
            if k:
                byk[k].append((per[disp] * scale, short))
        for k, v in byk.items():
            n = launches.get(LAUNCH_KEY.get(k, k[3:]), 0) or len(v)
            keep = v[-n:]
            e = out.setdefault(k, {"launches": len(keep), "kernels": sorted({s for _, s in keep})})
            e[key] = sum(b for b, _ in keep) / max(1, len(keep))
    for k, e in out.items():
        e["traffic_bytes"] = e.get("fetch_bytes", 0) + e.get("write_bytes", 0)
    # the library build of both passes (bench.py uses no pass of another build)
    ids = {bench_line(d, c).get("build_id") for c in ("FETCH_SIZE", "WRITE_SIZE")}
    bl = bench_line(d, "FETCH_SIZE")
    sh = bl.get("config", {}).get("shard") or {}
    out["_build"] = {"build_id": ids.pop() if len(ids) == 1 else None, "config": bl.get("config", {}).get("config_id"),
                     "value": bl.get("value"), "n_shards": sh.get("n_shards", 1), "rank": sh.get("rank", 0)}
    json.dump(out, open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1, sort_keys=True)
    print(f"build {out['_build']['build_id']}")
    for k, e in sorted(((k, e) for k, e in out.items() if not k.startswith("_")), key=lambda kv: -kv[1]["traffic_bytes"]):
        print(f"{k:10s} launches/step {e['launches']:3d}  fetch {e.get('fetch_bytes', 0) / 1e9:8.3f} GB  "
              f"write {e.get('write_bytes', 0) / 1e9:8.3f} GB per launch  ({', '.join(e['kernels'])})")


if __name__ == "__main__":
    main()
