"""Per-kernel duration summary of a rocprofv3 kernel trace, restricted to the
timed region of bench.py.

bench.py runs counted renders (reference + SAH topology, which may use other
kernel instantiations) and `warmup` renders before the timed steps; rocprofv3
--stats averages over all of them.  With the bench line (--json), this script
keeps the timed region only: the last steps x launches_per_step calls of the
dominant kernel and every call from the end of the render before them, and
reports count / total / mean / min / max per kernel, so the mean of the
dominant kernel can be compared with bench.py's HIP-event `roofline.avg_launch_ms`.

Usage: python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --skip-renders 2 [--json bench.json]
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_csv")
    ap.add_argument("--skip-renders", type=int, default=2, help="untimed renders before the timed steps")
    ap.add_argument("--json", help="bench JSON line (file) to compare against")
    args = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(args.trace_csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    bench = None
    if args.json:
        for line in open(args.json):
            line = line.strip()
            if line.startswith("{"):
                bench = json.loads(line)
    t0 = None
    if bench:
        # the timed region: the last steps x launches_per_step calls of the dominant kernel, back to the end of the
        # render before them (the wf_reduce preceding the first of those calls).  The untimed renders before it
        # (counted passes, warm-up) may run other instantiations, so counting calls per name is not enough.
        rf = bench["roofline"]
        n_dom = int(round(bench["steps"] * rf["launches_per_step"]))
        dom = [i for i, (_, _, n) in enumerate(rows) if is_dominant(n, rf)]
        if len(dom) >= n_dom > 0:
            first = dom[-n_dom]
            j = first
            while j > 0 and "wf_reduce" not in rows[j - 1][2]:
                j -= 1
            t0 = rows[j][0]
    per = defaultdict(list)
    for t, d, n in rows:
        if t0 is None or t >= t0:
            per[n].append(d)
    if t0 is None and bench:
        print("(timed region not found: every call)")
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'mean_us':>10s} {'min_us':>9s} {'max_us':>9s}")
    for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:70]:70s} {len(d):6d} {sum(d) / 1e6:10.3f} {sum(d) / len(d) / 1e3:10.1f} "
              f"{min(d) / 1e3:9.1f} {max(d) / 1e3:9.1f}")
    if bench:
        rf = bench["roofline"]
        fam = [d for n, ds in per.items() if is_dominant(n, rf) for d in ds]
        if fam and t0 is not None:
            print(f"dominant family in the timed region: {len(fam)} calls, mean {sum(fam) / len(fam) / 1e3:.1f} us "
                  f"({rf['kernel']})")
        print(f"bench.py HIP events: dominant kernel {rf['kernel']} avg {rf['avg_launch_ms'] * 1e3:.1f} us "
              f"over {rf['launches_per_step']} launches/step")


def is_dominant(name, rf):
    """One of the dominant kernel's instantiations (bench.py's roofline.kernels; a round-5 line names one)."""
    base = name.split("(")[0]
    return any(base.endswith(k) or k in name for k in rf.get("kernels") or [rf["kernel"]])


if __name__ == "__main__":
    main()
