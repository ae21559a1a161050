"""Per-kernel duration summary of a rocprofv3 kernel trace, restricted to the
timed region of bench.py.

bench.py runs 2 counted renders (reference + SAH topology) and `warmup`
renders before the timed steps; rocprofv3 --stats averages over all of them.
This script drops the first `--skip` dispatches of every kernel name (the
untimed ones) and reports count / total / mean / min / max of the rest, so the
mean of the dominant kernel can be compared with bench.py's HIP-event
`roofline.avg_launch_ms`.

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
    per = defaultdict(list)
    for r in csv.DictReader(open(args.trace_csv)):
        per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    n_renders = None
    bench = None
    if args.json:
        for line in open(args.json):
            line = line.strip()
            if line.startswith("{"):
                bench = json.loads(line)
        if bench:
            n_renders = bench["steps"] + bench["warmup"] + args.skip_renders
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'mean_us':>10s} {'min_us':>9s} {'max_us':>9s}")
    for name, recs in sorted(per.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        recs.sort()
        skip = 0
        if n_renders and len(recs) % n_renders == 0:
            per_render = len(recs) // n_renders
            skip = per_render * (args.skip_renders + bench["warmup"])
        d = [x for _, x in recs[skip:]]
        if not d:
            continue
        print(f"{name[:70]:70s} {len(d):6d} {sum(d) / 1e6:10.3f} {sum(d) / len(d) / 1e3:10.1f} "
              f"{min(d) / 1e3:9.1f} {max(d) / 1e3:9.1f}")
    if bench:
        rf = bench["roofline"]
        print(f"bench.py HIP events: dominant kernel {rf['kernel']} avg {rf['avg_launch_ms'] * 1e3:.1f} us "
              f"over {rf['launches_per_step']} launches/step")


if __name__ == "__main__":
    main()
