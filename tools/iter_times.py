#!/usr/bin/env python3
"""Per-wavefront-iteration kernel times from a rocprofv3 kernel trace of one render (tools/render_once.py).

Every batch launches wf_gen (split path) or the first wf_step (fused path), then one trace+shade pair (or
one fused step) per iteration, the tail and the reduce.  The i-th launch of a kernel name after the
batch's first launch is iteration i; the script sums each iteration's time over the batches and prints
one JSON line: {kernel: [ms of iteration 0, 1, ...], ...} plus the totals.
Usage: python tools/iter_times.py gpurun_out/it/x_kernel_trace.csv [label]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?(\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                  for r in csv.DictReader(open(sys.argv[1])))
    per_iter = defaultdict(lambda: defaultdict(float))
    totals = defaultdict(float)
    count = defaultdict(int)
    for s, e, k in rows:
        if k in ("wf_gen", "wf_tile_lists", "wf_tile_lists_walk", "wf_reduce"):
            if k in ("wf_gen", "wf_reduce"):
                count.clear()  # a batch boundary
        ms = (e - s) / 1e6
        totals[k] += ms
        if k.startswith(("wf_trace", "wf_shade", "wf_step")):
            per_iter[k][count[k]] += ms
            count[k] += 1
    out = {"label": sys.argv[2] if len(sys.argv) > 2 else "",
           "per_iteration_ms": {k: [round(v[i], 3) for i in sorted(v)] for k, v in per_iter.items()},
           "total_ms": {k: round(v, 3) for k, v in sorted(totals.items(), key=lambda kv: -kv[1])}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
