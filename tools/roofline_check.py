"""Recompute the roofline fractions of a committed bench line from profiles/.

  python tools/roofline_check.py profiles/r2_c2_bench.json

VALU (the bound): lane-instructions per launch of the dominant kernel
(profiles/pmc_valu_<config>_<bvh>.json, tools/pmc_valu.sh) / the bench's HIP-event
average launch time / the measured VALU issue peak (bench.py VALU_PEAK_TLOPS: one wave64 instruction
per SIMD per 2 clocks, profiles/r4_valu_peak/).
HBM: PMC traffic per launch (profiles/pmc_traffic_<config>_<bvh>.json,
tools/pmc_traffic.sh) / the same launch time / 8 TB/s.
Prints both and exits non-zero if the line's numbers disagree with the
recomputation by more than 0.5 % or any fraction exceeds 1.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def bench_line(path):
    with open(path) as f:
        return json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])


def recompute(line):
    import bench
    r = line["roofline"]
    launch_s = r["avg_launch_ms"] / 1e3
    out = {}
    src = r["valu"]["source"]
    if src:
        e = json.load(open(os.path.join(REPO, src)))[r["valu"]["kind"]]
        # the peak the line was computed against: rounds 1-3 assumed 4 clocks per wave64 VALU instruction
        # (39.3 T, issue busy from SQ_ACTIVE_INST_VALU); from round 4 the measured 2 clocks (78.6 T,
        # profiles/r4_valu_peak/), issue busy from SQ_INSTS_VALU
        cyc = bench.N_SIMD * 64 * bench.CLOCK_HZ / (r["peak"] * 1e12)
        out["valu_frac"] = e["lane_ops"] / launch_s / 1e12 / r["peak"]
        out["valu_lane_util"] = e["thread_cycles_valu"] / (64 * e["active_inst_valu"])
        insts = e["active_inst_valu"] if round(cyc) == 4 else e["insts_valu"]
        out["valu_issue_busy"] = insts * round(cyc) / (bench.N_SIMD * launch_s * bench.CLOCK_HZ)
    hsrc = r["hbm"]["source"]
    if hsrc:
        t = json.load(open(os.path.join(REPO, hsrc)))[r["hbm"]["kind"]]["traffic_bytes"]
        out["hbm_frac"] = t / launch_s / 1e9 / bench.HBM_PEAK_GBS
    wk = r.get("walk") or {}
    if wk.get("source") and wk.get("frac") is not None:  # the walk roofline (round 5)
        c = json.load(open(os.path.join(REPO, wk["source"])))
        assert c["build_id"] == line["build_id"], "walk ceiling of another build"
        out["walk_frac"] = wk["device_steps_per_render"] / (wk["render_ms"] / 1e3) / c["ceiling"]
    return out


def main():
    line = bench_line(sys.argv[1])
    r = line["roofline"]
    got = recompute(line)
    ok = True
    pairs = (("valu_frac", r["frac"]), ("hbm_frac", r["hbm"]["frac"]), ("valu_lane_util", r["valu"]["lane_util"]),
             ("valu_issue_busy", r["valu"]["issue_busy"]), ("walk_frac", (r.get("walk") or {}).get("frac")))
    for k, v in pairs:
        if k not in got:
            continue
        good = v is not None and abs(got[k] - v) <= 5e-3 * max(abs(v), 1e-9) + 1e-4
        ok &= good
        print(f"{k:16s} line {v}  recomputed {got[k]:.4f}  {'ok' if good else 'MISMATCH'}")
    for k in ("valu_frac", "hbm_frac", "walk_frac"):
        if k in got and not got[k] <= 1.0:
            print(f"{k} > 1")
            ok = False
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
