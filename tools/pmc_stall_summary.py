"""Per-launch stall breakdown of the bench's kernels from tools/pmc_stall.sh output.

Each group g<i>/ is one rocprofv3 --pmc pass over `bench.py --steps 1 --warmup 0`; as in
tools/pmc_summary.py the LAST n launches of each kernel kind are the timed step's (n from the bench
line in g<i>.log).  Counters of the same (kind, launch) are merged across passes.

Derived per launch (MI355X_MICROARCH.md § rocprofv3 PMC slots: SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles per wave, WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES):
  wait_any      SQ_WAIT_ANY / SQ_WAVE_CYCLES         waves parked on s_waitcnt / barrier
  wait_inst     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES    ready waves not issued (pipe / dependency)
  active        SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES  issuing
  wait_lds      SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES    (a sub-bucket of wait_inst)
  lane_util     SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)
  valu_issue2   2 x SQ_INSTS_VALU / (1024 SIMDs x per-XCD GRBM_GUI_ACTIVE): the fraction of SIMD
                cycles issuing VALU at the measured 2-cycle wave64 rate (profiles/r4_valu_peak/)
  lds_conflict  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  dual_issue    SQ_ACTIVE_INST_VALU2 / SQ_ACTIVE_INST_VALU: VALU quad-cycles with two instructions issued
  share_*       SQ_INSTS_VALU_<class> / SQ_INSTS_VALU
Writes <dir>/pmc_stall.json {kind: [per-launch dicts]}.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import LAUNCH_KEY, kind_of  # noqa: E402


def group(dirname, log):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            disp = int(r["Dispatch_Id"])
            per[disp][r["Counter_Name"]] += float(r["Counter_Value"])
            names[disp] = r["Kernel_Name"]
    launches = {}
    if os.path.exists(log):
        for line in open(log, errors="replace"):
            if line.startswith("{"):
                try:
                    launches = json.loads(line)["roofline"]["launches"]
                except (ValueError, KeyError):
                    pass
    byk = defaultdict(list)
    for disp in sorted(per):
        k, short = kind_of(names[disp])
        if k:
            byk[k].append((dict(per[disp]), short))
    out = {}
    for k, v in byk.items():
        n = launches.get(LAUNCH_KEY.get(k, k[3:]), 0) or len(v)
        out[k] = v[-n:]
    return out


def derive(c):
    w = c.get("SQ_WAVE_CYCLES")
    e = {}
    if w:
        for key, n in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                       ("active", "SQ_ACTIVE_INST_ANY"), ("wait_lds", "SQ_WAIT_INST_LDS"),
                       ("active_valu", "SQ_ACTIVE_INST_VALU"), ("active_lds", "SQ_ACTIVE_INST_LDS"),
                       ("active_sca", "SQ_ACTIVE_INST_SCA"), ("active_vmem", "SQ_ACTIVE_INST_VMEM"),
                       ("active_flat", "SQ_ACTIVE_INST_FLAT"), ("active_misc", "SQ_ACTIVE_INST_MISC")):
            if n in c:
                e[key] = c[n] / w
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_ACTIVE_INST_VALU2" in c:
        e["dual_issue"] = c["SQ_ACTIVE_INST_VALU2"] / c["SQ_ACTIVE_INST_VALU"]
    if c.get("SQ_INSTS_VALU"):
        for n in ("SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_INT32",
                  "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_CVT"):
            if n in c:
                e["share_" + n[len("SQ_INSTS_VALU_"):].lower()] = c[n] / c["SQ_INSTS_VALU"]
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        e["lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if c.get("GRBM_GUI_ACTIVE") and "SQ_INSTS_VALU" in c:
        e["valu_issue2"] = 2.0 * c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0)
    if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
        e["lds_conflict"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
    if hit is not None and miss is not None and hit + miss > 0:
        e["l2_hit"] = hit / (hit + miss)
    for n in ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TA_FLAT_READ_WAVEFRONTS_sum", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_VMEM_WR", "TA_BUSY_avr"):
        if n in c:
            e[n.lower().replace("_sum", "").replace("_avr", "")] = c[n]
    if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") and "TCP_TCC_READ_REQ_sum" in c:
        e["l1_miss_to_l2"] = c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if c.get("SQ_WAVES"):
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM",
                  "SQ_INSTS_BRANCH"):
            if n in c:
                e[n.lower().replace("sq_", "") + "_per_wave"] = c[n] / c["SQ_WAVES"]
    return e


def main():
    d = sys.argv[1]
    merged = defaultdict(lambda: defaultdict(dict))
    kernels = defaultdict(set)
    for g in sorted(glob.glob(os.path.join(d, "g*"))):
        if not os.path.isdir(g):
            continue
        for k, lst in group(g, g + ".log").items():
            for j, (c, short) in enumerate(lst):
                merged[k][j].update(c)
                kernels[k].add(short)
    out = {}
    for k in sorted(merged):
        rows = []
        print(f"== {k} ({', '.join(sorted(kernels[k]))})")
        for j in sorted(merged[k]):
            c = merged[k][j]
            e = derive(c)
            rows.append({"launch": j, "counters": c, "derived": e})
            print(f"  launch {j}: " + "  ".join(f"{n} {v:.3f}" if abs(v) < 1e4 else f"{n} {v:.4g}"
                                                for n, v in e.items()))
        tot = defaultdict(float)
        for r in rows:
            for n, v in r["counters"].items():
                tot[n] += v
        e = derive(tot)
        print("  all:      " + "  ".join(f"{n} {v:.3f}" if abs(v) < 1e4 else f"{n} {v:.4g}" for n, v in e.items()))
        out[k] = {"kernels": sorted(kernels[k]), "launches": rows, "total": {"counters": dict(tot), "derived": e}}
    # the build and workload the passes ran (bench.py's line in each group's log): every group must agree
    builds = set()
    for g in sorted(glob.glob(os.path.join(d, "g*.log"))):
        for line in open(g, errors="replace"):
            if line.startswith("{"):
                try:
                    x = json.loads(line)
                    builds.add((x["roofline"]["valu"]["build_id"], x["config"]["config_id"]))
                except (ValueError, KeyError):
                    pass
    out["_build"] = {"build_id": sorted(b for b, _ in builds), "workload": sorted(w for _, w in builds),
                     "consistent": len(builds) == 1}
    print("build", out["_build"])
    json.dump(out, open(os.path.join(d, "pmc_stall.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
