"""Per-launch VALU issue counters of the bench's kernels from tools/pmc_valu.sh output.

The profiled command is `bench.py --steps 1 --warmup 0`; as in tools/pmc_summary.py
the LAST n launches of each kernel kind are kept (n = that kind's launches per step
in the bench line of the same run), i.e. the timed step's launches, and averaged.

Per launch (sums over the launch's waves, rocprofv3 units):
  insts_valu          SQ_INSTS_VALU          wave-instructions issued to the VALU
  active_inst_valu    SQ_ACTIVE_INST_VALU    VALU-busy quad-cycles
  thread_cycles_valu  SQ_THREAD_CYCLES_VALU  active lanes x VALU quad-cycles
  wave_cycles         SQ_WAVE_CYCLES         resident-wave quad-cycles
  gui_active          GRBM_GUI_ACTIVE        GPU-busy clocks of the launch
Derived (unit-free ratios of counters of the same launch):
  lane_util = thread_cycles_valu / (64 * active_inst_valu)   useful lanes per VALU cycle
  lane_ops  = insts_valu * 64 * lane_util                    useful lane-instructions
Writes <dir>/pmc_valu.json {kind: {...}}; bench.py reads the copy in profiles/.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import LAUNCH_KEY, kind_of  # noqa: E402

FIELDS = {"SQ_INSTS_VALU": "insts_valu", "SQ_ACTIVE_INST_VALU": "active_inst_valu",
          "SQ_THREAD_CYCLES_VALU": "thread_cycles_valu", "SQ_WAVE_CYCLES": "wave_cycles", "SQ_WAVES": "waves",
          "SQ_BUSY_CYCLES": "sq_busy_cycles", "GRBM_GUI_ACTIVE": "gui_active", "GRBM_COUNT": "grbm_count"}


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(float))
    names, dur = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            c = r.get("Counter_Name")
            if c in FIELDS:
                disp = int(r["Dispatch_Id"])
                per[disp][FIELDS[c]] += float(r["Counter_Value"])
                names[disp] = r["Kernel_Name"]
    launches, build = {}, None
    for line in open(os.path.join(d, "valu.log"), errors="replace"):
        if line.startswith("{"):
            try:
                bl = json.loads(line)
                launches = bl["roofline"]["launches"]
                sh = bl["config"].get("shard") or {}
                build = {"build_id": bl.get("build_id"), "config": bl["config"].get("config_id"),
                         "value": bl.get("value"), "n_shards": sh.get("n_shards", 1), "rank": sh.get("rank", 0)}
            except (ValueError, KeyError):
                pass
    byk = defaultdict(list)
    for disp in sorted(per):
        k, short = kind_of(names[disp])
        if k:
            byk[k].append((per[disp], short))
    out = {}
    for k, v in byk.items():
        n = launches.get(LAUNCH_KEY.get(k, k[3:]), 0) or len(v)
        keep = v[-n:]
        e = {"launches": len(keep), "kernels": sorted({s for _, s in keep})}
        for f in FIELDS.values():
            e[f] = sum(c.get(f, 0.0) for c, _ in keep) / max(1, len(keep))
        if e["active_inst_valu"] > 0:
            e["lane_util"] = e["thread_cycles_valu"] / (64.0 * e["active_inst_valu"])
            e["lane_ops"] = e["insts_valu"] * 64.0 * e["lane_util"]
        # every launch of the timed step in launch order (the fused step: one per wavefront iteration)
        e["per_launch"] = [{"insts_valu": c.get("insts_valu", 0.0), "gui_active": c.get("gui_active", 0.0),
                            "lane_util": (c.get("thread_cycles_valu", 0.0) / (64.0 * c["active_inst_valu"])
                                          if c.get("active_inst_valu") else None),
                            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD clocks x 1024 SIMDs;
                            # one wave64 VALU instruction per SIMD per 2 clocks (profiles/r4_valu_peak/)
                            "valu_busy": (c.get("insts_valu", 0.0) * 2.0 / (1024.0 * c["gui_active"] / 8.0)
                                          if c.get("gui_active") else None)} for c, _ in keep]
        out[k] = e
    # the library build the pass was taken on (bench.py uses no pass of another build)
    out["_build"] = build or {"build_id": None}
    json.dump(out, open(os.path.join(d, "pmc_valu.json"), "w"), indent=1, sort_keys=True)
    print(f"build {out['_build'].get('build_id')}")
    for k, e in sorted(((k, e) for k, e in out.items() if not k.startswith("_")), key=lambda kv: -kv[1]["insts_valu"]):
        print(f"{k:10s} launches/step {e['launches']:3d}  VALU insts {e['insts_valu']:.4g}  "
              f"lane_util {e.get('lane_util', 0):.3f}  lane-ops {e.get('lane_ops', 0):.4g}  "
              f"GUI_ACTIVE {e['gui_active']:.4g}  ({', '.join(e['kernels'])})")
        if e["launches"] > 1:
            for j, pl in enumerate(e["per_launch"]):
                lu = pl["lane_util"]
                vb = pl["valu_busy"]
                print(f"    launch {j}: VALU insts {pl['insts_valu']:.4g}  lane_util "
                      f"{lu if lu is None else round(lu, 3)}  VALU issue busy (x2 / 1024 SIMD / per-XCD GUI_ACTIVE) "
                      f"{vb if vb is None else round(vb, 3)}  GUI_ACTIVE {pl['gui_active']:.4g}")


if __name__ == "__main__":
    main()
