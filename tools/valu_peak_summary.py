"""Summary of tools/valu_peak.sh: the VALU issue ceiling of gfx950 per (instruction, waves/SIMD).

Inputs: <dir>/plain.jsonl (diag/valu_peak's own HIP-event timing, one line per case) and
<dir>/pmc/**/*counter_collection.csv + *kernel_trace.csv (one rocprofv3 --pmc pass over the same
binary).  The binary launches every case 4 times (one warm-up + 3 timed) in case order, so
dispatch 4k+3 is case k's last timed launch.

Per case (the last launch):
  cyc/inst (events)  SIMD cycles per wave-instruction at the nominal 2.4 GHz from the HIP events
  clock              GRBM_GUI_ACTIVE / 8 XCDs / kernel-trace duration (the clock held under load)
  cyc/inst (clock)   the same at that measured clock
  active/insts       SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU
  busy4              4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x per-XCD GUI_ACTIVE): bench.py's old
                     'issue busy' (1.0 = one instruction per SIMD per 4 clocks)
  dual               SQ_ACTIVE_INST_VALU2 / SQ_ACTIVE_INST_VALU: quad-cycles in which the SIMD issued
                     two VALU instructions (dual issue) per VALU quad-cycle
Writes <dir>/valu_peak.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    plain = [json.loads(line) for line in open(os.path.join(d, "plain.jsonl")) if line.startswith("{")]
    ctr = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ctr[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(d, "pmc", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    disp = sorted(ctr)
    out = []
    print(f"{'case':24s} {'w/SIMD':>6s} {'Tlane-op/s':>10s} {'cyc/inst@2.4':>12s} {'clock GHz':>9s} "
          f"{'cyc/inst@clk':>12s} {'active/insts':>12s} {'busy4':>6s} {'dual':>6s}")
    for k, c in enumerate(plain):
        e = dict(c)
        if "tlane_ops_per_s" not in c:  # LDS-latency / placement lines: reported as measured
            out.append(e)
            print(json.dumps(c))
            continue
        j = 4 * k + 3
        if j < len(disp):
            p = ctr[disp[j]]
            t = dur.get(disp[j])
            gui = p.get("GRBM_GUI_ACTIVE", 0.0)
            insts = p.get("SQ_INSTS_VALU", 0.0)
            act = p.get("SQ_ACTIVE_INST_VALU", 0.0)
            e["pmc"] = dict(p)
            e["pmc_kernel_s"] = t
            if t and gui:
                clk = gui / 8.0 / t
                e["clock_ghz"] = clk / 1e9
                e["simd_cycles_per_wave_inst_at_clock"] = (gui / 8.0) * 1024 / insts if insts else None
                e["busy4"] = 4.0 * act / (1024 * gui / 8.0)
            e["active_over_insts"] = act / insts if insts else None
            e["dual_issue_frac"] = p.get("SQ_ACTIVE_INST_VALU2", 0.0) / act if act else None
            e["insts_valu_expected"] = c["wave_insts"]
        out.append(e)
        print(f"{e['case']:24s} {e['waves_per_simd']:6d} {e['tlane_ops_per_s']:10.3f} "
              f"{e['simd_cycles_per_wave_inst_at_2p4GHz']:12.3f} {e.get('clock_ghz', 0):9.3f} "
              f"{e.get('simd_cycles_per_wave_inst_at_clock') or 0:12.3f} {e.get('active_over_insts') or 0:12.3f} "
              f"{e.get('busy4', 0):6.3f} {e.get('dual_issue_frac') or 0:6.3f}")
    json.dump(out, open(os.path.join(d, "valu_peak.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
