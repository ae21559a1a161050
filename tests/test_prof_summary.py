"""tools/prof_summary.py finds bench.py's timed region in a rocprofv3 kernel trace and averages the dominant
kernel over all of its instantiations (round 6: iteration 0 and the later iterations of the fused step are two),
as bench.py's HIP events do -- the agreement test_bench_contract checks on the committed summary."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IT0 = "void (anonymous namespace)::wf_step_clds2<0u, 768u, 0, 1>(rtw_launch, rtw_wf, unsigned int)"
ITN = "void (anonymous namespace)::wf_step_clds2<0u, 768u, 0, 0>(rtw_launch, rtw_wf, unsigned int)"
CNT = "void (anonymous namespace)::wf_step_clds2<0u, 768u, 1, 2>(rtw_launch, rtw_wf, unsigned int)"
TAIL = "void (anonymous namespace)::wf_tail_clds2<0u, 768u, 0>(rtw_launch, rtw_wf, unsigned int)"
RED = "(anonymous namespace)::wf_reduce(rtw_launch, rtw_wf)"


def write_trace(path):
    """a counted render (other instantiations, slower) then two product renders: it0 12 us, its 1-3 8 us"""
    rows, t = [], 0
    def k(name, d):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + d})
        t += d + 100
    for _ in range(4):
        k(CNT, 30000)
    k(TAIL, 20000)
    k(RED, 1000)
    for _ in range(2):
        k(IT0, 12000)
        for _ in range(3):
            k(ITN, 8000)
        k(TAIL, 13000)
        k(RED, 1000)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def run(tmp_path, roofline):
    write_trace(tmp_path / "trace.csv")
    (tmp_path / "bench.json").write_text(json.dumps({"steps": 2, "roofline": roofline}) + "\n")
    rc = subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_summary.py"), str(tmp_path / "trace.csv"),
                         "--json", str(tmp_path / "bench.json")], capture_output=True, text=True)
    assert rc.returncode == 0, rc.stderr
    return rc.stdout


def test_family_mean_over_the_timed_region(tmp_path):
    out = run(tmp_path, {"kernel": "wf_step_clds2<0u, 768u, 0, 0> + wf_step_clds2<0u, 768u, 0, 1>",
                         "kernels": ["wf_step_clds2<0u, 768u, 0, 0>", "wf_step_clds2<0u, 768u, 0, 1>"],
                         "launches_per_step": 4.0, "avg_launch_ms": 9.0})
    assert "timed region not found" not in out
    fam = [ln for ln in out.splitlines() if ln.startswith("dominant family in the timed region:")]
    assert fam and "8 calls, mean 9.0 us" in fam[0], out  # (12 + 3 x 8) / 4 us; the counted render excluded
    # the counted pass's instantiation and the first render's tail are outside the timed region
    assert "wf_step_clds2<0u, 768u, 1, 2>" not in out
    tail = [ln for ln in out.splitlines() if "wf_tail_clds2" in ln]
    assert tail and tail[0].split()[-5] == "2", tail


def test_one_instantiation_line_still_found(tmp_path):
    """a round-5 line names one instantiation (no `kernels`): its calls alone define the region"""
    out = run(tmp_path, {"kernel": "wf_step_clds2<0u, 768u, 0, 0>", "launches_per_step": 3.0,
                         "avg_launch_ms": 8.0})
    assert "timed region not found" not in out
    assert "6 calls, mean 8.0 us" in out
