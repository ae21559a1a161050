"""Per-launch durations (us) of one kernel name prefix from a rocprofv3 kernel trace CSV,
in dispatch order, grouped `per` launches to a line: python tools/launch_durations.py trace.csv wf_step_clds 9"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
per = int(sys.argv[3]) if len(sys.argv) > 3 else len(d)
for k in range(0, len(d), per):
    print(" ".join(f"{x:8.1f}" for x in d[k:k + per]))
