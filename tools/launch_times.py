"""DIAGNOSTIC: per-launch durations of the wavefront kernels (rocprofv3 kernel trace CSV), in dispatch order."""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if k.startswith("wf_"):
        rows.append((int(r["Dispatch_Id"]), k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
rows.sort()
last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
for d, k, us in rows[-last:]:
    print(f"{d:6d} {k[:28]:28s} {us:10.1f} us")
