"""Print the tail of a rocprofv3 kernel trace with per-dispatch durations and inter-kernel gaps,
plus the per-kernel summary. Usage: python tools/trace_gaps.py gpurun_out/prof [N]"""
import csv
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
r = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
r = [x for x in r if "copyBuffer" not in x["Kernel_Name"]]
prev = None
for x in r[-n:]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{x['Kernel_Name'][:44]:44s} dur={(e - s) / 1e3:8.2f} gap={gap:7.2f} "
          f"grid={x['Grid_Size_X']}x{x['Grid_Size_Y']} wg={x['Workgroup_Size_X']} "
          f"lds={x['LDS_Block_Size']} vgpr={x['VGPR_Count']}")
    prev = e
print()
for x in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
    print(f"{x['Name'][:56]:56s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e3:9.2f} us")
