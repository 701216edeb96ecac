"""Per-grid average durations of the GEMM kernels in a rocprofv3 kernel trace: python tools/pair_shapes.py <trace.csv>"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm" in r["Kernel_Name"]:
        k = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-30:], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    print(f"{k[0]:>32} wgs={k[1]:5d} n={len(v):4d} avg={sum(v) / len(v):6.1f} us")
