"""Timeline of the last replayed step in a rocprofv3 kernel trace: per kernel start / end relative to the step's
first kernel, queue id, and the step's span; with --summary only the span and per-queue busy time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step ends with the adamw launch; take the span between the last two adamw launches
ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
a, b = ad[-2] + 1, ad[-1] + 1
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
print(f"kernels {len(step)} span {(t1 - t0) / 1000:.1f} us")
busy = {}
for r in step:
    q = r["Queue_Id"]
    busy[q] = busy.get(q, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print("busy per queue (us):", {q: round(v / 1000, 1) for q, v in busy.items()})
if "--summary" not in sys.argv:
    for r in step:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1000:8.1f} {e / 1000:8.1f} {(e - s) / 1000:6.1f} q{r['Queue_Id']} g{r['Grid_Size_X']:>7} "
              f"{r['Kernel_Name'][:70]}")
