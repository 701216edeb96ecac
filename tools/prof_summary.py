"""Per-step summary of a rocprofv3 --stats kernel CSV: python tools/prof_summary.py <kernel_stats.csv> [steps] [top]
(steps defaults to the call count of the loss reduce kernel = one per step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else None
if n is None:
    n = next(int(r["Calls"]) for r in rows if "reduce_kernel" in r["Name"])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"steps={n}  GPU time/step {tot / n / 1e3:.1f} us  kernels/step {calls / n:.1f}")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / n / 1e3:8.1f}us/step {int(r['Calls']) / n:6.1f}/step "
          f"{float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:90]}")
