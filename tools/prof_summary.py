"""Per-step summary of a rocprofv3 --stats kernel CSV (normalised by the loss kernel's call count = steps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else None
if n is None:
    n = next(int(r["Calls"]) for r in rows if "event_kernel" in r["Name"])
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"steps={n}  GPU time/step {tot / n / 1e6:.3f} ms")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{float(r['TotalDurationNs']) / n / 1e3:8.1f}us/step {int(r['Calls']) / n:6.1f}/step "
          f"{float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")
