"""Per-step kernel breakdown from a rocprofv3 --kernel-trace --stats CSV directory (one adamw launch per step).

    python tools/prof_step.py gpurun_out/step_prof2 [--trace]
"""
import csv
import os
import sys


def main(d, trace=False):
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    step = rows[a + 1: b + 1]
    agg = {}
    for r in step:
        d_us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = r["Kernel_Name"][:100]
        t, c = agg.get(n, (0.0, 0))
        agg[n] = (t + d_us, c + 1)
        if trace:
            print(f"{d_us:7.2f} grid={r['Grid_Size_X']:>8} wg={r['Workgroup_Size_X']:>5} {n}")
    tot = sum(t for t, _ in agg.values())
    span = (int(step[-1]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{t:8.1f} us  {c:3d}x  {t / c:7.2f}  {n}")
    print(f"kernel sum {tot:.1f} us; step span {span:.1f} us; launches {len(step)}")


if __name__ == "__main__":
    main(sys.argv[1], "--trace" in sys.argv)
