"""HBM traffic per launch of the roofline kernels from two rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section):

    rocprofv3 --pmc FETCH_SIZE -d <dirF> ... -- python bench.py --roofline-only
    rocprofv3 --pmc WRITE_SIZE -d <dirW> ... -- python bench.py --roofline-only
    python tools/pmc_traffic.py <dirF> <dirW> [out.json]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores. Averages over every dispatch of a
kernel symbol; bench.py reads bytes_per_launch[symbol] into roofline.traffic.
"""
import csv
import glob
import json
import sys
from collections import defaultdict

SYMBOLS = ["attn_fwd_mfma_kernel<64, true>", "attn_fwd_mfma_kernel<64, false>", "attn_bwd_kernel<64, true>",
           "gemm_kernel<true, true, 3, 1, 1>", "gemm_bwd_pair_kernel", "embed_joint_fwd_kernel<4, 1>",
           "attn_decode_kernel<float, 64>"]
# kernels launched at several shapes by bench.py: keyed "<symbol>@grid<work-items>"
BY_GRID = {"attn_decode_kernel<float, 64>"}
# the C5 embedding microbench runs the JOINT kernel on a grid far larger than C2's: its dispatches are keyed "@c5"
C5_GRID_MIN = 4 << 20
# multi-kernel launch sets: bytes per set = the sum over the member kernels' dispatches / the anchor's dispatches
GROUPS = {
    "embed_bag_bwd": (["bag_block_sort_kernel", "bag_col_prefix_kernel", "bag_row_scan_kernel", "bag_scatter_kernel",
                       "bag_reduce_kernel", "bag_combine_kernel", "bag_subject_part_kernel", "bag_subject_sum_kernel"],
                      "bag_block_sort_kernel"),
    "output_loss": (["::count_kernel(", "::event_lds_kernel<", "::event_kernel<", "::reduce_kernel(float const*"],
                    "::count_kernel("),
}


def averages(d: str, counter: str) -> dict:
    acc = defaultdict(list)
    group_sum = defaultdict(float)
    group_n = defaultdict(int)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name, val = r["Kernel_Name"], float(r["Counter_Value"])
            grid = int(r.get("Grid_Size", 0) or 0)
            for s in SYMBOLS:
                if s in name:
                    if s in BY_GRID:
                        key = f"{s}@grid{r.get('Grid_Size', '?')}"
                    elif s.startswith("embed_joint_fwd_kernel") and grid >= C5_GRID_MIN:
                        key = "embed_joint_fwd_kernel@c5"
                    else:
                        key = s
                    acc[key].append(val)
            for g, (members, anchor) in GROUPS.items():
                if any(m in name for m in members):
                    group_sum[g] += val
                if anchor in name:
                    group_n[g] += 1
    out = {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}
    for g in group_sum:
        if group_n[g]:
            out[g] = (group_sum[g] / group_n[g], group_n[g])
    return out


def main():
    fetch, write = averages(sys.argv[1], "FETCH_SIZE"), averages(sys.argv[2], "WRITE_SIZE")
    out = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "`python bench.py --roofline-only`; bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per dispatch "
                     "(gfx950 FETCH_SIZE calibration)",
           "bytes_per_launch": {}, "raw_kib": {}}
    for s in sorted(set(fetch) | set(write)):
        if s in fetch and s in write:
            out["bytes_per_launch"][s] = round((2 * fetch[s][0] + write[s][0]) * 1024)
            out["raw_kib"][s] = {"FETCH_SIZE": fetch[s][0], "WRITE_SIZE": write[s][0], "dispatches": fetch[s][1]}
    path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
