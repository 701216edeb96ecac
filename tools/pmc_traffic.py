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
           "gemm_kernel<true, true>", "gemm_bwd_pair_kernel", "embed_joint_fwd_kernel<4, 1>",
           "attn_decode_kernel<float, 64>"]
# kernels launched at several shapes by bench.py: keyed "<symbol>@grid<work-items>"
BY_GRID = {"attn_decode_kernel<float, 64>"}


def averages(d: str, counter: str) -> dict:
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for s in SYMBOLS:
                if s in r["Kernel_Name"]:
                    key = f"{s}@grid{r.get('Grid_Size', '?')}" if s in BY_GRID else s
                    acc[key].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


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
