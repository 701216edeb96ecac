"""HBM traffic per launch set of each roofline entry, from two rocprofv3 PMC passes over bench.py's marker-separated
launch sequence (MI355X_MICROARCH.md, HBM section):

    python bench.py --config C2 --roofline-only --pmc-pass gpurun_out/entries_C2.json          (no profiler: names)
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dirF> -- python bench.py --config C2 --roofline-only \
        --pmc-pass gpurun_out/entries_C2.json
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dirW> -- python bench.py ... (same)
    python tools/pmc_traffic.py --entries gpurun_out/entries_C2.json <dirF> <dirW> profiles/pmc_traffic_C2.json

bench.py ``pmc_pass`` launches, per entry, one seed_bank_kernel (the marker) and then ``reps`` launch sets of the
entry; the dispatches between marker i and marker i + 1 (Dispatch_Id order) belong to entry i, summed and divided
by ``reps``. FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores. bench.py reads
bytes_per_launch[entry] into each roofline entry's ``traffic``.
"""
import csv
import glob
import json
import sys

MARKER = "seed_bank_kernel"


def dispatches(d: str, counter: str) -> list:
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return rows


def per_entry(rows: list, n_entries: int, reps: int) -> tuple[list, list]:
    """Sum of the counter over each entry's segment / reps, and the kernel names seen in it."""
    marks = [i for i, (_, name, _) in enumerate(rows) if MARKER in name]
    if len(marks) < n_entries + 1:
        raise SystemExit(f"expected >= {n_entries + 1} markers, found {len(marks)}")
    marks = marks[-(n_entries + 1):]  # the pass's markers are the last ones (warm-up launches come first)
    vals, names = [], []
    for i in range(n_entries):
        seg = rows[marks[i] + 1: marks[i + 1]]
        vals.append(sum(v for _, _, v in seg) / reps)
        names.append(sorted({n.split("(")[0][-80:] for _, n, _ in seg}))
    return vals, names


def main():
    if sys.argv[1] != "--entries":
        raise SystemExit(__doc__)
    meta = json.load(open(sys.argv[2]))
    dir_f, dir_w = sys.argv[3], sys.argv[4]
    path = sys.argv[5] if len(sys.argv) > 5 else f"profiles/pmc_traffic_{meta['config']}.json"
    ents, reps = meta["entries"], meta["reps"]
    fetch, kn = per_entry(dispatches(dir_f, "FETCH_SIZE"), len(ents), reps)
    write, _ = per_entry(dispatches(dir_w, "WRITE_SIZE"), len(ents), reps)
    out = {"config": meta["config"],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over `python bench.py "
                     f"--config {meta['config']} --roofline-only --pmc-pass`; per entry, the dispatches between its "
                     f"seed_bank_kernel markers / {reps} launch sets; bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 "
                     "(gfx950 FETCH_SIZE calibration)",
           "bytes_per_launch": {}, "raw_kib": {}}
    for e, f, w, k in zip(ents, fetch, write, kn):
        out["bytes_per_launch"][e] = round((2 * f + w) * 1024)
        out["raw_kib"][e] = {"FETCH_SIZE": round(f, 2), "WRITE_SIZE": round(w, 2), "kernels": k}
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
