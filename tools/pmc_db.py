"""Per-kernel PMC counter means from rocprofv3 SQLite outputs (run_results.db): python tools/pmc_db.py db [db ...]
Counters summed over the chip per dispatch, averaged over dispatches; SQ_* also per wave (÷ SQ_WAVES of a pass that
has it)."""
import collections
import sqlite3
import sys


def load(path):
    c = sqlite3.connect(path)
    names = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    q = ("select s.kernel_name, d.event_id, p.pmc_id, p.value from rocpd_pmc_event p "
         "join rocpd_kernel_dispatch d on p.event_id = d.event_id "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for kn, ev, pid, val in c.execute(q):
        per[kn][ev][names[pid]] += val
    out = {}
    for kn, evs in per.items():
        tot = collections.defaultdict(float)
        for ev, vals in evs.items():
            for k, v in vals.items():
                tot[k] += v
        out[kn] = {k: v / len(evs) for k, v in tot.items()}
    return out


if __name__ == "__main__":
    merged = collections.defaultdict(dict)
    for p in sys.argv[1:]:
        for kn, vals in load(p).items():
            merged[kn].update(vals)
    for kn, vals in merged.items():
        print(kn[:100])
        waves = vals.get("SQ_WAVES")
        for k in sorted(vals):
            extra = f"   per wave {vals[k] / waves:10.1f}" if waves and k.startswith("SQ_") and k != "SQ_WAVES" else ""
            print(f"  {k:28s} {vals[k]:16.1f}{extra}")
