"""Summarises tools/loss_sections.sh outputs on the box: event_stream_kernel mean duration and per-wave SQ counts."""
import glob
import sqlite3
import sys

sys.path.insert(0, "tools")
import pmc_db  # noqa: E402

for s in sys.argv[1:]:
    t = glob.glob(f"gpurun_out/loss_sec/t{s}/**/*.db", recursive=True)
    p = glob.glob(f"gpurun_out/loss_sec/p{s}/**/*.db", recursive=True)
    c = sqlite3.connect(t[0])
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    kd = [x for x in tabs if x.startswith("rocpd_kernel_dispatch")][0]
    ks = [x for x in tabs if x.startswith("rocpd_info_kernel_symbol")][0]
    q = (f"select s.kernel_name, avg(d.end-d.start) from {kd} d join {ks} s on d.kernel_id=s.id "
         "group by s.kernel_name")
    dur = {k: v for k, v in c.execute(q)}
    pm = pmc_db.load(p[0])
    for kn in dur:
        if "event_stream" in kn or "count_kernel" in kn or "reduce_kernel" in kn:
            v = pm.get(kn, {})
            w = v.get("SQ_WAVES", 0) or 1
            print(f"skip={s:>3} {kn.split('N_1')[1][:22]:24s} {dur[kn]/1000:7.2f} us  VALU/w {v.get('SQ_INSTS_VALU',0)/w:7.1f}"
                  f"  SALU/w {v.get('SQ_INSTS_SALU',0)/w:7.1f}  LDS/w {v.get('SQ_INSTS_LDS',0)/w:6.1f}"
                  f"  cyc/w {v.get('SQ_WAVE_CYCLES',0)/w:8.1f} wait/w {v.get('SQ_WAIT_ANY',0)/w:8.1f}")
