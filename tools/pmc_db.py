"""Per-kernel averages of the PMC counters in a rocprofv3 rocpd .db (python tools/pmc_db.py DB [filter])."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
q = """select s.kernel_name, p.name, e.value, d.end - d.start, d.id
       from rocpd_pmc_event e join rocpd_info_pmc p on e.pmc_id = p.id
       join rocpd_kernel_dispatch d on d.event_id = e.event_id
       join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for k, name, v, dt, did in c.execute(q):
    if flt and flt not in k:
        continue
    acc[k][name].append(v)
    dur[k][did] = dt
for k in sorted(acc, key=lambda k: -sum(dur[k].values())):
    n = len(dur[k])
    print(f"{k[:90]}  dispatches {n}  avg {sum(dur[k].values()) / n / 1e3:.2f} us")
    for name, vs in sorted(acc[k].items()):
        print(f"    {name:24s} {sum(vs) / n:14.1f}")
