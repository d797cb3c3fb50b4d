"""Per-step dispatch list from a rocprofv3 kernel trace (tools/step_trace.sh): the stretches from one
k_world start to the next, three of them from the middle of the run (steady state), each dispatch
with its duration and the idle gap before it; then the median step period, GPU-busy time and
dispatch count over every stretch of the timed run.
usage: python tools/step_trace.py <kernel_trace.csv> [anchor-kernel-substring]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_world"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(anchor)]
if len(idx) < 5:
    sys.exit(f"only {len(idx)} {anchor} dispatches")
periods, busy, counts = [], [], []
stretches = list(zip(idx[:-1], idx[1:]))
# the steady-state steps: the most common dispatch count among stretches of more than one dispatch
# (bench.py also launches the step kernel alone, back to back, and the scenario program's calls
# after the timed region: those stretches have other counts)
import collections  # noqa: E402

n_common = collections.Counter(b - a for a, b in stretches if b - a > 1).most_common(1)[0][0]
stretches = [(a, b) for a, b in stretches if b - a == n_common]
for a, b in stretches:
    periods.append((rows[b]["s"] - rows[a]["s"]) / 1e3)
    busy.append(sum(rows[k]["e"] - rows[k]["s"] for k in range(a, b)) / 1e3)
    counts.append(b - a)
mid = len(stretches) // 2
for a, b in stretches[mid - 1: mid + 2]:
    print(f"--- step: period {(rows[b]['s'] - rows[a]['s']) / 1e3:.2f} us, {b - a} dispatches")
    for k in range(a, b):
        r, p = rows[k], rows[k - 1]
        print(f"  {r['Kernel_Name'][:70]:70s} {(r['e'] - r['s']) / 1e3:7.2f} us  gap {(r['s'] - p['e']) / 1e3:6.2f}")
print(f"median over {len(periods)} steps: period {statistics.median(periods):.2f} us, busy {statistics.median(busy):.2f} us, "
      f"dispatches {statistics.median(counts)}")
