"""Summarise a rocprofv3 kernel_stats.csv: name, calls, average us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    per = f" {int(r['Calls']) / steps:6.2f}/step" if steps else ""
    print(f"{r['Name'][:80]:80s} {r['Calls']:>6}{per} {float(r['AverageNs']) / 1e3:8.2f}us {float(r['Percentage']):6.2f}%")
print(f"total {tot / 1e6:.3f} ms" + (f", {tot / 1e3 / steps:.1f} us/step" if steps else ""))
