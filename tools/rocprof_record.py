"""Record the rocprofv3 kernel-trace summary of a bench run (profiles/rocprof_kernel.json): the
step kernel's average duration over every launch of the run, keyed -- like the PMC record -- by the
kernel's source sha256 and the workload, both read from the bench JSON line the same profiled
command printed.  bench.py reports it beside its own live timer (roofline.rocprof).
usage: python tools/rocprof_record.py <kernel_stats.csv> <bench log holding the JSON line> [summary path]
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
stats, log = Path(sys.argv[1]), Path(sys.argv[2])
summary = sys.argv[3] if len(sys.argv) > 3 else str(stats)
line = next(l for l in log.read_text().splitlines() if l.startswith("{"))
bench = json.loads(line)
rf = bench["roofline"]
kernel = rf["kernel"]
row = next(r for r in csv.DictReader(stats.open()) if r["Name"] == kernel or r["Name"].startswith(kernel + "("))
rec = {
    "kernel": kernel,
    "workload": bench["config"]["workload"],
    "kernel_source_sha256": rf["kernel_source_sha256"],
    "avg_us": round(float(row["AverageNs"]) / 1e3, 3),
    "min_us": round(float(row["MinNs"]) / 1e3, 3),
    "max_us": round(float(row["MaxNs"]) / 1e3, 3),
    "calls": int(row["Calls"]),
    "summary": summary,
    "bench_under_profiler": {"kernel_us_per_launch": rf.get("kernel_us_per_launch"), "timer": rf.get("timer"),
                             "kernel_us_timed_region": rf.get("kernel_us_timed_region"),
                             "ms_per_step": bench.get("ms_per_step")},
}
out = ROOT / "profiles" / "rocprof_kernel.json"
out.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps(rec))
