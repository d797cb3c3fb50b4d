"""Record the rocprofv3 kernel-trace summary of a bench run (profiles/rocprof_kernel.json), keyed
-- like the PMC record -- by the kernel's source sha256 and the workload, both read from the bench
JSON line the same profiled command printed.  bench.py reports it beside its own live timer
(roofline.rocprof).

With the kernel trace beside the stats (<prefix>_kernel_trace.csv) the record splits the step
kernel's launches as the bench ran them: `avg_us` = the last 50 launches, the bench's headline
timer (World.step() replayed back to back, the step kernel alone); `in_step_us` = the launches of
the timed steps (in a fused replay k_world also runs the scenario program as its epilogue);
`avg_all_us` = every launch.  Without the trace, `avg_us` is the stats' average over every launch.
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
avg_all = round(float(row["AverageNs"]) / 1e3, 3)
split = {}
trace = stats.with_name(stats.name.replace("kernel_stats", "kernel_trace"))
if trace.exists():
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(trace.open())
                if r["Kernel_Name"] == kernel or r["Kernel_Name"].startswith(kernel + "("))
    dur = [(e - s) / 1e3 for s, e in ks]
    timer_n = 50  # (bench.py time_step_kernel_graph: 5 replays x 10 launches, the run's last)
    w, n = int(bench.get("warmup", 0)), int(bench.get("steps", 0))
    split = {"avg_us": round(sum(dur[-timer_n:]) / timer_n, 3), "timer_launches": timer_n,
             "in_step_us": round(sum(dur[w:w + n]) / max(1, len(dur[w:w + n])), 3), "in_step_launches": len(dur[w:w + n]),
             "avg_all_us": avg_all, "trace": str(trace)}
    if (rf.get("plain") or {}).get("kernel_us"):  # (bench.py time_fused_chain: 5 warm + 50 right after the steps)
        fz = dur[w + n + 5:w + n + 55]
        split["fused_timer_us"] = round(sum(fz) / max(1, len(fz)), 3)
        split["fused_timer_launches"] = len(fz)
rec = {
    "kernel": kernel,
    "workload": bench["config"]["workload"],
    "kernel_source_sha256": rf["kernel_source_sha256"],
    "avg_us": split.get("avg_us", avg_all),
    "min_us": round(float(row["MinNs"]) / 1e3, 3),
    "max_us": round(float(row["MaxNs"]) / 1e3, 3),
    "calls": int(row["Calls"]),
    **{k: v for k, v in split.items() if k != "avg_us"},
    "summary": summary,
    "bench_under_profiler": {"kernel_us_per_launch": rf.get("kernel_us_per_launch"), "timer": rf.get("timer"),
                             "kernel_us_timed_region": rf.get("kernel_us_timed_region"),
                             "ms_per_step": bench.get("ms_per_step")},
}
out = ROOT / "profiles" / "rocprof_kernel.json"
out.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps(rec))
