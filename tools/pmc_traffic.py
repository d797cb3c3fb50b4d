"""Turn the rocprofv3 PMC passes of tools/pmc_session.sh into profiles/pmc_traffic.json, the
per-launch HBM bytes (and VALU instructions) of the step kernel that bench.py reports as
roofline.traffic -- only for the kernel source it was measured on.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports 1/2 of the bytes of
wide coalesced reads -> doubled; WRITE_SIZE is taken as reported.  Both counters are KiB.

The bench JSON line that each pass's log holds gives the workload and the generated kernel's
source sha256 (roofline.kernel_source_sha256); every pass must agree.  When that line's headline
is the fused variant (roofline.plain set: a graph-mode run whose replay launches k_world with the
scenario program as its epilogue), the record's per-launch figures are those of the fused timer's
launches -- k_world dispatches [warmup+steps+5, warmup+steps+55) in dispatch order, as
tools/rocprof_record.py splits them -- and `plain` holds the last 50 launches (the step kernel
alone, bench.py's graph timer); `all_launches` averages every k_world dispatch.  The counter CSVs are
copied under profiles/<dest>/ so that the record's evidence is tracked.

usage: python tools/pmc_traffic.py <pmc dir: p1/, p1.log, p2/, ...> <profiles dest dir> [kernel]
"""
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


SLICE = None  # (lo, hi) over the kernel's dispatches in order, or None for all of them


def per_launch(d, counter, kernel, sl=None):
    vals = {}
    for f in glob.glob(f"{d}/**/pmc_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].split("(")[0].strip()
            if name == kernel and row["Counter_Name"] == counter:
                k = int(row["Dispatch_Id"])
                vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    v = [vals[k] for k in sorted(vals)]
    sl = SLICE if sl is None else sl
    if sl == "all":
        sl = None
    if sl is not None:
        v = v[sl[0]:sl[1]]
        if not v:
            raise SystemExit(f"{counter}: no {kernel} dispatches in slice {sl} under {d}")
    return sum(v) / len(v), len(v)


def bench_line(log):
    for line in reversed(Path(log).read_text().splitlines()):
        if line.startswith("{") and '"roofline"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {log}")


def main():
    d, dest = Path(sys.argv[1]), ROOT / sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_world"
    lines = [bench_line(f) for f in sorted(glob.glob(f"{d}/p*.log"))]
    hashes = {b["roofline"]["kernel_source_sha256"] for b in lines}
    workloads = {b["config"]["workload"] for b in lines}
    if len(hashes) != 1 or len(workloads) != 1:
        raise SystemExit(f"passes disagree: {hashes} {workloads}")
    b = lines[0]
    alg = b["roofline"]["alg_bytes_per_env_step"] * b["config"]["num_envs_per_gpu"]
    global SLICE
    fused = bool(b["roofline"].get("plain"))
    in_step = bool(b["roofline"].get("fused_no_tail"))  # (the headline: the timed steps' own launches)
    w, n = int(b.get("warmup", 0)), int(b.get("steps", 0))
    if in_step:
        SLICE = (w, w + n)
    elif fused:
        SLICE = (w + n + 5, w + n + 55)
    plain = all_l = None
    if fused:
        pf, pw = per_launch(d, "FETCH_SIZE", kernel, (-50, None))[0], per_launch(d, "WRITE_SIZE", kernel, (-50, None))[0]
        plain = {"slice": "last 50 k_world dispatches (bench.py graph timer: the step kernel alone)",
                 "hbm_bytes_per_launch": round(2 * pf * 1024 + pw * 1024),
                 "traffic_over_alg": round((2 * pf * 1024 + pw * 1024) / alg, 3)}
        try:
            plain["valu_insts_per_launch"] = per_launch(d, "SQ_INSTS_VALU", kernel, (-50, None))[0]
        except SystemExit:
            pass
        af, aw = per_launch(d, "FETCH_SIZE", kernel, "all")[0], per_launch(d, "WRITE_SIZE", kernel, "all")[0]
        all_l = {"hbm_bytes_per_launch": round(2 * af * 1024 + aw * 1024)}
        if in_step:  # (the chain without the tail: bench.py's fused timer launches)
            sl = (w + n + 5, w + n + 55)
            ff, fw = per_launch(d, "FETCH_SIZE", kernel, sl)[0], per_launch(d, "WRITE_SIZE", kernel, sl)[0]
            all_l["fused_no_tail_hbm_bytes_per_launch"] = round(2 * ff * 1024 + fw * 1024)
    fetch_kib, n1 = per_launch(d, "FETCH_SIZE", kernel)
    write_kib, n2 = per_launch(d, "WRITE_SIZE", kernel)
    extra = {}
    for c in ("SQ_INSTS_VALU", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
        try:
            extra[c.lower() + "_per_launch"] = per_launch(d, c, kernel)[0]
        except SystemExit:
            pass
    hbm = 2 * fetch_kib * 1024 + write_kib * 1024
    dest.mkdir(parents=True, exist_ok=True)
    for f in glob.glob(f"{d}/**/pmc_counter_collection.csv", recursive=True):
        rel = Path(f).relative_to(d)
        shutil.copy(f, dest / ("_".join(rel.parts)))
    for f in glob.glob(f"{d}/p*.log"):
        shutil.copy(f, dest / Path(f).name)
    out = {
        "workload": b["config"]["workload"],
        "kernel": kernel,
        "kernel_source_sha256": hashes.pop(),
        "variant": (f"the timed steps' launches (k_world + epilogue + post-replay tail), dispatches "
                    f"[{SLICE[0]}, {SLICE[1]})" if in_step else
                    "fused: k_world + the scenario program as its epilogue, dispatches "
                    f"[{SLICE[0]}, {SLICE[1]}) (bench.py's fused timer)" if fused else "the step kernel alone"),
        "launches_sampled": [n1, n2],
        "fetch_size_kib_per_launch": round(fetch_kib, 1),
        "write_size_kib_per_launch": round(write_kib, 1),
        "hbm_bytes_per_launch": round(hbm),
        "alg_bytes_per_launch": round(alg),
        "traffic_over_alg": round(hbm / alg, 3),
        "alg_note": ("alg = SURVEY 8(d)'s physics bytes; the fused launch also writes the scenario "
                     "program's outputs and the state write-back's stores: bench.py reports "
                     "roofline.fused_alg.traffic_over_alg against the fused launch's own bytes") if fused else None,
        "valu_insts_per_launch": extra.get("sq_insts_valu_per_launch"),
        **{k: v for k, v in extra.items() if k != "sq_insts_valu_per_launch"},
        "plain": plain,
        "all_launches": all_l,
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads), WRITE_SIZE x1; KiB -> B",
        "source": str(dest.relative_to(ROOT)),
    }
    p = ROOT / "profiles" / "pmc_traffic.json"
    p.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
