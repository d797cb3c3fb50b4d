"""Turn a FETCH_SIZE / WRITE_SIZE rocprofv3 PMC pair (tools/pmc_session.sh) into
profiles/pmc_traffic.json, the HBM bytes per k_step launch that bench.py reports as
roofline.traffic.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports 1/2 of the bytes of
wide coalesced reads -> doubled; WRITE_SIZE is taken as reported.  Both counters are KiB.
usage: python tools/pmc_traffic.py <pmc dir with p1 (FETCH_SIZE) and p2 (WRITE_SIZE)> <workload> [kernel]
       <alg bytes per launch>
"""
import csv
import glob
import json
import sys
from pathlib import Path


def per_launch(d, counter):
    vals = {}
    for f in glob.glob(f"{d}/**/pmc_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if ("k_step" in row["Kernel_Name"] or "k_world" in row["Kernel_Name"]) and row["Counter_Name"] == counter:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for k_step under {d}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    d, workload, alg = sys.argv[1], sys.argv[2], float(sys.argv[3])
    fetch_kib, n1 = per_launch(d, "FETCH_SIZE")
    write_kib, n2 = per_launch(d, "WRITE_SIZE")
    try:  # wave-level VALU instructions per launch (VALU-issue roofline in bench.py)
        valu, _ = per_launch(d, "SQ_INSTS_VALU")
    except SystemExit:
        valu = None
    hbm = 2 * fetch_kib * 1024 + write_kib * 1024
    out = {
        "workload": workload,
        "kernel": sys.argv[4] if len(sys.argv) > 4 else "k_world",
        "launches_sampled": [n1, n2],
        "fetch_size_kib_per_launch": round(fetch_kib, 1),
        "write_size_kib_per_launch": round(write_kib, 1),
        "hbm_bytes_per_launch": round(hbm),
        "alg_bytes_per_launch": round(alg),
        "traffic_over_alg": round(hbm / alg, 3),
        "valu_insts_per_launch": valu,
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads), WRITE_SIZE x1; KiB -> B",
        "source": d,
    }
    p = Path(__file__).resolve().parent.parent / "profiles" / "pmc_traffic.json"
    p.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
