import csv, sys, collections, glob
for tag in sys.argv[1:]:
    tot = collections.defaultdict(float); n = collections.Counter(); dur = []
    for f in glob.glob(f"gpurun_out/pmc/{tag}/p*/pmc_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if "k_step" not in name and "k_world" not in name: continue
            key = (row["Counter_Name"])
            tot[key] += float(row["Counter_Value"])
            n[(key, row["Dispatch_Id"])] += 1
    disp = {}
    for (k, d) in n: disp.setdefault(k, set()).add(d)
    print("==", tag)
    for k in sorted(tot):
        print(f"  {k:28s} per-launch {tot[k]/len(disp[k]):.4g}  (launches {len(disp[k])})")
