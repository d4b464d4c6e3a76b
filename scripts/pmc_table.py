#!/usr/bin/env python
"""Print mean PMC counter values per kernel for every pass under a pmc dir.
usage: scripts/pmc_table.py gpurun_out/pmc TAG"""
import csv, collections, glob, os, sys
root, tag = sys.argv[1], sys.argv[2]
for d in sorted(glob.glob(os.path.join(root, f"{tag}_*"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith("__amd") or k.startswith("k_scatter"):
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"== {os.path.basename(d)}")
        for k, cs in acc.items():
            print("  ", k, "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
