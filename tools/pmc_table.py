#!/usr/bin/env python3
"""Mean per-dispatch PMC counters of kernels matching a regex from tools/pmc_passes.sh pass dirs.
usage: python tools/pmc_table.py gpurun_out/pmc_<tag> <kernel-regex>"""
import collections, csv, glob, re, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(sys.argv[1] + "/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if re.search(sys.argv[2], r["Kernel_Name"]):
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, d in agg.items():
    v = list(d.values())
    print(f"{c:30s} {sum(v) / len(v):14.5g}  (n={len(v)})")
