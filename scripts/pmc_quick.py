"""Per-launch medians of FETCH_SIZE (x2, MI355X_MICROARCH.md) and WRITE_SIZE for the persistent kernels
in rocprofv3 --pmc csv directories:  python scripts/pmc_quick.py LABEL DIR [DIR ...]"""
import collections
import csv
import glob
import os
import statistics
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if "k_paths" in name or "k_frame" in name:
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
for name, c in vals.items():
    fetch = statistics.median(c["FETCH_SIZE"]) * 2 if c.get("FETCH_SIZE") else None
    write = statistics.median(c["WRITE_SIZE"]) if c.get("WRITE_SIZE") else None
    print(f"{sys.argv[1]} {name}: fetch(x2) {fetch / 1e9 if fetch else float('nan'):.2f} GB, "
          f"write {write / 1e9 if write else float('nan'):.2f} GB per launch ({len(c.get('FETCH_SIZE', []))} launches)")
