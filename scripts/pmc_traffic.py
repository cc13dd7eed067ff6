"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs).

    python scripts/pmc_traffic.py OUT.json LABEL DIR [DIR ...]

Reads every *counter_collection.csv under the DIRs, and records per kernel (name up to '(') the
bytes of its largest dispatch (the bench's timed launch), corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950: FETCH_SIZE
(KB) reports half of a wide streaming read, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
The entry is keyed by LABEL (the bench configuration, e.g. "cornell-1920x1080-b8"); bench.py looks
it up for `roofline.traffic`.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    out, label, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    table = json.load(open(out)) if os.path.exists(out) else {}
    entry = {}
    for name, ctr in acc.items():
        if "FETCH_SIZE" not in ctr or "WRITE_SIZE" not in ctr:
            continue
        # the largest dispatch is the timed launch (warm-up launches cover fewer frames)
        fetch = max(ctr["FETCH_SIZE"])
        write = max(ctr["WRITE_SIZE"])
        entry[name] = {"fetch_bytes": 2.0 * fetch * 1024.0, "write_bytes": write * 1024.0,
                       "traffic_bytes": 2.0 * fetch * 1024.0 + write * 1024.0,
                       "dispatches": len(ctr["FETCH_SIZE"])}
    table[label] = entry
    json.dump(table, open(out, "w"), indent=1, sort_keys=True)
    for k, v in entry.items():
        print(f"{label} {k}: {v['traffic_bytes'] / 1e6:.1f} MB/launch over {v['dispatches']} dispatches")


if __name__ == "__main__":
    main()
