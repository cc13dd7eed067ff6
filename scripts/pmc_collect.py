"""Collate rocprofv3 PMC passes of one bench launch shape into profiles/pmc_r02.json.

    python scripts/pmc_collect.py OUT.json LABEL DIR [DIR ...]

Each DIR holds one `rocprofv3 --pmc ... --kernel-trace --output-format csv` run of the SAME bench
command (one pass per counter group: FETCH_SIZE | WRITE_SIZE | SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES
GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU). Per kernel (name up to the argument list) it keeps the median over that kernel's
dispatches (the warm-up and timed launches of one shape) of:
  traffic_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   (MI355X_MICROARCH.md HBM section: on
                  gfx950 FETCH_SIZE counts half of a wide streaming read; both counters in KB)
  valu_insts, salu_insts, waves                                (SQ counters, summed over the chip)
  duration_ns   = End_Timestamp - Start_Timestamp of the dispatch (median; duration_mean_ns: the mean)
  clock_ghz     = GRBM_GUI_ACTIVE / 8 XCDs / duration           (MI355X_MICROARCH.md, DVFS paragraph)
The record is keyed by LABEL (bench.py pmc_label: scene, size, bounces, ranks, frames per launch) and
stamped with the kernel-source hash bench.py checks, so it never describes another kernel or shape.
"""
import collections
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_source_hash() -> str:  # the same hash as bench.py's
    h = hashlib.sha256()
    for name in ("spt_kernels.hip", "spt_kernels.h", "spt_device.h", "spt_jit.hip"):
        with open(os.path.join(ROOT, "software-path-tracer_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def main():
    out, label, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (name, r["Dispatch_Id"])
                if key not in seen and "FETCH_SIZE" == r["Counter_Name"]:
                    seen.add(key)
                    dur[name].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    kernels = {}
    for name, ctr in vals.items():
        if "FETCH_SIZE" not in ctr or "WRITE_SIZE" not in ctr:
            continue
        med = {k: statistics.median(v) for k, v in ctr.items()}
        rec = {"traffic_bytes": 2.0 * med["FETCH_SIZE"] * 1024.0 + med["WRITE_SIZE"] * 1024.0,
               "fetch_bytes": 2.0 * med["FETCH_SIZE"] * 1024.0, "write_bytes": med["WRITE_SIZE"] * 1024.0,
               "dispatches": len(ctr["FETCH_SIZE"]), "duration_ns": statistics.median(dur[name]) if dur[name] else None,
               "duration_mean_ns": statistics.fmean(dur[name]) if dur[name] else None}
        if "SQ_INSTS_VALU" in med:
            rec["valu_insts"] = med["SQ_INSTS_VALU"]
            rec["salu_insts"] = med.get("SQ_INSTS_SALU")
            rec["waves"] = med.get("SQ_WAVES")
            rec["thread_cycles_valu"] = med.get("SQ_THREAD_CYCLES_VALU")
        if "GRBM_GUI_ACTIVE" in med and rec["duration_ns"]:
            rec["clock_ghz"] = round(med["GRBM_GUI_ACTIVE"] / 8.0 / rec["duration_ns"], 4)
        kernels[name] = rec
    table = json.load(open(out)) if os.path.exists(out) else {}
    table[label] = {"kernel_source": kernel_source_hash(), "kernels": kernels}
    json.dump(table, open(out, "w"), indent=1, sort_keys=True)
    for k, v in kernels.items():
        extra = ""
        if v.get("valu_insts") and v.get("duration_ns") and v.get("clock_ghz"):
            frac = v["valu_insts"] * 2.0 / (1024 * v["clock_ghz"] * v["duration_ns"])
            extra = f", VALU issue {frac:.3f} of peak at {v['clock_ghz']} GHz"
        print(f"{label} {k}: {v['traffic_bytes'] / 1e6:.1f} MB/launch over {v['dispatches']} dispatches{extra}")


if __name__ == "__main__":
    main()
