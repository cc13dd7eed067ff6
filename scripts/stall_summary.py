"""Sum rocprofv3 SQ counters of the timed kernel (k_paths, or the kernel named by $STALL_KERNEL, e.g.
k_frame) over its dispatches (gpu_stall_pmc.sh) and print per-wave-cycle fractions. SQ counters are
summed over the 8 XCDs by rocprofv3."""
import collections
import csv
import glob
import json
import os
import sys

tot = collections.Counter()
disp = collections.Counter()
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if os.environ.get("STALL_KERNEL", "k_paths") not in name or "<true" in name:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]] += 1
wc = tot["SQ_WAVE_CYCLES"] or 1.0
out = {k: tot[k] for k in sorted(tot)}
out["dispatches"] = dict(disp)
frac = {k: tot[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                                 "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")}
out["per_wave_cycle"] = frac
if tot["SQ_INSTS_LDS"]:
    out["lds_bank_conflict_cycles_per_lds_inst"] = tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_INSTS_LDS"]
if tot["SQ_INSTS_VALU"]:
    out["valu_thread_utilization"] = tot["SQ_THREAD_CYCLES_VALU"] / (64.0 * tot["SQ_INSTS_VALU"])
print(json.dumps(out, indent=1))
