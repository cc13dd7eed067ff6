#!/bin/bash
# PMC A/B of experiment libraries (LIBS="label=path ...", empty path = in-tree): one rocprofv3 --pmc pass
# per library over the same bench command (ARGS), then the per-dispatch medians of the k_paths counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
CTRS=${CTRS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"}
for lv in ${LIBS:-default=}; do
  label=${lv%%=*}; lib=${lv#*=}
  if [ -n "$lib" ]; then export SPT_LIB_PATH=$lib; else unset SPT_LIB_PATH; fi
  rm -rf gpurun_out/pmcab_$label
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d gpurun_out/pmcab_$label -o run -- python3 bench.py ${ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-profile} > gpurun_out/pmcab_$label.json 2> gpurun_out/pmcab_$label.err || { echo "pmc $label failed rc=$?"; tail -5 gpurun_out/pmcab_$label.err; exit 1; }
  python3 - "$label" <<'PY'
import csv, glob, statistics, sys, collections
label = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for f in glob.glob(f"gpurun_out/pmcab_{label}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if "k_paths" not in name and "k_frame" not in name:
            continue
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[name][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
for name, c in vals.items():
    med = {k: statistics.median(v) for k, v in c.items()}
    d = statistics.median(dur[name].values())
    print(label, name[:60], f"dispatches {len(dur[name])} dur_us {d/1e3:.1f}", " ".join(f"{k}={v:.4g}" for k, v in sorted(med.items())))
PY
done
