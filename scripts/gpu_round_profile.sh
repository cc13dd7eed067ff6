#!/bin/bash
# Round measurement set for one bench launch shape (one GPU call), every step its own time limit:
#   1. PMC passes of the bench command (FETCH_SIZE | WRITE_SIZE | SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES
#      GRBM_GUI_ACTIVE), each with --kernel-trace only -> profiles/pmc_r02.json (scripts/pmc_collect.py)
#   2. the bench line itself (now finds its PMC record: traffic + VALU roofline)
#   3. rocprofv3 --kernel-trace --stats of the same command (the k_paths average must agree with 2)
# BENCH_ARGS selects the shape (default: the driver's default line); TAG names the outputs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-rp}
ARGS=${BENCH_ARGS:-}
i=0
dirs=""
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/${T}_pmc$i -o run -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/${T}_pmc$i.json 2> gpurun_out/${T}_pmc$i.err || { echo "pmc pass $i failed rc=$?"; tail -5 gpurun_out/${T}_pmc$i.err; exit 1; }
  dirs="$dirs gpurun_out/${T}_pmc$i"
done
label=$(python3 -c "import json;print(json.loads(open('gpurun_out/${T}_pmc1.json').read().strip().splitlines()[-1])['pmc_label'])")
python3 scripts/pmc_collect.py profiles/pmc_r02.json "$label" $dirs || exit 1
timeout -k 10 300 python bench.py $ARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_rocprof -o run --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/${T}_rocprof_bench.json 2> gpurun_out/${T}_rocprof.err || { echo "rocprof failed rc=$?"; tail -5 gpurun_out/${T}_rocprof.err; exit 1; }
cp profiles/pmc_r02.json gpurun_out/${T}_pmc_r02.json
