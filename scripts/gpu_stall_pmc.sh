#!/bin/bash
# Issue / stall breakdown of the C2 k_paths launch: two 8-counter SQ passes, each its
# own rocprofv3 run (--kernel-trace only), summarized by scripts/stall_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ARGS=${BENCH_ARGS:---steps 10 --warmup 3}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" \
           "SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/stall_pmc$i -o run -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/stall_pmc$i.json 2> gpurun_out/stall_pmc$i.err || { echo "stall pass $i failed rc=$?"; tail -5 gpurun_out/stall_pmc$i.err; exit 1; }
done
python3 scripts/stall_summary.py gpurun_out/stall_pmc1 gpurun_out/stall_pmc2
