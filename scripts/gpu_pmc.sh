#!/bin/bash
# rocprofv3 PMC passes (each its own run, kernel-trace only alongside) over a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ARGS=${BENCH_ARGS:---steps 8 --warmup 1 --no-cpu-baseline --no-profile}
TAG=${TAG:-pmc}
i=0
SETS=${PMC_SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE|SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH"}
IFS='|' read -ra SET_LIST <<< "$SETS"
for set in "${SET_LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/${TAG}_$i -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  echo "pass $i ok: $set"
done
