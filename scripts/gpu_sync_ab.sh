#!/bin/bash
# Host-inclusive App pattern (scripts/app_pattern.py) for the in-tree library and each VARIANTS library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MODES=${MODES:-fused,sync,registered}
timeout -k 10 200 python scripts/app_pattern.py --frames 500 --modes $MODES > gpurun_out/sy_intree.jsonl 2> gpurun_out/sy_intree.err && echo intree && cat gpurun_out/sy_intree.jsonl || exit 1
for v in ${VARIANTS:-}; do
  n=$(basename $v .so)
  SPT_LIB_PATH=$v timeout -k 10 200 python scripts/app_pattern.py --frames 500 --modes $MODES > gpurun_out/sy_$n.jsonl 2> gpurun_out/sy_$n.err && echo $n && cat gpurun_out/sy_$n.jsonl || exit 1
done
