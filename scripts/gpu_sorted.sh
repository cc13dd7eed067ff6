#!/bin/bash
# Sorted ray queues (BVH): parity tests, then C4/C5 benches persistent vs split vs sorted.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sorted or bvh" > gpurun_out/so_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/so_pytest.log; exit 1; }
tail -1 gpurun_out/so_pytest.log
C4="--scene bunnylike --steps 4 --warmup 1 --no-cpu-baseline"
C5="--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32 --no-cpu-baseline"
for v in "c4sorted;$C4 --sorted" "c4split;$C4 --split" "c5sorted;$C5 --sorted" "c5split;$C5 --split" ${EXTRA_RUNS:-}; do
  IFS=';' read -r tag args <<< "$v"
  timeout -k 10 400 python bench.py $args > gpurun_out/so_$tag.json 2> gpurun_out/so_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/so_$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/so_$tag.json').read().strip().splitlines()[-1])
print('$tag', d['value'], d.get('schedule'), d.get('kernel_ms'))
"
done
