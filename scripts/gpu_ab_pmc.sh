#!/bin/bash
# A/B of experiment libraries with HBM counters: per variant and argument set, the bench line, then
# one rocprofv3 pass each for FETCH_SIZE and WRITE_SIZE of the same command (per-launch medians of
# the k_paths / k_frame dispatches printed by scripts/pmc_quick.py).
#   LIBS="label=path ..."  ARGSETS="tag;bench args|tag;bench args"  PMC=1  PARITY=1 PYTEST_K=...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
last=""
IFS='|' read -ra SETS <<< "${ARGSETS:-c2;--steps 10 --warmup 3 --no-cpu-baseline}"
for set in "${SETS[@]}"; do
  IFS=';' read -r tag args <<< "$set"
  for lv in ${LIBS:-default=}; do
    label=${lv%%=*}; lib=${lv#*=}
    if [ -n "$lib" ]; then export SPT_LIB_PATH=$lib; last=$lib; else unset SPT_LIB_PATH; fi
    timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/ab_${tag}_$label.json 2> gpurun_out/ab_${tag}_$label.err || { echo "$tag $label failed rc=$?"; tail -5 gpurun_out/ab_${tag}_$label.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab_${tag}_$label.json').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$tag', '$label', d['value'], d.get('schedule'), r.get('avg_launch_us'), d.get('lane_utilization'), d.get('bvh_per_traced_segment'))
"
    if [ -n "${PMC:-}" ]; then
      for ctr in FETCH_SIZE WRITE_SIZE; do
        rm -rf gpurun_out/abp_${tag}_${label}_$ctr
        timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/abp_${tag}_${label}_$ctr -o run -- python3 bench.py $args --no-cpu-baseline --no-profile > /dev/null 2> gpurun_out/abp_${tag}_${label}_$ctr.err || { echo "pmc $ctr failed rc=$?"; tail -5 gpurun_out/abp_${tag}_${label}_$ctr.err; exit 1; }
      done
      python3 scripts/pmc_quick.py "$tag $label" gpurun_out/abp_${tag}_${label}_FETCH_SIZE gpurun_out/abp_${tag}_${label}_WRITE_SIZE
    fi
  done
done
unset SPT_LIB_PATH
if [ -n "${PARITY:-}" ] && [ -n "$last" ]; then
  SPT_LIB_PATH=$last timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab_pytest.log 2>&1 || { echo "parity tests failed"; tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
