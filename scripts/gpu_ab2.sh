#!/bin/bash
# A/B of experiment libraries (build/libspt_exp_*.so via SPT_LIB_PATH) against the in-tree build:
# bench lines per variant, then the GPU parity tests against the LAST variant library.
#   LIBS="label=path ..."  ARGS="bench args"  PARITY=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
last=""
IFS='|' read -ra SETS <<< "${ARGSETS:-c2;--steps 10 --warmup 3 --no-cpu-baseline}"
for set in "${SETS[@]}"; do
  IFS=';' read -r tag args <<< "$set"
  for lv in ${LIBS:-default=}; do
    label=${lv%%=*}; lib=${lv#*=}
    if [ -n "$lib" ]; then export SPT_LIB_PATH=$lib; last=$lib; else unset SPT_LIB_PATH; fi
    timeout -k 10 170 python bench.py $args > gpurun_out/ab_${tag}_$label.json 2> gpurun_out/ab_${tag}_$label.err || { echo "$tag $label failed rc=$?"; tail -5 gpurun_out/ab_${tag}_$label.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab_${tag}_$label.json').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
sw=d.get('simulate_world') or {}
print('$tag', '$label', d['value'], d.get('schedule'), r.get('frac'), r.get('avg_launch_us'), d.get('lane_utilization'), (d.get('parity') or {}).get('exact_pixel_frac'), *([sw.get('max_ms_per_step'), sw.get('one_gpu_matched_ms_per_step'), sw.get('projected_speedup_matched')] if sw else []))
"
  done
done
unset SPT_LIB_PATH
if [ -n "${PARITY:-}" ] && [ -n "$last" ]; then
  SPT_LIB_PATH=$last timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab_pytest.log 2>&1 || { echo "parity tests failed"; tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
