#!/bin/bash
# Run bench.py under several env/arg variants in one GPU session; one summary line per variant.
# SWEEP="ENV=..;ARGS|ENV=..;ARGS|..."  (each item: space-separated env assignments, ';', extra bench args)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
BASE=${BASE_ARGS:---steps 32 --warmup 4 --no-cpu-baseline}
IFS='|' read -ra ITEMS <<< "${SWEEP}"
n=0
for item in "${ITEMS[@]}"; do
  n=$((n+1))
  envs=${item%%;*}; extra=${item#*;}
  out=gpurun_out/sweep_$n.json
  env $envs timeout -k 10 200 python bench.py $BASE $extra > $out 2> gpurun_out/sweep_$n.err || { echo "variant $n failed: $item"; tail -3 gpurun_out/sweep_$n.err; exit 1; }
  python3 -c "
import json,sys; r=json.load(open('$out')); k=r['kernel_ms']
print('%-45s %9.1f Ms/s  ext %.3f shade %.3f tail %.3f acc %.3f' % ('$item'[:45], r['value'], k['extend'], k['shade'], k['trace_tail'], k['accumulate']))"
done
