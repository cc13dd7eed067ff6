#!/bin/bash
# Specialized (run-time compiled) vs generic flat kernels: GPU tests, smoke, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/s_pytest.log; exit 1; }
tail -2 gpurun_out/s_pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/s_smoke.log; exit 1; }
cat gpurun_out/s_smoke.log | grep smoke
for v in "c2;--steps 10 --warmup 3 --no-cpu-baseline" "c2gen;--steps 10 --warmup 3 --no-cpu-baseline --no-specialize" \
         "f1;--steps 64 --warmup 8 --frames-per-step 1 --no-cpu-baseline" "f1gen;--steps 64 --warmup 8 --frames-per-step 1 --no-cpu-baseline --no-specialize"; do
  IFS=';' read -r tag args <<< "$v"
  timeout -k 10 240 python bench.py $args > gpurun_out/s_$tag.json 2> gpurun_out/s_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/s_$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/s_$tag.json').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$tag', d['value'], d.get('schedule'), d.get('specialized'), r.get('frac'), r.get('avg_launch_us'), d.get('lane_utilization'))
"
done
