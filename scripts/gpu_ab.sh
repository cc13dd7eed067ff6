#!/bin/bash
# GPU session: parity tests, then bench variants (VARIANTS="label;ENV;ARGS|..."), one JSON each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -n 25 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
IFS='|' read -ra VS <<< "${VARIANTS:-default;;--steps 64 --warmup 4}"
for v in "${VS[@]}"; do
  IFS=';' read -r label envs args <<< "$v"
  env $envs timeout -k 10 300 python bench.py $args > gpurun_out/ab_$label.json 2> gpurun_out/ab_$label.err
  rc=$?
  echo "== $label rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$label.err; exit $rc; fi
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_$label.json').read().strip().splitlines()[-1])
r=d['roofline'] or {}
print('$label', d['value'], d.get('schedule'), r.get('kernel'), r.get('frac'), r.get('avg_launch_us'), d.get('parity'), d.get('kernel_ms'))
"
done
