#!/bin/bash
# One GPU call: the whole -m gpu suite, smoke(), then bench lines (BENCH_SETS: "tag;args|tag;args").
# Every step under its own time limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-chk}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
  tail -2 gpurun_out/${T}_pytest.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  grep smoke gpurun_out/${T}_smoke.log
fi
IFS='|' read -ra SETS <<< "${BENCH_SETS:-c2;--no-cpu-baseline}"
for set in "${SETS[@]}"; do
  IFS=';' read -r tag args <<< "$set"
  timeout -k 10 300 python bench.py $args > gpurun_out/${T}_bench_$tag.json 2> gpurun_out/${T}_bench_$tag.err || { echo "bench $tag failed rc=$?"; tail -5 gpurun_out/${T}_bench_$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/${T}_bench_$tag.json').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$tag', d['value'], d.get('schedule'), 'frac', r.get('frac'), 'us', r.get('avg_launch_us'), 'lanes', d.get('lane_utilization'), 'traced/s', d.get('traced_segments_per_s'), 'parity', (d.get('parity') or {}).get('exact_pixel_frac'), 'sim', (d.get('simulate_world') or {}).get('projected_speedup'), 'matched', (d.get('simulate_world') or {}).get('projected_speedup_matched'))
"
done
