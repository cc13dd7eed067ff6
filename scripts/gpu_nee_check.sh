#!/bin/bash
# NEE on the GPU: the NEE parity suite, smoke, then the C2 / C4 NEE bench lines (the rates of the NEE
# kernels after a change to light_sample). Every step under its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${R:-r05_w}
timeout -k 10 600 python -u -m pytest tests/test_gpu_nee.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_nee_pytest.log 2>&1 || { echo "NEE tests failed"; tail -30 gpurun_out/${R}_nee_pytest.log; exit 1; }
tail -1 gpurun_out/${R}_nee_pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${R}_smoke.log; exit 1; }
grep smoke gpurun_out/${R}_smoke.log
for set in "c2nee;--nee --steps 20 --warmup 5" "c4nee;--scene bunnylike --steps 4 --warmup 1 --nee"; do
  tag=${set%%;*}; args=${set#*;}
  timeout -k 10 240 python bench.py $args --no-cpu-baseline > gpurun_out/${R}_bench_$tag.json 2> gpurun_out/${R}_bench_$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/${R}_bench_$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_bench_$tag.json').read().strip().splitlines()[-1])
print('$tag', d['value'], d['unit'], (d.get('roofline') or {}).get('avg_launch_us'), d.get('parity', {}) if isinstance(d.get('parity'), dict) else d.get('parity'))
"
done
