#!/bin/bash
# Round 3 (z): end-of-session check at HEAD — the -m gpu suite, smoke and the driver's default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/z_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/z_pytest.log; exit 1; }
tail -1 gpurun_out/z_pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/z_smoke.log; exit 1; }
grep smoke gpurun_out/z_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/z_bench.json 2> gpurun_out/z_bench.err || { echo "bench failed"; tail -20 gpurun_out/z_bench.err; exit 1; }
tail -1 gpurun_out/z_bench.json | cut -c1-300
