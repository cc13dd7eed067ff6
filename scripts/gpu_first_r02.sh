#!/bin/bash
# Round-2 first call: the driver's smoke, the -m gpu suite, and the bench at the driver's shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/r02_smoke.log; exit 1; }
cat gpurun_out/r02_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/r02_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02_pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02_bench_driver.json 2> gpurun_out/r02_bench_driver.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/r02_bench_driver.err; exit 1; }
tail -1 gpurun_out/r02_bench_driver.json | cut -c1-600
