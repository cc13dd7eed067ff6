#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_nee.py -x -v --timeout 200 --timeout-method thread > gpurun_out/nee1_pytest.log 2>&1; rc=$?
tail -40 gpurun_out/nee1_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/nee1_bench_c2.json 2> gpurun_out/nee1_bench_c2.err || { echo bench failed; tail -5 gpurun_out/nee1_bench_c2.err; exit 1; }
tail -1 gpurun_out/nee1_bench_c2.json | cut -c1-400
