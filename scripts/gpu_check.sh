#!/bin/bash
# One GPU session: parity tests, then a short bench. Stops at the first crash/timeout
# (a plain test failure, exit 1, still lets the bench run so the numbers are seen).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 16 --warmup 2} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -c 4000 gpurun_out/bench.log
exit $rc2
