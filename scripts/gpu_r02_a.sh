#!/bin/bash
# Round-2 GPU call A: the whole -m gpu suite, smoke, bench default, gloo multi-rank rehearsal,
# then the round profile (PMC -> profiles/pmc_r02.json, bench line, rocprof stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/a_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/a_pytest.log; exit 1; }
tail -2 gpurun_out/a_pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/a_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/a_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/a_bench.err; exit 1; }
tail -1 gpurun_out/a_bench.json | cut -c1-700
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/a_bench_driver.json 2> gpurun_out/a_bench_driver.err || { echo "bench driver failed"; tail -20 gpurun_out/a_bench_driver.err; exit 1; }
tail -1 gpurun_out/a_bench_driver.json | cut -c1-300
bash scripts/gpu_multirank.sh || exit 1
TAG=a_rp bash scripts/gpu_round_profile.sh || exit 1
