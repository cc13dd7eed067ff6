#!/bin/bash
# Round-3 final measurement, part A: the whole -m gpu suite, smoke, the driver's bench line (CPU
# baseline and parity included), the C2 round profile (PMC + rocprof), one frame per call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fa_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/fa_pytest.log; exit 1; }
tail -1 gpurun_out/fa_pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fa_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/fa_smoke.log; exit 1; }
grep smoke gpurun_out/fa_smoke.log
TAG=fa_c2 BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_round_profile.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fa_bench.json 2> gpurun_out/fa_bench.err || { echo "bench failed"; tail -20 gpurun_out/fa_bench.err; exit 1; }
tail -1 gpurun_out/fa_bench.json | cut -c1-400
TAG=fa_f1 BENCH_ARGS="--frames-per-step 1 --steps 64 --warmup 8" bash scripts/gpu_round_profile.sh || exit 1
TAG=fa_app BENCH_ARGS="--scene app --width 512 --height 512 --bounces 4 --frames-per-step 1 --steps 256 --warmup 32" bash scripts/gpu_round_profile.sh || exit 1
