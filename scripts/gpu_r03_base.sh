#!/bin/bash
# Round-3 baseline at HEAD: the -m gpu suite, the driver's bench shape, and C4/C5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/b3_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/b3_pytest.log; exit 1; }
tail -1 gpurun_out/b3_pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b3_bench.json 2> gpurun_out/b3_bench.err || { echo "bench failed"; tail -20 gpurun_out/b3_bench.err; exit 1; }
tail -1 gpurun_out/b3_bench.json | cut -c1-300
timeout -k 10 300 python bench.py --scene bunnylike --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/b3_c4.json 2> gpurun_out/b3_c4.err || { echo "c4 failed"; tail -20 gpurun_out/b3_c4.err; exit 1; }
tail -1 gpurun_out/b3_c4.json | cut -c1-300
timeout -k 10 300 python bench.py --scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32 --no-cpu-baseline > gpurun_out/b3_c5.json 2> gpurun_out/b3_c5.err || { echo "c5 failed"; tail -20 gpurun_out/b3_c5.err; exit 1; }
tail -1 gpurun_out/b3_c5.json | cut -c1-300
