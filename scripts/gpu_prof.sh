#!/bin/bash
# Bench + rocprofv3 kernel-trace/stats of the same bench command. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ARGS=${BENCH_ARGS:---steps 16 --warmup 2 --no-cpu-baseline}
TAG=${TAG:-prof}
timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_rocprof -o run --output-format csv -- python3 bench.py $ARGS --no-profile > gpurun_out/${TAG}_rocprof_bench.json 2> gpurun_out/${TAG}_rocprof.err || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/${TAG}_rocprof.err; exit 1; }
find gpurun_out/${TAG}_rocprof -name '*kernel_stats.csv' -exec cat {} \;
