#!/bin/bash
# Round-end measurement set (one GPU call): the default bench line, rocprofv3 kernel stats of the
# same command, FETCH_SIZE / WRITE_SIZE PMC passes of it (-> profiles/pmc_traffic.json via
# scripts/pmc_traffic.py), and the BVH configurations' bench lines. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-rp}
ARGS=${BENCH_ARGS:-}
timeout -k 10 300 python bench.py $ARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_rocprof -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_rocprof_bench.json 2> gpurun_out/${T}_rocprof.err || { echo "rocprof failed rc=$?"; tail -5 gpurun_out/${T}_rocprof.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${T}_pmc_$c -o run -- python3 bench.py $ARGS --no-cpu-baseline --no-profile > gpurun_out/${T}_pmc_$c.json 2> gpurun_out/${T}_pmc_$c.err || { echo "pmc $c failed rc=$?"; tail -5 gpurun_out/${T}_pmc_$c.err; exit 1; }
done
# C3: Cornell 4096 spp progressive (calls of 64 frames); the App's one frame per call (k_frame)
timeout -k 10 300 python bench.py --steps 4096 --warmup 64 --frames-per-call 64 --no-cpu-baseline > gpurun_out/${T}_bench_c3.json 2> gpurun_out/${T}_bench_c3.err || { echo "bench c3 failed rc=$?"; tail -5 gpurun_out/${T}_bench_c3.err; exit 1; }
tail -1 gpurun_out/${T}_bench_c3.json | cut -c1-300
timeout -k 10 300 python bench.py --steps 64 --warmup 4 --frames-per-call 1 --no-cpu-baseline > gpurun_out/${T}_bench_f1.json 2> gpurun_out/${T}_bench_f1.err || { echo "bench f1 failed rc=$?"; tail -5 gpurun_out/${T}_bench_f1.err; exit 1; }
tail -1 gpurun_out/${T}_bench_f1.json | cut -c1-300
for cfg in "bunnylike" "interior1m --width 3840 --height 2160 --steps 32"; do
  name=${cfg%% *}
  timeout -k 10 300 python bench.py --scene $cfg --no-cpu-baseline > gpurun_out/${T}_bench_$name.json 2> gpurun_out/${T}_bench_$name.err || { echo "bench $name failed rc=$?"; tail -5 gpurun_out/${T}_bench_$name.err; exit 1; }
  tail -1 gpurun_out/${T}_bench_$name.json | cut -c1-300
done
