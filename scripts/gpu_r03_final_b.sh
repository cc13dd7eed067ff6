#!/bin/bash
# Round-3 final measurement, part B: BVH scenes C4 / C5 with PMC (scene bytes vs traffic), then the
# multi-GPU shard preview (rank 0's shard of an N-GPU run) with PMC records for the driver's N-GPU lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
C4="--scene bunnylike --steps 4 --warmup 1"
C5="--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32"
TAG=fb_c4 BENCH_ARGS="$C4" bash scripts/gpu_round_profile.sh || exit 1
TAG=fb_c5 BENCH_ARGS="$C5" bash scripts/gpu_round_profile.sh || exit 1
for n in 2 4 8; do
  TAG=fb_sim$n BENCH_ARGS="--simulate-world $n --steps 10 --warmup 3" bash scripts/gpu_round_profile.sh || exit 1
done
bash scripts/gpu_multirank.sh || exit 1
