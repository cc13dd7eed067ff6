#!/bin/bash
# BVH scenes (C4, C5): bench lines with the §8d scene-byte accounting, PMC traffic for the same launch
# shapes, and the split wavefront schedule for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C4="--scene bunnylike --steps 4 --warmup 1"
C5="--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32"
TAG=c4 BENCH_ARGS="$C4" bash scripts/gpu_round_profile.sh || exit 1
TAG=c5 BENCH_ARGS="$C5" bash scripts/gpu_round_profile.sh || exit 1
for v in "c4split;$C4 --split --no-cpu-baseline"; do
  IFS=';' read -r tag args <<< "$v"
  timeout -k 10 300 python bench.py $args > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/$tag.err; exit 1; }
  tail -1 gpurun_out/$tag.json | cut -c1-200
done
