#!/bin/bash
# Round 5: the in-tree build (4-wide nodes, NEE with inline shadow rays) validated, then A/B of the
# 8-wide node variant (build/libspt_exp_w8.so, SPT_BVH_WIDTH=8) on the BVH configurations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=r05c BENCH_SETS="nee;--nee --no-cpu-baseline|c4nee;--scene bunnylike --steps 4 --warmup 1 --nee --no-cpu-baseline|neef1;--nee --frames-per-step 1 --steps 64 --warmup 8 --no-cpu-baseline" bash scripts/gpu_check.sh || exit 1
LIBS="default= w8=build/libspt_exp_w8.so" ARGSETS="c4;--scene bunnylike --steps 4 --warmup 1 --no-cpu-baseline|c5;--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32 --no-cpu-baseline|app;--scene app --width 512 --height 512 --bounces 4 --frames-per-step 1 --steps 256 --warmup 32 --no-cpu-baseline|c4f1;--scene bunnylike --frames-per-step 1 --steps 32 --warmup 4 --no-cpu-baseline" \
  PARITY=1 PYTEST_K="not deep_trees" bash scripts/gpu_ab2.sh
