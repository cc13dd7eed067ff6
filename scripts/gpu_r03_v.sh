#!/bin/bash
# Round 3 (v): BVH node order A/B (breadth-first throughout vs a breadth-first prefix of 64 / 256
# nodes with depth-first subtrees below) on C4 and C5, then the HEAD validation (scripts/gpu_r03_final_a.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
C4="--scene bunnylike --steps 4 --warmup 1 --no-cpu-baseline"
C5="--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32 --no-cpu-baseline"
LIBS="base=build/libspt_exp_base.so dfs64=build/libspt_exp_dfs64.so dfs256=build/libspt_exp_dfs256.so" \
ARGSETS="c4;$C4|c5;$C5|c4b;$C4" PARITY=1 PYTEST_K="bvh or bunny or interior or c4 or c5 or update" \
  bash scripts/gpu_ab2.sh > gpurun_out/v_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/v_ab.txt; exit 1; }
cat gpurun_out/v_ab.txt
bash scripts/gpu_r03_final_a.sh
