#!/bin/bash
# Round 3 (x): BVH k_paths traversal batch (SPT_BVH_BATCH = 24 (HEAD) / 16 / 20 / 32) at the final
# kernel on C4 (8-wave instantiation, twice) and C5 (7-wave instantiation).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
C4="--scene bunnylike --steps 4 --warmup 1 --no-cpu-baseline"
C5="--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32 --no-cpu-baseline"
LIBS="b24=build/libspt_exp_b24.so b16=build/libspt_exp_b16.so b20=build/libspt_exp_b20.so b32=build/libspt_exp_b32.so" \
ARGSETS="c4;$C4|c5;$C5|c4b;$C4" \
  bash scripts/gpu_ab2.sh > gpurun_out/x_ab.txt 2>&1 || { echo "ab failed"; tail -30 gpurun_out/x_ab.txt; exit 1; }
cat gpurun_out/x_ab.txt
