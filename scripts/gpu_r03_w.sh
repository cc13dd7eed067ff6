#!/bin/bash
# Round 3 (w): flat k_paths hand-out threshold A/B (SPT_FLAT_REFILL_MIN = 1 (HEAD) / 8 / 16 / 24) on
# C2 (twice) and the simulated 1/8 shard, then the whole -m gpu suite on the last variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
C2="--steps 20 --warmup 5 --no-cpu-baseline"
LIBS="r1=build/libspt_exp_r1.so r8=build/libspt_exp_r8.so r16=build/libspt_exp_r16.so r24=build/libspt_exp_r24.so" \
ARGSETS="c2;$C2|sim8;--simulate-world 8 --steps 10 --warmup 3 --no-cpu-baseline|c2b;$C2" PARITY=1 \
  bash scripts/gpu_ab2.sh > gpurun_out/w_ab.txt 2>&1 || { echo "ab failed"; tail -30 gpurun_out/w_ab.txt; exit 1; }
cat gpurun_out/w_ab.txt
