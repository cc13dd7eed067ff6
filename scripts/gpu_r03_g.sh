#!/bin/bash
# Round 3: C2 issue/stall PMC at HEAD (two SQ passes), then BVH batch-size A/B on C4/C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
BENCH_ARGS="--steps 10 --warmup 3" bash scripts/gpu_stall_pmc.sh > gpurun_out/g_stall.json 2> gpurun_out/g_stall.err || { echo "stall pmc failed"; tail -5 gpurun_out/g_stall.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/g_stall.json')); print({k: round(v, 3) for k, v in d['per_wave_cycle'].items()}, 'lane density', round(d.get('valu_thread_utilization', 0), 3), 'lds conflicts/inst', round(d.get('lds_bank_conflict_cycles_per_lds_inst', 0), 3))"
SKIP_TESTS=1 LIBS="cur= b16=build/libspt_exp_b16.so b32=build/libspt_exp_b32.so" ARGSETS="c4;--scene bunnylike --steps 4 --warmup 1 --no-cpu-baseline|c5;--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32 --no-cpu-baseline" bash scripts/gpu_ab_tests.sh
