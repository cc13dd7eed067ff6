#!/bin/bash
# The round's final measurement set, one GPU call per part (every step under its own time limit; the
# first failure ends the call). Replaces the round-stamped gpu_r0N_final_* drivers.
#   PART=a  the whole -m gpu suite, smoke, the driver's default bench line (CPU baseline + parity),
#           the C2 round profile (PMC + rocprof), one frame per call (Cornell 1080p, the App's 512²),
#           the C2 NEE round profile
#   PART=b  C4 / C5 round profiles (scene bytes vs PMC traffic), then the per-rank multi-GPU preview
#           (--simulate-world N: every rank's shard timed) of C2 / C4 / C5 at N = ${SIM_NS:-2 4 8}, the
#           N = ${SIM_PMC_N:-8} lines with their PMC records and rocprof stats (gpu_round_profile.sh);
#           first the C4 NEE round profile
#   PART=b1 / b2  the two halves of b (one GPU call's time limit each)
#   PART=c  the App's per-frame pattern with the host hand-off (scripts/app_pattern.py), plain and under
#           rocprofv3 --kernel-trace --memory-copy-trace --stats
#   PART=m  the multi-rank rehearsal on one GPU (scripts/gpu_multirank.sh)
# R names the outputs (gpurun_out/${R}_*); copy what is judged into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${R:-r06}
C4="--scene bunnylike --steps 4 --warmup 1"
C5="--scene interior1m --width 3840 --height 2160 --steps 1 --warmup 1 --frames-per-step 32"
case "${PART:-a}" in
a)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${R}_pytest.log; exit 1; }
  tail -1 gpurun_out/${R}_pytest.log
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${R}_smoke.log; exit 1; }
  grep smoke gpurun_out/${R}_smoke.log
  # (100 timed launches: the rocprof average then weighs the clock ramp of the first ~15 lightly)
  TAG=${R}_c2 BENCH_ARGS="--steps 100 --warmup 5" bash scripts/gpu_round_profile.sh || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${R}_bench.err; exit 1; }
  tail -1 gpurun_out/${R}_bench.json | cut -c1-400
  TAG=${R}_f1 BENCH_ARGS="--frames-per-step 1 --steps 64 --warmup 8" bash scripts/gpu_round_profile.sh || exit 1
  TAG=${R}_app BENCH_ARGS="--scene app --width 512 --height 512 --bounces 4 --frames-per-step 1 --steps 256 --warmup 32" bash scripts/gpu_round_profile.sh || exit 1
  TAG=${R}_nee BENCH_ARGS="--steps 20 --warmup 5 --nee" bash scripts/gpu_round_profile.sh || exit 1
  ;;
b|b1|b2)
  if [ "${PART}" != b2 ]; then  # b1: the BVH round profiles only
  TAG=${R}_c4nee BENCH_ARGS="$C4 --nee" bash scripts/gpu_round_profile.sh || exit 1
  TAG=${R}_c4 BENCH_ARGS="$C4" bash scripts/gpu_round_profile.sh || exit 1
  TAG=${R}_c5 BENCH_ARGS="$C5" bash scripts/gpu_round_profile.sh || exit 1
  fi
  [ "${PART}" = b1 ] && exit 0  # b2: the multi-GPU preview only
  for n in ${SIM_NS:-2 4 8}; do
    for cfg in c2 c4 c5; do
      case $cfg in c2) a="--steps 10 --warmup 3";; c4) a="$C4";; c5) a="$C5";; esac
      if [ "$n" = "${SIM_PMC_N:-8}" ]; then  # the N-GPU line the driver's scaling run is closest to: with PMC
        TAG=${R}_pmcsim${n}_$cfg BENCH_ARGS="$a --simulate-world $n" bash scripts/gpu_round_profile.sh > gpurun_out/${R}_pmcsim${n}_$cfg.txt 2>&1 || { echo "sim $n $cfg profile failed"; tail -5 gpurun_out/${R}_pmcsim${n}_$cfg.txt; exit 1; }
        cp gpurun_out/${R}_pmcsim${n}_${cfg}_bench.json gpurun_out/${R}_sim${n}_$cfg.json
      else
        timeout -k 10 600 python bench.py $a --simulate-world $n --no-cpu-baseline > gpurun_out/${R}_sim${n}_$cfg.json 2> gpurun_out/${R}_sim${n}_$cfg.err || { echo "sim $n $cfg failed"; tail -5 gpurun_out/${R}_sim${n}_$cfg.err; exit 1; }
      fi
      python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_sim${n}_$cfg.json').read().strip().splitlines()[-1])
s=d.get('simulate_world') or {}
print('sim $n $cfg', d['value'], {k: s.get(k) for k in ('projected_speedup', 'projected_speedup_matched', 'max_ms_per_step', 'min_ms_per_step', 'slowest_rank')})
"
    done
  done
  ;;
c)
  timeout -k 10 300 python scripts/app_pattern.py > gpurun_out/${R}_app_pattern.json 2> gpurun_out/${R}_app_pattern.err || { echo "app_pattern failed"; tail -5 gpurun_out/${R}_app_pattern.err; exit 1; }
  cat gpurun_out/${R}_app_pattern.json
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/${R}_app_pattern_rocprof -o run --output-format csv -- python3 scripts/app_pattern.py > gpurun_out/${R}_app_pattern_rocprof.json 2> gpurun_out/${R}_app_pattern_rocprof.err || { echo "app_pattern rocprof failed"; tail -5 gpurun_out/${R}_app_pattern_rocprof.err; exit 1; }
  ;;
m)
  bash scripts/gpu_multirank.sh || exit 1
  ;;
esac
