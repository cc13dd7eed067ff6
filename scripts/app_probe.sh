#!/bin/bash
# One-frame-per-call App probes: wall time per call vs kernel time, with and without per-launch events.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for cfg in "512 512 4 -" "512 512 4 --no-profile" "128 128 4 -" "128 128 4 --no-profile" "16 16 4 --no-profile" "16 16 4 -"; do
  set -- $cfg
  extra=$4; [ "$extra" = "-" ] && extra=""
  timeout -k 10 120 python3 bench.py --scene app --width $1 --height $2 --bounces $3 --frames-per-step 1 --steps 2000 --warmup 32 --no-cpu-baseline $extra > gpurun_out/probe.json 2>gpurun_out/probe.err || { echo fail; tail -3 gpurun_out/probe.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/probe.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('$1x$2 b$3 $extra', d['value'], 'us/step', round(d['ms_per_step']*1000,2), 'kernel us', r.get('avg_launch_us'))"
done
