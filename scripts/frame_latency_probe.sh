#!/bin/bash
# k_frame latency probe: kernel durations (rocprofv3 --kernel-trace --stats) of one-frame launches on
# tiny images (one wave) and the App size, over max bounces, for the App (BVH, LDS-resident) and the
# Cornell (flat) scenes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/flp
export TMPDIR=/tmp
for cfg in "app 16 16 0" "app 16 16 1" "app 16 16 2" "app 16 16 4" "app 512 512 4" "cornell 16 16 0" "cornell 16 16 1" "cornell 16 16 4" "cornell 16 16 8"; do
  set -- $cfg
  tag=$1_$2_b$4
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/flp/$tag -o run -- python3 bench.py --scene $1 --width $2 --height $3 --bounces $4 --frames-per-step 1 --steps 500 --warmup 32 --no-cpu-baseline --no-profile > gpurun_out/flp/$tag.json 2> gpurun_out/flp/$tag.err || { echo "fail $tag"; tail -3 gpurun_out/flp/$tag.err; exit 1; }
  python3 - "$tag" <<'PY'
import csv, glob, json, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/flp/{tag}/**/*kernel_stats.csv", recursive=True)[0]
d = json.loads(open(f"gpurun_out/flp/{tag}.json").read().strip().splitlines()[-1])
for r in csv.DictReader(open(f)):
    if "k_frame<false" in r["Name"]:
        print(tag, "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2), "min_us", round(float(r["MinNs"]) / 1e3, 2), "wall_us_per_step", round(d["ms_per_step"] * 1e3, 2))
PY
done
