#!/bin/bash
# The fused render+resolve (spt_render_resolve_rgba8): parity tests, the C++ backend tests, the App pattern
# host-inclusive timing (in-tree library and VARIANT), and an A/B of the one-frame bench lines against BASE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
BASE=${BASE:-build/libspt_exp_r6base.so}
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fused or registered" > gpurun_out/fz_pytest.log 2>&1 && tail -3 gpurun_out/fz_pytest.log &&
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cpp" > gpurun_out/fz_cpp.log 2>&1 && tail -2 gpurun_out/fz_cpp.log &&
timeout -k 10 240 python scripts/app_pattern.py --frames 300 --modes registered,fused,sync > gpurun_out/fz_app_pattern.jsonl 2> gpurun_out/fz_app_pattern.err && cat gpurun_out/fz_app_pattern.jsonl &&
if [ -n "${VARIANT:-}" ]; then
  SPT_LIB_PATH=$VARIANT timeout -k 10 240 python scripts/app_pattern.py --frames 300 --modes fused > gpurun_out/fz_app_pattern_variant.jsonl 2> gpurun_out/fz_app_pattern_variant.err && echo variant && cat gpurun_out/fz_app_pattern_variant.jsonl
fi &&
LIBS="base=$BASE new= base2=$BASE new2=" ARGSETS="app;--scene app --width 512 --height 512 --bounces 4 --frames-per-step 1 --steps 200 --warmup 20 --no-cpu-baseline|f1;--frames-per-step 1 --steps 64 --warmup 8 --no-cpu-baseline" bash scripts/gpu_ab2.sh
