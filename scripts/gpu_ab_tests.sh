#!/bin/bash
# A/B bench lines (scripts/gpu_ab2.sh) then the -m gpu suite against the in-tree library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_pytest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/t_pytest.log; exit 1; }
  tail -1 gpurun_out/t_pytest.log
fi
bash scripts/gpu_ab2.sh
