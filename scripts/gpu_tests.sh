#!/bin/bash
# GPU test run: the given pytest selection (default: the whole -m gpu suite), one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-tests}
SEL=${SEL:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
grep -E "bit-exact|identical|scene change|PASS|parity" gpurun_out/${T}_pytest.log | head -40
tail -2 gpurun_out/${T}_pytest.log
