#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) \
    bench.py --gpus $n --steps $((6/n)) --warmup 1 --dist-backend gloo --no-cpu-baseline --save-image gpurun_out/img_w$n.npy > gpurun_out/multirank_$n.json 2> gpurun_out/multirank_$n.err || { echo "world $n failed"; tail -20 gpurun_out/multirank_$n.err; exit 1; }
done
timeout -k 10 300 python scripts/dbg_multirank.py
rm -f gpurun_out/img_w*.npy
