#!/bin/bash
# Rehearse the multi-rank bench path on a 1-GPU box: 2 and 3 ranks share cuda:0 over gloo (RCCL
# cannot put two ranks on one GPU); the assembled image must equal a single-rank render of the same
# frames. Steps are scaled so every run renders the image at 384 spp (64 frames per GPU per step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) \
    bench.py --gpus $n --steps $((6/n)) --warmup 1 --dist-backend gloo --no-cpu-baseline --save-image gpurun_out/img_w$n.npy > gpurun_out/multirank_$n.json 2> gpurun_out/multirank_$n.err || { echo "world $n failed"; tail -20 gpurun_out/multirank_$n.err; exit 1; }
  head -c 400 gpurun_out/multirank_$n.json; echo
done
timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --save-image gpurun_out/img_w1.npy > gpurun_out/multirank_1.json 2>gpurun_out/multirank_1.err || exit 1
python3 - <<'PY' || { rm -f gpurun_out/img_w*.npy; exit 1; }
import numpy as np
a = np.load("gpurun_out/img_w1.npy")
assert np.all(a[..., 3] == 384.0), a[..., 3].max()
for n in (2, 3):
    b = np.load(f"gpurun_out/img_w{n}.npy")
    same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
    print(f"world {n}: assembled image bit-identical to 1 rank: {same}")
    assert same
PY
rm -f gpurun_out/img_w*.npy
