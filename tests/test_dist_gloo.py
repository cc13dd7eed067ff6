"""World-size-2 (and 3) gloo runs of the multi-GPU decomposition on CPU: each rank renders its
round-robin row shard (with the CPU oracle standing in for the GPU backend), the shards are gathered
to rank 0 with the same torch.distributed gather bench.py uses over RCCL, and the root's assembled
image must equal a single-process render bit for bit."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, FRAMES = 48, 29, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import cpu_ref

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spt = importlib.import_module("software-path-tracer_amd")
    sd = importlib.import_module("software-path-tracer_amd.distributed")
    prims, mats, env = spt.build_scene("cornell")
    shard = cpu_ref.RefScene(prims, mats, env).render(W, H, 0, FRAMES, 8, 2, 0, row_step=world, row_offset=rank)
    assert shard.shape[0] == len(sd.rows_of(H, rank, world))
    send = torch.from_numpy(sd.pad_shard(shard, H, world))
    gathered = sd.gather_to_root(send, world, rank)
    if rank == 0:
        img = sd.assemble_rows_host(torch.cat(gathered).numpy(), W, H, world)
        np.save(out_path, img)
    # max-over-ranks timing reduction, as bench.py does
    t = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert t.item() == world - 1
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_gather_equals_single_process(ref, spt, tmp_path, world):
    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    img = np.load(out)
    prims, mats, env = spt.build_scene("cornell")
    full = ref.RefScene(prims, mats, env).render(W, H, 0, FRAMES, 8, 2, 0)
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))
