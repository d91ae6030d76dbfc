"""CPU, world_size 2 (gloo): the multi-GPU decomposition of SURVEY.md §8(e).

Each rank renders only the 64x64 tiles the product's shard rule gives it
(mrt_shard_mask, the same rule the bounce kernel uses), non-owned pixels stay
0, and one SUM reduce to rank 0 must reproduce the single-device image
bitwise.  The per-rank render is the CPU oracle here (no device in this
container); on the GPU box test_gpu_parity.py::test_shard_invariance checks
the same identity on the HIP path.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import SEED

W, H, L, FRAMES = 150, 100, 3, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for sub in ("metal-renderer_amd", "oracle", "tests"):
        sys.path.insert(0, os.path.join(root, sub))
    import mrt
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mask, owned = mrt.shard_mask(W, H, rank, world)
    sc = oracle.OracleScene(mrt.scene_path("cornellbox"))
    img, _ = sc.render(W, H, L, SEED, FRAMES, threads=2, pixel_mask=np.ascontiguousarray(mask))
    t = torch.from_numpy(img.copy())
    n = torch.tensor([owned], dtype=torch.int64)
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)   # the single accumulation-image reduce
    dist.reduce(n, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out_path, t.numpy())
        assert int(n.item()) == W * H
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_tile_sharded_reduce_equals_single_device(tmp_path, oracle_mod, mrt_mod, world):
    out = str(tmp_path / "reduced.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    reduced = np.load(out)
    full, _ = oracle_mod.OracleScene(mrt_mod.scene_path("cornellbox")).render(W, H, L, SEED, FRAMES, threads=4)
    assert np.array_equal(reduced[..., :3], full[..., :3])
    assert np.all(reduced[..., 3] == 1.0)
