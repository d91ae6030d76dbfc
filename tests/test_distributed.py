"""CPU, world_size 2 (gloo): the multi-GPU decomposition of SURVEY.md §8(e).

Each rank renders only the 64x64 tiles the product's shard rule gives it
(mrt_shard_mask, the same rule the bounce kernel uses), non-owned pixels stay
0, and one exchange to rank 0 — a SUM reduce of the image, or (bench.py's
default) a gather of the densely packed owned tiles — must reproduce the
single-device image bitwise.  The per-rank render is the CPU oracle here (no device in this
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


def _worker(rank, world, port, out_path, exchange="reduce"):
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
    n = torch.tensor([owned], dtype=torch.int64)
    dist.reduce(n, dst=0, op=dist.ReduceOp.SUM)
    if exchange == "reduce":
        t = torch.from_numpy(img.copy())
        dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)   # the single accumulation-image reduce
        out = t.numpy()
    else:
        # bench.py's default: gather of the densely packed owned tiles
        # (mrt_tiles_pack layout), unpacked on rank 0
        n_max = mrt.tiles_packed_floats(W, H, 0, world)
        packed = np.zeros(n_max, np.float32)
        mine = mrt.tiles_pack_host(img, rank, world).reshape(-1)
        assert mine.size == mrt.tiles_packed_floats(W, H, rank, world)
        packed[:mine.size] = mine
        lst = [torch.zeros(n_max) for _ in range(world)] if rank == 0 else None
        dist.gather(torch.from_numpy(packed), lst, dst=0)
        out = img.copy()
        if rank == 0:
            for k in range(1, world):
                m = mrt.tiles_packed_floats(W, H, k, world)
                mrt.tiles_unpack_host(lst[k].numpy()[:m].reshape(-1, 64, 64, 4), out, k, world)
    if rank == 0:
        np.save(out_path, out)
        assert int(n.item()) == W * H
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange", [(2, "reduce"), (2, "gather"), (3, "gather")])
def test_tile_sharded_exchange_equals_single_device(tmp_path, oracle_mod, mrt_mod, world, exchange):
    out = str(tmp_path / "reduced.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, exchange), nprocs=world, join=True)
    reduced = np.load(out)
    full, _ = oracle_mod.OracleScene(mrt_mod.scene_path("cornellbox")).render(W, H, L, SEED, FRAMES, threads=4)
    assert np.array_equal(reduced[..., :3], full[..., :3])
    assert np.all(reduced[..., 3] == 1.0)
