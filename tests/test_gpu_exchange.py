"""GPU: the multi-GPU exchange of the accumulation image through the C ABI
(include/mrt.h mrt_comm_* / mrt_renderer_exchange).

One MI355X is available to the tests, so:
* libmrt's RCCL path runs with a 1-rank communicator: the gather (packed
  owned tiles -> rank 0 -> unpack), its overlapped form (collective on the
  communicator's stream, unpack deferred to the next exchange / flush,
  double-buffered packed tiles ordered by events) and the in-place SUM
  reduce must leave the 1-GPU image bitwise unchanged, over several steps;
* the whole N > 1 bench path (tile shards, exchange, max-over-ranks timing,
  --check-image: rank 0's exchanged image == a 1-GPU render, bitwise) runs
  as 2 and 3 ranks sharing the GPU, with the host transport (packed tiles to
  host memory, gloo gather, mrt_renderer_tiles_write on rank 0) — RCCL
  refuses two ranks on one device.
The per-rank renders themselves are pinned by the shard-invariance tests."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _render(mrt_mod, sc, W, H, L, frames, steps, comm=None, mode=0, shard=(0, 1)):
    r = mrt_mod.Renderer(sc, W, H, L, shard_rank=shard[0], shard_count=shard[1])
    for _ in range(steps):
        r.reset()
        r.draw(frames)
        if comm is not None:
            r.exchange(comm, mode)
    img = r.read_image()   # flushes a deferred exchange first
    r.close()
    return img


@pytest.mark.parametrize("inflight", ["1", "2"])
@pytest.mark.parametrize("mode", ["gather", "gather_overlap", "reduce"])
def test_rccl_exchange_single_rank(gpu, mrt_mod, monkeypatch, mode, inflight):
    """A 1-rank communicator: the exchange leaves the image bitwise as is.
    inflight 2 (a tile share's default: render launches on two streams) runs
    the overlapped gather on the renderer's main stream instead of the
    communicator's."""
    monkeypatch.setenv("MRT_INFLIGHT", inflight)
    sc = mrt_mod.Scene("cornellbox")
    W, H, L, frames = 200, 136, 4, 3
    ref = _render(mrt_mod, sc, W, H, L, frames, 1)
    comm = mrt_mod.Comm(mrt_mod.comm_unique_id(), 1, 0, 0)
    m = {"gather": mrt_mod.EXCHANGE_GATHER, "gather_overlap": mrt_mod.EXCHANGE_GATHER | mrt_mod.EXCHANGE_OVERLAP,
         "reduce": mrt_mod.EXCHANGE_REDUCE}[mode]
    got = _render(mrt_mod, sc, W, H, L, frames, 3, comm, m)
    comm.close()
    assert np.isfinite(ref).all() and ref[..., :3].max() > 0
    assert got.tobytes() == ref.tobytes()


def test_exchange_argument_checks(gpu, mrt_mod):
    sc = mrt_mod.Scene("cornellbox")
    comm = mrt_mod.Comm(mrt_mod.comm_unique_id(), 1, 0, 0)
    r = mrt_mod.Renderer(sc, 64, 64, 2, shard_rank=1, shard_count=2)
    with pytest.raises(mrt_mod.MrtError, match="shard"):
        r.exchange(comm, mrt_mod.EXCHANGE_GATHER)   # renderer shard != comm rank/size
    r.close()
    r = mrt_mod.Renderer(sc, 64, 64, 2)
    with pytest.raises(mrt_mod.MrtError, match="mode"):
        r.exchange(comm, mrt_mod.EXCHANGE_REDUCE | mrt_mod.EXCHANGE_OVERLAP)
    with pytest.raises(mrt_mod.MrtError, match="mode"):
        r.exchange(comm, 7)
    r.close()
    comm.close()


def test_host_tiles_roundtrip(gpu, mrt_mod):
    """mrt_renderer_tiles_read of every shard renderer, written into one
    renderer with mrt_renderer_tiles_write, rebuilds the 1-GPU image."""
    sc = mrt_mod.Scene("cornellbox")
    W, H, L, frames, S = 300, 170, 3, 2, 3
    ref = _render(mrt_mod, sc, W, H, L, frames, 1)
    r0 = mrt_mod.Renderer(sc, W, H, L, shard_rank=0, shard_count=S)
    r0.draw(frames)
    for k in range(1, S):
        rk = mrt_mod.Renderer(sc, W, H, L, shard_rank=k, shard_count=S)
        rk.draw(frames)
        packed = rk.tiles_read(k, S)
        assert packed.size == mrt_mod.tiles_packed_floats(W, H, k, S)
        rk.close()
        r0.tiles_write(k, packed)
    got = r0.read_image()
    r0.close()
    assert got[..., :3].tobytes() == ref[..., :3].tobytes()


@pytest.mark.parametrize("n", [2, 3, 8])
def test_rank0_unpacks_gathered_slabs(gpu, mrt_mod, n):
    """Rank 0's unpack of an N-rank ncclGather (renderer.cpp exchange_unpack:
    slab k at k * slab_floats, tile k*count + k-th of rank k) on one device:
    the receive buffer is filled with N synthetic packed slabs through the
    test entry mrt_debug_exchange_unpack, and the image must equal rank 0's
    own render with every other rank's tiles written by tiles_unpack_host,
    bitwise.  Slab 0 (rank 0's own tiles, never unpacked) is poisoned."""
    W, H = 3840, 2160
    sc = mrt_mod.Scene("cornellbox", device=0)
    r = mrt_mod.Renderer(sc, W, H, 1, shard_rank=0, shard_count=n)
    r.draw(1)
    expect = r.read_image()
    slab = mrt_mod.tiles_packed_floats(W, H, 0, n)
    gathered = np.zeros(n * slab, np.float32)
    gathered[:slab] = np.nan
    rng = np.random.default_rng(1000 + n)
    for k in range(1, n):
        m = mrt_mod.tiles_packed_floats(W, H, k, n)
        assert m <= slab
        data = rng.standard_normal(m).astype(np.float32)
        gathered[k * slab:k * slab + m] = data
        mrt_mod.tiles_unpack_host(data.reshape(-1, 64, 64, 4), expect, k, n)
    r.debug_exchange_unpack(n, gathered)
    got = r.read_image()
    r.close()
    assert got.tobytes() == expect.tobytes()
    # every pixel of the frame is rank 0's or came from a slab
    own = np.zeros((H, W), bool)
    mask = np.zeros((H, W), np.uint8)
    for k in range(n):
        mask[:] = 0
        mrt_mod.tiles_unpack_host(np.ones((mrt_mod.tiles_packed_floats(W, H, k, n) // 16384, 64, 64, 1), np.uint8),
                                  mask[..., None], k, n)
        assert not (own & mask.astype(bool)).any()
        own |= mask.astype(bool)
    assert own.all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_bench_multirank_rehearsal(gpu, world):
    """bench.py's N > 1 path, world ranks on the one GPU (host transport),
    --check-image asserts rank 0's exchanged image is the 1-GPU render."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--exchange-backend", "host", "--check-image"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == world and d["image_check"] == "bitwise equal to the 1-GPU render"
    assert d["value"] > 0


def test_bench_self_launches_ranks(gpu):
    """`bench.py --gpus 2` with no launcher starts its two ranks itself (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set before any HIP call) — never a
    silent single rank; rank 0's line reports n_gpus 2 and the bitwise image
    check of the exchanged frame."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--exchange-backend", "host", "--check-image"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["image_check"] == "bitwise equal to the 1-GPU render"


def test_overlapped_exchange_then_resize_reset_and_comm_close(gpu, mrt_mod):
    """A deferred (overlapped) gather is dropped, not unpacked, by resize (the
    buffers were packed for the old size) and by reset, and a flush after the
    communicator was destroyed never touches it: each image equals a plain
    render of the same frames."""
    sc = mrt_mod.Scene("cornellbox")
    L, frames = 3, 2
    mode = mrt_mod.EXCHANGE_GATHER | mrt_mod.EXCHANGE_OVERLAP
    comm = mrt_mod.Comm(mrt_mod.comm_unique_id(), 1, 0, 0)
    r = mrt_mod.Renderer(sc, 96, 64, L)
    r.draw(frames)
    r.exchange(comm, mode)
    r.resize(200, 130)                    # larger: the pending gather must not be unpacked into it
    r.draw(frames)
    big = r.read_image()
    r.exchange(comm, mode)
    r.reset()
    r.draw(frames)
    r.exchange(comm, mode)
    comm.close()                          # destroyed before the deferred unpack
    after = r.read_image()
    r.close()
    ref = _render(mrt_mod, sc, 200, 130, L, frames, 1)
    assert big.tobytes() == ref.tobytes() and after.tobytes() == ref.tobytes()


@pytest.mark.parametrize("failure", ["stuck", "async_error"])
def test_exchange_failure_aborts_communicator(gpu, mrt_mod, failure):
    """Failure handling of the exchange (SURVEY.md §5 "RCCL async error
    check"): on a 1-rank communicator the test entry mrt_debug_comm_fail makes
    the health checks see a collective that never completes (a stuck peer) or
    an asynchronous RCCL error.  mrt_renderer_sync / _exchange_flush then
    return MRT_ERR_COMM within the communicator's timeout (bounded wait, not a
    hang) after a real ncclCommAbort; every later use of the communicator
    fails cleanly with the same status; the renderer itself keeps rendering;
    the communicator closes and the process goes on."""
    import time
    sc = mrt_mod.Scene("cornellbox")
    W, H, L = 200, 136, 4
    comm = mrt_mod.Comm(mrt_mod.comm_unique_id(), 1, 0, 0)
    comm.set_timeout(300)
    r = mrt_mod.Renderer(sc, W, H, L)
    r.draw(2)
    r.exchange(comm, mrt_mod.EXCHANGE_GATHER | mrt_mod.EXCHANGE_OVERLAP)
    r.sync()   # healthy: the gather completes, nothing raised
    comm.check()
    r.draw(2)
    r.exchange(comm, mrt_mod.EXCHANGE_GATHER | mrt_mod.EXCHANGE_OVERLAP)
    comm.debug_fail(2 if failure == "stuck" else 1)
    t0 = time.time()
    with pytest.raises(mrt_mod.MrtError) as ei:
        if failure == "stuck":
            r.sync()
        else:
            r.exchange_flush()
    dt = time.time() - t0
    assert ei.value.status == mrt_mod.ERR_COMM, str(ei.value)
    assert ("did not complete" if failure == "stuck" else "asynchronous error") in str(ei.value)
    assert dt < 30.0 and (failure != "stuck" or dt >= 0.29), dt
    # later uses fail cleanly with the same status
    for call in (comm.check, lambda: r.exchange(comm, mrt_mod.EXCHANGE_GATHER)):
        with pytest.raises(mrt_mod.MrtError) as ei:
            call()
        assert ei.value.status == mrt_mod.ERR_COMM and "aborted" in str(ei.value)
    # the renderer is unaffected: it renders and reads back its own image
    r.reset()
    r.draw(3)
    img = r.read_image()
    ref = mrt_mod.Renderer(sc, W, H, L)
    ref.draw(3)
    assert img.tobytes() == ref.read_image().tobytes()
    ref.close()
    r.close()
    comm.close()
