"""Multi-rank sharding on CPU (gloo, world_size 2 and 3): every rank renders only the 16x16
tiles it owns (row-rotated t' % N == rank), shards are all-gathered and gathered to rank 0, rank 0
un-permutes, and the frame is
byte-identical to the single-process frame (partition invariance).
The per-tile pixels come from the oracle here; on GPUs the same layout is produced by
rt_render_shard_device and undone by rt_unshard_device (tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import Oracle, load_package

W, H, SPP, SCENE = 200, 150, 4, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rtm = load_package()
        full, _, _ = Oracle().render(SCENE, W, H, SPP, nthreads=2)
        shard = torch.from_numpy(rtm.shard_from_frame(full, rank, world).view(np.int32))
        gathered = rtm.all_gather_shards(shard, world)
        rooted = rtm.gather_shards(shard, world, dst=0)
        if rank == 0:
            img = rtm.frame_from_shards(gathered.numpy().view(np.uint32), W, H, world)
            img2 = rtm.frame_from_shards(rooted.numpy().view(np.uint32), W, H, world)
            q.put(("ok", bool(np.array_equal(img, full) and np.array_equal(img2, full)),
                   len(rtm.shard_tile_ids(W, H, 0, world))))
        else:
            assert rooted is None
        dist.barrier()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e), 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frame_is_partition_invariant(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, same, ntiles = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", same
    assert same
    assert ntiles == len(range(0, 13 * 10, world))


def test_shard_layout_roundtrip_many_ranks():
    rtm = load_package()
    rng = np.random.default_rng(0)
    img = rng.integers(0, 2**24, size=(77, 131), dtype=np.uint32)
    for n in (1, 2, 5, 8):
        g = np.concatenate([rtm.shard_from_frame(img, r, n) for r in range(n)])
        np.testing.assert_array_equal(rtm.frame_from_shards(g, 131, 77, n), img)
        assert g.size == n * rtm.shard_elems(131, 77, n)
