"""bench.py's multi-rank step (render shard -> gather -> rank-0 un-permute -> timing with
barrier + max over ranks, pipelined over two shard-buffer sets) driven under gloo on CPU,
world_size 2.  The GPU render is replaced by the oracle's frame of this rank's tiles, XORed with
the step number so a frame assembled from the wrong step or buffer set shows; everything else
is bench.run_steps itself."""
import os
import time
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import Oracle, load_package

W, H, SPP = 64, 48, 4


class CpuWorkload:
    def __init__(self, rtm, world, rank, scenes):
        self.rtm, self.world, self.rank = rtm, world, rank
        orc = Oracle()
        self.full = [orc.render(sid, W, H, SPP, nthreads=1)[0] for sid in scenes]
        n = rtm.shard_elems(W, H, world)
        self.bufs = [[torch.zeros(n, dtype=torch.int32) for _ in scenes] for _ in range(2)]
        self.frames = [None for _ in scenes]
        self.renders = 0
        self.sets = []
        self.active = list(range(len(scenes)))      # bench.per_scene_steps renders one scene at a time

    def expected(self, i, step):
        return self.full[i] ^ np.uint32(step)

    def render_all(self, p=0):
        step = self.renders // len(self.full)
        self.sets.append(p)
        for i in self.active:
            shard = self.rtm.shard_from_frame(self.expected(i, step), self.rank, self.world)
            self.bufs[p][i].copy_(torch.from_numpy(shard.view(np.int32)))
            self.renders += 1

    def unshard(self, i, gathered):
        self.frames[i] = self.rtm.frame_from_shards(gathered.numpy().view(np.uint32), W, H, self.world)

    def sync(self):
        pass

    def mark(self):
        return time.perf_counter()

    def reset_times(self):
        pass


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        bench.W, bench.H, bench.SPP = W, H, SPP
        rtm = load_package()
        work = CpuWorkload(rtm, world, rank, bench.SCENES)
        elapsed = bench.run_steps(work, world, rank, steps=3, warmup=1, dist=dist, clock_warmup=0.0)
        report = bench.dist_report(work, world, rank, dist, 3, elapsed, reps=3)
        renders = work.renders
        # the drained pipeline holds the last (4th) step's frames; steps alternate buffer sets
        same = all(np.array_equal(work.frames[i], work.expected(i, 3)) for i in range(len(bench.SCENES))) \
            if rank == 0 else True
        same = same and work.sets == [0, 1, 0, 1]
        # BASELINE.md §4's per-scene figures: each scene alone through the same step (2 + 1 steps each)
        work.renders = 0
        per = bench.per_scene_steps(work, world, rank, dist, 2, 1)
        if rank == 0:
            # scene i's frame of the last step (the renders count every scene's render) assembled alone
            same = same and work.renders == 3 * len(bench.SCENES) and work.active == [0, 1]
            q.put(("ok", same, elapsed, renders, report, per))
        else:
            assert report is None and per is None
        dist.barrier()
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), 0, 0, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_run_steps_gloo(world):
    """run_steps over `world` gloo ranks, then the N > 1 line's self-explaining fields
    (bench.dist_report): the collective that ran (the rooted gather: gloo gathers CPU tensors), the
    backend and the communicator's size, every rank's render span (max / min / mean) and the gathers'
    own duration, all on rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, same, elapsed, renders, rep, per = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", same
    assert same
    assert elapsed > 0
    assert renders == (3 + 1) * 2        # (steps + warmup) x scenes
    assert rep["backend"] == "gloo" and rep["world_size"] == world
    assert rep["collective"] == "gather" and rep["collective_fallback"] is None
    r = rep["render_ms"]
    assert len(r["per_rank"]) == world and all(x > 0 for x in r["per_rank"])
    assert r["min"] <= r["mean"] <= r["max"] == max(r["per_rank"])
    g = rep["gather_ms"]
    assert len(g["per_rank"]) == world and g["rank0"] > 0 and g["max"] >= g["rank0"]
    assert g["source"].startswith("host clock") and g["reps"] == 3
    assert rep["step_ms"] > 0
    # the per-scene legs (Cornell and killeroo reported separately at every N)
    assert sorted(per) == ["1", "8"]
    for v in per.values():
        assert v["ms_per_step"] > 0 and v["value"] > 0 and v["unit"] == "Msamples/s" and v["steps"] == 2


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_bench_two_ranks_one_gpu_rehearsal():
    """The whole N > 1 bench path on the GPU -- AUTO's shard kernels (wide section on
    killeroo), the all-gather, the K3 un-permute and the max-over-ranks timing -- as two
    processes on one device under gloo (RCCL needs one GPU per rank).  Rank 0's --check
    compares both assembled 1080p frames with a one-GPU render, byte for byte."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--check", "--dist-backend", "gloo",
           "--one-device"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, r.stderr[-2000:]
    line = next(l for l in r.stdout.splitlines() if l.startswith("{"))
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["check"] == "2 frames equal to the one-GPU render"
    d = out["distributed"]
    assert d["backend"] == "gloo" and d["world_size"] == 2 and d["collective"] == "all_gather"
    assert d["collective_fallback"] and len(d["render_ms"]["per_rank"]) == 2 and d["gather_ms"]["rank0"] > 0
    # the overlap setting, the one-stream figure beside the value, per-frame latency and each scene alone
    assert out["overlap"] is True and out["value_one_stream"] > 0 and out["one_stream"]["frame_latency_ms"] > 0
    assert out["frame_latency_ms"] > 0 and sorted(out["per_scene_steps"]) == ["1", "8"]
