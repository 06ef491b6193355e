"""The N>1 bench path on CPU: world_size-2 gloo processes run bench.py's
timed region (barrier + sync both sides, max over ranks) with a CPU step,
and the shard assignment gives every rank a disjoint buffer range with no
data-path collective. CPU only."""
import os
import socket
import time

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    delay = 0.002 * (rank + 1)          # rank 1 is the slow one
    step = lambda: time.sleep(delay)    # noqa: E731
    elapsed, per_step = bench.timed_region(step, steps=10, warmup=2, sync=lambda: None, dist=dist)
    q.put((rank, elapsed, per_step))
    dist.destroy_process_group()


def test_timed_region_max_over_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # Every rank reports the same (max) time, and it is the slow rank's.
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2]
    assert res[0][1] >= 10 * 0.004
    # Whole-job value counts every rank's bytes over that time.
    v = bench.aggregate_gibps(1 << 30, 10, world, res[0][1])
    assert v == pytest.approx(2 * 10 / res[0][1])


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_shards_are_disjoint(config):
    cfg = bench.CONFIGS[config]
    slots = cfg["count"] * cfg.get("nseg", 1)
    ranges = [(bench.shard_seed_base(r, slots), bench.shard_seed_base(r, slots) + slots) for r in range(8)]
    for a, b in zip(ranges, ranges[1:]):
        assert a[1] == b[0]  # contiguous, non-overlapping global buffer ids per rank


def test_bench_defaults():
    a = bench.parse([])
    assert a.gpus == 1 and a.config == "c2" and a.steps > 0 and a.warmup > 0
