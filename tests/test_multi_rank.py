"""CPU: the N>1 bench path (independent shards, MAX-of-time / MIN-of-ok
reductions, whole-job aggregation) over torch.distributed gloo, world_size 2."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from firedancer_amd import shard


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import time
    import torch
    import torch.distributed as dist
    from firedancer_amd import synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = shard.dist_env()
    assert (env.rank, env.world) == (rank, world)
    # each rank builds its own shard of synthetic txns
    pay, desc, exp, nsig = synth.make_batch(64, synth.LARGE_NOOP, seed=shard.shard_seed(1234, rank), threads=1)
    sig0 = torch.from_numpy(pay[1:65].copy())
    gathered = [torch.zeros_like(sig0) for _ in range(world)]
    dist.all_gather(gathered, sig0)
    # a step whose duration differs per rank: the reported time must be the slowest rank's
    def step():
        time.sleep(0.01 * (rank + 1))
    dt = shard.timed_steps(step, steps=3, warmup=1, sync=lambda: None, barrier=dist.barrier)
    dt_max, ok = shard.reduce_max_min(dist, dt, ok=(rank == 0 or True), device="cpu")
    _, not_ok = shard.reduce_max_min(dist, dt, ok=(rank == 0), device="cpu")
    value = shard.aggregate_rate(world, nsig, 3, dt_max)
    # the configs[4] stream aggregate: SUM of per-rank sigs over the MAX per-rank stream time
    ssum, smax, sw = shard.reduce_sum_max(dist, units=1000 * (rank + 1), seconds=0.5 * (rank + 1), device="cpu")
    assert (ssum, smax, sw) == (3000.0, 1.0, 2)
    # the per-GPU report: every rank's row, in rank order
    rows = shard.gather_rows(dist, [rank, 10.0 * rank + 0.5], device="cpu")
    assert rows == [[float(r), 10.0 * r + 0.5] for r in range(world)]
    q.put((rank, dt, dt_max, ok, not_ok, value, [g.numpy().tobytes() for g in gathered], nsig))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_and_reductions():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, dt0, max0, ok0, nok0, v0, g0, n0), (r1, dt1, max1, ok1, nok1, v1, g1, n1) = res
    assert max0 == max1 == pytest.approx(max(dt0, dt1))
    assert max0 >= 3 * 0.02                      # rank 1 sleeps 20 ms x 3
    assert ok0 and ok1 and not nok0 and not nok1
    assert v0 == v1 == pytest.approx(2 * n0 * 3 / max0)
    assert g0 == g1 and g0[0] != g0[1]            # shards are distinct transactions


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
    assert len({shard.shard_seed(1234, r) for r in range(8)}) == 8
