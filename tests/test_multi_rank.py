"""CPU: the N>1 bench path (independent shards, MAX-of-time / MIN-of-ok
reductions, whole-job aggregation) over torch.distributed gloo, world_size 2 and 4."""
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
    assert (ssum, smax, sw) == (1000.0 * world * (world + 1) / 2, 0.5 * world, world)
    # the per-GPU report: every rank's row, in rank order
    rows = shard.gather_rows(dist, [rank, 10.0 * rank + 0.5], device="cpu")
    assert rows == [[float(r), 10.0 * r + 0.5] for r in range(world)]
    q.put((rank, dt, dt_max, ok, not_ok, value, [g.numpy().tobytes() for g in gathered], nsig))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_rank_shards_and_reductions(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == list(range(world))
    dts, maxs = [r[1] for r in res], [r[2] for r in res]
    assert all(m == pytest.approx(max(dts)) for m in maxs)
    assert maxs[0] >= 3 * 0.01 * world           # the last rank sleeps 10 ms x world, 3 steps
    assert all(r[3] for r in res) and not any(r[4] for r in res)
    n0 = res[0][7]
    assert all(r[5] == pytest.approx(world * n0 * 3 / maxs[0]) for r in res)
    g0 = res[0][6]
    assert all(r[6] == g0 for r in res) and len(set(g0)) == world   # shards are distinct transactions


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
    assert len({shard.shard_seed(1234, r) for r in range(8)}) == 8
