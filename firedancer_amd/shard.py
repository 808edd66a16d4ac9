"""Multi-GPU orchestration: independent per-GPU shards, no data-path collective.

Verdicts are per signature, so each rank verifies its own
shard; the only collectives are the measurement ones (MAX of the timed
interval, MIN of the correctness flag).

Two sharding rules are used, one per bench line:
- the headline (configs[1]) gives every rank its own synthetic batch,
  generated from a distinct seed (`shard_seed`) and resident in that rank's
  HBM; no rank sees another's transactions;
- the configs[4] stream keeps the reference's verify-tile rule
  (src/disco/verify/fd_verify_tile.c:47-48): tile i of T keeps the frags
  with seq % T == i, and tile i runs on GPU i % G (fd_verify_gpu.c, the
  link).  That rule lives in the tile, not here.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass


@dataclass
class DistEnv:
    rank: int
    world: int
    local_rank: int


def dist_env() -> DistEnv:
    return DistEnv(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                   int(os.environ.get("LOCAL_RANK", "0")))


def shard_seed(base: int, rank: int) -> int:
    """Distinct, reproducible synthetic-data seed per rank."""
    return (base + 7919 * rank) & 0xFFFFFFFFFFFF


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous split of n_total items (used when one global batch is sharded)."""
    return n_total * rank // world, n_total * (rank + 1) // world


def timed_steps(step, steps: int, warmup: int, sync, barrier) -> float:
    """W untimed warmups, then exactly K steps bracketed by barrier + device sync on both sides."""
    for _ in range(warmup):
        step()
    sync()
    barrier(); sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync(); barrier()
    return time.perf_counter() - t0


def reduce_max_min(dist, dt: float, ok: bool, device) -> tuple[float, bool]:
    """MAX over ranks of the timed interval and MIN of the results flag."""
    import torch
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    o = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
    return float(t.item()), bool(o.item())


def aggregate_rate(world: int, units_per_rank: int, steps: int, dt_max: float) -> float:
    """Whole-job throughput: all ranks' units over the slowest rank's time (weak scaling)."""
    return world * units_per_rank * steps / dt_max


def reduce_sum_max(dist, units: float, seconds: float, device) -> tuple[float, float, int]:
    """SUM over ranks of units, MAX of seconds (a concurrent per-rank stream), and the rank count."""
    import torch
    u = torch.tensor([float(units)], dtype=torch.float64, device=device)
    s = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    w = 1
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        dist.all_reduce(s, op=dist.ReduceOp.MAX)
        w = dist.get_world_size()
    return float(u.item()), float(s.item()), w


def gather_rows(dist, row: list[float], device) -> list[list[float]]:
    """Every rank's small vector of measurements, in rank order (rank 0 uses them for the per-GPU report)."""
    import torch
    t = torch.tensor([float(x) for x in row], dtype=torch.float64, device=device)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [t.tolist()]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]
