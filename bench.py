#!/usr/bin/env python3
"""bench.py -- ed25519 verified sigs/s on MI355X (BASELINE.json metric).

A "step" is one pass of the verify hot path (expand -> prep -> dsm ->
reduce kernels) over one batch resident in HBM: BASELINE configs[1],
1,048,576 single-signature synthetic Solana transactions of 1232 bytes
(fd_benchg large_noop layout: 1167-byte signed message), all valid.
Each rank (one per GPU) verifies its own independent shard -- no
collective on the data path ("scaling": "weak"); the only collective is
the MAX over ranks of the timed interval.

Printed (rank 0, one JSON line): value = all ranks' signatures / max
rank time; roofline of the dominant kernel (fd_dsmh_kernel, the half-size walk: VALU integer,
priced in v_mad_u64_u32 multiply-accumulates against this device's own
measured v_mad_u64_u32 peak); cpu_baseline = the reference's AVX-512
fd_ed25519_verify (oracle/_ref, compiled from the reference sources) on
the host cores when the CPU has AVX-512 IFMA, else the oracle's portable C
restatement ("port").
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic work per signature: field ops of the
# reference algorithm, priced at 8x32-bit limb schoolbook products + the
# 2^256 = 38 fold: mul = 64+8, sqr = 36+8 32x32->64 multiply-accumulates.
MAC_PER_MUL, MAC_PER_SQR = 72, 44
DSM_MUL, DSM_SQR = 1341, 1008          # wNAF DSM (1008 S + 1339 M) + eq (2 M)
PREP_MUL, PREP_SQR = 38, 510           # decode of A and R: 2 x (255 S + 19 M)
DSM_MAC = DSM_MUL * MAC_PER_MUL + DSM_SQR * MAC_PER_SQR
# The half-size walk the engine runs by default (fd_gpu_lattice.h, fd_dsmh_kernel; bench.py with FDGPU_HALF=0 keeps
# the 252-doubling walk): 128 doublings (4 S + 3 M), 66 variable-base adds (A and R, 4 M + 4 M to
# extended), 16 base-point adds (3 M + 4 M), priced the same way.
HS_MUL, HS_SQR = 128 * 3 + 66 * 8 + 16 * 7, 128 * 4
HS_MAC = HS_MUL * MAC_PER_MUL + HS_SQR * MAC_PER_SQR
HALF = os.environ.get("FDGPU_HALF", "1") != "0"
# A/B: the largest batch that takes the unfolded (FM = 0, two waves per SIMD) throughput walk; -1 the engine's default
NOFOLD_MAX = int(os.environ.get("FDGPU_NOFOLD_MAX", "-1"))
WALK_MAC = HS_MAC if HALF else DSM_MAC
# MI355X_MICROARCH.md: 157.3 TF FP32 vector FMA = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz x 2 flops, i.e. a
# wave64 VALU instruction issues in 2 cycles per SIMD: 78.6 T lane-instructions/s for the whole chip
GUIDE_VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
# v_mad_u64_u32 is a half-rate instruction: 4.32 cycles per wave64 instruction per SIMD against 2.22 for
# v_fma_f32 / v_add_u32 (the guide's 2-cycle row) in the same probe (profiles/r03/ROOFLINE.md), so the
# guide's issue rate gives the MAC half the full-rate peak
GUIDE_MAD_PEAK = GUIDE_VALU_LANE_OPS / 2
PCIE_GBS = 63.0        # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s per direction (spec)
PCIE_DMA_GBS = 55.2    # hipMemcpyAsync H2D, measured (tools/gatherprobe, profiles/r02/stream/gather_probe.log)
PREP_MAC = PREP_MUL * MAC_PER_MUL + PREP_SQR * MAC_PER_SQR
# SHA-512 of R || A || M: ceil((msg_sz + 81) / 128) blocks of ~2.75K 64-bit operations, each two
# 32-bit VALU lane operations on CDNA4 -> priced against the full-rate VALU issue peak
SHA_BLOCK_OPS64 = 2750
# algorithmic bytes of a configs[1] signature over the whole path: R || S || A (96) + the 1167-byte message in, 1 out
ALGO_BYTES_PER_SIG = 96 + 1167 + 1


def roofline_per_kernel(nsig: int, ms_walk: float, ms_dec: float, ms_hash: float, pm: dict) -> dict:
    """The throughput path's three big kernels against their rooflines (all VALU issue-bound), with HIP-event
    times of this run and the work SURVEY §8(d) counts: the walk at its half-size work (HS_MAC) and at the
    reference DSM's (DSM_MAC); the decode kernel at the two decompressions (PREP_MAC; the -A / -R table
    additions on top are not priced); the hash kernel at SHA-512 (10 blocks for the 1167-byte message, two
    32-bit lane operations per 64-bit operation) against the full-rate issue peak.  Plus the per-signature
    tables' HBM traffic (PMC, profiles/dsm_pmc.json) against the path's algorithmic bytes."""
    blocks = -(-(1167 + 81) // 128)
    out = {}
    for name, ms, work, peak, unit in (("walk", ms_walk, WALK_MAC, GUIDE_MAD_PEAK, "v_mad_u64_u32"),
                                       ("walk_ref_equiv", ms_walk, DSM_MAC, GUIDE_MAD_PEAK, "v_mad_u64_u32"),
                                       ("decode", ms_dec, PREP_MAC, GUIDE_MAD_PEAK, "v_mad_u64_u32"),
                                       ("hash", ms_hash, blocks * SHA_BLOCK_OPS64 * 2, GUIDE_VALU_LANE_OPS, "32-bit lane op")):
        if ms and ms > 0:
            rate = work * nsig / (ms * 1e-3)
            out[name] = {"ms": round(ms, 4), "work_per_sig": work, "work_unit": unit, "achieved_t_per_s": round(rate / 1e12, 3),
                         "peak_t_per_s": round(peak / 1e12, 2), "frac": round(rate / peak, 4)}
    k = {"walk": pm.get("fd_dsmh_kernel<1>") or {}, "decode": pm.get("fd_decode_kernel") or {},
         "hash": pm.get("fd_hashh_kernel") or {}}
    for name, e in k.items():
        if name in out and e:
            out[name]["valu_insts_per_wave"] = e.get("valu_insts_per_wave")
            out[name]["valu_busy_flat4"] = round(e["valu_busy_flat4"], 4) if e.get("valu_busy_flat4") else None
    wr, rd = (k["decode"].get("hbm_write_bytes") or 0), (k["walk"].get("hbm_read_bytes") or 0)
    if wr and rd:
        per_sig = (wr + rd) / (1 << 20)
        out["table_traffic"] = {"decode_writes_gb_per_1m": round(wr / 1e9, 3), "walk_reads_gb_per_1m": round(rd / 1e9, 3),
                                "bytes_per_sig": round(per_sig), "algorithmic_bytes_per_sig": ALGO_BYTES_PER_SIG,
                                "vs_algorithmic": round(rd / (1 << 20) / ALGO_BYTES_PER_SIG, 2),
                                "source": "profiles/dsm_pmc.json (PMC FETCH_SIZE x2 / WRITE_SIZE, KiB, per 1M-sig launch)"}
    return out


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores() -> tuple[int, dict]:
    """Host cores this process may use: its affinity mask, capped by a cgroup CPU quota if one is set
    (the GPU box's share of a larger host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, {"affinity": aff, "cgroup_quota": quota}


def cpu_baseline(payload, desc, nsig_total, threads, target_s=1.5):
    """Time the reference (or the port) on a bounded prefix of the same workload, every signature verified
    once (fd_txn_verify's batch call; no separate per-signature pass)."""
    from oracle.oracle import Oracle, Reference, cpu_has_avx512_ifma
    kind, impl = "port", None
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libfdref_avx512.so")
    if os.path.exists(ref_path) and cpu_has_avx512_ifma():
        impl, kind = Reference("avx512"), "reference"
    else:
        impl = Oracle()

    def run(n, t):
        d = desc[:n]
        ns = int(d["sig_cnt"].astype(np.int64).sum())
        t0 = time.perf_counter()
        if kind == "reference":
            out, _ = impl.verify_txns(payload, d, ns, threads=t, want_sig_codes=False)
        else:
            out, _ = impl.verify_txns(payload, d, ns, threads=t)
        return time.perf_counter() - t0, ns, out
    # calibrate on a small prefix, then size the sample for ~target_s wall (~10-30 CPU-s)
    dt, ns, _ = run(min(len(desc), 2048 * threads), threads)
    rate = ns / dt
    n = int(min(len(desc), max(2048 * threads, rate * target_s)))
    dt, ns, out = run(n, threads)
    assert (out == 0).all(), "CPU baseline rejected valid signatures"
    return {"value": ns / dt, "unit": "sigs/s", "cores": threads, "kind": kind,
            "sample": f"first {n} txns ({ns} sigs) of the same 1232-byte workload, {threads} threads, "
                      f"{dt:.2f} s wall; host CPU: {cpu_model()}",
            "impl": "reference fd_ed25519_verify_batch_single_msg, AVX-512 r43x6 build (oracle/_ref)"
                    if kind == "reference" else "oracle/fd_ed25519_oracle.c portable C restatement"}, impl, kind


def cpu_sweep_configs0(impl, kind, max_threads, gen_threads, point_s=0.6):
    """BASELINE configs[0] on the host: 64K single-signature txns with 200-byte messages, all valid, the
    reference timed at 1, 2, 4, ... up to max_threads threads (SURVEY.md §6 measured 29.8K/s on 1 thread and
    211K/s on 8 of the survey box).  Each point is a bounded prefix sized to ~point_s of wall time."""
    from firedancer_amd import synth
    payload, desc, _, nsig = synth.make_batch(1 << 16, synth.SMALL_MSG, seed=77, threads=gen_threads)
    ts = sorted({t for t in (1, 2, 4, 8, 16, 32, 64, 128) if t <= max_threads} | {max_threads})
    pts = []
    for t in ts:
        n = min(len(desc), 512 * t)
        for _ in range(2):          # calibrate, then the sized run
            t0 = time.perf_counter()
            if kind == "reference":
                out, _ = impl.verify_txns(payload, desc[:n], n, threads=t, want_sig_codes=False)
            else:
                out, _ = impl.verify_txns(payload, desc[:n], n, threads=t)
            dt = time.perf_counter() - t0
            assert (out == 0).all()
            rate = n / dt
            n2 = int(min(len(desc), max(512 * t, rate * point_s)))
            if n2 <= n:
                break
            n = n2
        pts.append({"threads": t, "sigs_per_s": rate, "sigs": n})
    return {"workload": "BASELINE configs[0]: 65,536 single-sig txns, 200-byte messages, all valid",
            "points": pts}


# ---- host budget of the configs[4] stream at N GPUs -------------------------------------------------------
# Each GPU's stream child spins one thread per verify tile plus one per producer link (the reference pins
# every tile to a core of its own, src/app/fdctl/topology.c:167-170 sizes the verify stage by tile count).
# Every record also crosses host DRAM twice (the GPU's gather reads it, the write-back lands in the out
# dcache): ~34 GB/s each way per GPU at the measured 25.6M frags/s.
HOST_GBS_PER_GPU_EACH_WAY = 34.0


def _cpulist(path: str) -> set[int]:
    out = set()
    try:
        for part in open(path).read().strip().split(","):
            if part:
                a, _, b = part.partition("-")
                out.update(range(int(a), int(b or a) + 1))
    except (OSError, ValueError):
        pass
    return out


def host_topology(gpus: int = 8, sysfs_root: str = "/sys") -> tuple[dict, list]:
    """({NUMA node: usable physical cores (one hardware thread each, within this process's affinity)},
    [NUMA node of HIP devices 0..gpus-1, or -1]) from sysfs.  A device's node is that of its own PCI function,
    found as HIP numbers the devices -- the KFD topology's GPU nodes in order after ROCR_VISIBLE_DEVICES and
    HIP_VISIBLE_DEVICES (fdgpu_gpu_numa_node_sysfs, the same lookup the link's CPU choice makes) -- not the
    host's PCI order of every AMD GPU, which named the wrong node for a one-GPU job."""
    aff = os.sched_getaffinity(0)
    nodes = {}
    base = f"{sysfs_root}/devices/system/node"
    names = sorted(n for n in (os.listdir(base) if os.path.isdir(base) else []) if n.startswith("node") and n[4:].isdigit())
    for n in names:
        cpus = _cpulist(f"{base}/{n}/cpulist") & aff
        phys = {c for c in cpus
                if min(_cpulist(f"{sysfs_root}/devices/system/cpu/cpu{c}/topology/thread_siblings_list") & aff or {c}) == c}
        if phys:
            nodes[int(n[4:])] = len(phys)
    if not nodes:
        nodes = {0: len(aff)}
    try:
        from firedancer_amd import vtile
        gn = [vtile.gpu_numa_node(d, sysfs_root) for d in range(gpus)]
    except Exception:
        gn = []
    return nodes, [g for g in gn if g >= 0]


def host_plan(args, gpus: int, cores: int | None = None, nodes: dict | None = None,
              gpu_nodes: list | None = None) -> dict:
    """The host cores the configs[4] stream children of `gpus` GPUs need -- per GPU, its max-rate tiles or
    its paced tiles, plus its producers, each a spinning thread on a core of its own -- against what this
    job may use (affinity, cgroup quota, and per NUMA node: each child pins to its GPU's node first).  Where
    they do not fit, tiles per GPU are lowered (never below 1) instead of oversubscribing, and the plan says
    so.  cores / nodes / gpu_nodes override the probes (tests, --plan-cores)."""
    if cores is None:
        cores = usable_cores()[0] if not getattr(args, "plan_cores", 0) else int(args.plan_cores)
    if nodes is None:
        nodes, probed = host_topology(1 if os.environ.get("FDGPU_BENCH_ONE_DEVICE") == "1" else gpus)
        if getattr(args, "plan_cores", 0):
            nodes = {0: int(args.plan_cores)}
        gpu_nodes = probed if gpu_nodes is None else gpu_nodes
    nodes = {int(k): int(v) for k, v in nodes.items()}
    node_ids = sorted(nodes)
    gn = list(gpu_nodes or [])[:gpus]
    if os.environ.get("FDGPU_BENCH_ONE_DEVICE") == "1" and len(gn) == 1:   # (rehearsal: every rank on device 0)
        gn = gn * gpus
    if len(gn) < gpus or any(g not in nodes for g in gn):     # unknown placement: spread the GPUs over the nodes
        gn = [node_ids[i * len(node_ids) // gpus] for i in range(gpus)]
    P = args.stream_producers
    want_t, want_l = args.stream_tiles, args.stream_lat_tiles
    want_lc = 1 if getattr(args, "stream_lat_launcher", 0) else 0   # paced tiles' launch threads: a core each
    want_h = int(getattr(args, "stream_copy_threads", 0) or 0)      # max-rate tiles' host copy threads: a core each
    budget = max(1, cores // gpus)                          # the job's cores, an equal share per GPU
    per_node = {n: sum(1 for g in gn if g == n) for n in node_ids}
    node_budget = min(nodes[n] // per_node[n] for n in node_ids if per_node[n])
    b = min(budget, max(1, node_budget))
    h = want_h if b - P >= 1 + want_h else max(0, b - P - 1)    # copy threads only beside at least one tile
    tiles = min(want_t, max(1, (b - P) // (1 + h)))
    lc = want_lc if b - P >= 1 + want_lc else 0               # a launch thread only where a paced tile fits beside it
    lat_tiles = min(want_l, max(1, (b - P) // (1 + lc)))
    # served paced legs (--stream-svc-tiles): T tile processes + the verify service (+ its launch thread) per GPU
    want_s = max([int(x) for x in str(getattr(args, "stream_svc_tiles", "") or "").split(",") if x.strip()] or [0])
    svc_tiles = min(want_s, max(0, b - P - 1 - lc)) if want_s else 0
    need = gpus * (max(want_t * (1 + want_h), want_l * (1 + want_lc), want_s + 1 + want_lc if want_s else 0) + P)
    used = gpus * (max(tiles * (1 + h), lat_tiles * (1 + lc), svc_tiles + 1 + lc if svc_tiles else 0) + P)
    capped = tiles < want_t or lat_tiles < want_l or lc < want_lc or h < want_h or svc_tiles < want_s
    plan = {"gpus": gpus, "usable_cores": cores, "cores_per_numa_node": {str(k): v for k, v in nodes.items()},
            "gpu_numa_nodes": gn, "producers_per_gpu": P,
            "requested": {"tiles_per_gpu": want_t, "paced_tiles_per_gpu": want_l, "paced_launchers": want_lc,
                          "copy_threads_per_tile": want_h, "served_tiles_per_gpu": want_s, "cores": need},
            "applied": {"tiles_per_gpu": tiles, "paced_tiles_per_gpu": lat_tiles, "paced_launchers": lc,
                        "copy_threads_per_tile": h, "served_tiles_per_gpu": svc_tiles, "cores": used},
            "capped": capped, "oversubscribed": used > cores or b < 1 + P,
            "host_dram_gbs_est": round(gpus * 2 * HOST_GBS_PER_GPU_EACH_WAY, 1)}
    if capped:
        plan["cap"] = (f"{cores} usable cores ({min(budget, node_budget)} per GPU, {P} producer(s) each): tiles per GPU "
                       f"{want_t} -> {tiles}, paced {want_l} -> {lat_tiles}, paced launch threads {want_lc} -> {lc}, "
                       f"copy threads per tile {want_h} -> {h}, served tiles {want_s} -> {svc_tiles}")
    return plan


# ---- BASELINE configs[4]: the verify stage as the reference wires it ------------------------------------
# One producer link (mcache + in dcache) read by T = tiles_per_gpu x G verify tiles; tile i takes
# seq % T == i (before_frag, fd_verify_tile.c:47-48) and drives GPU i % G from that GPU's process.  With
# G > 1 the link lives in a /dev/shm file that rank 0's child creates and the other ranks' children join.

def stream_legs(args) -> list[str]:
    """cal, max, one paced leg per --stream-rates entry (frags/s per GPU), unrel (--stream-only-paced: the paced
    legs alone, e.g. under a kernel trace)"""
    if getattr(args, "stream_svc", 0):       # served: the paced legs (and, --stream-svc-max, the max rate first)
        return (["max"] if getattr(args, "stream_svc_max", 0) else []) + [f"paced@{r}" for r in _rates(args)]
    if getattr(args, "stream_only_paced", False):
        return [f"paced@{r}" for r in _rates(args)]
    return ["cal", "max"] + [f"paced@{r}" for r in _rates(args)] + ["unrel"]


def _rates(args) -> list[float]:
    return [float(x) for x in str(args.stream_rates).split(",") if x.strip()]


def _pow2_clamp(x: float, lo: int, hi: int) -> int:
    p = lo
    while p < x and p < hi:
        p *= 2
    return p


def _leg_cfg(args, leg, procs, cal_fps):
    # every tile and producer thread spins on its core: keep them within the host cores this job may
    # use (affinity and cgroup quota), split over the GPUs' processes
    plan = host_plan(args, procs)
    T = plan["applied"]["tiles_per_gpu"] * procs
    Tl = plan["applied"]["paced_tiles_per_gpu"] * procs
    Lc = plan["applied"]["paced_launchers"]
    H = plan["applied"]["copy_threads_per_tile"]
    # the max-rate legs batch for throughput (a GPU batch under one wave per SIMD costs about one wave's
    # DSM chain, ~1 ms, whatever its size), the paced leg for latency
    paced = leg.startswith("paced@")
    tput = leg in ("cal", "max")
    rate = float(leg.split("@")[1]) if paced else 0.0
    # paced legs: a batch limit of about 4 ms of one tile's share of the offered load (8K..64K), so batches
    # stay small at low load (latency path) and can grow with it; adaptive launch sizes them below that
    pb = _pow2_clamp(rate / max(1, args.stream_lat_tiles) * 4e-3, args.stream_batch, args.stream_max_batch)
    # NUMA placement of each producer's mcache, in dcache part and thread: its GPU's node (the process it runs in,
    # q % G), or (--stream-place opposite, the cross-socket arm) a node other than that GPU's
    gn = plan["gpu_numa_nodes"]
    nodes = sorted(int(k) for k in plan["cores_per_numa_node"])
    Qn = args.stream_producers * procs

    def pnode(q):
        g = gn[q % procs] if q % procs < len(gn) else None
        if args.stream_place == "none" or g is None:
            return None
        if args.stream_place == "opposite":
            return next((n for n in nodes if n != g), g)
        return g
    base = dict(prod_node=[pnode(q) for q in range(Qn)],
                batch_txn=args.stream_max_batch if not paced else pb,
                max_inflight=args.stream_inflight if not paced else args.stream_lat_inflight,
                zero_copy=not args.stream_copy, gpus=procs,
                producers=args.stream_producers * procs,   # the reference's QUIC tiles: producer q in process q % G
                # per link: its producer runs depth/2 ahead of the slowest tile; with one producer per GPU a
                # link carries 1/G of the frags but is read by all 2G tiles -> twice the single-GPU depth
                mcache_depth=args.stream_depth * min(procs, 2) if not paced else 1 << 18,
                nctx=args.stream_lat_ctx if paced else args.stream_ctx,
                # the reliable max-rate legs copy in bigger gathers (a gather's PCIe rate grows with its size,
                # tools/gatherprobe): ~20K records per gather (copy after 2 ms or 32K waiting frags, 128K
                # uncopied at most), max rate 25.7-25.8M vs 23.3-23.5M at ~2.6K (profiles/r04/gs); the paced and
                # the unreliable legs keep the tile's defaults (a later copy leaves a frag exposed to overruns
                # longer: unreliable goodput 17.0M vs 19.1M, profiles/r04/s)
                copy_wait_ns=int((args.stream_tput_copy_wait_us if tput else
                                  args.stream_lat_copy_wait_us if paced else args.stream_copy_wait_us) * 1000),
                gather_cus=args.stream_gather_cus,
                max_uncopied=args.stream_tput_max_uncopied if tput else args.stream_max_uncopied,
                copy_min=args.stream_tput_copy_min if tput else 0, prof=1 if args.stream_prof else 0, pf_dist=args.stream_pf_dist,
                no_huge_pages=1 if args.stream_no_huge else 0,
                cu_split=(args.stream_lat_cu_split if paced else args.stream_cu_split),
                cu_exclusive=args.stream_cu_exclusive,
                # paced legs: each tile's batch launches and copies on a launch thread of its own (the tile's
                # thread only queues them), when the host plan has the cores
                launcher=Lc if paced else 0,
                # max-rate and unreliable legs: host threads copy each record into the out dcache (the GPU copy only
                # reads it), so a record crosses PCIe once (--stream-copy-threads)
                copy_threads=0 if paced else H,
                # max-rate legs: a partial batch waits (up to 2 ms) until it holds --stream-tput-min-batch frags, so
                # it takes the throughput path (the latency path's 4-lane walk does twice the work per signature)
                min_batch=args.stream_tput_min_batch if tput else 0,
                # max-rate legs: batches above --stream-tput-small-max signatures take the throughput path
                small_max=args.stream_tput_small_max if tput else args.stream_lat_small_max if paced else 0,
                hk_ns=int(args.stream_lat_hk_us * 1000) if paced else 0,
                lat_share=args.stream_lat_share)
    if leg == "cal":
        return dict(base, tiles=T, n_frags=args.stream_frags if args.stream_frags > 0 else 2_000_000 * procs,
                    rate_fps=0.0, reliable=True)
    if leg == "max" and getattr(args, "stream_svc", 0):
        # served max rate: T tile processes per GPU and the verify service on the reliable link (credit-based),
        # with the max-rate legs' batching; sized for ~SVC_MAX_FPS_EST frags/s per GPU over --stream-seconds
        n = args.stream_frags if args.stream_frags > 0 else int(SVC_MAX_FPS_EST * procs * args.stream_seconds)
        # the service holds the engine contexts the one-process max leg's tiles hold together (tiles x contexts)
        return dict(base, tiles=args.stream_svc * procs, n_frags=n, rate_fps=0.0, reliable=True, svc=1,
                    nctx=min(3, args.stream_ctx * args.stream_tiles))
    if leg == "max":            # credit-based: the sustained rate with no frag lost
        n = args.stream_frags if args.stream_frags > 0 else int(1.2 * cal_fps * args.stream_seconds)
        return dict(base, tiles=T, n_frags=n, rate_fps=0.0, reliable=True)
    if paced and getattr(args, "stream_svc", 0):
        # served tiles: T verify-tile processes per GPU (no GPU context each), one verify service process per
        # GPU batching all of their frags -- at the same offered load per GPU as the one-process paced legs
        n = args.stream_frags if args.stream_frags > 0 else int(rate * procs * args.stream_paced_seconds)
        return dict(base, tiles=args.stream_svc * procs, n_frags=n, rate_fps=rate * procs, reliable=False, svc=1)
    if paced:                   # the reference's unreliable link at a fixed offered load (per GPU)
        n = args.stream_frags if args.stream_frags > 0 else int(rate * procs * args.stream_paced_seconds)
        return dict(base, tiles=Tl, n_frags=n, rate_fps=rate * procs, reliable=False)
    # unreliable, producer unthrottled: tiles that fall a lap behind are overrun and skip frags
    n = args.stream_frags if args.stream_frags > 0 else int(cal_fps * args.stream_unrel_seconds)
    return dict(base, tiles=T, n_frags=n, rate_fps=0.0, reliable=False)


KNEE_P99_US = 1000.0
SVC_MAX_FPS_EST = 30e6          # the served max-rate leg's frag count per GPU-second (its length, not a bound)


def knee_of(curve: list) -> float | None:
    """The highest offered rate (frags/s per GPU) such that it and every lower tried rate kept p99 within
    KNEE_P99_US with no frag lost and none overrun while copied; None if the lowest rate already fails."""
    knee = None
    for c in sorted(curve, key=lambda c: c["offered_frags_per_s_per_gpu"]):
        if c["p99_us"] > KNEE_P99_US or c["lost"] != 0 or c["overruns_at_verdict"] != 0:
            break
        knee = c["offered_frags_per_s_per_gpu"]
    return knee


def served_summary(args, raw: dict, knee_one_process) -> dict:
    """stream.served: per T tile processes per GPU (one verify service each GPU), the paced curve and knee next
    to the one-process knee (the same offered loads per GPU)."""
    out = {"def": "T verify-tile processes per GPU (fdgpu_tile: no GPU context) + one verify service process per GPU "
                  "batching all of their frags (fdgpu_vsvc_*); paced unreliable link, offered frags/s per GPU",
           "knee_one_process": knee_one_process, "by_tiles": {}}
    for T, r in raw.items():
        if "error" in r:
            out["by_tiles"][str(T)] = {"error": r["error"][-400:]}
            continue
        legs = r["legs"]
        curve = [dict(legs[f"paced@{x}"], offered_frags_per_s_per_gpu=x) for x in _rates(args)]
        mx = legs.get("max")
        out["by_tiles"][str(T)] = {
            "knee": knee_of(curve),
            # the reliable max-rate leg (--stream-svc-max): sigs/s of the GPU's T tile processes, every frag published
            "max": ({"sigs_per_s": mx["sigs_per_s"], "lost": mx["lost"], "published_all": mx["published"] == mx["frags"],
                     "tile_host_ns_per_frag": mx.get("tile_host_ns_per_frag"), "pcie": mx.get("pcie"),
                     "served": mx.get("served")} if mx else None),
            "paced_fps_p50_p99_us": [[c["offered_frags_per_s_per_gpu"], c["p50_us"], c["p99_us"]] for c in curve],
            "lost": [c["lost"] for c in curve], "overruns": [c["overruns_at_verdict"] for c in curve],
            "all_published": all(c["metrics"][:4] == [0, 0, 0, 0] for c in curve),
            "lost_frac": [round((c["lost"] + c["overruns_at_verdict"]) / max(c["frags"], 1), 3) for c in curve],
            "anomalies": anomaly_summary(r.get("anomalies"))[0],
            "dedup_recycled": dedup_recycled(r.get("anomalies")),
            "gpu_pauses_over_250us": [(c.get("gather_gpu") or {}).get("issue_to_start_over_250us") for c in curve],
            "mean_batch_txns": [round(c["mean_batch_txns"], 1) for c in curve],
            "served": [c.get("served") for c in curve],
            "curve": curve}
    return out


def _phases(ph) -> dict:
    n, ng = max(ph[0], 1), max(ph[8], 1)
    return {"batches": ph[0], "launch_to_kernels_mean": ph[1] / n * 1e-3, "launch_to_kernels_max": ph[2] * 1e-3,
            "kernels_mean": ph[3] / n * 1e-3, "kernels_max": ph[4] * 1e-3,
            "end_to_seen_mean": ph[5] / n * 1e-3, "end_to_seen_max": ph[6] * 1e-3,
            "launch_to_last_gather_end_mean": ph[7] / ng * 1e-3 if ph[8] else None}


def cpu_place(cpu: int) -> dict | None:
    """Where a CPU sits: its L3 group (the lowest CPU sharing its L3: one CCD on EPYC) and NUMA node, from sysfs."""
    if cpu is None or cpu < 0:
        return None
    l3 = _cpulist(f"/sys/devices/system/cpu/cpu{cpu}/cache/index3/shared_cpu_list")
    base = "/sys/devices/system/node"
    node = next((int(n[4:]) for n in (os.listdir(base) if os.path.isdir(base) else [])
                 if n.startswith("node") and n[4:].isdigit() and cpu in _cpulist(f"{base}/{n}/cpulist")), None)
    return {"cpu": cpu, "l3": min(l3) if l3 else None, "node": node}


def _pair_place(st: dict) -> dict:
    """Producer 0 and tile 0 (a paced leg's one link): their CPUs, and whether they share an L3 / a NUMA node --
    a frag's mcache line and record header cross from the producer's core to the tile's, each a coherence miss
    that costs more across L3 groups (the tile's intake ns per frag)."""
    pc = (st.get("prod_cpu") or [-1])[0]
    tc = (st.get("tile_cpu") or [-1])[0]
    p, t = cpu_place(pc), cpu_place(tc)
    same = (lambda k: (p[k] == t[k]) if p and t and p[k] is not None and t[k] is not None else None)
    return {"producer": p, "tile": t, "same_l3": same("l3"), "same_node": same("node")}


def _leg_summary(st: dict, cfg: dict) -> dict:
    n = max(st["verdicts"], 1)
    hist = st["gpu_lat_hist"]
    tot = sum(hist)

    def hq(q):   # GPU batch latency quantile: upper edge of the quarter-octave bucket (fdgpu_lat_bucket), us
        c = 0
        for i, h in enumerate(hist):
            c += h
            if tot and c > q * tot:
                return round(32.0 * 2 ** (i / 4), 1)
        return None
    return {"tiles": cfg["tiles"], "gpus": cfg["gpus"], "reliable": bool(cfg["reliable"]),
            "rate_fps": cfg["rate_fps"] or None, "frags": st["frags"], "verdicts": st["verdicts"],
            "lost": st["lost"], "overruns_at_verdict": st["overruns"],
            "lost_per_frag": st["lost"] / max(st["frags"], 1),
            "seconds": st["seconds"], "frags_per_s": st["frags_per_s"], "sigs_per_s": st["sigs_per_s"],
            "p50_us": st["lat_p50_us"], "p99_us": st["lat_p99_us"], "max_us": st["lat_max_us"],
            "published": st["published"], "metrics": st["metrics"],
            "tile_host_ns_per_frag": [round(x / n, 1) for x in st["tile_ns"]],
            "tile_after_split_ns_per_frag": {k: round(st[k] / n, 1) for k in ("gpu_wait_ns", "poll_ns", "after_ns", "launch_ns")},
            "tile_idle_ns_per_frag": round(st["tile_idle_ns"] / n, 1), "producer_seconds": st["prod_seconds"],
            "producer_credit_wait_s": st["prod_wait_ns"] * 1e-9,
            "batches": st["batches"], "mean_batch_txns": st["batch_txns"] / max(st["batches"], 1),
            "batch_limit": cfg["batch_txn"], "engine_contexts_per_tile": cfg["nctx"],
            # zero-copy intake: the GPU copies (the stem's during_frag copy, done by the GPU) started early
            "copies": st["copies"], "copy_lat_mean_us": st["copy_lat_ns_sum"] / max(st["copy_lat_n"], 1) * 1e-3,
            "copy_lat_max_us": st["copy_lat_ns_max"] * 1e-3,
            # every GPU copy on the GPU clock: host launch -> first block's start, start -> last block's end
            "gather_gpu": {"n": st["gather_gpu"][0],
                           "launch_to_start_mean_us": st["gather_gpu"][1] / max(st["gather_gpu"][0], 1) * 1e-3,
                           "launch_to_start_max_us": st["gather_gpu"][2] * 1e-3,
                           "run_mean_us": st["gather_gpu"][3] / max(st["gather_gpu"][0], 1) * 1e-3,
                           "run_max_us": st["gather_gpu"][4] * 1e-3,
                           # the runtime call that issued it (the launch thread's, after its queue) -> start
                           "issue_to_start_mean_us": st["gather_gpu"][5] / max(st["gather_gpu"][0], 1) * 1e-3,
                           "issue_to_start_max_us": st["gather_gpu"][6] * 1e-3,
                           "issue_to_start_over_250us": st["gather_gpu"][7]},
            # each batch's GPU time split (fdgpu_ed25519_phase_stats): launch -> its verify kernels start (its
            # gathers and the stream's earlier batch), kernels, end -> the tile saw it; launch -> last gather end
            "batch_phases_us": _phases(st["phase"]),
            "copy_backlog_refusals": st["copy_backlog"],
            # the host link at this leg's rate: each verdict's fd_txn_m_t record (80 + 1232 B) is read over PCIe
            # by the GPU copy and written back into the out dcache (plus its fd_txn_t image)
            # (with copy threads the record is not written back: only the fd_txn_t image and txn_t_sz go out)
            "pcie": {"record_bytes": 1312, "in_gbs": st["frags_per_s"] * 1312 / 1e9,
                     "out_gbs_at_least": st["frags_per_s"] * (0 if cfg.get("copy_threads") else 1312) / 1e9,
                     "peak_gbs_each_way": PCIE_GBS,
                     "frac_each_way": st["frags_per_s"] * 1312 / 1e9 / PCIE_GBS} if cfg.get("zero_copy") else None,
            # --stream-prof: rdtsc sections of the tile loop, ns per own frag (fdgpu_stream_stats_t.prof_ns)
            "tile_prof_ns_per_frag": (dict(zip(("mcache_poll", "during_frag", "prefetch_credit", "drain_after_frags",
                                                "hk_after_frags", "account", "credit", "housekeep"),
                                               [round(x / n, 1) for x in st["prof_ns"]]))
                                      if any(st["prof_ns"]) else None),
            "inflight_max": st["inflight_max"], "gpu_batch_lat_p50_us_le": hq(0.5),
            "gpu_batch_lat_p99_us_le": hq(0.99),
            # host contention: the spinning threads' CPU time over their wall time (1.0 = kept their cores),
            # involuntary context switches, and the CPUs the tiles were pinned to
            "host_cpu": {"tile_share": round(st["tile_cpu_ns"] / max(st["tile_wall_ns"], 1), 4),
                         "tile_share_min": round(st["tile_cpu_share_min"], 4), "tile_nivcsw": st["tile_nivcsw"],
                         "producer_share": round(st["prod_cpu_ns"] / max(st["prod_wall_ns"], 1), 4),
                         "producer_nivcsw": st["prod_nivcsw"],
                         "tile_cpus": [c for c in st["tile_cpu"][:min(cfg["tiles"], 8)]],
                         "producer_cpus": [c for c in (st.get("prod_cpu") or []) if c >= 0],
                         "producer_tile": _pair_place(st)},
            # the tiles' copy threads (cfg copy_threads): records copied, their ns per frag, overrun after the copy,
            # ns per frag the tile waited for a copy
            "host_copy": ({"records": st["host_copy"][0], "copy_ns_per_frag": round(st["host_copy"][1] / n, 1),
                           "overrun": st["host_copy"][2], "tile_wait_ns_per_frag": round(st["host_copy"][3] / n, 1)}
                          if cfg.get("copy_threads") else None),
            # the tiles' launch threads (cfg launcher): commands, their ns per frag, deepest queue, full-queue waits
            "launcher": ({"commands": st["launcher"][0], "busy_ns_per_frag": round(st["launcher"][1] / n, 1),
                          "depth_max": st["launcher"][2], "full_waits": st["launcher"][3],
                          "cmd_max_us": round(st["launcher"][4] * 1e-3, 1), "cmds_over_250us": st["launcher"][5]}
                         if cfg.get("launcher") else None)}


def _anon_huge_mb() -> float | None:
    """This process's memory in transparent huge pages (the link region's backing, when the kernel allows)."""
    try:
        for line in open("/proc/self/smaps_rollup"):
            if line.startswith("AnonHugePages:"):
                return int(line.split()[1]) / 1024.0
    except OSError:
        pass
    return None


def page_config() -> dict:
    """The host's page setup the links live on: transparent huge pages for anonymous memory (a one-process link)
    and for shared memory (/dev/shm: the link of several processes, the verify service's segment), and
    reserved hugetlb pages (none: shared memory is then in 4 KiB pages)."""
    def rd(p):
        try:
            return open(p).read().strip()
        except OSError:
            return None
    sel = lambda v: (v.split("[")[1].split("]")[0] if v and "[" in v else v)
    mounts = []
    try:
        mounts = [l.split()[1] for l in open("/proc/mounts") if l.split()[2:3] == ["hugetlbfs"]]
    except OSError:
        pass
    return {"thp": sel(rd("/sys/kernel/mm/transparent_hugepage/enabled")),
            "shmem_thp": sel(rd("/sys/kernel/mm/transparent_hugepage/shmem_enabled")),
            "hugetlb_pages": rd("/proc/sys/vm/nr_hugepages"), "hugetlbfs_mounts": mounts}


LINK_BYTES_PER_PAYLOAD = 1.1 * 1312      # a link's bytes per distinct payload (record + mcache line, measured map_mb)


def link_dir(choice: str, need_bytes: int, mounts_file: str = "/proc/mounts",
             sys_hp: str = "/sys/kernel/mm/hugepages") -> str:
    """Where a link of several processes lives.  "auto": a writable hugetlbfs mount whose huge pages have room for
    the link (the reference's workspaces live on fd_shmem's hugetlbfs mounts, src/util/shmem/fd_shmem_admin.c),
    else /dev/shm (4 KiB pages where shmem_enabled is never).  Every process of a run picks the same one (the
    same host state).  Any other value: that directory."""
    if choice != "auto":
        return choice
    try:
        mounts = [l.split() for l in open(mounts_file) if l.split()[2:3] == ["hugetlbfs"]]
    except OSError:
        mounts = []
    for m in mounts:
        d, opts = m[1], m[3].split(",")
        ps = next((o.split("=")[1] for o in opts if o.startswith("pagesize=")), "2M")
        kb = {"2M": 2048, "1G": 1048576, "2048k": 2048, "1048576k": 1048576}.get(ps, 2048)
        try:
            free = int(open(f"{sys_hp}/hugepages-{kb}kB/free_hugepages").read())
        except (OSError, ValueError):
            continue
        if free * kb * 1024 >= 1.25 * need_bytes and os.access(d, os.W_OK):
            return d
    return "/dev/shm"


def _kfd_gpu_ids() -> set[str]:
    """KFD gpu_ids of the GPUs this process sees (topology nodes with SIMDs)."""
    ids, base = set(), "/sys/class/kfd/kfd/topology/nodes"
    try:
        for n in os.listdir(base):
            try:
                props = open(f"{base}/{n}/properties").read()
                gid = open(f"{base}/{n}/gpu_id").read().strip()
            except OSError:
                continue
            if any(l.split()[:2] == ["simd_count", "0"] for l in props.splitlines()) or gid in ("", "0"):
                continue
            ids.add(gid)
    except OSError:
        pass
    return ids


def kfd_queues() -> dict | None:
    """The HSA user queues on this process's GPU(s) as KFD lists them (/sys/class/kfd/kfd/proc/<pid>/queues/
    <q>/gpuid; pids of every process on the node, in the host's pid space): how many, of how many processes,
    and the milliseconds those processes' queues have spent evicted (stats_<gpuid>/evicted_ms: KFD takes a
    process's queues off the GPU while it re-validates its memory, e.g. when the kernel invalidates pages of
    registered host memory).  A GPU maps at most num_cp_queues compute queues (24 on MI355X) at once."""
    base, gids = "/sys/class/kfd/kfd/proc", _kfd_gpu_ids()
    try:
        pids = os.listdir(base)
    except OSError:
        return None
    tot = procs = 0
    ev = 0.0
    for p in pids:
        try:
            qs = os.listdir(f"{base}/{p}/queues")
        except OSError:
            continue
        n = 0
        for q in qs:
            try:
                g = open(f"{base}/{p}/queues/{q}/gpuid").read().strip()
            except OSError:
                continue
            n += (not gids) or g in gids
        procs += n > 0
        tot += n
        for g in gids:
            try:
                ev += float(open(f"{base}/{p}/stats_{g}/evicted_ms").read().split()[0])
            except (OSError, ValueError, IndexError):
                pass
    return {"queues": tot, "procs": procs, "evicted_ms": ev}


class KfdSampler:
    """Samples kfd_queues() every 250 ms on a thread while a leg runs (the tile threads run in C, without the
    GIL); keeps the largest queue counts seen and the growth of the evicted time over the leg."""

    def __init__(self):
        import threading
        self.peak, self._first, self._stop = None, None, threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while True:
            stopped = self._stop.is_set()          # (one last sample after the leg)
            q = kfd_queues()
            if q is None:
                return
            if self._first is None:
                self._first = q
            self.peak = dict(queues=max(q["queues"], (self.peak or q)["queues"]),
                             procs=max(q["procs"], (self.peak or q)["procs"]),
                             evicted_ms=round(q["evicted_ms"] - self._first["evicted_ms"], 3))
            if stopped:
                return
            self._stop.wait(0.25)

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join(1.0)


def gpu_pause_log(reset: bool = True) -> dict | None:
    """The engine's GPU pause log (fdgpu_debug_gather_pauses, read through the tile library this process has
    loaded, without torch): copies held over 250 us on the GPU after their runtime call, grouped into episodes
    (events within 2 ms of each other): [start ms from the first, longest hold us, copies]."""
    import ctypes
    from firedancer_amd import vtile
    L = vtile.load()
    f = getattr(L, "fdgpu_debug_gather_pauses", None)
    if f is None:
        return None
    f.restype, f.argtypes = ctypes.c_ulong, [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int]
    buf = (ctypes.c_ulong * 1024)()
    tot = int(f(buf, 512, 1 if reset else 0))
    ev = sorted((buf[2 * i], buf[2 * i + 1]) for i in range(min(tot, 512)))
    eps = []
    for t, d in ev:
        if eps and t - eps[-1][3] <= 2_000_000:
            eps[-1][1] = max(eps[-1][1], d); eps[-1][2] += 1; eps[-1][3] = t
        else:
            eps.append([t, d, 1, t])
    t0 = eps[0][0] if eps else 0
    return {"copies": tot, "episodes": [[round((e[0] - t0) * 1e-6, 2), round(e[1] * 1e-3), e[2]] for e in eps[:40]]}


def stream_child_main(args) -> None:
    """--stream-child: the configs[4] legs for one process (one GPU); no torch GPU context here.  Process 0
    regenerates the payloads (same seed), creates each leg's link and runs the producer; the others join."""
    from firedancer_amd import vtile
    proc, procs, dev = args.stream_proc, args.stream_procs, args.stream_device
    out, cal_fps, anom = {}, 0.0, {}

    def anomalies(link, leg):
        # verdicts neither published nor overrun: in these all-valid streams every one is an anomaly
        # (and, apart, the dedups of payloads a tile had published before: the payloads recycle, so after a tile
        # lost most of its frags a tag can still be in its tcache -- correct drops, fdgpu_link_anomaly_results)
        n, first, by = 0, [], [0] * 8
        for t in vtile.tiles_of(int(link.cfg()["tiles"]), procs, proc):
            c, f = link.anomalies(t)
            n += c
            first += [dict(e, tile=t) for e in f]
            by = [a + b for a, b in zip(by, link.anomaly_results(t))]
        if n or by[0]:
            anom[leg] = {"count": n, "first": first[:8],
                         "by_result": {RESULT_NAMES[i]: c for i, c in enumerate(by) if c and i < len(RESULT_NAMES)}}
    wb = {"gather": 0, "none": 1, "finish": 2}[args.stream_writeback]
    if wb or args.stream_poll_prefetch or args.stream_gather_rpb or args.stream_gather_cu_spread or args.stream_quad_sha:
        from firedancer_amd import engine
        engine.debug_set_opts(gather_no_writeback=wb, poll_prefetch=args.stream_poll_prefetch,
                              gather_rpb=args.stream_gather_rpb, gather_cu_spread=args.stream_gather_cu_spread,
                              quad_sha=args.stream_quad_sha)
    payload = desc = None
    # distinct payloads: every tile's share must exceed its HA dedup depth (1 << 16), or each
    # payload's second round through the link would be dropped as a duplicate (correct dedup,
    # but then the legs would verify-and-drop instead of verify-and-publish)
    tiles = max(args.stream_tiles, args.stream_lat_tiles, args.stream_svc) * procs
    n_pay = max(args.txns, 2 * tiles * (1 << 16))
    ldir = link_dir(args.stream_link_dir, int(n_pay * LINK_BYTES_PER_PAYLOAD))
    if proc == 0:
        from firedancer_amd import synth
        payload, desc, _, _ = synth.make_batch(n_pay, synth.LARGE_NOOP, seed=args.stream_seed,
                                               threads=min(16, os.cpu_count() or 1))
    svc_stats = {}
    for leg in stream_legs(args):
        # (served tiles are processes of their own that join the link by its file)
        path = (f"{ldir}/fdgpu_link_{args.stream_token}_{leg.replace('@', '_')}"
                if procs > 1 or args.stream_svc else None)
        if proc == 0:
            cfg = _leg_cfg(args, leg, procs, cal_fps)
            link = vtile.Link(path, create=True, payload=payload, off=desc["payload_off"], sz=desc["payload_sz"], **cfg)
            huge_mb = _anon_huge_mb()
            place = dict(link.placement(), gpu_node=vtile.gpu_numa_node(dev), place=args.stream_place,
                         page_config=page_config(), link_dir=ldir if path else None)
            gpu_pause_log(reset=True)                 # (a fresh log for this leg)
            try:
                with KfdSampler() as kq:
                    rc = link.run(0, dev, True)
                    if rc:
                        raise RuntimeError(f"leg {leg}: fdgpu_link_run {rc}")
                    st = link.result(timeout_s=120.0)
                anomalies(link, leg)
                if args.stream_svc:
                    svc_stats[leg] = link.svc_stats()
            finally:
                link.close()
                if path and os.path.exists(path):
                    os.unlink(path)
            if leg == "cal":
                cal_fps = st["frags_per_s"]
            else:
                out[leg] = dict(_leg_summary(st, cfg), anon_huge_mb=huge_mb, kfd_queues_peak=kq.peak,
                                gpu_pauses=gpu_pause_log(reset=True), placement=place)
                if args.stream_svc:
                    sv = svc_stats[leg]
                    out[leg]["served"] = {"tile_processes": cfg["tiles"], "tiles_gpu_open": st["tiles_gpu_open"],
                                          "service_cpu": sv["cpu"], "mixed_batches": sv["mixed_batches"],
                                          "batches": sv["gm"]["batches"], "fault_completions": sv["fault_completions"],
                                          "service_busy_ns_per_frag": round(sv["busy_ns"] / max(sv["completed"], 1), 1),
                                          "service_loop_ns_per_frag": round(sv["loop_ns"] / max(sv["completed"], 1), 1)}
        else:
            link = vtile.Link(path, create=False, timeout_s=180.0 if leg == "cal" else 120.0)   # bounded if process 0 failed
            try:
                rc = link.run(proc, dev, True)          # its producers: q % G == proc
                anomalies(link, leg)
            finally:
                link.close()
            if rc:
                raise RuntimeError(f"leg {leg}: fdgpu_link_run {rc} (process {proc})")
    print(json.dumps({"legs": out, "cal_frags_per_s": cal_fps, "anomalies": anom}), flush=True)


def run_stream_child(args, dev, proc, procs, token) -> dict:
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--stream-child", "--stream-device", str(dev),
           "--stream-proc", str(proc), "--stream-procs", str(procs), "--stream-token", token,
           "--stream-seed", "1234", "--txns", str(args.txns), "--stream-frags", str(args.stream_frags),
           "--stream-seconds", str(args.stream_seconds), "--stream-unrel-seconds", str(args.stream_unrel_seconds),
           "--stream-tiles", str(args.stream_tiles), "--stream-batch", str(args.stream_batch),
           "--stream-max-batch", str(args.stream_max_batch),
           "--stream-lat-tiles", str(args.stream_lat_tiles),
           "--stream-inflight", str(args.stream_inflight), "--stream-depth", str(args.stream_depth),
           "--stream-lat-inflight", str(args.stream_lat_inflight), "--stream-producers", str(args.stream_producers),
           "--stream-ctx", str(args.stream_ctx), "--stream-lat-ctx", str(args.stream_lat_ctx),
           "--stream-rates", str(args.stream_rates), "--stream-paced-seconds", str(args.stream_paced_seconds),
           "--stream-copy-wait-us", str(args.stream_copy_wait_us), "--stream-gather-cus", str(args.stream_gather_cus),
           "--stream-tput-copy-wait-us", str(args.stream_tput_copy_wait_us),
           "--stream-tput-max-uncopied", str(args.stream_tput_max_uncopied),
           "--stream-tput-copy-min", str(args.stream_tput_copy_min),
           "--stream-lat-copy-wait-us", str(args.stream_lat_copy_wait_us),
           "--stream-max-uncopied", str(args.stream_max_uncopied), "--stream-pf-dist", str(args.stream_pf_dist),
           "--plan-cores", str(args.plan_cores)] + \
        (["--stream-prof"] if args.stream_prof else []) + (["--stream-no-huge"] if args.stream_no_huge else []) + \
        (["--stream-gather-rpb", str(args.stream_gather_rpb)] if args.stream_gather_rpb else []) + \
        (["--stream-gather-cu-spread", str(args.stream_gather_cu_spread)] if args.stream_gather_cu_spread else []) + \
        (["--stream-only-paced"] if args.stream_only_paced else []) + \
        ["--stream-cu-split", str(args.stream_cu_split), "--stream-lat-cu-split", str(args.stream_lat_cu_split),
         "--stream-cu-exclusive", str(args.stream_cu_exclusive), "--stream-lat-launcher", str(args.stream_lat_launcher),
         "--stream-copy-threads", str(args.stream_copy_threads),
         "--stream-tput-min-batch", str(args.stream_tput_min_batch),
         "--stream-tput-small-max", str(args.stream_tput_small_max), "--stream-lat-hk-us", str(args.stream_lat_hk_us),
         "--stream-lat-small-max", str(args.stream_lat_small_max), "--stream-quad-sha", str(args.stream_quad_sha),
         "--stream-lat-share", str(args.stream_lat_share), "--stream-svc", str(getattr(args, "stream_svc", 0)),
         "--stream-svc-max", str(getattr(args, "stream_svc_max", 0)),
         "--stream-place", args.stream_place, "--stream-link-dir", args.stream_link_dir]
    if args.stream_copy:
        cmd.append("--stream-copy")
    env = dict(os.environ)
    if args.stream_hw_queues:
        # HIP maps a process's streams onto at most GPU_MAX_HW_QUEUES hardware queues (default 4); streams beyond
        # that share a queue and serialise behind each other's packets (2 tiles x 2 contexts x 2 streams = 8)
        env["GPU_MAX_HW_QUEUES"] = str(args.stream_hw_queues)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode or not lines:
        raise RuntimeError(f"stream child rc={r.returncode}: {r.stderr[-1500:]}")
    return json.loads(lines[-1])


ROOF_STEPS = 3                 # steps of the roofline pass (per-kernel timing, one launch per kernel)
HEADLINE_MAX_BYTES = 4096      # the driver keeps the last ~8 KB of stdout: the headline line stays well inside


def _r(x, nd=4):
    """Round a float to nd significant digits (compact line); None / non-floats pass through."""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}")
    return x


PATH_NAMES = {8: "latency8", 4: "latency4", 2: "latency2", 1: "latency1", 0: "throughput", -1: "throughput_full",
              -2: "none"}


# fdgpu_link_anomaly_results' slots (FDGPU_VTILE_*): slot 0 (PUBLISH, never an anomaly) counts the dedups of
# payloads the tile had published before -- correct drops of the recycled synthetic payloads, not anomalies
RESULT_NAMES = ("dedup_recycled", "parse", "verify", "dedup", "bundle_peer", "overrun", "gpu_fault")


def dedup_recycled(anomalies: dict | None) -> int:
    """The correct dedups of recycled payloads over a stream's legs (not in the anomaly count)."""
    return sum(int((v.get("by_result") or {}).get("dedup_recycled", 0)) for v in (anomalies or {}).values())


def anomaly_summary(anomalies: dict | None) -> tuple[int, dict | None]:
    """(count, the first record) of a stream's anomalies (fdgpu_link_anomalies, merged per leg over ranks)."""
    n, first = 0, None
    for leg, v in (anomalies or {}).items():
        n += int(v.get("count", 0))
        if first is None and v.get("first"):
            first = dict(v["first"][0], leg=leg)
            if "path" in first:
                first["path"] = PATH_NAMES.get(first["path"], first["path"])
    return n, first


def compact_record(full: dict, detail_path: str | None) -> dict:
    """The one JSON line the driver parses (printed last on stdout, <= HEADLINE_MAX_BYTES): the BASELINE
    metric, its roofline and CPU baseline, and one-number summaries of the side measurements.  Everything
    else (stream legs, latency curve, sweeps, per-leg host splits) stays in `full`, written to detail_path."""
    rf = full.get("roofline") or {}
    cpu = full.get("cpu_baseline")
    rec = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    cfg = full.get("config") or {}
    rec["config"] = {k: cfg[k] for k in ("workload", "txns_per_gpu", "sigs_per_gpu", "signed_msg_bytes", "parallelism",
                                         "semantics", "contexts_per_gpu") if k in cfg}
    rec["results_ok"] = full.get("results_ok")
    rec["kernel_ms"] = {k: _r(v) for k, v in (full.get("kernel_ms") or {}).items()}
    rec["roofline"] = {
        "bound": rf.get("bound"), "kernel": rf.get("kernel"), "unit": rf.get("unit"),
        "achieved": _r(rf.get("achieved")),
        # peak / frac: MI355X_MICROARCH.md's VALU issue rate with v_mad_u64_u32 at half rate (39.3 T MAC/s)
        "peak": _r(rf.get("peak_guide")), "frac": _r(rf.get("frac_guide")),
        "peak_source": "guide: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / 2 (v_mad_u64_u32 half rate)",
        # the same achieved rate against this device's measured v_mad_u64_u32 peak at its sustained clock
        "peak_live": _r(rf.get("peak")), "frac_live": _r(rf.get("frac")),
        "frac_fullrate": _r(rf.get("frac_guide_fullrate")), "frac_ref_equiv": _r(rf.get("frac_ref_equiv")),
        "mac_per_sig": rf.get("mac_per_sig"), "valu_busy": _r(rf.get("valu_busy")),
        "traffic": rf.get("traffic"), "traffic_unit": "HBM bytes per 1M-sig launch (PMC, profiles/dsm_pmc.json)",
        "hbm_frac": _r((rf.get("hbm") or {}).get("frac")),
        # each big kernel's fraction of its roofline, same pricing, and the -A / -R tables' HBM
        # traffic against the path's algorithmic bytes
        "per_kernel_frac": {k: v.get("frac") for k, v in (rf.get("per_kernel") or {}).items() if "frac" in v},
        "table_traffic_vs_algorithmic": ((rf.get("per_kernel") or {}).get("table_traffic") or {}).get("vs_algorithmic"),
    }
    if cpu:
        sw = (cpu.get("sweep_configs0") or {}).get("points") or []
        rec["cpu_baseline"] = {"value": _r(cpu.get("value")), "unit": cpu.get("unit"), "cores": cpu.get("cores"),
                               "kind": cpu.get("kind"), "sample": cpu.get("sample"),
                               "configs0_sigs_per_s_by_threads": {str(p["threads"]): _r(p["sigs_per_s"], 3) for p in sw}}
    else:
        rec["cpu_baseline"] = None
    # per-GPU VALU utilisation (north star): [rank, sigs/s, frac of the guide peak, frac of the live peak]
    rec["per_gpu"] = [[g["rank"], _r(g["sigs_per_s"]), _r(g.get("frac_guide"), 3), _r(g.get("frac"), 3)]
                      for g in (full.get("per_gpu") or [])]
    rec["per_gpu_cols"] = ["rank", "sigs_per_s", "frac", "frac_live"]
    two = full.get("headline_two_contexts")
    rec["two_contexts_sigs_per_s"] = _r(two["sigs_per_s"]) if two else None
    lat = full.get("latency")
    if lat:
        rec["latency"] = {"batch_txns": lat["batch_txns"], "p50_ms": _r(lat["p50_ms"]), "p99_ms": _r(lat["p99_ms"]),
                          "device_p99_ms": _r(lat.get("device_p99_ms")), "pinned_p99_ms": _r(lat.get("pinned_p99_ms")),
                          "dropin_call_p99_us": _r(lat.get("dropin_call_p99_us"))}
    hs = full.get("host_staged")
    if hs:
        rec["host_staged_sigs_per_s"] = _r(hs["sigs_per_s"])
    ex = full.get("extra_configs")
    if ex:
        rec["extra_configs"] = {k.split("_")[0]: [_r(v["sigs_per_s"]), v["results_ok"]] for k, v in ex.items()}
    st = full.get("stream")
    if st:
        n_anom, first_anom = anomaly_summary(st.get("anomalies"))
        if "error" in st:
            rec["stream"] = {"error": str(st["error"])[-300:]}
            rec["stream_ok"] = False
        elif "only_paced" in st:
            rec["stream"] = {"only_paced": {k: [_r(v["p50_us"]), _r(v["p99_us"])] for k, v in st["only_paced"].items()},
                             "anomalies": n_anom, "anomaly_first": first_anom}
            rec["stream_ok"] = n_anom == 0
        else:
            curve = st.get("latency_curve") or []
            rec["stream"] = {
                "sigs_per_s": _r(st["sigs_per_s"]), "n_gpus": st["n_gpus"], "tiles_per_gpu": st["tiles_per_gpu"],
                "knee": (st.get("knee") or {}).get("frags_per_s_per_gpu"),
                "knee_def": "highest offered frags/s per GPU with p99 <= 1 ms and no frag lost",
                "paced_fps_p50_p99_us": [[_r(c["offered_frags_per_s_per_gpu"], 3), _r(c["p50_us"]), _r(c["p99_us"])]
                                         for c in curve],
                # per paced leg, the longest a GPU copy waited on the GPU after the runtime call that issued it
                # (a GPU-side pause holds every queue at once: DESIGN §12, the paced tail)
                "paced_gpu_pause_max_us": [_r((c.get("gather_gpu") or {}).get("issue_to_start_max_us"), 3)
                                           for c in curve],
                "paced_gpu_pauses_over_250us": [(c.get("gather_gpu") or {}).get("issue_to_start_over_250us")
                                                for c in curve],
                "p99_us": _r(curve[0]["p99_us"]) if curve else None,
                "unreliable_vs_max": _r(st.get("unreliable_goodput_vs_max"), 3),
                "tile_host_ns_per_frag": (st.get("max_rate") or {}).get("tile_host_ns_per_frag"),
                # per paced leg, the tile loop's intake ns per frag, and whether its producer shared the tile's L3
                # (a host that runs the intake at half speed laps the paced tile from 7.5M on: DESIGN §12)
                "paced_intake_ns_per_frag": [_r((c.get("tile_host_ns_per_frag") or [None])[0], 3) for c in curve],
                "paced_producer_tile_same_l3": [((c.get("host_cpu") or {}).get("producer_tile") or {}).get("same_l3")
                                                for c in curve],
                "all_published": st.get("all_published"),
                # where the max-rate leg's link memory was: the GPU's node, each producer's dcache part node, and the
                # link's bytes in 2 MiB pages / in all in the tile process (shared memory has no THP on shmem_thp never)
                "link_placement": {k: (st.get("max_rate") or {}).get("placement", {}).get(k)
                                   for k in ("place", "gpu_node", "dcache_nodes", "huge_mb", "map_mb")},
                "host_cpu_share_min": _r(st.get("host_cpu_share_min")),
                # verdicts neither published nor overrun (none expected in these all-valid streams), and the
                # first one with the GPU batch that produced it (leg, tile, ctx, seq, payload, code, path)
                "anomalies": n_anom, "anomaly_first": first_anom}
            rec["stream_ok"] = bool(st.get("all_published")) and n_anom == 0
        sv = st.get("served") if "error" not in st else None
        if sv:   # T tile processes per GPU served by one verify service: knee and p99 per offered rate
            rec["stream"]["served"] = {
                T: ({"error": v["error"][-200:]} if "error" in v else
                    {"knee": v["knee"], "p99_us": [_r(x[2]) for x in v["paced_fps_p50_p99_us"]],
                     **({"max_sigs_per_s": _r(v["max"]["sigs_per_s"])} if v.get("max") else {}),
                     "all_published": v["all_published"], "anomalies": v["anomalies"],
                     "tiles_gpu_open": sum((x or {}).get("tiles_gpu_open", 0) for x in v["served"])})
                for T, v in sv["by_tiles"].items()}
            rec["stream"]["served_knee_one_process"] = sv.get("knee_one_process")
    hp = full.get("host_plan")
    if hp:      # the configs[4] stream's host budget at this N (cores for its spinning tiles and producers)
        rec["host_plan"] = {"usable_cores": hp["usable_cores"], "need_cores": hp["requested"]["cores"],
                            "used_cores": hp["applied"]["cores"], "tiles_per_gpu": hp["applied"]["tiles_per_gpu"],
                            "paced_tiles_per_gpu": hp["applied"]["paced_tiles_per_gpu"],
                            "paced_launchers": hp["applied"]["paced_launchers"], "capped": hp["capped"],
                            "oversubscribed": hp["oversubscribed"], "host_dram_gbs_est": hp["host_dram_gbs_est"]}
        if hp.get("cap"):
            rec["host_plan"]["cap"] = hp["cap"]
    rec["detail"] = detail_path
    return rec


def emit_record(full: dict, detail_path: str | None) -> str:
    """Write the full record to detail_path (best effort) and return the compact headline line."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(full, f, indent=1)
        except OSError:
            detail_path = None
    line = json.dumps(compact_record(full, detail_path), separators=(",", ":"))
    if len(line) > HEADLINE_MAX_BYTES:       # never again an unparseable line: drop the side summaries first
        rec = compact_record(full, detail_path)
        st = rec.get("stream") if isinstance(rec.get("stream"), dict) else {}
        # the stream's diagnostics first (all in the detail file), then whole side summaries
        drops = [(st, k) for k in ("knee_def", "paced_producer_tile_same_l3", "paced_intake_ns_per_frag",
                                   "paced_gpu_pause_max_us", "tile_host_ns_per_frag", "link_placement",
                                   "host_cpu_share_min", "anomaly_first")] + \
                [(rec, k) for k in ("extra_configs", "latency", "per_gpu", "stream")]
        for d, k in drops:
            d.pop(k, None)
            line = json.dumps(rec, separators=(",", ":"))
            if len(line) <= HEADLINE_MAX_BYTES:
                break
    return line


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _stdout_to_stderr:
    """fd 1 -> fd 2 for the block (C++ libraries' prints, e.g. gloo's "[Gloo] Rank r is connected ..." at
    init_process_group, which torchrun passes through on the ranks' shared stdout)."""
    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def launch_ranks(n: int, argv: list[str], script: str | None = None, timeout_s: float = 3000.0) -> int:
    """`bench.py --gpus N` without torchrun: start N rank processes of this script, one per GPU, with the
    torch.distributed env (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), as the
    reference starts N verify tiles (src/app/fdctl/topology.c:167-170).  This process never touches the GPU.
    Rank 0's stdout is the bench line.  A rank that fails takes the others down (they would wait in a
    barrier forever); the exit code is the first failure's."""
    import subprocess
    port = _free_port()
    script = script or os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # only rank 0's stdout is the bench's: the other ranks' (gloo's connection notes, ...) go to stderr
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env, stdout=None if r == 0 else sys.stderr))
    t0, rc = time.time(), 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or time.time() - t0 > timeout_s:
            rc = bad[0] if bad else 124
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return rc
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.2)


def rank_env(gpus: int | None):
    """(rank, world, local_rank) from the launcher's / torchrun's env; --gpus N must equal the world size."""
    from firedancer_amd import shard
    env = shard.dist_env()
    if gpus is not None and env.world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={env.world}")
    return env.rank, env.world, env.local_rank


def dry_run_main(args) -> None:
    """--dry-run (CPU test of the launcher and the record): every GPU leg replaced by a stub of known
    duration; the same rank env, gloo reductions, per-GPU rows and compact line as the real run."""
    import torch.distributed as dist
    from firedancer_amd import shard
    rank, world, _ = rank_env(args.gpus)
    if world > 1:
        with _stdout_to_stderr():
            dist.init_process_group("gloo")
    dd = dist if world > 1 else None
    nsig = args.txns

    def step():
        time.sleep(0.002 * (rank + 1))
    dt = shard.timed_steps(step, args.steps, args.warmup, lambda: None, (lambda: dist.barrier()) if world > 1 else (lambda: None))
    dt_max, ok = shard.reduce_max_min(dd, dt, True, "cpu")
    rows = shard.gather_rows(dd, [rank, 1.0, 1.0, 0.5 * GUIDE_MAD_PEAK, GUIDE_MAD_PEAK, dt], "cpu")
    if rank == 0:
        full = {"metric": "dry-run", "value": shard.aggregate_rate(world, nsig, args.steps, dt_max), "unit": "sigs/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt_max * 1e3 / args.steps,
                "results_ok": ok, "roofline": {"bound": "valu", "frac_guide": 0.5, "peak_guide": GUIDE_MAD_PEAK / 1e9},
                "per_gpu": [{"rank": int(r[0]), "sigs_per_s": nsig * args.steps / r[5], "frac_guide": r[3] / r[4],
                             "frac": r[3] / r[4]} for r in rows],
                "host_plan": host_plan(args, world)}
        print(emit_record(full, args.detail_out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); without torchrun's env, bench.py starts the N ranks itself")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where the full record goes (stream legs, latency curve, sweeps); the stdout line is compact")
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--plan-cores", type=int, default=0,
                    help="(planning) host cores to budget the configs[4] stream children against instead of this "
                         "job's usable cores (e.g. --gpus 8 --dry-run --plan-cores 16)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--txns", type=int, default=1 << 20, help="txns per GPU per step (BASELINE configs[1]: 1M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipe", type=int, default=1,
                    help="engine contexts (each on its own stream) that consecutive headline steps alternate over")
    ap.add_argument("--latency-batch", type=int, default=8192)
    ap.add_argument("--stream-frags", type=int, default=-1,
                    help="BASELINE configs[4]: frags per stream leg (0 = skip the stream; default: sized to "
                         "--stream-seconds from a short calibration leg)")
    ap.add_argument("--stream-seconds", type=float, default=10.0,
                    help="sustained length of the reliable max-rate leg and of the paced leg")
    ap.add_argument("--stream-unrel-seconds", type=float, default=4.0,
                    help="frags of the unreliable unthrottled leg, in seconds of the calibrated rate")
    ap.add_argument("--stream-tiles", type=int, default=2,
                    help="verify tiles per GPU of the max-rate legs (profiles/r02/stream/sweep_depth.md: at depth 2^20 "
                         "2 tiles 16.2-17.6M, 3 tiles 15-17.3M, 4 tiles 13.1-16.1M, 6 tiles 12.4-14.1M sigs/s)")
    ap.add_argument("--stream-copy", action="store_true",
                    help="stream tiles copy each frag into the out dcache on the host (the reference tile's "
                         "during_frag) instead of the zero-copy intake (GPU gathers from the registered in dcache)")
    ap.add_argument("--stream-batch", type=int, default=8192, help="GPU batch (txns) of the paced latency leg")
    ap.add_argument("--stream-max-batch", type=int, default=65536,
                    help="GPU batch limit (txns) of the max-rate legs (profiles/r02/stream: batches of 8192 give "
                         "7.2M, of up to 32768 13.7M sigs/s on 2 tiles)")
    ap.add_argument("--stream-inflight", type=int, default=2,
                    help="batches a tile's engine context keeps launched before housekeeping launches its filling "
                         "one (a full batch launches regardless); 2: 17.5M vs 16.8M sigs/s at 1 on 2 tiles "
                         "(profiles/r02/stream/sweep_depth.md)")
    ap.add_argument("--stream-producers", type=int, default=1,
                    help="producer links (the reference's QUIC tiles) per GPU; every tile reads every link")
    ap.add_argument("--stream-ctx", type=int, default=1,
                    help="engine contexts per verify tile on the max-rate and unreliable legs (FDGPU_VTILE_CTX; "
                         "1 beat 2 by 2.5-5.6 %% in 4 interleaved pairs, profiles/r02/stream/sweep_ctx_per_tile.md)")
    ap.add_argument("--stream-lat-ctx", type=int, default=2,
                    help="engine contexts per verify tile on the paced leg (staggered batches: one stages while "
                         "the other runs)")
    ap.add_argument("--stream-lat-inflight", type=int, default=1,
                    help="--stream-inflight of the paced leg (1: few, larger batches; 2 gave p50/p99 0.82/1.53 ms "
                         "against 0.72/1.02 ms at 1, with 277-txn mean batches)")
    ap.add_argument("--stream-depth", type=int, default=1 << 20,
                    help="mcache lines of the max-rate legs' link: a reliable producer runs depth/2 ahead of the "
                         "oldest frag a tile still holds, so the depth bounds the frags in flight (2^18: 13.8M, "
                         "2^20: 16-17.6M sigs/s on 2 tiles, profiles/r02/stream/sweep_depth.log)")
    ap.add_argument("--stream-rates", default="2e6,5e6,7.5e6,10e6,12.5e6,15e6",
                    help="paced legs (the latency-under-load curve): offered frags/s per GPU, comma separated; "
                         "stream.knee = the highest whose p99 is <= 1 ms with no frag lost")
    ap.add_argument("--stream-paced-seconds", type=float, default=3.0, help="length of each paced leg")
    ap.add_argument("--stream-gather-cus", type=int, default=16,
                    help="zero-copy intake: CUs each tile's engine contexts reserve for the copies (fdgpu_vtile_opts_t; "
                         "16 vs 0 on 2 tiles: max 21.6M vs 18.7M sigs/s, paced 10M/s p99 2.0 vs 4.6 ms, "
                         "profiles/r03/stream_tiles)")
    ap.add_argument("--stream-first", action="store_true",
                    help="run the configs[4] stream legs before the headline, before this process initialises the GPU")
    ap.add_argument("--stream-gather-rpb", type=int, default=0,
                    help="(stream child, A/B) records per gather workgroup (fdgpu_debug_opts_t.gather_rpb; 0 = default 4)")
    ap.add_argument("--stream-no-huge", action="store_true",
                    help="(A/B) the link region in 4 KiB pages instead of transparent huge pages")
    ap.add_argument("--stream-gather-cu-spread", type=int, default=0, choices=(0, 1, 2),
                    help="(stream child, A/B) the CUs each tile context reserves for its gathers: 0 the last n, "
                         "1 every (CUs/n)-th, 2 the first n (fdgpu_debug_opts_t.gather_cu_spread)")
    ap.add_argument("--stream-prof", action="store_true",
                    help="rdtsc section profile of the tile loop (fdgpu_stream_cfg_t.prof), in each leg's summary")
    ap.add_argument("--stream-max-uncopied", type=int, default=0,
                    help="paced / unreliable legs, zero-copy intake: frags a tile may hold whose GPU copy has not completed (fdgpu_vtile_opts_t."
                         "max_uncopied; 0 = its default)")
    ap.add_argument("--stream-poll-prefetch", type=int, default=0,
                    help="(stream child only, A/B) software prefetch distance of the tiles' completion polls "
                         "(fdgpu_debug_opts_t.poll_prefetch; 0 = none)")
    ap.add_argument("--stream-pf-dist", type=int, default=0,
                    help="tile loop prefetch distance in own frags (fdgpu_stream_cfg_t.pf_dist; 0 = its default)")
    ap.add_argument("--stream-writeback", choices=("gather", "finish", "none"), default="gather",
                    help="(stream child only) who writes a gathered record into the out dcache: the gather kernel as it "
                         "copies (default), the batch's finish kernel (A/B), or nobody (DIAGNOSTIC: published records lack "
                         "their payload -- what the write-back costs; never a result)")
    ap.add_argument("--stream-copy-wait-us", type=float, default=0.0,
                    help="unreliable legs, zero-copy intake: a tile starts the GPU copy of the frags it took once the oldest has "
                         "waited this long (0 = fdgpu_vtile default, FDGPU_VTILE_COPY_WAIT_NS)")
    ap.add_argument("--stream-tput-copy-wait-us", type=float, default=2000.0,
                    help="reliable max-rate legs (cal, max): --stream-copy-wait-us of their tiles (bigger gathers)")
    ap.add_argument("--stream-tput-max-uncopied", type=int, default=131072,
                    help="reliable max-rate legs (cal, max): --stream-max-uncopied of their tiles")
    ap.add_argument("--stream-lat-copy-wait-us", type=float, default=25.0,
                    help="paced legs: --stream-copy-wait-us of their tile (25 us: p99 at 10M frags/s 0.91 ms against "
                         "0.92-0.95 at the tile's default 50 us, profiles/r04/pcw)")
    ap.add_argument("--stream-tput-copy-min", type=int, default=32768,
                    help="reliable max-rate legs (cal, max): a tile starts a copy once this many frags wait "
                         "(fdgpu_vtile_opts_t.copy_min; 0 = the tile's default, 4,096)")
    ap.add_argument("--stream-lat-tiles", type=int, default=1,
                    help="verify tiles per GPU of the paced legs (fewer tiles = fewer HIP streams sharing the "
                         "device: 1 tile x 2 contexts p99 0.81 / 0.99 / 1.37 ms at 2 / 5 / 10M frags/s against "
                         "1.09 / 1.16 / 1.61 with 2 tiles, profiles/r03/stream_fused)")
    ap.add_argument("--stream-cu-split", type=int, default=0, choices=(0, 1),
                    help="max-rate legs: each tile's engine contexts on disjoint CU shares (fdgpu_vtile_opts_t.cu_split)")
    ap.add_argument("--stream-lat-cu-split", type=int, default=0, choices=(0, 1),
                    help="paced legs: each tile's engine contexts on disjoint CU shares (fdgpu_vtile_opts_t.cu_split)")
    ap.add_argument("--stream-cu-exclusive", type=int, default=0, choices=(-1, 0, 1, 2, 3, 4),
                    help="every leg: latency-path workgroups alone on their CU (fdgpu_vtile_opts_t.cu_exclusive; "
                         "0 = the tile's default, on; -1 off; A/B: 2 at most two per CU, 3 the walk only, 4 the prep "
                         "only; profiles/r04/p, q)")
    ap.add_argument("--stream-lat-share", type=int, default=0,
                    help="every leg: each engine context's exclusive latency-path walk fits 1/n of the CUs left by the "
                         "gathers (fdgpu_vtile_opts_t.lat_share; 0 = the tile's default, 1/contexts; -1 = no limit, A/B)")
    ap.add_argument("--stream-lat-launcher", type=int, default=1, choices=(0, 1),
                    help="paced legs: each tile's batch launches and copies on a launch thread of its own, a core "
                         "each (fdgpu_vtile_opts_t.launcher; the host plan drops it when the cores are short).  On by "
                         "default: p99 neutral (profiles/r05/lc, hk), but it takes ~15 ns per frag of runtime calls "
                         "off the single paced tile, which at 10M frags/s has no other headroom; 1 tile + 1 launch "
                         "thread + 1 producer is the max-rate legs' 3 cores per GPU")
    ap.add_argument("--stream-tput-min-batch", type=int, default=0,
                    help="max-rate legs: batches wait (up to 2 ms) for at least this many frags (fdgpu_vtile_opts_t."
                         "min_batch; 0 = launch when the GPU has room)")
    ap.add_argument("--stream-tput-small-max", type=int, default=0,
                    help="max-rate legs: batches of at most this many signatures take the latency path "
                         "(fdgpu_vtile_opts_t.small_max; 0 = the tile's default, half the batch limit)")
    ap.add_argument("--stream-quad-sha", type=int, default=0, choices=(-1, 0),
                    help="A/B: -1 = the latency path's hash role on one lane per signature instead of a quad "
                         "(fdgpu_debug_opts_t.quad_sha; engine test hook)")
    ap.add_argument("--stream-lat-small-max", type=int, default=0,
                    help="paced legs: batches of at most this many signatures take the latency path (fdgpu_vtile_opts_t."
                         "small_max; 0 = the tile's default, half the batch limit)")
    ap.add_argument("--stream-lat-hk-us", type=float, default=2.5,
                    help="paced legs: the tile loop's housekeeping (launch decision, copies, verdict poll) at most "
                         "every this many us while frags flow (0 = the link's 10 us; 2.5: verdicts seen ~5 us "
                         "sooner, p99 at 10M 0.889 / 0.889 vs 0.897 / 0.938 ms, profiles/r05/hk)")
    ap.add_argument("--stream-copy-threads", type=int, default=0, choices=range(0, 9),
                    help="max-rate and unreliable legs: host threads per tile that copy each record into the out dcache "
                         "while the GPU copy only reads it (fdgpu_vtile_opts_t.copy_threads; a core each in the host plan)")
    ap.add_argument("--stream-svc-tiles", default="2",
                    help="served paced legs: for each T in this comma list, T verify-tile processes per GPU (the fdgpu_tile "
                         "program, no GPU context each) served by one verify service process per GPU (fdgpu_vsvc_*), at "
                         "the --stream-rates offered loads per GPU; stream.served[T] holds the curve and knee (empty: skip)")
    ap.add_argument("--stream-svc", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--stream-svc-max", type=int, default=0, choices=(0, 1),
                    help="served legs: also a reliable max-rate leg with the T tile processes (stream.served[T].max)")
    ap.add_argument("--stream-place", choices=("gpu", "opposite", "none"), default="gpu",
                    help="NUMA node of each producer's mcache, in dcache part and thread: its GPU's (default), the node "
                         "opposite its GPU (the cross-socket arm), or unplaced (first touch by the link's creator)")
    ap.add_argument("--stream-link-dir", default="/dev/shm",
                    help="directory of the link file of several processes (N > 1, served legs); auto = a writable "
                         "hugetlbfs mount with free huge pages for it (2 MiB pages, as the reference's workspaces), "
                         "else /dev/shm.  Not the default: no GPU box here has a hugetlbfs mount with pages, so the "
                         "hugetlbfs path has not run on hardware")
    ap.add_argument("--stream-only-paced", action="store_true",
                    help="(diagnostic) run only the paced legs (no stream summary line: max_rate is absent)")
    ap.add_argument("--stream-hw-queues", type=int, default=0, choices=range(0, 17), metavar="0..16",
                    help="GPU_MAX_HW_QUEUES of the tile processes (0 = the runtime's default, 4): hardware queues "
                         "their HIP streams are spread over")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the BASELINE configs[0,2,3] side measurements (small / adversarial / multi-sig)")
    ap.add_argument("--stream-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stream-device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--stream-proc", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--stream-procs", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--stream-token", default="x", help=argparse.SUPPRESS)
    ap.add_argument("--stream-seed", type=int, default=1234, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.stream_child:
        stream_child_main(args)
        return
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.dry_run:
        dry_run_main(args)
        return

    import torch
    import torch.distributed as dist
    from firedancer_amd import Engine, load_library, shard, synth

    rank, world, local_rank = rank_env(args.gpus)
    # rehearsal knob for the N>1 flow on a one-GPU box: FDGPU_BENCH_ONE_DEVICE=1 puts every rank on GPU 0
    dev = 0 if os.environ.get("FDGPU_BENCH_ONE_DEVICE") == "1" else local_rank
    # The data path has no collective (independent shards); the measurement reductions (MAX of time, MIN of
    # the results flag, SUM of signatures) are a few scalars, so they go over gloo on CPU tensors: no RCCL.
    if world > 1:
        with _stdout_to_stderr():       # gloo's connection notes: stdout carries only rank 0's bench line
            dist.init_process_group("gloo")
    dd = dist if world > 1 else None

    def barrier():
        if world > 1:
            dist.barrier()

    def stream_section():
        """BASELINE configs[4] on every rank (its tile process), merged on rank 0; None elsewhere."""
        stream = None
        barrier()
        token = f"{os.getpid()}_{int(time.time())}" if rank == 0 else ""
        if world > 1:
            obj = [token]
            dist.broadcast_object_list(obj, src=0)
            token = obj[0]
        res, err = None, None
        kq0 = kfd_queues()            # the queues already open on the node when the tile processes start
        try:
            res = run_stream_child(args, dev, rank, world, token)
        except Exception as e:      # keep the headline line even if the stream leg fails
            err = str(e)[-2000:]
        # served paced legs (--stream-svc-tiles): T tile processes + one verify service process per GPU, a fresh
        # stream child per T, every rank in step
        served_raw = {}
        svc_max = host_plan(args, world)["applied"]["served_tiles_per_gpu"]
        for T in [int(x) for x in str(args.stream_svc_tiles).split(",") if x.strip() and int(x) <= svc_max]:
            a2 = argparse.Namespace(**vars(args))
            a2.stream_svc = T
            try:
                served_raw[T] = run_stream_child(a2, dev, rank, world, f"{token}_s{T}")
            except Exception as e:
                served_raw[T] = {"error": str(e)[-1500:]}
            barrier()
        # every rank takes part in the same collectives, whatever happened locally
        _, stream_ok = shard.reduce_max_min(dd, 0.0, err is None, "cpu")
        mine = (res or {}).get("anomalies", {})
        all_anom = [mine]
        if world > 1:
            all_anom = [None] * world
            dist.all_gather_object(all_anom, mine)
        anomalies = {}
        for r, a in enumerate(all_anom):
            for leg, v in (a or {}).items():
                m = anomalies.setdefault(leg, {"count": 0, "first": []})
                m["count"] += v["count"]
                for k, c in (v.get("by_result") or {}).items():
                    m.setdefault("by_result", {})[k] = m.get("by_result", {}).get(k, 0) + c
                m["first"] = (m["first"] + [dict(e, rank=r) for e in v["first"]])[:8]
        if rank == 0:
            if res is not None and stream_ok and args.stream_only_paced:
                stream = {"only_paced": dict(res["legs"]), "anomalies": anomalies}
            elif res is not None and stream_ok:
                legs = res["legs"]
                mx, ur = legs["max"], legs["unrel"]
                curve = [dict(legs[f"paced@{r}"], offered_frags_per_s_per_gpu=r) for r in _rates(args)]
                pc = curve[0]
                ok_s = (mx["metrics"][:4] == [0, 0, 0, 0] and mx["published"] == mx["frags"] and mx["lost"] == 0
                        and all(c["metrics"][:4] == [0, 0, 0, 0] for c in curve))
                # the knee: the highest offered rate whose p99 (tsorig -> verdict) stays within 1 ms with
                # every frag verified (none lost to overruns, none overrun while copied)
                # every rate up to the knee must hold the bound (a curve that fails at a lower rate and passes
                # at a higher one has its knee below the failure)
                knee = {"frags_per_s_per_gpu": knee_of(curve), "p99_bound_us": KNEE_P99_US, "rates_tried": _rates(args)}
                stream = {"workload": "BASELINE configs[4]: 1232-byte txns, Q producer mcache links over one in dcache "
                                      "-> T verify tiles reading every link (seq % T round robin per link, tile i -> "
                                      "GPU i % G; device fd_txn_parse + verify, in-order after_frag, dedup tcache) -> "
                                      "out dcache",
                          "sigs_per_s": mx["sigs_per_s"], "per_gpu_sigs_per_s": mx["sigs_per_s"] / world,
                          "n_gpus": world, "tiles_per_gpu": mx["tiles"] // world, "batch_max": args.stream_max_batch,
                          "batch_paced": pc["batch_limit"],
                          "max_inflight": args.stream_inflight, "max_inflight_paced": args.stream_lat_inflight,
                          "link_depth": args.stream_depth * min(world, 2),
                          "producers": args.stream_producers * world,
                          "engine_contexts_per_tile": args.stream_ctx, "engine_contexts_per_tile_paced": args.stream_lat_ctx,
                          "tiles_per_gpu_paced": args.stream_lat_tiles, "hw_queues": args.stream_hw_queues or 4,
                          "process": "one tile process per GPU without a torch GPU context (as a C verify tile); "
                                     "link in /dev/shm when G > 1",
                          "intake": "zero-copy (GPU gathers frags from the registered in dcache)"
                                    if not args.stream_copy else "host copy into the out dcache (reference during_frag)",
                          "max_rate": mx, "paced": pc, "latency_curve": curve, "knee": knee, "unreliable_max": ur,
                          # goodput of the reference's own link mode under overload, against the reliable max rate
                          "unreliable_goodput_vs_max": ur["sigs_per_s"] / mx["sigs_per_s"] if mx["sigs_per_s"] else None,
                          "all_published": bool(ok_s),
                          # verdicts neither published nor overrun, per leg (fdgpu_link_anomalies): none expected
                          "anomalies": anomalies,
                          # the lowest share of wall time any leg's tile thread kept its core (a shared host
                          # that steals it inflates that leg's latency tail; 1.0 = undisturbed)
                          "host_cpu_share_min": min((l.get("host_cpu") or {}).get("tile_share_min", 1.0)
                                                    for l in [mx, ur] + curve),
                          "latency_def": "producer mcache publish (tsorig) -> after_frag verdict on the host",
                          "kfd_queues_before": kq0, "pages": page_config()}
            else:
                stream = {"error": err or "a stream child failed on another rank"}
            if served_raw:
                k1 = (stream.get("knee") or {}).get("frags_per_s_per_gpu")
                if "only_paced" in stream:      # the one-process knee over the same offered rates
                    k1 = knee_of([dict(stream["only_paced"][f"paced@{r}"], offered_frags_per_s_per_gpu=r)
                                  for r in _rates(args)])
                stream["served"] = served_summary(args, served_raw, k1)

        return stream


    # --stream-first: the configs[4] legs before this process touches the GPU (its HIP context, queues and
    # torch's allocations then do not exist yet while the tile processes run)
    stream = stream_section() if args.stream_frags != 0 and args.stream_first else None
    torch.cuda.set_device(dev)

    n = args.txns
    gen_threads = min(16, os.cpu_count() or 1)
    t_gen = time.time()
    payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, seed=shard.shard_seed(1234, rank),
                                                   threads=gen_threads)
    t_gen = time.time() - t_gen

    pay_d = torch.from_numpy(payload).cuda()
    desc_d = torch.from_numpy(desc.view(np.uint8)).cuda()
    out_d = torch.empty(n, dtype=torch.int8, device="cuda")
    if not HALF or NOFOLD_MAX >= 0:   # A/B: the full-length walk / the unfolded walk's batch limit (the
        from firedancer_amd import engine as _engine   # engine's explicit test hook, not an env read)
        _engine.debug_set_opts(half=1 if HALF else 0, nofold_max=NOFOLD_MAX)
    eng = Engine(device=dev, max_txn=n, max_sig=nsig)
    st = torch.cuda.current_stream().cuda_stream
    # --pipe P: consecutive steps alternate over P engine contexts, each on its own stream, so one batch's
    # prep can fill the SIMDs its predecessor's walk leaves idle in its last partial round of waves
    pipe = [(eng, st, out_d)]
    for _ in range(1, args.pipe):
        pipe.append((Engine(device=dev, max_txn=n, max_sig=nsig), torch.cuda.Stream().cuda_stream,
                     torch.empty(n, dtype=torch.int8, device="cuda")))
    step_i = [0]

    def step():
        e, s, o = pipe[step_i[0] % len(pipe)]
        step_i[0] += 1
        e.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, o.data_ptr(), None, s)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dt = shard.timed_steps(step, args.steps, 0, torch.cuda.synchronize, barrier)
    ok = all(bool(np.array_equal(o.cpu().numpy(), expect)) for _, _, o in pipe)

    # the roofline pass: a few more steps of the same batch with per-kernel HIP events on the launch stream
    # (the headline steps above run without event records between their kernels)
    eng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, out_d.data_ptr(), None, st)
    torch.cuda.synchronize()
    eng.set_timing(True)
    for _ in range(ROOF_STEPS):
        eng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, out_d.data_ptr(), None, st)
    torch.cuda.synchronize()
    ms_prep, ms_dsm, ms_red = eng.kernel_ms(0), eng.kernel_ms(1), eng.kernel_ms(2)
    ms_dec, ms_hash = eng.kernel_ms(3), eng.kernel_ms(4)    # the prep's two kernels (throughput path)
    eng.set_timing(False)
    ok = ok and bool(np.array_equal(out_d.cpu().numpy(), expect))
    # the same steps alternating over two contexts / streams (one batch's prep overlaps the other's walk
    # tail): the engine's best whole-job rate on this workload.  Reported beside `value`, which stays the
    # one-context rate so that the roofline's per-launch kernel times are not stretched by the overlap
    # (A/B: 104.4-104.8M vs 101.0-101.2M, profiles/r03/pipe_ab.log)
    pipelined = None
    if args.pipe == 1 and not args.no_extra_configs:
        e2 = Engine(device=dev, max_txn=n, max_sig=nsig)
        p2 = [(eng, st, out_d), (e2, torch.cuda.Stream().cuda_stream, torch.empty(n, dtype=torch.int8, device="cuda"))]
        k2 = [0]

        def step2():
            e, s, o = p2[k2[0] % 2]
            k2[0] += 1
            e.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, o.data_ptr(), None, s)
        for _ in range(2):
            step2()
        dt2 = shard.timed_steps(step2, args.steps, 0, torch.cuda.synchronize, barrier)
        ok2 = all(bool(np.array_equal(o.cpu().numpy(), expect)) for _, _, o in p2)
        dt2_max, ok2 = shard.reduce_max_min(dd, dt2, ok2, "cpu")
        pipelined = {"sigs_per_s": shard.aggregate_rate(world, nsig, args.steps, dt2_max),
                     "ms_per_step": dt2_max * 1e3 / args.steps, "contexts_per_gpu": 2, "results_ok": ok2}
        e2.close()
    for e, _, _ in pipe[1:]:
        e.close()
    dt_max, all_ok = shard.reduce_max_min(dd, dt, ok, "cpu")

    # BASELINE configs[0] / [2] / [3] on the same device path, rank 0 only:
    # throughput with HBM-resident input plus a check of every result code
    # against the generator's intended code (the GPU parity tests pin those
    # workloads against the oracle and the reference)
    extra = None
    if rank == 0 and not args.no_extra_configs:
        extra = {}
        for name, kind, nt, ms, inv in (("configs0_small_msg_200B", synth.SMALL_MSG, 1 << 16, 1, 0.0),
                                        ("configs2_adversarial_10pct", synth.LARGE_NOOP, 1 << 20, 1, 0.1),
                                        ("configs3_multisig_1to12", synth.MULTI, 1 << 18, 12, 0.1)):
            xp, xd, xe, xn = synth.make_batch(nt, kind, ms, inv, seed=shard.shard_seed(4321, rank), threads=gen_threads)
            xe_d = Engine(device=dev, max_txn=nt, max_sig=xn)
            xpd = torch.from_numpy(xp).cuda()
            xdd = torch.from_numpy(xd.view(np.uint8)).cuda()
            xo = torch.empty(nt, dtype=torch.int8, device="cuda")

            def xstep():
                xe_d.verify_txns_device(xpd.data_ptr(), xdd.data_ptr(), nt, xn, xo.data_ptr(), None, st)
            xstep(); torch.cuda.synchronize()
            xk = max(3, (1 << 20) // nt)          # ~1M signatures' worth of launches: 16 for configs[0]'s 64K
            # warm the clock first (a short kernel train right after another config runs slow), then the
            # median of 3 timed trains
            xdt = sorted(shard.timed_steps(xstep, xk, xk, torch.cuda.synchronize, lambda: None)
                         for _ in range(3))[1]
            xok = bool(np.array_equal(xo.cpu().numpy(), xe))
            xe_d.close()
            codes = {int(c): int(k) for c, k in zip(*np.unique(xe, return_counts=True))}
            extra[name] = {"sigs_per_s": xn * xk / xdt, "txns": nt, "sigs": xn, "launches": xk, "results_ok": xok,
                           "txn_codes": codes}
            del xpd, xdd, xo

    lat = None
    if rank == 0 and args.latency_batch > 0:
        # p99 batch latency: host-staged batches (H2D + kernels + D2H), submit -> verdict
        lb = min(args.latency_batch, n)
        lpay = payload[: int(desc["payload_off"][lb - 1]) + 1232 + 64]
        leng = Engine(device=dev, max_txn=lb, max_sig=lb, max_payload=lpay.nbytes)
        ld = desc[:lb].copy()
        leng.verify_txns_host(lpay, ld, want_sig_codes=False)
        times = []
        for _ in range(1000):          # p99 of 1000 calls: the 10th-worst, not one host hiccup
            t1 = time.perf_counter()
            lo, _ = leng.verify_txns_host(lpay, ld, want_sig_codes=False)
            times.append((time.perf_counter() - t1) * 1e3)
            assert (lo == 0).all()
        # the same batch already resident in HBM: kernels only (launch -> stream idle)
        lo_d = torch.empty(lb, dtype=torch.int8, device="cuda")
        dtimes = []
        for _ in range(1000):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            leng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), lb, lb, lo_d.data_ptr(), None, st)
            torch.cuda.synchronize()
            dtimes.append((time.perf_counter() - t1) * 1e3)
        assert (lo_d.cpu().numpy() == 0).all()
        # the same batch from a pinned (registered) host buffer, as a tile's dcache is: direct DMA, no staging copy
        from firedancer_amd import engine as _engine
        ppay = np.array(lpay, copy=True)
        _engine.host_register(ppay)
        ptimes = []
        try:
            leng.verify_txns_host(ppay, ld, want_sig_codes=False)
            for _ in range(1000):
                t1 = time.perf_counter()
                lo, _ = leng.verify_txns_host(ppay, ld, want_sig_codes=False)
                ptimes.append((time.perf_counter() - t1) * 1e3)
                assert (lo == 0).all()
        finally:
            _engine.host_unregister(ppay)
        leng.close()
        lat = {"batch_txns": lb, "p50_ms": float(np.percentile(times, 50)), "p99_ms": float(np.percentile(times, 99)),
               "path": "fdgpu_ed25519_verify_txns_host: pinned staging in 1-MB chunks overlapped with H2D, "
                       "latency path (one fused launch: decode A + -A table / decode R + -R table / hash + half-size "
                       "scalars; half-size walk on four lanes per signature; reduce), D2H",
               "device_p50_ms": float(np.percentile(dtimes, 50)), "device_p99_ms": float(np.percentile(dtimes, 99)),
               "device_path": "same batch resident in HBM: kernels only, launch -> stream idle",
               "pinned_p50_ms": float(np.percentile(ptimes, 50)), "pinned_p99_ms": float(np.percentile(ptimes, 99)),
               "pinned_path": "same call with the payload in a registered (pinned) host buffer, as a tile's dcache: "
                              "one direct H2D DMA, no staging copy",
               "samples": len(times)}

    # configs[1] from host memory: the whole 1M-txn batch handed over in a pinned host buffer each step
    # (chunked H2D on a copy stream overlapped with the kernels, fdgpu_ed25519_verify_txns_host) --
    # the PCIe-inclusive rate, next to the HBM-resident headline
    host_staged = None
    if rank == 0 and not args.no_extra_configs:
        from firedancer_amd import engine as _engine
        heng = Engine(device=dev, max_txn=n, max_sig=nsig, max_payload=payload.nbytes)
        hpay = np.array(payload, copy=True)
        _engine.host_register(hpay)
        try:
            heng.verify_txns_host(hpay, desc, want_sig_codes=False)
            hts = []
            for _ in range(5):
                t1 = time.perf_counter()
                ho, _ = heng.verify_txns_host(hpay, desc, want_sig_codes=False)
                hts.append(time.perf_counter() - t1)
            hok = bool(np.array_equal(ho, expect))
        finally:
            _engine.host_unregister(hpay)
        heng.close()
        hgbs = payload.nbytes / float(np.median(hts)) / 1e9
        host_staged = {"sigs_per_s": nsig / float(np.median(hts)), "ms_per_batch": 1e3 * float(np.median(hts)),
                       "batch_txns": n, "bytes_per_batch": int(payload.nbytes), "results_ok": hok,
                       # the host -> device link: the batch's payload bytes over the step's wall time
                       "roofline": {"bound": "pcie", "achieved": hgbs, "peak": PCIE_GBS, "unit": "GB/s",
                                    "frac": hgbs / PCIE_GBS, "dma_measured_peak": PCIE_DMA_GBS,
                                    "frac_of_dma_peak": hgbs / PCIE_DMA_GBS,
                                    "peak_source": "MI355X_MICROARCH.md host link: PCIe Gen5 x16, 63 GB/s (spec); "
                                                   "dma_measured_peak: hipMemcpyAsync H2D of 32K records, "
                                                   "profiles/r02/stream/gather_probe.log"},
                       "path": "payload in a registered (pinned) host buffer -> H2D in 1-MB chunks on a copy stream, "
                               "kernels on the compute stream, verdicts D2H; synchronous per batch"}

    eng.close()     # the headline context's stream is idle from here: free it before the tiles open theirs
    # BASELINE configs[4]: the same 1232-byte payloads through the verify stage as the reference wires it
    # (one producer link, T = tiles x G verify tiles, tile i -> GPU i % G), in a child process per GPU that
    # never initialises torch's GPU context: a verify tile is a plain C process, and torch's context in this
    # one measurably inflates the tiles' tail latency (tools/stream_seq.py, TORCH=1: paced p99 1.2 -> 2.2 ms).
    stream = stream_section() if args.stream_frags != 0 and not args.stream_first else stream
    if lat is not None:
        # after the stream leg: the drop-in's process-wide context (and its stream) lives until exit
        # the link-level drop-in: one synchronous fd_ed25519_verify call (one signature, one GPU round trip)
        from firedancer_amd import engine as _engine
        d0 = desc[0]
        b0 = payload[int(d0["payload_off"]): int(d0["payload_off"]) + int(d0["payload_sz"])].tobytes()
        so, ao, mo = int(d0["signature_off"]), int(d0["acct_addr_off"]), int(d0["message_off"])
        sig0, pub0, msg0 = b0[so:so + 64], b0[ao:ao + 32], b0[mo:]
        assert _engine.fd_ed25519_verify(msg0, sig0, pub0) == 0
        ctimes = []
        for _ in range(200):
            t1 = time.perf_counter()
            rc0 = _engine.fd_ed25519_verify(msg0, sig0, pub0)
            ctimes.append((time.perf_counter() - t1) * 1e6)
            assert rc0 == 0
        lat.update({"dropin_call_p50_us": float(np.percentile(ctimes, 50)),
                    "dropin_call_p99_us": float(np.percentile(ctimes, 99)),
                    "dropin_path": "fd_ed25519_verify (link-level drop-in, fd_ed25519.h:96-101): one 1167-byte "
                                   "message, one synchronous GPU round trip per call"})
    # per-GPU VALU utilisation (north star): every rank prices its own DSM launches against its own
    # measured v_mad_u64_u32 peak; rank 0 reports the list
    L = load_library()
    L.fdgpu_mad_peak_per_s.restype = ctypes.c_double
    L.fdgpu_mad_peak_per_s.argtypes = [ctypes.c_int]
    my_peak = max(float(L.fdgpu_mad_peak_per_s(dev)) for _ in range(3))
    my_ach = WALK_MAC * nsig / (ms_dsm * 1e-3)
    rows = shard.gather_rows(dd, [rank, ms_dsm, ms_prep, my_ach, my_peak, dt], "cpu")
    per_gpu = [{"rank": int(r[0]), "dsm_ms": r[1], "prep_ms": r[2], "achieved_gmac_s": r[3] / 1e9,
                "peak_gmac_s": r[4] / 1e9, "frac": r[3] / r[4] if r[4] > 0 else None,
                "frac_guide": r[3] / GUIDE_MAD_PEAK if r[3] > 0 else None,
                "sigs_per_s": nsig * args.steps / r[5]} for r in rows]

    if rank == 0:
        peak = my_peak
        dom_ms = ms_dsm
        achieved = WALK_MAC * nsig / (dom_ms * 1e-3)
        ref_equiv = DSM_MAC * nsig / (dom_ms * 1e-3)     # the reference algorithm's work at this rate
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "dsm_pmc.json")
        valu_busy, pm_k = None, {}
        if os.path.exists(pmc):
            try:
                pm = json.load(open(pmc))
                traffic, valu_busy, pm_k = pm.get("hbm_bytes_per_launch"), pm.get("valu_busy"), pm.get("per_kernel") or {}
            except Exception:
                traffic = None
        per_kernel = roofline_per_kernel(nsig, ms_dsm, ms_dec, ms_hash, pm_k)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cores, core_src = usable_cores()
            cpu, impl, kind = cpu_baseline(payload, desc, nsig, threads=cores)
            cpu["cores_source"] = dict(core_src, used=cores)
            cpu["sweep_configs0"] = cpu_sweep_configs0(impl, kind, cores, gen_threads)
        value = shard.aggregate_rate(world, nsig, args.steps, dt_max)
        rec = {
            "metric": "ed25519 verified sigs/sec at 1/8 MI355X vs host AVX-512; p99 batch latency",
            "value": value,
            "unit": "sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (fd_benchg large_noop layout, seeded ed25519 keys/signatures)",
            "config": {"workload": "BASELINE configs[1]: 1M single-sig 1232-byte synthetic Solana txns, all valid",
                       "txns_per_gpu": n, "sigs_per_gpu": nsig, "signed_msg_bytes": 1167,
                       "parallelism": f"independent per-GPU shards x{world}", "semantics": "avx512",
                       "contexts_per_gpu": args.pipe},
            "results_ok": all_ok,
            "kernel_ms": {"prep": ms_prep, "dsm": ms_dsm, "reduce": ms_red, "decode": ms_dec, "hash": ms_hash,
                          "source": f"roofline pass: {ROOF_STEPS} more steps of the same batch, HIP events"},
            "roofline": {"bound": "valu", "achieved": achieved / 1e9, "peak": peak / 1e9, "unit": "GMAC/s",
                         "frac": achieved / peak if peak > 0 else None, "traffic": traffic,
                         # rocprof name of the 1M launch (carry-fold instantiation)
                         "kernel": "fd_dsmh_kernel<1>" if HALF else "fd_dsm_kernel<1>",
                         "mac_per_sig": WALK_MAC,
                         "work_per_sig": (f"{HS_MAC} v_mad_u64_u32 ({HS_SQR} S + {HS_MUL} M of the half-size walk: "
                                          f"128 doublings, 66 variable + 16 base-point adds; S=44 M=72 MAC)" if HALF else
                                          f"{DSM_MAC} v_mad_u64_u32 (1008 S + 1341 M of the reference wNAF DSM, "
                                          f"S=44 M=72 MAC)"),
                         # the reference's own DSM work (SURVEY §8d, 1008 S + 1341 M) over the same time: what
                         # this walk is worth in the reference algorithm's terms (not a hardware efficiency)
                         "achieved_ref_equiv": ref_equiv / 1e9,
                         "frac_ref_equiv": ref_equiv / peak if peak > 0 else None,
                         "peak_source": "fdgpu_mad_peak_per_s: measured v_mad_u64_u32 throughput of this device at "
                                        "its sustained clock (8 waves/SIMD, 16 chains; max of 3)",
                         # the same achieved rate against MI355X_MICROARCH.md's VALU issue rate: 2 cycles per
                         # full-rate wave64 instruction (78.6 T lane-ops/s at 2.4 GHz), and v_mad_u64_u32 measured
                         # at twice that cost -> 39.3 T MAC/s
                         "peak_guide": GUIDE_MAD_PEAK / 1e9,
                         "frac_guide": achieved / GUIDE_MAD_PEAK,
                         "peak_guide_source": "MI355X_MICROARCH.md: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T "
                                              "full-rate lane-ops/s; v_mad_u64_u32 is half rate (4.32 vs 2.22 cycles per "
                                              "wave-instruction, tools/instprobe/instprobe2 + PMC clock) -> 39.3 T MAC/s; "
                                              "profiles/r03/ROOFLINE.md",
                         "frac_guide_fullrate": achieved / GUIDE_VALU_LANE_OPS,
                         "valu_busy": valu_busy,
                         "valu_busy_source": "profiles/dsm_pmc.json: issue cycles of the walk kernel's ISA priced at "
                                             "the measured per-instruction costs (tools/dsm_issue_model.py, "
                                             "profiles/r03/roofline/issue_model_dsmh_r03c.json, every row measured) / measured kernel cycles",
                         # the same kernel against the HBM roofline: PMC bytes per launch / this run's launch time
                         "hbm": ({"achieved": traffic * nsig / (1 << 20) / (dom_ms * 1e-3) / 1e9, "peak": 8000.0,
                                  "unit": "GB/s",
                                  "frac": traffic * nsig / (1 << 20) / (dom_ms * 1e-3) / 8e12,
                                  "note": "PMC bytes (FETCH_SIZE x1024 x2 + WRITE_SIZE x1024) per 1M-sig launch, scaled "
                                          "to this launch: the walk reads each signature's -A / -R tables, which the "
                                          "decode kernel wrote to HBM (per-signature tables: 2.3 GB per 1M does not fit "
                                          "the 256 MB MALL; only the B tables stay L2/MALL-resident).  Not the bound "
                                          "(frac ~0.2): the walk is VALU issue-bound"}
                                 if traffic else None),
                         # each big kernel of the step against its roofline, priced as SURVEY §8(d) prices it, and
                         # the -A / -R tables' traffic against the algorithmic bytes
                         "per_kernel": per_kernel},
            "cpu_baseline": cpu,
            "per_gpu": per_gpu,
            "latency": lat,
            "host_staged": host_staged,
            "stream": stream,
            "host_plan": host_plan(args, world) if args.stream_frags != 0 else None,
            "extra_configs": extra,
            "headline_two_contexts": pipelined,
            "gen_s": t_gen,
        }
        print(emit_record(rec, args.detail_out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
