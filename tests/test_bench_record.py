"""CPU: bench.py's driver contract -- the compact headline line (<= 4 KB, last on stdout, the keys the
driver reads) built from a canned full record of the size round 3's grew to, and `--gpus N` starting N
ranks itself (gloo on CPU, GPU legs stubbed by --dry-run)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _leg(rate):
    return {"tiles": 2, "gpus": 8, "reliable": False, "rate_fps": rate, "frags": 10 ** 8, "verdicts": 10 ** 8, "lost": 0,
            "overruns_at_verdict": 0, "p50_us": 512.123456, "p99_us": 812.987654, "max_us": 1999.1,
            "published": 10 ** 8, "metrics": [0, 0, 0, 0, 10 ** 8], "tile_host_ns_per_frag": [30.8, 46.7, 10.9, 92.3],
            "sigs_per_s": rate, "frags_per_s": rate, "batch_limit": 8192, "offered_frags_per_s_per_gpu": rate,
            "gather_gpu": {"n": 90000, "issue_to_start_max_us": 850.123456, "issue_to_start_over_250us": 3},
            "padding": "x" * 1500}


def canned_full(n_gpus=8):
    curve = [_leg(r) for r in (2e6, 5e6, 7.5e6, 10e6, 15e6)]
    return {
        "metric": "ed25519 verified sigs/sec at 1/8 MI355X vs host AVX-512; p99 batch latency",
        "value": 8.3e8, "unit": "sigs/s", "n_gpus": n_gpus, "steps": 20, "warmup": 5, "ms_per_step": 10.1,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (fd_benchg large_noop layout, seeded ed25519 keys/signatures)",
        "config": {"workload": "BASELINE configs[1]: 1M single-sig 1232-byte synthetic Solana txns, all valid",
                   "txns_per_gpu": 1 << 20, "sigs_per_gpu": 1 << 20, "signed_msg_bytes": 1167,
                   "parallelism": "independent per-GPU shards x8", "semantics": "avx512", "contexts_per_gpu": 1},
        "results_ok": True, "kernel_ms": {"prep": 3.9123456, "dsm": 6.7298765, "reduce": 0.05},
        "roofline": {"bound": "valu", "achieved": 15000.123, "peak": 31400.0, "unit": "GMAC/s", "frac": 0.4777,
                     "traffic": 10.1e9, "kernel": "fd_dsmh_kernel<1>", "mac_per_sig": 96256,
                     "frac_ref_equiv": 0.56, "peak_guide": 39321.6, "frac_guide": 0.3815,
                     "frac_guide_fullrate": 0.19, "valu_busy": 0.99, "work_per_sig": "y" * 300,
                     "hbm": {"frac": 0.2}},
        "cpu_baseline": {"value": 900457.2, "unit": "sigs/s", "cores": 16, "kind": "reference",
                         "sample": "first 1048576 txns (1048576 sigs) of the same 1232-byte workload, 16 threads, "
                                   "1.16 s wall; host CPU: AMD EPYC 9575F 64-Core Processor",
                         "sweep_configs0": {"points": [{"threads": t, "sigs_per_s": 59000.0 * t, "sigs": 65536}
                                                       for t in (1, 2, 4, 8, 16)]}},
        "per_gpu": [{"rank": r, "dsm_ms": 6.7, "prep_ms": 3.9, "achieved_gmac_s": 15000.0, "peak_gmac_s": 31400.0,
                     "frac": 0.4777123, "frac_guide": 0.3815123, "sigs_per_s": 1.04e8} for r in range(n_gpus)],
        "latency": {"batch_txns": 8192, "p50_ms": 0.64, "p99_ms": 0.66, "device_p99_ms": 0.33, "pinned_p99_ms": 0.55,
                    "dropin_call_p99_us": 379.5, "path": "z" * 500},
        "host_staged": {"sigs_per_s": 3.97e7, "roofline": {"x": "w" * 400}},
        "stream": {"sigs_per_s": 1.7e8, "n_gpus": n_gpus, "tiles_per_gpu": 2, "max_rate": curve[0], "paced": curve[0],
                   "latency_curve": curve, "knee": {"frags_per_s_per_gpu": 7.5e6}, "unreliable_max": curve[0],
                   "unreliable_goodput_vs_max": 0.86, "all_published": True},
        "extra_configs": {"configs0_small_msg_200B": {"sigs_per_s": 9.5e7, "results_ok": True},
                          "configs2_adversarial_10pct": {"sigs_per_s": 1.06e8, "results_ok": True},
                          "configs3_multisig_1to12": {"sigs_per_s": 9.9e7, "results_ok": True}},
        "headline_two_contexts": {"sigs_per_s": 1.07e8},
    }


def test_compact_line_fits_and_carries_the_contract(tmp_path):
    full = canned_full()
    assert len(json.dumps(full)) > 15000            # the round-3 size that the driver could not parse
    detail = str(tmp_path / "d" / "bench_detail.json")
    line = bench.emit_record(full, detail)
    assert len(line) <= bench.HEADLINE_MAX_BYTES and "\n" not in line
    rec = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "results_ok", "kernel_ms", "roofline", "cpu_baseline"):
        assert k in rec, k
    assert rec["value"] == full["value"] and rec["n_gpus"] == 8
    rf = rec["roofline"]
    assert rf["frac"] == pytest.approx(0.3815, rel=1e-3) and rf["frac_live"] == pytest.approx(0.4777, rel=1e-3)
    assert rf["peak"] == pytest.approx(39321.6, rel=1e-3) and rf["traffic"] == 10.1e9
    assert rec["cpu_baseline"]["cores"] == 16 and rec["cpu_baseline"]["kind"] == "reference"
    assert len(rec["per_gpu"]) == 8
    assert rec["stream"]["knee"] == 7.5e6 and len(rec["stream"]["paced_fps_p50_p99_us"]) == 5
    # per paced leg: the longest GPU-side hold of a copy and how many were held over 250 us (the GPU pauses)
    assert rec["stream"]["paced_gpu_pause_max_us"] == [850.0] * 5
    assert rec["stream"]["paced_gpu_pauses_over_250us"] == [3] * 5
    assert json.load(open(detail)) == full          # the detail file keeps everything


def test_stream_ok_and_first_anomaly(tmp_path):
    """A clean stream sets stream_ok; an anomaly (a verdict neither published nor overrun) clears it and the
    compact line names the first one: leg, tile, seq, payload, the GPU's code and the batch that produced it."""
    full = canned_full()
    rec = json.loads(bench.emit_record(full, None))
    assert rec["stream_ok"] is True and rec["stream"]["anomalies"] == 0 and rec["stream"]["anomaly_first"] is None
    first = {"seq": 123457, "in_idx": 0, "payload_idx": 99, "tag": 7, "result": 2, "code": -3, "ctx": 1,
             "batch_txns": 2049, "batch_pos": 2048, "path": 8, "tile": 0, "rank": 0}
    full["stream"]["anomalies"] = {"paced@2000000": {"count": 1, "first": [first]}}
    rec = json.loads(bench.emit_record(full, None))
    assert rec["stream_ok"] is False and rec["stream"]["anomalies"] == 1
    a = rec["stream"]["anomaly_first"]
    assert a["leg"] == "paced@2000000" and a["path"] == "latency8" and a["code"] == -3 and a["batch_pos"] == 2048
    full["stream"] = {"error": "child failed"}
    assert json.loads(bench.emit_record(full, None))["stream_ok"] is False


def test_oversized_summaries_are_dropped_not_the_headline(tmp_path):
    full = canned_full(n_gpus=8)
    full["stream"] = {"error": "e" * 10000}
    full["per_gpu"] = full["per_gpu"] * 40            # absurdly many rows
    line = bench.emit_record(full, None)
    rec = json.loads(line)
    assert len(line) <= bench.HEADLINE_MAX_BYTES
    assert rec["roofline"]["frac"] and rec["cpu_baseline"]["value"]


@pytest.mark.parametrize("n", [2])
def test_gpus_n_starts_n_ranks(tmp_path, n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    detail = str(tmp_path / "detail.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "3", "--warmup",
                        "1", "--txns", "1000", "--dry-run", "--detail-out", detail],
                       capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    rec = json.loads(lines[-1])
    assert rec["n_gpus"] == n and [row[0] for row in rec["per_gpu"]] == list(range(n))
    # rank 1 sleeps 4 ms per step: the value is all ranks' units over the slowest rank's time
    assert rec["ms_per_step"] >= 4.0
    assert rec["value"] == pytest.approx(n * 1000 * 1e3 / rec["ms_per_step"], rel=1e-6)


def test_gpus_mismatch_refused():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_failed_rank_takes_the_others_down(tmp_path):
    stub = tmp_path / "stub.py"
    stub.write_text("import os, sys, time\n"
                    "sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(600)\n")
    import time
    t0 = time.time()
    rc = bench.launch_ranks(2, [], script=str(stub), timeout_s=120)
    assert rc == 3 and time.time() - t0 < 60


def _pt(rate, p99, lost=0, ovr=0):
    return {"offered_frags_per_s_per_gpu": rate, "p99_us": p99, "lost": lost, "overruns_at_verdict": ovr}


def test_knee_is_monotone():
    """stream.knee: every tried rate up to the knee holds p99 <= 1 ms with nothing lost or overrun."""
    assert bench.knee_of([_pt(2e6, 600), _pt(5e6, 640), _pt(10e6, 960), _pt(15e6, 1700)]) == 10e6
    assert bench.knee_of([_pt(15e6, 1700), _pt(2e6, 600), _pt(10e6, 960)]) == 10e6           # order-free
    assert bench.knee_of([_pt(2e6, 600), _pt(5e6, 1200), _pt(10e6, 960)]) == 2e6             # a lower rate failed
    assert bench.knee_of([_pt(2e6, 600), _pt(5e6, 700, lost=3), _pt(10e6, 900)]) == 2e6      # frags lost
    assert bench.knee_of([_pt(2e6, 600, ovr=1)]) is None
    assert bench.knee_of([_pt(2e6, 1000.0)]) == 2e6                                          # the bound is inclusive


def test_leg_copy_settings():
    """The reliable max-rate legs (cal, max) copy in bigger gathers; paced and unreliable legs keep the tile's
    defaults (0 = fdgpu_vtile_opts_t default)."""
    args = bench.parse_args([]) if hasattr(bench, "parse_args") else None
    if args is None:
        pytest.skip("bench.parse_args not available")
    for leg, tput in (("cal", True), ("max", True), ("paced@5000000.0", False), ("unrel", False)):
        cfg = bench._leg_cfg(args, leg, 1, 20e6)
        want = int(args.stream_tput_copy_wait_us * 1000) if tput else \
            int(args.stream_lat_copy_wait_us * 1000) if leg.startswith("paced") else 0
        assert cfg["copy_wait_ns"] == want, leg
        assert cfg["max_uncopied"] == (args.stream_tput_max_uncopied if tput else 0), leg
    assert args.stream_tput_copy_wait_us == 2000.0 and args.stream_tput_max_uncopied == 131072
    assert bench._leg_cfg(args, "max", 1, 20e6)["copy_min"] == 32768 and bench._leg_cfg(args, "unrel", 1, 20e6)["copy_min"] == 0


@pytest.mark.parametrize("cores,gpus,tiles,capped", [(128, 8, 2, False), (24, 8, 2, False), (16, 8, 1, True),
                                                     (8, 8, 1, True), (4, 1, 2, False), (2, 1, 1, True)])
def test_host_plan_caps_tiles_to_the_cores(cores, gpus, tiles, capped):
    """VERDICT r04 Missing 3: per GPU 2 max-rate tiles (or 1 paced tile) + 1 producer, each spinning on a core
    of its own (topology.c:167-170); tiles per GPU drop, never below 1, when the job's cores cannot hold them."""
    args = bench.parse_args(["--stream-svc-tiles", ""])       # (the served legs' budget: below)
    plan = bench.host_plan(args, gpus, cores=cores, nodes={0: cores}, gpu_nodes=[0] * gpus)
    assert plan["requested"]["cores"] == gpus * 3
    assert plan["applied"]["tiles_per_gpu"] == tiles and plan["capped"] is capped
    assert plan["applied"]["paced_tiles_per_gpu"] == 1
    assert plan["oversubscribed"] is (gpus * (tiles + 1) > cores)
    assert ("cap" in plan) is capped
    assert plan["host_dram_gbs_est"] == pytest.approx(gpus * 68.0)


@pytest.mark.parametrize("cores,gpus,launchers", [(128, 8, 1), (24, 8, 1), (16, 8, 0), (3, 1, 1), (2, 1, 0)])
def test_host_plan_paced_launch_threads(cores, gpus, launchers):
    """--stream-lat-launcher: a paced tile's launch thread takes a core of its own; where a GPU's share
    cannot hold tile + launch thread + producer the plan drops the thread (and says so), never the tile."""
    args = bench.parse_args(["--stream-lat-launcher", "1", "--stream-svc-tiles", ""])
    plan = bench.host_plan(args, gpus, cores=cores, nodes={0: cores}, gpu_nodes=[0] * gpus)
    assert plan["requested"]["paced_launchers"] == 1 and plan["applied"]["paced_launchers"] == launchers
    assert plan["applied"]["paced_tiles_per_gpu"] == 1
    assert plan["applied"]["cores"] == gpus * (max(plan["applied"]["tiles_per_gpu"], 1 + launchers) + 1)
    assert plan["capped"] is (launchers == 0 or plan["applied"]["tiles_per_gpu"] < 2)
    args = bench.parse_args(["--stream-lat-launcher", "1", "--plan-cores", str(cores), "--stream-svc-tiles", ""])
    assert bench._leg_cfg(args, "paced@5000000.0", gpus, 20e6)["launcher"] == launchers
    assert bench._leg_cfg(args, "max", gpus, 20e6)["launcher"] == 0


@pytest.mark.parametrize("cores,gpus,h,tiles", [(128, 8, 2, 2), (56, 8, 2, 2), (40, 8, 2, 1), (24, 8, 1, 1), (16, 8, 0, 1)])
def test_host_plan_copy_threads(cores, gpus, h, tiles):
    """--stream-copy-threads 2: each max-rate tile's copy threads take a core each; short of cores the plan
    lowers tiles first, then copy threads (never below one tile)."""
    args = bench.parse_args(["--stream-copy-threads", "2", "--plan-cores", str(cores)])
    plan = bench.host_plan(args, gpus, cores=cores, nodes={0: cores}, gpu_nodes=[0] * gpus)
    assert plan["requested"]["cores"] == gpus * (2 * 3 + 1)
    assert plan["applied"]["copy_threads_per_tile"] == h and plan["applied"]["tiles_per_gpu"] == tiles
    assert plan["applied"]["cores"] <= max(cores, gpus * 2)
    assert bench._leg_cfg(args, "max", gpus, 20e6)["copy_threads"] == h
    assert bench._leg_cfg(args, "paced@5000000.0", gpus, 20e6)["copy_threads"] == 0


def test_host_plan_per_numa_node():
    """Each child pins to its GPU's NUMA node first: 4 GPUs on a 6-core node and 4 on a 64-core node get the
    small node's share (1 tile each) rather than oversubscribing it."""
    args = bench.parse_args([])
    plan = bench.host_plan(args, 8, cores=70, nodes={0: 6, 1: 64}, gpu_nodes=[0, 0, 0, 0, 1, 1, 1, 1])
    assert plan["applied"]["tiles_per_gpu"] == 1 and plan["capped"]
    plan = bench.host_plan(args, 8, cores=140, nodes={0: 70, 1: 70}, gpu_nodes=[0, 0, 0, 0, 1, 1, 1, 1])
    assert plan["applied"]["tiles_per_gpu"] == 2 and not plan["capped"]


def test_host_topology_gpu_nodes_in_hip_order(tmp_path, monkeypatch):
    """The plan's GPU -> NUMA node comes from each HIP device's own PCI function, in HIP's device order (the
    KFD topology's GPU nodes after ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES), not from the host's PCI order
    of every AMD GPU: a job given only the host's 6th GPU (on node 1) plans for node 1 (VERDICT r05 weak 3:
    the plan said node 0 while the link pinned to node 1)."""
    from test_vsvc import _fake_sysfs
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "FDGPU_BENCH_ONE_DEVICE"):
        monkeypatch.delenv(k, raising=False)
    root = str(tmp_path)
    _fake_sysfs(root, [(0x0500 + 0x1000 * i, 0, 0 if i < 4 else 1) for i in range(8)])
    for n in (0, 1):
        d = tmp_path / f"devices/system/node/node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(f"{64 * n}-{64 * n + 63}\n")
    _, gn = bench.host_topology(8, root)
    assert gn == [0, 0, 0, 0, 1, 1, 1, 1]
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "5")
    _, gn = bench.host_topology(1, root)
    assert gn == [1]
    args = bench.parse_args([])
    assert bench.host_plan(args, 1, cores=16, nodes={0: 64, 1: 64}, gpu_nodes=gn)["gpu_numa_nodes"] == [1]


def test_dry_run_prints_the_plan(tmp_path):
    """`--gpus 8 --dry-run --plan-cores 16` prints the plan and the cap it applied in the compact line."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run", "--plan-cores", "16",
                        "--steps", "2", "--warmup", "1", "--detail-out", str(tmp_path / "d.json")],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    hp = json.loads(r.stdout.strip().splitlines()[-1])["host_plan"]
    # per GPU the served legs ask the most: 2 tile processes + the verify service + its launch thread + a producer
    assert hp["need_cores"] == 40 and hp["used_cores"] == 16 and hp["tiles_per_gpu"] == 1 and hp["capped"]
    assert "2 -> 1" in hp["cap"] and "served tiles 2 -> 0" in hp["cap"]


def test_kfd_queues_without_kfd():
    """The KFD queue / eviction sampler reads only sysfs: off a GPU host (no /sys/class/kfd) it reports
    nothing and its thread ends at once."""
    q = bench.kfd_queues()
    assert q is None or set(q) == {"queues", "procs", "evicted_ms"}
    with bench.KfdSampler() as s:
        pass
    assert s.peak is None or s.peak["evicted_ms"] >= 0.0



def test_producer_tile_placement():
    """_pair_place: the paced link's producer 0 and tile 0 CPUs, their L3 group and NUMA node from sysfs, and
    whether they share them (None where a CPU is unknown)."""
    cpus = sorted(os.sched_getaffinity(0))
    p = bench._pair_place({"prod_cpu": [cpus[0], -1, -1, -1], "tile_cpu": [cpus[0]] + [0] * 7})
    assert p["producer"]["cpu"] == cpus[0] and p["tile"]["cpu"] == cpus[0]
    if p["producer"]["l3"] is not None:
        assert p["same_l3"] is True
    q = bench._pair_place({"prod_cpu": [-1] * 4, "tile_cpu": [cpus[0]] + [0] * 7})
    assert q["producer"] is None and q["same_l3"] is None and q["same_node"] is None
    assert bench.cpu_place(-1) is None


@pytest.mark.parametrize("cores,gpus,want,got", [(16, 1, "1,2,3", 3), (16, 8, "1,2,3", 0), (64, 8, "1,2,3", 3),
                                                  (40, 8, "2,3", 2), (16, 1, "", 0), (16, 1, None, 2)])
def test_host_plan_served_tiles(cores, gpus, want, got):
    """Served paced legs need T tile processes + the verify service + its launch thread + the producer per
    GPU: the plan caps T to the cores (0: the served legs are skipped rather than oversubscribe).  The default
    (None) runs T = 2."""
    args = bench.parse_args(["--stream-svc-tiles", want] if want is not None else [])
    plan = bench.host_plan(args, gpus, cores=cores, nodes={0: cores}, gpu_nodes=[0] * gpus)
    assert plan["applied"]["served_tiles_per_gpu"] == got
    assert plan["applied"]["cores"] <= max(cores, gpus * 2)


def test_recycled_dedups_are_not_anomalies():
    """The link counts apart the dedup failures of payloads a tile had published before (the synthetic payloads
    recycle; after a tile lost most of its frags their tags can still be in its tcache: profiles/r06/n2svc,
    r06/final): the record keeps them as dedup_recycled, and they are not in the anomaly count."""
    anom = {"paced@2500000.0": {"count": 0, "first": [], "by_result": {"dedup_recycled": 10}},
            "paced@1000000.0": {"count": 1, "first": [{"result": 6, "path": 0}], "by_result": {"gpu_fault": 1}}}
    n, first = bench.anomaly_summary(anom)
    assert n == 1 and first["leg"] == "paced@1000000.0"
    assert bench.dedup_recycled(anom) == 10
    assert bench.RESULT_NAMES[0] == "dedup_recycled" and bench.RESULT_NAMES[3] == "dedup"

def test_link_dir_prefers_hugetlbfs_with_room(tmp_path):
    """The link of several processes goes on a writable hugetlbfs mount with free pages for it (2 MiB pages, as the
    reference's workspaces), else /dev/shm."""
    import bench
    mnt = tmp_path / "huge"; mnt.mkdir()
    hp = tmp_path / "hp" / "hugepages-2048kB"; hp.mkdir(parents=True)
    (hp / "free_hugepages").write_text("1024\n")                       # 2 GiB free
    mounts = tmp_path / "mounts"
    mounts.write_text(f"tmpfs /dev/shm tmpfs rw 0 0\nnone {mnt} hugetlbfs rw,relatime,pagesize=2M 0 0\n")
    f = lambda need, choice="auto": bench.link_dir(choice, need, str(mounts), str(tmp_path / "hp"))
    assert f(1 << 30) == str(mnt)
    assert f(2 << 30) == "/dev/shm"                                    # not room for 1.25 x the link
    assert f(1 << 30, "/tmp/x") == "/tmp/x"
    mounts.write_text("tmpfs /dev/shm tmpfs rw 0 0\n")
    assert f(1 << 20) == "/dev/shm"


def test_n8_line_keeps_the_stream_knee():
    """At N = 8 the line grows (8 per_gpu rows, the host plan's cap text): the stream's diagnostics go first, so
    the knee and the served curve stay in it (the default run of profiles/r06/dflt, widened to 8 ranks)."""
    full = json.load(open(os.path.join(ROOT, "profiles", "r06", "dflt", "detail.json")))
    full["n_gpus"] = 8
    full["per_gpu"] = [dict(full["per_gpu"][0], rank=r) for r in range(8)]
    full["host_plan"]["capped"] = True
    full["host_plan"]["cap"] = "c" * 260
    line = bench.emit_record(full, None)
    rec = json.loads(line)
    assert len(line) <= bench.HEADLINE_MAX_BYTES
    assert rec["stream"]["knee"] == 10e6 and rec["stream"]["served"]["2"]["knee"] == 10e6
    assert len(rec["per_gpu"]) == 8 and rec["host_plan"]["cap"]


def test_served_max_leg_cfg():
    """--stream-svc-max: the served legs start with a reliable max-rate leg over the T tile processes, batched
    as the max-rate legs are (throughput path), sized by SVC_MAX_FPS_EST."""
    args = bench.parse_args(["--stream-svc-max", "1"])
    args.stream_svc = 3
    assert bench.stream_legs(args)[0] == "max" and bench.stream_legs(args)[1].startswith("paced@")
    c = bench._leg_cfg(args, "max", 2, 0.0)
    assert c["svc"] == 1 and c["tiles"] == 6 and c["reliable"] and c["rate_fps"] == 0.0
    assert c["n_frags"] == int(bench.SVC_MAX_FPS_EST * 2 * args.stream_seconds)
    assert c["batch_txn"] == bench._leg_cfg(args, "cal", 2, 0.0)["batch_txn"]
    assert c["nctx"] == args.stream_ctx * args.stream_tiles     # the contexts of the one-process max leg's tiles
    args.stream_svc_max = 0
    assert "max" not in bench.stream_legs(args)
