#!/usr/bin/env python3
"""The round-6 tables of DESIGN.md §13, rebuilt from the bench records under profiles/r06/.

usage: python3 tools/r06_tables.py [profiles/r06]
  cmp   : paced p99 at equal device load -- one tile process, served T = 1, 2, 3, two processes with own contexts
  place : producer + dcache part on the GPU's node vs the opposite node (max rate, intake, gather GB/s, p99 at 10M)
  hi    : served legs above the knee (10 / 12.5 / 15M)
  final : the final builds' stream curves, one-process and served
"""
import json
import os
import sys

R = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "profiles", "r06")


def load(*p):
    return json.load(open(os.path.join(R, *p)))


def one_curve(st):
    """the one-process paced legs of a record: (offered per GPU, leg) in offered order"""
    if st.get("latency_curve"):
        return [(c["offered_frags_per_s_per_gpu"], c) for c in st["latency_curve"]]
    return sorted((float(k.split("@")[1]), v) for k, v in st["only_paced"].items())


def us(x):
    return f"{x:.0f}" + ("*" if x > 1000 else "")


def cmp_table():
    print("## cmp: paced p99 (us) at equal device load; * = over 1 ms")
    for run in ("a1", "a2"):
        st = load("cmp", f"{run}.json")["stream"]
        print(f"{run} one process      ", [us(c["p99_us"]) for _, c in one_curve(st)])
        for T, v in st["served"]["by_tiles"].items():
            print(f"{run} served T={T}        ", [us(x[2]) for x in v["paced_fps_p50_p99_us"]], "knee", v["knee"])
    st = load("cmp", "own2.json")["stream"]
    print("own2 two processes (device rate 2x per-rank)", [(2 * r / 1e6, us(c["p99_us"])) for r, c in one_curve(st)])


def place_table():
    print("## place: same vs opposite node")
    for run in ("g1", "o1", "g2", "o2"):
        st = load("place", f"{run}.json")["stream"]
        mx, pc = st["max_rate"], st["latency_curve"][0]
        gb = lambda leg: leg["frags"] * 1232 / leg["gather_gpu"]["n"] / leg["gather_gpu"]["run_mean_us"] / 1e3
        print(run, "dcache node", mx["placement"]["dcache_nodes"], "gpu node", mx["placement"]["gpu_node"],
              f"max {mx['sigs_per_s'] / 1e6:.2f}M", "intake", mx["tile_host_ns_per_frag"][0],
              f"gather GB/s {gb(mx):.1f} / {gb(pc):.1f}", "p99@10M", round(pc["p99_us"]),
              "pauses>250us", pc["gather_gpu"]["issue_to_start_over_250us"])


def hi_table():
    print("## hi / smax / smax2: above the knee, p99 (us)")
    for d, runs in (("hi", ("h1", "h2")), ("smax", ("s1",)), ("smax2", ("s2",))):
        for run in runs:
            st = load(d, f"{run}.json")["stream"]
            print(f"{d}/{run} one process", [(r / 1e6, us(c["p99_us"])) for r, c in one_curve(st)])
            for T, v in st["served"]["by_tiles"].items():
                mx = v.get("max")
                print(f"{d}/{run} served T={T}", [(x[0] / 1e6, us(x[2])) for x in v["paced_fps_p50_p99_us"]],
                      f"max {mx['sigs_per_s'] / 1e6:.1f}M" if mx else "")


def final_table():
    print("## final builds")
    for d in ("final_a", "final_b"):
        f = load(d, "bench_line.json")
        st = f["stream"]
        print(d, f"{f['value'] / 1e6:.1f}M sigs/s", "knee", st["knee"], [us(x[2]) for x in st["paced_fps_p50_p99_us"]],
              "served", {T: (v.get("knee"), [us(x) for x in v.get("p99_us", [])]) for T, v in st.get("served", {}).items()})


if __name__ == "__main__":
    cmp_table(); place_table(); hi_table(); final_table()
