"""Table of paced-only A/B arms (bench.py --stream-only-paced --detail-out): per arm and rate, p99 in ms, mean
batch (txns) and the latest gather start (us); and the knee (every rate up to it at p99 <= 1 ms).
usage: python tools/paced_table.py <dir>..."""
import glob
import json
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/*.json")):
        st = json.load(open(f)).get("stream")
        if not st:                       # (other records in the same directory)
            continue
        legs = st.get("only_paced") or {f"paced@{l['rate_fps']}": l for l in st.get("latency_curve", [])}
        row, knee, ok = [], 0.0, True
        for k, v in sorted(legs.items(), key=lambda kv: float(kv[0].split("@")[1])):
            r = float(k.split("@")[1])
            ok = ok and v["p99_us"] <= 1000.0 and v["lost"] == 0
            knee = r if ok else knee
            row.append(f"{r / 1e6:g}M {v['p99_us'] / 1e3:.3f} b{v['mean_batch_txns']:.0f} g{v['gather_gpu']['launch_to_start_max_us']:.0f}"
                       + (f"/i{v['gather_gpu']['issue_to_start_max_us']:.0f}" if 'issue_to_start_max_us' in v['gather_gpu'] else ""))
        print(f"{f.split('/')[-1]:10s} knee {knee / 1e6:g}M | " + " | ".join(row))
