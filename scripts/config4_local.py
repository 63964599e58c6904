"""Config 4 at full size on ONE GPU, stream-segment ownership:
G ranks x 1,048,576 txns of the config-2 workload; rank r owns positions [r n, (r+1) n) of every
CommandStore.  Each rank is a resident store on this GPU, measured ALONE (synced, HIP events on
its own stream, median of --reps):
  * summary  -- accord_segment_summary: per key, what later txns can still reach of the segment;
  * carry    -- accord_segment_carry: the fold of the earlier ranks' summaries into the
                CommandsForKey state at the segment's start (the all-gather's payload);
  * compute  -- accord_deps_compute: the segment's node-level deps.
Reported per rank with the summary size (the bytes the rank sends), the output size (the bytes its
deps occupy) and, for the whole job, the projection  max_r(summary + carry + compute) + all-gather
time at --link-gbs (ring all-gather: (G-1) x padded summary bytes through each link)  against one
store computing the whole G x n stream on this GPU.  --check compares every segment's deps with a
resident store fed the whole stream (and segment 1's first txns with the oracle).
python scripts/config4_local.py [--ranks 8] [--reps 5] [--check] [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from accord_amd import CommandStore, generate_stream, segment_bounds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--n", type=int, default=1 << 20, help="txns per rank (weak scaling)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--link-gbs", type=float, default=150.0, help="per-link all-gather rate (SURVEY.md §5)")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    G, ks, W = a.ranks, 100_000, 256
    n_total = a.n * G
    t0 = time.perf_counter()
    s = generate_stream(n_total, 8, ks, 0.99, 0.5, seed=2)       # bench.py PRESETS[2], as --gpus G builds it
    S = 8 * G
    bounds = [b * ks // S for b in range(S)] + [0xFFFFFFFF]
    out = {"workload": f"config4 segments: {G} ranks x {a.n} txns x 8 keys, Zipf(0.99) over {ks} keys, W={W}, "
                       f"{S} EvenSplit CommandStores, seed 2", "ranks": G, "n_total": n_total,
           "generate_s": round(time.perf_counter() - t0, 2)}
    segs = segment_bounds(n_total, G)
    stores, parts, ranks = [], [], []
    try:
        for r, (lo, hi) in enumerate(segs):
            st = CommandStore(device=0, key_lo=0, key_hi=ks, window=W, profile=True, resident=True, store_bounds=bounds)
            st.segment_begin(lo)
            st.upload(s.slice(lo, hi))
            ms = []
            for _ in range(a.reps + 1):
                p = st.segment_summary()
                ms.append(st.segment_timing()[0])
            parts.append(p)
            stores.append(st)
            ranks.append({"rank": r, "segment": [lo, hi], "pairs": int(s.key_off[hi] - s.key_off[lo]),
                          "summary_ms": float(np.median(ms[1:])), "summary_entries": p[0],
                          "summary_bytes": 8 * p[0]})
        m = max(p[0] for p in parts)
        for r, st in enumerate(stores):
            cm, dm = [], []
            for _ in range(a.reps + 1):
                st.segment_carry(parts[:r])
                cm.append(st.segment_timing()[1])
                st.compute()
                dm.append(st.timing().total_ms)
            v = st.device_view()
            d = st.download()
            out_bytes = 4 * (int(v["kd_keys_total"]) + int(d.kd_val_off[-1]) + int(v["kd_k2v_total"])) + 12 * (a.n + 1)
            ranks[r].update({"carry_ms": float(np.median(cm[1:])), "compute_ms": float(np.median(dm[1:])),
                             "carry_entries": st.state()["carry_entries"], "output_bytes": out_bytes,
                             # a ring all-gather of padded summaries: every rank sends its own and forwards
                             # G - 2 others through one link
                             "allgather_bytes_per_link": 8 * m * (G - 1),
                             "remote_frac_of_output": 8 * m * (G - 1) / out_bytes})
            ranks[r]["step_ms"] = ranks[r]["summary_ms"] + ranks[r]["carry_ms"] + ranks[r]["compute_ms"]
            print(json.dumps(ranks[r]), flush=True)
            del d
        if a.check:
            import oracle_lib as O
            bad = []
            with CommandStore(device=0, key_lo=0, key_hi=ks, window=W, resident=True) as one:
                for r, (lo, hi) in enumerate(segs):
                    stores[r].segment_carry(parts[:r])
                    stores[r].compute()
                    got = stores[r].download()
                    one.upload(s.slice(lo, hi))
                    one.compute()
                    diff = got.first_difference(one.download())
                    if diff is not None:
                        bad.append([r, str(diff)])
                    if r == 1:
                        k = 20_000
                        exp = O.deps_fast(s.prefix(lo + k), W).txns(lo, lo + k)
                        out["oracle_boundary_equal"] = got.txns(0, k).first_difference(exp) is None
            out["segments_equal_single_store"] = not bad
            out["mismatch"] = bad
    finally:
        for st in stores:
            st.close()
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W, profile=True) as one:
        one.upload(s)
        ms = []
        for _ in range(3):
            one.compute()
            ms.append(one.timing().total_ms)
        out["single_gpu_whole_stream_ms"] = float(min(ms))
    comp = [r["compute_ms"] for r in ranks]
    step = [r["step_ms"] for r in ranks]
    xfer_ms = 8 * max(p[0] for p in parts) * (G - 1) / (a.link_gbs * 1e9) * 1e3
    proj = max(step) + xfer_ms
    out.update({"per_rank": ranks, "compute_max_over_mean": max(comp) / (sum(comp) / G),
                "step_max_ms": max(step), "allgather_ms_at_link_gbs": xfer_ms, "link_gbs": a.link_gbs,
                "projected_step_ms": proj,
                "projected_speedup_vs_one_gpu": out["single_gpu_whole_stream_ms"] / proj,
                "max_remote_frac_of_output": max(r["remote_frac_of_output"] for r in ranks)})
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    if out.get("segments_equal_single_store") is False or out.get("oracle_boundary_equal") is False:
        sys.exit(1)


if __name__ == "__main__":
    main()
