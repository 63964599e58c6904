"""Config 4 at full size on ONE GPU: G ranks x 1,048,576 txns of the config-2
workload, every rank a CommandStore over its key block (rank r hosts EvenSplit stores [8r, 8r+8),
local/ShardDistributor.java:46-157) holding the partial deps of the txns that touch it, then
accord_deps_exchange_local -- the RCCL exchange's plan and on-device union (PreAccept.reduce,
messages/PreAccept.java:140-156) with the transport replaced by device copies.

Prints one JSON object: per-rank txns / pairs / device compute ms (median of --reps computes, the
store's own HIP events), the partial's KeyDeps sizes (what the rank ships, less its own block), the
exchange's wall ms and per-rank plan/merge ms, and two parity checks:
  * every rank's exchanged block equals the same txns' deps from ONE store computing the whole
    G x 1 Mi stream (config-2 txns are key-only, so store slicing cannot change a dep);
  * the first --oracle-prefix txns of rank 0's block equal the C oracle on that stream prefix
    (deps of txn i depend on txns < i only).
python scripts/config4_local.py [--ranks 8] [--reps 5] [--oracle-prefix 20000] [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from accord_amd import CommandStore, generate_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--n", type=int, default=1 << 20, help="txns per rank (weak scaling)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--oracle-prefix", type=int, default=20000)
    ap.add_argument("--no-single", action="store_true", help="skip the single-store comparison")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    G, ks, W = a.ranks, 100_000, 256
    n_total = a.n * G
    t0 = time.perf_counter()
    s = generate_stream(n_total, 8, ks, 0.99, 0.5, seed=2)       # bench.py PRESETS[2], as --gpus G builds it
    gen_s = time.perf_counter() - t0
    S = 8 * G
    bounds = [b * ks // S for b in range(S)] + [0xFFFFFFFF]
    ranks, stores = [], []
    out = {"workload": f"config4-local: {G} ranks x {a.n} txns x 8 keys, Zipf(0.99) over {ks} keys, seed 2",
           "ranks": G, "n_total": n_total, "generate_s": round(gen_s, 2)}
    try:
        for r in range(G):
            lo, hi = (8 * r) * ks // S, (8 * r + 8) * ks // S
            sr = s.restrict_keys(lo, hi, drop_empty=True)
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W, profile=True,
                              store_bounds=bounds[8 * r:8 * r + 9])
            st.upload(sr)
            ms = []
            for _ in range(a.reps + 1):
                st.compute()
                ms.append(st.timing().total_ms)
            dv = st.device_view()
            hot = int(np.bincount(np.asarray(sr.key_ord, np.int64) - lo).max()) if sr.pairs else 0
            ranks.append({"rank": r, "keys": [lo, hi], "txns": sr.n, "pairs": int(sr.pairs), "hottest_key_txns": hot,
                          "compute_ms_median": round(float(np.median(ms[1:])), 4),
                          "compute_ms_min": round(float(min(ms[1:])), 4),
                          # the partial this rank sends (all but its own txn block): KeyDeps words
                          "partial_keys": int(dv["kd_keys_total"]), "partial_vals_ub": int(dv["kd_vals_total"]),
                          "partial_k2v": int(dv["kd_k2v_total"])})
            stores.append(st)
            print(json.dumps(ranks[-1]), flush=True)
        t1 = time.perf_counter()
        CommandStore.exchange_local(stores, n_total)
        out["exchange_wall_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
        for r, st in enumerate(stores):
            plan, merge = st.shard_timing()
            ranks[r]["exchange_plan_ms"], ranks[r]["exchange_merge_ms"] = round(plan, 4), round(merge, 4)
        got = [st.download() for st in stores]
        for r, d in enumerate(got):
            ranks[r]["node_level_deps"] = d.totals()["vals"]
    finally:
        for st in stores:
            st.close()
    out["per_rank"] = ranks
    out["max_rank_compute_ms"] = max(r["compute_ms_median"] for r in ranks)
    bad = []
    if not a.no_single:
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=W, profile=True) as one:
            one.upload(s)
            one.compute()
            out["single_store_compute_ms"] = round(one.timing().total_ms, 4)
            whole = one.download()
        for r, d in enumerate(got):
            lo, hi = r * n_total // G, (r + 1) * n_total // G
            diff = d.first_difference(whole.txns(lo, hi))
            if diff is not None:
                bad.append([r, str(diff)])
        out["ranks_equal_single_store"] = not bad
        out["mismatch"] = bad
        del whole
    if a.oracle_prefix:
        import oracle_lib as O
        m = min(a.oracle_prefix, n_total // G)
        exp = O.deps_fast(s.prefix(m), W)
        diff = got[0].txns(0, m).first_difference(exp)
        out["oracle_prefix"] = m
        out["oracle_prefix_equal"] = diff is None
        if diff is not None:
            out["oracle_prefix_diff"] = str(diff)
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    if bad or out.get("oracle_prefix_equal") is False:
        sys.exit(1)


if __name__ == "__main__":
    main()
