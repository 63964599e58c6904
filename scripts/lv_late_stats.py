"""Config 5's reduced DAG (tests/oracle_lib.reduced_dag): per 64-txn chunk, the predecessor pairs and
distinct predecessors within the previous K chunks (the levelling resolver's late work), and the
share of edges older than the resolver's LDS ring.  CPU only: python scripts/lv_late_stats.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import oracle_lib as O  # noqa: E402
from accord_amd import generate_stream  # noqa: E402

p = bench.PRESETS[5]
s = generate_stream(p["n"], p["keys_per_txn"], p["keyspace"], 0.99, p["write_frac"], seed=p["seed"])
off, preds = O.reduced_dag(s)
n = s.n
off = off.astype(np.int64)
preds = preds.astype(np.int64)
tgt = np.repeat(np.arange(n), np.diff(off))
base = (tgt // 64) * 64
ch, nch = tgt // 64, n // 64
for K in (1, 2, 3, 4):
    w = (preds < base) & (preds + 64 * K >= base)
    pairs = np.bincount(ch[w], minlength=nch)
    dist = np.bincount(np.unique(ch[w] * (1 << 23) + preds[w]) >> 23, minlength=nch)
    print(f"K={K}: pairs mean {pairs.mean():.1f} max {pairs.max()}, distinct preds mean {dist.mean():.1f} max {dist.max()}")
for R in (8192, 16384, 32768):
    print(f"edges older than a {R}-entry ring: {(preds + R < base).mean():.3f}")
