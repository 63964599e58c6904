"""Debug: replay test_gpu_schedule_equals_oracle[2500-30-250-7-0.1] and, at the first executesAtLeast
difference, print the txn, its deps and their statuses / executeAts."""
import os
import sys

import numpy as np

os.environ.setdefault("ACCORD_READY_TRACE", "2107,2091,2104")

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "cassandra-accord_amd")]
import test_ready as T  # noqa: E402
from accord_amd import CommandStore, WINDOW_NONE  # noqa: E402

parts = {}
orig_batch = T.Driver.batch


def batch(self, lo, hi):
    p = orig_batch(self, lo, hi)
    parts[lo] = (hi, p)
    return p


def find(g):
    for lo, (hi, p) in parts.items():
        if lo <= g < hi:
            return lo, p
    raise KeyError(g)


def show(d, g):
    s = d.s
    lo, p = find(g)
    t = g - lo
    kind = (int(s.lsb[g]) >> 1) & 7
    print(f"txn {g} kind {kind} rdom {int(s.lsb[g]) & 1} tid hlc {int(s.lsb[g]) >> 16} node {int(s.node[g])} "
          f"status {d.status[g]} exec {d.execs[g]}")
    keys, vals, k2v = p.key_deps(t)
    K = len(keys)
    for q, k in enumerate(keys):
        d0 = K if q == 0 else int(k2v[q - 1]); d1 = int(k2v[q])
        print("  key", int(k), "deps", [int(vals[int(x)]) for x in k2v[d0:d1]])
    for u in vals:
        u = int(u)
        print(f"   kdep {u} kind {(int(s.lsb[u]) >> 1) & 7} rdom {int(s.lsb[u]) & 1} status {d.status[u]} exec {d.execs[u]}")
    _, _, rv, _ = p.range_deps(t)
    for u in rv:
        u = int(u)
        print(f"   rdep {u} kind {(int(s.lsb[u]) >> 1) & 7} status {d.status[u]} exec {d.execs[u]}")

def rnd(self):
    want, weal = self.ora.ready_ex()
    got, waiting, geal = self.dev.ready_update_ex()
    self.eal = weal
    assert np.array_equal(got, want), (got[:20], want[:20])
    for i in range(len(got)):
        if any(int(a[i]) != int(b[i]) for a, b in zip(geal, weal)):
            print("MISMATCH txn", int(got[i]), "dev", [int(a[i]) for a in geal], "ora", [int(b[i]) for b in weal])
            show(self, int(got[i]))
            raise SystemExit(1)
    return want


T.Driver.batch = batch
T.Driver.round = rnd
s = T.stable_stream(2500, 30, 7, 0.1)
with CommandStore(device=0, key_lo=0, key_hi=30, window=WINDOW_NONE, resident=True) as dev:
    T.schedule(s, 30, 250, 7, dev)
print("no mismatch")
