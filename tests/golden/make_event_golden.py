"""Freezes the event-exact readiness restatement (or_lstore_event_mode, oracle/oracle.c) over the
20k-txn schedule of tests/test_ready.py::test_gpu_event_mode_20k_golden: per ready call the released
txns, their executesAtLeast and the waiting count -> tests/golden/events_20k.npz.  CPU only, ~9 min.
Run from the repo root: python tests/golden/make_event_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "cassandra-accord_amd"))
import test_ready as T  # noqa: E402

p = T.EV20K
s = T.stable_stream(p["n"], p["ks"], p["seed"], p["rf"])
txn, off, waiting, em, el, en = [], [0], [], [], [], []


class Rec(T.Driver):
    def round(self):
        want = super().round()
        txn.append(np.asarray(want, np.uint32))
        off.append(off[-1] + len(want))
        waiting.append(self.ev.waiting)
        em.append(np.asarray(self.eal[0], np.uint64)); el.append(np.asarray(self.eal[1], np.uint64))
        en.append(np.asarray(self.eal[2], np.int32))
        return want


d = Rec(s, p["ks"], None, dev_events=True)
out, _ = T.schedule(s, p["ks"], p["bsz"], p["seed"], driver=d)
cat = lambda xs, t: np.concatenate(xs).astype(t) if xs else np.zeros(0, t)  # noqa: E731
np.savez_compressed(os.path.join(HERE, "events_20k.npz"), txn=cat(txn, np.uint32), off=np.asarray(off, np.uint32),
                    waiting=np.asarray(waiting, np.uint32), eal_msb=cat(em, np.uint64), eal_lsb=cat(el, np.uint64),
                    eal_node=cat(en, np.int32), released=np.uint64(sum(len(r) for r in out)))
print("calls", len(off) - 1, "released", sum(len(r) for r in out))
