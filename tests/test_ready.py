"""Execution readiness of a registered-status store: CommandsForKey.notify /
registerUnmanaged / notifyUnmanaged (local/CommandsForKey.java:1163-1215, 1315-1498, 1512-1635) and
Commands.updateWaitingOn (local/Commands.java:755-830) clearing WaitingOn as statuses change, until a
txn is ReadyToExecute (Commands.maybeExecute, :656-733).

CPU: the oracle restatement (or_lstore_ready, over literal CommandsForKey objects) against
hand-derived known answers -- a Read waits for the Write before it, a Write for the Reads and Writes
before it, a STABLE txn for a dep that is still uncommitted (until it commits executing later), an
unmanaged range txn for every committed txn on the key up to its latest dep (notifyUnmanaged(APPLY,
next)) -- and, with every txn STABLE at executeAt = TxnId, the rounds of the ready -> APPLIED loop
equal the independent CommandsForKey-side simulation or_levels_cfk.
GPU: accord_ready_update == the oracle, round by round, over event schedules that interleave
batches, STABLE events (some executeAt past the TxnId, some txns committing late) and APPLIED
feedback, with range txns and EphemeralReads, through the C ABI.
"""
import numpy as np
import pytest

from accord_amd import NO_TXN, CommandStore, IllegalStateException, Stream, WINDOW_NONE, generate_stream
import oracle_lib as O
from status_events import APPLIED, INVALID, STABLE, rb_map

KIND = {"R": 0, "W": 1, "ER": 2, "SP": 3, "XSP": 4}


def mk(txns):
    """txns: [(hlc, kind, node, keys or None, ranges or None)], epoch 1; ranges make a Range-domain txn."""
    n = len(txns)
    msb = np.full(n, 1 << 15, np.uint64)
    lsb = np.array([(h << 16) | (KIND[k] << 1) | (1 if rs is not None else 0) for h, k, _, _, rs in txns], np.uint64)
    node = np.array([t[2] for t in txns], np.int32)
    key_off = np.zeros(n + 1, np.uint32)
    key_off[1:] = np.cumsum([len(t[3] or []) for t in txns])
    key_ord = np.array([k for t in txns for k in (t[3] or [])], np.uint32)
    rng_off = np.zeros(n + 1, np.uint32)
    rng_off[1:] = np.cumsum([len(t[4] or []) for t in txns])
    rs = np.array([a for t in txns for a, _ in (t[4] or [])], np.uint32)
    re = np.array([b for t in txns for _, b in (t[4] or [])], np.uint32)
    return Stream(msb, lsb, node, key_off, key_ord, rng_off, rs, re)


class Driver:
    """One schedule driven into the oracle and (optionally) the device store in lockstep."""

    def __init__(self, s, nkeys, dev=None, events=False, dev_events=False):
        self.s, self.ora, self.dev = s, O.LStore(nkeys), dev
        self.status = np.zeros(s.n, np.uint8)
        self.execs = [None] * s.n
        # events: an event-driven restatement (or_lstore_event_mode) fed the same schedule in lockstep;
        # ev_rounds[c] = what it releases at call c.  dev_events: the device runs event-exact
        # (accord_ready_set_mode ACCORD_READY_EVENTS) and is compared with that restatement instead
        self.dev_events = dev_events
        self.ev = O.LStore(nkeys, event_mode=True) if (events or dev_events) else None
        self.ev_rounds = []
        if dev is not None and dev_events:
            dev.ready_mode(True)

    def batch(self, lo, hi):
        if self.ev is not None:
            self.ev.batch(self.s.slice(lo, hi))
        part = self.ora.batch(self.s.slice(lo, hi))
        if self.dev is not None:
            got = self.dev.calculate_deps_batch(self.s.slice(lo, hi))
            assert got.first_difference(part) is None, got.first_difference(part)
        self.status[lo:hi] = 2
        return part

    def register(self, idx, st, execs=None):
        idx = np.asarray(idx, np.int64)
        if idx.size == 0:
            return
        order = np.argsort(idx)
        idx = idx[order]
        s = self.s
        em = s.msb[idx].copy(); el = s.lsb[idx].copy(); en = s.node[idx].copy()
        for r, g in enumerate(idx):
            if execs is not None and execs[order[r]] is not None:
                self.execs[g] = execs[order[r]]
            if self.execs[g] is None:
                self.execs[g] = (int(s.msb[g]), int(s.lsb[g]), int(s.node[g]))
            em[r], el[r], en[r] = self.execs[g]
        stv = np.full(idx.size, st, np.uint8)
        self.ora.register(s.msb[idx], s.lsb[idx], s.node[idx], stv, em, el, en)
        if self.ev is not None:
            self.ev.register(s.msb[idx], s.lsb[idx], s.node[idx], stv, em, el, en)
        if self.dev is not None:
            self.dev.register(s.msb[idx], s.lsb[idx], s.node[idx], stv, em, el, en)
        self.status[idx] = st

    def initialise(self, lo, part):
        self.ora.waiting_add(lo, part)
        if self.ev is not None:
            self.ev.waiting_add(lo, part)
        if self.dev is not None:
            self.dev.waiting_on_initialise()

    def round(self):
        if self.dev_events:
            want, weal = self.ev.ready_ex()
            self.ev_rounds.append(want)
            self.eal = weal
            if self.dev is not None:
                got, waiting, geal = self.dev.ready_update_ex()
                assert np.array_equal(got, want), (got[:20], want[:20])
                assert waiting == self.ev.waiting
                for a, b in zip(geal, weal):
                    assert np.array_equal(a, b), (got, a, b)
            self.ora.ready_ex()                            # the polling restatement keeps pace
            return want
        if self.ev is not None:
            self.ev_rounds.append(self.ev.ready())
        want, weal = self.ora.ready_ex()
        self.eal = weal                                   # Command.executesAtLeast of the ready txns
        if self.dev is not None:
            got, waiting, geal = self.dev.ready_update_ex()
            assert np.array_equal(got, want), (got[:20], want[:20])
            assert waiting == self.ora.waiting
            for a, b in zip(geal, weal):
                assert np.array_equal(a, b), (got, a, b)
        return want

    def redundant(self, start, end, locally_applied, bootstrapped_at, stale=None, start_epoch=None, end_epoch=None):
        """The store's RedundantBefore with the rest of each entry (removeRedundantDependencies); the
        shard bound stays NONE (no truncation, no collectDeps union)."""
        m = len(start)
        se = [0] * m if start_epoch is None else start_epoch
        ee = [1 << 62] * m if end_epoch is None else end_epoch
        st = [0] * m if stale is None else stale
        self.ora.redundant(start, end, se, ee, locally_applied, bootstrapped_at, st)
        if self.dev is not None:
            self.dev.redundant_before(start=start, end=end, start_epoch=se, end_epoch=ee, bound=[NO_TXN] * m,
                                      min_epoch=0, locally_applied=locally_applied, bootstrapped_at=bootstrapped_at,
                                      stale=st)

    def apply(self, ready):
        self.register(ready, APPLIED)


def drain(d, limit=100000):
    rounds = []
    for _ in range(limit):
        r = d.round()
        if r.size == 0:
            break
        rounds.append(r)
        d.apply(r)
    return rounds


# ---- hand-derived known answers (CPU oracle; GPU below) ----
# k1: t0 W, t1 R, t2 W, t3 R; t4 a Range-domain Write over (0, 1] (unmanaged on k1); k2: t5 W stays
# PREACCEPTED, t6 R (dep t5), t7 W (deps t5, t6)
KAT = [(10, "W", 1, [1], None), (11, "R", 1, [1], None), (12, "W", 1, [1], None), (13, "R", 1, [1], None),
       (14, "W", 1, None, [(0, 1)]), (15, "W", 1, [2], None), (16, "R", 1, [2], None), (17, "W", 1, [2], None)]


def kat_run(dev=None):
    s = mk(KAT)
    d = Driver(s, 4, dev)
    part = d.batch(0, 8)
    d.register([0, 1, 2, 3, 4, 6, 7], STABLE)            # t5 stays PREACCEPTED
    d.initialise(0, part)
    r0 = d.round()
    # t0 has no deps; t5 is not STABLE; t6 waits for t5 (uncommitted dep), t7 for t5 and t6
    assert list(r0) == [0]
    d.apply(r0)
    r1 = d.round()
    assert list(r1) == [1]                                # t1 R after t0 applied; t2 W waits for t1
    d.apply(r1)
    r2 = d.round()
    assert list(r2) == [2]
    d.apply(r2)
    r3 = d.round()
    # t3 R: its Write applied.  t4 (unmanaged, deps t0..t3 committed): notifyUnmanaged(APPLY, next)
    # releases it once every committed txn up to its latest dep (t3) has applied -- not yet
    assert list(r3) == [3]
    d.apply(r3)
    assert list(d.round()) == [4]
    d.apply([4])
    assert list(d.round()) == []                          # t6 / t7 still wait for t5
    # t5 commits at its TxnId: no longer an uncommitted dep of t6, but now an unapplied Write before
    # it; t5 itself has no deps
    d.register([5], STABLE)
    assert list(d.round()) == [5]
    d.apply([5])
    assert list(d.round()) == [6]                         # t7 (W) waits for t6 (R)
    d.apply([6])
    assert list(d.round()) == [7]
    d.apply([7])
    assert d.ora.waiting == 0
    return d


def test_kat_oracle():
    kat_run()


# ---- the reference's event order (CommandsForKey.notifyAndUpdatePending, :1163-1215) ----
# The device (and or_lstore_ready) re-test a waiting txn whenever an input of its test changed; the
# reference tests it only when an event reaches the key.  KAT of the difference: t1 (R) waits for t0
# (W, uncommitted).  t0 COMMITs at an executeAt after t1: t1's test holds (nothing unapplied executes
# before it, no dep uncommitted), but a COMMITTED event executing no later than nextWrite (t0 itself)
# notifies nobody -- the reference releases t1 only at t0's STABLE event, one call later.
EV_KAT = [(10, "W", 1, [1], None), (11, "R", 1, [1], None)]


def test_event_order_kat():
    s = mk(EV_KAT)
    d = Driver(s, 4, events=True)
    part = d.batch(0, 2)
    d.register([1], STABLE)
    d.initialise(0, part)
    assert list(d.round()) == [] and list(d.ev_rounds[-1]) == []
    t0x = (int(s.msb[0]), 20 << 16 | int(s.lsb[0]) & 0xFFFF, 1)
    d.register([0], 4, [t0x])                             # COMMITTED at hlc 20
    assert list(d.round()) == [1]                         # device / polling: at once
    assert list(d.ev_rounds[-1]) == []                    # reference: not notified
    d.register([0], STABLE)
    assert list(d.round()) == [0]
    assert list(d.ev_rounds[-1]) == [0, 1]                # t0's STABLE event notifies t1


def event_schedule(s, nkeys, bsz, seed, late_frac=0.15, delay=0.2, cf=0.0, rounds=3):
    """The interleaved schedule of the GPU tests (batches; STABLE, some late, some at an executeAt past
    the TxnId, a share cf COMMITTED one batch before STABLE; ready -> APPLIED rounds), fed ONE event at a
    time to the polling restatement (or_lstore_ready, what the device computes) and to the event-driven
    one (or_lstore_event_mode), both asked for ready txns after every event.  Returns, per txn, the
    index of the event after which each released it (int64 max: never)."""
    rng = np.random.default_rng(seed)
    poll, ev = O.LStore(nkeys), O.LStore(nkeys, event_mode=True)
    never = np.iinfo(np.int64).max
    at_p, at_e = np.full(s.n, never, np.int64), np.full(s.n, never, np.int64)
    clock = [0]
    execs = [None] * s.n

    def step():
        for o, at in ((poll, at_p), (ev, at_e)):
            r = o.ready().astype(np.int64)
            at[r] = np.minimum(at[r], clock[0])
        clock[0] += 1

    def event(g, st):
        e = execs[g] or (int(s.msb[g]), int(s.lsb[g]), int(s.node[g]))
        for o in (poll, ev):
            o.register(s.msb[g:g + 1], s.lsb[g:g + 1], s.node[g:g + 1], np.array([st], np.uint8),
                       np.array([e[0]], np.uint64), np.array([e[1]], np.uint64), np.array([e[2]], np.int32))
        step()

    late, applied = np.zeros(0, np.int64), np.zeros(s.n, bool)
    for lo in range(0, s.n, bsz):
        hi = min(s.n, lo + bsz)
        part = poll.batch(s.slice(lo, hi))
        ev.batch(s.slice(lo, hi))
        idx = np.arange(lo, hi)
        is_late = rng.random(hi - lo) < late_frac
        now = np.concatenate([late, idx[~is_late]])
        first = []
        for g in now:
            if g >= lo and rng.random() < delay:
                execs[g] = (int(s.msb[g]), ((int(s.lsb[g]) >> 16) + int(rng.integers(1, 30))) << 16, int(rng.integers(8, 16)))
            if g >= lo and rng.random() < cf:
                first.append(g)
                event(g, 4)                                  # COMMITTED first, STABLE next batch
            else:
                event(g, STABLE)
        late = np.concatenate([idx[is_late], np.array(first, np.int64)]).astype(np.int64)
        poll.waiting_add(lo, part)
        ev.waiting_add(lo, part)
        step()
        for _ in range(rounds):                              # the polling releases are executed
            r = np.nonzero((at_p < never) & ~applied)[0]
            for g in r:
                applied[g] = True
                event(g, APPLIED)
    for g in np.sort(late):
        event(g, STABLE)
    for _ in range(5000):
        r = np.nonzero((at_p < never) & ~applied)[0]
        if r.size == 0:
            break
        for g in r:
            applied[g] = True
            event(g, APPLIED)
    return at_p, at_e


@pytest.mark.parametrize("seed,rf,sp,delay,cf", [(31, 0.0, False, 0.2, 0.0), (32, 0.1, False, 0.2, 0.0),
                                                (33, 0.1, True, 0.0, 0.0), (34, 0.05, False, 0.2, 0.3)])
def test_event_order_never_later(seed, rf, sp, delay, cf):
    """Event by event, the polling restatement (the device's semantics: tests/test_ready.py GPU cases
    check device == polling round by round) releases every txn the event-driven restatement releases
    no later; it releases some strictly earlier (EV_KAT: a test that holds between events), and a txn
    no event reaches stays for the reference's progress log.  (Between calls the device sees only the
    state after all of a call's events; a transient state inside one call -- e.g. next before a
    non-dep commits earlier -- can release an unmanaged APPLY record in the reference and not at the
    call's end: the device is event-exact at one event per call, as here.)"""
    s = stable_stream(900, 40, seed, rf, sync_points=sp)
    at_p, at_e = event_schedule(s, 40, 150, seed, delay=delay, cf=cf)
    never = np.iinfo(np.int64).max
    released = at_e < never
    assert released.sum() > s.n // 4
    assert (at_p[released] <= at_e[released]).all(), np.nonzero(at_p > at_e)[0][:10]
    print("event-driven releases", int(released.sum()), "of", s.n, "; polling earlier for",
          int((at_p[released] < at_e[released]).sum()), "; never reached by an event:", int((~released).sum()))


# removeRedundantDependencies (local/CommandStore.java:601-670) KAT over keys 0..13, every txn Write:
# t0 (0,4], t3 (4,8], t6 (6,10], t8 (8,12] are range txns that never commit; t1 range (0,2] and t2
# key 3 wait on t0; t4 key 6 and t5 keys {5, 9} on t3; t7 key 7 on t3, t6; t9 key 9 on t6, t8.
RR_KAT = [(10, "W", 1, None, [(0, 4)]), (11, "W", 1, None, [(0, 2)]), (12, "W", 1, [3], None),
          (13, "W", 1, None, [(4, 8)]), (14, "W", 1, [6], None), (15, "W", 1, [5, 9], None),
          (16, "W", 1, None, [(6, 10)]), (17, "W", 1, [7], None), (18, "W", 1, None, [(8, 12)]),
          (19, "W", 1, [9], None)]


def rr_kat_run(dev=None):
    s = mk(RR_KAT)
    d = Driver(s, 14, dev)
    part = d.batch(0, 10)
    d.register([1, 2, 4, 5, 7, 9], STABLE)
    d.initialise(0, part)
    assert list(d.round()) == []                          # every one waits on an uncommitted range txn
    # (0,4] locally applied before t1: t0 is redundant for t1, t2 (rule 1: [bootstrapIdx 0, appliedIdx 1));
    # (4,10] bootstrapped at t7: t3's range (4,8] lies inside it -> fully bootstrapping for t4, t5, t7
    # (rule 2); t6 (position 6 < 7) too, for t7; t9's deps t6 (6,10] covered, t8 (8,12] not (its
    # bootstrapIdx is 1: t8 follows t7)
    d.redundant(start=[0, 4], end=[4, 10], locally_applied=[1, NO_TXN], bootstrapped_at=[NO_TXN, 7])
    assert list(d.round()) == [1, 2, 4, 5, 7]
    d.apply([1, 2, 4, 5, 7])                              # t9's key 9 waits for t5 (a Write) to apply
    # bootstrapped at t9 over (4,10] and (10,12]: t8's range is covered only with (10,12], which t9's
    # key 9 does not touch -- not in the fold, so (10,12] remains and t9 keeps waiting
    d.redundant(start=[0, 4, 10], end=[4, 10, 12], locally_applied=[1, NO_TXN, NO_TXN],
                bootstrapped_at=[NO_TXN, 9, 9])
    assert list(d.round()) == []
    d.redundant(start=[0, 4], end=[4, 12], locally_applied=[1, NO_TXN], bootstrapped_at=[NO_TXN, 9])
    assert list(d.round()) == [9]
    return d


def test_rr_kat_oracle():
    rr_kat_run()


def test_rr_gate_epoch_oracle():
    """hasLocallyRedundantDependencies folds only in-bounds entries (Entry.outOfBounds): with the
    entry's epochs after the txns', nothing is removed."""
    s = mk(RR_KAT)
    d = Driver(s, 14)
    part = d.batch(0, 10)
    d.register([1, 2, 4, 5, 7, 9], STABLE)
    d.initialise(0, part)
    d.redundant(start=[0, 4], end=[4, 10], locally_applied=[1, NO_TXN], bootstrapped_at=[NO_TXN, 7],
                start_epoch=[5, 5], end_epoch=[9, 9])
    assert list(d.round()) == []


# executeAtLeast (WaitingOn.updateExecuteAtLeast, local/Command.java:1511-1514): t1, an
# ExclusiveSyncPoint over (0,2] (awaitsOnlyDeps), waits on t0 (key 1) committed at an executeAt after
# t1's TxnId (registerUnmanaged leaves an APPLY record: executesAt = t0's executeAt); t2 a range Write
# over (0,2] (not awaitsOnlyDeps: executesAtLeast = its own executeAt)
EAL_KAT = [(10, "W", 1, [1], None), (11, "XSP", 1, None, [(0, 2)]), (12, "W", 1, None, [(0, 2)])]


def eal_kat_run(dev=None):
    s = mk(EAL_KAT)
    d = Driver(s, 4, dev)
    part = d.batch(0, 3)
    t0x = (int(s.msb[0]), 30 << 16 | int(s.lsb[0]) & 0xFFFF, 1)    # t0 executes at hlc 30
    d.register([0, 1, 2], STABLE, [t0x, None, None])
    d.initialise(0, part)
    # t2 (not awaitsOnlyDeps) stops waiting for t0, which executes after it (removeWaitingOn)
    assert list(d.round()) == [0, 2]
    assert int(d.eal[1][1]) >> 16 == 12                            # t2: its own executeAt (= TxnId)
    d.apply([0, 2])
    assert list(d.round()) == [1]
    em, el, en = d.eal
    assert (int(em[0]), int(el[0]), int(en[0])) == t0x             # t1: the dep's executeAt
    return d


def test_eal_kat_oracle():
    eal_kat_run()


# executeAtLeast over candidates on different nodes: t2, an EphemeralRead of key 1 (awaitsOnlyDeps),
# has range deps t0 (executes at hlc 14 on node 13) and t1 (hlc 27 on node 9), both committed when
# its WaitingOn is initialised; Timestamp.max keeps every field of the later one (t1, node 9).  The
# device's running merge once combined t1's hlc with t0's node (profiles/r05_eal).
EAL_MIX_KAT = [(10, "W", 1, None, [(0, 2)]), (11, "W", 1, None, [(0, 2)]), (12, "ER", 1, [1], None)]


def eal_mix_run(dev=None):
    s = mk(EAL_MIX_KAT)
    d = Driver(s, 4, dev)
    part = d.batch(0, 3)
    x0 = (int(s.msb[0]), 14 << 16 | int(s.lsb[0]) & 0xFFFF, 13)
    x1 = (int(s.msb[1]), 27 << 16 | int(s.lsb[1]) & 0xFFFF, 9)
    d.register([0, 1, 2], STABLE, [x0, x1, None])
    d.initialise(0, part)
    for _ in range(4):
        r = list(d.round())
        if 2 in r:
            em, el, en = d.eal
            i = r.index(2)
            assert (int(em[i]), int(el[i]), int(en[i])) == x1
            return d
        d.apply(r)
    raise AssertionError("t2 never became ready")


def test_eal_mixed_nodes_oracle():
    eal_mix_run()


# setAppliedAndPropagate (local/Command.java:1569-1583): t1, a Range-domain ExclusiveSyncPoint
# (awaitsOnlyDeps), waits on t0, a range Write executing at hlc 30; t0 applied, t1 records it in its
# appliedOrInvalidated and is applied.  t2, another ExclusiveSyncPoint over the same range, is
# initialised only then: updateWaitingOn walks its range deps in reverse (forEachWaitingOnId), so t1
# comes first and propagates t0 -- t0's bit is cleared without its executeAt ever reaching
# updateExecuteAtLeast, and t2 executes at least at its own TxnId (hlc 12), not at t0's hlc 30.
PROP_KAT = [(10, "W", 1, None, [(0, 4)]), (11, "XSP", 1, None, [(0, 4)]), (12, "XSP", 1, None, [(0, 4)])]


def prop_kat_run(dev=None):
    s = mk(PROP_KAT)
    d = Driver(s, 6, dev)
    part = d.batch(0, 2)
    x0 = (int(s.msb[0]), 30 << 16 | int(s.lsb[0]) & 0xFFFF, 1)
    d.register([0, 1], STABLE, [x0, None])
    d.initialise(0, part)
    assert list(d.round()) == [0]
    d.apply([0])
    assert list(d.round()) == [1]
    em, el, en = d.eal
    assert (int(em[0]), int(el[0]), int(en[0])) == x0                # t1 waited on t0 (awaitsOnlyDeps)
    d.apply([1])
    part2 = d.batch(2, 3)
    assert list(part2.range_deps(0)[2]) == [0, 1], part2.range_deps(0)
    d.register([2], STABLE)
    d.initialise(2, part2)
    assert list(d.round()) == [2]
    em, el, en = d.eal
    assert (int(em[0]), int(el[0]), int(en[0])) == (int(s.msb[2]), int(s.lsb[2]), int(s.node[2]))
    return d


def test_propagate_kat_oracle():
    prop_kat_run()


# TruncatedApply carries its executeAt (ACCORD_ST_TRUNCATED_APPLY; local/SaveStatus.java:79-81): t0, a
# range Write over (0,2] committed at hlc 30, is TruncatedApply when t1 -- an ExclusiveSyncPoint over
# (0,2], awaitsOnlyDeps -- initialises its WaitingOn.  updateWaitingOn reads ExecuteAtKnown before the
# truncation branch (local/Commands.java:782-783), so t1 executes at least at t0's executeAt and its
# bit clears as applied-or-invalidated; with t0 Erased / Invalidated (INVALID: no executeAt) t1
# executes at its own TxnId.  t2, a range Write (not awaitsOnlyDeps) executing at its TxnId (hlc 12)
# before t0's executeAt, breaks checkState(executeAt < waitingExecuteAt || awaitsOnlyDeps) (:789-791):
# an IllegalStateException.
TRUNC_KAT = [(10, "W", 1, None, [(0, 2)]), (11, "XSP", 1, None, [(0, 2)]), (12, "W", 1, None, [(0, 2)])]
TRUNCATED_APPLY = 9


def trunc_kat_run(dev=None, status=TRUNCATED_APPLY):
    s = mk(TRUNC_KAT)
    d = Driver(s, 4, dev)
    part = d.batch(0, 2)
    x0 = (int(s.msb[0]), 30 << 16 | int(s.lsb[0]) & 0xFFFF, 1)
    d.register([0], STABLE, [x0])
    d.register([0], status, [x0])
    d.register([1], STABLE)
    d.initialise(0, part)
    assert list(d.round()) == [1]
    em, el, en = d.eal
    own = (int(s.msb[1]), int(s.lsb[1]), int(s.node[1]))
    assert (int(em[0]), int(el[0]), int(en[0])) == (x0 if status == TRUNCATED_APPLY else own)
    return d, s, x0


def trunc_kat_violation(dev=None):
    d, s, x0 = trunc_kat_run(dev)
    part = d.batch(2, 3)
    assert list(part.range_deps(0)[2]) == [0]           # a Write does not witness the ExclusiveSyncPoint
    d.register([2], STABLE)
    if dev is not None:
        with pytest.raises(IllegalStateException):
            dev.waiting_on_initialise()                 # the initial updateWaitingOn visits t0
        return
    d.ora.waiting_add(2, part)
    with pytest.raises(O.OracleError) as e:
        d.ora.ready_ex()
    assert e.value.rc == -10


def test_truncated_apply_kat_oracle():
    trunc_kat_run()
    trunc_kat_run(status=INVALID)
    trunc_kat_violation()


def test_truncated_apply_status_order_oracle():
    # statuses advance in SaveStatus order: TruncatedApply after Applied, before Invalid / Erased
    s = mk(TRUNC_KAT)
    L = O.LStore(4)
    L.batch(s)
    x = (s.msb[:1], s.lsb[:1], s.node[:1])
    L.register(*x, np.array([APPLIED], np.uint8), *x)
    L.register(*x, np.array([TRUNCATED_APPLY], np.uint8), *x)
    L.register(*x, np.array([INVALID], np.uint8), *x)
    with pytest.raises(O.OracleError):
        L.register(*x, np.array([TRUNCATED_APPLY], np.uint8), *x)     # back from Invalid
    L.close()


def stable_stream(n, ks, seed, range_frac=0.0, sync_points=False, range_len_max=8):
    s = generate_stream(n, 3, ks, 0.9, 0.5, seed=seed, range_frac=range_frac, range_len_max=range_len_max)
    # kinds: Read / Write / EphemeralRead (key txns); range txns keep their kind.  sync_points: also
    # SyncPoint / ExclusiveSyncPoint, key and range domain (Txn.Kind ordinals 3, 4)
    rng = np.random.default_rng(seed)
    if sync_points:
        k = rng.choice([0, 1, 2, 3, 4], size=n, p=[0.3, 0.4, 0.1, 0.1, 0.1]).astype(np.uint64)
        rk = rng.choice([0, 1, 3, 4], size=n, p=[0.3, 0.3, 0.2, 0.2]).astype(np.uint64)
    else:
        k = rng.choice([0, 1, 2], size=n, p=[0.4, 0.5, 0.1]).astype(np.uint64)
        rk = (s.lsb >> np.uint64(1)) & np.uint64(7)
    dom = s.lsb & np.uint64(1)
    kind = np.where(dom == 1, rk, k)
    lsb = (s.lsb & ~np.uint64(0xE)) | (kind << np.uint64(1))
    return Stream(s.msb, lsb, s.node, s.key_off, s.key_ord, s.rng_off, s.rng_start, s.rng_end)


@pytest.mark.parametrize("n,ks,seed,rf", [(600, 40, 1, 0.0), (800, 60, 2, 0.1), (500, 20, 3, 0.05)])
def test_all_stable_rounds_equal_cfk_simulation(n, ks, seed, rf):
    """Every txn STABLE at executeAt = TxnId from the start: the ready -> APPLIED rounds of the
    readiness restatement equal or_levels_cfk (an independent CommandsForKey-side simulation) on
    the same deps."""
    s = stable_stream(n, ks, seed, rf)
    d = Driver(s, ks)
    part = d.batch(0, n)
    d.register(np.arange(n), STABLE)
    d.initialise(0, part)
    rounds = drain(d)
    got = np.zeros(n, np.int64)
    for r, txns in enumerate(rounds):
        got[txns] = r
    assert sum(len(r) for r in rounds) == n
    want = O.levels_cfk(s, part)
    assert np.array_equal(got, want.astype(np.int64))


def schedule(s, nkeys, bsz, seed, dev=None, late_frac=0.15, delay_frac=0.2, rounds_per_batch=2, dev_events=False,
             driver=None):
    """Batches of bsz: computed, then STABLE for most txns (some at an executeAt past their TxnId),
    the rest (late) STABLE one batch later; WaitingOn initialised; a few ready -> APPLIED rounds per
    batch; finally drained.  Returns every round's ready list.  driver: another object with the
    Driver's interface (the golden replay below)."""
    rng = np.random.default_rng(seed)
    d = driver if driver is not None else Driver(s, nkeys, dev, dev_events=dev_events)
    out, late = [], np.zeros(0, np.int64)
    for lo in range(0, s.n, bsz):
        hi = min(s.n, lo + bsz)
        part = d.batch(lo, hi)
        idx = np.arange(lo, hi)
        is_late = rng.random(hi - lo) < late_frac
        now = np.concatenate([late, idx[~is_late]])
        execs = []
        for g in now:
            if g >= lo and rng.random() < delay_frac:
                execs.append((int(s.msb[g]), ((int(s.lsb[g]) >> 16) + int(rng.integers(1, 30))) << 16,
                              int(rng.integers(8, 16))))
            else:
                execs.append(None)
        d.register(now, STABLE, execs)
        late = idx[is_late]
        d.initialise(lo, part)
        for _ in range(rounds_per_batch):
            r = d.round()
            out.append(r)
            d.apply(r)
    d.register(late, STABLE)
    out.extend(drain(d))
    return out, d


def test_event_schedule_driver_oracle():
    """The event-exact comparison path of the Driver on the CPU (the GPU test's reference side)."""
    s = stable_stream(500, 30, 71, 0.1)
    out, d = schedule(s, 30, 100, 71, dev_events=True)
    assert sum(len(r) for r in out) > 500 // 4


def test_schedule_oracle_progress():
    """The schedule drains: every txn becomes ready exactly once."""
    s = stable_stream(1500, 50, 4, 0.05)
    out, d = schedule(s, 50, 300, 4)
    allr = np.concatenate(out)
    assert np.array_equal(np.sort(allr), np.arange(s.n))
    assert d.ora.waiting == 0


# ---- GPU: the device readiness == the oracle, round by round ----

@pytest.mark.gpu
def test_gpu_kat(gpu_device):
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        kat_run(dev)


@pytest.mark.gpu
def test_gpu_rr_kat(gpu_device):
    with CommandStore(device=gpu_device, key_lo=0, key_hi=14, window=WINDOW_NONE, resident=True) as dev:
        rr_kat_run(dev)


@pytest.mark.gpu
def test_gpu_eal_kat(gpu_device):
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        eal_kat_run(dev)


@pytest.mark.gpu
def test_gpu_event_order_kat(gpu_device):
    """EV_KAT on the device in event-exact mode: t1 is released only at t0's STABLE event."""
    s = mk(EV_KAT)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        d = Driver(s, 4, dev, dev_events=True)
        part = d.batch(0, 2)
        d.register([1], STABLE)
        d.initialise(0, part)
        assert list(d.round()) == []
        t0x = (int(s.msb[0]), 20 << 16 | int(s.lsb[0]) & 0xFFFF, 1)
        d.register([0], 4, [t0x])                         # COMMITTED: notifies nobody
        assert list(d.round()) == []
        d.register([0], STABLE)
        assert list(d.round()) == [0, 1]


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed,rf,sp", [(600, 30, 100, 71, 0.0, False), (700, 40, 140, 72, 0.1, False),
                                                  (600, 30, 120, 73, 0.1, True)])
def test_gpu_event_mode_equals_event_oracle(gpu_device, n, ks, bsz, seed, rf, sp):
    """Event-exact device readiness == or_lstore_event_mode call by call over the interleaved
    schedule (batches; STABLE in bulk registrations, some late, some past their TxnId; ready ->
    APPLIED rounds), incl. range txns (unmanaged records) and sync points."""
    s = stable_stream(n, ks, seed, rf, sync_points=sp)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, d = schedule(s, ks, bsz, seed, dev=dev, dev_events=True)
    # every call compared inside Driver.round; the event-driven reference releases fewer (sync points
    # wait for an event that may never reach their keys)
    assert sum(len(r) for r in out) > 0


# Event-exact readiness at 20k txns: the event restatement takes ~9 min on one core for this
# schedule, so its per-call releases and executesAtLeast are frozen in tests/golden/events_20k.npz
# (tests/golden/make_event_golden.py) and the device replays the same schedule against them.
EV20K = dict(n=20000, ks=2000, bsz=1000, seed=91, rf=0.05)


class GoldenReplay:
    """Driver's interface over the device alone: every ready call compared with the frozen
    event-restatement output of the same call (releases, executesAtLeast, waiting count)."""

    def __init__(self, s, dev, g):
        self.s, self.dev, self.g, self.call = s, dev, g, 0
        self.execs = [None] * s.n
        dev.ready_mode(True)

    def batch(self, lo, hi):
        self.dev.calculate_deps_batch(self.s.slice(lo, hi))
        return None

    def register(self, idx, st, execs=None):
        idx = np.asarray(idx, np.int64)
        if idx.size == 0:
            return
        order = np.argsort(idx)
        idx = idx[order]
        s = self.s
        em = s.msb[idx].copy(); el = s.lsb[idx].copy(); en = s.node[idx].copy()
        for r, g in enumerate(idx):
            if execs is not None and execs[order[r]] is not None:
                self.execs[g] = execs[order[r]]
            if self.execs[g] is None:
                self.execs[g] = (int(s.msb[g]), int(s.lsb[g]), int(s.node[g]))
            em[r], el[r], en[r] = self.execs[g]
        self.dev.register(s.msb[idx], s.lsb[idx], s.node[idx], np.full(idx.size, st, np.uint8), em, el, en)

    def initialise(self, lo, part):
        self.dev.waiting_on_initialise()

    def round(self):
        g, c = self.g, self.call
        a, b = int(g["off"][c]), int(g["off"][c + 1])
        want = g["txn"][a:b]
        got, waiting, geal = self.dev.ready_update_ex()
        assert np.array_equal(got, want), (c, got[:20], want[:20])
        assert waiting == int(g["waiting"][c]), (c, waiting, int(g["waiting"][c]))
        for x, y in zip(geal, (g["eal_msb"][a:b], g["eal_lsb"][a:b], g["eal_node"][a:b])):
            assert np.array_equal(x, y), c
        self.call += 1
        return want

    def apply(self, ready):
        self.register(ready, APPLIED)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_event_mode_20k_golden(gpu_device):
    """Event-exact device readiness over 20,000 txns (2,000 keys, 5 % range txns) == the frozen
    or_lstore_event_mode output, call by call."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "events_20k.npz"))
    p = EV20K
    s = stable_stream(p["n"], p["ks"], p["seed"], p["rf"])
    with CommandStore(device=gpu_device, key_lo=0, key_hi=p["ks"], window=WINDOW_NONE, resident=True) as dev:
        d = GoldenReplay(s, dev, g)
        out, _ = schedule(s, p["ks"], p["bsz"], p["seed"], driver=d)
    assert d.call == len(g["off"]) - 1
    assert sum(len(r) for r in out) == int(g["released"])


def single_event_schedule(s, nkeys, bsz, seed, dev=None, cf=0.3, delay=0.2, rounds=3):
    """event_schedule's shape through the Driver: ONE event per registration (a share cf COMMITTED one
    batch before STABLE, executeAt sometimes past the TxnId), a ready call after every event and its
    releases applied at once; the device (if any) runs event-exact and is compared at every call."""
    rng = np.random.default_rng(seed)
    d = Driver(s, nkeys, dev, dev_events=True)
    total = [0]

    def event(g, st, ex=None):
        d.register([g], st, [ex] if ex is not None else None)
        r = d.round()
        total[0] += len(r)
        if len(r):
            d.apply(r)
            total[0] += 0

    late = np.zeros(0, np.int64)
    for lo in range(0, s.n, bsz):
        hi = min(s.n, lo + bsz)
        part = d.batch(lo, hi)
        idx = np.arange(lo, hi)
        is_late = rng.random(hi - lo) < 0.15
        now = np.concatenate([late, idx[~is_late]])
        first = []
        for g in now:
            ex = None
            if g >= lo and rng.random() < delay:
                ex = (int(s.msb[g]), ((int(s.lsb[g]) >> 16) + int(rng.integers(1, 30))) << 16, int(rng.integers(8, 16)))
            if g >= lo and rng.random() < cf:
                first.append(g)
                event(g, 4, ex if ex is not None else (int(s.msb[g]), int(s.lsb[g]), int(s.node[g])))
            else:
                event(g, STABLE, ex)
        late = np.concatenate([idx[is_late], np.array(first, np.int64)]).astype(np.int64)
        d.initialise(lo, part)
        for _ in range(rounds):
            r = d.round()
            total[0] += len(r)
            if len(r):
                d.apply(r)
    for g in np.sort(late):
        event(int(g), STABLE)
    for _ in range(2000):
        r = d.round()
        if not len(r):
            break
        total[0] += len(r)
        d.apply(r)
    return total[0], d


def test_single_event_schedule_oracle():
    s = stable_stream(300, 20, 81, 0.1)
    released, _ = single_event_schedule(s, 20, 60, 81)
    assert released > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed,rf,sp", [(400, 20, 80, 81, 0.1, False), (400, 24, 100, 82, 0.1, True)])
def test_gpu_event_mode_single_events(gpu_device, n, ks, bsz, seed, rf, sp):
    """Event-exact device readiness == or_lstore_event_mode with one event per registration and a
    ready call after each, COMMITTED-before-STABLE events included (their nextWrite skip)."""
    s = stable_stream(n, ks, seed, rf, sync_points=sp)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        released, _ = single_event_schedule(s, ks, bsz, seed, dev=dev)
    assert released > 0


@pytest.mark.gpu
def test_gpu_ready_mode_guards(gpu_device):
    """accord_ready_set_mode: registered-status stores only, never with txns waiting; the mode
    survives accord_store_reset (a store setting, not state)."""
    s = mk(EV_KAT)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=256) as plain:
        with pytest.raises(IllegalStateException):
            plain.ready_mode(True)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        dev.ready_mode(True)
        d = Driver(s, 4, dev, dev_events=True)
        part = d.batch(0, 2)
        d.register([0, 1], STABLE)
        d.initialise(0, part)
        with pytest.raises(IllegalStateException):
            dev.ready_mode(False)                         # txns wait
        assert list(d.round()) == [0]
        dev.reset()
        dev.ready_mode(False)


@pytest.mark.gpu
def test_gpu_propagate_kat(gpu_device):
    with CommandStore(device=gpu_device, key_lo=0, key_hi=6, window=WINDOW_NONE, resident=True) as dev:
        prop_kat_run(dev)


@pytest.mark.gpu
def test_gpu_truncated_apply_kat(gpu_device):
    for status in (TRUNCATED_APPLY, INVALID):
        with CommandStore(device=0, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
            trunc_kat_run(dev, status)
    with CommandStore(device=0, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        trunc_kat_violation(dev)
    with CommandStore(device=0, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        s = mk(TRUNC_KAT)
        dev.calculate_deps_batch(s)
        x = (s.msb[:1], s.lsb[:1], s.node[:1])
        dev.register(*x, np.array([INVALID], np.uint8), *x)
        with pytest.raises(IllegalStateException):
            dev.register(*x, np.array([TRUNCATED_APPLY], np.uint8), *x)   # statuses never go back


@pytest.mark.gpu
def test_gpu_eal_mixed_nodes(gpu_device):
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        eal_mix_run(dev)


def schedule_rr(s, nkeys, bsz, seed, dev=None, late_frac=0.1, rounds_per_batch=4, nent=5, remove=True):
    """Range and key txns, some committing two batches late (late_frac), and after every batch a new
    RedundantBefore map of nent entries over the keyspace with random locallyAppliedOrInvalidatedBefore
    (mostly recent) / bootstrappedAt positions (some NONE, some stale): readiness removes redundant
    range deps (removeRedundantDependencies) == the oracle's literal fold, round by round.
    remove=False: the same maps with NONE bounds (nothing removable).  Returns the rounds and the driver."""
    rng = np.random.default_rng(seed)
    d = Driver(s, nkeys, dev)
    out, late = [], []
    for b, lo in enumerate(range(0, s.n, bsz)):
        hi = min(s.n, lo + bsz)
        part = d.batch(lo, hi)
        idx = np.arange(lo, hi)
        is_late = rng.random(hi - lo) < late_frac
        d.register(idx[~is_late], STABLE)
        if b >= 2 and late[b - 2].size:
            d.register(late[b - 2], STABLE)
        late.append(idx[is_late])
        d.initialise(lo, part)
        cuts = np.sort(rng.choice(np.arange(1, nkeys - 1), size=nent - 1, replace=False))
        bounds = np.concatenate([[0], cuts, [nkeys - 1]])
        keep = rng.random(nent) < 0.8                       # a few gaps in the map
        st, en = bounds[:-1][keep], bounds[1:][keep]
        m = len(st)
        loc = np.where(rng.random(m) < 0.7, rng.integers(max(0, hi - 2 * bsz), hi + 1, m), NO_TXN).astype(np.uint32)
        boot = np.where(rng.random(m) < 0.4, rng.integers(0, hi + 1, m), NO_TXN).astype(np.uint32)
        # Entry.merge clears a locallyAppliedOrInvalidatedBefore at or below bootstrappedAt
        loc = np.where((boot != NO_TXN) & (loc != NO_TXN) & (boot >= loc), NO_TXN, loc).astype(np.uint32)
        stale = (rng.random(m) < 0.1).astype(np.uint8)
        if not remove:
            loc[:] = NO_TXN; boot[:] = NO_TXN; stale[:] = 0
        d.redundant(start=st, end=en, locally_applied=loc, bootstrapped_at=boot, stale=stale)
        for _ in range(rounds_per_batch):
            r = d.round()
            out.append(r)
            d.apply(r)
    for x in late[-2:]:
        d.register(x, STABLE)
    out.extend(drain(d))
    return out, d


@pytest.mark.parametrize("seed", [21, 22])
def test_schedule_rr_oracle(seed):
    """The maps release range-dep waiters earlier than the same schedule without removable bounds."""
    s = stable_stream(900, 30, seed, 0.25, sync_points=True)
    out, d = schedule_rr(s, 30, 150, seed)
    got = np.concatenate(out)
    assert np.unique(got).size == got.size
    out0, _ = schedule_rr(s, 30, 150, seed, remove=False)
    nb = (900 // 150) * 4                                  # rounds before the final drain
    assert sum(len(r) for r in out[:nb]) > sum(len(r) for r in out0[:nb])


def spill_stream():
    """Range txns up to 300 keys long over 400 keys, maps of 200 entries: most range txns touch more
    RedundantBefore entries than the removal's LDS scratch holds (RR_MAXE = 64)."""
    return stable_stream(700, 400, 31, 0.3, sync_points=True, range_len_max=300)


def test_schedule_rr_spill_shape():
    """The spill schedule really exceeds the LDS caps: some range txn's ranges meet > 64 map entries."""
    s = spill_stream()
    wide = [int(np.sum(s.rng_end[s.rng_off[i]:s.rng_off[i + 1]] - s.rng_start[s.rng_off[i]:s.rng_off[i + 1]]))
            for i in range(s.n) if s.rng_off[i + 1] > s.rng_off[i]]
    assert max(wide) > 2 * 64 * 400 // 200


@pytest.mark.gpu
def test_gpu_schedule_rr_spill(gpu_device):
    """Txns over the removal's LDS caps go through the HBM spill pass: no capacity error,
    and device == the literal oracle fold round by round, at initialise and at every evaluation."""
    s = spill_stream()
    with CommandStore(device=gpu_device, key_lo=0, key_hi=400, window=WINDOW_NONE, resident=True) as dev:
        out, d = schedule_rr(s, 400, 175, 31, dev, nent=200)
    got = np.concatenate(out)
    assert np.array_equal(np.sort(got), np.arange(s.n))


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed,rf", [(2000, 40, 250, 23, 0.25), (3000, 100, 500, 24, 0.15)])
def test_gpu_schedule_rr_equals_oracle(gpu_device, n, ks, bsz, seed, rf):
    """removeRedundantDependencies + executeAtLeast under random maps: device == literal oracle fold."""
    s = stable_stream(n, ks, seed, rf, sync_points=True)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, d = schedule_rr(s, ks, bsz, seed, dev)


@pytest.mark.gpu
def test_gpu_initialise_twice(gpu_device):
    """A second accord_waiting_on_initialise of the same batch replaces its unevaluated generation (no
    txn reported twice, the waiting count unchanged); after an accord_ready_update has evaluated it,
    a third is refused (its released txns were reported already)."""
    from accord_amd import IllegalStateException
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        s = mk(KAT)
        d = Driver(s, 4, dev)
        part = d.batch(0, 8)
        d.register([0, 1, 2, 3, 4, 6, 7], STABLE)
        d.initialise(0, part)
        dev.waiting_on_initialise()                       # again: replaces the first generation
        assert list(d.round()) == [0]                     # Driver.round: == oracle, waiting counts equal
        with pytest.raises(IllegalStateException):
            dev.waiting_on_initialise()
        d.apply([0])
        assert list(d.round()) == [1]


@pytest.mark.gpu
def test_gpu_initialise_failure_leaves_set(gpu_device, monkeypatch):
    """A generation that fails half built (ACCORD_INJECT_FAIL=ready_gen: after its buffers are
    allocated and partly copied) never joins the waiting set: the waiting count and the next calls
    are those of the set without it, and initialising the batch again afterwards works."""
    from accord_amd import AccordError
    with CommandStore(device=gpu_device, key_lo=0, key_hi=4, window=WINDOW_NONE, resident=True) as dev:
        s = mk(KAT)
        d = Driver(s, 4, dev)
        part = d.batch(0, 4)
        d.register([0, 1, 2, 3], STABLE)
        d.initialise(0, part)
        part2 = d.batch(4, 8)
        d.register([4, 6, 7], STABLE)
        monkeypatch.setenv("ACCORD_INJECT_FAIL", "ready_gen")
        with pytest.raises(AccordError):
            dev.waiting_on_initialise()
        monkeypatch.delenv("ACCORD_INJECT_FAIL")
        assert list(d.round()) == [0]                     # == the oracle, which has only batch 1 waiting
        d.apply([0])
        d.initialise(4, part2)                            # the retry joins batch 2
        released = [0] + [int(x) for r in drain(d) for x in r]   # every round == the oracle
        assert sorted(released) == [0, 1, 2, 3, 4]        # t5 stays PREACCEPTED: t6 / t7 wait on it


def test_sync_points_oracle_progress():
    """SyncPoints / ExclusiveSyncPoints (awaitsOnlyDeps, witness everything) at executeAt = TxnId
    drain too.  (With executeAts past the TxnId a range XSP's unmanaged APPLY record can wait for a
    later key-domain XSP that waits for it in turn -- the restated notifyUnmanaged holds the XSP until
    every committed txn of the key executing before its last dep has applied; the GPU test below
    checks the device against the restatement round by round there, without a drain assertion.)"""
    s = stable_stream(1500, 40, 13, 0.1, sync_points=True)
    out, d = schedule(s, 40, 300, 13, delay_frac=0.0)
    assert np.array_equal(np.sort(np.concatenate(out)), np.arange(s.n))


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed,delay", [(3000, 60, 300, 14, 0.0), (5000, 400, 1000, 15, 0.0),
                                                 (3000, 60, 300, 16, 0.2)])
def test_gpu_sync_points_equal_oracle(gpu_device, n, ks, bsz, seed, delay):
    s = stable_stream(n, ks, seed, 0.1, sync_points=True)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, d = schedule(s, ks, bsz, seed, dev, delay_frac=delay)    # == oracle at every round
    got = np.concatenate(out)
    assert np.unique(got).size == got.size
    if delay == 0.0:
        assert np.array_equal(np.sort(got), np.arange(n))


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed,rf", [(3000, 80, 500, 5, 0.0), (4000, 200, 400, 6, 0.08),
                                              (2500, 30, 250, 7, 0.1), (6000, 500, 1000, 8, 0.05)])
def test_gpu_schedule_equals_oracle(gpu_device, n, ks, bsz, seed, rf):
    s = stable_stream(n, ks, seed, rf)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, d = schedule(s, ks, bsz, seed, dev)
    assert np.array_equal(np.sort(np.concatenate(out)), np.arange(n))


@pytest.mark.gpu
def test_gpu_all_stable_levels(gpu_device):
    """All STABLE at TxnId in one batch: the device's ready rounds equal or_levels_cfk."""
    n, ks = 3000, 100
    s = stable_stream(n, ks, 9, 0.05)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        d = Driver(s, ks, dev)
        part = d.batch(0, n)
        d.register(np.arange(n), STABLE)
        d.initialise(0, part)
        rounds = drain(d)
    got = np.zeros(n, np.int64)
    for r, txns in enumerate(rounds):
        got[txns] = r
    assert np.array_equal(got, O.levels_cfk(s, part).astype(np.int64))


# ---- RedundantBefore truncation and invalidations under readiness ----

def redundant(s, lo, hi, ks, bound):
    """RedundantBefore.collectDeps of txns [lo, hi) under the one-entry map (as
    tests/test_registered_schedule.py)."""
    return O.redundant_collect(s.prefix(hi), **rb_map(ks, bound), min_epoch=0).txns(lo, hi)


def schedule_rb(s, nkeys, bsz, seed, dev=None, inval_frac=0.05, rb_every=3, rounds_per_batch=3, dev_events=False):
    """Batches STABLE at executeAt = TxnId except a few txns INVALIDATED (they never become ready;
    their dependents stop waiting for them), a few ready -> APPLIED rounds per batch, and every
    rb_every batches the store's RedundantBefore moves to shardAppliedOrInvalidatedBefore (the
    first txn not yet APPLIED / INVALID): CommandsForKey.withRedundantBefore truncates the keys'
    histories (a new carry on the device: everything re-evaluated) and collectDeps adds the bound to
    the next batches' deps.  Returns every round's ready list, the invalidated txns and the driver."""
    rng = np.random.default_rng(seed)
    d = Driver(s, nkeys, dev, dev_events=dev_events)
    out, bound, inval = [], None, []
    for b, lo in enumerate(range(0, s.n, bsz)):
        hi = min(s.n, lo + bsz)
        part = d.ora.batch(s.slice(lo, hi))
        if d.ev is not None:
            d.ev.batch(s.slice(lo, hi))
        if bound is not None:
            part = O.deps_union([part, redundant(s, lo, hi, nkeys, bound)])
        if dev is not None:
            got = dev.calculate_deps_batch(s.slice(lo, hi))
            assert got.first_difference(part) is None, got.first_difference(part)
        d.status[lo:hi] = 2
        idx = np.arange(lo, hi)
        bad = rng.random(hi - lo) < inval_frac
        d.register(idx[~bad], STABLE)
        d.register(idx[bad], INVALID)
        inval.extend(idx[bad].tolist())
        d.initialise(lo, part)
        for _ in range(rounds_per_batch):
            r = d.round()
            out.append(r)
            d.apply(r)
        if b % rb_every == rb_every - 1:
            done = (d.status[:hi] == APPLIED) | (d.status[:hi] == INVALID)
            p = int(np.argmin(done)) if not done.all() else hi - 1
            if p > 0 and (bound is None or p > bound):
                m = rb_map(nkeys, p)
                d.ora.truncate(m["start"], m["end"], m["bound"])
                if d.ev is not None:                     # event mode: notifyAndUpdatePending(prevCfk)
                    d.ev.truncate(m["start"], m["end"], m["bound"])
                if dev is not None:
                    dev.redundant_before(**m, min_epoch=0)
                bound = p
    out.extend(drain(d))
    return out, np.array(sorted(inval), np.int64), d


def test_schedule_rb_oracle_progress():
    s = stable_stream(1800, 40, 10)
    out, inval, d = schedule_rb(s, 40, 300, 10)
    allr = np.concatenate(out)
    assert np.array_equal(np.sort(np.concatenate([allr, inval])), np.arange(s.n))
    assert d.ora.waiting == 0                            # invalidated txns leave the set, never ready


def test_schedule_rb_events_oracle():
    s = stable_stream(900, 30, 13, 0.1)
    out, _, _ = schedule_rb(s, 30, 150, 13, dev_events=True)
    assert sum(len(r) for r in out) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed,rf", [(1500, 40, 250, 13, 0.1), (1200, 30, 200, 14, 0.0)])
def test_gpu_event_mode_truncation(gpu_device, n, ks, bsz, seed, rf):
    """Event-exact mode with invalidations and RedundantBefore truncations (the truncated keys'
    unmanaged records notified, or_lstore_truncate's notifyAndUpdatePending) == the event oracle."""
    s = stable_stream(n, ks, seed, rf)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, _, _ = schedule_rb(s, ks, bsz, seed, dev, dev_events=True)
    assert sum(len(r) for r in out) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed", [(3000, 60, 300, 11), (5000, 300, 500, 12)])
def test_gpu_schedule_rb_equals_oracle(gpu_device, n, ks, bsz, seed):
    s = stable_stream(n, ks, seed)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, inval, d = schedule_rb(s, ks, bsz, seed, dev)
    assert np.array_equal(np.sort(np.concatenate(out + [inval])), np.arange(n))
