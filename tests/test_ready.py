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

from accord_amd import CommandStore, Stream, WINDOW_NONE, generate_stream
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

    def __init__(self, s, nkeys, dev=None):
        self.s, self.ora, self.dev = s, O.LStore(nkeys), dev
        self.status = np.zeros(s.n, np.uint8)
        self.execs = [None] * s.n

    def batch(self, lo, hi):
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
        if self.dev is not None:
            self.dev.register(s.msb[idx], s.lsb[idx], s.node[idx], stv, em, el, en)
        self.status[idx] = st

    def initialise(self, lo, part):
        self.ora.waiting_add(lo, part)
        if self.dev is not None:
            self.dev.waiting_on_initialise()

    def round(self):
        want = self.ora.ready()
        if self.dev is not None:
            got, waiting = self.dev.ready_update()
            assert np.array_equal(got, want), (got[:20], want[:20])
            assert waiting == self.ora.waiting
        return want

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


def stable_stream(n, ks, seed, range_frac=0.0, sync_points=False):
    s = generate_stream(n, 3, ks, 0.9, 0.5, seed=seed, range_frac=range_frac, range_len_max=8)
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


def schedule(s, nkeys, bsz, seed, dev=None, late_frac=0.15, delay_frac=0.2, rounds_per_batch=2):
    """Batches of bsz: computed, then STABLE for most txns (some at an executeAt past their TxnId),
    the rest (late) STABLE one batch later; WaitingOn initialised; a few ready -> APPLIED rounds per
    batch; finally drained.  Returns every round's ready list."""
    rng = np.random.default_rng(seed)
    d = Driver(s, nkeys, dev)
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


def schedule_rb(s, nkeys, bsz, seed, dev=None, inval_frac=0.05, rb_every=3, rounds_per_batch=3):
    """Batches STABLE at executeAt = TxnId except a few txns INVALIDATED (they never become ready;
    their dependents stop waiting for them), a few ready -> APPLIED rounds per batch, and every
    rb_every batches the store's RedundantBefore moves to shardAppliedOrInvalidatedBefore (the
    first txn not yet APPLIED / INVALID): CommandsForKey.withRedundantBefore truncates the keys'
    histories (a new carry on the device: everything re-evaluated) and collectDeps adds the bound to
    the next batches' deps.  Returns every round's ready list, the invalidated txns and the driver."""
    rng = np.random.default_rng(seed)
    d = Driver(s, nkeys, dev)
    out, bound, inval = [], None, []
    for b, lo in enumerate(range(0, s.n, bsz)):
        hi = min(s.n, lo + bsz)
        part = d.ora.batch(s.slice(lo, hi))
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


@pytest.mark.gpu
@pytest.mark.parametrize("n,ks,bsz,seed", [(3000, 60, 300, 11), (5000, 300, 500, 12)])
def test_gpu_schedule_rb_equals_oracle(gpu_device, n, ks, bsz, seed):
    s = stable_stream(n, ks, seed)
    with CommandStore(device=gpu_device, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as dev:
        out, inval, d = schedule_rb(s, ks, bsz, seed, dev)
    assert np.array_equal(np.sort(np.concatenate(out + [inval])), np.arange(n))
