"""Real status events on a resident store (SURVEY.md §8a a4, §8b accord_txn_register, §8f row 1):
no status-at-time model (window ACCORD_WINDOW_NONE); batches enter PREACCEPTED, InternalStatus /
executeAt events arrive between batches, and every batch's deps must equal the stateful literal
oracle fed the same batches and events (real CommandsForKey objects: insert, update, committed[]
rebuilt per change, mapReduceActive with maxCommittedBefore pruning, local/CommandsForKey.java:
422-470, 614-706)."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalArgumentException, IllegalStateException, WINDOW_NONE, generate_stream
import oracle_lib as O
from status_events import APPLIED, COMMITTED, ERASED, INVALID, PREACCEPTED, events_for

pytestmark = pytest.mark.gpu


def run(s, ks, pts, seed, frac=0.5, delay=40, accept=None, erased=False):
    rng = np.random.default_rng(seed)
    status = np.full(s.n, PREACCEPTED, np.uint8)
    execs = [None] * s.n
    ora = O.LStore(ks)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as st:
        for b, (a, c) in enumerate(zip(pts[:-1], pts[1:])):
            part = s.slice(a, c) if accept is None else accept.slice(a, c)
            got = st.calculate_deps_batch(part)
            want = ora.batch(part)
            diff = got.first_difference(want)
            assert diff is None, (b, diff)
            idx, stt, em, el, en = events_for(s, 0, c, status, execs, rng, frac=frac, delay=delay, erased=erased)
            st.register(s.msb[idx], s.lsb[idx], s.node[idx], stt, em, el, en)
            ora.register(s.msb[idx], s.lsb[idx], s.node[idx], stt, em, el, en)
        return st.state()


@pytest.mark.parametrize("n,k,ks,z,wf,parts,seed", [
    (4000, 4, 300, 0.99, 0.5, 6, 1),
    (3000, 2, 40, 0.0, 0.7, 10, 2),        # hot keys: long general-path histories
    (5000, 8, 2000, 0.99, 0.3, 4, 3),
    (2000, 3, 10, 0.0, 1.0, 12, 4),        # all writes on 10 keys
])
def test_events_match_literal_oracle(gpu_device, n, k, ks, z, wf, parts, seed):
    s = generate_stream(n, k, ks, z, wf, seed=seed)
    pts = [i * n // parts for i in range(parts + 1)]
    run(s, ks, pts, seed)


def test_events_uneven_batches(gpu_device):
    # batches that grow and shrink: after the first, the compute fills speculatively into the arrays
    # (and the general pass's history extension) an earlier batch sized -- a larger batch aborts it,
    # grows them and fills again (store.cpp, SpecCheck); the deps stay the oracle's
    s = generate_stream(6000, 4, 150, 0.99, 0.5, seed=31)
    run(s, 150, [0, 60, 2500, 2560, 2700, 6000], 31)


def test_events_with_accept_batches(gpu_device):
    s = generate_stream(3000, 4, 200, 0.99, 0.5, seed=5)
    acc = s.accept(frac=0.5, max_delay=30, seed=5)
    run(s, 200, [0, 700, 1500, 2200, 3000], 5, accept=acc)


def test_truncated_entries_leave_the_state(gpu_device):
    s = generate_stream(4000, 4, 100, 0.0, 0.5, seed=6)
    with CommandStore(device=0, key_lo=0, key_hi=100, window=WINDOW_NONE, resident=True) as st:
        st.calculate_deps_batch(s.slice(0, 2000))
        before = st.state()["carry_entries"]
        idx = np.arange(0, 1500)
        ex = (s.msb[idx], s.lsb[idx], s.node[idx])
        st.register(s.msb[idx], s.lsb[idx], s.node[idx], np.full(idx.size, APPLIED, np.uint8), *ex)
        st.register(s.msb[idx], s.lsb[idx], s.node[idx], np.full(idx.size, INVALID, np.uint8))
        st.calculate_deps_batch(s.slice(2000, 2001))
        after = st.state()["carry_entries"]
        assert after < before - 1500 * 4 * 0.9


def test_register_errors_apply_nothing(gpu_device):
    s = generate_stream(200, 2, 50, 0.0, 0.5, seed=7)
    with CommandStore(device=0, key_lo=0, key_hi=50, window=256, resident=True) as st:
        st.calculate_deps_batch(s)
        with pytest.raises(IllegalStateException):          # the status-at-time model is in force
            st.register(s.msb[:1], s.lsb[:1], s.node[:1], [APPLIED], s.msb[:1], s.lsb[:1], s.node[:1])
    with CommandStore(device=0, key_lo=0, key_hi=50, window=WINDOW_NONE, resident=True) as st:
        st.calculate_deps_batch(s.slice(0, 100))
        ex = (s.msb[:2], s.lsb[:2], s.node[:2])
        st.register(s.msb[:2], s.lsb[:2], s.node[:2], [COMMITTED, COMMITTED], *ex)
        with pytest.raises(IllegalStateException):          # goes back
            st.register(s.msb[:1], s.lsb[:1], s.node[:1], [PREACCEPTED])
        with pytest.raises(IllegalArgumentException):       # not a txn of the store (yet)
            st.register(s.msb[150:151], s.lsb[150:151], s.node[150:151], [PREACCEPTED])
        with pytest.raises(IllegalArgumentException):       # unsorted
            st.register(s.msb[[3, 2]], s.lsb[[3, 2]], s.node[[3, 2]], [PREACCEPTED, PREACCEPTED])
        # a rejected call applied nothing: t1 can still be committed at its TxnId
        st.register(s.msb[1:2], s.lsb[1:2], s.node[1:2], [APPLIED], s.msb[1:2], s.lsb[1:2], s.node[1:2])


@pytest.mark.parametrize("n,k,ks,rf,rl,parts,seed", [
    (3000, 4, 300, 0.2, 40, 6, 11),
    (2000, 2, 60, 0.3, 10, 8, 12),          # hot keys, short ranges
    (2500, 6, 1000, 0.1, 300, 5, 13),
])
def test_range_txns_with_events(gpu_device, n, k, ks, rf, rl, parts, seed):
    # range commands stay until ERASED (SaveStatus >= Erased); INVALID_OR_TRUNCATED ones are still
    # visited (SURVEY.md §8c KAT 5); range txns' KeyDeps run the CFK filter on their ranges' keys
    s = generate_stream(n, k, ks, 0.99, 0.5, range_frac=rf, range_len_max=rl, seed=seed)
    pts = [i * n // parts for i in range(parts + 1)]
    run(s, ks, pts, seed, erased=True)


def test_range_txns_with_events_accept(gpu_device):
    s = generate_stream(2500, 4, 300, 0.99, 0.5, range_frac=0.2, range_len_max=50, seed=14)
    acc = s.accept(frac=0.5, max_delay=30, seed=14)
    run(s, 300, [0, 600, 1300, 1900, 2500], 14, accept=acc, erased=True)


def test_kat5_erased_or_invalidated_on_gpu(gpu_device):
    # SURVEY.md §8c KAT 5 through the C ABI (the oracle KAT: test_oracle_events.py): a range command
    # at INVALID_OR_TRUNCATED (ErasedOrInvalidated) is still a dependency, at ERASED it is not
    from test_oracle_events import mk_mixed, range_deps_of, reg
    s = mk_mixed([(10, "W", 1, None, [(0, 5)]), (11, "W", 1, None, [(3, 9)]), (12, "W", 1, [4], None),
                  (13, "W", 1, [4], None), (14, "W", 1, [4], None)])
    ora = O.LStore(16)
    with CommandStore(device=0, key_lo=0, key_hi=16, window=WINDOW_NONE, resident=True) as st:
        def both(a, b):
            got, want = st.calculate_deps_batch(s.slice(a, b)), ora.batch(s.slice(a, b))
            assert got.first_difference(want) is None
            return got
        assert range_deps_of(both(0, 3), 2) == {(0, 5): [0], (3, 9): [1]}
        reg(st, s, [0], [INVALID]); reg(ora, s, [0], [INVALID])
        assert range_deps_of(both(3, 4), 0) == {(0, 5): [0], (3, 9): [1]}
        reg(st, s, [0, 1], [ERASED, INVALID]); reg(ora, s, [0, 1], [ERASED, INVALID])
        assert range_deps_of(both(4, 5), 0) == {(3, 9): [1]}
