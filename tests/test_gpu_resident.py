"""Resident CommandsForKey state across batches.

A store created resident keeps each key's reachable history in HBM between batches and prunes the
rest (local/CommandsForKey.java:620-645,1654-1684).  Feeding a stream to it as consecutive batches
must give, byte for byte, the deps of one batch over the whole stream (txnIds are global stream
positions) -- checked against the GPU single-batch run, the literal oracle fed the same batch
sequence (real CFK objects, per-status-change copies) and, at config-2 size, the fast oracle."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalArgumentException, IllegalStateException, PartialDeps, generate_stream
import oracle_lib as O

pytestmark = pytest.mark.gpu


def split_points(n, parts, seed):
    rng = np.random.default_rng(seed)
    cuts = np.sort(rng.choice(np.arange(1, n), size=parts - 1, replace=False)) if parts > 1 else []
    return [0, *[int(c) for c in cuts], n]


def run_batches(s, ks, W, pts, lo=0):
    outs = []
    with CommandStore(device=0, key_lo=lo, key_hi=ks, window=W, resident=True) as st:
        for a, b in zip(pts[:-1], pts[1:]):
            outs.append(st.calculate_deps_batch(s.slice(a, b)))
        state = st.state()
    return PartialDeps.concat(outs), state


def single(s, ks, W, lo=0):
    with CommandStore(device=0, key_lo=lo, key_hi=ks, window=W) as st:
        return st.calculate_deps_batch(s)


CASES = [
    # n, k, keyspace, zipf, write_frac, W, seed, parts
    (12000, 8, 2000, 0.99, 0.5, 256, 1, 8),
    (20000, 4, 300, 0.0, 0.1, 64, 2, 13),       # read-heavy: long carried read runs
    (15000, 2, 20, 0.0, 1.0, 1000, 3, 5),       # hot keys, window spans batches
    (12000, 8, 50000, 0.99, 0.5, 0, 4, 7),      # W = 0
    (9000, 3, 100, 0.0, 0.0, 32, 5, 4),         # reads only: nothing is ever pruned
    (8000, 6, 500, 0.99, 0.5, 3000, 6, 16),     # window longer than most batches
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_batches_equal_single_and_literal(gpu_device, case):
    n, k, ks, z, wf, W, seed, parts = case
    s = generate_stream(n, k, ks, z, wf, seed=seed)
    pts = split_points(n, parts, seed)
    got, state = run_batches(s, ks, W, pts)
    assert state["next_global"] == n
    one = single(s, ks, W)
    assert got.first_difference(one) is None
    lit = O.deps_literal(s, W)
    assert got.first_difference(lit) is None


# batch pair counts around the merge join's chunk and size limits (csrc/radix_sort.hip: 1024-pair
# chunks, up to 16 of them; a batch over 16 Ki pairs, or the first one, re-sorts with the radix passes)
MERGE_CASES = [
    # keys per txn, keyspace, batch sizes (txns)
    (1, 3000, [5, 1, 1024, 1025, 1023, 16384, 16385, 3000, 2]),
    (8, 100000, [7, 128, 2048, 2049, 1, 300]),
]


@pytest.mark.parametrize("case", MERGE_CASES, ids=[f"m{i}" for i in range(len(MERGE_CASES))])
def test_merge_join_batch_sizes(gpu_device, case):
    k, ks, sizes = case
    n = sum(sizes)
    s = generate_stream(n, k, ks, 0.99, 0.5, seed=11 + k)
    pts = [0]
    for b in sizes:
        pts.append(pts[-1] + b)
    got, state = run_batches(s, ks, 256, pts)
    assert state["next_global"] == n
    assert got.first_difference(single(s, ks, 256)) is None


def test_uploads_without_compute_between(gpu_device):
    """accord_batch_upload leaves a small batch's copy running (two page-locked staging halves in
    turn): uploads back to back, then one compute, give the last batch's deps, for plain and
    resident stores"""
    parts = [generate_stream(700 + 50 * i, 4, 500, 0.99, 0.5, seed=40 + i) for i in range(4)]
    for resident in (False, True):
        with CommandStore(device=0, key_lo=0, key_hi=500, window=64, resident=resident) as st:
            for p in parts:
                st.upload(p)
            st.compute()
            got = st.download()
        assert got.first_difference(single(parts[-1], 500, 64)) is None


def test_accept_batches_see_only_registered_txns(gpu_device):
    # executeAt past the end of its batch: only txns registered so far are candidates
    n, ks, W = 12000, 400, 128
    s = generate_stream(n, 4, ks, 0.99, 0.5, seed=21).accept(frac=0.6, max_delay=300, seed=21)
    pts = split_points(n, 6, 21)
    got, _ = run_batches(s, ks, W, pts)
    ends = O.batch_ends(np.diff(pts))
    assert got.first_difference(O.deps_literal(s, W, batch_end=ends)) is None
    assert got.first_difference(O.deps_fast(s, W, batch_end=ends)) is None


def test_store_subset_with_global_positions(gpu_device):
    # a store owning keys [300, 700) of a 1000-key stream, fed batch by batch with txn_index
    full = generate_stream(30000, 4, 1000, 0.99, 0.5, seed=22)
    sub = full.restrict_keys(300, 700, drop_empty=True)
    pts = split_points(sub.n, 9, 22)
    got, state = run_batches(sub, 700, 256, pts, lo=300)
    assert got.first_difference(single(sub, 700, 256, lo=300)) is None
    assert state["next_global"] == int(sub.txn_index[-1]) + 1


def test_state_is_pruned_and_rejections_leave_it(gpu_device):
    s = generate_stream(20000, 8, 2000, 0.99, 0.5, seed=23)
    with CommandStore(device=0, key_lo=0, key_hi=2000, window=256, resident=True) as st:
        a = st.calculate_deps_batch(s.slice(0, 10000))
        with pytest.raises(IllegalStateException):              # the same upload cannot be registered twice
            st.compute()
        st0 = st.state()
        assert st0["next_global"] == 10000
        assert 0 < st0["carry_entries"] < s.key_off[10000]      # pruned below each key's last old Write
        with pytest.raises(IllegalArgumentException):           # out of order: replays an earlier batch
            st.calculate_deps_batch(s.slice(5000, 10000))
        assert st.state() == st0                                # a rejected batch leaves the state
        b = st.calculate_deps_batch(s.slice(10000, 20000))
        first = single(s, 2000, 256)
        assert PartialDeps.concat([a, b]).first_difference(first) is None
        st.reset()
        assert st.state()["next_global"] == 0
        again = st.calculate_deps_batch(s)
        assert again.first_difference(first) is None


@pytest.mark.timeout(600)
def test_config2_full_in_8_batches(gpu_device):
    """BASELINE configs[1] (1,048,576 txns, k = 8, Zipf 0.99 over 100k keys, W = 256) fed as 8
    consecutive batches to one resident store == the single-batch run == the fast oracle."""
    n, ks, W = 1 << 20, 100_000, 256
    s = generate_stream(n, 8, ks, 0.99, 0.5, seed=2)
    pts = [i * n // 8 for i in range(9)]
    got, state = run_batches(s, ks, W, pts)
    one = single(s, ks, W)
    assert got.first_difference(one) is None
    assert got.first_difference(O.deps_fast(s, W)) is None
    assert state["carry_entries"] < n                           # far less than the 8.4 M history pairs


# range txns in a resident store: the range commands a later batch's window can still reach travel
# with the key history (owner positions >= next_global - W), so RangeDeps and the range txns'
# KeyDeps of every batch equal the single-batch run over the whole stream
RANGE_CASES = [
    # n, k, keyspace, zipf, write_frac, range_frac, range_len_max, W, seed, parts
    (6000, 4, 2000, 0.99, 0.5, 0.2, 200, 256, 31, 8),
    (8000, 3, 500, 0.0, 0.3, 0.1, 60, 64, 32, 23),
    (5000, 2, 3000, 0.99, 0.5, 0.05, 1500, 3000, 33, 11),     # window spans most batches
    (6000, 4, 1000, 0.99, 0.5, 0.3, 100, 0, 34, 6),           # W = 0: nothing carries
    (4000, 4, 800, 0.99, 0.5, 0.02, 300, 512, 35, 80),        # short batches, most without ranges
    (9000, 4, 20000, 0.99, 0.5, 0.15, 400, 4500, 36, 5),      # windows span checkpoint blocks
]


@pytest.mark.parametrize("case", RANGE_CASES, ids=[f"r{i}" for i in range(len(RANGE_CASES))])
def test_range_batches_equal_single(gpu_device, case):
    n, k, ks, z, wf, rf, rl, W, seed, parts = case
    s = generate_stream(n, k, ks, z, wf, range_frac=rf, range_len_max=rl, seed=seed)
    assert int(s.rng_off[-1]) > 0
    pts = split_points(n, parts, seed)
    got, state = run_batches(s, ks, W, pts)
    assert state["next_global"] == n
    one = single(s, ks, W)
    assert got.first_difference(one) is None
    assert got.first_difference(O.deps_fast(s, W)) is None


def test_range_accept_batches(gpu_device):
    n, ks, W = 6000, 600, 128
    s = generate_stream(n, 4, ks, 0.99, 0.5, range_frac=0.15, range_len_max=80, seed=37)
    s = s.accept(frac=0.5, max_delay=200, seed=37)
    pts = split_points(n, 7, 37)
    got, _ = run_batches(s, ks, W, pts)
    ends = O.batch_ends(np.diff(pts))
    assert got.first_difference(O.deps_fast(s, W, batch_end=ends)) is None


def test_range_carry_resets(gpu_device):
    s = generate_stream(4000, 4, 500, 0.99, 0.5, range_frac=0.2, range_len_max=100, seed=38)
    with CommandStore(device=0, key_lo=0, key_hi=500, window=300, resident=True) as st:
        a = st.calculate_deps_batch(s.slice(0, 2000))
        b = st.calculate_deps_batch(s.slice(2000, 4000))
        st.reset()
        again = PartialDeps.concat([st.calculate_deps_batch(s.slice(0, 2000)),
                                    st.calculate_deps_batch(s.slice(2000, 4000))])
    assert PartialDeps.concat([a, b]).first_difference(again) is None
    assert again.first_difference(single(s, 500, 300)) is None


def test_registered_store_takes_ranges(gpu_device):
    # no events yet: every txn PREACCEPTED, no window -- the stateful literal oracle's result
    from accord_amd import WINDOW_NONE
    s = generate_stream(200, 2, 100, 0.0, 0.5, range_frac=0.3, range_len_max=10, seed=39)
    with CommandStore(device=0, key_lo=0, key_hi=100, window=WINDOW_NONE, resident=True) as st:
        got = st.calculate_deps_batch(s)
    assert got.first_difference(O.LStore(100).batch(s)) is None


@pytest.mark.timeout(600)
def test_config3_full_in_8_batches(gpu_device):
    """BASELINE configs[2] (config 2 with 20% range txns of up to 1000 keys) fed as 8 consecutive
    batches to one resident store == the single-batch run == the fast oracle."""
    n, ks, W = 1 << 20, 100_000, 256
    s = generate_stream(n, 8, ks, 0.99, 0.5, range_frac=0.2, range_len_max=1000, seed=3)
    pts = [i * n // 8 for i in range(9)]
    got, _ = run_batches(s, ks, W, pts)
    one = single(s, ks, W)
    assert got.first_difference(one) is None
    assert got.first_difference(O.deps_fast(s, W)) is None
