"""WaitingOn bitsets and execution levelling on the GPU vs the
oracle (or_waiting_on) and, for streams without SyncPoint kinds, the CommandsForKey-side readiness
simulation or_levels_cfk (notify with missing[] counts, registerUnmanaged; test_oracle_stream.py).  Bit-exact: levels and every bitset word."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalStateException, generate_stream
import oracle_lib as O
from test_oracle_stream import with_random_kinds

pytestmark = pytest.mark.gpu

CASES = [
    # n, k, keyspace, zipf, write_frac, window, seed, range_frac, range_len, random kinds
    (20000, 4, 2000, 0.99, 0.9, 256, 51, 0.0, 0, False),     # config 5 shape, small
    (20000, 8, 5000, 0.99, 0.5, 64, 52, 0.0, 0, False),
    (12000, 4, 500, 0.0, 0.5, 32, 53, 0.2, 50, False),       # range txns: full pred lists
    (15000, 4, 300, 0.99, 0.7, 16, 54, 0.0, 0, True),        # SyncPoints keep full lists
    (10000, 2, 20, 0.0, 1.0, 1000, 55, 0.0, 0, False),       # deep chains (~1000 per key)
    (3000, 1, 1, 0.0, 1.0, 4096, 56, 0.0, 0, False),         # one key, all writes: level = i
    (60000, 4, 50000, 0.99, 0.9, 256, 59, 0.0, 0, False),    # cold keys: predecessors beyond the LDS ring
    (20000, 6, 40, 0.0, 0.3, 2000, 60, 0.0, 0, False),       # read-heavy: writes with many far predecessors
]


def _check(s, ks, W, cfk=False):
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        st.upload(s)
        st.compute()
        wo = st.waiting_on()
        d = st.download()
    level, wo_off, words = O.waiting_on(d)
    assert np.array_equal(wo.wo_off, wo_off)
    assert np.array_equal(wo.words, words)
    bad = np.nonzero(wo.level != level)[0]
    assert bad.size == 0, (bad[:5], wo.level[bad[:5]], level[bad[:5]])
    assert wo.max_level == int(level.max(initial=0))
    if cfk:
        # readiness restated from CommandsForKey notify / registerUnmanaged (or_levels_cfk)
        assert np.array_equal(wo.level, O.levels_cfk(s, d))
    return wo


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_waiting_on_matches_oracle(gpu_device, case):
    n, k, ks, z, wf, W, seed, rf, rl, kinds = case
    s = generate_stream(n, k, ks, z, wf, seed=seed, range_frac=rf, range_len_max=rl)
    if kinds:
        s = with_random_kinds(s, seed)
    wo = _check(s, ks, W, cfk=not kinds)
    if ks == 1:
        assert np.array_equal(wo.level, np.arange(n, dtype=np.uint32))


def test_waiting_on_reduced_dag_is_smaller(gpu_device):
    s = generate_stream(30000, 4, 1000, 0.99, 0.9, seed=57)
    with CommandStore(device=0, key_lo=0, key_hi=1000, window=256) as st:
        st.upload(s)
        st.compute()
        wo = st.waiting_on()
        full_edges = st.download().totals()["vals"]
    assert wo.preds_total < full_edges


def test_waiting_on_requires_full_stream(gpu_device):
    s = generate_stream(2000, 4, 1000, 0.0, 0.5, seed=58)
    sub = s.restrict_keys(0, 500, drop_empty=True)
    with CommandStore(device=0, key_lo=0, key_hi=500, window=16) as st:
        with pytest.raises(IllegalStateException):
            st.waiting_on()
        st.upload(sub)
        st.compute()
        with pytest.raises(IllegalStateException):
            st.waiting_on()


@pytest.mark.timeout(900)
def test_config5_full_size(gpu_device):
    """BASELINE.json configs[4] at full size: 4,194,304 key txns, k = 4 over
    10,000 keys, Zipf(0.99), 90% writes, W = 256, seed 5 -- deps byte-compared with the fast oracle,
    then level[], wo_off and every bitset word with or_waiting_on over those deps."""
    n, ks, W = 1 << 22, 10_000, 256
    s = generate_stream(n, 4, ks, 0.99, 0.9, seed=5)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        st.upload(s)
        st.compute()
        wo = st.waiting_on()
        d = st.download()
    want = O.deps_fast(s, W)
    diff = d.first_difference(want)
    assert diff is None, diff
    del want
    level, wo_off, words = O.waiting_on(d)
    assert np.array_equal(wo.wo_off, wo_off)
    assert np.array_equal(wo.words, words)
    bad = np.nonzero(wo.level != level)[0]
    assert bad.size == 0, (bad[:5], wo.level[bad[:5]], level[bad[:5]])
    assert wo.max_level == int(level.max(initial=0))
    assert np.array_equal(wo.level, O.levels_cfk(s, d))
