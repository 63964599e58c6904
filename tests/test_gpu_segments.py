"""Stream segments on the device (config 4; include/accord_deps.h accord_segment_*).

Rank r owns positions [a_r, b_r) of every CommandStore.  Here the G ranks are G resident stores on
one GPU: each uploads its segment and builds its CommandsForKey summary; each then folds the
summaries of the segments before it into its carry (the transport -- one all-gather over RCCL in
bench.py, tests/test_segments.py under gloo -- replaced by the stores' own device pointers) and
computes.  Checked byte for byte:
  * every device summary == the oracle's (or_cfk_reachable), every carry's size == the prefix state;
  * every segment's deps == the oracle's deps of the whole stream for those txns (small streams),
    == one resident store fed the whole stream (config 4 at full size: 8 x 1,048,576 txns), and the
    txns right after a segment boundary == the oracle on that prefix."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalArgumentException, IllegalStateException, generate_stream, segment_bounds
import oracle_lib as O

pytestmark = pytest.mark.gpu


def device_summary(st):
    import torch
    n, _, _ = st.segment_summary()
    buf = torch.empty((2, max(n, 1)), dtype=torch.int32, device="cuda")
    st.segment_summary_copy(buf[0].data_ptr(), buf[1].data_ptr(), max(n, 1))
    h = buf.cpu().numpy().view(np.uint32)
    return h[0, :n].copy(), h[1, :n].copy()


def run_segments(s, G, ks, W, check_summary=True):
    """G segment stores of one GPU: summaries, carries, computes.  Returns the stores (open)."""
    bounds = segment_bounds(s.n, G)
    stores, parts = [], []
    for r, (a, b) in enumerate(bounds):
        st = CommandStore(device=0, key_lo=0, key_hi=ks, window=W, resident=True)
        st.segment_begin(a)
        st.upload(s.slice(a, b))
        parts.append(st.segment_summary())
        if check_summary:
            got = device_summary(st)
            wk, we = O.cfk_reachable(s, a, b, b - W)              # key-major; the device's is in stream order
            o = np.lexsort((wk, we & 0x1FFFFFFF))
            assert np.array_equal(got[0], wk[o]) and np.array_equal(got[1], we[o]), r
        stores.append(st)
    for r, st in enumerate(stores):
        st.segment_carry(parts[:r])
    return bounds, stores


CASES = [
    # n, k, keyspace, zipf, write_frac, W, seed, G
    (12000, 8, 2000, 0.99, 0.5, 256, 1, 4),
    (20000, 4, 300, 0.0, 0.1, 64, 2, 5),        # read-heavy: carries reach back over several segments
    (9000, 3, 100, 0.0, 0.0, 32, 5, 3),         # reads only: the carry is every earlier entry
    (8000, 6, 500, 0.99, 0.5, 3000, 6, 8),      # window longer than a segment
    (6000, 2, 40, 0.0, 1.0, 0, 7, 6),           # W = 0, writes only
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_segments_equal_whole_stream(gpu_device, case):
    n, k, ks, z, wf, W, seed, G = case
    s = generate_stream(n, k, ks, z, wf, seed=seed)
    want = O.deps_fast(s, W)
    bounds, stores = run_segments(s, G, ks, W)
    try:
        for r, (st, (a, b)) in enumerate(zip(stores, bounds)):
            assert st.state()["carry_entries"] == O.cfk_reachable(s, 0, a, a - W)[0].size, r
            st.compute()
            d = st.download()
            assert d.first_difference(want.txns(a, b)) is None, r
            # a step again: carry rewinds the store to the segment's start
            st.segment_carry([stores[q].segment_summary() for q in range(r)])
            st.compute()
            assert st.download().first_difference(want.txns(a, b)) is None, r
    finally:
        for st in stores:
            st.close()


def test_segment_call_order_and_arguments(gpu_device):
    s = generate_stream(2000, 4, 500, 0.0, 0.5, seed=9)
    with CommandStore(device=0, key_lo=0, key_hi=500, window=64) as plain:
        with pytest.raises(IllegalStateException):
            plain.segment_begin(0)                          # not resident
    with CommandStore(device=0, key_lo=0, key_hi=500, window=64, resident=True) as st:
        with pytest.raises(IllegalStateException):
            st.segment_summary()                            # before segment_begin
        st.segment_begin(1000)
        with pytest.raises(IllegalStateException):
            st.segment_summary()                            # before the upload
        st.upload(s.slice(1000, 2000))
        n, _, _ = st.segment_summary()
        import torch
        small = torch.empty((2, 1), dtype=torch.int32, device="cuda")
        if n > 1:
            from accord_amd import AccordError
            with pytest.raises(AccordError):
                st.segment_summary_copy(small[0].data_ptr(), small[1].data_ptr(), 1)
    r = generate_stream(1000, 4, 500, 0.0, 0.5, range_frac=0.2, range_len_max=20, seed=10)
    with CommandStore(device=0, key_lo=0, key_hi=500, window=64, resident=True) as st:
        st.segment_begin(0)
        st.upload(r)
        with pytest.raises(IllegalArgumentException):
            st.segment_summary()                            # range txns
        st.segment_begin(0)
        st.upload(s.accept(seed=2))
        with pytest.raises(IllegalArgumentException):
            st.segment_summary()                            # Accept batch


@pytest.mark.timeout(600)
def test_config4_full_size_segments(gpu_device):
    """Config 4 at full size on one GPU: 8 segments x 1,048,576 config-2 txns (Zipf 0.99 over 100k
    keys, W = 256, seed 2 -- the stream bench.py --gpus 8 builds).  Every segment's deps == one
    resident store fed the whole stream segment by segment (== one batch over it: test_gpu_resident),
    and segment 1's first 20,000 txns == the fast oracle on the prefix that ends there."""
    G, n1, ks, W = 8, 1 << 20, 100_000, 256
    s = generate_stream(G * n1, 8, ks, 0.99, 0.5, seed=2)
    bounds, stores = run_segments(s, G, ks, W, check_summary=False)
    try:
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=W, resident=True) as one:
            for r, (st, (a, b)) in enumerate(zip(stores, bounds)):
                st.compute()
                got = st.download()
                one.upload(s.slice(a, b))
                one.compute()
                ref = one.download()
                assert got.first_difference(ref) is None, r
                if r == 1:
                    m = 20_000
                    exp = O.deps_fast(s.prefix(a + m), W).txns(a, a + m)
                    assert got.txns(0, m).first_difference(exp) is None
                del got, ref
                st.close()
    finally:
        for st in stores:
            st.close()
