"""Stream segments (config 4; include/accord_deps.h accord_segment_*): rank r owns
positions [a_r, b_r) of every CommandStore and needs the CommandsForKey state at a_r -- per key the
run from the last Write before a_r - W on (local/CommandsForKey.java:620-645).  CPU tests:

  * the decomposition: folding the per-segment summaries (oracle or_cfk_fold) gives exactly the state
    read off the whole prefix (or_cfk_reachable(0, a_r, a_r - W)), for segments longer and shorter
    than the window and streams where keys go long without a Write;
  * the exchange step itself (accord_amd.segment_exchange, the code bench.py runs over RCCL) under
    torch.distributed gloo with world sizes 2 and 3, the oracle standing in for the device summary
    and fold: every rank's carry equals the prefix state.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from accord_amd import generate_stream, segment_bounds, segment_exchange
import oracle_lib as O


def _fold_case(s, W, cuts):
    parts = []
    for q in range(len(cuts) - 1):
        a, b = cuts[q], cuts[q + 1]
        parts.append(O.cfk_reachable(s, a, b, b - W))
        want = O.cfk_reachable(s, 0, b, b - W)
        got = O.cfk_fold(parts, b - W)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), (W, cuts, q)


@pytest.mark.parametrize("W", [0, 8, 64, 256])
def test_fold_of_summaries_equals_prefix_state(W):
    s = generate_stream(6000, 4, 300, 0.99, 0.5, seed=51)
    _fold_case(s, W, [0, 1500, 3000, 4500, 6000])
    _fold_case(s, W, [0, 100, 130, 700, 701, 2500, 6000])       # segments shorter than the window


def test_fold_when_keys_go_long_without_writes():
    # 5 % Writes over a large keyspace: most keys carry no Write in a segment, so the carry reaches
    # back across several summaries (and to the first entry of keys never written)
    s = generate_stream(8000, 3, 2000, 0.5, 0.05, seed=52)
    _fold_case(s, 32, [0, 1000, 2000, 3000, 4000, 5000, 6000, 7000, 8000])
    k, e = O.cfk_reachable(s, 0, 8000, 8000 - 32)
    assert k.size > 8000 // 4                                   # the state is not a thin tail here


def test_summary_is_small_at_config4_scale():
    # config-2-shaped segment: the summary is a small fraction of the segment's pairs
    s = generate_stream(1 << 17, 8, 100_000, 0.99, 0.5, seed=2)
    k, _ = O.cfk_reachable(s, 0, s.n, s.n - 256)
    assert k.size < s.pairs // 3


class OracleSegmentStore:
    """The oracle playing a CommandStore's segment calls (summary on the host, carry = or_cfk_fold)
    so the exchange step can run on the CPU; buffers are CPU tensors, pointers are host pointers."""

    def __init__(self, s, a, b, W):
        self.s, self.a, self.b, self.W = s, a, b, W
        self.carry = None

    def segment_summary(self):
        self.k, self.e = O.cfk_reachable(self.s, self.a, self.b, self.b - self.W)
        return int(self.k.size), self.k.ctypes.data, self.e.ctypes.data

    def segment_summary_copy(self, key_ptr, ent_ptr, cap):
        assert cap >= self.k.size
        C.memmove(key_ptr, self.k.ctypes.data, 4 * self.k.size)
        C.memmove(ent_ptr, self.e.ctypes.data, 4 * self.e.size)

    def segment_carry(self, parts):
        got = []
        for n, kp, ep in parts:
            k = np.ctypeslib.as_array((C.c_uint32 * max(n, 1)).from_address(kp))[:n].copy()
            e = np.ctypeslib.as_array((C.c_uint32 * max(n, 1)).from_address(ep))[:n].copy()
            got.append((k, e))
        self.carry = O.cfk_fold(got, self.a - self.W)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        W = 48
        s = generate_stream(3000 * world, 4, 400, 0.99, 0.4, seed=60 + world)   # the same stream on every rank
        a, b = segment_bounds(s.n, world)[rank]
        st = OracleSegmentStore(s, a, b, W)
        info = segment_exchange(st, rank, world, "cpu")
        want = O.cfk_reachable(s, 0, a, a - W)
        ok = np.array_equal(st.carry[0], want[0]) and np.array_equal(st.carry[1], want[1])
        dist.destroy_process_group()
        q.put((rank, ok, int(want[0].size), info["summary_entries"]))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), 0, None))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_segment_exchange_builds_every_carry(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, size, counts in res:
        assert ok is True, (rank, ok)
        assert rank == 0 or size > 0
        assert counts is not None and len(counts) == world
