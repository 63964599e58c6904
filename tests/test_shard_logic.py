"""CPU rehearsal (gloo, world_size 2) of the multi-GPU partitioning that bench.py and
accord_deps_exchange_merge implement: every rank owns a contiguous EvenSplit block of stores
(local/ShardDistributor.java:46-157), computes the partial deps of the txns intersecting it, sends
each txn's partial to its owner rank floor(g*G/N), and the owner unions the parts
(PreAccept.reduce, messages/PreAccept.java:140-156).  The union must equal single-store deps.
The oracle plays the device's role here; the RCCL transport itself needs GPUs."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from accord_amd import generate_stream
import oracle_lib as O

KS, W, N = 600, 16, 1200


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        s = generate_stream(N, 4, KS, 0.99, 0.5, seed=41)      # identical on every rank
        lo, hi = rank * KS // world, (rank + 1) * KS // world
        part = O.deps_fast(s.restrict_keys(lo, hi), W)        # this rank's stores, global coordinates
        home = [(d * N // world, (d + 1) * N // world) for d in range(world)]
        outgoing = []
        for (a, b) in home:
            outgoing.append([tuple(np.asarray(x).tolist() for x in part.key_deps(t)) for t in range(a, b)])
        received = [None] * world
        for src in range(world):
            obj = [outgoing] if src == rank else [None]
            dist.broadcast_object_list(obj, src=src)
            received[src] = obj[0][rank]
        tm = s.msb.astype(np.uint64)
        tl = s.lsb.astype(np.uint64)
        tn = s.node.astype(np.int32)
        full = O.deps_fast(s, W)
        a, b = home[rank]
        bad = 0
        for t in range(a, b):
            acc = None
            for src in range(world):
                p = tuple(np.asarray(x) for x in received[src][t - a])
                if acc is None:
                    acc = p
                elif len(p[0]):
                    acc = p if len(acc[0]) == 0 else O.keydeps_union(acc, p, tm, tl, tn)
            want = full.key_deps(t)
            if not all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(acc, want)):
                bad += 1
        dist.destroy_process_group()
        q.put((rank, bad, b - a))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), 0))


def _worker_ranges(rank, world, port, q):
    """Range txns: each rank's partial is a whole PartialDeps (KeyDeps + RangeDeps) of its stores;
    the owner unions the parts it receives with Deps.merge (or_deps_union) -- what the device does
    through accord_deps_union -- and the result is the node-level deps over all the stores."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        s = generate_stream(N, 4, KS, 0.99, 0.5, seed=42, range_frac=0.15, range_len_max=120)
        # 4 EvenSplit CommandStores per rank: every store slices the range commands and queries to
        # its own range (InMemoryCommandStore.java:757-760), so a rank's part holds its stores' slices
        bounds = O.store_bounds(KS, 4 * world)
        part = O.deps_stores(s, W, bounds[4 * rank:4 * rank + 5])
        parts = [None] * world
        for src in range(world):
            obj = [part] if src == rank else [None]
            dist.broadcast_object_list(obj, src=src)
            parts[src] = obj[0]
        merged = O.deps_union(parts)
        full = O.deps_stores(s, W, bounds)
        a, b = rank * N // world, (rank + 1) * N // world
        bad = 0
        for t in range(a, b):
            x, y = merged.key_deps(t), full.key_deps(t)
            u, v = merged.range_deps(t), full.range_deps(t)
            if not all(np.array_equal(np.asarray(i), np.asarray(j)) for i, j in zip(tuple(x) + tuple(u), tuple(y) + tuple(v))):
                bad += 1
        dist.destroy_process_group()
        q.put((rank, bad, b - a))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), 0))


@pytest.mark.parametrize("worker", [_worker, _worker_ranges], ids=["keys", "ranges"])
def test_two_rank_shard_union_equals_full_deps(worker):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, bad, cnt in results:
        assert bad == 0, (rank, bad)
        assert cnt > 0
