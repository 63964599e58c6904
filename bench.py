#!/usr/bin/env python3
"""Benchmark of the MI355X-native Accord deps path (BASELINE.json metric).

One "step" = one pass of the hot path over one batch: batched PreAccept deps for every txn of
the stream (validate/pack -> (key, txn) radix bucketing into CommandsForKey histories ->
history annotation -> per-txn conflict scan + KeyDeps linearisation, count and fill), with the
batch already resident in HBM.  Default workload (BASELINE.json configs[1]): 1,048,576 key txns,
8 keys each, Zipf(0.99) over 100,000 keys, 50% writes, window W=256, seed 2.

Multi-GPU (`bench.py --gpus G`, which starts the G ranks itself, or `torchrun --nproc-per-node G`;
config 4): one global stream of G x 1,048,576 txns (weak scaling: every GPU gets a config-2-sized
share) over 8G EvenSplit CommandStores (local/ShardDistributor.java:46-157).  Default partition
(`--partition segments`): rank r owns the r-th segment of the stream -- positions
[r n, (r+1) n) -- of every CommandStore.  A step is: the segment's CommandsForKey summary (per key,
what later txns can still reach), one all-gather of the summaries over RCCL/xGMI
(torch.distributed nccl), the fold of the earlier segments' summaries into the CommandsForKey state
at the segment's start, and the deps of the segment's txns -- node-level deps, the union
PreAccept.reduce (messages/PreAccept.java:140-156) would assemble, so no partial deps travel.
`--partition keys`: rank r owns the key block of stores [8r, 8r+8), computes the partial deps of
the txns touching it, and one RCCL exchange moves every partial to the txn's owner for the on-device
union (the round-3..5 design, kept for comparison).  `--one-device`: every rank on GPU 0 with the
exchange over gloo (a one-GPU rehearsal of the multi-rank code path).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

import numpy as np  # noqa: E402

PEAK_HBM_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes(n, P, kc, U, D):
    """B = 20N + 4(N+1) + 4P + 8D + 4*sum(k_i) + 4U + 12N (keys only)."""
    return 20 * n + 4 * (n + 1) + 4 * P + 8 * D + 4 * kc + 4 * U + 12 * n


def fill_kernel_bytes(n, P, kc, U, D):
    """Algorithmic bytes of ONE pass of the fill stage (txnrec_kernel + keydeps_fast_kernel<16> +
    keydeps_kernel<1,8> over the fast kernel's fallback list; every txn is filled once): reads lsb (8N),
    key_off (4(N+1)), key_ord (4P), the pair slices poslo (8P), each raw candidate once (4D), the
    three offset arrays (12(N+1)); writes the txnIds count (4N), keys (4kc), txnIds (4U) and
    keysToTxnIds (4(kc+D))."""
    return 8 * n + 4 * (n + 1) + 4 * P + 8 * P + 4 * D + 12 * (n + 1) + 4 * n + 4 * kc + 4 * U + 4 * (kc + D)


# SURVEY.md §8d workloads
PRESETS = {
    2: dict(n=1 << 20, keys_per_txn=8, keyspace=100_000, seed=2, range_frac=0.0, write_frac=0.5),
    3: dict(n=1 << 20, keys_per_txn=8, keyspace=100_000, seed=3, range_frac=0.2, write_frac=0.5),
    5: dict(n=1 << 22, keys_per_txn=4, keyspace=10_000, seed=5, range_frac=0.0, write_frac=0.9),
}


def launch(gpus, argv, dry_run=False):
    """`bench.py --gpus G` without a launcher: start G ranks of this script, one process per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = G, rendezvous on 127.0.0.1), before anything in this process
    touches the GPU -- the parent imports no HIP / torch.cuda / accord_amd.  The parent relays rank
    0's stdout (the JSON line; every rank's with --launch-dry-run) and exits with the first failing
    rank's code; a rank that fails ends the others."""
    import socket
    import subprocess
    import tempfile
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs, outs = [], []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        f = tempfile.TemporaryFile(mode="w+")
        outs.append(f)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, stdout=f))
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            time.sleep(5)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
        if rc == 0 and p.returncode != 0:
            rc = p.returncode
    for r, f in enumerate(outs):
        if r == 0 or dry_run:
            f.seek(0)
            sys.stdout.write(f.read())
        f.close()
    sys.stdout.flush()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 5),
                    help="BASELINE.json configs[1] (2), configs[2] (3: 20%% range txns), configs[4] "
                         "(5: 4M txns, deep chains, + WaitingOn levelling)")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--keys-per-txn", type=int, default=None)
    ap.add_argument("--keyspace", type=int, default=None)
    ap.add_argument("--zipf", type=float, default=0.99)
    ap.add_argument("--window", type=int, default=256)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--range-frac", type=float, default=None)
    ap.add_argument("--range-len", type=int, default=1000)
    ap.add_argument("--write-frac", type=float, default=None)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="first txns of the CPU-baseline prefix sample (default: grown by doubling within --cpu-budget)")
    ap.add_argument("--cpu-budget", type=float, default=25.0,
                    help="seconds of CPU-baseline work: the prefix doubles while the next run fits (600 = the "
                         "largest prefix within 10 minutes)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--resident", action="store_true",
                    help="also time the stream fed as 8 batches to one resident store (resident_batches); "
                         "off by default so a kernel trace of the default run holds one batch size only")
    ap.add_argument("--registered", action="store_true",
                    help="also time the registered-status store (real status events, no status-at-time model) "
                         "on the config-2 stream fed in batches (registered_batches)")
    ap.add_argument("--ready", action="store_true",
                    help="also time execution readiness (accord_ready_update) over a registered-status "
                         "schedule: batches registered STABLE, ready txns registered APPLIED round by round")
    ap.add_argument("--ready-events", action="store_true",
                    help="--ready: also run the schedule in event-exact mode (accord_ready_set_mode EVENTS)")
    ap.add_argument("--ready-batch", type=int, default=4096, help="txns per batch of the --ready leg")
    ap.add_argument("--ready-batches", type=int, default=16, help="batches of the --ready leg")
    ap.add_argument("--ready-cpu-batch", type=int, default=2048,
                    help="--ready: one batch of this many txns drained by the oracle's readiness restatement "
                         "(CPU) and by the device (0: skip)")
    ap.add_argument("--reg-batch", type=int, default=1024, help="txns per batch of the --registered leg")
    ap.add_argument("--reg-batches", type=int, default=64, help="batches of the --registered leg")
    ap.add_argument("--partition", choices=("segments", "keys"), default="segments",
                    help="--gpus G > 1: ownership by stream segments (default) or by key blocks of stores")
    ap.add_argument("--one-device", action="store_true",
                    help="--gpus G > 1 on one GPU: every rank uses device 0, the exchange runs over gloo")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="--gpus G > 1: start the G ranks, each prints its rank / world and exits before any GPU work")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, sys.argv[1:], args.launch_dry_run))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}")
    if args.launch_dry_run:
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "world": int(os.environ.get("WORLD_SIZE", "1")), "master": os.environ.get("MASTER_ADDR"),
                          "port": os.environ.get("MASTER_PORT"), "gpus": args.gpus}))
        if os.environ.get("ACCORD_DRY_FAIL_RANK") == os.environ.get("RANK"):
            sys.exit(3)                 # the launcher's failure path (tests/test_bench_launch.py)
        return
    preset = PRESETS[args.config]
    for k, v in preset.items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    args.waiting_on = args.config == 5

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch = None
    segments = world > 1 and args.partition == "segments"
    device_index = 0 if (world == 1 or args.one_device) else local_rank
    xdev = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(device_index)
        dist.init_process_group("gloo" if args.one_device else "nccl", init_method="env://")
        xdev = torch.device("cpu") if args.one_device else torch.device("cuda", device_index)
        if not segments and args.one_device:
            raise SystemExit("--one-device rehearses --partition segments only")

    from accord_amd import CommandStore, generate_stream, segment_bounds, segment_exchange

    if args.waiting_on and world > 1:
        raise SystemExit("config 5 levels one full stream per GPU (replicas only): run it with --gpus 1")
    if world > 1 and args.range_frac > 0:
        raise SystemExit("config 4 is the key-txn workload of config 2")

    n_total = args.n * world
    # one global stream (identical on every rank); weak scaling: n per GPU
    s_full = generate_stream(n_total, args.keys_per_txn, args.keyspace, args.zipf, args.write_frac,
                             range_frac=args.range_frac, range_len_max=args.range_len, seed=args.seed)
    stores_total = 8 * world
    # EvenSplit over [0, keyspace): store b owns [b*ks/S, (b+1)*ks/S)
    bounds = [b * args.keyspace // stores_total for b in range(stores_total)] + [0xFFFFFFFF]
    rccl = None
    seg = None
    if segments:
        # rank r owns positions [a, b) of every CommandStore: one resident handle hosting all 8G
        # stores, standing at a with the CommandsForKey state the exchange builds
        a, b = segment_bounds(n_total, world)[rank]
        seg = (a, b)
        s = s_full.slice(a, b)
        store = CommandStore(device=device_index, key_lo=0, key_hi=args.keyspace, window=args.window, profile=True,
                             resident=True, store_bounds=bounds)
        store.segment_begin(a)
        store.upload(s)
    else:
        # rank r owns the key block of stores [8r, 8r+8) (one unbounded store at --gpus 1)
        key_lo = (8 * rank) * args.keyspace // stores_total
        key_hi = (8 * rank + 8) * args.keyspace // stores_total
        s = s_full if world == 1 else s_full.restrict_keys(key_lo, key_hi, drop_empty=True)
        store = CommandStore(device=device_index, key_lo=key_lo, key_hi=key_hi,
                             window=args.window, profile=True,
                             store_bounds=bounds[8 * rank:8 * rank + 9] if world > 1 else None)
        store.upload(s)
        if world > 1:
            uid = [CommandStore.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            store.comm_init(world, rank, uid[0])
            rccl = store.comm_size()

    xinfo = {}

    def step():
        if segments:
            xinfo.update(segment_exchange(store, rank, world, xdev, store_device=torch.device("cuda", device_index)))
        store.compute()
        if world > 1 and not segments:
            store.exchange_merge(n_total)
        if args.waiting_on:
            store.waiting_on_compute()

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()

    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    # the timed steps run without the profiling events (their records cost host time and marker
    # packets between the kernels); the stage split comes from a profiled pass over the same batch
    store.set_profile(False)
    barrier()
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    hip.hipDeviceSynchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_local = elapsed
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    store.set_profile(True)
    prof_steps = max(1, min(args.steps, 5))
    stage = {"validate": 0.0, "sort": 0.0, "segment": 0.0, "count": 0.0, "scan": 0.0, "fill": 0.0, "range_fill": 0.0,
             "compact": 0.0, "total": 0.0, "exchange": 0.0, "merge": 0.0, "wo_bits": 0.0, "wo_preds": 0.0, "wo_level": 0.0}
    if segments:
        stage.update({"cfk_summary": 0.0, "cfk_carry": 0.0, "exchange_wall": 0.0})
    count_detail, scan_spins, scan_fallbacks = {}, 0, 0
    for _ in range(prof_steps):
        tx = time.perf_counter()
        step()
        if segments:
            a_ms, c_ms = store.segment_timing()
            stage["cfk_summary"] += a_ms
            stage["cfk_carry"] += c_ms
            stage["exchange_wall"] += (time.perf_counter() - tx) * 1e3     # summary + all-gather + carry + compute
        t = store.timing()
        stage["validate"] += t.validate_ms
        stage["sort"] += t.sort_ms
        stage["segment"] += t.segment_ms
        stage["count"] += t.count_ms
        stage["scan"] += t.scan_ms
        stage["fill"] += t.fill_ms
        stage["range_fill"] += t.range_ms
        stage["compact"] += t.compact_ms
        stage["total"] += t.total_ms
        for k, v in t.count_detail.items():
            count_detail[k] = count_detail.get(k, 0.0) + v
        scan_spins += t.scan_spins
        scan_fallbacks += t.scan_fallbacks
        if world > 1 and not segments:
            xms, mms = store.shard_timing()
            stage["exchange"] += xms
            stage["merge"] += mms
        if args.waiting_on:
            a, b, c = store.waiting_on_timing()
            stage["wo_bits"] += a
            stage["wo_preds"] += b
            stage["wo_level"] += c
    for k in stage:
        stage[k] /= prof_steps
    for k in count_detail:
        count_detail[k] /= prof_steps
    per_rank = None
    if segments:
        stage["exchange_wall"] -= stage["total"]        # host wall of summary + all-gather + carry
    if dist is not None:
        mine = {"rank": rank, "txns": s.n, "pairs": s.pairs, "compute_ms": stage["total"], "elapsed_s": elapsed_local}
        if segments:
            mine.update({"segment": list(seg), "cfk_summary_ms": stage["cfk_summary"], "cfk_carry_ms": stage["cfk_carry"],
                         "exchange_wall_ms": stage["exchange_wall"], "carry_entries": store.state()["carry_entries"],
                         "summary_entries": xinfo["summary_entries"][rank], "allgather_bytes_sent": xinfo["bytes_sent"],
                         "collective": "gloo (one-device rehearsal)" if args.one_device else "RCCL all_gather (torch.distributed nccl)"})
        else:
            mine.update({"rccl": list(rccl), "exchange_ms": stage["exchange"], "merge_ms": stage["merge"]})
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)

    # sizes for the byte model: the rank's own computed deps (keys: the partial before the exchange;
    # segments: the node-level deps of the segment's txns)
    if segments:
        step()
    else:
        store.compute()
    view = store.device_view()
    n = s.n
    P = s.pairs
    kc = int(view["kd_keys_total"])
    # the exact |txnIds| (the device view's txnIds are gapped: kd_vals_total is the array length)
    dd = store.download()
    U = int(dd.kd_val_off[-1])
    D = int(view["kd_k2v_total"]) - kc
    fill_sizes = (n, P, kc, U, D)
    if s.rng_off[-1] > 0:
        # the fill stage only builds key txns' KeyDeps (range txns' come from range_fill): size the
        # roofline unit by the key txns alone
        key_txn = ~s.domains().astype(bool)
        d_keys = np.diff(dd.kd_key_off.astype(np.int64))[key_txn]
        d_vals = np.diff(dd.kd_val_off.astype(np.int64))[key_txn]
        d_k2v = np.diff(dd.kd_k2v_off.astype(np.int64))[key_txn]
        kc_k = int(d_keys.sum())
        fill_sizes = (int(key_txn.sum()), int(np.diff(s.key_off.astype(np.int64))[key_txn].sum()), kc_k,
                      int(d_vals.sum()), int(d_k2v.sum()) - kc_k)
    wo_info = None
    if args.waiting_on:
        wo = store.waiting_on()
        wo_info = {"max_level": wo.max_level, "reduced_edges": wo.preds_total,
                   "bitset_words": int(wo.wo_off[-1]), "level_histogram_top": int(np.bincount(wo.level).max())}

    boundary = None
    resident = None
    registered = None
    ready = None
    if world == 1 and not args.waiting_on:
        boundary = boundary_rate(store, s)
        if s.rng_off[-1] == 0 and args.resident:
            resident = resident_split(s, args, stage["total"])
        if s.rng_off[-1] == 0 and args.registered:
            registered = registered_batches(s, args)
        if s.rng_off[-1] == 0 and args.ready:
            ready = ready_schedule(s, args)
            if args.ready_events:
                ready["events_mode"] = ready_schedule(s, args, events=True)
            if args.ready_cpu_batch:
                one = types.SimpleNamespace(ready_batch=args.ready_cpu_batch, ready_batches=1, keyspace=args.keyspace)
                ready["same_sample"] = {"device": ready_schedule(s, one), "cpu_baseline": ready_cpu(s, args)}

    if rank != 0:
        store.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    txns_total = n_total * args.steps
    value = txns_total / elapsed
    B = algorithmic_bytes(n, P, kc, U, D)
    Bf = fill_kernel_bytes(*fill_sizes)
    fill_gbs = Bf / (stage["fill"] * 1e-3) / 1e9 if stage["fill"] > 0 else None
    pipe_gbs = B / (stage["total"] * 1e-3) / 1e9 if stage["total"] > 0 else None

    traffic = measured_traffic(args.config)
    cpu = None
    if not args.no_cpu:
        cpu = cpu_baseline(s_full, args)
        if args.waiting_on and cpu is not None:
            cpu["levelling_1core"] = levelling_cpu(s_full, wo.level if wo_info is not None else None,
                                                   stage["wo_level"])

    line = {
        "metric": "PreAccept deps/sec (batched txns)",
        "value": value,
        "unit": "txns/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 integer",
        "data": "synthetic (SURVEY.md §8d stream, splitmix64 + Zipf rejection-inversion)",
        "config": {"workload": workload_name(args, world),
                   "n_txns_per_gpu": args.n, "keys_per_txn": args.keys_per_txn, "keyspace": args.keyspace,
                   "zipf": args.zipf, "window": args.window, "seed": args.seed,
                   "n_txns_total": n_total,
                   "gpu_stores": world, "evensplit_stores": stores_total if world > 1 else None,
                   "parallelism": (f"stream segments x{world}: every rank owns 1/{world} of the stream for all "
                                   f"{stores_total} CommandStores; CFK summaries all-gathered" if segments else
                                   f"keyspace-sharded x{world}" + (" + RCCL exchange/union" if world > 1 else ""))},
        "rccl_ranks": (per_rank[0]["rccl"][0] if per_rank and not segments else world if per_rank else None),
        "deps_per_s": D * world * args.steps / elapsed,
        "sizes": {"N": n, "P": P, "keys_out": kc, "U": U, "D": D},
        "stage_ms": stage,
        "stage_ms_source": f"HIP events on the store's stream, mean of a profiled pass of {prof_steps} steps "
                           "after the timed steps (which run without the events)",
        "count_stage_ms": count_detail,
        "scan_lookback": {"spins_per_step": scan_spins / prof_steps,
                          "fallbacks_total": scan_fallbacks},
        "roofline": {"kernel": "fill stage: txnrec_kernel + keydeps_fast_kernel<16> + keydeps_kernel<1,8>",
                     "bound": "hbm",
                     "achieved": fill_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": (fill_gbs / PEAK_HBM_GBS) if fill_gbs else None,
                     "traffic": traffic["traffic_bytes"] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None,
                     "algorithmic_bytes_per_launch": Bf},
        "pipeline_roofline": {"bytes": B, "achieved": pipe_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                              "frac": (pipe_gbs / PEAK_HBM_GBS) if pipe_gbs else None,
                              "formula": "SURVEY.md §8d B / device time of the whole pipeline"},
        "cpu_baseline": cpu,
    }
    if per_rank is not None:
        line["ranks"] = per_rank
    if wo_info is not None:
        line["waiting_on"] = wo_info
    if boundary is not None:
        line["boundary_inclusive"] = boundary
    if resident is not None:
        line["resident_batches"] = resident
    if registered is not None:
        line["registered_batches"] = registered
    if ready is not None:
        line["readiness"] = ready
    print(json.dumps(line))
    store.close()
    if dist is not None:
        dist.destroy_process_group()


def workload_name(args, world=1):
    if world > 1 and args.partition == "segments":
        return (f"config4: {world} x {args.n} key txns x {args.keys_per_txn} keys, Zipf({args.zipf}) over "
                f"{args.keyspace} keys, {8 * world} EvenSplit CommandStores, W={args.window}; rank r owns stream "
                f"segment r of every store: CFK summary + one all-gather + carry + node-level deps")
    if world > 1:
        return (f"config4: {world} x {args.n} key txns x {args.keys_per_txn} keys, Zipf({args.zipf}) over "
                f"{args.keyspace} keys, {8 * world} EvenSplit CommandStores (8 per GPU), W={args.window}; per-rank "
                f"partial deps + one RCCL exchange + on-device union")
    if args.waiting_on:
        return (f"config5: {args.n} key txns x {args.keys_per_txn} keys, Zipf({args.zipf}) over {args.keyspace} "
                f"keys, {args.write_frac:.0%} writes, W={args.window}; deps + WaitingOn bitsets + levelling "
                f"(all STABLE, executeAt = txnId)")
    if args.range_frac > 0:
        return (f"config3: {args.n} txns ({args.range_frac:.0%} range txns, 1-2 ranges len<= {args.range_len}), "
                f"{args.keys_per_txn} keys/key txn, Zipf({args.zipf}) over {args.keyspace} keys, W={args.window}")
    return (f"config2: {args.n} key txns x {args.keys_per_txn} keys, Zipf({args.zipf}) over {args.keyspace} keys, "
            f"{args.write_frac:.0%} writes, W={args.window}")


def boundary_rate(store, s):
    """PCIe-inclusive rate of the C-ABI entry accord_deps_batch (host SoA batch in, host CSR out:
    H2D upload + pipeline + D2H of every output array), as a Java caller would see it.  Reported
    next to `value`, never as it; the second of two calls is timed (the first sizes the buffers)."""
    import ctypes as C
    from accord_amd import _Deps, lib
    b = s.c_batch()
    ms = None
    for _ in range(2):
        d = _Deps()
        t0 = time.perf_counter()
        rc = lib().accord_deps_batch(store._h, C.byref(b), C.byref(d))
        ms = (time.perf_counter() - t0) * 1e3
        lib().accord_deps_release(C.byref(d))
        if rc != 0:
            return None
    return {"ms": ms, "txns_per_s": s.n / (ms * 1e-3), "path": "accord_deps_batch, host buffers in and out"}


def resident_split(s, args, single_ms, batch_counts=(8, 64, 512), reps=3):
    """The same stream fed as B consecutive batches to one resident store (CommandsForKey state kept
    in HBM across batches, deps identical to the single batch), for each B of batch_counts: device
    time of the computes (HIP events, with the per-stage split) and host wall time around them
    (uploads excluded), per full stream, against the single-batch device time."""
    from accord_amd import CommandStore
    out = []
    with CommandStore(device=0, key_lo=0, key_hi=args.keyspace, window=args.window, profile=True,
                      resident=True) as st:
        for batches in batch_counts:
            pts = [i * s.n // batches for i in range(batches + 1)]
            parts = [s.slice(a, b) for a, b in zip(pts[:-1], pts[1:])]
            best = None
            for _ in range(reps + 1):
                st.reset()
                acc = {"device_ms": 0.0, "compute_wall_ms": 0.0, "validate_ms": 0.0, "sort_ms": 0.0,
                       "segment_ms": 0.0, "count_ms": 0.0, "scan_ms": 0.0, "fill_ms": 0.0, "compact_ms": 0.0}
                for p in parts:
                    st.upload(p)
                    t0 = time.perf_counter()
                    st.compute()
                    acc["compute_wall_ms"] += (time.perf_counter() - t0) * 1e3
                    t = st.timing()
                    acc["device_ms"] += t.total_ms
                    for k in ("validate_ms", "sort_ms", "segment_ms", "count_ms", "scan_ms", "fill_ms", "compact_ms"):
                        acc[k] += getattr(t, k)
                if best is None or acc["device_ms"] < best["device_ms"]:
                    best = acc
            best["batches"] = batches
            best["single_batch_device_ms"] = single_ms
            best["device_ratio"] = best["device_ms"] / single_ms if single_ms else None
            best["wall_ratio"] = best["compute_wall_ms"] / single_ms if single_ms else None
            out.append(best)
    return out


ST_COMMITTED, ST_APPLIED = 4, 6


def registered_batches(s, args, lag_applied=4, lag_rb=8, reps=2):
    """The real drop-in mode: a resident store with no status-at-time model (window
    ACCORD_WINDOW_NONE) fed the first reg_batches x reg_batch txns of the stream, with the event
    schedule of tests/status_events.py committed_schedule -- right after batch b is computed its txns
    are registered COMMITTED at executeAt = TxnId and those of batch b - 4 APPLIED
    (accord_txn_register), and the store's RedundantBefore moves to the first txn of batch b - 8
    (accord_redundant_before_set: CommandsForKey.withRedundantBefore truncates the resident history,
    RedundantBefore.collectDeps adds the bound to every later txn's deps).  Per batch: the compute's
    device time (HIP events) and stages, and the host wall time of compute, register and
    RedundantBefore calls (uploads excluded) -- the walls from a second pass over a store without the
    profiling events (compute_wall_profiled_ms_per_batch: with them).  Beside it: the status-at-time resident store (window
    W) fed the same batches, for the fill-stage comparison."""
    from accord_amd import CommandStore, WINDOW_NONE
    bsz, nb = args.reg_batch, args.reg_batches
    nb = min(nb, s.n // bsz)
    parts = [s.slice(b * bsz, (b + 1) * bsz) for b in range(nb)]
    starts = [b * bsz for b in range(nb + 1)]
    ks = args.keyspace

    def events(b):
        idx = np.arange(starts[b], starts[b + 1])
        st = np.full(idx.size, ST_COMMITTED, np.uint8)
        if b >= lag_applied:
            a = np.arange(starts[b - lag_applied], starts[b - lag_applied + 1])
            idx = np.concatenate([a, idx])
            st = np.concatenate([np.full(a.size, ST_APPLIED, np.uint8), st])
        return (s.msb[idx], s.lsb[idx], s.node[idx], st, s.msb[idx], s.lsb[idx], s.node[idx])

    evs = [events(b) for b in range(nb)]

    def run(window, with_events, profile=True):
        best = None
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=window, profile=profile, resident=True) as st:
            for _ in range(reps + 1):
                st.reset()
                st.redundant_before()
                acc = {"device_ms": 0.0, "fill_ms": 0.0, "count_ms": 0.0, "sort_ms": 0.0, "segment_ms": 0.0,
                       "compact_ms": 0.0, "compute_wall_ms": 0.0, "register_wall_ms": 0.0, "rb_wall_ms": 0.0,
                       "upload_wall_ms": 0.0}
                for b, p in enumerate(parts):
                    tu = time.perf_counter()
                    st.upload(p)
                    acc["upload_wall_ms"] += (time.perf_counter() - tu) * 1e3
                    t0 = time.perf_counter()
                    st.compute()
                    t1 = time.perf_counter()
                    if profile:
                        t = st.timing()
                        acc["device_ms"] += t.total_ms
                        acc["fill_ms"] += t.fill_ms
                        acc["count_ms"] += t.count_ms
                        acc["sort_ms"] += t.sort_ms
                        acc["segment_ms"] += t.segment_ms
                        acc["compact_ms"] += t.compact_ms
                    acc["compute_wall_ms"] += (t1 - t0) * 1e3
                    if with_events:
                        t2 = time.perf_counter()
                        st.register(*evs[b])
                        t3 = time.perf_counter()
                        acc["register_wall_ms"] += (t3 - t2) * 1e3
                        if b >= lag_rb and starts[b - lag_rb] > 0:
                            st.redundant_before(start=[0], end=[ks - 1], start_epoch=[0], end_epoch=[1 << 62],
                                                bound=[starts[b - lag_rb]], min_epoch=0)
                            acc["rb_wall_ms"] += (time.perf_counter() - t3) * 1e3
                carry = st.state()["carry_entries"]
                if best is None or acc["compute_wall_ms"] < best[0]["compute_wall_ms"]:
                    best = (acc, carry)
        acc, carry = best
        per = {k.replace("_ms", "_ms_per_batch"): v / nb for k, v in acc.items()}
        per["carry_entries_end"] = carry
        return per, acc

    # device stages from a profiled store (HIP events on its stream); the host walls from a store
    # without them (the events' records cost ~2 us of host time each, a dozen per compute)
    reg, racc = run(WINDOW_NONE, True)
    sat, _ = run(args.window, False)
    for per, win in ((reg, run(WINDOW_NONE, True, profile=False)[0]), (sat, run(args.window, False, profile=False)[0])):
        per["compute_wall_profiled_ms_per_batch"] = per["compute_wall_ms_per_batch"]
        for k in ("compute_wall_ms_per_batch", "register_wall_ms_per_batch", "rb_wall_ms_per_batch", "upload_wall_ms_per_batch"):
            per[k] = win[k]
    wall = (reg["compute_wall_ms_per_batch"] + reg["register_wall_ms_per_batch"] + reg["rb_wall_ms_per_batch"]) * nb
    return {"schedule": f"{nb} batches x {bsz} txns of the config-2 stream; after batch b: COMMITTED "
                        f"(executeAt = TxnId) for b, APPLIED for b-{lag_applied}, RedundantBefore = first txn "
                        f"of b-{lag_rb}",
            "txns": nb * bsz,
            "txns_per_s_wall": nb * bsz / (wall * 1e-3),
            "txns_per_s_device": nb * bsz / (racc["device_ms"] * 1e-3),
            "registered": reg,
            "status_at_time_W": sat,
            "fill_ratio_vs_status_at_time": (reg["fill_ms_per_batch"] / sat["fill_ms_per_batch"])
            if sat["fill_ms_per_batch"] else None,
            "device_ratio_vs_status_at_time": (reg["device_ms_per_batch"] / sat["device_ms_per_batch"])
            if sat["device_ms_per_batch"] else None}


ST_STABLE = 5


def ready_schedule(s, args, rounds_per_batch=4, events=False):
    """Execution readiness (include/accord_deps.h accord_ready_update) over the
    first ready_batches x ready_batch txns of the stream in a registered-status store: per batch the
    deps are computed, the batch is registered STABLE at executeAt = TxnId and its WaitingOn
    initialised (the txns join the waiting set), then up to rounds_per_batch rounds of
    accord_ready_update -> the ready txns registered APPLIED; finally the set is drained.  Reports the
    wall time of the ready_update calls (device summaries + evaluation + one host read) against the
    txns they released.  events: the store in event-exact mode (accord_ready_set_mode(ACCORD_READY_
    EVENTS)), where key bits clear when a registration's events reach the key -- that work is in the
    registration calls, reported as register_ms_per_call beside the update calls."""
    from accord_amd import CommandStore, WINDOW_NONE
    bsz, nb = args.ready_batch, min(args.ready_batches, s.n // args.ready_batch)
    upd_ms, app_ms, calls, released, rounds = 0.0, 0.0, 0, 0, 0
    reg_ms, regs = 0.0, 0

    def rnd(st):
        nonlocal upd_ms, app_ms, calls, released, rounds
        t0 = time.perf_counter()
        ready, waiting = st.ready_update()
        upd_ms += (time.perf_counter() - t0) * 1e3
        calls += 1
        if ready.size:
            released += ready.size
            rounds += 1
            t1 = time.perf_counter()
            st.register(s.msb[ready], s.lsb[ready], s.node[ready], np.full(ready.size, ST_APPLIED, np.uint8),
                        s.msb[ready], s.lsb[ready], s.node[ready])
            app_ms += (time.perf_counter() - t1) * 1e3
        return ready.size, waiting

    with CommandStore(device=0, key_lo=0, key_hi=args.keyspace, window=WINDOW_NONE, resident=True) as st:
        if events:
            st.ready_mode(True)
        for b in range(nb):
            lo, hi = b * bsz, (b + 1) * bsz
            st.upload(s.slice(lo, hi))
            st.compute()
            idx = np.arange(lo, hi)
            t2 = time.perf_counter()
            st.register(s.msb[idx], s.lsb[idx], s.node[idx], np.full(bsz, ST_STABLE, np.uint8),
                        s.msb[idx], s.lsb[idx], s.node[idx])
            reg_ms += (time.perf_counter() - t2) * 1e3
            regs += 1
            st.waiting_on_initialise()
            for _ in range(rounds_per_batch):
                if rnd(st)[0] == 0:
                    break
        waiting = 1
        for _ in range(100000):
            r, waiting = rnd(st)
            if r == 0:
                break
    return {"schedule": f"{nb} batches x {bsz} txns of the config-2 stream, registered-status store: each batch "
                        f"STABLE (executeAt = TxnId) and initialised, <= {rounds_per_batch} ready -> APPLIED rounds "
                        f"per batch, then drained",
            "txns": nb * bsz, "released": released, "left_waiting": waiting, "update_calls": calls,
            "release_rounds": rounds, "update_ms_per_call": upd_ms / max(1, calls),
            "mode": "events" if events else "poll",
            "register_stable_ms_per_batch": reg_ms / max(1, regs),
            "register_applied_ms_per_call": app_ms / max(1, rounds),
            "per_call_ms_update_plus_register": (upd_ms + app_ms) / max(1, calls),
            "released_txns_per_s_update_wall": released / (upd_ms * 1e-3) if upd_ms else None,
            "apply_register_ms_total": app_ms}


def ready_cpu(s, args):
    """CPU baseline of the readiness leg: the oracle's restatement (or_lstore_ready over literal
    CommandsForKey objects: the count test of every waiting txn at every call, one thread) draining
    one batch of --ready-cpu-batch txns registered STABLE -- the same schedule the device runs beside
    it ("device" in the same dict)."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        bsz = min(args.ready_cpu_batch, s.n)
        L = oracle_lib.LStore(args.keyspace)
        idx = np.arange(bsz)
        part = L.batch(s.slice(0, bsz))
        L.register(s.msb[idx], s.lsb[idx], s.node[idx], np.full(bsz, ST_STABLE, np.uint8), s.msb[idx], s.lsb[idx],
                   s.node[idx])
        L.waiting_add(0, part)
        upd, calls, released = 0.0, 0, 0
        for _ in range(100000):
            t0 = time.perf_counter()
            r = L.ready()
            upd += time.perf_counter() - t0
            calls += 1
            if r.size == 0:
                break
            released += r.size
            L.register(s.msb[r], s.lsb[r], s.node[r], np.full(r.size, ST_APPLIED, np.uint8), s.msb[r], s.lsb[r], s.node[r])
        L.close()
        return {"value": released / upd if upd else None, "unit": "released txns/s (ready calls)", "cores": 1,
                "kind": "port", "update_calls": calls, "update_ms_per_call": upd * 1e3 / max(1, calls),
                "sample": f"one batch of {bsz} config-2 txns STABLE at TxnId, drained ready -> APPLIED; literal "
                          f"restatement, every waiting txn re-tested per call ({upd:.1f} s)"}
    except Exception as e:  # pragma: no cover
        return {"value": None, "sample": f"failed: {e}"}


def measured_traffic(config):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC passes of the
    same workload (profiles/traffic_config<N>.json, written by scripts/traffic_json.py): PMC
    counters need their own rocprofv3 run, so a bench run reports the last committed measurement."""
    path = os.path.join(ROOT, "profiles", f"traffic_config{config}.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(s, args):
    """The oracle's literal restatement of the reference algorithm (sorted-array CommandsForKey
    copied/re-sorted on every status change, linear mapReduceActive scan, RelationMultiMap
    builder) on a prefix of the same stream.  Key-only streams run the reference's node-level
    shape: S = 8 CommandStores (EvenSplit of the keyspace), one thread per store
    (impl/InMemoryCommandStore.java:1131-1148; ctypes releases the GIL for each store's call), then
    the coordinator's union of the 8 partials (PreAccept.reduce / Deps.merge) -- the same deps the
    GPU's single store produces.  The prefix starts at --cpu-sample (8192) and doubles while the
    next run is expected to fit --cpu-budget seconds; the largest completed run is reported.  Beside
    it, config 1 (64k txns x 4 keys, uniform 100k keys, one store) at full size."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        from concurrent.futures import ThreadPoolExecutor
        key_only = int(s.rng_off[-1]) == 0 and not args.waiting_on
        threads = min(8, os.cpu_count() or 1) if key_only else 1

        def run(m):
            pre = s.prefix(m)
            t0 = time.perf_counter()
            if key_only:
                stores = [pre.restrict_keys(b * args.keyspace // 8, (b + 1) * args.keyspace // 8) for b in range(8)]
                with ThreadPoolExecutor(threads) as ex:
                    parts = list(ex.map(lambda st: oracle_lib.deps_literal(st, args.window), stores))
                oracle_lib.deps_union(parts)
            else:
                d = oracle_lib.deps_literal(pre, args.window)
                if args.waiting_on:
                    oracle_lib.waiting_on(d)
            return time.perf_counter() - t0

        m = min(args.cpu_sample or 8192, s.n)
        spent = 0.0
        while True:
            dt = run(m)
            spent += dt
            done = (m, dt)
            # a doubled prefix costs >= 2x (CommandsForKey histories grow with it): stop unless it fits
            if m >= s.n or spent + 2.5 * dt > args.cpu_budget:
                break
            m = min(2 * m, s.n)
        m, dt = done
        how = (f"8 stores on {threads} threads + union of the partials" if key_only else "1 store, 1 thread") + \
              (" + levelling" if args.waiting_on else "")
        out = {"value": m / dt, "unit": "txns/s", "cores": threads, "kind": "port",
               "sample": f"first {m} txns of the config-{args.config} stream, literal reference algorithm, "
                         f"{how}, {dt:.1f} s; CFK histories grow with the prefix so the full run would be slower",
               "nproc": os.cpu_count(), "cpu_model": _cpu_model()}
        from accord_amd import generate_stream
        c1 = generate_stream(65536, 4, 100_000, 0.0, 0.5, seed=1)
        t0 = time.perf_counter()
        oracle_lib.deps_literal(c1, args.window)
        t1 = time.perf_counter() - t0
        out["config1_full"] = {"value": c1.n / t1, "unit": "txns/s", "seconds": t1, "cores": 1,
                               "sample": f"config 1 at full size: 65536 txns x 4 keys, uniform over 100000 keys, "
                                         f"50% writes, W={args.window}, one store, literal reference algorithm"}
        return out
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "txns/s", "cores": 1, "kind": "port", "sample": f"failed: {e}"}


def levelling_cpu(s, gpu_level, gpu_ms):
    """One host core levelling the same reduced DAG the device levels (config 5): the oracle's
    reduction of the stream (tests/oracle_lib.reduced_dag; built untimed) and or_levels_csr timed
    alone, best of three; its levels compared with the device's."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        off, preds = oracle_lib.reduced_dag(s)
        best, lv = None, None
        for _ in range(3):
            t0 = time.perf_counter()
            lv = oracle_lib.levels_csr(off, preds)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return {"ms": best * 1e3, "edges": int(preds.size), "cores": 1, "kind": "port",
                "levels_equal_device": (bool(np.array_equal(lv, gpu_level)) if gpu_level is not None else None),
                "device_wo_level_ms": gpu_ms,
                "sample": "the whole reduced DAG of config 5 (every txn), or_levels_csr -O2, best of 3"}
    except Exception as e:  # pragma: no cover
        return {"ms": None, "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
