"""Readiness call latency (and, --registered, the registered-batches compute leg) (accord_ready_update) on the bench's readiness schedule (bench.py
ready_schedule): per-call host wall, and -- with --trace CSV from `rocprofv3 --kernel-trace
--memory-copy-trace --output-format csv` -- the device work inside the calls (kernel busy time, copy
time, idle gaps).  python scripts/ready_latency.py [--batches 4] [--batch 4096]
python scripts/ready_latency.py --analyse DIR (the rocprofv3 output directory)"""
import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, ROOT)


def run_registered(a):
    """the bench's registered-batches leg (bench.py registered_batches) alone"""
    import types
    import bench
    from accord_amd import generate_stream
    s = generate_stream(a.batches * a.batch, 8, 100_000, 0.99, 0.5, seed=2)
    args = types.SimpleNamespace(reg_batch=a.batch, reg_batches=a.batches, keyspace=100_000, window=256)
    print(json.dumps(bench.registered_batches(s, args)), flush=True)


def run(a):
    import types
    import numpy as np
    import bench
    from accord_amd import generate_stream
    s = generate_stream(a.batches * a.batch, 8, 100_000, 0.99, 0.5, seed=2)
    args = types.SimpleNamespace(ready_batch=a.batch, ready_batches=a.batches, keyspace=100_000)
    t0 = time.perf_counter()
    r = bench.ready_schedule(s, args)
    r["wall_s"] = round(time.perf_counter() - t0, 3)
    print(json.dumps(r), flush=True)


def analyse(d):
    ks = [f for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)]
    ms = [f for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)]
    ev = []
    for f in ks:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"].split("(")[0][-40:]))
    for f in ms:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r.get("Direction", "copy")))
    ev.sort()
    # calls: a run of events that ends with the device-to-host copy after rd_eval_kernel
    calls, cur = [], []
    for e in ev:
        cur.append(e)
        if e[2].startswith("C:") and "DEVICE_TO_HOST" in e[2].upper() and any("rd_eval" in x[2] for x in cur):
            calls.append(cur)
            cur = []
    # only the events from the first readiness kernel on belong to the call
    rows = []
    for c in calls:
        i = next((k for k, x in enumerate(c) if "rd_part" in x[2] or "rd_summary" in x[2]), None)
        if i is None:
            continue
        c = c[max(0, i - 1):]
        span = c[-1][1] - c[0][0]
        busy = sum(x[1] - x[0] for x in c)
        rows.append((span, busy, len(c), [(x[2], x[1] - x[0]) for x in c]))
    rows.sort(key=lambda r: r[0])
    med = rows[len(rows) // 2]
    out = {"calls": len(rows), "span_us_median": med[0] / 1e3, "busy_us_median": med[1] / 1e3, "ops_median": med[2],
           "median_call": [(n, round(t / 1e3, 1)) for n, t in med[3]]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--analyse", default=None)
    ap.add_argument("--registered", action="store_true", help="the registered-batches leg instead")
    a = ap.parse_args()
    analyse(a.analyse) if a.analyse else run_registered(a) if a.registered else run(a)
