"""The --registered and --resident legs of bench.py alone (config-2 stream prefix), for kernel traces:
rocprofv3 --kernel-trace -- python3 scripts/reg_trace.py [registered|resident|ready]"""
import json
import os
import sys
import types

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "cassandra-accord_amd")]
import bench  # noqa: E402
from accord_amd import generate_stream  # noqa: E402

leg = sys.argv[1] if len(sys.argv) > 1 else "registered"
n = 1 << 17
s = generate_stream(n, 8, 100_000, 0.99, 0.5, seed=2)
args = types.SimpleNamespace(reg_batch=1024, reg_batches=64, keyspace=100_000, window=256,
                             ready_batch=4096, ready_batches=4)
if leg == "registered":
    out = bench.registered_batches(s, args, reps=1)
elif leg == "resident":
    out = bench.resident_split(s, args, 0.0, batch_counts=(1, 8, 64), reps=1)
else:
    out = bench.ready_schedule(s, args)
print(json.dumps(out))
