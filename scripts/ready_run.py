"""The bench --ready schedule alone (profiling helper): python scripts/ready_run.py [batches] [batch]"""
import os, sys, time, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import generate_stream
import bench
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16
bsz = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
s = generate_stream(nb * bsz, 8, 100_000, 0.99, 0.5, seed=2)
args = types.SimpleNamespace(ready_batch=bsz, ready_batches=nb, keyspace=100_000)
t0 = time.perf_counter()
print(bench.ready_schedule(s, args), f"{time.perf_counter() - t0:.1f} s", flush=True)
