"""Config-2 stream as B resident batches (profiling helper): python scripts/resident_run.py [B] [reps]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import CommandStore, generate_stream
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << 20
s = generate_stream(n, 8, 100_000, 0.99, 0.5, seed=2)
pts = [i * n // B for i in range(B + 1)]
parts = [s.slice(a, b) for a, b in zip(pts[:-1], pts[1:])]
with CommandStore(device=0, key_lo=0, key_hi=100_000, window=256, profile=True, resident=True) as st:
    for r in range(reps):
        st.reset()
        dev = wall = 0.0
        for p in parts:
            st.upload(p)
            t0 = time.perf_counter()
            st.compute()
            wall += time.perf_counter() - t0
            t = st.timing()
            dev += t.total_ms
        print(f"rep {r}: device {dev:.3f} ms, compute wall {wall*1e3:.3f} ms", flush=True)
