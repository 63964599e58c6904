"""Per-rank compute of the N-GPU weak-scaling bench on one GPU (no exchange): the N x config-2
stream restricted to rank r's key block, as bench.py --gpus N builds it.
python scripts/rank_sim.py [N] [rank]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import CommandStore, generate_stream
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
r = int(sys.argv[2]) if len(sys.argv) > 2 else 0
n, ks = 1 << 20, 100_000
s_full = generate_stream(n * N, 8, ks, 0.99, 0.5, seed=2)
lo, hi = (8 * r) * ks // (8 * N), (8 * r + 8) * ks // (8 * N)
s = s_full.restrict_keys(lo, hi, drop_empty=True)
print(f"N={N} rank={r}: {s.n} txns, {s.pairs} pairs in keys [{lo},{hi})", flush=True)
with CommandStore(device=0, key_lo=lo, key_hi=hi, window=256, profile=True) as st:
    st.upload(s)
    for i in range(6):
        st.compute()
        t = st.timing()
        if i >= 2:
            print({k: round(getattr(t, k), 3) for k in ("validate_ms", "sort_ms", "segment_ms", "count_ms", "scan_ms",
                                                         "fill_ms", "range_ms", "compact_ms", "total_ms")}, flush=True)
