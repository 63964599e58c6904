"""Device time of accord_max_conflicts_fold on the config-2 stream (HIP events on the store's stream)."""
import ctypes as C
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cassandra-accord_amd"))
from accord_amd import CommandStore, generate_stream, lib

s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, seed=2)
with CommandStore(device=0, key_lo=0, key_hi=100_000, window=256, profile=True) as st:
    ms = []
    for i in range(8):
        st.upload(s)                       # a batch folds once: a new upload starts it again
        st.max_conflicts_reset()
        st.max_conflicts_fold(download=False)
        f = C.c_float()
        lib().accord_ops_timing(st._h, C.byref(f))
        ms.append(f.value)
    ms = sorted(ms[2:])
    P = int(s.key_off[-1])
    print(f"max_conflicts_fold config2: median {ms[len(ms)//2]:.3f} ms over {len(ms)} runs; "
          f"{(1 << 20) / ms[len(ms)//2] / 1e3:.1f} M txns/s; pairs {P}; "
          f"~130 B/pair -> {P * 130 / ms[len(ms)//2] / 1e6:.0f} GB/s")
