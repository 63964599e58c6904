"""Segment shares of the striped levelling's stripe walk (csrc/levels.hip lv_stripe_kernel) from a
-DACCORD_LV_STAMPS build: ACCORD_LIB=<stamps build> python3 scripts/lv_stamps.py [stripe ...]
(config 5 stream; stamps drain the wave's LDS queue, so read the shares, not the run time)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import CommandStore, generate_stream, lib  # noqa: E402

NAMES = ["chunk start", "classify", "ext edges", "gather+fold", "serial step", "row stores"]
s = generate_stream(1 << 22, 4, 10_000, 0.99, 0.9, seed=5)
L = lib()
f = L.accord_dbg_lv_stamps
f.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * 16)()
for z in (sys.argv[1:] or ["2048", "4096"]):
    os.environ["ACCORD_LV_STRIPE"] = z
    with CommandStore(device=0, key_lo=0, key_hi=10_000, window=256) as st:
        st.upload(s)
        st.compute()
        st.waiting_on_compute()
        f(buf)
        st.waiting_on_compute()
        f(buf)
    tot = sum(buf[q] for q in range(6))
    ch = buf[7]
    print(f"stripe {z}: chunks {ch}, waves {buf[8]}, cycles/chunk/wave {tot / max(1, ch):.0f}")
    for q, nm in enumerate(NAMES):
        print(f"  {nm:14s} {100.0 * buf[q] / max(1, tot):5.1f} %   {buf[q] / max(1, ch):8.0f} cyc/chunk")
