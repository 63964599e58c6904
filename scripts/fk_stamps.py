"""Segment shares of the fast fill kernel's txn loop from a -DACCORD_FK_STAMPS build:
ACCORD_LIB=<stamps build> python3 scripts/fk_stamps.py [config-2 args]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import CommandStore, generate_stream, lib  # noqa: E402

NAMES = ["prefetch issue", "phase 1", "far deps", "union", "keys+header", "phase 2", "rotation"]
s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, seed=2)
L = lib()
f = L.accord_dbg_fk_stamps
f.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * 16)()
with CommandStore(device=0, key_lo=0, key_hi=100_000, window=256) as st:
    st.upload(s)
    st.compute()
    f(buf)
    for _ in range(3):
        st.compute()
    f(buf)
tot = sum(buf[q] for q in range(7))
txns = buf[7]
print(f"txn iterations {txns}, waves {buf[8]}, cycles/txn/wave {tot / max(1, txns):.0f}")
for q, nm in enumerate(NAMES):
    print(f"  {nm:16s} {100.0 * buf[q] / tot:5.1f} %   {buf[q] / max(1, txns):7.0f} cyc/txn")
