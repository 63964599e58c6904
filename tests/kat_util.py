"""Helpers shared by the KAT tests (CPU oracle and GPU)."""
import json
import os

import numpy as np

from accord_amd import Stream

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KIND = {"R": 0, "W": 1, "E": 2, "S": 3, "X": 4, "L": 5}


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)["kats"]


def kat_stream(kat) -> Stream:
    txns = kat["txns"]
    n = len(txns)
    msb = np.zeros(n, np.uint64)
    lsb = np.zeros(n, np.uint64)
    node = np.zeros(n, np.int32)
    key_off = np.zeros(n + 1, np.uint32)
    rng_off = np.zeros(n + 1, np.uint32)
    keys, rs, re = [], [], []
    accept = any("exec" in t for t in txns)
    emsb = np.zeros(n, np.uint64)
    elsb = np.zeros(n, np.uint64)
    enode = np.zeros(n, np.int32)
    for i, t in enumerate(txns):
        hlc = t.get("hlc", 1_000_000 + i)
        is_range = "ranges" in t
        flags = (KIND[t["kind"]] << 1) | (1 if is_range else 0)
        msb[i] = (1 << 15) | (hlc >> 48)
        lsb[i] = ((hlc << 16) | flags) & ((1 << 64) - 1)
        node[i] = t.get("node", 1 + i % 7)
        for k in t.get("keys", []):
            keys.append(k)
        for (a, b) in t.get("ranges", []):
            rs.append(a)
            re.append(b)
        key_off[i + 1] = len(keys)
        rng_off[i + 1] = len(rs)
        # Accept: startedBefore = executeAt (a Timestamp: hlc, flags, node), default = the txnId
        e = t.get("exec")
        emsb[i], elsb[i], enode[i] = msb[i], lsb[i], node[i]
        if e is not None:
            ehlc = e["hlc"]
            emsb[i] = (1 << 15) | (ehlc >> 48)
            elsb[i] = ((ehlc << 16) | e.get("flags", 0)) & ((1 << 64) - 1)
            enode[i] = e["node"]
    ex = dict(exec_msb=emsb, exec_lsb=elsb, exec_node=enode) if accept else {}
    return Stream(msb, lsb, node, key_off, np.array(keys, np.uint32), rng_off, np.array(rs, np.uint32),
                  np.array(re, np.uint32), **ex)


def max_key(s: Stream) -> int:
    m = 0
    if s.key_ord.size:
        m = max(m, int(s.key_ord.max()))
    if s.rng_end.size:
        m = max(m, int(s.rng_end.max()))
    return m
