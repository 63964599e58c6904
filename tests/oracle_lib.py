"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (as the checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from accord_amd import PartialDeps, Stream

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(_ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

_u32p = C.POINTER(C.c_uint32)
_i32p = C.POINTER(C.c_int32)
_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)


class _OrStream(C.Structure):
    _fields_ = [("n", C.c_uint32), ("msb", _u64p), ("lsb", _u64p), ("node", _i32p),
                ("key_off", _u32p), ("key_ord", _u32p), ("rng_off", _u32p), ("rng_start", _u32p),
                ("rng_end", _u32p), ("window", C.c_uint32),
                ("exec_msb", _u64p), ("exec_lsb", _u64p), ("exec_node", _i32p), ("batch_end", _u32p),
                ("applied_before", _u32p), ("floor", _u32p)]


class _OrDeps(C.Structure):
    _fields_ = [("n", C.c_uint32),
                ("kd_key_off", _u32p), ("kd_keys", _u32p), ("kd_val_off", _u32p), ("kd_vals", _u32p),
                ("kd_k2v_off", _u32p), ("kd_k2v", _i32p),
                ("rd_rng_off", _u32p), ("rd_rng_start", _u32p), ("rd_rng_end", _u32p), ("rd_val_off", _u32p),
                ("rd_vals", _u32p), ("rd_r2v_off", _u32p), ("rd_r2v", _i32p)]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        L = C.CDLL(ORACLE_SO)
        L.or_stream_deps_literal.argtypes = [C.POINTER(_OrStream), C.POINTER(_OrDeps)]
        L.or_stream_deps_fast.argtypes = [C.POINTER(_OrStream), C.POINTER(_OrDeps)]
        L.or_stream_deps_literal_prefix.argtypes = [C.POINTER(_OrStream), C.c_uint32, C.POINTER(_OrDeps)]
        L.or_deps_free.argtypes = [C.POINTER(_OrDeps)]
        L.or_deps_free.restype = None
        L.or_max_conflicts.argtypes = ([C.c_uint32, _u64p, _u64p, _i32p, _u32p, _u32p, _u64p, _u64p, _i32p,
                                        C.c_uint32, C.c_uint32, _u64p, _u64p, _i32p, _u8p]
                                       + [_u64p, _u64p, _i32p, _u8p, _u8p]
                                       + [C.c_uint32, C.c_int, C.c_uint64, C.c_uint64, C.c_int32, _u32p])
        L.or_ts_compare.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32]
        L.or_ts_equals.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32]
        L.or_keydeps_build.argtypes = [C.c_uint32, _u32p, _u32p, C.c_uint32, _u64p, _u64p, _i32p,
                                       C.POINTER(_OrDeps)]
        L.or_keydeps_union.argtypes = [C.POINTER(_OrDeps), C.c_uint32, C.POINTER(_OrDeps), C.c_uint32,
                                       _u64p, _u64p, _i32p, C.POINTER(_OrDeps)]
        L.or_stab_key.argtypes = [C.c_uint32, _u32p, _u32p, C.c_uint32, _u32p]
        L.or_stab_key.restype = C.c_uint32
        L.or_waiting_on.argtypes = [C.POINTER(_OrDeps), C.c_uint32, _u32p, _u32p, C.POINTER(_u64p)]
        L.or_waiting_on_events.argtypes = [C.POINTER(_OrDeps), C.c_uint32, _u32p]
        L.or_initialise_waiting_on.argtypes = [C.POINTER(_OrDeps), C.c_uint32, _u64p, _u64p, _u64p, _i32p, _u8p,
                                               _u64p, _u64p, _i32p, _u32p, C.POINTER(_u64p), C.POINTER(_u64p)]
        L.or_levels_cfk.argtypes = [C.POINTER(_OrStream), C.POINTER(_OrDeps), _u32p]
        L.or_levels_csr.argtypes = [C.c_uint32, _u32p, _u32p, _u32p]
        L.or_deps_union.argtypes = [C.c_uint32, C.POINTER(_OrDeps), C.POINTER(_OrDeps)]
        L.or_stream_deps_stores.argtypes = [C.POINTER(_OrStream), C.c_uint32, _u32p, C.c_int, C.POINTER(_OrDeps)]
        L.or_deps_slice.argtypes = [C.POINTER(_OrDeps), _u32p, _u32p, _u32p, C.c_uint32, C.POINTER(_OrDeps)]
        L.or_deps_invert.argtypes = [C.POINTER(_OrDeps), C.c_int, _u32p, C.POINTER(_i32p)]
        L.or_redundant_collect.argtypes = [C.POINTER(_OrStream), C.c_uint32, _u32p, _u32p, _u64p, _u64p, _u32p,
                                           C.c_uint64, C.POINTER(_OrDeps)]
        L.or_cfk_reachable.argtypes = [C.POINTER(_OrStream), C.c_uint32, C.c_uint32, C.c_uint32, _u32p,
                                       C.POINTER(_u32p), C.POINTER(_u32p)]
        L.or_cfk_fold.argtypes = [C.c_uint32, _u32p, C.POINTER(_u32p), C.POINTER(_u32p), C.c_uint32, _u32p,
                                  C.POINTER(_u32p), C.POINTER(_u32p)]
        L.or_free.argtypes = [C.c_void_p]
        L.or_free.restype = None
        _LIB = L
    return _LIB


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def _to_partial(d: _OrDeps) -> PartialDeps:
    n = d.n
    kw = {}
    for f in ("kd_key_off", "kd_val_off", "kd_k2v_off", "rd_rng_off", "rd_val_off", "rd_r2v_off"):
        kw[f] = _arr(getattr(d, f), n + 1, np.uint32)
    kw["kd_keys"] = _arr(d.kd_keys, int(kw["kd_key_off"][-1]), np.uint32)
    kw["kd_vals"] = _arr(d.kd_vals, int(kw["kd_val_off"][-1]), np.uint32)
    kw["kd_k2v"] = _arr(d.kd_k2v, int(kw["kd_k2v_off"][-1]), np.int32)
    R = int(kw["rd_rng_off"][-1])
    kw["rd_rng_start"] = _arr(d.rd_rng_start, R, np.uint32)
    kw["rd_rng_end"] = _arr(d.rd_rng_end, R, np.uint32)
    kw["rd_vals"] = _arr(d.rd_vals, int(kw["rd_val_off"][-1]), np.uint32)
    kw["rd_r2v"] = _arr(d.rd_r2v, int(kw["rd_r2v_off"][-1]), np.int32)
    return PartialDeps(**kw)


def _or_stream(s: Stream, window: int, batch_end=None, applied_before=None, floor=None):
    keep = [np.ascontiguousarray(a) for a in (s.msb, s.lsb, s.node, s.key_off, s.key_ord, s.rng_off,
                                              s.rng_start, s.rng_end)]
    msb, lsb, node, ko, kord, ro, rs, re = keep
    o = _OrStream()
    o.n = s.n
    o.msb = msb.ctypes.data_as(_u64p)
    o.lsb = lsb.ctypes.data_as(_u64p)
    o.node = node.ctypes.data_as(_i32p)
    o.key_off = ko.ctypes.data_as(_u32p)
    o.key_ord = kord.ctypes.data_as(_u32p)
    o.rng_off = ro.ctypes.data_as(_u32p)
    o.rng_start = rs.ctypes.data_as(_u32p)
    o.rng_end = re.ctypes.data_as(_u32p)
    o.window = window
    if s.exec_msb is not None:
        ex = [np.ascontiguousarray(s.exec_msb, dtype=np.uint64), np.ascontiguousarray(s.exec_lsb, dtype=np.uint64),
              np.ascontiguousarray(s.exec_node, dtype=np.int32)]
        keep += ex
        o.exec_msb = ex[0].ctypes.data_as(_u64p)
        o.exec_lsb = ex[1].ctypes.data_as(_u64p)
        o.exec_node = ex[2].ctypes.data_as(_i32p)
    if batch_end is not None:
        be = np.ascontiguousarray(batch_end, dtype=np.uint32)
        keep.append(be)
        o.batch_end = be.ctypes.data_as(_u32p)
    if applied_before is not None:
        ab = np.ascontiguousarray(applied_before, dtype=np.uint32)
        keep.append(ab)
        o.applied_before = ab.ctypes.data_as(_u32p)
    if floor is not None:
        fl = np.ascontiguousarray(floor, dtype=np.uint32)
        keep.append(fl)
        o.floor = fl.ctypes.data_as(_u32p)
    return o, keep


class OracleError(RuntimeError):
    def __init__(self, rc):
        super().__init__(f"oracle rc={rc}")
        self.rc = rc


def batch_starts(sizes):
    """applied_before[i] of the committed-per-batch schedule: the first position of i's batch."""
    starts = np.cumsum(np.asarray(sizes, np.int64)) - np.asarray(sizes, np.int64)
    return np.repeat(starts, sizes).astype(np.uint32)


def batch_ends(sizes):
    """batch_end[i] for a stream fed as consecutive batches of the given sizes."""
    ends = np.cumsum(np.asarray(sizes, np.int64))
    return np.repeat(ends, sizes).astype(np.uint32)


def deps_literal(s: Stream, window: int, limit: int | None = None, batch_end=None) -> PartialDeps:
    """Literal restatement (real CFK objects, per-status-change copies).  batch_end: the stream is
    fed batch by batch to one resident store (see batch_ends)."""
    o, keep = _or_stream(s, window, batch_end)
    d = _OrDeps()
    if limit is None:
        rc = lib().or_stream_deps_literal(C.byref(o), C.byref(d))
    else:
        rc = lib().or_stream_deps_literal_prefix(C.byref(o), limit, C.byref(d))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(d)
    finally:
        lib().or_deps_free(C.byref(d))


def deps_fast(s: Stream, window: int, batch_end=None, applied_before=None, floor=None) -> PartialDeps:
    """Fast restatement; applied_before[i] (optional) replaces i - W as the position below which
    txns are committed at executeAt = txnId, floor[i] (optional) is the shardRedundantBefore below
    which key entries were truncated (see oracle.h)."""
    o, keep = _or_stream(s, window, batch_end, applied_before, floor)
    d = _OrDeps()
    rc = lib().or_stream_deps_fast(C.byref(o), C.byref(d))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(d)
    finally:
        lib().or_deps_free(C.byref(d))


def _take_entries(n, kp, ep):
    try:
        return _arr(kp, n.value, np.uint32), _arr(ep, n.value, np.uint32)
    finally:
        lib().or_free(C.cast(kp, C.c_void_p))
        lib().or_free(C.cast(ep, C.c_void_p))


def cfk_reachable(s: Stream, lo: int, hi: int, thr: int):
    """or_cfk_reachable: per key, the CommandsForKey entries of txns [lo, hi) a txn at position
    >= thr + W can still reach -- (key[], ent[] = kind << 29 | position), key-major.  A segment's
    summary is cfk_reachable(s, a, b, b - W); the state at the start of segment r is
    cfk_reachable(s, 0, a_r, a_r - W)."""
    o, keep = _or_stream(s, 0)
    n, kp, ep = C.c_uint32(), _u32p(), _u32p()
    rc = lib().or_cfk_reachable(C.byref(o), lo, hi, max(0, thr), C.byref(n), C.byref(kp), C.byref(ep))
    if rc != 0:
        raise OracleError(rc)
    return _take_entries(n, kp, ep)


def cfk_fold(parts, thr: int):
    """or_cfk_fold: the state at the start of a segment (thr = its first position - W) from the
    summaries [(key[], ent[]), ...] of every earlier segment, in stream order."""
    keep = [(np.ascontiguousarray(k, np.uint32), np.ascontiguousarray(e, np.uint32)) for k, e in parts]
    G = len(keep)
    pn = np.array([k.size for k, _ in keep], np.uint32)
    kt = (_u32p * max(G, 1))(*[k.ctypes.data_as(_u32p) for k, _ in keep])
    et = (_u32p * max(G, 1))(*[e.ctypes.data_as(_u32p) for _, e in keep])
    n, kp, ep = C.c_uint32(), _u32p(), _u32p()
    rc = lib().or_cfk_fold(G, pn.ctypes.data_as(_u32p), kt, et, max(0, thr), C.byref(n), C.byref(kp), C.byref(ep))
    if rc != 0:
        raise OracleError(rc)
    return _take_entries(n, kp, ep)


KEY_END = 0xFFFFFFFF     # an open upper store bound (include/accord_deps.h ACCORD_KEY_END)


def store_bounds(keyspace: int, stores: int):
    """EvenSplit boundaries of `stores` CommandStores over ordinals [0, keyspace)
    (local/ShardDistributor.java:46-157): store b owns [bounds[b], bounds[b+1]); the outer stores
    are open (the node owns the whole key domain)."""
    b = [j * keyspace // stores for j in range(stores)] + [KEY_END]
    b[0] = 0
    return b


def deps_stores(s: Stream, window: int, bounds, literal: bool = False, batch_end=None) -> PartialDeps:
    """Node-level deps over the CommandStores with the given bounds (oracle.h or_stream_deps_stores):
    every store slices the range commands and queries to its own range, the parts are unioned."""
    o, keep = _or_stream(s, window, batch_end)
    b = np.ascontiguousarray(bounds, np.uint32)
    d = _OrDeps()
    rc = lib().or_stream_deps_stores(C.byref(o), len(b) - 1, b.ctypes.data_as(_u32p), int(literal), C.byref(d))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(d)
    finally:
        lib().or_deps_free(C.byref(d))


def redundant_collect(s: Stream, start, end, start_epoch, end_epoch, bound, min_epoch: int) -> PartialDeps:
    """RedundantBefore.collectDeps of every txn (the redundant PartialDeps of
    PreAccept.calculatePartialDeps, messages/PreAccept.java:260-262); bound 0xFFFFFFFF = NONE."""
    o, keep = _or_stream(s, 0)
    a = [np.ascontiguousarray(start, np.uint32), np.ascontiguousarray(end, np.uint32),
         np.ascontiguousarray(start_epoch, np.uint64), np.ascontiguousarray(end_epoch, np.uint64),
         np.ascontiguousarray(bound, np.uint32)]
    d = _OrDeps()
    rc = lib().or_redundant_collect(C.byref(o), len(a[0]), a[0].ctypes.data_as(_u32p), a[1].ctypes.data_as(_u32p),
                                    a[2].ctypes.data_as(_u64p), a[3].ctypes.data_as(_u64p), a[4].ctypes.data_as(_u32p),
                                    min_epoch, C.byref(d))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(d)
    finally:
        lib().or_deps_free(C.byref(d))


def ts_compare(a, b) -> int:
    return lib().or_ts_compare(a[0], a[1], a[2], b[0], b[1], b[2])


def ts_equals(a, b) -> bool:
    return bool(lib().or_ts_equals(a[0], a[1], a[2], b[0], b[1], b[2]))


def keydeps_build(keys, vals, tbl_msb, tbl_lsb, tbl_node):
    """KeyDeps.Builder over (key, value-index) adds; returns (keys, vals, k2v) or None on throw."""
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    vals = np.ascontiguousarray(vals, dtype=np.uint32)
    tm = np.ascontiguousarray(tbl_msb, dtype=np.uint64)
    tl = np.ascontiguousarray(tbl_lsb, dtype=np.uint64)
    tn = np.ascontiguousarray(tbl_node, dtype=np.int32)
    d = _OrDeps()
    rc = lib().or_keydeps_build(len(keys), keys.ctypes.data_as(_u32p), vals.ctypes.data_as(_u32p), len(tm),
                                tm.ctypes.data_as(_u64p), tl.ctypes.data_as(_u64p), tn.ctypes.data_as(_i32p),
                                C.byref(d))
    if rc != 0:
        return None
    try:
        return _to_partial(d).key_deps(0)
    finally:
        lib().or_deps_free(C.byref(d))


def _single(keys, vals, k2v) -> PartialDeps:
    z = np.zeros(2, dtype=np.uint32)
    return PartialDeps(np.array([0, len(keys)], np.uint32), np.asarray(keys, np.uint32),
                       np.array([0, len(vals)], np.uint32), np.asarray(vals, np.uint32),
                       np.array([0, len(k2v)], np.uint32), np.asarray(k2v, np.int32),
                       z.copy(), np.zeros(0, np.uint32), np.zeros(0, np.uint32), z.copy(), np.zeros(0, np.uint32),
                       z.copy(), np.zeros(0, np.int32))


def _c_deps(p: PartialDeps):
    keep = [np.ascontiguousarray(getattr(p, f)) for f in PartialDeps.FIELDS]
    d = _OrDeps()
    d.n = p.n
    for f, a in zip(PartialDeps.FIELDS, keep):
        setattr(d, f, a.ctypes.data_as(_i32p if a.dtype == np.int32 else _u32p))
    return d, keep


def keydeps_union(a, b, tbl_msb, tbl_lsb, tbl_node):
    """RelationMultiMap.linearUnion of two (keys, vals, k2v) KeyDeps."""
    x, kx = _c_deps(_single(*a))
    y, ky = _c_deps(_single(*b))
    tm = np.ascontiguousarray(tbl_msb, dtype=np.uint64)
    tl = np.ascontiguousarray(tbl_lsb, dtype=np.uint64)
    tn = np.ascontiguousarray(tbl_node, dtype=np.int32)
    d = _OrDeps()
    rc = lib().or_keydeps_union(C.byref(x), 0, C.byref(y), 0, tm.ctypes.data_as(_u64p), tl.ctypes.data_as(_u64p),
                                tn.ctypes.data_as(_i32p), C.byref(d))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(d).key_deps(0)
    finally:
        lib().or_deps_free(C.byref(d))


def stab_key(starts, ends, key):
    rs = np.ascontiguousarray(starts, dtype=np.uint32)
    re = np.ascontiguousarray(ends, dtype=np.uint32)
    out = np.zeros(max(1, len(rs)), dtype=np.uint32)
    c = lib().or_stab_key(len(rs), rs.ctypes.data_as(_u32p), re.ctypes.data_as(_u32p), key, out.ctypes.data_as(_u32p))
    return out[:c].copy()


def reduced_dag(s: Stream):
    """The reduced WaitingOn DAG of a key-only Read/Write stream: on each key a txn
    keeps the last Write before it and, when it is a Write, the Reads since that Write -- every other
    dep on the key is implied through them (a Write depends on everything before it in its slice).
    Independent of the window: the slice [lcw, i) always holds the key's last Write before i.
    Returns the predecessor CSR (pred_off [n+1], preds) in txn order."""
    n = s.n
    kind = ((s.lsb >> np.uint64(1)) & np.uint64(7)).astype(np.int64)
    if np.any((s.lsb & np.uint64(1)) != 0) or np.any(kind > 1):
        raise ValueError("reduced_dag: key Read/Write streams only")
    ko = s.key_off.astype(np.int64)
    txn = np.repeat(np.arange(n, dtype=np.int64), np.diff(ko))
    keys = s.key_ord.astype(np.int64)
    w = kind[txn] == 1
    order = np.lexsort((txn, keys))                      # key-major, TxnId order within a key
    k_s, t_s, w_s = keys[order], txn[order], w[order]
    idx = np.arange(order.size)
    first = np.r_[True, k_s[1:] != k_s[:-1]]
    seg = np.cumsum(first) - 1
    seg_lo = np.flatnonzero(first)[seg]
    seg_hi = np.r_[np.flatnonzero(first)[1:], order.size][seg]
    last_w = np.maximum.accumulate(np.where(w_s, idx, -1))
    prev_w = np.r_[-1, last_w[:-1]]
    prev_w = np.where(prev_w >= seg_lo, prev_w, -1)
    m = prev_w >= 0                                      # last Write before the entry
    src = [t_s[prev_w[m]]]
    dst = [t_s[m]]
    next_w = np.minimum.accumulate(np.where(w_s, idx, order.size)[::-1])[::-1]
    nxt = np.r_[next_w[1:], order.size]                  # first Write after the entry
    r = (~w_s) & (nxt < seg_hi)                          # a Read -> the next Write on its key
    src.append(t_s[r])
    dst.append(t_s[nxt[r]])
    src = np.concatenate(src)
    dst = np.concatenate(dst)
    o = np.lexsort((src, dst))
    src, dst = src[o], dst[o]
    off = np.zeros(n + 1, np.int64)
    np.add.at(off, dst + 1, 1)
    return np.cumsum(off).astype(np.uint32), src.astype(np.uint32)


def levels_csr(pred_off: np.ndarray, preds: np.ndarray) -> np.ndarray:
    """or_levels_csr: level[i] = 0 without preds, else 1 + max level(p) (one core, txn order)."""
    n = int(pred_off.size) - 1
    pred_off = np.ascontiguousarray(pred_off, np.uint32)
    preds = np.ascontiguousarray(preds, np.uint32)
    level = np.zeros(max(1, n), np.uint32)
    rc = lib().or_levels_csr(n, pred_off.ctypes.data_as(_u32p), preds.ctypes.data_as(_u32p),
                             level.ctypes.data_as(_u32p))
    if rc != 0:
        raise OracleError(rc)
    return level[:n]


def waiting_on(p: PartialDeps):
    d, keep = _c_deps(p)
    n = p.n
    level = np.zeros(max(1, n), dtype=np.uint32)
    wo_off = np.zeros(n + 1, dtype=np.uint32)
    words = _u64p()
    rc = lib().or_waiting_on(C.byref(d), n, level.ctypes.data_as(_u32p), wo_off.ctypes.data_as(_u32p),
                             C.byref(words))
    if rc != 0:
        raise OracleError(rc)
    w = _arr(words, int(wo_off[-1]), np.uint64)
    C.CDLL(None).free(words)
    return level[:n].copy(), wo_off, w


def initialise_waiting_on(p: PartialDeps, s: Stream, g0: int, status, execs):
    """Commands.initialiseWaitingOn + the initial updateWaitingOn (or_initialise_waiting_on) of
    batch s (txn t at global position g0 + t, deps p with global positions) against status[g] /
    execs[g] (None or (msb, lsb, node)) of every position.  Returns (wo_off, words, aoi)."""
    n = s.n
    G = len(status)
    st = np.ascontiguousarray(status, dtype=np.uint8)
    em = np.zeros(max(1, G), np.uint64); el = np.zeros(max(1, G), np.uint64); en = np.zeros(max(1, G), np.int32)
    for g, x in enumerate(execs):
        if x is not None:
            em[g], el[g], en[g] = x
    om = s.msb.astype(np.uint64).copy(); ol = s.lsb.astype(np.uint64).copy(); on = s.node.astype(np.int32).copy()
    for t in range(n):
        g = g0 + t
        if 3 <= int(st[g]) <= 6 and execs[g] is not None:      # ACCEPTED..APPLIED carry an executeAt
            om[t], ol[t], on[t] = execs[g]
    d, keep = _c_deps(p)
    wo_off = np.zeros(n + 1, dtype=np.uint32)
    words, aoi = _u64p(), _u64p()
    lsb = np.ascontiguousarray(s.lsb, dtype=np.uint64)
    rc = lib().or_initialise_waiting_on(C.byref(d), n, lsb.ctypes.data_as(_u64p), om.ctypes.data_as(_u64p),
                                        ol.ctypes.data_as(_u64p), on.ctypes.data_as(_i32p), st.ctypes.data_as(_u8p),
                                        em.ctypes.data_as(_u64p), el.ctypes.data_as(_u64p), en.ctypes.data_as(_i32p),
                                        wo_off.ctypes.data_as(_u32p), C.byref(words), C.byref(aoi))
    if rc != 0:
        raise OracleError(rc)
    w = _arr(words, int(wo_off[-1]), np.uint64)
    a = _arr(aoi, int(wo_off[-1]), np.uint64)
    C.CDLL(None).free(words)
    C.CDLL(None).free(aoi)
    return wo_off, w, a


def waiting_on_events(p: PartialDeps):
    """Event-driven readiness rounds (independent restatement; must equal waiting_on's levels)."""
    d, keep = _c_deps(p)
    n = p.n
    rounds = np.zeros(max(1, n), dtype=np.uint32)
    rc = lib().or_waiting_on_events(C.byref(d), n, rounds.ctypes.data_as(_u32p))
    if rc != 0:
        raise OracleError(rc)
    return rounds[:n].copy()


def levels_cfk(s: Stream, p: PartialDeps):
    """Readiness rounds restated from the CommandsForKey side (notify + missing[] counts,
    registerUnmanaged / notifyUnmanaged, range-dep bits): or_levels_cfk."""
    o, keep = _or_stream(s, 0)
    d, keep2 = _c_deps(p)
    rounds = np.zeros(max(1, s.n), dtype=np.uint32)
    rc = lib().or_levels_cfk(C.byref(o), C.byref(d), rounds.ctypes.data_as(_u32p))
    if rc != 0:
        raise OracleError(rc)
    return rounds[:s.n].copy()


def deps_union(parts):
    """Deps.merge (left fold of RelationMultiMap.linearUnion) of G PartialDeps of the same txns."""
    cs = [_c_deps(p) for p in parts]
    arr = (_OrDeps * len(parts))(*[c[0] for c in cs])
    d = _OrDeps()
    rc = lib().or_deps_union(len(parts), arr, C.byref(d))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(d)
    finally:
        lib().or_deps_free(C.byref(d))


def deps_slice(p: PartialDeps, sel_start, sel_end, sel_off=None):
    """KeyDeps.slice + RangeDeps.slice of every txn to select ranges (per-txn CSR or shared)."""
    d, keep = _c_deps(p)
    ss = np.ascontiguousarray(sel_start, dtype=np.uint32)
    se = np.ascontiguousarray(sel_end, dtype=np.uint32)
    so = None if sel_off is None else np.ascontiguousarray(sel_off, dtype=np.uint32)
    o = _OrDeps()
    rc = lib().or_deps_slice(C.byref(d), None if so is None else so.ctypes.data_as(_u32p), ss.ctypes.data_as(_u32p),
                             se.ctypes.data_as(_u32p), len(ss), C.byref(o))
    if rc != 0:
        raise OracleError(rc)
    try:
        return _to_partial(o)
    finally:
        lib().or_deps_free(C.byref(o))


def deps_invert(p: PartialDeps, range_side: bool = False):
    """RelationMultiMap.invert of every txn: (off[n+1], ints) of txnIdsToKeys / txnIdsToRanges."""
    d, keep = _c_deps(p)
    off = np.zeros(p.n + 1, dtype=np.uint32)
    out = _i32p()
    rc = lib().or_deps_invert(C.byref(d), 1 if range_side else 0, off.ctypes.data_as(_u32p), C.byref(out))
    if rc != 0:
        raise OracleError(rc)
    a = _arr(out, int(off[-1]), np.int32)
    C.CDLL(None).free(out)
    return off, a


def max_conflicts(s, key_lo: int, nkeys: int, state=None, first: int = 0, exec_at=None, out=None,
                  intervals=None):
    """or_max_conflicts: per-txn (msb, lsb, node, present, fast), the updated per-key map and the
    number of txns merged (`folded`: the fold stops at a slow-path txn whose executeAt is unknown).
    `state` = (msb, lsb, node, present) arrays of nkeys entries (None = MaxConflicts.EMPTY);
    first/exec_at continue a stopped fold with the caller's executeAt for txn `first`.
    intervals: use or_max_conflicts_rm (the map as disjoint intervals; key and range txns);
    None = only when the stream has range txns."""
    n = len(s.msb)
    if state is None:
        state = (np.zeros(nkeys, np.uint64), np.zeros(nkeys, np.uint64), np.zeros(nkeys, np.int32),
                 np.zeros(nkeys, np.uint8))
    st = tuple(np.array(a, copy=True) for a in state)
    msb = np.ascontiguousarray(s.msb, np.uint64); lsb = np.ascontiguousarray(s.lsb, np.uint64)
    node = np.ascontiguousarray(s.node, np.int32)
    ko = np.ascontiguousarray(s.key_off, np.uint32); kk = np.ascontiguousarray(s.key_ord, np.uint32)
    ex = getattr(s, "exec_msb", None)
    em = el = en = None
    if ex is not None:
        em = np.ascontiguousarray(s.exec_msb, np.uint64); el = np.ascontiguousarray(s.exec_lsb, np.uint64)
        en = np.ascontiguousarray(s.exec_node, np.int32)
    if out is None:
        out = (np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(n, np.int32), np.zeros(n, np.uint8),
               np.zeros(n, np.uint8))
    else:
        out = tuple(np.array(a, copy=True) for a in out[:5])
    folded = C.c_uint32(0)
    ov = exec_at if exec_at is not None else (0, 0, 0)
    p = lambda a, t: None if a is None else a.ctypes.data_as(t)
    if intervals is None:
        intervals = bool(np.any(lsb & np.uint64(1)))
    if intervals:
        L = lib()
        if not getattr(L, "_mcrm_typed", False):
            L.or_max_conflicts_rm.argtypes = ([C.c_uint32, _u64p, _u64p, _i32p, _u32p, _u32p, _u32p, _u32p, _u32p,
                                               _u64p, _u64p, _i32p, C.c_uint32, C.c_uint32, _u64p, _u64p, _i32p, _u8p]
                                              + [_u64p, _u64p, _i32p, _u8p, _u8p]
                                              + [C.c_uint32, C.c_int, C.c_uint64, C.c_uint64, C.c_int32, _u32p])
            L._mcrm_typed = True
        ro = np.ascontiguousarray(s.rng_off if s.rng_off is not None else np.zeros(n + 1), np.uint32)
        rs = np.ascontiguousarray(s.rng_start if s.rng_start is not None else np.zeros(1), np.uint32)
        re = np.ascontiguousarray(s.rng_end if s.rng_end is not None else np.zeros(1), np.uint32)
        rc = L.or_max_conflicts_rm(n, p(msb, _u64p), p(lsb, _u64p), p(node, _i32p), p(ko, _u32p), p(kk, _u32p),
                                   p(ro, _u32p), p(rs, _u32p), p(re, _u32p),
                                   p(em, _u64p), p(el, _u64p), p(en, _i32p), key_lo, nkeys,
                                   p(st[0], _u64p), p(st[1], _u64p), p(st[2], _i32p), p(st[3], _u8p),
                                   p(out[0], _u64p), p(out[1], _u64p), p(out[2], _i32p), p(out[3], _u8p),
                                   p(out[4], _u8p), first, 1 if exec_at is not None else 0, int(ov[0]), int(ov[1]),
                                   int(ov[2]), C.byref(folded))
        if rc != 0:
            raise OracleError(rc)
        return out, st, int(folded.value)
    rc = lib().or_max_conflicts(n, p(msb, _u64p), p(lsb, _u64p), p(node, _i32p), p(ko, _u32p), p(kk, _u32p),
                                p(em, _u64p), p(el, _u64p), p(en, _i32p), key_lo, nkeys,
                                p(st[0], _u64p), p(st[1], _u64p), p(st[2], _i32p), p(st[3], _u8p),
                                p(out[0], _u64p), p(out[1], _u64p), p(out[2], _i32p), p(out[3], _u8p),
                                p(out[4], _u8p), first, 1 if exec_at is not None else 0, int(ov[0]), int(ov[1]),
                                int(ov[2]), C.byref(folded))
    if rc != 0:
        raise OracleError(rc)
    return out, st, int(folded.value)


class LStore:
    """Stateful literal CommandStore (or_lstore_*): batches fed in order, InternalStatus events in
    between; deps values are global positions.  Range txns join rangeCommands; status 8 (ERASED) is
    SaveStatus Erased / Invalidated: off the range scan, INVALID_OR_TRUNCATED for CommandsForKey."""
    TK, HISTORICAL, PREACCEPTED, ACCEPTED, COMMITTED, STABLE, APPLIED, INVALID, ERASED = range(9)

    def __init__(self, nkeys: int, event_mode: bool = False):
        L = lib()
        if not getattr(L, "_lstore_typed", False):
            L.or_lstore_create.argtypes = [C.c_uint32]
            L.or_lstore_create.restype = C.c_void_p
            L.or_lstore_free.argtypes = [C.c_void_p]
            L.or_lstore_free.restype = None
            L.or_lstore_batch.argtypes = [C.c_void_p, C.POINTER(_OrStream), C.POINTER(_OrDeps)]
            L.or_lstore_register.argtypes = [C.c_void_p, C.c_uint32, _u64p, _u64p, _i32p, _u8p, _u64p, _u64p, _i32p]
            L.or_lstore_size.argtypes = [C.c_void_p]
            L.or_lstore_size.restype = C.c_uint32
            L.or_lstore_truncate.argtypes = [C.c_void_p, C.c_uint32, _u32p, _u32p, _u32p]
            L.or_lstore_waiting_add.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_OrDeps), C.c_uint32]
            L.or_lstore_ready.argtypes = [C.c_void_p, _u32p, _u32p]
            L.or_lstore_ready_ex.argtypes = [C.c_void_p, _u32p, _u32p, _u64p, _u64p, _i32p]
            L.or_lstore_redundant.argtypes = [C.c_void_p, C.c_uint32, _u32p, _u32p, _u64p, _u64p, _u32p, _u32p, _u8p]
            L.or_lstore_event_mode.argtypes = [C.c_void_p, C.c_int]
            L.or_lstore_event_mode.restype = None
            L.or_lstore_waiting.argtypes = [C.c_void_p]
            L.or_lstore_waiting.restype = C.c_uint32
            L._lstore_typed = True
        self._h = L.or_lstore_create(nkeys)
        if event_mode:      # key bits cleared only on notifyAndUpdatePending's events (oracle.h)
            L.or_lstore_event_mode(self._h, 1)

    def close(self):
        if self._h:
            lib().or_lstore_free(self._h)
            self._h = None

    __del__ = close

    @property
    def size(self) -> int:
        return lib().or_lstore_size(self._h)

    def batch(self, s: Stream) -> PartialDeps:
        o, keep = _or_stream(s, 0)
        d = _OrDeps()
        rc = lib().or_lstore_batch(self._h, C.byref(o), C.byref(d))
        if rc != 0:
            raise OracleError(rc)
        try:
            return _to_partial(d)
        finally:
            lib().or_deps_free(C.byref(d))

    def waiting_add(self, base: int, p: PartialDeps):
        """The txns at positions base.. (deps p, positions as values) join the waiting set with every
        WaitingOn bit set (or_lstore_waiting_add)."""
        d, keep = _c_deps(p)
        rc = lib().or_lstore_waiting_add(self._h, base, C.byref(d), p.n)
        if rc != 0:
            raise OracleError(rc)

    def ready(self):
        """Execution readiness (or_lstore_ready): the waiting txns that became ReadyToExecute,
        ascending positions; they leave the set."""
        return self.ready_ex()[0]

    def ready_ex(self):
        """ready(), plus each ready txn's Command.executesAtLeast as (msb, lsb, node) arrays."""
        w = lib().or_lstore_waiting(self._h)
        out = np.zeros(max(1, w), np.uint32)
        em = np.zeros(max(1, w), np.uint64); el = np.zeros(max(1, w), np.uint64); en = np.zeros(max(1, w), np.int32)
        cnt = np.zeros(1, np.uint32)
        rc = lib().or_lstore_ready_ex(self._h, out.ctypes.data_as(_u32p), cnt.ctypes.data_as(_u32p),
                                      em.ctypes.data_as(_u64p), el.ctypes.data_as(_u64p), en.ctypes.data_as(_i32p))
        if rc != 0:
            raise OracleError(rc)
        c = int(cnt[0])
        return out[:c].copy(), (em[:c].copy(), el[:c].copy(), en[:c].copy())

    def redundant(self, start, end, start_epoch, end_epoch, locally_applied, bootstrapped_at, stale):
        """The RedundantBefore map readiness reads (or_lstore_redundant): removeRedundantDependencies."""
        a = [np.ascontiguousarray(start, np.uint32), np.ascontiguousarray(end, np.uint32),
             np.ascontiguousarray(start_epoch, np.uint64), np.ascontiguousarray(end_epoch, np.uint64),
             np.ascontiguousarray(locally_applied, np.uint32), np.ascontiguousarray(bootstrapped_at, np.uint32),
             np.ascontiguousarray(stale, np.uint8)]
        rc = lib().or_lstore_redundant(self._h, len(a[0]), a[0].ctypes.data_as(_u32p), a[1].ctypes.data_as(_u32p),
                                       a[2].ctypes.data_as(_u64p), a[3].ctypes.data_as(_u64p), a[4].ctypes.data_as(_u32p),
                                       a[5].ctypes.data_as(_u32p), a[6].ctypes.data_as(_u8p))
        if rc != 0:
            raise OracleError(rc)

    @property
    def waiting(self) -> int:
        return lib().or_lstore_waiting(self._h)

    def truncate(self, start, end, bound):
        """CommandsForKey.withRedundantBefore on every key of the map's entries (oracle.h)."""
        a = [np.ascontiguousarray(x, np.uint32) for x in (start, end, bound)]
        rc = lib().or_lstore_truncate(self._h, len(a[0]), *[x.ctypes.data_as(_u32p) for x in a])
        if rc != 0:
            raise OracleError(rc)

    def register(self, msb, lsb, node, status, exec_msb=None, exec_lsb=None, exec_node=None):
        a = [np.ascontiguousarray(msb, np.uint64), np.ascontiguousarray(lsb, np.uint64),
             np.ascontiguousarray(node, np.int32), np.ascontiguousarray(status, np.uint8)]
        e = None if exec_msb is None else [np.ascontiguousarray(exec_msb, np.uint64),
                                           np.ascontiguousarray(exec_lsb, np.uint64),
                                           np.ascontiguousarray(exec_node, np.int32)]
        rc = lib().or_lstore_register(self._h, len(a[0]), a[0].ctypes.data_as(_u64p), a[1].ctypes.data_as(_u64p),
                                      a[2].ctypes.data_as(_i32p), a[3].ctypes.data_as(_u8p),
                                      None if e is None else e[0].ctypes.data_as(_u64p),
                                      None if e is None else e[1].ctypes.data_as(_u64p),
                                      None if e is None else e[2].ctypes.data_as(_i32p))
        if rc != 0:
            raise OracleError(rc)
