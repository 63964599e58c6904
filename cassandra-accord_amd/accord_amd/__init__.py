"""Host-side mirror of the Accord deps path over the C ABI of libaccord_deps.so.

This package mirrors the reference's operator surface for the dependency-calculation path
(accord-core, see include/accord_deps.h for file:line citations):

  * :class:`CommandStore` ~ ``accord.local.CommandStore`` / ``SafeCommandStore`` with the new
    batched entry ``calculate_deps_batch`` (PreAccept.calculatePartialDeps for a whole stream).
  * :class:`PartialDeps` ~ per-txn ``KeyDeps``/``RangeDeps`` in their exact serialised layout
    (``KeyDeps.SerializerSupport.create(keys, txnIds, keysToTxnIds)``).
  * :func:`txn_id_str`, :func:`keydeps_str` ~ ``TxnId.toString`` / ``KeyDeps.toString``.

Errors map to :class:`IllegalStateException` / :class:`IllegalArgumentException` like the
reference's ``Invariants`` (utils/Invariants.java:43-60).  There is no CPU fallback: compute
calls fail loudly when the HIP library or a device is missing.
"""
from __future__ import annotations

import ctypes as C
import os
import dataclasses
from dataclasses import dataclass
from typing import Optional

import numpy as np

__all__ = [
    "AccordError", "IllegalStateException", "IllegalArgumentException", "lib", "lib_path",
    "Stream", "generate_stream", "CommandStore", "PartialDeps", "Timing", "WaitingOn",
    "txn_id_str", "keydeps_str", "rangedeps_str", "EXPORTED_SYMBOLS", "segment_bounds", "segment_exchange",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG_ROOT = os.path.dirname(_HERE)
lib_path = os.environ.get("ACCORD_LIB") or os.path.join(_PKG_ROOT, "libaccord_deps.so")   # ACCORD_LIB: measurement builds

ACCORD_OK = 0
ERR = {
    -1: "ARG", -2: "UNSORTED", -3: "KIND", -4: "KEYS", -5: "DOMAIN", -6: "RANGES",
    -7: "CAPACITY", -8: "HIP", -9: "OOM", -10: "STATE",
}
STORE_PROFILE = 1
STORE_RESIDENT = 2
WINDOW_NONE = 0xFFFFFFFF     # no status-at-time model: statuses from CommandStore.register
KEY_END = 0xFFFFFFFF         # an open upper store bound (accord_store_cfg.store_bounds)
READY_POLL, READY_EVENTS = 0, 1   # accord_ready_set_mode
ST_ERASED = 8                # register(): SaveStatus Erased / Invalidated (range commands leave the range scan)
ST_TRUNCATED_APPLY = 9       # register(): SaveStatus TruncatedApply* (INVALID for CFK, executeAt known)

EXPORTED_SYMBOLS = [
    "accord_store_create", "accord_store_destroy", "accord_last_error", "accord_store_stream",
    "accord_deps_batch", "accord_deps_release", "accord_batch_upload", "accord_deps_compute",
    "accord_deps_device_view", "accord_deps_download", "accord_store_timing", "accord_store_set_profile",
    "accord_workload_generate", "accord_workload_free", "accord_deps_merge", "accord_comm_unique_id",
    "accord_comm_init", "accord_comm_size", "accord_deps_exchange_merge", "accord_deps_exchange_local", "accord_shard_timing",
    "accord_ready_update", "accord_ready_set_mode",
    "accord_waiting_on_compute", "accord_waiting_on_levelling", "accord_waiting_on_initialise", "accord_waiting_on_download", "accord_waiting_on_release",
    "accord_waiting_on_timing", "accord_deps_union", "accord_deps_slice", "accord_deps_invert",
    "accord_deps_inverse_release", "accord_ops_timing", "accord_deps_upload",
    "accord_max_conflicts_fold", "accord_max_conflicts_reset", "accord_max_conflicts_state",
    "accord_max_conflicts_fold_from", "accord_store_state", "accord_store_reset", "accord_txn_register",
    "accord_deps_visit", "accord_deps_range_stab", "accord_range_stab_release",
    "accord_redundant_before_set", "accord_redundant_before_set_ex", "accord_abi_version",
    "accord_segment_begin", "accord_segment_summary", "accord_segment_summary_copy", "accord_segment_carry",
    "accord_segment_timing",
]
ABI_VERSION = 6              # include/accord_deps.h ACCORD_ABI_VERSION this mirror follows
NO_TXN = 0xFFFFFFFF          # RedundantBefore bound Timestamp.NONE
VISIT_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32)


class AccordError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{ERR.get(code, code)}] {msg}")
        self.code = code


class IllegalStateException(AccordError):
    pass


class IllegalArgumentException(AccordError):
    pass


def _raise(code: int, msg: str):
    if code in (-1, -2, -3, -4, -5, -6):
        raise IllegalArgumentException(code, msg)
    raise IllegalStateException(code, msg)


# ---------------------------------------------------------------- ctypes structures
_u32p = C.POINTER(C.c_uint32)
_i32p = C.POINTER(C.c_int32)
_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)


class _MaxConflictsOut(C.Structure):
    _fields_ = [("msb", _u64p), ("lsb", _u64p), ("node", _i32p), ("present", _u8p), ("fast", _u8p),
                ("folded", C.c_uint32), ("reserved", C.c_uint32)]


class _StoreCfg(C.Structure):
    _fields_ = [("device", C.c_int32), ("key_lo", C.c_uint32), ("key_hi", C.c_uint32),
                ("window", C.c_uint32), ("flags", C.c_uint32), ("nstores", C.c_uint32),
                ("store_bounds", _u32p)]


class _Batch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("msb", _u64p), ("lsb", _u64p), ("node", _i32p),
                ("key_off", _u32p), ("key_ord", _u32p), ("rng_off", _u32p),
                ("rng_start", _u32p), ("rng_end", _u32p), ("txn_index", _u32p),
                ("exec_msb", _u64p), ("exec_lsb", _u64p), ("exec_node", _i32p)]


class _Deps(C.Structure):
    _fields_ = [("n", C.c_uint32), ("reserved", C.c_uint32),
                ("kd_keys_total", C.c_uint64), ("kd_vals_total", C.c_uint64), ("kd_k2v_total", C.c_uint64),
                ("rd_rngs_total", C.c_uint64), ("rd_vals_total", C.c_uint64), ("rd_r2v_total", C.c_uint64),
                ("kd_key_off", _u32p), ("kd_keys", _u32p), ("kd_val_off", _u32p), ("kd_vals", _u32p),
                ("kd_k2v_off", _u32p), ("kd_k2v", _i32p),
                ("rd_rng_off", _u32p), ("rd_rng_start", _u32p), ("rd_rng_end", _u32p),
                ("rd_val_off", _u32p), ("rd_vals", _u32p), ("rd_r2v_off", _u32p), ("rd_r2v", _i32p),
                ("kd_val_cnt", _u32p), ("owner", C.c_void_p)]


class _Ready(C.Structure):
    _fields_ = [("n", C.c_uint32), ("reserved", C.c_uint32), ("waiting", C.c_uint64), ("txn", C.POINTER(C.c_uint32)),
                ("eal_msb", _u64p), ("eal_lsb", _u64p), ("eal_node", _i32p)]


class _WaitingOn(C.Structure):
    _fields_ = [("n", C.c_uint32), ("max_level", C.c_uint32), ("words_total", C.c_uint64),
                ("preds_total", C.c_uint64), ("level", _u32p), ("wo_off", _u32p), ("words", _u64p),
                ("owner", C.c_void_p), ("applied_or_invalidated", _u64p)]


class _RangeStab(C.Structure):
    _fields_ = [("nq", C.c_uint32), ("reserved", C.c_uint32), ("total", C.c_uint64), ("off", _u32p),
                ("txn", _u32p), ("owner", C.c_void_p)]


class _Inverse(C.Structure):
    _fields_ = [("n", C.c_uint32), ("reserved", C.c_uint32), ("kd_total", C.c_uint64), ("rd_total", C.c_uint64),
                ("kd_t2k_off", _u32p), ("kd_t2k", _i32p), ("rd_t2r_off", _u32p), ("rd_t2r", _i32p),
                ("owner", C.c_void_p)]


class _StoreState(C.Structure):
    _fields_ = [("next_global", C.c_uint64), ("carry_entries", C.c_uint64), ("txns_registered", C.c_uint64),
                ("reserved", C.c_uint64)]


class _Timing(C.Structure):
    _fields_ = [("validate_ms", C.c_float), ("sort_ms", C.c_float), ("segment_ms", C.c_float),
                ("count_ms", C.c_float), ("scan_ms", C.c_float), ("fill_ms", C.c_float),
                ("range_ms", C.c_float), ("total_ms", C.c_float),
                ("compact_ms", C.c_float), ("reserved_ms", C.c_float),
                ("pairs", C.c_uint64), ("hist_entries", C.c_uint64),
                ("count_rk_cp_ms", C.c_float), ("count_rk_nkeys_ms", C.c_float), ("count_kd_sizes_ms", C.c_float),
                ("count_rk_ms", C.c_float), ("count_rd_ms", C.c_float), ("reserved2_ms", C.c_float),
                ("scan_spins", C.c_uint64), ("scan_fallbacks", C.c_uint64)]


class _CfkPart(C.Structure):
    """accord_cfk_part: a stream segment's CommandsForKey summary in device memory."""
    _fields_ = [("n", C.c_uint64), ("key", C.c_void_p), ("ent", C.c_void_p)]


class _WorkloadCfg(C.Structure):
    _fields_ = [("n", C.c_uint32), ("keys_per_txn", C.c_uint32), ("keyspace", C.c_uint32),
                ("ranges_max", C.c_uint32), ("zipf_s", C.c_double), ("write_frac", C.c_double),
                ("range_frac", C.c_double), ("range_len_max", C.c_uint32), ("node_mod", C.c_uint32),
                ("seed", C.c_uint64)]


_LIB: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load the in-tree HIP library; raise loudly if it is missing (no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(lib_path):
            raise ImportError(f"libaccord_deps.so not built at {lib_path}: run __graft_entry__.build()")
        L = C.CDLL(lib_path)
        L.accord_store_create.argtypes = [C.POINTER(_StoreCfg), C.POINTER(C.c_void_p)]
        L.accord_store_destroy.argtypes = [C.c_void_p]
        L.accord_last_error.argtypes = [C.c_void_p]
        L.accord_last_error.restype = C.c_char_p
        L.accord_store_stream.argtypes = [C.c_void_p]
        L.accord_store_stream.restype = C.c_void_p
        L.accord_deps_batch.argtypes = [C.c_void_p, C.POINTER(_Batch), C.POINTER(_Deps)]
        L.accord_deps_release.argtypes = [C.POINTER(_Deps)]
        L.accord_deps_release.restype = None
        L.accord_batch_upload.argtypes = [C.c_void_p, C.POINTER(_Batch)]
        L.accord_deps_compute.argtypes = [C.c_void_p]
        L.accord_deps_device_view.argtypes = [C.c_void_p, C.POINTER(_Deps)]
        L.accord_deps_download.argtypes = [C.c_void_p, C.POINTER(_Deps)]
        L.accord_store_timing.argtypes = [C.c_void_p, C.POINTER(_Timing)]
        L.accord_store_set_profile.argtypes = [C.c_void_p, C.c_uint32]
        L.accord_workload_generate.argtypes = [C.POINTER(_WorkloadCfg), C.POINTER(_Batch)]
        L.accord_workload_free.argtypes = [C.POINTER(_Batch)]
        L.accord_workload_free.restype = None
        L.accord_deps_merge.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_Deps), C.c_uint32]
        L.accord_comm_unique_id.argtypes = [C.c_void_p]
        L.accord_comm_init.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.accord_deps_exchange_merge.argtypes = [C.c_void_p, C.c_uint32]
        L.accord_deps_exchange_local.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.c_uint32]
        L.accord_shard_timing.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.accord_waiting_on_compute.argtypes = [C.c_void_p]
        L.accord_waiting_on_levelling.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.accord_waiting_on_initialise.argtypes = [C.c_void_p]
        L.accord_ready_update.argtypes = [C.c_void_p, C.POINTER(_Ready)]
        L.accord_ready_set_mode.argtypes = [C.c_void_p, C.c_uint32]
        L.accord_waiting_on_download.argtypes = [C.c_void_p, C.POINTER(_WaitingOn)]
        L.accord_waiting_on_release.argtypes = [C.POINTER(_WaitingOn)]
        L.accord_waiting_on_release.restype = None
        L.accord_waiting_on_timing.argtypes = [C.c_void_p] + [C.POINTER(C.c_float)] * 3
        L.accord_deps_union.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_Deps)]
        L.accord_deps_slice.argtypes = [C.c_void_p, C.POINTER(_Deps), _u32p, _u32p, _u32p, C.c_uint32]
        L.accord_deps_invert.argtypes = [C.c_void_p, C.POINTER(_Deps), C.POINTER(_Inverse)]
        L.accord_deps_inverse_release.argtypes = [C.POINTER(_Inverse)]
        L.accord_deps_inverse_release.restype = None
        L.accord_ops_timing.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
        L.accord_deps_upload.argtypes = [C.c_void_p, C.POINTER(_Deps)]
        L.accord_max_conflicts_fold.argtypes = [C.c_void_p, C.POINTER(_MaxConflictsOut)]
        L.accord_max_conflicts_fold_from.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_int32,
                                                     C.POINTER(_MaxConflictsOut)]
        L.accord_max_conflicts_reset.argtypes = [C.c_void_p]
        L.accord_redundant_before_set.argtypes = [C.c_void_p, C.c_uint32, _u32p, _u32p, _u64p, _u64p, _u32p,
                                                  C.c_uint64]
        L.accord_redundant_before_set_ex.argtypes = [C.c_void_p, C.c_uint32, _u32p, _u32p, _u64p, _u64p, _u32p,
                                                     _u32p, _u32p, _u8p, C.c_uint64]
        L.accord_store_state.argtypes = [C.c_void_p, C.POINTER(_StoreState)]
        L.accord_store_reset.argtypes = [C.c_void_p]
        L.accord_deps_visit.argtypes = [C.POINTER(_Deps), C.c_uint32, VISIT_FN, C.c_void_p]
        L.accord_txn_register.argtypes = [C.c_void_p, C.c_uint32, _u64p, _u64p, _i32p, _u8p, _u64p, _u64p, _i32p]
        L.accord_max_conflicts_state.argtypes = [C.c_void_p, _u64p, _u64p, _i32p, _u8p]
        L.accord_deps_range_stab.argtypes = [C.c_void_p, C.POINTER(_Deps), _u32p, _u32p, _u32p, C.POINTER(_RangeStab)]
        L.accord_range_stab_release.argtypes = [C.POINTER(_RangeStab)]
        L.accord_range_stab_release.restype = None
        L.accord_abi_version.argtypes = []
        L.accord_abi_version.restype = C.c_uint32
        L.accord_segment_begin.argtypes = [C.c_void_p, C.c_uint32]
        L.accord_segment_summary.argtypes = [C.c_void_p, C.POINTER(_CfkPart)]
        L.accord_segment_summary_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.accord_segment_carry.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_CfkPart)]
        L.accord_segment_timing.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        if L.accord_abi_version() != ABI_VERSION:
            raise ImportError(f"{lib_path}: ABI version {L.accord_abi_version()}, this mirror follows {ABI_VERSION}")
        for name in EXPORTED_SYMBOLS:
            f = getattr(L, name)
            if f.restype is C.c_int:  # default
                f.restype = C.c_int32
        _LIB = L
    return _LIB


# ---------------------------------------------------------------- streams
@dataclass
class Stream:
    """A batch of transactions in TxnId order (SoA), plus the model window."""
    msb: np.ndarray
    lsb: np.ndarray
    node: np.ndarray
    key_off: np.ndarray
    key_ord: np.ndarray
    rng_off: np.ndarray
    rng_start: np.ndarray
    rng_end: np.ndarray
    txn_index: Optional[np.ndarray] = None   # global stream positions (store subsets)
    # Accept batches (messages/Accept.java:113-117): startedBefore = executeAt per txn
    # (msb, lsb, node); None = PreAccept (startedBefore = txnId)
    exec_msb: Optional[np.ndarray] = None
    exec_lsb: Optional[np.ndarray] = None
    exec_node: Optional[np.ndarray] = None

    @property
    def n(self) -> int:
        return int(self.msb.shape[0])

    @property
    def pairs(self) -> int:
        return int(self.key_off[-1])

    def kinds(self) -> np.ndarray:
        return ((self.lsb >> np.uint64(1)) & np.uint64(7)).astype(np.uint8)

    def domains(self) -> np.ndarray:
        return (self.lsb & np.uint64(1)).astype(np.uint8)

    def slice(self, a: int, b: int) -> "Stream":
        """Txns [a, b) as a batch of their own (CSR rebased); txn_index / executeAt follow."""
        k0, k1 = int(self.key_off[a]), int(self.key_off[b])
        r0, r1 = int(self.rng_off[a]), int(self.rng_off[b])
        ex = {}
        if self.exec_msb is not None:
            ex = dict(exec_msb=self.exec_msb[a:b].copy(), exec_lsb=self.exec_lsb[a:b].copy(),
                      exec_node=self.exec_node[a:b].copy())
        ti = None if self.txn_index is None else self.txn_index[a:b].copy()
        return Stream(self.msb[a:b].copy(), self.lsb[a:b].copy(), self.node[a:b].copy(),
                      (self.key_off[a:b + 1] - self.key_off[a]).astype(np.uint32), self.key_ord[k0:k1].copy(),
                      (self.rng_off[a:b + 1] - self.rng_off[a]).astype(np.uint32), self.rng_start[r0:r1].copy(),
                      self.rng_end[r0:r1].copy(), txn_index=ti, **ex)

    def prefix(self, m: int) -> "Stream":
        m = min(m, self.n)
        k1 = int(self.key_off[m])
        r1 = int(self.rng_off[m])
        ex = {}
        if self.exec_msb is not None:
            ex = dict(exec_msb=self.exec_msb[:m].copy(), exec_lsb=self.exec_lsb[:m].copy(),
                      exec_node=self.exec_node[:m].copy())
        return Stream(self.msb[:m].copy(), self.lsb[:m].copy(), self.node[:m].copy(),
                      self.key_off[:m + 1].copy(), self.key_ord[:k1].copy(), self.rng_off[:m + 1].copy(),
                      self.rng_start[:r1].copy(), self.rng_end[:r1].copy(), **ex)

    def accept(self, frac: float = 1.0, max_delay: int = 64, node_mod: int = 7, seed: int = 1) -> "Stream":
        """The Accept batch of the same txns (messages/Accept.java:113-117): a `frac` of them get an
        executeAt later than their TxnId (hlc + U[0, max_delay], Timestamp flags 0, a seeded node;
        never before the TxnId), the rest executeAt = txnId (p1 = null, PreAccept-equivalent)."""
        rng = np.random.default_rng(seed)
        n = self.n
        em, el, en = self.msb.copy(), self.lsb.copy(), self.node.copy()
        pick = rng.random(n) < frac
        delay = rng.integers(0, max_delay + 1, n).astype(np.uint64)
        node = rng.integers(1, node_mod + 1, n).astype(np.int32)
        hlc = (self.lsb >> np.uint64(16)) + delay
        cand_lsb = hlc << np.uint64(16)
        # Timestamp.compareTo (primitives/Timestamp.java:208-217) with equal msb: hlc, the identity
        # flags (lsb & 0x1E; the candidate's are 0), then the signed node id
        flags = self.lsb & np.uint64(0x1E)
        later = (delay > 0) | ((flags == 0) & (node > self.node))
        use = pick & later
        el[use] = cand_lsb[use]
        en[use] = node[use]
        return dataclasses.replace(self, exec_msb=em, exec_lsb=el, exec_node=en)

    def restrict_keys(self, lo: int, hi: int, drop_empty: bool = False) -> "Stream":
        """Slice every txn's keys to the store block [lo, hi) (CommandStores.mapReduce fan-out,
        local/CommandStores.java:575-592).  drop_empty keeps only the txns intersecting the block
        and records their global positions in txn_index (key txns only)."""
        keep = (self.key_ord >= lo) & (self.key_ord < hi)
        csum = np.zeros(self.pairs + 1, np.int64)
        np.cumsum(keep, out=csum[1:])
        counts = (csum[self.key_off[1:].astype(np.int64)] - csum[self.key_off[:-1].astype(np.int64)]).astype(np.uint32)
        kord = self.key_ord[keep].copy()
        accept = self.exec_msb is not None
        if not drop_empty:
            ko = np.zeros(self.n + 1, np.uint32)
            np.cumsum(counts, out=ko[1:])
            return Stream(self.msb, self.lsb, self.node, ko, kord, self.rng_off, self.rng_start, self.rng_end,
                          exec_msb=self.exec_msb, exec_lsb=self.exec_lsb, exec_node=self.exec_node)
        if int(self.rng_off[-1]) != 0:
            raise IllegalArgumentException(-1, "drop_empty restriction supports key txns only")
        sel = np.nonzero(counts > 0)[0].astype(np.uint32)
        ko = np.zeros(sel.size + 1, np.uint32)
        np.cumsum(counts[sel], out=ko[1:])
        base = np.zeros(sel.size + 1, np.uint32)
        ex = dict(exec_msb=self.exec_msb[sel].copy(), exec_lsb=self.exec_lsb[sel].copy(),
                  exec_node=self.exec_node[sel].copy()) if accept else {}
        return Stream(self.msb[sel].copy(), self.lsb[sel].copy(), self.node[sel].copy(), ko, kord, base,
                      np.zeros(0, np.uint32), np.zeros(0, np.uint32), txn_index=sel, **ex)

    def c_batch(self) -> _Batch:
        self._keep = [np.ascontiguousarray(a) for a in (self.msb, self.lsb, self.node, self.key_off, self.key_ord,
                                                        self.rng_off, self.rng_start, self.rng_end)]
        if self.txn_index is not None:
            self._keep.append(np.ascontiguousarray(self.txn_index, dtype=np.uint32))
        msb, lsb, node, ko, kord, ro, rs, re = self._keep[:8]
        b = _Batch()
        b.n = self.n
        b.msb = msb.ctypes.data_as(_u64p)
        b.lsb = lsb.ctypes.data_as(_u64p)
        b.node = node.ctypes.data_as(_i32p)
        b.key_off = ko.ctypes.data_as(_u32p)
        b.key_ord = kord.ctypes.data_as(_u32p)
        has_ranges = ro.shape[0] > 0 and int(ro[-1]) > 0
        b.rng_off = ro.ctypes.data_as(_u32p) if has_ranges else None
        b.rng_start = rs.ctypes.data_as(_u32p) if has_ranges else None
        b.rng_end = re.ctypes.data_as(_u32p) if has_ranges else None
        b.txn_index = self._keep[8].ctypes.data_as(_u32p) if self.txn_index is not None else None
        if self.exec_msb is not None:
            ex = [np.ascontiguousarray(self.exec_msb, dtype=np.uint64), np.ascontiguousarray(self.exec_lsb, dtype=np.uint64),
                  np.ascontiguousarray(self.exec_node, dtype=np.int32)]
            self._keep += ex
            b.exec_msb = ex[0].ctypes.data_as(_u64p)
            b.exec_lsb = ex[1].ctypes.data_as(_u64p)
            b.exec_node = ex[2].ctypes.data_as(_i32p)
        return b



def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def _dense_vals(off: np.ndarray, cnt: np.ndarray, vals: np.ndarray):
    """Gapped txnIds (txn i: vals[off[i] .. off[i] + cnt[i])) -> dense CSR (offsets, values)."""
    n = cnt.size
    dense = np.zeros(n + 1, np.int64)
    np.cumsum(cnt, out=dense[1:])
    if np.any(off[:-1].astype(np.int64) + cnt > off[1:]):
        raise ValueError("gapped txnIds: a count runs past the next txn's offset")
    idx = np.repeat(off[:-1].astype(np.int64) - dense[:-1], cnt.astype(np.int64))
    idx += np.arange(int(dense[-1]), dtype=np.int64)
    return dense.astype(np.uint32), vals[idx]


def generate_stream(n: int, keys_per_txn: int = 4, keyspace: int = 100_000, zipf_s: float = 0.0,
                    write_frac: float = 0.5, range_frac: float = 0.0, ranges_max: int = 2,
                    range_len_max: int = 1000, node_mod: int = 7, seed: int = 1) -> Stream:
    """SURVEY.md §8d synthetic stream (generated by the library's host code)."""
    cfg = _WorkloadCfg(n, keys_per_txn, keyspace, ranges_max, zipf_s, write_frac, range_frac,
                       range_len_max, node_mod, seed)
    b = _Batch()
    rc = lib().accord_workload_generate(C.byref(cfg), C.byref(b))
    if rc != ACCORD_OK:
        _raise(rc, lib().accord_last_error(None).decode())
    try:
        P = b.key_off[n] if n else 0
        R = b.rng_off[n] if n else 0
        s = Stream(_arr(b.msb, n, np.uint64), _arr(b.lsb, n, np.uint64), _arr(b.node, n, np.int32),
                   _arr(b.key_off, n + 1, np.uint32), _arr(b.key_ord, P, np.uint32),
                   _arr(b.rng_off, n + 1, np.uint32), _arr(b.rng_start, R, np.uint32), _arr(b.rng_end, R, np.uint32))
    finally:
        lib().accord_workload_free(C.byref(b))
    return s


# ---------------------------------------------------------------- deps
@dataclass
class PartialDeps:
    """Per-txn KeyDeps/RangeDeps of a batch in the exact reference layout (CSR over txns)."""
    kd_key_off: np.ndarray
    kd_keys: np.ndarray
    kd_val_off: np.ndarray
    kd_vals: np.ndarray
    kd_k2v_off: np.ndarray
    kd_k2v: np.ndarray
    rd_rng_off: np.ndarray
    rd_rng_start: np.ndarray
    rd_rng_end: np.ndarray
    rd_val_off: np.ndarray
    rd_vals: np.ndarray
    rd_r2v_off: np.ndarray
    rd_r2v: np.ndarray

    FIELDS = ("kd_key_off", "kd_keys", "kd_val_off", "kd_vals", "kd_k2v_off", "kd_k2v",
              "rd_rng_off", "rd_rng_start", "rd_rng_end", "rd_val_off", "rd_vals", "rd_r2v_off", "rd_r2v")

    @property
    def n(self) -> int:
        return int(self.kd_key_off.shape[0]) - 1

    def key_deps(self, i: int):
        """(keys, txnIds as stream indices, keysToTxnIds) of txn i -- KeyDeps.SerializerSupport."""
        return (self.kd_keys[self.kd_key_off[i]:self.kd_key_off[i + 1]],
                self.kd_vals[self.kd_val_off[i]:self.kd_val_off[i + 1]],
                self.kd_k2v[self.kd_k2v_off[i]:self.kd_k2v_off[i + 1]])

    def range_deps(self, i: int):
        a, b = self.rd_rng_off[i], self.rd_rng_off[i + 1]
        return (self.rd_rng_start[a:b], self.rd_rng_end[a:b],
                self.rd_vals[self.rd_val_off[i]:self.rd_val_off[i + 1]],
                self.rd_r2v[self.rd_r2v_off[i]:self.rd_r2v_off[i + 1]])

    def txns(self, a: int, b: int) -> "PartialDeps":
        """The deps of txns [a, b) as a set of their own (offset arrays rebased)."""
        kw = {}
        for off, datas in (("kd_key_off", ("kd_keys",)), ("kd_val_off", ("kd_vals",)), ("kd_k2v_off", ("kd_k2v",)),
                           ("rd_rng_off", ("rd_rng_start", "rd_rng_end")), ("rd_val_off", ("rd_vals",)),
                           ("rd_r2v_off", ("rd_r2v",))):
            o = getattr(self, off)
            lo, hi = int(o[a]), int(o[b])
            kw[off] = (o[a:b + 1].astype(np.int64) - lo).astype(np.uint32)
            for dname in datas:
                kw[dname] = getattr(self, dname)[lo:hi].copy()
        return PartialDeps(**kw)

    def totals(self):
        return dict(keys=int(self.kd_key_off[-1]), vals=int(self.kd_val_off[-1]), k2v=int(self.kd_k2v_off[-1]),
                    body=int(self.kd_k2v_off[-1] - self.kd_key_off[-1]), rd_vals=int(self.rd_val_off[-1]))

    @staticmethod
    def from_c(d: _Deps) -> "PartialDeps":
        """From a host accord_deps (accord_deps_download / _batch).  A compute result's txnIds are
        gapped (kd_val_cnt, include/accord_deps.h): each txn's list is read by (start, count), as
        KeyDeps.SerializerSupport.create takes it per txn, and the set here is kept dense."""
        n = d.n
        kw = {}
        kw["kd_key_off"] = _arr(d.kd_key_off, n + 1, np.uint32)
        kw["kd_k2v_off"] = _arr(d.kd_k2v_off, n + 1, np.uint32)
        kw["kd_keys"] = _arr(d.kd_keys, int(kw["kd_key_off"][-1]), np.uint32)
        voff = _arr(d.kd_val_off, n + 1, np.uint32)
        vals = _arr(d.kd_vals, int(voff[-1]), np.uint32)
        if d.kd_val_cnt:
            voff, vals = _dense_vals(voff, _arr(d.kd_val_cnt, n, np.uint32), vals)
        kw["kd_val_off"], kw["kd_vals"] = voff, vals
        kw["kd_k2v"] = _arr(d.kd_k2v, int(kw["kd_k2v_off"][-1]), np.int32)
        kw["rd_rng_off"] = _arr(d.rd_rng_off, n + 1, np.uint32)
        kw["rd_val_off"] = _arr(d.rd_val_off, n + 1, np.uint32)
        kw["rd_r2v_off"] = _arr(d.rd_r2v_off, n + 1, np.uint32)
        R = int(kw["rd_rng_off"][-1])
        kw["rd_rng_start"] = _arr(d.rd_rng_start, R, np.uint32)
        kw["rd_rng_end"] = _arr(d.rd_rng_end, R, np.uint32)
        kw["rd_vals"] = _arr(d.rd_vals, int(kw["rd_val_off"][-1]), np.uint32)
        kw["rd_r2v"] = _arr(d.rd_r2v, int(kw["rd_r2v_off"][-1]), np.int32)
        return PartialDeps(**kw)

    @staticmethod
    def concat(parts) -> "PartialDeps":
        """The PartialDeps of consecutive batches as one (offset arrays rebased)."""
        kw = {}
        for f in PartialDeps.FIELDS:
            arrs = [getattr(p, f) for p in parts]
            if f.endswith("_off"):
                out, base = [np.zeros(1, np.uint32)], 0
                for a in arrs:
                    out.append((a[1:].astype(np.int64) + base).astype(np.uint32))
                    base += int(a[-1])
                kw[f] = np.concatenate(out)
            else:
                kw[f] = np.concatenate(arrs) if arrs else np.zeros(0, np.uint32)
        return PartialDeps(**kw)

    def to_c(self):
        """A host accord_deps view of this set (arrays kept alive by the returned tuple)."""
        keep = [np.ascontiguousarray(getattr(self, f)) for f in PartialDeps.FIELDS]
        d = _Deps()
        d.n = self.n
        for f, a in zip(PartialDeps.FIELDS, keep):
            setattr(d, f, a.ctypes.data_as(_i32p if a.dtype == np.int32 else _u32p))
        d.kd_keys_total = int(self.kd_key_off[-1]); d.kd_vals_total = int(self.kd_val_off[-1])
        d.kd_k2v_total = int(self.kd_k2v_off[-1]); d.rd_rngs_total = int(self.rd_rng_off[-1])
        d.rd_vals_total = int(self.rd_val_off[-1]); d.rd_r2v_total = int(self.rd_r2v_off[-1])
        return d, keep

    def visit(self, i: int):
        """SafeCommandStore.mapReduceActive replay of txn i through the C ABI (accord_deps_visit):
        [(is_range, key_or_start, range_end, txn_value)] in the visitor contract order."""
        d, keep = self.to_c()
        seen = []

        def cb(ctx, is_range, a, b, v):
            seen.append((is_range, a, b, v))
            return 0
        f = VISIT_FN(cb)
        rc = lib().accord_deps_visit(C.byref(d), i, f, None)
        if rc != ACCORD_OK:
            _raise(rc, lib().accord_last_error(None).decode())
        return seen

    def equals(self, other: "PartialDeps") -> bool:
        return all(np.array_equal(getattr(self, f), getattr(other, f)) for f in self.FIELDS)

    def first_difference(self, other: "PartialDeps"):
        for f in self.FIELDS:
            a, b = getattr(self, f), getattr(other, f)
            if a.shape != b.shape:
                return f, "shape", a.shape, b.shape
            bad = np.nonzero(a != b)[0]
            if bad.size:
                j = int(bad[0])
                return f, j, a[j], b[j]
        return None


@dataclass
class WaitingOn:
    """Per-txn WaitingOn bitsets (Command.WaitingOn, local/Command.java:1403-1437: range-dep txn
    bits, then key bits) and execution levels."""
    level: np.ndarray
    wo_off: np.ndarray
    words: np.ndarray
    max_level: int
    preds_total: int
    applied_or_invalidated: "np.ndarray | None" = None   # accord_waiting_on_initialise only

    def bits(self, i: int) -> np.ndarray:
        return self.words[self.wo_off[i]:self.wo_off[i + 1]]


@dataclass
class Timing:
    validate_ms: float
    sort_ms: float
    segment_ms: float
    count_ms: float
    scan_ms: float
    fill_ms: float
    range_ms: float
    total_ms: float
    pairs: int
    hist_entries: int
    compact_ms: float = 0.0
    count_detail: dict = dataclasses.field(default_factory=dict)   # count stage by kernel (ms)
    scan_spins: int = 0          # look-back spin iterations of the compute's scans
    scan_fallbacks: int = 0      # look-backs that summed their inputs instead of waiting


class CommandStore:
    """One CommandStore == one HIP stream on one device (impl/InMemoryCommandStore.java:89)."""

    def __init__(self, device: int = 0, key_lo: int = 0, key_hi: int = 100_000, window: int = 256,
                 profile: bool = False, resident: bool = False, store_bounds=None):
        """resident=True: the store keeps its CommandsForKey state across batches (every batch
        continues the store's stream; deps values are global stream positions).
        store_bounds: the CommandStores this handle hosts as S + 1 ascending key ordinals (store j
        owns [b[j], b[j+1]); b[0] == 0 open below, b[S] == KEY_END open above); every range is
        sliced Minimal to them (impl/InMemoryCommandStore.java:757-760).  None: one unbounded store."""
        flags = (STORE_PROFILE if profile else 0) | (STORE_RESIDENT if resident else 0)
        if store_bounds is None:
            cfg = _StoreCfg(device, key_lo, key_hi, window, flags, 0, None)
        else:
            b = np.ascontiguousarray(store_bounds, np.uint32)
            cfg = _StoreCfg(device, key_lo, key_hi, window, flags, len(b) - 1, b.ctypes.data_as(_u32p))
        h = C.c_void_p()
        rc = lib().accord_store_create(C.byref(cfg), C.byref(h))
        if rc != ACCORD_OK:
            _raise(rc, lib().accord_last_error(None).decode())
        self._h = h
        self.window = window
        self.key_lo, self.key_hi = key_lo, key_hi

    def state(self) -> dict:
        """Resident CFK state: next global position, carried history entries."""
        st = _StoreState()
        self._check(lib().accord_store_state(self._h, C.byref(st)))
        return {"next_global": st.next_global, "carry_entries": st.carry_entries,
                "txns_registered": st.txns_registered}

    def register(self, msb, lsb, node, status, exec_msb=None, exec_lsb=None, exec_node=None):
        """InternalStatus events (CommandsForKey.update) for txns this resident store holds, named by
        TxnId (strictly ascending); window must be WINDOW_NONE.  status: 0 TRANSITIVELY_KNOWN ..
        7 INVALID_OR_TRUNCATED, 8 ST_ERASED (SaveStatus Erased / Invalidated); executeAt for
        ACCEPTED..APPLIED."""
        a = [np.ascontiguousarray(msb, np.uint64), np.ascontiguousarray(lsb, np.uint64),
             np.ascontiguousarray(node, np.int32), np.ascontiguousarray(status, np.uint8)]
        e = None if exec_msb is None else [np.ascontiguousarray(exec_msb, np.uint64),
                                           np.ascontiguousarray(exec_lsb, np.uint64),
                                           np.ascontiguousarray(exec_node, np.int32)]
        self._check(lib().accord_txn_register(self._h, len(a[0]), a[0].ctypes.data_as(_u64p), a[1].ctypes.data_as(_u64p),
                                              a[2].ctypes.data_as(_i32p), a[3].ctypes.data_as(_u8p),
                                              None if e is None else e[0].ctypes.data_as(_u64p),
                                              None if e is None else e[1].ctypes.data_as(_u64p),
                                              None if e is None else e[2].ctypes.data_as(_i32p)))

    def reset(self):
        """Back to an empty CommandStore (resident state cleared)."""
        self._check(lib().accord_store_reset(self._h))

    def close(self):
        if getattr(self, "_h", None):
            lib().accord_store_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != ACCORD_OK:
            _raise(rc, lib().accord_last_error(self._h).decode())

    @property
    def stream_handle(self) -> int:
        return int(lib().accord_store_stream(self._h) or 0)

    def calculate_deps_batch(self, s: Stream) -> PartialDeps:
        """PreAccept.calculatePartialDeps for every txn of the batch, in TxnId order."""
        b = s.c_batch()
        d = _Deps()
        self._check(lib().accord_deps_batch(self._h, C.byref(b), C.byref(d)))
        try:
            return PartialDeps.from_c(d)
        finally:
            lib().accord_deps_release(C.byref(d))

    # device-resident pipeline
    def upload(self, s: Stream):
        b = s.c_batch()
        self._check(lib().accord_batch_upload(self._h, C.byref(b)))
        self._n_uploaded = len(s.msb)

    def compute(self):
        self._check(lib().accord_deps_compute(self._h))

    def download(self) -> PartialDeps:
        d = _Deps()
        self._check(lib().accord_deps_download(self._h, C.byref(d)))
        try:
            return PartialDeps.from_c(d)
        finally:
            lib().accord_deps_release(C.byref(d))

    # MaxConflicts (include/accord_deps.h; local/MaxConflicts.java, local/CommandStore.java:320-349)
    def max_conflicts_fold(self, s: "Stream | None" = None, download: bool = True, first: int = 0,
                           exec_at=None, out=None):
        """For every txn of the uploaded batch (or `s`, uploaded first): minNonConflicting =
        maxConflicts.get(keys) before the txn's own update, and the fast-path test.  Returns
        (msb, lsb, node, present, fast, folded): numpy arrays over the batch and the number of txns
        merged so far -- the fold stops at the first globally visible slow-path txn of a PreAccept
        batch (its executeAt is the caller's uniqueNow); continue with first=folded and exec_at =
        (msb, lsb, node) of that txn's executeAt, passing the previous result as `out`."""
        if s is not None:
            self.upload(s)
        if not download:
            self._check(lib().accord_max_conflicts_fold(self._h, None))
            return None
        n = self._n_uploaded if s is None else len(s.msb)
        if out is None:
            msb = np.zeros(n, np.uint64); lsb = np.zeros(n, np.uint64); node = np.zeros(n, np.int32)
            present = np.zeros(n, np.uint8); fast = np.zeros(n, np.uint8)
        else:
            msb, lsb, node, present, fast = out[:5]
        o = _MaxConflictsOut(msb.ctypes.data_as(_u64p), lsb.ctypes.data_as(_u64p), node.ctypes.data_as(_i32p),
                             present.ctypes.data_as(_u8p), fast.ctypes.data_as(_u8p), 0, 0)
        if exec_at is None:
            if first != 0:
                raise IllegalArgumentException(-1, "a continued fold needs the executeAt of txn `first`")
            self._check(lib().accord_max_conflicts_fold(self._h, C.byref(o)))
        else:
            em, el, en = exec_at
            self._check(lib().accord_max_conflicts_fold_from(self._h, first, int(em), int(el), int(en), C.byref(o)))
        return msb, lsb, node, present, fast, int(o.folded)

    def redundant_before(self, start=(), end=(), start_epoch=(), end_epoch=(), bound=(), min_epoch: int = 0,
                         locally_applied=None, bootstrapped_at=None, stale=None):
        """RedundantBefore of this store (local/RedundantBefore.java): its non-null entries (start, end]
        ascending and disjoint, with [start_epoch, end_epoch) and shardAppliedOrInvalidatedBefore as a
        stream position (NO_TXN = NONE); min_epoch = minUnsyncedEpoch.  Every later calculation returns
        builder.build().with(RedundantBefore.collectDeps(...)) (messages/PreAccept.java:260-263).  No
        entries = RedundantBefore.EMPTY.  locally_applied / bootstrapped_at (positions, NO_TXN = NONE)
        and stale (staleUntilAtLeast != null) complete each Entry: readiness then applies
        removeRedundantDependencies (accord_redundant_before_set_ex)."""
        a = [np.ascontiguousarray(start, np.uint32), np.ascontiguousarray(end, np.uint32),
             np.ascontiguousarray(start_epoch, np.uint64), np.ascontiguousarray(end_epoch, np.uint64),
             np.ascontiguousarray(bound, np.uint32)]
        ext = [None if x is None else np.ascontiguousarray(x, t)
               for x, t in ((locally_applied, np.uint32), (bootstrapped_at, np.uint32), (stale, np.uint8))]
        if len({len(x) for x in a + [e for e in ext if e is not None]}) != 1:
            raise IllegalArgumentException(-1, "RedundantBefore arrays differ in length")
        self._check(lib().accord_redundant_before_set_ex(
            self._h, len(a[0]), a[0].ctypes.data_as(_u32p), a[1].ctypes.data_as(_u32p), a[2].ctypes.data_as(_u64p),
            a[3].ctypes.data_as(_u64p), a[4].ctypes.data_as(_u32p),
            None if ext[0] is None else ext[0].ctypes.data_as(_u32p),
            None if ext[1] is None else ext[1].ctypes.data_as(_u32p),
            None if ext[2] is None else ext[2].ctypes.data_as(_u8p), int(min_epoch)))

    def max_conflicts_reset(self):
        self._check(lib().accord_max_conflicts_reset(self._h))

    def max_conflicts_state(self):
        nk = self.key_hi - self.key_lo
        msb = np.zeros(nk, np.uint64); lsb = np.zeros(nk, np.uint64); node = np.zeros(nk, np.int32)
        present = np.zeros(nk, np.uint8)
        self._check(lib().accord_max_conflicts_state(self._h, msb.ctypes.data_as(_u64p), lsb.ctypes.data_as(_u64p),
                                                     node.ctypes.data_as(_i32p), present.ctypes.data_as(_u8p)))
        return msb, lsb, node, present

    def device_view(self) -> dict:
        d = _Deps()
        self._check(lib().accord_deps_device_view(self._h, C.byref(d)))
        out = {"n": d.n, "kd_keys_total": d.kd_keys_total, "kd_vals_total": d.kd_vals_total,
               "kd_k2v_total": d.kd_k2v_total}
        for f in PartialDeps.FIELDS + ("kd_val_cnt",):
            out[f] = C.cast(getattr(d, f), C.c_void_p).value or 0
        return out

    def _device_view_c(self) -> _Deps:
        d = _Deps()
        self._check(lib().accord_deps_device_view(self._h, C.byref(d)))
        return d

    def merge(self, parts, txn_lo: int = 0):
        """Union of per-store partials (each a CommandStore on this GPU, key-disjoint, ordered by
        key block) -- PreAccept.reduce; the result becomes this store's deps."""
        arr = (_Deps * len(parts))(*[p._device_view_c() for p in parts])
        self._check(lib().accord_deps_merge(self._h, len(parts), arr, txn_lo))

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        rc = lib().accord_comm_unique_id(buf)
        if rc != ACCORD_OK:
            _raise(rc, lib().accord_last_error(None).decode())
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = C.create_string_buffer(uid, 128)
        self._check(lib().accord_comm_init(self._h, nranks, rank, buf))

    def comm_size(self):
        """(ranks, rank) of the store's RCCL communicator as RCCL reports them (ncclCommCount)."""
        a, b = C.c_int32(), C.c_int32()
        self._check(lib().accord_comm_size(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def exchange_merge(self, n_total: int):
        self._check(lib().accord_deps_exchange_merge(self._h, n_total))

    @staticmethod
    def exchange_local(stores, n_total: int):
        """accord_deps_exchange_merge for len(stores) simulated ranks on one device: stores[r] acts
        as rank r (each holding its key block's partial of the stream), the plan and the union are
        the RCCL path's, the transport is device copies.  Afterwards stores[r] holds the node-level
        deps of its own txns [r*n_total/G, (r+1)*n_total/G)."""
        arr = (C.c_void_p * len(stores))(*[st._h for st in stores])
        rc = lib().accord_deps_exchange_local(arr, len(stores), n_total)
        if rc != ACCORD_OK:
            msgs = [lib().accord_last_error(st._h).decode() for st in stores]
            _raise(rc, "; ".join(m for m in msgs if m) or lib().accord_last_error(None).decode())

    def shard_timing(self):
        a, b = C.c_float(), C.c_float()
        self._check(lib().accord_shard_timing(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    # deps-set operations (a9 general union, a10 slice / invert); sources are CommandStores on this
    # device whose current deps index the same TxnId table
    def union(self, parts):
        """Deps.merge of the current deps of `parts` (keys may overlap: KeyDeps.merge /
        RangeDeps.merge -> RelationMultiMap.linearUnion); the result becomes this store's deps."""
        arr = (_Deps * len(parts))(*[p._device_view_c() for p in parts])
        self._check(lib().accord_deps_union(self._h, len(parts), arr))

    def slice(self, src: "CommandStore", sel_start, sel_end, sel_off=None):
        """KeyDeps.slice + RangeDeps.slice of src's deps to (start, end] select ranges (shared, or
        per txn with sel_off[n+1]); the result becomes this store's deps."""
        v = src._device_view_c()
        ss = np.ascontiguousarray(sel_start, dtype=np.uint32)
        se = np.ascontiguousarray(sel_end, dtype=np.uint32)
        so = None if sel_off is None else np.ascontiguousarray(sel_off, dtype=np.uint32)
        self._check(lib().accord_deps_slice(self._h, C.byref(v), None if so is None else so.ctypes.data_as(_u32p),
                                            ss.ctypes.data_as(_u32p), se.ctypes.data_as(_u32p), len(ss)))

    def invert(self, src: "CommandStore"):
        """txnIdsToKeys / txnIdsToRanges of src's deps (RelationMultiMap.invert):
        (kd_off[n+1], kd_ints, rd_off[n+1], rd_ints)."""
        v = src._device_view_c()
        w = _Inverse()
        self._check(lib().accord_deps_invert(self._h, C.byref(v), C.byref(w)))
        try:
            return (_arr(w.kd_t2k_off, w.n + 1, np.uint32), _arr(w.kd_t2k, w.kd_total, np.int32),
                    _arr(w.rd_t2r_off, w.n + 1, np.uint32), _arr(w.rd_t2r, w.rd_total, np.int32))
        finally:
            lib().accord_deps_inverse_release(C.byref(w))

    def range_stab(self, src: "CommandStore", q_off, q_start, q_end):
        """SearchableRangeList stabbing of src's RangeDeps, built on the device: for each query
        (q_start, q_end] of txn i (queries [q_off[i], q_off[i+1])), the txnIds of txn i's RangeDeps
        ranges intersecting it, ascending (RangeDeps.forEach / computeTxnIds).  Returns
        (off[nq+1], txns)."""
        v = src._device_view_c()
        qo = np.ascontiguousarray(q_off, dtype=np.uint32)
        qs = np.ascontiguousarray(q_start, dtype=np.uint32)
        qe = np.ascontiguousarray(q_end, dtype=np.uint32)
        r = _RangeStab()
        self._check(lib().accord_deps_range_stab(self._h, C.byref(v), qo.ctypes.data_as(_u32p),
                                                 qs.ctypes.data_as(_u32p), qe.ctypes.data_as(_u32p), C.byref(r)))
        try:
            return _arr(r.off, r.nq + 1, np.uint32), _arr(r.txn, r.total, np.uint32)
        finally:
            lib().accord_range_stab_release(C.byref(r))

    def upload_deps(self, p: "PartialDeps"):
        """A host PartialDeps set becomes this store's current deps (e.g. replica replies)."""
        keep = [np.ascontiguousarray(getattr(p, f)) for f in PartialDeps.FIELDS]
        d = _Deps()
        d.n = p.n
        for f, a in zip(PartialDeps.FIELDS, keep):
            setattr(d, f, a.ctypes.data_as(_i32p if a.dtype == np.int32 else _u32p))
        d.kd_keys_total = int(p.kd_key_off[-1]); d.kd_vals_total = int(p.kd_val_off[-1])
        d.kd_k2v_total = int(p.kd_k2v_off[-1]); d.rd_rngs_total = int(p.rd_rng_off[-1])
        d.rd_vals_total = int(p.rd_val_off[-1]); d.rd_r2v_total = int(p.rd_r2v_off[-1])
        self._check(lib().accord_deps_upload(self._h, C.byref(d)))

    def ops_ms(self) -> float:
        f = C.c_float()
        self._check(lib().accord_ops_timing(self._h, C.byref(f)))
        return f.value

    # stream segments (config 4; include/accord_deps.h accord_segment_*)
    def segment_begin(self, seg_base: int):
        """This (resident) store owns stream positions seg_base.. of every CommandStore: reset, then
        upload the segment's txns."""
        self._check(lib().accord_segment_begin(self._h, int(seg_base)))

    def segment_summary(self):
        """The uploaded segment's CommandsForKey summary in device memory: (n, key_ptr, ent_ptr)."""
        p = _CfkPart()
        self._check(lib().accord_segment_summary(self._h, C.byref(p)))
        return int(p.n), int(p.key or 0), int(p.ent or 0)

    def segment_summary_copy(self, key_ptr: int, ent_ptr: int, cap: int):
        """Copy the summary into caller device buffers of cap entries each."""
        self._check(lib().accord_segment_summary_copy(self._h, C.c_void_p(key_ptr), C.c_void_p(ent_ptr), int(cap)))

    def segment_carry(self, parts):
        """The CommandsForKey state at the segment's start from the summaries [(n, key_ptr, ent_ptr)]
        of every earlier segment, in stream order (device pointers); compute() then gives the
        segment's node-level deps."""
        arr = (_CfkPart * max(1, len(parts)))(*[_CfkPart(int(n), C.c_void_p(k), C.c_void_p(e)) for n, k, e in parts])
        self._check(lib().accord_segment_carry(self._h, len(parts), arr))

    def segment_timing(self):
        a, b = C.c_float(), C.c_float()
        self._check(lib().accord_segment_timing(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def waiting_on_compute(self):
        """WaitingOn bitsets + execution levels of the computed deps (device-resident)."""
        self._check(lib().accord_waiting_on_compute(self._h))

    def waiting_on_download(self) -> "WaitingOn":
        w = _WaitingOn()
        self._check(lib().accord_waiting_on_download(self._h, C.byref(w)))
        try:
            return WaitingOn(level=_arr(w.level, w.n, np.uint32).copy(),
                             wo_off=_arr(w.wo_off, w.n + 1, np.uint32).copy(),
                             words=_arr(w.words, w.words_total, np.uint64).copy(),
                             max_level=int(w.max_level), preds_total=int(w.preds_total),
                             applied_or_invalidated=(_arr(w.applied_or_invalidated, w.words_total, np.uint64).copy()
                                                     if w.applied_or_invalidated else None))
        finally:
            lib().accord_waiting_on_release(C.byref(w))

    def waiting_on(self) -> "WaitingOn":
        self.waiting_on_compute()
        return self.waiting_on_download()

    def waiting_on_initialise(self) -> "WaitingOn":
        """Commands.initialiseWaitingOn + updateWaitingOn of the last batch against the registered
        statuses (registered-status stores; include/accord_deps.h accord_waiting_on_initialise)."""
        self._check(lib().accord_waiting_on_initialise(self._h))
        return self.waiting_on_download()

    def ready_mode(self, events: bool):
        """accord_ready_set_mode: ACCORD_READY_EVENTS (event-exact: key bits clear only when
        notifyAndUpdatePending's events reach the key, replayed at registration) or ACCORD_READY_POLL
        (the default: every call re-tests the waiting txns whose inputs changed).  Empty waiting set only."""
        self._check(lib().accord_ready_set_mode(self._h, READY_EVENTS if events else READY_POLL))

    def ready_update(self):
        """Execution readiness (include/accord_deps.h accord_ready_update): re-evaluates every txn of
        the waiting set (batches whose WaitingOn was initialised) against the registered statuses --
        Commands.updateWaitingOn for range deps, CommandsForKey.notify / notifyUnmanaged for keys --
        and returns the global positions (ascending) of the txns now ReadyToExecute, and how many
        txns still wait."""
        got, waiting, _ = self.ready_update_ex()
        return got, waiting

    def ready_update_ex(self):
        """ready_update, plus each ready txn's Command.executesAtLeast as (msb, lsb, node) arrays."""
        r = _Ready()
        self._check(lib().accord_ready_update(self._h, C.byref(r)))
        if not r.n:
            z = np.zeros(0, np.uint64)
            return np.zeros(0, np.uint32), int(r.waiting), (z, z.copy(), np.zeros(0, np.int32))
        got = np.ctypeslib.as_array(r.txn, shape=(r.n,)).copy()
        eal = (np.ctypeslib.as_array(r.eal_msb, shape=(r.n,)).copy(), np.ctypeslib.as_array(r.eal_lsb, shape=(r.n,)).copy(),
               np.ctypeslib.as_array(r.eal_node, shape=(r.n,)).copy())
        return got, int(r.waiting), eal

    def waiting_on_levelling(self):
        """(stripe length, fell back to the serial resolver) of the last waiting_on_compute
        (include/accord_deps.h accord_waiting_on_levelling)."""
        a, b = C.c_uint32(), C.c_uint32()
        self._check(lib().accord_waiting_on_levelling(self._h, C.byref(a), C.byref(b)))
        return int(a.value), bool(b.value)

    def waiting_on_timing(self):
        a, b, c = C.c_float(), C.c_float(), C.c_float()
        self._check(lib().accord_waiting_on_timing(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def set_profile(self, on: bool):
        """Profiling events on / off from the next call on (include/accord_deps.h accord_store_set_profile)."""
        self._check(lib().accord_store_set_profile(self._h, 1 if on else 0))

    def timing(self) -> Timing:
        t = _Timing()
        self._check(lib().accord_store_timing(self._h, C.byref(t)))
        return Timing(t.validate_ms, t.sort_ms, t.segment_ms, t.count_ms, t.scan_ms, t.fill_ms, t.range_ms,
                      t.total_ms, t.pairs, t.hist_entries, t.compact_ms,
                      {"rk_checkpoints": t.count_rk_cp_ms, "rk_nkeys": t.count_rk_nkeys_ms,
                       "kd_sizes": t.count_kd_sizes_ms, "rk_count": t.count_rk_ms, "rd_count": t.count_rd_ms},
                      int(t.scan_spins), int(t.scan_fallbacks))


# ---------------------------------------------------------------- string forms
_DOMAIN = "KR"
_KIND = "RWESXL"


def segment_bounds(n_total: int, world: int):
    """Segment r of a stream of n_total txns over `world` ranks: positions [a_r, b_r)."""
    return [(r * n_total // world, (r + 1) * n_total // world) for r in range(world)]


def segment_exchange(store, rank: int, world: int, device, group=None, store_device=None) -> dict:
    """The config-4 exchange step: every rank's CommandsForKey summary reaches every
    other rank with one all-gather over torch.distributed (nccl = RCCL over xGMI on the GPU box, gloo
    on the CPU), and each rank folds the summaries of the segments before its own into the carry
    (store.segment_carry).  `store` is a CommandStore after segment_begin + upload (or any object with
    its segment_summary / segment_summary_copy / segment_carry methods); `device` is where the
    exchange buffers live (the store's device, or the CPU for gloo); store_device, when it differs
    from `device`, is where the received summaries are staged for the store's carry (a GPU store
    exchanging over gloo).  Returns the byte counts."""
    import torch
    import torch.distributed as dist
    n = store.segment_summary()[0]
    mine_n = torch.tensor([n], dtype=torch.int64, device=device)
    counts = [torch.empty(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(counts, mine_n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(1, max(counts))
    mine = torch.empty((2, m), dtype=torch.int32, device=device)
    store.segment_summary_copy(mine[0].data_ptr(), mine[1].data_ptr(), m)
    gathered = [torch.empty((2, m), dtype=torch.int32, device=device) for _ in range(world)]
    dist.all_gather(gathered, mine, group=group)
    if store_device is not None and torch.device(store_device) != torch.device(device):
        gathered = [g.to(store_device) for g in gathered[:rank]]
    for d in (device, store_device):
        if d is not None and torch.device(d).type == "cuda":
            torch.cuda.synchronize(d)
    store.segment_carry([(counts[q], gathered[q][0].data_ptr(), gathered[q][1].data_ptr()) for q in range(rank)])
    return {"summary_entries": counts, "padded_entries": m, "bytes_sent": 8 * m * (world - 1),
            "bytes_used": 8 * sum(counts[:rank])}


def txn_id_str(msb: int, lsb: int, node: int) -> str:
    """TxnId.toString (primitives/TxnId.java:118-122): [epoch,hlc,flags(DK),node]."""
    msb, lsb = int(msb), int(lsb)
    epoch = msb >> 15
    hlc = ((msb & 0x7FFF) << 48) | (lsb >> 16)
    flags = lsb & 0xFFFF
    return f"[{epoch},{hlc},{flags}({_DOMAIN[flags & 1]}{_KIND[(flags >> 1) & 7]}),{int(node)}]"


def keydeps_str(keys, vals, k2v, s: Stream) -> str:
    """KeyDeps.toString -> RelationMultiMap.toSimpleString (utils/RelationMultiMap.java:963-987)."""
    keys = list(keys)
    if len(keys) == len(k2v):
        return "{}"
    out, t = [], len(keys)
    for k, key in enumerate(keys):
        ids = []
        while t < k2v[k]:
            j = int(vals[k2v[t]])
            ids.append(txn_id_str(s.msb[j], s.lsb[j], s.node[j]))
            t += 1
        out.append(f"{int(key)}:[{', '.join(ids)}]")
    return "{" + ", ".join(out) + "}"


def rangedeps_str(starts, ends, vals, r2v, s: Stream) -> str:
    """RangeDeps.toString with IntKey ranges printed as (s,e] (Range.java:433-440)."""
    if len(starts) == len(r2v):
        return "{}"
    out, t = [], len(starts)
    for k in range(len(starts)):
        ids = []
        while t < r2v[k]:
            j = int(vals[r2v[t]])
            ids.append(txn_id_str(s.msb[j], s.lsb[j], s.node[j]))
            t += 1
        out.append(f"({int(starts[k])},{int(ends[k])}]:[{', '.join(ids)}]")
    return "{" + ", ".join(out) + "}"
