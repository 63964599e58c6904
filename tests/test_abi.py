"""The C ABI library loads on CPU, exports every symbol include/accord_deps.h declares, and its
structs match the ctypes mirror byte for byte (no compute calls: no GPU here)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import accord_amd as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "accord_deps.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(accord_[a-z_]+)\s*\(", text)))


def test_library_loads_and_exports_all_declared():
    L = A.lib()
    decl = declared_symbols()
    assert decl, "no declarations parsed"
    for name in decl:
        assert hasattr(L, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", A.lib_path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (accord_\w+)", nm))
    assert set(decl) <= exported
    assert set(A.EXPORTED_SYMBOLS) == set(decl)


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", A.lib_path], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(A.lib_path, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts_match_header():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "accord_deps.h"
int main(void){
 printf("%zu %zu %zu %zu %zu\n", sizeof(accord_store_cfg), sizeof(accord_batch), sizeof(accord_deps),
        sizeof(accord_timing), sizeof(accord_workload_cfg));
 printf("%zu %zu %zu %zu %zu\n", offsetof(accord_deps, kd_key_off), offsetof(accord_deps, rd_r2v),
        offsetof(accord_workload_cfg, seed), offsetof(accord_timing, pairs), offsetof(accord_deps, kd_val_cnt));
 return 0;}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = [int(x) for x in lines[0].split()]
    offs = [int(x) for x in lines[1].split()]
    assert sizes == [C.sizeof(A._StoreCfg), C.sizeof(A._Batch), C.sizeof(A._Deps), C.sizeof(A._Timing),
                     C.sizeof(A._WorkloadCfg)]
    assert offs == [A._Deps.kd_key_off.offset, A._Deps.rd_r2v.offset, A._WorkloadCfg.seed.offset,
                    A._Timing.pairs.offset, A._Deps.kd_val_cnt.offset]


def test_store_create_without_gpu_fails_loudly():
    # this container has no GPU: the product must refuse, never fall back to the CPU
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    with pytest.raises(A.AccordError):
        A.CommandStore(device=0, key_lo=0, key_hi=10)


def test_generator_deterministic_and_shaped():
    a = A.generate_stream(5000, 8, 100_000, 0.99, 0.5, seed=2)
    b = A.generate_stream(5000, 8, 100_000, 0.99, 0.5, seed=2)
    c = A.generate_stream(5000, 8, 100_000, 0.99, 0.5, seed=3)
    for f in ("msb", "lsb", "node", "key_off", "key_ord"):
        assert np.array_equal(getattr(a, f), getattr(b, f))
    assert not np.array_equal(a.key_ord, c.key_ord)
    assert a.n == 5000 and a.pairs == 5000 * 8
    # TxnId packing: epoch 1, hlc 1_000_000 + i, node 1 + i % 7
    i = np.arange(5000, dtype=np.uint64)
    assert np.all(a.msb == np.uint64(1 << 15))
    assert np.all((a.lsb >> np.uint64(16)) == np.uint64(1_000_000) + i)
    assert np.all(a.node == (1 + np.arange(5000) % 7))
    # keys sorted unique per txn
    for t in range(0, 5000, 97):
        ks = a.key_ord[a.key_off[t]:a.key_off[t + 1]]
        assert np.all(np.diff(ks.astype(np.int64)) > 0)
    kinds = a.kinds()
    assert set(np.unique(kinds)) <= {0, 1}
    assert 0.45 < kinds.mean() < 0.55


def test_generator_zipf_statistics():
    s = A.generate_stream(200_000, 1, 100_000, 0.99, 0.5, seed=4)
    counts = np.bincount(s.key_ord, minlength=100_000)
    p1 = counts.max() / s.pairs
    # Zipf(0.99) over 100k keys: p1 ~= 0.078 (SURVEY.md §7 hard part 3)
    assert 0.07 < p1 < 0.087, p1


def test_generator_ranges_normalised():
    s = A.generate_stream(4000, 4, 10_000, 0.0, 0.5, range_frac=0.2, range_len_max=1000, seed=3)
    d = s.domains()
    assert 0.15 < d.mean() < 0.25
    for t in range(s.n):
        r0, r1 = s.rng_off[t], s.rng_off[t + 1]
        if d[t]:
            assert s.key_off[t + 1] == s.key_off[t] and r1 > r0
            st, en = s.rng_start[r0:r1].astype(np.int64), s.rng_end[r0:r1].astype(np.int64)
            assert np.all(st < en) and np.all(en[:-1] <= st[1:])
        else:
            assert r1 == r0


def test_txn_id_string_format():
    # TxnId.toString (primitives/TxnId.java:118-122)
    msb = (1 << 15)
    lsb = (1_000_000 << 16) | (1 << 1)
    assert A.txn_id_str(msb, lsb, 3) == "[1,1000000,2(KW),3]"
    assert A.txn_id_str(msb, (5 << 16) | 1, 1) == "[1,5,1(RR),1]"


def test_deps_visit_replays_mapreduceactive_order():
    """accord_deps_visit (host-only) over oracle deps: keys ascending then ranges ascending, txnIds
    ascending within each (local/SafeCommandStore.java:269-273); feeding the visits to
    KeyDeps/RangeDeps builders (the oracle's RelationMultiMap builder) rebuilds the same deps."""
    import oracle_lib as O
    s = A.generate_stream(3000, 4, 500, 0.99, 0.5, range_frac=0.2, range_len_max=40, seed=11)
    d = O.deps_fast(s, 64)
    for i in (0, 5, 777, 1500, 2999):
        seen = d.visit(i)
        keys = [(a, v) for r, a, b, v in seen if r == 0]
        rngs = [((a, b), v) for r, a, b, v in seen if r == 1]
        assert all(r == 0 for r, *_ in seen[:len(keys)])                  # keys first
        assert [k for k, _ in keys] == sorted(k for k, _ in keys)         # ascending keys
        assert [r for r, _ in rngs] == sorted(r for r, _ in rngs)         # ascending ranges
        rebuilt = O.keydeps_build([k for k, _ in keys], [v for _, v in keys], s.msb, s.lsb, s.node)
        kk, vv, xx = d.key_deps(i)
        if len(keys):
            assert np.array_equal(rebuilt[0], kk) and np.array_equal(rebuilt[1], vv) and np.array_equal(rebuilt[2], xx)
        else:
            assert len(kk) == 0
        rs, re_, rv, rx = d.range_deps(i)
        want = [((int(rs[r]), int(re_[r])), int(rv[rx[b]])) for r in range(len(rs))
                for b in range(len(rs) if r == 0 else rx[r - 1], rx[r])]
        assert rngs == want


def test_deps_visit_stops_on_nonzero():
    import oracle_lib as O
    s = A.generate_stream(500, 4, 50, 0.0, 0.5, seed=12)
    d = O.deps_fast(s, 64)
    i = int(np.argmax(np.diff(d.kd_val_off)))
    dd, keep = d.to_c()
    calls = []
    f = A.VISIT_FN(lambda ctx, r, a, b, v: (calls.append(v), 7)[1])
    assert A.lib().accord_deps_visit(C.byref(dd), i, f, None) == 7 and len(calls) == 1
