"""Regenerates tests/golden/stream_small.npz: a small seeded mixed key+range stream and the
oracle's literal (reference-algorithm) PartialDeps for it.  The stream comes from the library's
SURVEY.md §8d generator; the expected outputs are additionally pinned by the hand-derived KATs in
kats.json and the restated reference property tests, which this vector only freezes for
regression."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "tests")]

from accord_amd import generate_stream  # noqa: E402
import oracle_lib as O  # noqa: E402

WINDOW = 32
s = generate_stream(600, 4, 120, 0.99, 0.5, range_frac=0.15, range_len_max=20, seed=2024)
d = O.deps_literal(s, WINDOW)
arrays = {f: getattr(s, f) for f in ("msb", "lsb", "node", "key_off", "key_ord", "rng_off", "rng_start", "rng_end")}
arrays["window"] = np.array(WINDOW)
for f in d.FIELDS:
    arrays["out_" + f] = getattr(d, f)
np.savez_compressed(os.path.join(HERE, "stream_small.npz"), **arrays)
print("wrote stream_small.npz", d.totals())
