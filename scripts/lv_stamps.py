"""Analyse ACCORD_LV_DEBUG stamps of the levelling resolve pass (dev aid)."""
import sys
import numpy as np
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 5).astype(np.int64)
a = a[a[:, 4] > 0]
pub = a[:, 4]
per = np.diff(pub)
handoff = a[1:, 3] - pub[:-1]          # x-1 published -> x sees it
late = a[:, 4] - a[:, 3]
early = a[:, 2] - a[:, 1]
slack = a[1:, 3] - a[1:, 2]             # early done -> late ready (negative: early was late)
print("chunks", len(a), "period median", np.median(per), "mean", per.mean())
print("handoff median", np.median(handoff), "late median", np.median(late), "early median", np.median(early))
print("early-done before late-ready (frac)", (slack > 0).mean(), "median slack", np.median(slack))
