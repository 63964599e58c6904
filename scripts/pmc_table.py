"""Per-kernel averages of every counter in rocprofv3 --pmc pass directories (dev helper)."""
import csv
import collections
import sys


def kname(s):
    s = s.replace("(anonymous namespace)::", "").replace("accord::", "")
    return s.split("(")[0].replace("void ", "")


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in [a.rstrip("/") for a in sys.argv[1:]]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        agg[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    if k.startswith("__amd") or k.startswith("sc_"):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:24s} {sum(v) / len(v):16.0f}")
