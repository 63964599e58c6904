"""Per-kernel table of a rocprofv3 counter-collection csv: python3 pmc_table.py <csv> [name-filter]."""
import csv, sys
from collections import defaultdict
rows = csv.DictReader(open(sys.argv[1]))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(float))
for r in rows:
    n = r["Kernel_Name"]
    if filt not in n:
        continue
    key = n.replace("(anonymous namespace)::", "").split("(")[0][-60:]
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k)
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
