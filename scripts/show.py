"""Print a bench JSON line and a kernel-stats CSV compactly (dev helper)."""
import csv
import json
import sys


def kname(s):
    s = s.replace("(anonymous namespace)::", "").replace("accord::", "")
    return s.split("(")[0].replace("void ", "")


for f in sys.argv[1:]:
    if f.endswith(".json"):
        d = json.load(open(f))
        print(f, round(d["value"]), round(d["ms_per_step"], 4))
        print("  stage", {k: round(v, 3) for k, v in d["stage_ms"].items() if v})
        r = d.get("roofline") or {}
        print("  roofline", r.get("achieved"), r.get("frac"))
    else:
        for r in csv.DictReader(open(f)):
            print(f"  {kname(r['Name'])[:40]:40s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs']) / 1e3:9.1f}")
