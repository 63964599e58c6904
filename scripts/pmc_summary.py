"""Summarise rocprofv3 --pmc CSVs (FETCH_SIZE / WRITE_SIZE passes) per kernel."""
import csv
import collections
import sys


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    return s.split("(")[0].replace("void ", "")


def main(dirs):
    print("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; values are KB per dispatch;")
    print("gfx950 FETCH_SIZE reports ~1/2 of wide coalesced streams (MI355X_MICROARCH.md §HBM)")
    for d in dirs:
        agg = collections.defaultdict(lambda: [0, 0.0])
        with open(f"{d}/run_counter_collection.csv") as f:
            for r in csv.DictReader(f):
                k = (kname(r["Kernel_Name"]), r["Counter_Name"])
                agg[k][0] += 1
                agg[k][1] += float(r["Counter_Value"])
        for (k, c), (n, v) in sorted(agg.items(), key=lambda x: -x[1][1]):
            print(f"{c:11s} dispatches={n:3d} avg_KB={v / n:14.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1:])
