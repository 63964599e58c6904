"""Per-step HBM traffic of the roofline unit (one or more kernels, comma-separated substrings) from rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE in separate runs; values in KB per dispatch).  gfx950 correction (MI355X_MICROARCH.md,
HBM): FETCH_SIZE reports half the bytes of wide coalesced reads, so traffic = 2*FETCH + WRITE; the
raw counters are kept next to it.  With a request-size pass (TCC_EA0_RDREQ_{32B,64B,128B}_sum and
TCC_EA0_RDREQ_sum in one run, [rdreq_dir]) the read bytes are resolved per request size instead
(32/64/128-byte requests at their sizes) and traffic = resolved reads + WRITE_SIZE.  Usage:
traffic_json.py <fetch_dir> <write_dir> <substr[,substr..]> <profile-dir-to-cite> <out.json> [rdreq_dir]"""
import csv
import json
import sys


def per_dispatch(d, counter, ksub):
    vals = []
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter and ksub in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {ksub} in {d}")
    return sum(vals) / len(vals), len(vals)


fetch_dir, write_dir, ksubs, cite, out = sys.argv[1:6]
rdreq_dir = sys.argv[6] if len(sys.argv) > 6 else None
fkb = wkb = rb = 0.0
per = {}
for ksub in ksubs.split(","):        # every kernel of the unit runs once per step
    f, nf = per_dispatch(fetch_dir, "FETCH_SIZE", ksub)
    w, nw = per_dispatch(write_dir, "WRITE_SIZE", ksub)
    per[ksub] = {"fetch_size_kb": f, "write_size_kb": w, "dispatches": [nf, nw]}
    if rdreq_dir:
        q = {c: per_dispatch(rdreq_dir, f"TCC_EA0_RDREQ{c}_sum", ksub)[0] for c in ("_32B", "_64B", "_128B", "")}
        b = 32 * q["_32B"] + 64 * q["_64B"] + 128 * q["_128B"]
        per[ksub].update({"rdreq": q, "read_bytes_resolved": b})
        rb += b
    fkb += f
    wkb += w
doc = {"kernel": ksubs, "fetch_size_kb": fkb, "write_size_kb": wkb, "per_kernel": per,
       "traffic_bytes": (2 * fkb + wkb) * 1024.0,
       "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide reads)",
       "source": cite}
parts_ok = rdreq_dir and all(abs(v["rdreq"]["_32B"] + v["rdreq"]["_64B"] + v["rdreq"]["_128B"] - v["rdreq"][""])
                             <= 0.02 * max(1.0, v["rdreq"][""]) for v in per.values())
if rdreq_dir and not parts_ok:        # the size classes do not partition RDREQ: keep the x2 estimate
    doc["read_bytes_resolved"] = rb
    doc["rdreq_note"] = "RDREQ_32B + RDREQ_64B + RDREQ_128B != RDREQ: request-size resolution not used"
if parts_ok:
    doc["traffic_bytes_fetch_x2"] = doc["traffic_bytes"]
    doc["read_bytes_resolved"] = rb
    doc["traffic_bytes"] = rb + wkb * 1024.0
    doc["correction"] = ("reads resolved by request size (32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B) "
                         "+ WRITE_SIZE; the 2*FETCH_SIZE estimate kept as traffic_bytes_fetch_x2")
json.dump(doc, open(out, "w"), indent=1)
print(json.dumps(doc))
