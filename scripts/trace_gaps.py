"""GPU busy vs idle inside a kernel trace (rocprofv3 --kernel-trace csv): the union of kernel
intervals against the span from the first to the last kernel, over the last `tail` fraction of the
trace (the steady state).  python3 scripts/trace_gaps.py <run_kernel_trace.csv> [tail=0.3]"""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
tail = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
iv = iv[int(len(iv) * (1 - tail)):]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
print(f"kernels {len(iv)}, span {span/1e6:.3f} ms, busy {busy/1e6:.3f} ms ({100*busy/span:.1f} %), "
      f"idle {(span-busy)/1e6:.3f} ms, mean kernel {busy/len(iv)/1e3:.1f} us")
