#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace csv: per step window, the busy
union of all kernels, each stream's kernels in order with the gaps between
them, and which kernels run while a big streaming kernel (name filter) is
alone on the GPU.
    python tools/trace_timeline.py run_kernel_trace.csv [--big correct_hist,welford]
        [--last-ms 40]"""
import argparse
import csv
import re


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "").replace("tmh::", "").replace("(anonymous namespace)::", "")
    return n[:48]


ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last-ms", type=float, default=40.0, help="analyse the trace's last N ms")
ap.add_argument("--streams", action="store_true", help="print every stream's kernel sequence")
ap.add_argument("--anchor", default=None,
                help="window = from the K-th last kernel whose name contains this, to the end "
                     "of the last one (K = --anchor-count)")
ap.add_argument("--anchor-count", type=int, default=4)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]),
       int(r["Queue_Id"]), short(r["Kernel_Name"])) for r in rows]
ks.sort()
if a.anchor:
    an = [k for k in ks if a.anchor in k[4]]
    t0 = an[-a.anchor_count][0]
    t_end = an[-1][1]
    ks = [k for k in ks if k[0] >= t0 and k[1] <= t_end]
else:
    t_end = max(k[1] for k in ks)
    t0 = t_end - int(a.last_ms * 1e6)
    ks = [k for k in ks if k[0] >= t0]
span = (ks[-1][1] - ks[0][0]) / 1e6
# busy union
busy, cur_s, cur_e = 0, None, None
for s, e, *_ in ks:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("window %.3f ms, %d kernels, busy union %.3f ms (idle %.3f ms)" %
      (span, len(ks), busy / 1e6, span - busy / 1e6))
agg = {}
for s, e, st, q, n in ks:
    d = agg.setdefault(n, [0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1e6
print("%-50s %6s %10s %9s" % ("kernel", "calls", "sum ms", "avg ms"))
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("%-50s %6d %10.3f %9.4f" % (n, c, t, t / c))
if a.streams:
    by = {}
    for k in ks:
        by.setdefault(k[2], []).append(k)
    for st, lst in sorted(by.items()):
        print("\nstream %d (queue %s): %d kernels" % (st, sorted({k[3] for k in lst}), len(lst)))
        prev = None
        for s, e, _, q, n in lst:
            gap = (s - prev) / 1e3 if prev else 0
            print("  +%8.1f us gap  %8.1f us  %s" % (gap, (e - s) / 1e3, n))
            prev = e
