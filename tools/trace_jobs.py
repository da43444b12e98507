#!/usr/bin/env python3
"""Kernel-by-kernel listing of a rocprofv3 --kernel-trace csv between the
K-th last launch of an anchor kernel and the end of the last one (ms from the
window start, duration, stream, queue):
    python tools/trace_jobs.py run_kernel_trace.csv [--anchor correct_hist] [-k 4]"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--anchor", default="correct_hist")
ap.add_argument("-k", type=int, default=4)
ap.add_argument("--min-us", type=float, default=0.0, help="hide kernels shorter than this")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]),
             int(r["Queue_Id"]),
             re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tmh::", "")[:44])
            for r in rows)
an = [k for k in ks if a.anchor in k[4]]
t0, t1 = an[-a.k][0], an[-1][1]
base = t0
for k in ks:
    if k[0] >= t0 and k[1] <= t1 and (k[1] - k[0]) / 1e3 >= a.min_us:
        print("%8.3f %8.3f %7.3f  s%-3d q%-2d %s" % ((k[0] - base) / 1e6, (k[1] - base) / 1e6,
                                                   (k[1] - k[0]) / 1e6, k[2], k[3], k[4]))
