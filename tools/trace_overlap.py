#!/usr/bin/env python3
"""Where the histogram tail runs: from a rocprofv3 --kernel-trace csv, the
time each of the job's passes (k_correct_hist, k_welford_vec8) shares with
the tail kernels (k_hist_finalize*, k_pct_acc, k_pooled_colsum*), per pass
launch and in total:
    python tools/trace_overlap.py run_kernel_trace.csv [-o out.json]"""
import argparse
import csv
import json
import re

TAIL = ("k_hist_finalize", "k_pct_acc", "k_pooled_colsum")
PASSES = ("k_correct_hist", "k_welford_vec8")


def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "").replace("tmh::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
          for r in rows]
    tails = [k for k in ks if any(t in k[2] for t in TAIL)]
    res = {}
    for p in PASSES:
        launches = sorted(k for k in ks if p in k[2])
        if not launches:
            continue
        big = max(k[1] - k[0] for k in launches)
        launches = [k for k in launches if k[1] - k[0] >= 0.25 * big]  # the job's own launches
        per = []
        for s0, s1, _ in launches:
            ov = {}
            for t0, t1, tn in tails:
                o = min(s1, t1) - max(s0, t0)
                if o > 0:
                    key = next(t for t in TAIL if t in tn)
                    ov[key] = ov.get(key, 0) + o
            per.append({"ms": round((s1 - s0) / 1e6, 4),
                        "tail_overlap_ms": {k: round(v / 1e6, 4) for k, v in ov.items()}})
        res[p] = {"launches": len(per),
                  "avg_ms": round(sum(x["ms"] for x in per) / len(per), 4),
                  "launches_sharing_with_tail": sum(1 for x in per if x["tail_overlap_ms"]),
                  "avg_tail_overlap_ms": round(sum(sum(x["tail_overlap_ms"].values())
                                                   for x in per) / len(per), 4),
                  "per_launch": per}
    out = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "per_launch"}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
