"""One timed step of a rocprofv3 kernel + HIP runtime trace: every GPU
activity (kernels, copies) with its start offset and duration, and each idle
gap over --min-gap-us with the long host calls that span it.

  python3 tools/trace_gaps.py gpurun_out/rocprof_dist432h_TAG [--anchor correct_hist] [--index 3]
"""
import argparse
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--anchor", default="correct_hist", help="kernel name part marking step ends")
    ap.add_argument("--index", type=int, default=3, help="the step after the index-th anchor launch")
    ap.add_argument("--min-gap-us", type=float, default=20.0)
    ap.add_argument("--summary", action="store_true", help="only the busy/idle totals per step")
    a = ap.parse_args()
    rd = lambda n: list(csv.DictReader(open(os.path.join(a.dir, n))))  # noqa: E731
    k = rd("run_kernel_trace.csv")
    api = rd("run_hip_api_trace.csv") if os.path.exists(os.path.join(a.dir, "run_hip_api_trace.csv")) else []
    mc = rd("run_memory_copy_trace.csv") if os.path.exists(os.path.join(a.dir, "run_memory_copy_trace.csv")) else []
    anc = sorted((x for x in k if a.anchor in x["Kernel_Name"]), key=lambda x: int(x["Start_Timestamp"]))
    steps = range(len(anc) - 1) if a.summary else [a.index]
    for idx in steps:
        t0, t1 = int(anc[idx]["End_Timestamp"]), int(anc[idx + 1]["End_Timestamp"])
        ev = []
        for x in k:
            s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
            if e > t0 and s < t1:
                n = x["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
                ev.append((s, e, "K s%s %s" % (x["Stream_Id"], n)))
        for x in mc:
            s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
            if e > t0 and s < t1:
                ev.append((s, e, "M %s" % x.get("Direction", "")))
        ev.sort()
        busy_end, idle = t0, 0
        for s, e, n in ev:
            gap = s - busy_end
            if gap > a.min_gap_us * 1e3:
                idle += gap
                if not a.summary:
                    hs = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Function"]) for x in api
                          if int(x["End_Timestamp"]) > busy_end and int(x["Start_Timestamp"]) < s and
                          int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) > a.min_gap_us * 1e3]
                    print("   GAP %.1f us; long host calls: %s" % (
                        gap / 1e3, [(f, round((q - p) / 1e3, 1), round((p - t0) / 1e3, 1))
                                    for p, q, f in hs][:6]))
            if not a.summary:
                print("%8.1f %8.1f %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))
            busy_end = max(busy_end, e)
        print("step after anchor %d: %.3f ms, idle gaps > %.0f us: %.3f ms" % (
            idx, (t1 - t0) / 1e6, a.min_gap_us, idle / 1e6))


if __name__ == "__main__":
    main()
