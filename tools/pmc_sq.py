#!/usr/bin/env python3
"""Per-kernel SQ / GRBM counter summary from rocprofv3 --pmc runs.

Each pass is its own rocprofv3 run (at most 8 SQ and 2 GRBM counters, see
tools/gpu.sh step pmcsq); this merges the passes' counter_collection.csv files
and prints, per kernel (full name), the per-dispatch median of every counter
over the headline-sized dispatches (>= 1/4 of the kernel's largest
SQ_WAVE_CYCLES or first counter), plus derived ratios:

  gui_per_xcd     GRBM_GUI_ACTIVE / n_xcd (the counter is summed over the 8
                  XCDs' GRBMs on gfx950: 222.0M over a 12.82 ms dispatch is
                  8 x 2.16 GHz; SQ_BUSY_CYCLES / 32 SEs agrees)
  valu_busy       SQ_ACTIVE_INST_VALU * 4 / (n_simd * gui_per_xcd)
                  (ACTIVE_INST_* count quad-cycles, summed over waves; a
                  SIMD issues for one wave at a time)
  lds_busy        SQ_LDS_IDX_ACTIVE / (n_cu * gui_per_xcd)
  lds_conflict    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait_any        SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves waiting on anything)
  wait_inst_any   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting for an
                  instruction's dependency: vmcnt / lgkmcnt)
  *_per_px        instructions (wave-level) per pixel of the dispatch
  clock_mhz       gui_per_xcd / dispatch duration (when the csv has
                  timestamps)

    python tools/pmc_sq.py DIR [DIR ...] --pixels N -o out.json
    python tools/pmc_sq.py --rederive OLD.json -o out.json   (counters kept, ratios recomputed)
"""
from __future__ import annotations

import argparse
import csv
import glob
import hashlib
import json
import os
from collections import defaultdict


def read_dirs(dirs):
    """{kernel: {dispatch: {counter: value, '_ns': duration}}}"""
    out = defaultdict(lambda: defaultdict(dict))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name") or row.get("KernelName") or ""
                    c = row.get("Counter_Name") or row.get("CounterName") or ""
                    v = float(row.get("Counter_Value") or row.get("CounterValue") or 0)
                    disp = (d, row.get("Dispatch_Id") or row.get("DispatchId") or "")
                    rec = out[name][disp]
                    rec[c] = rec.get(c, 0.0) + v
                    t0, t1 = row.get("Start_Timestamp"), row.get("End_Timestamp")
                    if t0 and t1:
                        rec["_ns"] = float(t1) - float(t0)
    return out


def derive(med, pixels, n_cu, n_xcd):
    g = med.get("GRBM_GUI_ACTIVE")
    dv = {}
    if g:
        g = g / n_xcd
        if "SQ_ACTIVE_INST_VALU" in med:
            dv["valu_busy"] = med["SQ_ACTIVE_INST_VALU"] * 4 / (4 * n_cu * g)
        if "SQ_LDS_IDX_ACTIVE" in med:
            dv["lds_busy"] = med["SQ_LDS_IDX_ACTIVE"] / (n_cu * g)
        if "_ns" in med and med["_ns"] > 0:
            dv["clock_mhz"] = g / med["_ns"] * 1e3
    if med.get("SQ_LDS_IDX_ACTIVE"):
        dv["lds_conflict"] = med.get("SQ_LDS_BANK_CONFLICT", 0.0) / med["SQ_LDS_IDX_ACTIVE"]
    if med.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in med:
                dv[c.lower()[3:]] = med[c] / med["SQ_WAVE_CYCLES"]
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_VMEM_WR"):
        if c in med:
            dv[c.lower()[3:] + "_per_px"] = med[c] / pixels
    return {k: round(v, 4) for k, v in dv.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dirs", nargs="*")
    p.add_argument("--pixels", type=float,
                   help="pixels one headline dispatch of the kernels of interest processes")
    p.add_argument("--n-cu", type=int, default=256)
    p.add_argument("--n-xcd", type=int, default=8)
    p.add_argument("--rederive", help="recompute the ratios of an earlier output's counters")
    p.add_argument("--kernels", default="k_correct_hist,k_welford_vec8",
                   help="comma list of kernel-name substrings to report")
    p.add_argument("-o", "--out", required=True)
    a = p.parse_args()
    if a.rederive:
        with open(a.rederive) as fh:
            res = json.load(fh)
        res["note"] = __doc__.split("\n\n")[1]
        for v in res["kernels"].values():
            v["derived"] = derive(v["counters"], res["pixels_per_dispatch"], a.n_cu, a.n_xcd)
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
        return
    if not a.dirs or a.pixels is None:
        p.error("DIR ... and --pixels are required")
    data = read_dirs(a.dirs)
    want = [k for k in a.kernels.split(",") if k]
    lib = os.environ.get("TMH_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                 "tmlibrary_amd", "hip", "libtmhip.so"))
    with open(lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    res = {"library_sha256": lib_sha, "pixels_per_dispatch": a.pixels,
           "note": __doc__.split("\n\n")[1], "kernels": {}}
    for name, disps in data.items():
        if want and not any(w in name for w in want):
            continue
        # per pass (directory), the dispatches of headline size; counters of
        # different passes are medians over their own passes' dispatches
        per_counter = defaultdict(list)
        by_dir = defaultdict(list)
        for (d, _), rec in disps.items():
            by_dir[d].append(rec)
        for d, recs in by_dir.items():
            key = "SQ_WAVE_CYCLES" if any("SQ_WAVE_CYCLES" in r for r in recs) else None
            if key is None:
                key = next((c for c in recs[0] if not c.startswith("_")), None)
            top = max(r.get(key, 0.0) for r in recs) if key else 0.0
            for r in recs:
                if key and r.get(key, 0.0) < 0.25 * top:
                    continue
                for c, v in r.items():
                    per_counter[c].append(v)
        med = {}
        for c, vs in per_counter.items():
            vs = sorted(vs)
            med[c] = vs[len(vs) // 2]
        res["kernels"][name] = {"counters": med, "derived": derive(med, a.pixels, a.n_cu, a.n_xcd),
                                "dispatches": len(disps)}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
