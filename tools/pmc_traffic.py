#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC counters.

Follows MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
  * FETCH_SIZE and WRITE_SIZE are collected in SEPARATE passes (their TCC
    slot costs do not fit one pass), each with --kernel-trace only;
  * both are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
    streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
    write bytes = WRITE_SIZE * 1024 (exact for 16-B-per-lane stores).

Usage on the GPU box (each step under its own timeout):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
      python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-profile
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
      python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-profile
  python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
      --sites 3456 --height 2160 --width 2560 -o profiles/pmc_traffic.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import hashlib
import json
import os
import re
from collections import defaultdict

SHORT = {
    "k_welford_vec8": "welford",
    "k_hist_scatter": "hist",
    "k_hist_finalize": "hist_finalize",
    "k_correct_hist": "correct_hist",
    "k_correct_u16_vec8": "correct",
    "k_pct_acc": "pct_acc",
    "k_wf_merge_parts": "welford_merge",
    "k_chain_u8": "chain",
    "k_pooled_colsum": "colsum",
}


def short_name(kernel: str):
    for k, v in SHORT.items():
        if k in kernel:
            return v
    return None


def read_counter(d, counter):
    """{short kernel: [values per dispatch]} from a rocprofv3 counter csv."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    out = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("KernelName") or ""
                cname = row.get("Counter_Name") or row.get("CounterName") or ""
                if cname != counter:
                    continue
                k = short_name(name)
                if k:
                    out[k].append(float(row.get("Counter_Value") or row.get("CounterValue")))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--sites", type=int, required=True)
    p.add_argument("--height", type=int, required=True)
    p.add_argument("--width", type=int, required=True)
    p.add_argument("--distribution", default="synthetic")
    p.add_argument("-o", "--out", required=True)
    a = p.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    npx = a.height * a.width
    site_bytes = 2 * npx
    alg = {"welford": a.sites * site_bytes + 32 * npx, "hist": a.sites * site_bytes,
           "correct": 2 * a.sites * site_bytes + 16 * npx,
           "correct_hist": 2 * a.sites * site_bytes + 8 * npx,
           "chain": 3 * a.sites * npx}
    lib = os.environ.get("TMH_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                 "tmlibrary_amd", "hip", "libtmhip.so"))
    with open(lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    res = {"config": {"sites": a.sites, "height": a.height, "width": a.width,
                      "distribution": a.distribution},
           "library_sha256": lib_sha,
           "method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per launch (separate --pmc passes; "
                     "gfx950 FETCH_SIZE halving corrected); median over the headline-sized launches "
                     "(>= 1/4 of the kernel's largest)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        # the headline job's launches only: the bench's extras (e.g. the
        # host-path batches) launch the same kernels on a few sites
        f = sorted(fetch.get(k, []))
        w = sorted(write.get(k, []))
        f = [x for x in f if x >= 0.25 * f[-1]] if f else f
        w = [x for x in w if x >= 0.25 * w[-1]] if w else w
        fm = f[len(f) // 2] if f else None
        wm = w[len(w) // 2] if w else None
        rd = 2 * fm * 1024 if fm is not None else None
        wr = wm * 1024 if wm is not None else None
        tot = (rd or 0) + (wr or 0) if (rd is not None or wr is not None) else None
        res["kernels"][k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": tot,
                             "alg_bytes_per_launch": alg.get(k),
                             "traffic_over_alg": (tot / alg[k]) if (tot and k in alg) else None,
                             "launches": max(len(f), len(w))}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
