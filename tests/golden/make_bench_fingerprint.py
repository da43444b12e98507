#!/usr/bin/env python3
"""Oracle fingerprint of bench.py's full-size input (VERDICT r1 "bench pin").

bench.py fills HBM with tmh_synth_sites_device; tmlibrary_amd/synth.py
(synth_exact_host) regenerates the same pixels bit for bit on the host, so the
CPU oracle (oracle/corilla_oracle.py) can be run on exactly the bench's
sites.  This script does that once, in this container, and commits the
result under tests/golden/ as data; bench.py compares its last step against
it and prints ``check_vs_oracle``.

Per channel job (reference: tmlib/workflow/corilla/stats.py:64-121,
tmlib/image.py:599-631, :1172-1193):
  n; pooled 65,536-bin histogram (exact) and its sha256; the f64 percentile
  sums (sequential site-order sum, bit-exact) as a sha256; mean / std and the
  smoothed planes at fixed sample pixels; the corrected uint16 values of
  three sites (first, middle, last) at sample pixels.
The Welford state is built per block of sites in worker processes and merged
with Chan's formula (oracle.chan_merge; ~1e-14 from one sequential pass, the
bar is 1e-6); percentile vectors come back per site and are summed in site
order in this process, so the sums are the reference's sequential sums.

    python tests/golden/make_bench_fingerprint.py [--sites 3456] [--distribution synthetic]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from bench import fingerprint_name  # noqa: E402
from oracle import corilla_oracle as orc  # noqa: E402
from tmlibrary_amd import synth  # noqa: E402

N_STAT_SAMPLES = 16384
N_CORR_SAMPLES = 65536




def _block(args):
    H, W, seed, channel, a, b, dist = args
    st = orc.OracleOnlineStatistics((H, W), keep_site_percentiles=True)
    hist = np.zeros(65536, dtype=np.uint64)
    for s in range(a, b):
        img = synth.synth_exact_host(H, W, seed, channel, s, dist)
        hist += orc.histogram_u16(img)
        st.update(img)
    return a, st.n, st._mean, st._M2, np.stack(st.site_percentiles), hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=3456)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=2560)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--channel", type=int, default=0)
    ap.add_argument("--distribution", choices=sorted(synth.DISTRIBUTIONS), default="synthetic")
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--block", type=int, default=48)
    a = ap.parse_args()
    H, W, S = a.height, a.width, a.sites
    dist = synth.DISTRIBUTIONS[a.distribution]
    t0 = time.time()
    jobs = [(H, W, a.seed, a.channel, s, min(S, s + a.block), dist) for s in range(0, S, a.block)]
    acc = np.zeros(100000)
    hist = np.zeros(65536, dtype=np.uint64)
    parts = []
    with mp.get_context("fork").Pool(a.workers) as pool:
        for first, n, mean, m2, pcts, h in pool.imap(_block, jobs):  # in site order
            for p in pcts:
                acc += p  # stats.py:76, sequential in site order
            hist += h
            parts.append((n, mean, m2))
            print("sites %d..%d done (%.0f s)" % (first, first + n, time.time() - t0), flush=True)
    n, mean, m2 = orc.chan_merge(parts)
    std = np.sqrt(m2 / (n - 1))
    smean = orc.smooth_reflect(mean, 5)
    sstd = orc.smooth_reflect(std, 5)
    npx = H * W
    rng = np.random.default_rng(0)
    sp = np.sort(rng.choice(npx, min(npx, N_STAT_SAMPLES), replace=False))
    cp = np.sort(rng.choice(npx, min(npx, N_CORR_SAMPLES), replace=False))
    corr_sites = np.array(sorted({0, S // 2, S - 1}), dtype=np.int64)
    corr = []
    corr_hist = []
    for s in corr_sites:
        img = synth.synth_exact_host(H, W, a.seed, a.channel, int(s), dist)
        c = orc.correct_illumination(img, smean, sstd).ravel()
        corr.append(c[cp])
        corr_hist.append(np.bincount(c, minlength=65536).astype(np.uint32))
    out = dict(
        n=np.int64(n), height=np.int64(H), width=np.int64(W), sites=np.int64(S),
        seed=np.int64(a.seed), channel=np.int64(a.channel), distribution=np.int64(dist),
        pct_sums_sha256=np.str_(hashlib.sha256(acc.tobytes()).hexdigest()),
        hist=hist, hist_sha256=np.str_(hashlib.sha256(hist.tobytes()).hexdigest()),
        mean_sum=np.float64(mean.sum()), std_sum=np.float64(std.sum()),
        stat_px=sp.astype(np.int64), mean_samples=mean.ravel()[sp], std_samples=std.ravel()[sp],
        smean_samples=smean.ravel()[sp], sstd_samples=sstd.ravel()[sp],
        corr_sites=corr_sites, corr_px=cp.astype(np.int64), corr_samples=np.stack(corr),
        corr_hist=np.stack(corr_hist),
    )
    path = os.path.join(REPO, "tests", "golden",
                        fingerprint_name(H, W, S, a.seed, a.channel, a.distribution))
    np.savez_compressed(path, **out)
    print(json.dumps({"written": os.path.relpath(path, REPO), "n": int(n),
                      "pct_sums_sha256": str(out["pct_sums_sha256"])[:16],
                      "hist_sha256": str(out["hist_sha256"])[:16],
                      "seconds": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main()
