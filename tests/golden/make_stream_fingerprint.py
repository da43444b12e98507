#!/usr/bin/env python3
"""Oracle fingerprint of ``bench.py --stream-host`` (configs[4]) input.

The stream bench feeds every channel from a pinned host ring of R distinct
sites -- the device generator's sites 0 .. R-1 of (SEED, channel 0) --
channel c's global site g being ring site (g + 7 c) % R
(``bench.stream_ring_index``), on every rank.  tmlibrary_amd/synth.py
regenerates the ring bit for bit, so the oracle (oracle/corilla_oracle.py)
can be evaluated on exactly the streamed sequence without walking 24,576
full-size sites per channel:

  * percentile sums: each ring site's percentile vector once
    (stats.py:76), then the reference's sequential ``+=`` in the channel's
    site order -- the same f64 adds in the same order (bit-exact);
  * pooled histogram: sum of (multiplicity x ring-site histogram), exact;
  * mean / std of the log10 planes (stats.py:78-112) from the ring sites
    with their multiplicities, two-pass f64, at fixed sample pixels (the GPU's
    Welford result agrees to ~1e-12; the bar is 1e-6).

    python tests/golden/make_stream_fingerprint.py [--sites 24576] [--channels 5]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from bench import SEED, STREAM_RING, stream_fingerprint_name, stream_ring_index  # noqa: E402
from oracle import corilla_oracle as orc  # noqa: E402
from tmlibrary_amd import synth  # noqa: E402

N_STAT_SAMPLES = 16384


def log10_plane(img):
    """stats.py:78-85: astype(float), log10, zeros -> 0"""
    x = img.astype(np.float64)
    with np.errstate(divide="ignore"):
        x = np.log10(x)
    x[img == 0] = 0.0
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=2560)
    ap.add_argument("--sites", type=int, default=24576)
    ap.add_argument("--channels", type=int, default=5)
    ap.add_argument("--ring", type=int, default=STREAM_RING)
    a = ap.parse_args()
    H, W, S, CH, R = a.height, a.width, a.sites, a.channels, a.ring
    q = np.linspace(0, 100, 100000)
    rng = np.random.default_rng(2024)
    stat_px = np.sort(rng.choice(H * W, N_STAT_SAMPLES, replace=False))
    t0 = time.time()
    pv, hist, xs = [], [], []
    for k in range(R):
        img = synth.synth_exact_host(H, W, SEED, 0, k)
        pv.append(orc.percentile_linear(img, q))
        hist.append(orc.histogram_u16(img))
        xs.append(log10_plane(img).ravel()[stat_px])
        print("ring site %d/%d  %.0f s" % (k + 1, R, time.time() - t0), flush=True)
    xs = np.stack(xs)
    out = {"n": np.int64(S), "stat_px": stat_px, "mean_samples": [], "std_samples": [],
           "pct_sums_sha256": [], "hist_sha256": []}
    for c in range(CH):
        order = np.array([stream_ring_index(g, c, R) for g in range(S)])
        m = np.bincount(order, minlength=R).astype(np.float64)
        mean = (m[:, None] * xs).sum(axis=0) / S
        m2 = (m[:, None] * (xs - mean) ** 2).sum(axis=0)
        std = np.sqrt(m2 / (S - 1)) if S > 1 else np.full_like(mean, np.nan)
        acc = np.zeros(len(q))
        for k in order:  # the reference's sequential sum, in site order
            acc += pv[k]
        h = np.zeros(65536, np.uint64)
        for k in range(R):
            h += np.uint64(int(m[k])) * hist[k]
        out["mean_samples"].append(mean)
        out["std_samples"].append(std)
        out["pct_sums_sha256"].append(hashlib.sha256(acc.tobytes()).hexdigest())
        out["hist_sha256"].append(hashlib.sha256(h.tobytes()).hexdigest())
        print("channel %d done  %.0f s" % (c, time.time() - t0), flush=True)
    path = os.path.join(REPO, "tests", "golden", stream_fingerprint_name(H, W, S, CH, R))
    np.savez_compressed(path, n=out["n"], stat_px=out["stat_px"],
                        mean_samples=np.stack(out["mean_samples"]),
                        std_samples=np.stack(out["std_samples"]),
                        pct_sums_sha256=np.array(out["pct_sums_sha256"]),
                        hist_sha256=np.array(out["hist_sha256"]),
                        ring=np.int64(R), channels=np.int64(CH))
    print("wrote", path)


if __name__ == "__main__":
    main()
