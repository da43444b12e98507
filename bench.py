#!/usr/bin/env python3
"""Benchmark: illumstats + correct throughput (sites/s) on MI355X.

Metric (BASELINE.json): sites/sec for 2160x2560 uint16 site images through
corilla illumination statistics AND ChannelImage.correct.  One *step* is the
whole job over one channel's resident batch of sites (configs[1]: 384 wells x
9 sites = 3,456 sites per GPU):

    reset stats -> Welford + per-site histogram/percentiles over every site
    (tmh_stats_update_device) -> [N>1: RCCL Welford all-reduce merge + ordered
    percentile chain] -> finalize mean/std -> smooth both planes (sigma 5)
    -> correction coefficients -> correct every site (tmh_correct_u16_device)

Inputs are synthetic (counter-hash generator, SURVEY.md §8(d) distribution)
and resident in HBM before timing starts.  With N GPUs each rank owns its own
3,456 sites (weak scaling) and the merged statistics are identical on every
rank.  Prints ONE JSON line on rank 0.

    python bench.py                      # N=1, default steps
    torchrun --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

METRIC = "sites/sec (2160×2560 uint16) illumstats+correct; % of HBM roofline at 1–8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--sites", type=int, default=3456,
                   help="sites per channel per GPU (configs[1]: 384 wells x 9 sites)")
    p.add_argument("--channels", type=int, default=1,
                   help="channels per GPU, each its own job on its own stream (configs[2]/[3]: 4)")
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=2560)
    p.add_argument("--cpu-sample", type=int, default=24,
                   help="sites in the bounded CPU-baseline sample (0 disables)")
    p.add_argument("--no-profile", action="store_true", help="skip per-kernel event timing")
    p.add_argument("--pipeline", choices=["fused", "separate"], default="fused",
                   help="fused: histograms built from the correction's read (6 B/px); "
                        "separate: Welford || histogram pass, then correct (8 B/px)")
    p.add_argument("--serial-stats", action="store_true",
                   help="run the histogram pass after Welford instead of concurrently")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the extra (non-headline) measurements: the illuminati chain pass")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return p.parse_args()


def cpu_baseline(n_sites, H, W, total_sites):
    """Bounded sample of the CPU oracle (numpy, 1 process, single-threaded
    elementwise ops) over the same op sequence: per-site stats update +
    correct, plus the one-time smoothing amortised over the full job."""
    from oracle import corilla_oracle as orc
    from tmlibrary_amd.synth import synth_sites_host
    sites = synth_sites_host(n_sites, H, W, seed=2024)
    st = orc.OracleOnlineStatistics((H, W), percentile="numpy")  # stats.py:76 as written
    t0 = time.perf_counter()
    for s in sites:
        st.update(s)
    t1 = time.perf_counter()
    sm_mean = orc.smooth_reflect(st.mean, 5)
    sm_std = orc.smooth_reflect(st.std, 5)
    t2 = time.perf_counter()
    for s in sites:
        orc.correct_illumination(s, sm_mean, sm_std)
    t3 = time.perf_counter()
    per_site = ((t1 - t0) + (t3 - t2)) / n_sites + (t2 - t1) / total_sites
    return {
        "value": round(1.0 / per_site, 4),
        "unit": "sites/s",
        "cores": 1,
        "kind": "port",
        "sample": "%d synthetic %dx%d sites: oracle OnlineStatistics.update (np.percentile "
                  "with 100,000 q, log10, Welford) x%d + "
                  "correct_illumination x%d (numpy, 1 process) + smoothing of 2 planes "
                  "amortised over %d sites; stats %.1f ms/site, correct %.1f ms/site"
                  % (n_sites, H, W, n_sites, n_sites, total_sites,
                     1e3 * (t1 - t0) / n_sites, 1e3 * (t3 - t2) / n_sites),
    }


def bench_chain(L, corr, S_ptr, S, H, W, dev, sp, reps=3):
    """§8(f) rank 3, measured beside the headline: the illuminati chain
    (correct -> align(crop=False) -> clip -> scale to uint8, illuminati/api.py:
    396-405) over the same resident sites with per-site shifts; 3 B/px
    algorithmic (uint16 in, uint8 out)."""
    import torch

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import align_window
    wins = np.stack([align_window((H, W), s % 7 - 3, s % 9 - 4, 3, 3, 4, 4, crop=False)[0]
                     for s in range(S)])
    out8 = torch.empty((S, H, W), dtype=torch.uint8, device=dev)
    O8 = C.c_void_p(out8.data_ptr())
    lo, hi = 110, 4000
    hip.check(L.tmh_correct_chain_u8_device(corr, S_ptr, O8, S, hip.ptr(wins), lo, hi, sp))
    L.tmh_profile_enable(1)
    L.tmh_profile_reset()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        hip.check(L.tmh_correct_chain_u8_device(corr, S_ptr, O8, S, hip.ptr(wins), lo, hi, sp))
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / reps
    ms, k = C.c_double(), C.c_int64()
    hip.check(L.tmh_profile_read(b"chain", C.byref(ms), C.byref(k)))
    L.tmh_profile_enable(0)
    kern_ms = ms.value / max(k.value, 1)
    alg = S * H * W * 3
    del out8
    return {"workload": "illumination correct + align(crop=False, per-site shifts) + clip + "
                        "scale to uint8, %d sites of %dx%d" % (S, H, W),
            "value": round(S / el, 1), "unit": "sites/s", "kernel_avg_ms": round(kern_ms, 4),
            "alg_bytes_per_launch": alg,
            "achieved_GBs": round(alg / (kern_ms * 1e-3) / 1e9, 1),
            "frac_of_8TBs": round(alg / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def bench_host_path(H, W, n_sites=64, reps=3):
    """PCIe-inclusive rate of the drop-in host-buffer path (SURVEY §8(d) C5
    note; never the headline): numpy sites in host memory through
    OnlineStatistics.update_batch (tmh_stats_update) and Corrector.apply
    (tmh_correct_u16), double-buffered device slots on copy streams."""
    from tmlibrary_amd.image import Corrector
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    sites = np.ascontiguousarray(np.stack(synth_sites_host(n_sites, H, W, seed=7)))
    st = OnlineStatistics((H, W), batch_size=32)
    st.update_batch(sites)  # warm-up: both pinned and device slots allocated
    corr = Corrector(st.mean.array, st.std.array)
    corr.apply(sites)
    t_stats = t_corr = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        st.update_batch(sites)
        t_stats = min(t_stats, time.perf_counter() - t0)
        t0 = time.perf_counter()
        corr.apply(sites)
        t_corr = min(t_corr, time.perf_counter() - t0)
    out = np.empty_like(sites)
    corr.apply(sites, out=out)
    t_out = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        corr.apply(sites, out=out)
        t_out = min(t_out, time.perf_counter() - t0)
    st.close()
    corr.close()
    site_b = H * W * 2
    return {"workload": "%d host (numpy, pageable) sites of %dx%d: stats update (H2D 2 B/px) then "
                        "correct (H2D + D2H 4 B/px), PCIe-inclusive" % (n_sites, H, W),
            "stats_sites_per_s": round(n_sites / t_stats, 1),
            "stats_h2d_GBs": round(n_sites * site_b / t_stats / 1e9, 1),
            "correct_sites_per_s": round(n_sites / t_corr, 1),
            "correct_pcie_GBs": round(2 * n_sites * site_b / t_corr / 1e9, 1),
            "correct_reused_out_sites_per_s": round(n_sites / t_out, 1),
            "correct_reused_out_pcie_GBs": round(2 * n_sites * site_b / t_out / 1e9, 1),
            "job_sites_per_s": round(n_sites / (t_stats + t_corr), 1)}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    from tmlibrary_amd.workflow.corilla.sharded import StatsOps, merge_percentiles, merge_welford

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # TMH_BENCH_FORCE_DIST=1 runs the multi-GPU code path (RCCL merge,
    # deferred percentiles, pipelined chain) even with one rank
    dist_on = world > 1 or os.environ.get("TMH_BENCH_FORCE_DIST") == "1"
    if dist_on:
        dist.init_process_group("nccl", device_id=dev)
    L = hip.lib()
    hip.check(L.tmh_set_device(local_rank))
    H, W, S = a.height, a.width, a.sites
    npx = H * W
    Q = 100000
    # one non-null stream for our launches AND torch/RCCL work, so they order
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = C.c_void_p(stream.cuda_stream)

    # resident inputs / outputs (int16 tensors = raw uint16 bytes); channel c
    # owns sites [c*S, (c+1)*S)
    CH = a.channels
    sites = torch.empty((CH * S, H, W), dtype=torch.int16, device=dev)
    out = torch.empty_like(sites)
    for c in range(CH):
        hip.check(L.tmh_synth_sites_device(C.c_void_p(sites[c * S].data_ptr()), S, H, W, 12345, c,
                                           rank * S, sp))
    lo, hi, gamma = quantile_table(npx, np.linspace(0, 100, Q))
    lut = stats_log10_lut()
    flags = hip.TMH_STATS_DEFERRED_PCT if dist_on else 0
    if a.serial_stats:
        flags |= hip.TMH_STATS_SERIAL
    fused = a.pipeline == "fused"

    class Channel(object):
        """One channel's job: its sites, statistics handle, corrector and
        stream (channel 0 runs on the main stream; with several channels the
        others overlap on their own streams, configs[2]/[3])."""

        def __init__(self, c):
            self.stream = stream if c == 0 else torch.cuda.Stream(dev)
            self.sp = C.c_void_p(self.stream.cuda_stream)
            self.S_ptr = C.c_void_p(sites[c * S].data_ptr())
            self.O_ptr = C.c_void_p(out[c * S].data_ptr())
            self.mean = torch.empty(npx, dtype=torch.float64, device=dev)
            self.std = torch.empty_like(self.mean)
            self.smean = torch.empty_like(self.mean)
            self.sstd = torch.empty_like(self.mean)
            self.tmp = torch.empty_like(self.mean)
            self.h = C.c_void_p()
            hip.check(L.tmh_stats_create(H, W, Q, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                         hip.ptr(lut), 1, flags, C.byref(self.h)))
            hip.check(L.tmh_stats_set_stream(self.h, self.sp))
            self.corr = C.c_void_p()
            torch.cuda.synchronize(dev)
            hip.check(L.tmh_corrector_create_device(C.c_void_p(self.mean.data_ptr()),
                                                    C.c_void_p(self.std.data_ptr()), H, W, 1,
                                                    ZERO_LOG10, self.sp, C.byref(self.corr)))
            self.ops = StatsOps(L, self.h, npx, Q, dev)

        def stats(self):
            hip.check(L.tmh_stats_reset(self.h))
            if fused:  # Welford pass; histograms come from the correction's read
                hip.check(L.tmh_stats_update_welford_device(self.h, self.S_ptr, S, 1, self.sp))
            else:
                hip.check(L.tmh_stats_update_device(self.h, self.S_ptr, S, 1, self.sp))

        def apply(self):
            p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
            hip.check(L.tmh_stats_finalize_device(self.h, p(self.mean), p(self.std), self.sp))
            hip.check(L.tmh_smooth_f64_device(p(self.mean), p(self.smean), p(self.tmp), H, W, 5.0,
                                              self.sp))
            hip.check(L.tmh_smooth_f64_device(p(self.std), p(self.sstd), p(self.tmp), H, W, 5.0,
                                              self.sp))
            hip.check(L.tmh_corrector_update_device(self.corr, p(self.smean), p(self.sstd),
                                                    self.sp))
            if fused:
                hip.check(L.tmh_correct_u16_hist_device(self.corr, self.h, self.S_ptr, self.O_ptr,
                                                        S, -1, -1, self.sp))
            else:
                hip.check(L.tmh_correct_u16_device(self.corr, self.S_ptr, self.O_ptr, S, -1, -1,
                                                   self.sp))

        def close(self):
            L.tmh_corrector_destroy(self.corr)
            L.tmh_stats_destroy(self.h)

    chans = [Channel(c) for c in range(CH)]
    h, corr, S_ptr = chans[0].h, chans[0].corr, chans[0].S_ptr  # single-channel extras / check

    def step():
        for ch in chans:
            ch.stats()
        if dist_on:
            for ch in chans:
                with torch.cuda.stream(ch.stream):
                    merge_welford(ch.ops, dist)
        for ch in chans:
            ch.apply()
        if dist_on:
            for ch in chans:
                with torch.cuda.stream(ch.stream):
                    merge_percentiles(ch.ops, dist)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    prof = not a.no_profile
    if prof:
        L.tmh_profile_enable(1)
        L.tmh_profile_reset()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel event timing on the launch stream (live roofline)
    kern = {}
    if prof:
        for name in ("welford", "hist", "pct_acc", "finalize", "smooth", "coeffs", "correct",
                     "correct_hist", "hist_finalize"):
            ms, k = C.c_double(), C.c_int64()
            hip.check(L.tmh_profile_read(name.encode(), C.byref(ms), C.byref(k)))
            if k.value:
                kern[name] = (ms.value / k.value, k.value)
        L.tmh_profile_enable(0)

    # result fingerprint of the last step (identical on every rank and for
    # any N: merged mean/std and the bit-exact percentile sums)
    nn = C.c_int64()
    m_h = np.empty(npx)
    s_h = np.empty(npx)
    acc_h = np.empty(Q)
    hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(m_h), hip.ptr(s_h), hip.ptr(acc_h), None))
    import hashlib
    check = {"n": int(nn.value), "mean_sum": float(m_h.sum()), "std_sum": float(s_h.sum()),
             "pct_sums_sha256": hashlib.sha256(acc_h.tobytes()).hexdigest()[:16]}

    extras = {}
    if not a.no_extras and world == 1:
        extras["chain_u8"] = bench_chain(L, corr, S_ptr, S, H, W, dev, sp)
        extras["host_path"] = bench_host_path(H, W)

    if rank == 0:
        site_bytes = npx * 2
        alg = {  # algorithmic HBM bytes per launch (per-site figure x sites)
            "welford": S * site_bytes + 4 * 8 * npx,       # sites + mean/M2 read & write
            "hist": S * site_bytes,                        # sites
            "correct": S * site_bytes * 2 + 16 * npx,      # sites in + out, coefficients
            "correct_hist": S * site_bytes * 2 + 8 * npx,  # sites in + out, coefficients
            "pct_acc": S * Q * 4,                          # per-site order statistics
        }
        kdetail = {}
        for name, (avg_ms, k) in kern.items():
            d = {"avg_ms": round(avg_ms, 4), "launches": k}
            if name in alg:
                gbs = alg[name] / (avg_ms * 1e-3) / 1e9
                d["alg_GBs"] = round(gbs, 1)
                d["frac_of_8TBs"] = round(gbs / HBM_PEAK_GBS, 4)
            kdetail[name] = d
        dominant = max((n for n in kern if n in alg), key=lambda n: kern[n][0], default=None)
        roofline = None
        if dominant:
            avg_ms = kern[dominant][0]
            ach = alg[dominant] / (avg_ms * 1e-3) / 1e9
            traffic = None
            try:
                with open(a.traffic_json) as f:
                    tj = json.load(f)
                cfg = tj.get("config", {})
                if cfg.get("sites") == S and cfg.get("height") == H and cfg.get("width") == W:
                    traffic = tj.get("kernels", {}).get(dominant, {}).get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                pass
            roofline = {"bound": "hbm", "kernel": dominant, "achieved": round(ach, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "alg_bytes_per_launch": alg[dominant]}
        total_sites = world * CH * S * a.steps
        value = total_sites / elapsed
        job_bytes = world * CH * S * 6 * npx  # 6 B/px algorithmic per site-image
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "sites/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device counter-hash generator, SURVEY.md §8(d) distribution), "
                    "resident in HBM",
            "config": {"workload": ("illumstats+correct, 1 channel, %d sites/GPU of %dx%d uint16 "
                                    "(configs[1]: 384 wells x 9 sites)" % (S, H, W)) if CH == 1
                       else ("illumstats+correct, %d channels x %d sites/GPU of %dx%d uint16, "
                             "one job per channel on its own stream" % (CH, S, H, W)),
                       "sites_per_gpu": CH * S, "channels": CH, "height": H, "width": W,
                       "decimals": 3,
                       "smoothing_sigma": 5, "clip": None,
                       "parallelism": "sites sharded (contiguous); RCCL all-reduce Welford "
                                      "merge + ordered percentile chain" if world > 1
                                      else "single GPU",
                       "pipeline": a.pipeline},
            "job_hbm_roofline_frac": round(job_bytes * a.steps / elapsed / 1e9 / (HBM_PEAK_GBS * world), 4),
            "roofline": roofline,
            "kernels": kdetail,
        }
        res["check"] = check
        if extras:
            res["extras"] = extras
        if world == 1 and a.cpu_sample > 0:
            res["cpu_baseline"] = cpu_baseline(a.cpu_sample, H, W, S)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)

    for ch in chans:
        ch.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
