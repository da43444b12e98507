#!/usr/bin/env python3
"""Benchmark: illumstats + correct throughput (sites/s) on MI355X.

Metric (BASELINE.json): sites/sec for 2160x2560 uint16 site images through
corilla illumination statistics AND ChannelImage.correct.  One *step* is the
whole job over every channel's resident batch of sites:

    reset stats -> Welford (tmh_stats_update_welford_device)
    -> [N>1: RCCL Welford all-reduce merge] -> finalize mean/std -> smooth both
    planes (sigma 5) -> correction coefficients -> fused correct + per-site
    histogram pass -> order statistics -> ordered percentile sum
    (tmh_correct_u16_hist_device) -> [N>1: ordered percentile chain +
    histogram all-reduce]

Workloads:
  N = 1   configs[1]: one channel, 3,456 sites (384 wells x 9 sites) on one GPU.
  N > 1   configs[2]: 4 channels x 3,456 sites, each channel's sites sharded
          contiguously over the ranks (432 per channel per GPU at N = 8); one
          job per channel on its own stream, so a channel's merge overlaps the
          next channel's kernels.  Total work is fixed: "scaling": "strong".
  --layout per-gpu gives every rank its own 3,456 sites per channel instead
  (weak scaling).

Inputs come from the device generator (tmh_synth_sites_device), resident in
HBM before timing starts.  Its host twin (tmlibrary_amd/synth.py) regenerates
the same pixels, so the last step's results are compared against an oracle
fingerprint committed under tests/golden/ (make_bench_fingerprint.py):
``check_vs_oracle``.  Prints ONE JSON line on rank 0.

    python bench.py                      # N=1, default steps
    python bench.py --gpus N             # starts N rank processes itself (launch())
    torchrun --nproc-per-node N bench.py --gpus N
    python bench.py --gpus 1 --channels 4 --layout sharded   # configs[2]'s workload on 1 GPU
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

METRIC = "sites/sec (2160×2560 uint16) illumstats+correct; % of HBM roofline at 1–8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
SEED = 12345


def log(msg):
    """Progress on stderr (a long silent run looks hung to the GPU harness)."""
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one process per GPU).  Without WORLD_SIZE in the environment and "
                        "N > 1, bench.py starts the N rank processes itself; under torchrun it "
                        "must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: every rank joins a gloo group and rank 0 "
                        "prints the ranks' environments as its JSON line")
    p.add_argument("--deadline", type=float, default=1500.0,
                   help="--gpus N launcher: seconds the whole run may take; past it every rank's "
                        "process group is killed and the launcher exits 3 naming each rank's "
                        "last stage (the reference's failed job: exit non-zero with the cause, "
                        "tmlib/workflow/cli.py:287-293)")
    p.add_argument("--stall-timeout", type=float, default=300.0,
                   help="--gpus N launcher: seconds without a heartbeat from ANY rank (every "
                        "rank stuck, e.g. all waiting in a collective) before the ranks are "
                        "killed and the launcher exits 3 naming each rank's last stage")
    p.add_argument("--coll-timeout", type=float, default=600.0,
                   help="timeout (s) of the ranks' process group (init and every collective)")
    p.add_argument("--share-gpu", action="store_true",
                   help="N > 1 ranks on GPU 0 of a one-GPU box (parity runs only): gloo group, "
                        "collectives staged through host memory (sharded.HostStagedDist)")
    p.add_argument("--share-outputs", choices=["auto", "yes", "no"], default="auto",
                   help="several channels: their corrected outputs share HBM blocks except the "
                        "blocks holding the sites checked against the oracle (auto: when private "
                        "outputs would not fit, e.g. 4 channels x 3,456 sites on one GPU)")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--sites", type=int, default=3456,
                   help="sites per channel (384 wells x 9 sites); per GPU with --layout per-gpu")
    p.add_argument("--channels", type=int, default=None,
                   help="channels, each its own job on its own stream (default 1 at N=1, "
                        "4 when sharded: configs[2])")
    p.add_argument("--layout", choices=["auto", "per-gpu", "sharded"], default="auto",
                   help="sharded: each channel's sites split over the ranks (default for N>1); "
                        "per-gpu: every rank has its own --sites per channel")
    p.add_argument("--distribution", choices=["synthetic", "bright", "uniform"],
                   default="synthetic",
                   help="pixel distribution of the generated sites (tmlibrary_amd/synth.py)")
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=2560)
    p.add_argument("--cpu-sample", type=int, default=96,
                   help="sites of the CPU-baseline job (configs[0]: 96; 0 disables)")
    p.add_argument("--cpu-procs", type=int, default=4,
                   help="P of the P-process CPU variant (one channel job per process; "
                        "P = min(this, cores))")
    p.add_argument("--fused-cus", type=int, default=None,
                   help="TMH_OPT_FUSED_CUS: CUs' worth of workgroups of the fused pass's "
                        "persistent grid (default: the library's, all CUs)")
    p.add_argument("--welford-parts", type=int, default=None,
                   help="TMH_OPT_WELFORD_PARTS (1..4 forces that split and the standard pass; "
                        "default: automatic, from the job's site probe)")
    p.add_argument("--welford-cus", type=int, default=None,
                   help="(experiment) one channel: run each job lane's stream -- its Welford "
                        "pass and planes -- on a stream CU-masked to this many CUs, leaving the "
                        "rest to the previous job's histogram tail; several channels "
                        "(pipelined order): the Welford passes on a stream so masked, the "
                        "channels' merges and plane chains beside them on the rest")
    p.add_argument("--fused-config", type=int, default=None,
                   help="fused pass (sites per unit, threads, LDS bins) configuration 0..5 "
                        "(TMH_OPT_FUSED_CONFIG; default: automatic, from the job's site probe)")
    p.add_argument("--block-sites", type=int, default=64,
                   help="sites per HBM allocation of the corrected output (a power of two >= 4; "
                        "blocked site layout); 0: one contiguous buffer")
    p.add_argument("--in-layout", choices=["contiguous", "blocked"], default="contiguous",
                   help="with --block-sites B: the input sites in one buffer (the Welford pass "
                        "takes its contiguous path, the fused pass a block table into it) or in "
                        "B-site blocks allocated alternately with the output blocks")
    p.add_argument("--no-profile", action="store_true", help="skip per-kernel event timing")
    p.add_argument("--no-box", action="store_true",
                   help="skip the box probe (the box's copy / read rate and shader clock over "
                        "the job's own buffers, reported as 'box')")
    p.add_argument("--hbm-skip-gb", type=float, default=0.0,
                   help="hold an allocation of this many GB before the sites' buffers "
                        "(placement study: which HBM region the first buffer lands in)")
    p.add_argument("--jobs-in-flight", type=int, default=2,
                   help="one channel on one rank: consecutive jobs (steps) alternate between "
                        "this many statistics handles / correctors / streams, so job k+1's "
                        "Welford pass runs while job k's histogram tail finishes (each job "
                        "still complete and checked; 1 = one job at a time)")
    p.add_argument("--jobs-order", choices=["welford", "planes", "corrected"], default="welford",
                   help="jobs in flight: job k+1's Welford pass starts after job k's Welford pass "
                        "(sharing HBM with job k's corrected pass, hiding job k's small kernels "
                        "and tail), after job k's planes, or after job k's corrected pass "
                        "(hiding only the tail); a pipelined order measured no better "
                        "(DESIGN.md 9.5, 10.7)")
    p.add_argument("--planes", choices=["multi", "per-job"], default="multi",
                   help="finalize -> smoothing -> coefficients: every channel's in one launch per "
                        "kernel (tmh_job_planes_multi_device) or per channel (finalize, "
                        "smooth2, corrector update)")
    p.add_argument("--merge", choices=["batched", "per-channel"], default="batched",
                   help="N > 1 / forced distributed: the channels' merges with one collective per "
                        "quantity for all channels (sharded.merge_*_multi) or per channel")
    p.add_argument("--channel-order", choices=["pipelined", "deep", "serial", "concurrent"],
                   default="pipelined",
                   help="several channels: their Welford passes, then their corrected passes, "
                        "one after another on one pass stream, each channel's merges and planes "
                        "on its own stream under the other channels' passes (pipelined); the "
                        "same with every channel's merge and planes batched between the two "
                        "sweeps (serial); or each channel's passes on its own stream at once "
                        "(concurrent); or job p+1's Welford passes before job p's corrected "
                        "pass, every small step of the jobs in flight under a Welford pass (deep, "
                        "three channel sets: measured slower, DESIGN.md 10.3)")
    p.add_argument("--prefetch-probe", choices=["on", "off"], default="off",
                   help="jobs in flight: queue the next job's reset and site probe right after "
                        "this job's Welford pass (on): its Welford launch then does not wait "
                        "for the probe behind this job's corrected pass (measured 0.5-1%% "
                        "slower, profiles/r5/ab_jobs_order_prefetch_r6j.jsonl)")
    p.add_argument("--pass-launch", choices=["multi", "per-channel"], default="multi",
                   help="several channels, serial or pipelined order: every channel's corrected "
                        "pass in ONE fused launch (tmh_correct_u16_hist_multi_blocks_device) or "
                        "one launch per channel")
    p.add_argument("--fused-bands", type=int, default=None,
                   help="TMH_OPT_FUSED_BANDS: pixel bands of the fused pass (default: automatic)")
    p.add_argument("--channel-streams", choices=["per-channel", "one"], default="per-channel",
                   help="several channels: each on its own stream (its merges overlap the "
                        "others' kernels), or all on one stream")
    p.add_argument("--no-same-workload", action="store_true",
                   help="N > 1: skip rank 0's single-GPU run of the same (unsharded) workload")
    p.add_argument("--pipeline", choices=["fused", "separate"], default="fused",
                   help="fused: histograms built from the correction's read (6 B/px); "
                        "separate: Welford || histogram pass, then correct (8 B/px)")
    p.add_argument("--serial-stats", action="store_true",
                   help="run the histogram pass after Welford instead of concurrently")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the extra (non-headline) measurements: chain pass, host path")
    p.add_argument("--stream-host", action="store_true",
                   help="configs[4]: sites streamed from pinned host memory over PCIe (one JSON "
                        "line of its own; never the HBM headline)")
    p.add_argument("--stream-sites", type=int, default=24576,
                   help="--stream-host: sites per channel (4 plates x 384 wells x 16 sites), "
                        "sharded over the ranks")
    p.add_argument("--stream-channels", type=int, default=5)
    p.add_argument("--resident-gb", type=float, default=160.0,
                   help="--stream-host: HBM for the two in-flight channels' resident sites; a "
                        "channel share beyond half of it is streamed twice (stats, then correct)")
    p.add_argument("--traffic-json", default=None,
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py; "
                        "default profiles/pmc_traffic.json, profiles/pmc_traffic_bright.json for "
                        "--distribution bright)")
    a = p.parse_args()
    if a.traffic_json is None:
        a.traffic_json = os.path.join(REPO, "profiles", "pmc_traffic%s.json" % (
            "" if a.distribution == "synthetic" else "_" + a.distribution))
    return a


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1 only; the oracle is the timed thing here, never
# the GPU path's checker)
# ---------------------------------------------------------------------------

def _cpu_job(args):
    """One channel job of the numpy oracle on a process's own core: per-site
    OnlineStatistics.update (np.percentile with 100,000 q as stats.py:76,
    log10, Welford), smoothing of both planes once, per-site correct."""
    n_sites, H, W, seed, distinct = args
    sys.path.insert(0, REPO)
    from oracle import corilla_oracle as orc
    from tmlibrary_amd.synth import synth_exact_host
    base = [synth_exact_host(H, W, seed, 0, i) for i in range(min(distinct, n_sites))]
    st = orc.OracleOnlineStatistics((H, W), percentile="numpy")  # stats.py:76 as written
    t0 = time.perf_counter()
    for i in range(n_sites):
        st.update(base[i % len(base)])
    t1 = time.perf_counter()
    sm_mean = orc.smooth_reflect(st.mean, 5)
    sm_std = orc.smooth_reflect(st.std, 5)
    t2 = time.perf_counter()
    for i in range(n_sites):
        orc.correct_illumination(base[i % len(base)], sm_mean, sm_std)
    t3 = time.perf_counter()
    return t1 - t0, t2 - t1, t3 - t2


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n_sites, H, W, procs):
    """configs[0] on the host: one process (the reference's cores=1 job,
    workflow/args.py:538-545) over n_sites, plus P processes each running
    its own channel job (the reference's one-job-per-channel parallelism,
    corilla/api.py:64-105).  Both in fresh spawned interpreters."""
    import multiprocessing as mp
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    distinct = 8  # the timing does not depend on which sites repeat
    env_keep = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS")}
    os.environ["OMP_NUM_THREADS"] = os.environ["OPENBLAS_NUM_THREADS"] = "1"
    try:
        ctx = mp.get_context("spawn")
        with ctx.Pool(1) as pool:
            ts, tsm, tc = pool.apply(_cpu_job, ((n_sites, H, W, SEED, distinct),))
        P = max(1, min(procs, cores))
        per = max(1, n_sites // 4)
        with ctx.Pool(P) as pool:
            # concurrent jobs; each times its own job (site generation excluded)
            times = pool.map(_cpu_job, [(per, H, W, SEED + k, distinct) for k in range(P)])
        rate_p = sum(per / sum(t) for t in times)
    finally:
        for k, v in env_keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    job = ts + tsm + tc
    return {
        "value": round(n_sites / job, 4),
        "unit": "sites/s",
        "cores": 1,
        "kind": "port",
        "cpu": cpu_model(),
        "nproc": cores,
        "sample": "configs[0]: one channel job of %d synthetic %dx%d sites (%d distinct, cycled) "
                  "in the numpy oracle, 1 process: OnlineStatistics.update (np.percentile with "
                  "100,000 q, log10, Welford) %.1f ms/site + smoothing of both planes once "
                  "%.2f s + correct_illumination %.1f ms/site"
                  % (n_sites, H, W, distinct, 1e3 * ts / n_sites, tsm, 1e3 * tc / n_sites),
        "multi_process": {"processes": P, "sites_per_process": per,
                          "value": round(rate_p, 4), "unit": "sites/s",
                          "note": "P = min(%d channels, %d cores) processes, one channel job "
                                  "each (the reference's job-level parallelism)" % (procs, cores)},
    }


# ---------------------------------------------------------------------------
# extras beside the headline (N = 1)
# ---------------------------------------------------------------------------

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
    from tmlibrary_amd.synth import synth_exact_host
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    base = [synth_exact_host(H, W, 7, 0, i) for i in range(8)]
    sites = np.ascontiguousarray(np.stack([base[i % 8] for i in range(n_sites)]))
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


def bench_input_path(H, W, dev, distinct=8, block=64, reps=2):
    """§8(f) rank 1 beside the headline: site images from gzip HDF5 files
    (the reference's ChannelImageFile layout: level 4, h5py's own 135 x 160
    chunks, models/file.py h5py_chunk_shape) into HBM -- decoded on the host
    (libhdf5 + zlib on the granted cores) vs inflated on the GPU (compressed
    chunks read by pread, PCIe, tmh_inflate_device + placement), one block at
    a time and as a stream of blocks (the host read of block k+1 under the
    GPU work of block k, as run_job does); the GPU result is checked against
    the host one.  Never the headline."""
    import shutil
    import tempfile

    import torch

    from tmlibrary_amd.models.device_decode import DeviceChunkDecoder
    from tmlibrary_amd.models.file import (default_decode_threads, read_channel_images,
                                           write_channel_image)
    from tmlibrary_amd.synth import synth_exact_host
    d = tempfile.mkdtemp(prefix="tmh_bench_input_")
    try:
        files = []
        for i in range(distinct):
            p = os.path.join(d, "channel_image_file_%d.h5" % i)
            write_channel_image(p, synth_exact_host(H, W, SEED, 0, i), 4)
            files.append(p)
        paths = [files[i % distinct] for i in range(block)]
        nt = default_decode_threads()
        host = np.empty((block, H, W), np.uint16)
        read_channel_images(paths, nt, out=host)
        t_host = 1e30
        for _ in range(reps):
            t0 = time.perf_counter()
            read_channel_images(paths, nt, out=host)
            t_host = min(t_host, time.perf_counter() - t0)
        out = torch.empty((block, H, W), dtype=torch.int16, device=dev)
        dec = DeviceChunkDecoder(device=dev, n_threads=nt)
        dec.decode(paths, out.data_ptr())
        dec.check()
        torch.cuda.synchronize(dev)
        same = bool(np.array_equal(out.cpu().numpy().view(np.uint16), host))
        t_gpu = 1e30
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            dec.decode(paths, out.data_ptr())
            dec.check()
            torch.cuda.synchronize(dev)
            t_gpu = min(t_gpu, time.perf_counter() - t0)
        out2 = torch.empty_like(out)
        n_pipe = 16
        torch.cuda.synchronize(dev)
        dec.times = {k: 0.0 for k in dec.times}
        t0 = time.perf_counter()
        for k in range(n_pipe):
            dec.decode(paths, (out if k % 2 == 0 else out2).data_ptr())
        dec.check()
        torch.cuda.synchronize(dev)
        t_pipe = time.perf_counter() - t0
        host_ms = {k: round(v / n_pipe * 1e3, 1) for k, v in dec.times.items()}
        comp = sum(os.path.getsize(p) for p in paths)
        del out, out2
        from tmlibrary_amd.models.file import h5py_chunk_shape
        return {"workload": "%d gzip HDF5 site files of %dx%d uint16 (%d distinct, cycled; level 4, "
                            "%dx%d chunks) decoded into HBM" % ((block, H, W, distinct)
                                                                + h5py_chunk_shape((H, W), 2)),
                "compressed_MB_per_site": round(comp / block / 1e6, 2),
                "host_threads": nt,
                "host_inflate_sites_per_s": round(block / t_host, 1),
                "gpu_inflate_sites_per_s": round(block / t_gpu, 1),
                "gpu_inflate_stream_sites_per_s": round(n_pipe * block / t_pipe, 1),
                "gpu_inflate_stream_host_ms_per_block": host_ms,
                "gpu_equals_host": same}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def sysfs_clocks(torch, dev):
    """The GPU's current sclk / mclk DPM levels from sysfs (best effort: the
    levels the driver selected, '*' in pp_dpm_*), or the reason they are not
    readable."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        path = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (
            getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id)
    except Exception as e:  # noqa: BLE001 -- report, never fail the line
        return {"error": "%s: %s" % (type(e).__name__, e)}
    out = {"device": path}
    for k in ("sclk", "mclk", "fclk"):
        try:
            with open(os.path.join(path, "pp_dpm_%s" % k)) as f:
                lines = [ln.strip() for ln in f if ln.strip()]
            cur = [ln for ln in lines if ln.endswith("*")]
            out[k] = cur[0].split(":", 1)[1].rstrip("*").strip() if cur else lines
        except OSError as e:
            out[k] = "unreadable (%s)" % e.strerror
    return out


def cu_masked_stream(torch, dev, n_cus):
    """A HIP stream restricted to n_cus of the device's CUs
    (hipExtStreamCreateWithCUMask; the CUs left out spread evenly over the CU
    indices), wrapped for torch.  The mask call goes to the HIP runtime torch
    already loaded (one runtime per process)."""
    total = torch.cuda.get_device_properties(dev).multi_processor_count
    n_cus = max(1, min(int(n_cus), total))
    keep = [True] * total
    drop = total - n_cus
    for j in range(drop):
        keep[(j * total) // drop] = False
    words = [0] * ((total + 31) // 32)
    for i, k in enumerate(keep):
        if k:
            words[i // 32] |= 1 << (i % 32)
    path = None
    with open("/proc/self/maps") as f:
        for ln in f:
            if "libamdhip64.so" in ln:
                path = ln.split()[-1]
                break
    rt = C.CDLL(path or "libamdhip64.so")
    h = C.c_void_p()
    rc = rt.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(len(words)),
                                         (C.c_uint32 * len(words))(*words))
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed (%d)" % rc)
    return torch.cuda.ExternalStream(h.value, device=dev)


def box_probe(L, hip, ch, S, H, W, sp, reps=3):
    """The box's own copy and read rates over the job's buffers (the fused
    pass's 2 + 2 B/px and the Welford pass's 2 B/px; tmh_box_probe_device) in
    two shapes (persistent grid-strided, one thread per 16 B), the shader
    clock measured inside the persistent probe kernel.  The box's rate for a
    pass's bytes is the faster shape's."""
    res = {}
    npx = H * W
    for kind, nbytes, modes in (("copy", 4 * S * npx, (0, 2)), ("read", 2 * S * npx, (1, 3))):
        shapes = {}
        for mode in modes:
            ms, mhz = C.c_double(), C.c_double()
            hip.check(L.tmh_box_probe_device(ch["t_in"], ch["t_out"], ch["shift"], S, H, W, mode,
                                             reps, sp, C.byref(ms), C.byref(mhz)))
            d = {"ms": round(ms.value, 4), "GBs": round(nbytes / (ms.value * 1e-3) / 1e9, 1)}
            if mhz.value > 0:
                d["sclk_mhz_measured"] = round(mhz.value, 1)
            shapes["persistent" if mode < 2 else "flat"] = d
        best = max(shapes.values(), key=lambda d: d["GBs"])
        res[kind] = {"ms": best["ms"], "GBs": best["GBs"], "bytes": nbytes, "shapes": shapes}
    return res


def link_rates(dev, nbytes=2 << 30):
    """Pinned host <-> HBM copy rates on this box (GB/s): H2D alone, D2H alone,
    both at once on two streams -- the PCIe roofline of --stream-host."""
    import torch
    h_in = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def run(h2d, d2h):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_in, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_out.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize(dev)
        return nbytes / (time.perf_counter() - t0) / 1e9

    run(True, True)
    r = {"h2d_GBs": round(max(run(True, False) for _ in range(2)), 1),
         "d2h_GBs": round(max(run(False, True) for _ in range(2)), 1)}
    both = max(run(True, True) for _ in range(2))
    r["duplex_each_way_GBs"] = round(both, 1)
    del h_in, h_out, d_a, d_b
    return r


STREAM_RING = 64   # distinct host sites of --stream-host, cycled
STREAM_CHUNK = 32  # sites per copy / Welford launch
STREAM_STEP = 7    # channel c's global site g is ring site (g + 7 c) % ring


def stream_ring_index(g, c, ring=STREAM_RING):
    """configs[4]'s host input: global site g of channel c is site (g + 7c) %
    ring of the host ring (the generator's sites 0 .. ring-1 of (SEED, channel
    0)); the same on every rank, so results do not depend on the rank count."""
    return (int(g) + STREAM_STEP * int(c)) % int(ring)


class HostStreamJob(object):
    """configs[4] on one rank: every channel's share of sites streamed from a
    pinned host ring (corilla/api.py:69-83 reads them from files one site at a
    time), the sites of one channel job per rank, contiguous in site order.

    A channel share that fits (resident_gb) crosses the link once: streamed in
    (H2D 2 B/px) chunk by chunk with the Welford pass chasing the arrivals,
    kept resident for the fused correct + histogram pass, and the corrected
    sites streamed out (D2H 2 B/px) while the NEXT channel streams in on the
    other copy engine.  Sites beyond the resident budget are streamed twice
    (stats, then correct).  Two statistics handles alternate between
    channels; each channel's results (mean, std, percentile sums, pooled
    histogram, smoothed planes) are copied to device buffers of its own at the
    end of its job, on its stream, so a caller can check every channel without
    stalling the pipeline; ``keep`` = {(channel, global site)} also keeps
    those sites' corrected planes."""

    def __init__(self, L, dev, H, W, S_total, world=1, rank=0, resident_gb=160.0,
                 ring=STREAM_RING, chunk=STREAM_CHUNK, dist=None, keep=(), seed=SEED):
        import torch

        from tmlibrary_amd import hip
        from tmlibrary_amd.image import ZERO_LOG10
        from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
        from tmlibrary_amd.workflow.corilla.sharded import StatsOps, shard_bounds
        self.torch, self.hip, self.L, self.dev = torch, hip, L, dev
        self.H, self.W, self.npx = H, W, H * W
        self.S_total, self.world, self.rank, self.dist = S_total, world, rank, dist
        self.ring, self.CK = ring, chunk
        self.s_begin, self.s_end = shard_bounds(S_total, world, rank)
        self.S = self.s_end - self.s_begin
        site_b = self.npx * 2
        self.R = min(self.S, int(resident_gb * 1e9 / 2 / site_b) // chunk * chunk)
        Q = 100000
        CK = chunk
        # the host ring: the generator's sites 0 .. ring-1, pinned
        self.h_ring = torch.empty((ring, H, W), dtype=torch.int16, pin_memory=True)
        tmp = torch.empty((ring, H, W), dtype=torch.int16, device=dev)
        hip.check(L.tmh_synth_sites_device(C.c_void_p(tmp.data_ptr()), ring, H, W, seed, 0, 0,
                                           hip.TMH_SYNTH_STANDARD, None))
        self.h_ring.copy_(tmp)
        del tmp
        self.h_out = torch.empty((4, CK, H, W), dtype=torch.int16, pin_memory=True)
        self.resident = [torch.empty((max(self.R, 1), H, W), dtype=torch.int16, device=dev)
                         for _ in range(2)]
        self.stage = [torch.empty((CK, H, W), dtype=torch.int16, device=dev) for _ in range(2)]
        self.d_out = [torch.empty((CK, H, W), dtype=torch.int16, device=dev) for _ in range(4)]
        self.s_h2d, self.s_d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        self.comp = [torch.cuda.Stream(dev) for _ in range(2)]
        lo, hi, gamma = quantile_table(self.npx, np.linspace(0, 100, Q))
        lut = stats_log10_lut()
        flags = hip.TMH_STATS_DEFERRED_PCT if dist is not None else 0
        self.handles = []
        for b in range(2):
            h, corr = C.c_void_p(), C.c_void_p()
            hip.check(L.tmh_stats_create(H, W, Q, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                         hip.ptr(lut), 1, flags, C.byref(h)))
            sp = C.c_void_p(self.comp[b].cuda_stream)
            hip.check(L.tmh_stats_set_stream(h, sp))
            planes = [torch.empty(self.npx, dtype=torch.float64, device=dev) for _ in range(6)]
            torch.cuda.synchronize(dev)
            hip.check(L.tmh_corrector_create_device(C.c_void_p(planes[0].data_ptr()),
                                                    C.c_void_p(planes[1].data_ptr()), H, W, 1,
                                                    ZERO_LOG10, sp, C.byref(corr)))
            self.handles.append((h, corr, sp, planes, StatsOps(L, h, self.npx, Q, dev)))
        self.keep = set((int(c), int(g)) for c, g in keep)
        self.kept = {}   # (channel, global site) -> device plane
        self.res = {}    # channel -> device result buffers
        self.reset_state()
        self.marks = []  # (channel, phase, timing event)
        self.host_t = {}

    def reset_state(self):
        self.state = {"buf_free": [None, None], "stage_free": [None, None],
                      "out_free": [None] * 4, "k_in": 0, "k_out": 0}

    def _record(self, stream, timing=False):
        e = self.torch.cuda.Event(enable_timing=timing)
        e.record(stream)
        return e

    def mark(self, c, phase, stream):
        self.marks.append((c, phase, self._record(stream, True)))
        self.host_t.setdefault("c%d" % c, {})["enq_" + phase] = time.perf_counter()

    def h2d(self, dst, g0, n, c):
        """global sites g0 .. g0+n-1 of channel c from the host ring into dst
        (contiguous runs of the ring; on the H2D engine)"""
        torch = self.torch
        i = 0
        with torch.cuda.stream(self.s_h2d):
            while i < n:
                k = stream_ring_index(g0 + i, c, self.ring)
                m = min(n - i, self.ring - k)
                dst[i:i + m].copy_(self.h_ring[k:k + m], non_blocking=True)
                i += m
        return self._record(self.s_h2d)

    def channel(self, c):
        torch, hip, L = self.torch, self.hip, self.L
        from tmlibrary_amd.workflow.corilla.sharded import merge_counts, merge_welford
        H, W, CK, S, R = self.H, self.W, self.CK, self.S, self.R
        st = self.state
        b = c % 2
        h, corr, sp, planes, ops = self.handles[b]
        cs = self.comp[b]
        mean, std, smean, sstd, ptmp, ptmp2 = planes
        buf = self.resident[b]
        ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        if st["buf_free"][b] is not None:
            self.s_h2d.wait_event(st["buf_free"][b])
        hip.check(L.tmh_stats_reset(h))
        nch = (S + CK - 1) // CK
        self.mark(c, "h2d_begin", self.s_h2d)
        for j in range(nch):  # pass 1: arrivals -> Welford
            n = min(CK, S - j * CK)
            g0 = self.s_begin + j * CK
            if j * CK < R:
                dst = buf[j * CK:j * CK + n]
            else:
                k = st["k_in"] % 2
                st["k_in"] += 1
                if st["stage_free"][k] is not None:
                    self.s_h2d.wait_event(st["stage_free"][k])
                dst = self.stage[k][:n]
            cs.wait_event(self.h2d(dst, g0, n, c))
            hip.check(L.tmh_stats_update_welford_device(h, ptr(dst), n, 1, sp))
            if j * CK >= R:
                st["stage_free"][k] = self._record(cs)
        self.mark(c, "h2d_end", self.s_h2d)
        with torch.cuda.stream(cs):
            if self.dist is not None:
                merge_welford(ops, self.dist, n_total=self.S_total)
            hip.check(L.tmh_stats_finalize_device(h, ptr(mean), ptr(std), sp))
            hip.check(L.tmh_smooth2_f64_device(ptr(mean), ptr(std), ptr(smean), ptr(sstd),
                                               ptr(ptmp), ptr(ptmp2), H, W, 5.0, sp))
            hip.check(L.tmh_corrector_update_device(corr, ptr(smean), ptr(sstd), sp))
        for j in range(nch):  # pass 2: correct + histogram -> out slots -> host
            n = min(CK, S - j * CK)
            g0 = self.s_begin + j * CK
            if j * CK < R:
                src = buf[j * CK:j * CK + n]
            else:
                k = st["k_in"] % 2
                st["k_in"] += 1
                if st["stage_free"][k] is not None:
                    self.s_h2d.wait_event(st["stage_free"][k])
                src = self.stage[k][:n]
                cs.wait_event(self.h2d(src, g0, n, c))
            o = st["k_out"] % 4
            st["k_out"] += 1
            if st["out_free"][o] is not None:
                cs.wait_event(st["out_free"][o])
            hip.check(L.tmh_correct_u16_hist_device(corr, h, ptr(src), ptr(self.d_out[o]), n, -1,
                                                    -1, sp))
            with torch.cuda.stream(cs):  # corrected planes kept for a check
                for g in range(g0, g0 + n):
                    if (c, g) in self.keep:
                        self.kept[(c, g)] = self.d_out[o][g - g0].clone()
            e = self._record(cs)
            if j * CK >= R:
                st["stage_free"][k] = e
            self.s_d2h.wait_event(e)
            with torch.cuda.stream(self.s_d2h):
                self.h_out[o][:n].copy_(self.d_out[o][:n], non_blocking=True)
            st["out_free"][o] = self._record(self.s_d2h)
        self.mark(c, "d2h_end", self.s_d2h)
        with torch.cuda.stream(cs):
            if self.dist is not None:
                merge_counts(ops, self.dist)
            # the channel's results, before the handle serves channel c + 2
            r = self.res.get(c)
            if r is None:
                r = self.res[c] = {k: torch.empty(self.npx, dtype=torch.float64, device=self.dev)
                                   for k in ("mean", "std", "smean", "sstd")}
                r["acc"] = torch.empty(100000, dtype=torch.float64, device=self.dev)
                r["hist"] = torch.empty(65536, dtype=torch.int64, device=self.dev)
            for k, t in (("mean", mean), ("std", std), ("smean", smean), ("sstd", sstd)):
                r[k].copy_(t)
            hip.check(L.tmh_stats_get_pct_sum_device(h, ptr(r["acc"]), sp))
            hip.check(L.tmh_stats_get_hist_device(h, ptr(r["hist"]), sp))
        st["buf_free"][b] = self._record(cs)

    def results(self, c):
        """channel c's results on the host (synchronises)"""
        self.torch.cuda.synchronize(self.dev)
        r = self.res[c]
        out = {k: r[k].cpu().numpy() for k in ("mean", "std", "smean", "sstd", "acc")}
        out["hist"] = r["hist"].cpu().numpy().astype(np.uint64)
        out["n"] = self.S_total
        out["kept"] = {g: t.cpu().numpy().view(np.uint16)
                       for (cc, g), t in self.kept.items() if cc == c}
        return out

    def close(self):
        self.torch.cuda.synchronize(self.dev)
        for h, corr, *_ in self.handles:
            self.L.tmh_corrector_destroy(corr)
            self.L.tmh_stats_destroy(h)
        self.handles = []


def stream_fingerprint_name(H, W, S, CH, ring):
    return "stream_fp_%dx%d_s%d_ch%d_ring%d_seed%d.npz" % (H, W, S, CH, ring, SEED)


def check_stream_channel(fp, c, res):
    """One channel of --stream-host against the committed oracle fingerprint
    (tests/golden/make_stream_fingerprint.py): n, percentile sums and pooled
    histogram bit-exact, mean/std at the sampled pixels within 1e-6."""
    sp = fp["stat_px"]
    return {
        "n": int(res["n"]) == int(fp["n"]),
        "pct_sums_bit_exact": hashlib.sha256(res["acc"].tobytes()).hexdigest() ==
        str(fp["pct_sums_sha256"][c]),
        "hist_bit_exact": hashlib.sha256(res["hist"].tobytes()).hexdigest() ==
        str(fp["hist_sha256"][c]),
        "mean_1e-6": _close(res["mean"][sp], fp["mean_samples"][c]),
        "std_1e-6": _close(res["std"][sp], fp["std_samples"][c]),
    }


def bench_stream_host(a, world, rank, local_rank, dist_on):
    """configs[4]: a multi-plate batch (4 plates x 384 wells x 16 sites = 24,576
    sites per channel, 5 channels) that does not live in HBM: HostStreamJob
    on every rank, timed over all channels (PCIe-bound: never the headline)."""
    import torch
    import torch.distributed as dist

    from tmlibrary_amd import hip
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if dist_on:
        import datetime
        Heartbeat(rank)("init_process_group")
        dist.init_process_group("nccl", device_id=dev,
                                timeout=datetime.timedelta(seconds=a.coll_timeout))
    H, W = a.height, a.width
    site_b = H * W * 2
    CH = a.stream_channels
    S_total = a.stream_sites
    L = hip.lib()
    hip.check(L.tmh_set_device(local_rank))
    log("stream-host: link test")
    link = link_rates(dev)
    log("link: %s" % link)
    job = HostStreamJob(L, dev, H, W, S_total, world, rank, a.resident_gb,
                        dist=dist if dist_on else None)
    log("stream-host: %d channels x %d sites/rank (%d resident, %d streamed twice); warm-up"
        % (CH, job.S, job.R, job.S - job.R))
    job.channel(0)
    job.channel(1)
    torch.cuda.synchronize(dev)
    job.reset_state()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    log("stream-host: timing %d channels" % CH)
    job.marks.clear()
    job.host_t.clear()
    t0 = time.perf_counter()
    for c in range(CH):
        job.channel(c)
    torch.cuda.synchronize(dev)
    timeline = {}
    if job.marks:
        e0 = job.marks[0][2]
        for c, phase, e in job.marks:
            timeline.setdefault("c%d" % c, {})[phase] = round(e0.elapsed_time(e), 1)
        for c, d in job.host_t.items():  # host enqueue times, same origin (approximately)
            for k, v in d.items():
                timeline[c][k] = round(1e3 * (v - t0), 1)
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # every channel's results against the oracle fingerprint of the same input
    path = os.path.join(REPO, "tests", "golden",
                        stream_fingerprint_name(H, W, S_total, CH, job.ring))
    checks, check_ok = {}, None
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as z:
            fp = {k: z[k] for k in z.files}
        for c in range(CH):
            checks["c%d" % c] = check_stream_channel(fp, c, job.results(c))
        check_ok = all(all(v.values()) for v in checks.values())
    job.close()
    if dist_on:
        dist.destroy_process_group()
    if rank != 0:
        return None
    sites_done = CH * S_total
    R_all = job.R * world
    h2d_b = CH * (S_total * site_b + (S_total - min(S_total, R_all)) * site_b)
    d2h_b = CH * S_total * site_b
    per_link = elapsed * world
    return {
        "metric": "sites/sec (2160x2560 uint16) illumstats+correct streamed from host (PCIe-bound)",
        "value": round(sites_done / elapsed, 1), "unit": "sites/s", "n_gpus": world,
        "ms_total": round(1e3 * elapsed, 1), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64 stats / f32 correct (±1 DN)",
        "data": "synthetic, %d distinct sites in a pinned host ring, cycled (channel c's site g "
                "is ring site (g + 7c) %% %d)" % (job.ring, job.ring),
        "config": {"workload": "configs[4]: %d channels x %d sites (4 plates x 384 wells x 16 "
                               "sites) of %dx%d uint16 streamed from host, sharded over %d GPU(s)"
                               % (CH, S_total, H, W, world),
                   "resident_sites_per_channel_per_gpu": job.R,
                   "sites_per_channel_per_gpu": job.S, "chunk_sites": job.CK},
        "pcie": {"h2d_bytes": h2d_b, "d2h_bytes": d2h_b,
                 "h2d_GBs_per_gpu": round(h2d_b / per_link / 1e9, 1),
                 "d2h_GBs_per_gpu": round(d2h_b / per_link / 1e9, 1),
                 "link": link,
                 "frac_of_duplex_link": round(max(h2d_b, d2h_b) / per_link / 1e9 /
                                              link["duplex_each_way_GBs"], 4)},
        "timeline_ms": timeline,
        "check": checks,
        "check_vs_oracle": check_ok,
        "fingerprint": os.path.relpath(path, REPO) if check_ok is not None else None,
    }


# ---------------------------------------------------------------------------
# oracle fingerprint check
# ---------------------------------------------------------------------------

def fingerprint_name(H, W, S, seed, channel, distribution):
    """File (under tests/golden/) of the oracle fingerprint for one channel
    job; written by tests/golden/make_bench_fingerprint.py."""
    return "bench_fp_%dx%d_s%d_seed%d_c%d_%s.npz" % (H, W, S, seed, channel, distribution)


def load_fingerprint(H, W, S_total, distribution, channel=0):
    path = os.path.join(REPO, "tests", "golden",
                        fingerprint_name(H, W, S_total, SEED, channel, distribution))
    if not os.path.exists(path):
        return None, path
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}, path


def _close(got, want, rtol=1e-6, atol=1e-9):
    return bool(np.all(np.abs(got - want) <= atol + rtol * np.abs(want)))


def check_against_fingerprint(fp, res, smean, sstd, corr_sites):
    """This rank's view of the channel-0 job vs the oracle fingerprint.
    corr_sites: {global site index: corrected uint16 plane} for the
    fingerprint's sampled sites that this rank holds."""
    sp = fp["stat_px"]
    out = {
        "n": int(res["n"]) == int(fp["n"]),
        "pct_sums_bit_exact": hashlib.sha256(res["acc"].tobytes()).hexdigest() ==
        str(fp["pct_sums_sha256"]),
        "hist_bit_exact": hashlib.sha256(res["hist"].tobytes()).hexdigest() ==
        str(fp["hist_sha256"]),
        "mean_1e-6": _close(res["mean"].ravel()[sp], fp["mean_samples"]),
        "std_1e-6": _close(res["std"].ravel()[sp], fp["std_samples"]),
        "smoothed_1e-6": _close(smean[sp], fp["smean_samples"]) and
        _close(sstd[sp], fp["sstd_samples"]),
    }
    cnt = np.zeros(5, dtype=np.int64)  # equal, +1, -1, |d| > 1, wrap flips
    for k, s in enumerate(fp["corr_sites"].tolist()):
        if s not in corr_sites:
            continue
        got = corr_sites[s].ravel()[fp["corr_px"]].astype(np.int64)
        d = got - fp["corr_samples"][k].astype(np.int64)
        flips = np.abs(d) == 65535
        cnt += [np.count_nonzero(d == 0), np.count_nonzero(d == 1), np.count_nonzero(d == -1),
                np.count_nonzero((np.abs(d) > 1) & ~flips), np.count_nonzero(flips)]
    return out, cnt


# ---------------------------------------------------------------------------
# multi-GPU cost model
# ---------------------------------------------------------------------------

class CollectiveTimer(object):
    """``timer(name)`` context for sharded.merge_*: synchronises the device
    before the collective (so no kernel of any stream is in flight), then
    brackets it with events on torch's current stream -- each collective's own
    time, including the wait for its peers, isolated from the kernels."""

    def __init__(self, torch, dev):
        self.torch, self.dev = torch, dev
        self.events = []
        self._name = None

    def __call__(self, name):
        self._name = name
        return self

    def __enter__(self):
        self.torch.cuda.synchronize(self.dev)
        self._a = self.torch.cuda.Event(enable_timing=True)
        self._a.record(self.torch.cuda.current_stream(self.dev))
        return self

    def __exit__(self, *exc):
        b = self.torch.cuda.Event(enable_timing=True)
        b.record(self.torch.cuda.current_stream(self.dev))
        self.events.append((self._name, self._a, b))
        return False

    def summary(self):
        self.torch.cuda.synchronize(self.dev)
        out = {}
        for name, a, b in self.events:
            d = out.setdefault(name, {"calls": 0, "total_ms": 0.0})
            d["calls"] += 1
            d["total_ms"] += a.elapsed_time(b)
        for d in out.values():
            d["mean_ms"] = round(d["total_ms"] / d["calls"], 4)
            d["total_ms"] = round(d["total_ms"], 4)
        return out


def single_gpu_same_workload(L, dev, H, W, CH, S_total, dist_id, steps=3, warmup=1, B=64):
    """configs[2]/[3] on ONE GPU: the CH channel jobs of S_total sites that an
    N > 1 run shards over its ranks, run here one after another on one stream
    -- every channel's sites resident in B-site blocks, one set of output
    blocks reused by every channel (CH x 2 x 38 GB would not fit) -- the
    like-for-like N = 1 point of the strong-scaling curve."""
    import torch

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    npx = H * W
    shift = B.bit_length() - 1
    stream = torch.cuda.Stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    ins, outs = [], []
    for c in range(CH):
        blk = []
        for b0 in range(0, S_total, B):
            m = min(B, S_total - b0)
            blk.append(torch.empty((m, H, W), dtype=torch.int16, device=dev))
            if c == 0:
                outs.append(torch.empty((m, H, W), dtype=torch.int16, device=dev))
            hip.check(L.tmh_synth_sites_device(ptr(blk[-1]), m, H, W, SEED, c, b0, dist_id, sp))
        ins.append(blk)
    t_in = [torch.tensor([t.data_ptr() for t in blk], dtype=torch.int64, device=dev) for blk in ins]
    t_out = torch.tensor([t.data_ptr() for t in outs], dtype=torch.int64, device=dev)
    lo, hi, gamma = quantile_table(npx, np.linspace(0, 100, 100000))
    lut = stats_log10_lut()
    h, corr = C.c_void_p(), C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, 100000, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 1, 0, C.byref(h)))
    hip.check(L.tmh_stats_set_stream(h, sp))
    mean, std, smean, sstd, tmp, tmp2 = [torch.empty(npx, dtype=torch.float64, device=dev)
                                         for _ in range(6)]
    torch.cuda.synchronize(dev)
    hip.check(L.tmh_corrector_create_device(ptr(mean), ptr(std), H, W, 1, ZERO_LOG10, sp,
                                            C.byref(corr)))

    def job(c):
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_blocks_device(h, ptr(t_in[c]), shift, S_total, 1, sp))
        hip.check(L.tmh_stats_finalize_device(h, ptr(mean), ptr(std), sp))
        hip.check(L.tmh_smooth2_f64_device(ptr(mean), ptr(std), ptr(smean), ptr(sstd), ptr(tmp),
                                           ptr(tmp2), H, W, 5.0, sp))
        hip.check(L.tmh_corrector_update_device(corr, ptr(smean), ptr(sstd), sp))
        hip.check(L.tmh_correct_u16_hist_blocks_device(corr, h, ptr(t_in[c]), ptr(t_out), shift,
                                                       S_total, -1, -1, sp))

    for _ in range(warmup):
        for c in range(CH):
            job(c)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        for c in range(CH):
            job(c)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    L.tmh_corrector_destroy(corr)
    L.tmh_stats_destroy(h)
    del ins, outs, t_in, t_out
    torch.cuda.empty_cache()
    return {"workload": "%d channels x %d sites of %dx%d uint16 on one GPU, channel jobs one "
                        "after another (the N > 1 workload unsharded)" % (CH, S_total, H, W),
            "value": round(CH * S_total * steps / el, 1), "unit": "sites/s",
            "ms_per_step": round(1e3 * el / steps, 3), "steps": steps}


# ---------------------------------------------------------------------------

def claim_stdout():
    """The one JSON line keeps stdout; everything else written to fd 1 (RCCL's
    version banner, library prints) goes to stderr."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


class Heartbeat(object):
    """A rank's progress for the launcher (``bench.py --gpus N``): the stage it
    is in -- "init_process_group", "step 3", "all_reduce #41 (step 3)" -- one
    line per stage to the file $TMH_BENCH_HEARTBEAT names (rewritten each
    time; the launcher reads it and its mtime) and, for collectives and
    phases, to stderr.  Inactive without that variable (a plain one-rank run
    prints nothing more)."""

    def __init__(self, rank):
        self.rank = rank
        self.path = os.environ.get("TMH_BENCH_HEARTBEAT")
        self.n = 0
        self.step = ""

    def __call__(self, stage, echo=True):
        if not self.path:
            return
        line = "%.3f %s%s" % (time.time(), stage, self.step)
        with open(self.path, "w") as f:
            f.write(line + "\n")
        if echo:
            log("[rank %d] %s%s" % (self.rank, stage, self.step))


class BeatingDist(object):
    """The collectives' module with a heartbeat before every collective call:
    a rank that never returns from one is named with it by the launcher."""

    COLLECTIVES = ("all_reduce", "broadcast", "send", "recv", "barrier", "all_gather",
                   "all_gather_object", "reduce_scatter")

    def __init__(self, d, beat):
        self._d = d
        self._beat = beat

    def __getattr__(self, name):
        f = getattr(self._d, name)
        if name not in self.COLLECTIVES or not callable(f):
            return f
        beat = self._beat

        def call(*args, **kw):
            beat.n += 1
            beat("%s #%d" % (name, beat.n), echo=False)
            return f(*args, **kw)
        return call


def read_heartbeats(paths):
    """{rank: (seconds since the beat, stage)} from the ranks' heartbeat files."""
    now = time.time()
    out = {}
    for r, p in enumerate(paths):
        try:
            with open(p) as f:
                t, _, stage = f.read().strip().partition(" ")
            out[r] = (now - float(t), stage)
        except (OSError, ValueError):
            out[r] = (None, "no heartbeat yet")
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(a, argv):
    """``bench.py --gpus N`` without WORLD_SIZE: start N rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as
    torchrun sets them) BEFORE anything touches the GPU, forward rank 0's JSON
    line, and exit non-zero if any rank fails.  The parent never initialises
    HIP (torch.cuda.device_count() does not, on this image) and never execs:
    the ranks are child processes.  Returns the exit code."""
    import signal
    import subprocess
    N = a.gpus
    if not a.dry_run:
        import torch
        have = torch.cuda.device_count()
        need = 1 if a.share_gpu else N
        if have < need:
            log("--gpus %d needs %d visible GPU(s), found %d (one process per GPU; "
                "--share-gpu runs parity ranks on one GPU)" % (N, need, have))
            return 2
    import shutil
    import tempfile
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    hb_dir = tempfile.mkdtemp(prefix="tmh_bench_hb_")
    hb = [os.path.join(hb_dir, "rank%d" % r) for r in range(N)]
    procs = []
    for r in range(N):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(0 if a.share_gpu else r),
                   WORLD_SIZE=str(N), LOCAL_WORLD_SIZE=str(N), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, TMH_BENCH_LAUNCHED="1", TMH_BENCH_HEARTBEAT=hb[r])
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))
    import threading
    buf = []
    reader = threading.Thread(target=lambda: buf.append(procs[0].stdout.read()), daemon=True)
    reader.start()  # rank 0's stdout, while the ranks are watched below
    rcs = [None] * N
    failed = None  # exit code of the first rank seen failing (the cause)
    why = None
    t_start = time.time()
    while any(rc is None for rc in rcs):
        for r, pr in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = pr.poll()
                if rcs[r] not in (None, 0) and failed is None:
                    failed = rcs[r]
                    why = "rank %d exited with %d" % (r, rcs[r])
        if failed is not None:
            break
        now = time.time()
        if now - t_start > a.deadline:
            failed, why = 3, "deadline of %.0f s passed" % a.deadline
            break
        beats = read_heartbeats(hb)
        ages = [b[0] for b in beats.values() if b[0] is not None]
        newest = min(ages) if ages else now - t_start
        if newest > a.stall_timeout:  # no rank has moved: every one is stuck
            failed, why = 3, "no rank made progress for %.0f s" % newest
            break
        time.sleep(0.2)
    if failed is not None:  # a rank died or hangs: the others would wait forever in a collective
        beats = read_heartbeats(hb)
        log("launcher: %s; killing the ranks.  Last stage of each rank:" % why)
        for r in range(N):
            age, stage = beats[r]
            state = "running" if procs[r].poll() is None else "exited %s" % procs[r].poll()
            log("  rank %d (%s): %s%s" % (r, state, stage,
                                         "" if age is None else " (%.1f s ago)" % age))
        for r, pr in enumerate(procs):
            if pr.poll() is None:
                os.killpg(pr.pid, signal.SIGTERM)
        for r, pr in enumerate(procs):
            try:
                rcs[r] = pr.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(pr.pid, signal.SIGKILL)
                rcs[r] = pr.wait()
        log("rank exit codes: %s" % rcs)
        shutil.rmtree(hb_dir, ignore_errors=True)
        return failed if 0 < failed < 256 else 1
    shutil.rmtree(hb_dir, ignore_errors=True)
    reader.join(timeout=30)
    out0 = buf[0].decode(errors="replace") if buf else ""
    lines = [ln for ln in out0.splitlines() if ln.strip().startswith("{")]
    if not lines:
        log("rank 0 printed no JSON line")
        return 1
    print(lines[-1], flush=True)
    return 0


def dry_run(world, rank, a):
    """--dry-run rank body: a gloo group, one all_reduce, and the ranks' launch
    environment.  Launcher tests: TMH_BENCH_DRY_FAIL_RANK=r makes rank r die,
    TMH_BENCH_DRY_STALL_RANK=r makes rank r hang before the all_reduce (the
    others then wait inside it)."""
    import datetime

    import torch
    import torch.distributed as dist
    beat = Heartbeat(rank)
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
    if os.environ.get("TMH_BENCH_DRY_FAIL_RANK") == str(rank):  # launcher test: a rank dies
        sys.exit(3)
    beat("init_process_group")
    if world == 1:  # a lone rank needs no launcher's rendezvous address
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=a.coll_timeout))
    D = BeatingDist(dist, beat)
    if os.environ.get("TMH_BENCH_DRY_STALL_RANK") == str(rank):
        beat("stalled on purpose (launcher test)")
        time.sleep(3600)
    t = torch.ones(1)
    D.all_reduce(t)
    envs = [None] * world
    D.all_gather_object(envs, {k: os.environ.get(k) for k in keys})
    ws = dist.get_world_size()
    merges = rehearse_merges(a, world, rank, D, torch) if world > 1 else None
    beat("done")
    dist.destroy_process_group()
    if rank == 0:
        r = {"dry_run": True, "n_gpus": world, "world_size": ws, "ranks": envs}
        if merges is not None:
            r["merges"] = merges
        return r
    return None


class DryOps(object):
    """Synthetic per-rank state for the dry run's merge rehearsal (no
    statistics are computed): channel c's local site i contributes the
    percentile vector p(c, i) below, its Welford state and histogram are
    seeded by (c, rank).  Same interface as sharded.StatsOps, on CPU tensors,
    so the dry run moves the real collectives' shapes through the real
    sequencing code (sharded.merge_*)."""

    def __init__(self, torch, c, rank, world, S_total, npx, Q):
        from tmlibrary_amd.workflow.corilla.sharded import shard_bounds
        self.torch, self.c, self.Q = torch, c, Q
        self.a, self.b = shard_bounds(S_total, world, rank)
        rng = np.random.default_rng([c, rank])
        self.n = self.b - self.a
        self.mean = torch.from_numpy(rng.random(npx) * 4.0)
        self.m2 = torch.from_numpy(rng.random(npx) * self.n)
        self.hist = torch.from_numpy(rng.integers(0, 1000, 65536).astype(np.int64))
        self.acc = None
        self.device = "cpu"

    @staticmethod
    def pcts(c, i, q0, qn):
        """site i's synthetic percentiles [q0, q0 + qn): inexact products, so a
        reassociated sum differs in its last bits"""
        q = np.arange(q0, q0 + qn, dtype=np.int64)
        return ((q * 40503 + i * 2654435761 + c * 97) % 65536).astype(np.float64) * 1.0000001

    def n_local(self):
        return self.n

    def empty_plane(self):
        return self.torch.empty(self.mean.numel(), dtype=self.torch.float64)

    def empty_acc(self):
        return self.torch.zeros(self.Q, dtype=self.torch.float64)

    def stage1(self, buf):
        buf.copy_(self.n * self.mean)

    def stage2(self, sum_nmean, n_total, m2c):
        mu = sum_nmean / n_total
        d = self.mean - mu
        m2c.copy_(self.m2 + self.n * d * d)
        self.mean = mu.clone()

    def stage3(self, n_total, sum_m2c):
        self.m2, self.n = sum_m2c.clone(), n_total

    def pct_accumulate_range(self, part, q0, qn):
        acc = part.numpy().copy()
        for i in range(self.a, self.b):  # the rank's sites in order
            acc += self.pcts(self.c, i, q0, qn)
        part.copy_(self.torch.from_numpy(acc))

    def pct_accumulate(self, acc):
        self.pct_accumulate_range(acc, 0, self.Q)

    def set_pct_sum(self, acc):
        self.acc = acc.clone()

    def empty_hist(self):
        return self.torch.empty(65536, dtype=self.torch.int64)

    def get_hist(self, buf):
        buf.copy_(self.hist)

    def set_hist(self, buf):
        self.hist = buf.clone()


def rehearse_merges(a, world, rank, D, torch):
    """The N > 1 bench's exchange at its own geometry, on CPU (gloo): every
    channel's sites sharded over the ranks, the Welford all-reduce merges, the
    pipelined ordered percentile chain (chain_chunks(Q, N) chunks, N hops) and
    the histogram all-reduce, in the order --channel-order / --merge give the
    GPU run (per-channel merges for the default pipelined order, one batched
    collective per quantity for 'deep' / --merge batched); rank 0 then checks
    every channel against the sequential result (site-order sum bit for bit,
    pooled Welford and histogram)."""
    from tmlibrary_amd.workflow.corilla.sharded import (chain_chunks, merge_counts,
                                                         merge_counts_multi, merge_welford,
                                                         merge_welford_multi, shard_bounds)
    CH = a.channels if a.channels else 4
    S_total, Q, npx = a.sites, 100000, a.height * a.width
    batched = a.channel_order == "deep" or (a.channel_order != "pipelined" and a.merge == "batched")
    ops = [DryOps(torch, c, rank, world, S_total, npx, Q) for c in range(CH)]
    if batched:
        merge_welford_multi(ops, D, n_totals=[S_total] * CH)
        merge_counts_multi(ops, D)
    else:
        for o in ops:
            merge_welford(o, D, n_total=S_total)
        for o in ops:
            merge_counts(o, D)
    if rank != 0:
        return None
    out = {"channels": CH, "sites_per_channel": S_total, "height": a.height, "width": a.width,
           "n_quantiles": Q, "chain_chunks": len(chain_chunks(Q, world)),
           "merge": "batched" if batched else "per-channel", "check": {}}
    for c, o in enumerate(ops):
        want_acc = np.zeros(Q)
        for i in range(S_total):  # the reference's sequential += in site order
            want_acc += DryOps.pcts(c, i, 0, Q)
        parts = [DryOps(torch, c, r, world, S_total, npx, Q) for r in range(world)]
        n = sum(p.n for p in parts)
        mean = sum(p.n * p.mean for p in parts) / n
        m2 = sum(p.m2 + p.n * (p.mean - mean) ** 2 for p in parts)
        hist = sum(p.hist for p in parts)
        out["check"]["c%d" % c] = {
            "sites_per_rank": [shard_bounds(S_total, world, r)[1] - shard_bounds(S_total, world, r)[0]
                               for r in range(world)],
            "pct_sum_bit_exact": bool(np.array_equal(o.acc.numpy(), want_acc)),
            "welford_close": bool(torch.allclose(o.mean, mean, rtol=1e-12, atol=0) and
                                  torch.allclose(o.m2, m2, rtol=1e-12, atol=0) and o.n == n),
            "hist_equal": bool(torch.equal(o.hist, hist))}
    out["ok"] = all(all(v for k, v in d.items() if k != "sites_per_rank")
                    for d in out["check"].values())
    return out


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and a.gpus is not None and a.gpus != int(env_world):
        log("--gpus %d disagrees with WORLD_SIZE=%s" % (a.gpus, env_world))
        sys.exit(2)
    if env_world is None and (a.gpus or 1) > 1:
        sys.exit(launch(a, sys.argv[1:]))
    out = claim_stdout()
    if a.dry_run:
        r = dry_run(int(env_world or 1), int(os.environ.get("RANK", "0")), a)
        if r is not None:
            print(json.dumps(r), file=out, flush=True)
        return
    if a.stream_host:
        # HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 on the
        # box) round-robin; with the copy, compute and library streams of the
        # host pipeline that put the next channel's H2D behind the current
        # channel's kernels (profiles/r3/stream_host_hwq_r3t.jsonl: 2,988 sites/s
        # with 4, 3,408 with 8).  The resident multi-channel job runs best with
        # 4 (dist4_hwq_r3u.jsonl), so only this mode changes it, before HIP starts.
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.stream_host:
        r = bench_stream_host(a, world, rank, local_rank,
                              world > 1 or os.environ.get("TMH_BENCH_FORCE_DIST") == "1")
        if r is not None:
            print(json.dumps(r), file=out, flush=True)
        return
    H, W = a.height, a.width
    npx = H * W
    Q = 100000

    cpu = None
    if world == 1 and a.cpu_sample > 0:  # before the GPU is touched: nothing competes
        log("CPU baseline: %d sites, 1 process + %d processes" % (a.cpu_sample, a.cpu_procs))
        cpu = cpu_baseline(a.cpu_sample, H, W, a.cpu_procs)
        log("CPU baseline: %.3f sites/s" % cpu["value"])

    import torch
    import torch.distributed as dist

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.synth import DISTRIBUTIONS
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    from tmlibrary_amd.workflow.corilla.sharded import (StatsOps, merge_counts,
                                                         merge_counts_multi, merge_welford,
                                                         merge_welford_multi, shard_bounds)

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    clocks_start = sysfs_clocks(torch, dev)
    # TMH_BENCH_FORCE_DIST=1 runs the multi-GPU code path (RCCL merges,
    # deferred percentiles, pipelined chain) even with one rank
    dist_on = world > 1 or os.environ.get("TMH_BENCH_FORCE_DIST") == "1"
    D = dist  # the collectives' module: RCCL, or gloo staged through host memory
    staged = a.share_gpu and world > 1
    beat = Heartbeat(rank)
    if dist_on:
        import datetime
        tmo = datetime.timedelta(seconds=a.coll_timeout)
        beat("init_process_group")
        if staged:  # parity runs: N ranks on one GPU (RCCL needs a GPU per rank)
            from tmlibrary_amd.workflow.corilla.sharded import HostStagedDist
            dist.init_process_group("gloo", timeout=tmo)
            D = HostStagedDist(dist)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        D = BeatingDist(D, beat)
    coll_world = dist.get_world_size() if dist_on else 1
    sharded = a.layout == "sharded" or (a.layout == "auto" and world > 1)
    CH = a.channels if a.channels else (4 if sharded else 1)
    S_total = a.sites
    if sharded:
        s_begin, s_end = shard_bounds(S_total, world, rank)
    else:
        s_begin, s_end = rank * S_total, (rank + 1) * S_total
    S = s_end - s_begin  # this rank's sites per channel
    n_channel = S_total if sharded else world * S_total  # sites per channel job
    L = hip.lib()
    with open(hip.LIB_PATH, "rb") as fh:  # which build ran (profiles/ summaries name it too)
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    hip.check(L.tmh_set_device(local_rank))
    same = None
    if sharded and world > 1 and not a.no_same_workload and not staged:
        if rank == 0:  # before this run's buffers exist: the GPU's whole HBM is free
            beat("single-GPU run of the same workload")
            log("rank 0: the same %d-channel workload on this GPU alone" % CH)
            same = single_gpu_same_workload(L, dev, H, W, CH, S_total,
                                            DISTRIBUTIONS[a.distribution])
            log("single GPU, same workload: %.1f sites/s" % same["value"])
        D.barrier()
    # one non-null stream for our launches AND torch/RCCL work, so they order
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = C.c_void_p(stream.cuda_stream)

    # resident inputs / outputs (int16 tensors = raw uint16 bytes) of channel c
    # = its global sites [s_begin, s_end): one contiguous buffer each, or
    # (--block-sites B) blocks of B sites in separate allocations, input and
    # output blocks allocated alternately.  The fused pass's speed depends on
    # which HBM region holds its 38 GB output (12.8-15.2 ms for the same job
    # on different buffers of one process; blocks ran 13.1 on every draw:
    # DESIGN.md §3, profiles/r3/mb_place2_r3a.txt).
    dist_id = DISTRIBUTIONS[a.distribution]
    B = a.block_sites if a.pipeline == "fused" else 0  # the separate pipeline is contiguous
    if B:
        assert B >= 4 and B & (B - 1) == 0, "--block-sites must be a power of two >= 4"
    shift = B.bit_length() - 1 if B else 0
    # The Welford pass reads the sites once, in site order: its contiguous path
    # runs 0.25-0.3 ms faster than its block-table path (profiles/r3/
    # ab_block_sites_0_vs_64_r3f.jsonl, mb_place2_r3g.txt), while the fused
    # pass gains from blocked outputs; so by default the input is one buffer
    # (block views of it for the fused pass's table) and the outputs blocks.
    in_contig = not B or a.in_layout == "contiguous"
    skip = (torch.empty(int(a.hbm_skip_gb * 2 ** 30), dtype=torch.uint8, device=dev)
            if a.hbm_skip_gb > 0 else None)
    # Several channels' private outputs may not fit (4 channels x 3,456 sites
    # in + out = 306 GB on one GPU): the corrected outputs then share one set
    # of blocks, except the blocks holding the sites the oracle fingerprints
    # sample (global sites 0, S/2, S-1 of every channel), which stay private.
    out_b = CH * S * npx * 2
    share_out = B and CH > 1 and (a.share_outputs == "yes" or (
        a.share_outputs == "auto" and
        2 * out_b > 0.85 * torch.cuda.get_device_properties(dev).total_memory))
    checked = {s - s_begin for s in (0, S_total // 2, S_total - 1) if s_begin <= s < s_end}
    shared_out = {}
    chan_sites = []  # per channel: (input blocks, output blocks); one block if contiguous
    for c in range(CH):
        blk_in, blk_out = [], []
        big = None
        if B and in_contig:
            big = torch.empty((S, H, W), dtype=torch.int16, device=dev)
            hip.check(L.tmh_synth_sites_device(C.c_void_p(big.data_ptr()), S, H, W, SEED, c,
                                               s_begin, dist_id, sp))
        for b0 in range(0, S, B if B else S):
            m = min(B, S - b0) if B else S
            if big is not None:
                blk_in.append(big[b0:b0 + m])
            else:
                blk_in.append(torch.empty((m, H, W), dtype=torch.int16, device=dev))
                hip.check(L.tmh_synth_sites_device(C.c_void_p(blk_in[-1].data_ptr()), m, H, W,
                                                   SEED, c, s_begin + b0, dist_id, sp))
            if share_out and not any(b0 <= i < b0 + m for i in checked):
                if b0 not in shared_out:
                    shared_out[b0] = torch.empty((m, H, W), dtype=torch.int16, device=dev)
                blk_out.append(shared_out[b0])
            else:
                blk_out.append(torch.empty((m, H, W), dtype=torch.int16, device=dev))
        chan_sites.append((blk_in, blk_out))

    def local_site(c, i, outputs=False):
        """channel c's local site i (input or corrected output) as a tensor view"""
        blks = chan_sites[c][1 if outputs else 0]
        return blks[i // B][i % B] if B else blks[0][i]
    lo, hi, gamma = quantile_table(npx, np.linspace(0, 100, Q))
    lut = stats_log10_lut()
    flags = hip.TMH_STATS_DEFERRED_PCT if dist_on else 0
    if a.serial_stats:
        flags |= hip.TMH_STATS_SERIAL
    fused = a.pipeline == "fused"
    prof = not a.no_profile

    probe_sp = [None]  # several channels: the site probes' own stream (set below)

    class Channel(object):
        """One channel's job: its sites, statistics handle, corrector and
        stream (channel 0 runs on the main stream; with several channels the
        others overlap on their own streams, configs[2]/[3])."""

        def __init__(self, c, lane=0):
            self.lane = lane
            # (high-priority channel streams measured slower: 14.97 vs 12.74 ms
            # for 4 x 432 sites, profiles/r5/dist432_stream_priority_r5y.jsonl)
            self.stream = (stream if (c == 0 and lane == 0) or a.channel_streams == "one"
                           else torch.cuda.Stream(dev))
            if a.welford_cus and CH == 1:  # (experiment) the lane's Welford pass and planes on fewer CUs
                self.stream = cu_masked_stream(torch, dev, a.welford_cus)
            self.sp = C.c_void_p(self.stream.cuda_stream)
            # jobs in flight: the corrected pass on a stream of its own, so the
            # histogram tail runs on the statistics handle's stream after it
            # (tmhip.h stream contract) and the next job need not wait for it
            # (one stream for every lane's corrected pass: they run in job order)
            if jobs_in_flight > 1 and "cstream" not in shared_streams:
                shared_streams["cstream"] = torch.cuda.Stream(dev)
            self.cstream = shared_streams["cstream"] if jobs_in_flight > 1 else self.stream
            self.csp = C.c_void_p(self.cstream.cuda_stream)
            blk_in, blk_out = chan_sites[c]
            self.blocks = (blk_in, blk_out)
            self.S_ptr = C.c_void_p(blk_in[0].data_ptr())
            self.O_ptr = C.c_void_p(blk_out[0].data_ptr())
            if B:  # device tables of the block base pointers
                self.t_in = torch.tensor([t.data_ptr() for t in blk_in], dtype=torch.int64,
                                         device=dev)
                self.t_out = torch.tensor([t.data_ptr() for t in blk_out], dtype=torch.int64,
                                          device=dev)
                self.T_in = C.c_void_p(self.t_in.data_ptr())
                self.T_out = C.c_void_p(self.t_out.data_ptr())
            self.mean = torch.empty(npx, dtype=torch.float64, device=dev)
            self.std = torch.empty_like(self.mean)
            self.smean = torch.empty_like(self.mean)
            self.sstd = torch.empty_like(self.mean)
            self.tmp = torch.empty_like(self.mean)
            self.tmp2 = torch.empty_like(self.mean)
            self.h = C.c_void_p()
            hip.check(L.tmh_stats_create(H, W, Q, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                         hip.ptr(lut), 1, flags, C.byref(self.h)))
            hip.check(L.tmh_stats_set_stream(self.h, self.sp))
            if a.welford_parts is not None:
                hip.check(L.tmh_stats_set_option(self.h, hip.TMH_OPT_WELFORD_PARTS, a.welford_parts))
            if a.fused_config is not None:
                hip.check(L.tmh_stats_set_option(self.h, hip.TMH_OPT_FUSED_CONFIG, a.fused_config))
            self.corr = C.c_void_p()
            torch.cuda.synchronize(dev)
            hip.check(L.tmh_corrector_create_device(C.c_void_p(self.mean.data_ptr()),
                                                    C.c_void_p(self.std.data_ptr()), H, W, 1,
                                                    ZERO_LOG10, self.sp, C.byref(self.corr)))
            if a.fused_cus is not None:
                hip.check(L.tmh_corrector_set_option(self.corr, hip.TMH_OPT_FUSED_CUS, a.fused_cus))
            if a.fused_bands is not None:
                hip.check(L.tmh_corrector_set_option(self.corr, hip.TMH_OPT_FUSED_BANDS,
                                                     a.fused_bands))
            self.ops = StatsOps(L, self.h, npx, Q, dev)
            self.merge_ev = []  # (welford start, end, counts start, end) per timed step

        def reset_probe(self):
            """The job's reset, and its site probe queued at once (no wait):
            with several channels every probe is in flight before any
            channel's Welford launch waits for its own.  The probe reads only
            the (resident) sites: on the probe stream it need not wait for
            the handle's queued work (tmhip.h)."""
            hip.check(L.tmh_stats_reset(self.h))
            sp = probe_sp[0] or self.sp
            if fused and B and not in_contig:
                hip.check(L.tmh_stats_probe_blocks_device(self.h, self.T_in, shift, S, sp))
            else:
                hip.check(L.tmh_stats_probe_device(self.h, self.S_ptr, S, sp))

        def welford(self, sp=None):
            sp = sp or self.sp  # another stream: the library orders it against the handle's
            if fused and B and not in_contig:  # Welford pass; histograms from the correction's read
                hip.check(L.tmh_stats_update_welford_blocks_device(self.h, self.T_in, shift, S, 1,
                                                                   sp))
            elif fused:
                hip.check(L.tmh_stats_update_welford_device(self.h, self.S_ptr, S, 1, sp))
            else:
                hip.check(L.tmh_stats_update_device(self.h, self.S_ptr, S, 1, sp))

        def stats(self):
            self.reset_probe()
            self.welford()

        def planes(self):
            """finalize -> smoothing -> coefficients of this job alone"""
            p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
            if a.planes == "multi":
                planes_multi([self], unsmoothed=False)
                return
            hip.check(L.tmh_stats_finalize_device(self.h, p(self.mean), p(self.std), self.sp))
            hip.check(L.tmh_smooth2_f64_device(p(self.mean), p(self.std), p(self.smean),
                                               p(self.sstd), p(self.tmp), p(self.tmp2), H, W, 5.0,
                                               self.sp))
            hip.check(L.tmh_corrector_update_device(self.corr, p(self.smean), p(self.sstd),
                                                    self.sp))

        def apply(self):
            self.planes()
            self.corrected()

        def corrected(self, sp=None):
            csp = sp or self.csp
            if fused and B:
                hip.check(L.tmh_correct_u16_hist_blocks_device(self.corr, self.h, self.T_in,
                                                               self.T_out, shift, S, -1, -1,
                                                               csp))
            elif fused:
                hip.check(L.tmh_correct_u16_hist_device(self.corr, self.h, self.S_ptr, self.O_ptr,
                                                        S, -1, -1, csp))
            else:
                hip.check(L.tmh_correct_u16_device(self.corr, self.S_ptr, self.O_ptr, S, -1, -1,
                                                   self.sp))

        def event(self):
            e = torch.cuda.Event(enable_timing=True)
            e.record(self.stream)
            return e

        def close(self):
            L.tmh_corrector_destroy(self.corr)
            L.tmh_stats_destroy(self.h)

    def planes_multi(jobs, sp=None, unsmoothed=False):
        """The planes step of several jobs (a rank's channels) in one launch per
        kernel (tmh_job_planes_multi_device), on the first job's stream (or
        sp): the library orders it after every job's stream and every job's
        stream after it.  unsmoothed=False: only the smoothed planes the
        correction needs (no finalize launch)."""
        n = len(jobs)
        arr = lambda xs: (C.c_void_p * n)(*[C.c_void_p(x) for x in xs])  # noqa: E731
        hip.check(L.tmh_job_planes_multi_device(
            arr([j.h.value for j in jobs]), arr([j.corr.value for j in jobs]), n,
            arr([j.mean.data_ptr() for j in jobs]) if unsmoothed else None,
            arr([j.std.data_ptr() for j in jobs]) if unsmoothed else None,
            arr([j.smean.data_ptr() for j in jobs]), arr([j.sstd.data_ptr() for j in jobs]),
            5.0, sp or jobs[0].sp))

    def corrected_multi(jobs, sp):
        """Every job's corrected pass in one fused launch on sp (the library
        orders it after each job's handle stream; each job's histogram tail on
        its handle's tail stream)."""
        n = len(jobs)
        arr = lambda xs: (C.c_void_p * n)(*[C.c_void_p(x) for x in xs])  # noqa: E731
        ns = (C.c_int64 * n)(*[S] * n)
        if B:
            hip.check(L.tmh_correct_u16_hist_multi_blocks_device(
                arr([j.corr.value for j in jobs]), arr([j.h.value for j in jobs]), n,
                arr([j.T_in.value for j in jobs]), arr([j.T_out.value for j in jobs]), shift, ns,
                -1, -1, sp))
        else:
            hip.check(L.tmh_correct_u16_hist_multi_device(
                arr([j.corr.value for j in jobs]), arr([j.h.value for j in jobs]), n,
                arr([j.S_ptr.value for j in jobs]), arr([j.O_ptr.value for j in jobs]), ns,
                -1, -1, sp))

    # jobs in flight (one channel, one rank): lanes share the sites and the
    # output blocks; job k runs on lane k % J after job k-1's corrected pass
    # (outputs written in job order, HBM passes one at a time), so what
    # overlaps is job k's Welford pass with job k-1's histogram tail
    shared_streams = {}
    J = jobs_in_flight = max(1, a.jobs_in_flight) if (CH == 1 and not dist_on and fused) else 1
    chans = [Channel(c) for c in range(CH)]
    lanes = chans + [Channel(0, lane=j) for j in range(1, J)]
    # several channels, --channel-order serial: every channel's Welford pass,
    # then every channel's corrected pass, one after another on one stream of
    # their own (each streaming pass alone on the GPU; the library orders it
    # against the channel's handle stream, and each channel's histogram tail
    # runs on its handle's tail stream under the next channel's pass)
    pass_stream = (torch.cuda.Stream(dev) if CH > 1 and a.channel_order in ("serial", "pipelined",
                                                                         "deep")
                   else None)
    evs_p = {}
    # the pipelined order merges each channel on its own stream as soon as its
    # pass is done (one collective per quantity and channel)
    merge_mode = ("per-channel" if a.channel_order == "pipelined" and CH > 1 else
                  "batched" if a.channel_order == "deep" and CH > 1 else a.merge)
    pass_sp = C.c_void_p(pass_stream.cuda_stream) if pass_stream is not None else None
    # (experiment, --welford-cus with several channels) the Welford passes on
    # a CU-masked stream of their own, so the channels' plane chains queued
    # beside them find free CUs; the corrected passes stay on the pass stream
    wf_sp = pass_sp
    if a.welford_cus and pass_stream is not None:
        wf_stream = cu_masked_stream(torch, dev, a.welford_cus)
        wf_sp = C.c_void_p(wf_stream.cuda_stream)
    multi_pass = pass_sp is not None and fused and a.pass_launch == "multi"
    # several channels on the pass stream: consecutive jobs (steps) alternate
    # between --jobs-in-flight sets of channel handles / correctors, so the
    # next job's reset and site probe are queued under this job's passes and
    # its first Welford pass needs nothing of this job's histogram tails and
    # count merges (the same jobs in flight as the one-channel headline)
    CJ = max(1, a.jobs_in_flight) if (pass_sp is not None and fused) else 1
    # --channel-order deep: job p+1's Welford passes run before job p's
    # corrected pass, so job p's merges and planes (and job p-1's count
    # merges, histogram tails and the next job's probe) all run under Welford
    # passes; three channel sets (jobs p-1, p, p+1 in flight)
    deep = a.channel_order == "deep" and pass_sp is not None and fused and B
    if pass_sp is not None or (J > 1 and a.prefetch_probe == "on"):
        probe_stream = torch.cuda.Stream(dev)
        probe_sp[0] = C.c_void_p(probe_stream.cuda_stream)
    if deep:
        CJ = max(3, CJ)
        small_stream = torch.cuda.Stream(dev)
        small_sp = C.c_void_p(small_stream.cuda_stream)
    sets = [chans] + [[Channel(c, lane=j) for c in range(CH)] for j in range(1, CJ)]

    def corrected_all(X):
        if multi_pass:
            corrected_multi(X, pass_sp)
        else:
            for ch in X:
                ch.corrected(pass_sp)
    jobs = {"k": 0, "applied": None, "welford": None, "probed": set(), "p": None,
            "counts": None}

    def deep_step(last=False):
        """One period of the deep order (job p): job p+1's Welford passes,
        job p-1's count merges, job p+2's reset and probe, job p's merges and
        planes, job p's corrected pass.  Per period exactly one job's passes;
        the first period's job p+1 Welford passes follow a prologue (job p's)."""
        S_ = lambda j: sets[j % CJ]  # noqa: E731
        if jobs["p"] is None:  # prologue (warm-up): job 0's reset, probe and Welford passes
            jobs["p"] = 0
            for ch in S_(0):
                ch.reset_probe()
            for ch in S_(0):
                ch.welford(wf_sp)
            for ch in S_(1):
                ch.reset_probe()
        p = jobs["p"]
        for ch in S_(p + 1):  # probed a period ago: no host wait
            ch.welford(wf_sp)
        if jobs["counts"] is not None:  # job p-1's count merges (after its tails)
            if dist_on:
                with torch.cuda.stream(small_stream):
                    merge_counts_multi([ch.ops for ch in jobs["counts"]], D)
            jobs["counts"] = None
        if not last:  # job p+2 reuses job p-1's set: after its count merges
            for ch in S_(p + 2):
                ch.reset_probe()
        X = S_(p)
        if dist_on:
            with torch.cuda.stream(small_stream):
                merge_welford_multi([ch.ops for ch in X], D, n_totals=[n_channel] * CH)
        planes_multi(X, sp=small_sp, unsmoothed=False)
        corrected_all(X)
        jobs["counts"] = X
        jobs["p"] = p + 1

    def deep_drain():
        """Untimed, after the timed periods: the in-flight jobs completed
        (job p-1's count merges; job p's merges, planes and corrected pass)."""
        if jobs["counts"] is not None and dist_on:
            with torch.cuda.stream(small_stream):
                merge_counts_multi([ch.ops for ch in jobs["counts"]], D)
        X = sets[jobs["p"] % CJ]
        if dist_on:
            with torch.cuda.stream(small_stream):
                merge_welford_multi([ch.ops for ch in X], D, n_totals=[n_channel] * CH)
        planes_multi(X, sp=small_sp, unsmoothed=False)
        corrected_all(X)
        if dist_on:
            with torch.cuda.stream(small_stream):
                merge_counts_multi([ch.ops for ch in X], D)
        jobs["counts"] = None

    log("%d channel(s) x %d sites resident; warm-up" % (CH, S))
    beat("warm-up")

    timing = {"on": False}

    def step(last=False):
        if deep:
            deep_step(last)
            return
        if J > 1:
            ch = lanes[jobs["k"] % J]
            nxt = lanes[(jobs["k"] + 1) % J]
            jobs["k"] += 1
            gate = {"welford": jobs["welford"], "planes": jobs.get("planes"),
                    "corrected": jobs["applied"]}[a.jobs_order]
            if gate is not None:  # after the previous job's Welford (or corrected) pass
                ch.stream.wait_event(gate)
            if id(ch) in jobs["probed"]:  # reset and probed one step ago
                jobs["probed"].discard(id(ch))
                ch.welford()
            else:
                ch.stats()
            ev_w = torch.cuda.Event()
            ev_w.record(ch.stream)
            jobs["welford"] = ev_w
            if a.prefetch_probe == "on" and not last and nxt is not ch:
                # the next job's reset (after its lane's previous job) and site
                # probe (on the probe stream, sites resident) now: they run
                # under this job's passes, so the next Welford launch finds
                # its probe done instead of waiting for it behind this job's
                # corrected pass
                nxt.reset_probe()
                jobs["probed"].add(id(nxt))
            ch.planes()
            ev_p = torch.cuda.Event()
            ev_p.record(ch.stream)
            jobs["planes"] = ev_p
            if jobs["applied"] is not None:  # corrected passes in job order (shared outputs)
                ch.cstream.wait_event(jobs["applied"])
            ch.corrected()
            ev = torch.cuda.Event()
            ev.record(ch.cstream)
            jobs["applied"] = ev
            return
        X = sets[jobs["k"] % CJ]
        Y = sets[(jobs["k"] + 1) % CJ]
        jobs["k"] += 1

        def reset_probe(Z):
            if id(Z) not in jobs["probed"]:
                for ch in Z:
                    ch.reset_probe()
            jobs["probed"].discard(id(Z))

        def prefetch():
            # the next job's reset and site probe (channel set Y), queued on
            # Y's streams now: they run under this job's passes
            if CJ > 1 and not last:
                for ch in Y:
                    ch.reset_probe()
                jobs["probed"].add(id(Y))
        if a.channel_order == "pipelined":
            # every channel's probe queued, then the Welford passes one after
            # another on the pass stream; channel c's merge and planes on its
            # own stream as soon as its pass is done (under the next channel's
            # Welford pass); the corrected passes one after another on the pass
            # stream (each after its channel's planes: the library's stream
            # contract), each channel's tail and count merge under the next
            # channel's corrected pass
            reset_probe(X)
            for ch in X:
                ch.welford(wf_sp)
            prefetch()
            for ch in X:
                with torch.cuda.stream(ch.stream):
                    if dist_on:
                        e0 = ch.event() if timing["on"] else None
                        merge_welford(ch.ops, D, n_total=n_channel)
                        evs_p[id(ch)] = [e0, ch.event() if timing["on"] else None]
                ch.planes()
            corrected_all(X)
            if dist_on:
                for ch in X:
                    with torch.cuda.stream(ch.stream):
                        e2 = ch.event() if timing["on"] else None
                        merge_counts(ch.ops, D)
                        if timing["on"]:
                            ch.merge_ev.append(evs_p[id(ch)] + [e2, ch.event()])
            return
        reset_probe(X)  # every channel's probe queued before any Welford launch waits
        for ch in X:
            ch.welford(wf_sp)
        prefetch()
        evs = {}
        if dist_on and merge_mode == "batched":
            # every channel's merge on the main stream, one collective per
            # quantity for all channels (the library orders each handle's
            # stream against it: tmhip.h stream contract)
            with torch.cuda.stream(stream):
                e0 = X[0].event() if timing["on"] else None
                merge_welford_multi([ch.ops for ch in X], D, n_totals=[n_channel] * CH)
                evs["batched"] = [e0, X[0].event() if timing["on"] else None]
        elif dist_on:
            for ch in X:
                with torch.cuda.stream(ch.stream):
                    e0 = ch.event() if timing["on"] else None
                    merge_welford(ch.ops, D, n_total=n_channel)
                    evs[id(ch)] = [e0, ch.event() if timing["on"] else None]
        if a.planes == "multi":
            planes_multi(X, unsmoothed=False)
        else:
            for ch in X:
                ch.planes()
        corrected_all(X)
        if dist_on and merge_mode == "batched":
            with torch.cuda.stream(stream):
                e2 = X[0].event() if timing["on"] else None
                merge_counts_multi([ch.ops for ch in X], D)
                if timing["on"]:
                    X[0].merge_ev.append(evs["batched"] + [e2, X[0].event()])
        elif dist_on:
            for ch in X:
                with torch.cuda.stream(ch.stream):
                    e2 = ch.event() if timing["on"] else None
                    merge_counts(ch.ops, D)
                    if timing["on"]:
                        ch.merge_ev.append(evs[id(ch)] + [e2, ch.event()])

    for i in range(a.warmup):
        beat.step = " (warm-up step %d)" % i
        step()
    beat("synchronize after warm-up")
    torch.cuda.synchronize(dev)

    log("timing %d steps" % a.steps)
    if prof:
        L.tmh_profile_enable(1)
        L.tmh_profile_reset()
        timing["on"] = dist_on
    if dist_on:
        D.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    host_ms = []  # the host's time to queue each step (it runs ahead unless it waits)
    for i in range(a.steps):
        beat.step = " (timed step %d)" % i
        th = time.perf_counter()
        step(last=i == a.steps - 1)
        host_ms.append(1e3 * (time.perf_counter() - th))
    beat.step = ""
    beat("synchronize after the timed steps", echo=False)
    torch.cuda.synchronize(dev)
    if dist_on:
        D.barrier()
    elapsed = time.perf_counter() - t0
    beat("timed steps done: checks and report")
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        D.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel event timing on the launch stream (live roofline)
    kern = {}
    if prof:
        for name in ("welford", "hist", "pct_acc", "finalize", "smooth", "coeffs", "correct",
                     "correct_hist", "hist_finalize", "hist_u16", "colsum"):
            ms, k = C.c_double(), C.c_int64()
            hip.check(L.tmh_profile_read(name.encode(), C.byref(ms), C.byref(k)))
            if k.value:
                kern[name] = (ms.value / k.value, k.value)
        L.tmh_profile_enable(0)
    if deep:  # the jobs in flight completed (untimed) before the checks
        deep_drain()
        torch.cuda.synchronize(dev)
    collectives = None
    if dist_on and prof:  # one more step with every collective timed on its own
        ct = CollectiveTimer(torch, dev)
        for ch in chans:
            ch.stats()
        if merge_mode == "batched":
            with torch.cuda.stream(stream):
                merge_welford_multi([ch.ops for ch in chans], D, n_totals=[n_channel] * CH,
                                    timer=ct)
        else:
            for ch in chans:
                with torch.cuda.stream(ch.stream):
                    merge_welford(ch.ops, D, n_total=n_channel, timer=ct)
        for ch in chans:
            ch.apply()
        if merge_mode == "batched":
            with torch.cuda.stream(stream):
                merge_counts_multi([ch.ops for ch in chans], D, timer=ct)
        else:
            for ch in chans:
                with torch.cuda.stream(ch.stream):
                    merge_counts(ch.ops, D, timer=ct)
        collectives = ct.summary()
    merge_ms = None
    if dist_on and prof:
        merge_ms = []
        for ch in chans:
            if not ch.merge_ev:  # batched merges: timed on channel 0 for all channels
                continue
            w = [e[0].elapsed_time(e[1]) for e in ch.merge_ev]
            m = [e[2].elapsed_time(e[3]) for e in ch.merge_ev]
            merge_ms.append({"welford_allreduce_ms": round(float(np.mean(w)), 4),
                             "pct_chain_hist_allreduce_ms": round(float(np.mean(m)), 4)})

    # every channel's results after the last step (identical on every rank)
    # against its oracle fingerprint (tests/golden/make_bench_fingerprint.py)
    check, check_ok = {}, None
    per_channel = {}
    for c, ch in (list(enumerate(chans)) + [(0, ln) for ln in lanes[len(chans):]] +
                  [(c, ch) for X in sets[1:] for c, ch in enumerate(X)]):
        nn = C.c_int64()
        res = {"mean": np.empty(npx), "std": np.empty(npx), "acc": np.empty(Q),
               "hist": np.empty(65536, np.uint64)}
        hip.check(L.tmh_stats_finalize(ch.h, C.byref(nn), hip.ptr(res["mean"]),
                                       hip.ptr(res["std"]), hip.ptr(res["acc"]),
                                       hip.ptr(res["hist"])))
        res["n"] = nn.value
        chk = {"n": int(nn.value), "mean_sum": float(res["mean"].sum()),
               "std_sum": float(res["std"].sum()),
               "pct_sums_sha256": hashlib.sha256(res["acc"].tobytes()).hexdigest()[:16],
               "hist_sha256": hashlib.sha256(res["hist"].tobytes()).hexdigest()[:16]}
        fp, fp_path = load_fingerprint(H, W, S_total, a.distribution, channel=c)
        if fp is not None and n_channel == S_total and fused:
            held = {s: local_site(c, s - s_begin, outputs=True).cpu().numpy().view(np.uint16)
                    for s in fp["corr_sites"].tolist() if s_begin <= s < s_end}
            oks, cnt = check_against_fingerprint(fp, res, ch.smean.cpu().numpy(),
                                                 ch.sstd.cpu().numpy(), held)
            if dist_on:
                flags_t = torch.tensor([int(v) for v in oks.values()], dtype=torch.int64,
                                       device=dev)
                D.all_reduce(flags_t, op=dist.ReduceOp.MIN)
                oks = dict(zip(oks, (bool(v) for v in flags_t.tolist())))
                cnt_t = torch.tensor(cnt, dtype=torch.int64, device=dev)
                D.all_reduce(cnt_t)
                cnt = cnt_t.cpu().numpy()
            tot = max(int(cnt.sum()), 1)
            oks["corrected_within_1DN"] = bool(cnt[3] == 0 and cnt[4] == 0)
            chk["vs_oracle"] = dict(oks, fingerprint=os.path.relpath(fp_path, REPO))
            chk["corrected_vs_oracle"] = {
                "sampled_pixels": tot, "sites": fp["corr_sites"].tolist(),
                "frac_equal": round(cnt[0] / tot, 6), "frac_plus1": round(cnt[1] / tot, 6),
                "frac_minus1": round(cnt[2] / tot, 6), "beyond_1DN": int(cnt[3]),
                "wrap_flips": int(cnt[4])}
            per_channel[c] = per_channel.get(c, True) and all(oks.values())
        if ch.lane > 0:  # the other jobs-in-flight lane(s): their own statistics, same outputs
            check.setdefault("lanes", {})["lane%d" % ch.lane + ("_c%d" % c if c else "")] = chk
        elif c == 0:
            check = chk
        else:
            check.setdefault("channels", {})["c%d" % c] = chk
    if per_channel:
        check["channels_checked"] = sorted(per_channel)
        check_ok = all(per_channel.values())
        if len(per_channel) != CH:
            check["channels_unchecked"] = [c for c in range(CH) if c not in per_channel]
    ch0 = chans[0]
    choice = None
    if hasattr(L, "tmh_stats_job_choice"):  # (absent from A/B builds of earlier trees)
        pc, wb, fc = (C.c_uint32 * 3)(), C.c_int(), C.c_int()
        hip.check(L.tmh_stats_job_choice(ch0.h, pc, C.byref(wb), C.byref(fc)))
        choice = {"probe_groups": list(pc), "welford_bright": wb.value,
                  "fused_config": "no-histogram + per-site u16 pass" if fc.value == 100
                  else fc.value}

    log("%.1f ms/step; check_vs_oracle %s" % (1e3 * elapsed / a.steps, check_ok))
    extras = {}
    solo_kern = {}
    if J > 1 and not a.no_extras:
        # the same K jobs one at a time (lane 0 only), for comparison, with
        # each kernel's duration when no other job shares the GPU
        torch.cuda.synchronize(dev)
        if prof:
            L.tmh_profile_enable(1)
            L.tmh_profile_reset()
        t1 = time.perf_counter()
        for _ in range(a.steps):
            chans[0].stats()
            chans[0].apply()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter() - t1
        if prof:
            for name in ("welford", "correct_hist", "hist_finalize", "pct_acc"):
                ms, k = C.c_double(), C.c_int64()
                hip.check(L.tmh_profile_read(name.encode(), C.byref(ms), C.byref(k)))
                if k.value:
                    solo_kern[name] = ms.value / k.value
            L.tmh_profile_enable(0)
        extras["one_job_at_a_time"] = {"sites_per_s": round(CH * S * a.steps / t1, 1),
                                       "ms_per_step": round(1e3 * t1 / a.steps, 3),
                                       "kernel_avg_ms": {k: round(v, 4) for k, v in solo_kern.items()}}
    if not a.no_extras and world == 1:
        # the chain pass reads one contiguous run of sites
        if B:
            flat = torch.cat(chan_sites[0][0])
            extras["chain_u8"] = bench_chain(L, ch0.corr, C.c_void_p(flat.data_ptr()), S, H, W,
                                             dev, sp)
            del flat
        else:
            extras["chain_u8"] = bench_chain(L, ch0.corr, ch0.S_ptr, S, H, W, dev, sp)
        extras["host_path"] = bench_host_path(H, W)
        try:
            extras["input_path"] = bench_input_path(H, W, dev)
        except Exception as e:  # libhdf5 missing on the box: report, never fail the headline
            extras["input_path"] = {"error": "%s: %s" % (type(e).__name__, e)}
    box = None
    if not a.no_box and not staged and hasattr(L, "tmh_box_probe_device"):
        # (absent from A/B builds of earlier trees) the box's own copy / read rates over channel 0's buffers (after the
        # checks: the copy overwrites the corrected outputs), so the passes'
        # rates can be read against this box rather than the 8 TB/s spec
        torch.cuda.synchronize(dev)
        if B:
            tab = {"t_in": ch0.T_in, "t_out": ch0.T_out, "shift": shift}
        else:
            t_one = torch.tensor([ch0.S_ptr.value], dtype=torch.int64, device=dev)
            o_one = torch.tensor([ch0.O_ptr.value], dtype=torch.int64, device=dev)
            tab = {"t_in": C.c_void_p(t_one.data_ptr()), "t_out": C.c_void_p(o_one.data_ptr()),
                   "shift": 24}
        log("box probe: copy and read over the job's buffers")
        box = box_probe(L, hip, tab, S, H, W, sp)
        box["sysfs_clocks"] = {"start": clocks_start, "end": sysfs_clocks(torch, dev)}

    if rank == 0:
        site_bytes = npx * 2
        alg = {  # algorithmic HBM bytes per channel job (per-site figure x sites)
            "welford": S * site_bytes + 4 * 8 * npx,       # sites + mean/M2 read & write
            "hist": S * site_bytes,                        # sites
            "correct": S * site_bytes * 2 + 16 * npx,      # sites in + out, coefficients
            "correct_hist": S * site_bytes * 2 + 8 * npx,  # sites in + out, coefficients
            "pct_acc": S * Q * 4,                          # per-site order statistics
        }
        kdetail = {}
        for name, (avg_ms, k) in kern.items():
            # alg bytes are per channel job; a kernel may run in several launches
            # per job (pct_acc / hist_finalize in pieces): rate over its job time
            step_ms = avg_ms * k / (a.steps * CH)
            d = {"avg_ms": round(avg_ms, 4), "launches": k, "ms_per_job": round(step_ms, 4)}
            if name in alg:
                gbs = alg[name] / (step_ms * 1e-3) / 1e9
                d["alg_GBs"] = round(gbs, 1)
                d["frac_of_8TBs"] = round(gbs / HBM_PEAK_GBS, 4)
            kdetail[name] = d
        # the roofline's kernel: the one moving the most algorithmic bytes (the
        # fused correct + histogram pass, 4 of the job's 6 B/px).  (By time, a
        # Welford pass co-running with another job's kernels could be picked
        # on bright data, where both passes stretch.)
        dominant = max((n for n in kern if n in alg), key=lambda n: alg[n], default=None)
        roofline = None
        if dominant:
            avg_ms, k_launch = kern[dominant]
            # one launch may carry several channels' jobs (--pass-launch multi)
            jobs_per_launch = max(1, int(round(a.steps * CH / k_launch)))
            alg_launch = alg[dominant] * jobs_per_launch
            ach = alg_launch / (avg_ms * 1e-3) / 1e9
            # PMC traffic (tools/pmc_traffic.py) of THIS library build only:
            # the summary names the sha256 of the library it was measured on
            traffic, traffic_src = None, None
            try:
                with open(a.traffic_json) as f:
                    tj = json.load(f)
                cfg = tj.get("config", {})
                if cfg.get("sites") == S and cfg.get("height") == H and cfg.get("width") == W \
                        and cfg.get("distribution", "synthetic") == a.distribution:
                    if tj.get("library_sha256") == lib_sha:
                        traffic = tj.get("kernels", {}).get(dominant, {}).get("hbm_bytes_per_launch")
                        traffic_src = os.path.relpath(a.traffic_json, REPO)
                    else:
                        traffic_src = "%s was measured on another build (sha256 %s)" % (
                            os.path.relpath(a.traffic_json, REPO), str(tj.get("library_sha256"))[:16])
            except (OSError, ValueError):
                pass
            roofline = {"bound": "hbm", "kernel": dominant, "achieved": round(ach, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": traffic_src,
                        "alg_bytes_per_launch": alg_launch, "jobs_per_launch": jobs_per_launch,
                        "timed": "HIP events around the launch of the one configuration the job "
                                 "runs, on its stream (tmh_profile_*)"}
            if J > 1:
                roofline["note"] = ("%d jobs in flight: the pass holds every CU (persistent "
                                    "grid), so the next job's Welford pass runs after it; "
                                    "this job's histogram tail runs under that Welford pass "
                                    "(profiles/r5/trace_jobs_synthetic_r5a.txt)"
                                    % J) if a.jobs_order == "welford" else (
                                    "%d jobs in flight (the next job's Welford pass after this "
                                    "pass)" % J)
                if dominant in solo_kern:
                    solo = alg[dominant] / (solo_kern[dominant] * 1e-3) / 1e9
                    roofline["achieved_one_job_at_a_time"] = round(solo, 1)
                    roofline["frac_one_job_at_a_time"] = round(solo / HBM_PEAK_GBS, 4)
        total_sites = world * CH * S * a.steps if not sharded else CH * S_total * a.steps
        value = total_sites / elapsed
        job_bytes = total_sites // a.steps * 6 * npx  # 6 B/px algorithmic per site-image
        if sharded:
            workload = ("illumstats+correct, %d channels x %d sites of %dx%d uint16, each channel's "
                        "sites sharded over %d GPU(s) (%d per GPU), one job per channel on its own "
                        "stream (configs[2]: full plate 384 wells x 9 sites x 4 channels; the "
                        "same job is configs[3]: exact 65,536-bin per-site percentile histograms + "
                        "smoothed IllumstatsContainer apply, 4 channels at 2/4/8 GPUs)"
                        % (CH, S_total, H, W, world, S, ))
        elif CH == 1:
            workload = ("illumstats+correct, 1 channel, %d sites/GPU of %dx%d uint16 "
                        "(configs[1]: 384 wells x 9 sites)" % (S, H, W))
        else:
            workload = ("illumstats+correct, %d channels x %d sites/GPU of %dx%d uint16, "
                        "one job per channel on its own stream" % (CH, S, H, W))
        resd = {
            "metric": METRIC,
            "library_sha256": lib_sha,
            "value": round(value, 1),
            "unit": "sites/s",
            "n_gpus": 1 if staged else world,
            "ranks": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 3),
            "host_queue_ms_per_step": [round(float(np.median(host_ms)), 3),
                                       round(float(np.max(host_ms)), 3)],
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64 stats / f32 correct (±1 DN)",
            "data": "synthetic '%s' (integer-exact device generator, tmlibrary_amd/synth.py; "
                    "SURVEY.md §8(d) distribution), resident in HBM" % a.distribution,
            "config": {"workload": workload,
                       "sites_per_gpu": CH * S, "channels": CH, "sites_per_channel": n_channel,
                       "height": H, "width": W, "decimals": 3,
                       "smoothing_sigma": 5, "clip": None, "distribution": a.distribution,
                       "parallelism": ("sites sharded (contiguous); %s all-reduce Welford "
                                       "merge, ordered percentile chain, histogram all-reduce"
                                       % ("gloo (host-staged, ranks share GPU 0)" if staged
                                          else "RCCL"))
                       if dist_on else "single GPU",
                       "rccl_world_size": coll_world if dist_on and not staged else None,
                       "collective_world_size": coll_world,
                       "corrected_outputs": ("channels share output blocks except the checked "
                                             "sites' blocks" if share_out else "private"),
                       "pipeline": a.pipeline,
                       "jobs_in_flight": J if CH == 1 else CJ,
                       "prefetch_probe": a.prefetch_probe if J > 1 else None,
                       "planes": a.planes,
                       "channel_order": a.channel_order if CH > 1 else None,
                       "pass_launch": ("multi" if multi_pass else "per-channel") if CH > 1 else None,
                       "merge": merge_mode if dist_on else None,
                       "job_choice": choice,
                       "jobs_order": a.jobs_order if J > 1 else None,
                       "hbm_layout": (("sites in one buffer, corrected output in blocks of %d "
                                       "sites" % B) if in_contig else
                                      ("blocks of %d sites, input and output blocks allocated "
                                       "alternately" % B)) if B else "contiguous"},
            "job_hbm_roofline_frac": round(job_bytes * a.steps / elapsed / 1e9 /
                                           (HBM_PEAK_GBS * world), 4),
            "roofline": roofline,
            "kernels": kdetail,
        }
        if box is not None:
            # each pass's algorithmic rate over the box's own rate for its bytes
            # (copy: 2 + 2 B/px like the fused pass, read: 2 B/px like Welford)
            fr = {}
            for name, probe, alg_name in (("correct_hist", "copy", "correct_hist"),
                                          ("welford", "read", "welford")):
                if name in kdetail and kdetail[name].get("alg_GBs"):
                    fr[name] = round(kdetail[name]["alg_GBs"] / box[probe]["GBs"], 4)
                if name in solo_kern:
                    solo = alg[alg_name] / (solo_kern[name] * 1e-3) / 1e9
                    fr[name + "_one_job_at_a_time"] = round(solo / box[probe]["GBs"], 4)
                    # against the probe's persistent shape (a grid-strided
                    # loop, the passes' own shape): one-launch-per-block flat
                    # copies outrun every long-lived shape measured
                    # (profiles/r6/mb_stream_r6k.txt)
                    pers = box[probe].get("shapes", {}).get("persistent", {}).get("GBs")
                    if pers:
                        fr[name + "_one_job_at_a_time_vs_persistent_shape"] = round(solo / pers, 4)
            box["frac_of_box_copy"] = fr
            box["note"] = ("tmh_box_probe_device: 16-B non-temporal loads (+ stores) over the "
                           "job's own input and output blocks, %d sites, the faster of two "
                           "shapes; sclk_mhz_measured = clock64 / wall_clock64 ticks in the "
                           "persistent probe kernel" % S)
            resd["box"] = box
        if merge_ms:
            if merge_mode == "batched":
                resd["merge_all_channels"] = dict(merge_ms[0], note=(
                    "batched: one collective per quantity for the %d channels" % CH))
            else:
                resd["merge_per_channel"] = merge_ms
        if collectives is not None:
            resd["collectives_isolated"] = {
                "note": "one extra step, the device synchronised before each collective: its own "
                        "time incl. the wait for peers (%d channels' calls summed)" % CH,
                "per_collective": collectives}
        if same is not None:
            resd["single_gpu_same_workload"] = same
        resd["check"] = check
        resd["check_vs_oracle"] = check_ok
        if extras:
            resd["extras"] = extras
        resd["cpu_baseline"] = cpu
        print(json.dumps(resd), file=out, flush=True)

    for ch in lanes:
        ch.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
