"""GPU parity of the exact pipeline bench.py times, at full size.

bench.py's step (one channel job, configs[1]) is, on one stream:
    tmh_stats_reset -> tmh_stats_update_welford_device (site-split Welford)
    -> tmh_stats_finalize_device -> tmh_smooth_f64_device x2
    -> tmh_corrector_update_device -> tmh_correct_u16_hist_device (the fused
       correct + per-site histogram pass, then order statistics and the
       ordered percentile sum)
Here the same calls run on 128 device-resident 2160x2560 sites from the
bench's own generator -- once with the production launch shapes (one Welford
site part) and once with the launch split into 4 site parts (32 full-size
sites each, merged) -- and everything is compared with the CPU oracle on the
same pixels
(reference: tmlib/workflow/corilla/stats.py:64-121, tmlib/image.py:599-631,
:1172-1193): mean/std within 1e-6, pooled and per-site histograms and the
percentile sums bit-exact, corrected pixels within +-1 DN (non-modular) with
zero wrap flips.

test_bright_fullsize covers bright data (the wide log10 path and the
automatic wide fused configuration) at full size.

test_fused_multi_job_configs covers ADVICE r1: several jobs on one handle
(tmh_stats_reset between), high values in different 1,024-bin rounds per
job, every fused configuration, and the corrector on a different stream from
the statistics handle with no host synchronisation inside a job.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import corilla_oracle as orc
from test_gpu_parity import Dev, check_order_stats, site_order_stats
from util import assert_close_rel, dn_report

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from tmlibrary_amd import hip
    return hip.lib()


def _tables(H, W, Q=100000):
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    lo, hi, gamma = quantile_table(H * W, np.linspace(0, 100, Q))
    return lo, hi, gamma, stats_log10_lut()


def _stats_handle(L, H, W, flags):
    from tmlibrary_amd import hip
    lo, hi, gamma, lut = _tables(H, W)
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, len(lo), hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 1, flags, C.byref(h)))
    return h


def _results(L, h, H, W, n_sites, Q=100000):
    from tmlibrary_amd import hip
    nn = C.c_int64()
    mean = np.empty((H, W))
    std = np.empty((H, W))
    acc = np.empty(Q)
    hist = np.empty(65536, np.uint64)
    hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(mean), hip.ptr(std), hip.ptr(acc),
                                   hip.ptr(hist)))
    return dict(n=nn.value, mean=mean, std=std, acc=acc, hist=hist)


@pytest.mark.timeout(900)
def test_headline_pipeline_fullsize(L):
    import torch

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.synth import synth_exact_host
    H, W, N = 2160, 2560, 128
    seed, channel, first = 2026, 1, 1000
    npx = H * W
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    d_in, d_out = Dev(L, N * npx * 2), Dev(L, N * npx * 2)
    planes = [Dev(L, npx * 8) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    hip.check(L.tmh_synth_sites_device(d_in.p, N, H, W, seed, channel, first,
                                       hip.TMH_SYNTH_STANDARD, sp))
    h = _stats_handle(L, H, W, hip.TMH_STATS_KEEP_SITE_HIST)
    hip.check(L.tmh_stats_set_stream(h, sp))
    c = C.c_void_p()
    L.tmh_synchronize(None)
    hip.check(L.tmh_corrector_create_device(mean.p, std.p, H, W, 1, ZERO_LOG10, sp, C.byref(c)))

    def job():  # bench.py Channel.stats() + Channel.apply(), same calls, same stream
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_device(h, d_in.p, N, 1, sp))
        hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, sp))
        hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_corrector_update_device(c, smean.p, sstd.p, sp))
        hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, N, -1, -1, sp))
        return _results(L, h, H, W, N)

    r1 = job()  # the production launch shapes (one Welford site part)
    out1 = d_out.get(np.uint16, (N, npx))[::37].copy()
    # the second job on the same handle (bench warm-up -> timed) with the
    # Welford launch split into 4 site parts (32 full-size sites each) + merge
    hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_WELFORD_PARTS, 4))
    r = job()
    assert np.array_equal(r["acc"], r1["acc"]) and np.array_equal(r["hist"], r1["hist"])
    site_hist = {}
    for i in (0, 63, N - 1):
        sh = np.empty(65536, np.uint32)
        hip.check(L.tmh_stats_site_histogram(h, i, hip.ptr(sh)))
        site_hist[i] = sh
    order_stats = site_order_stats(L, h, (0, 63, N - 1), 100000)
    sites = d_in.get(np.uint16, (N, H, W))
    out = d_out.get(np.uint16, (N, H, W))
    assert np.array_equal(out.reshape(N, npx)[::37], out1), "fused pass not repeatable"
    gm, gs = smean.get(np.float64, (H, W)), sstd.get(np.float64, (H, W))
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    for b in planes + [d_in, d_out]:
        b.free()

    # the device generator is the bench's input: its host twin is bit-identical
    for i in (0, N - 1):
        assert np.array_equal(sites[i], synth_exact_host(H, W, seed, channel, first + i))
    ref = orc.OracleOnlineStatistics((H, W))
    pooled = np.zeros(65536, np.uint64)
    for i, s in enumerate(sites):
        ref.update(s)
        hs = orc.histogram_u16(s)
        pooled += hs
        if i in site_hist:
            assert np.array_equal(site_hist[i].astype(np.uint64), hs), "site %d histogram" % i
    assert r["n"] == r1["n"] == ref.n == N
    for res in (r1, r):  # one part, four parts
        assert_close_rel(res["mean"], ref.mean)
        assert_close_rel(res["std"], ref.std)
    check_order_stats([sites[i] for i in (0, 63, N - 1)], order_stats)
    assert np.array_equal(r["hist"], pooled), "pooled histogram not bit-exact"
    assert np.array_equal(r["acc"], ref.percentile_sums), "percentile sums not bit-exact"
    sm_ref, ss_ref = orc.smooth_reflect(ref.mean, 5), orc.smooth_reflect(ref.std, 5)
    assert_close_rel(gm, sm_ref)
    assert_close_rel(gs, ss_ref)
    tot = pm1 = 0
    for i in list(range(0, N, 16)) + [N - 1]:
        want = orc.correct_illumination(sites[i], sm_ref, ss_ref)
        worst, flips, n1 = dn_report(out[i], want)
        assert worst <= 1, "site %d: %d DN" % (i, worst)
        assert flips == 0, "site %d: %d wrap flips" % (i, flips)
        tot += want.size
        pm1 += n1
    print("fullsize headline pipeline: %d sites, +-1 DN pixels %.4f%%, wrap flips 0"
          % (N, 100.0 * pm1 / tot))


@pytest.mark.timeout(600)
def test_bright_fullsize(L):
    """bright 16-bit data (lognormal(8.5, 0.6), about a third
    of the pixels >= 4,096) at full size.  The Welford pass takes its wide
    log10 path for most pixel groups and counts them; the automatic fused
    configuration then runs kFusedWide: four sites per unit, 16,384 bins each
    as u16 counters packed two sites to a word (4, 1024, 65536; the flush's
    wrap check is exercised by test_packed_counters_wrap).  The same job with
    the narrow slices forced (global
    adds for every pixel >= 4,096) must give identical results, and both
    match the oracle.  (64 sites: below the 96 the bright Welford pass needs,
    so this covers the standard pass's rare log10 path; tests/test_gpu_blocked.py
    runs 100 bright sites through the bright pass and its 20,472-entry table.)"""
    import torch

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.synth import BRIGHT, synth_exact_host
    H, W, N = 2160, 2560, 64
    seed, channel, first = 4242, 2, 0
    npx = H * W
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    d_in, d_out = Dev(L, N * npx * 2), Dev(L, N * npx * 2)
    planes = [Dev(L, npx * 8) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    hip.check(L.tmh_synth_sites_device(d_in.p, N, H, W, seed, channel, first, hip.TMH_SYNTH_BRIGHT, sp))
    h = _stats_handle(L, H, W, hip.TMH_STATS_KEEP_SITE_HIST)
    hip.check(L.tmh_stats_set_stream(h, sp))
    c = C.c_void_p()
    L.tmh_synchronize(None)
    hip.check(L.tmh_corrector_create_device(mean.p, std.p, H, W, 1, ZERO_LOG10, sp, C.byref(c)))
    wide = []

    def job():
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_device(h, d_in.p, N, 1, sp))
        wg = C.c_uint64()
        hip.check(L.tmh_stats_wide_groups(h, C.byref(wg), None))
        wide.append(wg.value)
        hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, sp))
        hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_corrector_update_device(c, smean.p, sstd.p, sp))
        hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, N, -1, -1, sp))
        return _results(L, h, H, W, N)

    r = job()  # automatic: wide
    pc, wb, fc = (C.c_uint32 * 3)(), C.c_int(), C.c_int()
    hip.check(L.tmh_stats_job_choice(h, pc, C.byref(wb), C.byref(fc)))
    assert wb.value == 1 and fc.value == 5, (list(pc), wb.value, fc.value)  # bright: both choices
    out_auto = d_out.get(np.uint16, (N, npx))
    hist0 = np.empty(65536, np.uint32)
    hip.check(L.tmh_stats_site_histogram(h, 0, hip.ptr(hist0)))
    hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_FUSED_CONFIG, 3))  # narrow, forced
    rn = job()
    assert np.array_equal(d_out.get(np.uint16, (N, npx)), out_auto)
    assert np.array_equal(rn["acc"], r["acc"]) and np.array_equal(rn["hist"], r["hist"])
    assert np.array_equal(rn["mean"], r["mean"]) and np.array_equal(rn["std"], r["std"])
    sites = d_in.get(np.uint16, (N, H, W))
    gm, gs = smean.get(np.float64, (H, W)), sstd.get(np.float64, (H, W))
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    for b in planes + [d_in, d_out]:
        b.free()

    for i in (0, N - 1):
        assert np.array_equal(sites[i], synth_exact_host(H, W, seed, channel, first + i, BRIGHT))
    assert wide[0] == wide[1] == _wide_groups(sites)
    assert wide[0] >= 0.02 * N * npx // 8, wide[0] / (N * npx // 8)
    ref = orc.OracleOnlineStatistics((H, W))
    pooled = np.zeros(65536, np.uint64)
    for s in sites:
        ref.update(s)
        pooled += orc.histogram_u16(s)
    assert np.array_equal(hist0.astype(np.uint64), orc.histogram_u16(sites[0]))
    assert_close_rel(r["mean"], ref.mean)
    assert_close_rel(r["std"], ref.std)
    assert np.array_equal(r["hist"], pooled)
    assert np.array_equal(r["acc"], ref.percentile_sums)
    sm_ref, ss_ref = orc.smooth_reflect(ref.mean, 5), orc.smooth_reflect(ref.std, 5)
    assert_close_rel(gm, sm_ref)
    assert_close_rel(gs, ss_ref)
    for i in (0, N // 2, N - 1):
        want = orc.correct_illumination(sites[i], sm_ref, ss_ref)
        worst, flips, _ = dn_report(out_auto.reshape(N, H, W)[i], want)
        assert worst <= 1 and flips == 0, (i, worst, flips)


def _job_sites(k, n, H, W, dist=0):
    """Job k's sites: synthetic plus high values in job-specific 1,024-bin
    rounds (beyond every configuration's LDS slice) and saturated pixels."""
    from tmlibrary_amd.synth import synth_exact_host
    sites = np.stack([synth_exact_host(H, W, 77 + k, 0, i, dist) for i in range(n)])
    hi_vals = [(40000, 65535), (20000, 5000), (60000, 12345)][k % 3]
    sites[0, :3, :40] = hi_vals[0]
    sites[n // 2, 5, :17] = hi_vals[1]
    sites[n - 1, -1, -9:] = hi_vals[0] + 1024
    return sites


def _wide_groups(sites):
    """8-pixel groups (row-major, per site) holding a value >= 4,096."""
    g = sites.reshape(sites.shape[0], -1, 8)
    return int(np.count_nonzero((g >= 4096).any(axis=2)))


@pytest.mark.parametrize("cfg", [-1, 0, 1, 2, 3, 4, 5])
def test_fused_multi_job_configs(L, cfg):
    """cfg -1 is the automatic choice: job 1 is bright (lognormal(8.5, 0.6)),
    so the Welford count must select the wide configuration for it, and the
    synthetic jobs around it the narrow one."""
    import torch

    from tmlibrary_amd import hip, synth
    from tmlibrary_amd.image import ZERO_LOG10
    H, W, n = 240, 320, 9
    npx = H * W
    dev = torch.device("cuda", 0)
    s_stats, s_corr = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    sp1, sp2 = C.c_void_p(s_stats.cuda_stream), C.c_void_p(s_corr.cuda_stream)
    h = _stats_handle(L, H, W, hip.TMH_STATS_KEEP_SITE_HIST)
    hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_FUSED_CONFIG, cfg))
    hip.check(L.tmh_stats_set_stream(h, sp1))
    d_in, d_out = Dev(L, n * npx * 2), Dev(L, n * npx * 2)
    planes = [Dev(L, npx * 8) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    c = C.c_void_p()  # its stream is stream 2; coefficients come from each job below
    L.tmh_synchronize(None)
    hip.check(L.tmh_corrector_create_device(mean.p, std.p, H, W, 1, ZERO_LOG10, sp2, C.byref(c)))
    L.tmh_synchronize(None)
    for k in range(3):
        bright = cfg == -1 and k == 1
        sites = _job_sites(k, n, H, W, synth.BRIGHT if bright else synth.STANDARD)
        d_in.put(sites)
        # one job, no host synchronisation: statistics on stream 1, the
        # fused pass on stream 2 (tmh_correct_u16_hist_device orders itself
        # after stream 1 and makes stream 1 wait for it)
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_device(h, d_in.p, n, 1, None))
        hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, None))
        hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, sp1))
        hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, sp1))
        hip.check(L.tmh_corrector_update_device(c, smean.p, sstd.p, sp1))
        wg, ws = C.c_uint64(), C.c_int64()
        hip.check(L.tmh_stats_wide_groups(h, C.byref(wg), C.byref(ws)))
        groups = n * npx // 8
        assert ws.value == n
        assert wg.value == _wide_groups(sites), (cfg, k)
        if cfg == -1:  # the automatic choice's threshold: 2 % of the groups
            assert (wg.value >= 0.02 * groups) == bright, (k, wg.value / groups)
        # the configuration the job runs, chosen on the host from its site probe
        pc, wb, fc = (C.c_uint32 * 3)(), C.c_int(), C.c_int()
        hip.check(L.tmh_stats_job_choice(h, pc, C.byref(wb), C.byref(fc)))
        assert pc[0] == 16384 and wb.value == int(bright), (cfg, k, list(pc), wb.value)
        assert fc.value == (cfg if cfg >= 0 else (5 if bright else 3)), (cfg, k, fc.value)
        hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, n, -1, -1, None))
        r = _results(L, h, H, W, n)  # on stream 1: waits for stream 2's fused pass
        hip.check(L.tmh_stats_wide_groups(h, C.byref(wg), C.byref(ws)))
        assert wg.value == 0 and ws.value == 0  # consumed by the fused pass
        ref = orc.run_illumstats(list(sites))
        assert r["n"] == n
        assert_close_rel(r["mean"], ref.mean)
        assert np.array_equal(r["acc"], ref.percentile_sums), (cfg, k)
        assert np.array_equal(r["hist"], sum(orc.histogram_u16(s) for s in sites)), (cfg, k)
        for i in range(n):
            sh = np.empty(65536, np.uint32)
            hip.check(L.tmh_stats_site_histogram(h, i, hip.ptr(sh)))
            assert np.array_equal(sh.astype(np.uint64), orc.histogram_u16(sites[i])), (cfg, k, i)
        out = d_out.get(np.uint16, sites.shape)
        sm_ref, ss_ref = orc.smooth_reflect(ref.mean, 5), orc.smooth_reflect(ref.std, 5)
        for i in (0, n - 1):
            worst, flips, _ = dn_report(out[i], orc.correct_illumination(sites[i], sm_ref, ss_ref))
            assert worst <= 1 and flips == 0, (cfg, k, i, worst, flips)
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    for b in planes + [d_in, d_out]:
        b.free()


def _groups_ge(sites, v):
    """8-pixel groups (row-major, per site) holding a value >= v."""
    g = sites.reshape(sites.shape[0], -1, 8)
    return int(np.count_nonzero((g >= v).any(axis=2)))


@pytest.mark.parametrize("cfg", [-1, 3, 5])
def test_very_wide_jobs(L, cfg):
    """Very wide sites (a third or more of the 8-pixel groups hold a value
    >= 16,384): with the automatic configuration the fused pass runs without
    its histogram and k_hist_site_u16 builds the exact per-site histograms in
    LDS as u16 pairs from one more read of the sites.  Job 0 is uniform
    0..65535; job 1 adds a value held by more than 65,535 pixels of one site,
    two values sharing one u16 pair held by 45,000 pixels each, a hot upper
    half (each half spills 16,384 counts at a time to the global slab) and
    the extremes 0 / 65535.  cfg 3 forces the narrow slices
    (every value >= 4,096 by global atomics) on the same jobs.  Histograms,
    order statistics and percentile sums bit-exact, mean/std 1e-6, corrected
    values within 1 DN of the oracle (stats.py:64-121, image.py:599-631)."""
    import torch

    from tmlibrary_amd import hip, synth
    from tmlibrary_amd.image import ZERO_LOG10
    H, W, n = 288, 320, 6  # 92,160 pixels per site: room for a 70,000-pixel value
    npx = H * W
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    h = _stats_handle(L, H, W, hip.TMH_STATS_KEEP_SITE_HIST)
    hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_FUSED_CONFIG, cfg))
    hip.check(L.tmh_stats_set_stream(h, sp))
    d_in, d_out = Dev(L, n * npx * 2), Dev(L, n * npx * 2)
    planes = [Dev(L, npx * 8) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    c = C.c_void_p()
    L.tmh_synchronize(None)
    hip.check(L.tmh_corrector_create_device(mean.p, std.p, H, W, 1, ZERO_LOG10, sp, C.byref(c)))
    L.tmh_synchronize(None)
    for k in range(2):
        sites = np.stack([synth.synth_exact_host(H, W, 91 + k, 1, i, synth.UNIFORM)
                          for i in range(n)])
        if k == 1:
            sites[2].reshape(-1)[:70000] = 30000  # one bin beyond 65,535 pixels
            sites[3].reshape(-1)[:5] = 0
            sites[4].reshape(-1)[-7:] = 65535
            # both halves of one u16 pair hot at once (45,000 pixels each,
            # interleaved), and a hot upper half alone
            sites[1].reshape(-1)[:90000] = 40000 + np.arange(90000, dtype=np.uint16) % 2
            sites[5].reshape(-1)[:50000] = 12345
        d_in.put(sites)
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_device(h, d_in.p, n, 1, sp))
        hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, sp))
        hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_corrector_update_device(c, smean.p, sstd.p, sp))
        assert _groups_ge(sites, 16384) >= 0.33 * n * npx // 8  # very wide
        hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, n, -1, -1, sp))
        r = _results(L, h, H, W, n)
        ref = orc.run_illumstats(list(sites))
        assert r["n"] == n
        assert_close_rel(r["mean"], ref.mean)
        assert_close_rel(r["std"], ref.std)
        assert np.array_equal(r["hist"], sum(orc.histogram_u16(s) for s in sites)), (cfg, k)
        assert np.array_equal(r["acc"], ref.percentile_sums), (cfg, k)
        for i in range(n):
            sh = np.empty(65536, np.uint32)
            hip.check(L.tmh_stats_site_histogram(h, i, hip.ptr(sh)))
            assert np.array_equal(sh.astype(np.uint64), orc.histogram_u16(sites[i])), (cfg, k, i)
        check_order_stats([sites[i] for i in (0, 2)], site_order_stats(L, h, (0, 2), 100000))
        out = d_out.get(np.uint16, sites.shape)
        sm_ref, ss_ref = orc.smooth_reflect(ref.mean, 5), orc.smooth_reflect(ref.std, 5)
        for i in (0, 2, n - 1):
            worst, flips, _ = dn_report(out[i], orc.correct_illumination(sites[i], sm_ref, ss_ref))
            assert worst <= 1 and flips == 0, (cfg, k, i, worst, flips)
    # the slab is zero-maintained: a third job on the same handle starts clean
    sites = np.stack([synth.synth_exact_host(H, W, 99, 1, i, synth.STANDARD) for i in range(n)])
    d_in.put(sites)
    hip.check(L.tmh_stats_reset(h))
    hip.check(L.tmh_stats_update_welford_device(h, d_in.p, n, 1, sp))
    hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, sp))
    hip.check(L.tmh_corrector_update_device(c, mean.p, std.p, sp))
    hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, n, -1, -1, sp))
    r = _results(L, h, H, W, n)
    assert np.array_equal(r["hist"], sum(orc.histogram_u16(s) for s in sites))
    assert np.array_equal(r["acc"], orc.run_illumstats(list(sites)).percentile_sums)
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    for b in planes + [d_in, d_out]:
        b.free()


def test_packed_counters_wrap(L):
    """Fused configuration 5 (four sites per unit, u16 LDS counters packed two
    sites to a word, 8 bands): at 768 x 768 a band holds 73,728 pixels of a
    site, so a value filling a band wraps its 16-bit counter.  The flush's
    per-site sum check must catch it and recount the band from the pixels:
    sites of one value (5,000 and 16,383, the top LDS bin), a half-constant
    bright site, a bright site, and a site with a value >= 16,384 in every
    pixel group.  Per-site histograms, percentile sums bit-exact; mean/std
    1e-6 (stats.py:64-121)."""
    from tmlibrary_amd import hip, synth
    H, W, n = 768, 768, 5
    npx = H * W
    sites = np.stack([synth.synth_exact_host(H, W, 5 + i, 0, i, synth.BRIGHT) for i in range(n)])
    sites[0] = 5000
    sites[1] = 16383
    sites[2, : H // 2] = 3000
    sites[4, :, ::8] = 40000
    h = _stats_handle(L, H, W, hip.TMH_STATS_KEEP_SITE_HIST)
    hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_FUSED_CONFIG, 5))
    d_in, d_out = Dev(L, n * npx * 2), Dev(L, n * npx * 2)
    planes = [Dev(L, npx * 8) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    from tmlibrary_amd.image import ZERO_LOG10
    c = C.c_void_p()
    L.tmh_synchronize(None)
    hip.check(L.tmh_corrector_create_device(mean.p, std.p, H, W, 1, ZERO_LOG10, None, C.byref(c)))
    d_in.put(sites)
    hip.check(L.tmh_stats_reset(h))
    hip.check(L.tmh_stats_update_welford_device(h, d_in.p, n, 1, None))
    hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, None))
    hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, None))
    hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, None))
    hip.check(L.tmh_corrector_update_device(c, smean.p, sstd.p, None))
    hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, n, -1, -1, None))
    r = _results(L, h, H, W, n)
    ref = orc.run_illumstats(list(sites))
    assert r["n"] == n
    assert_close_rel(r["mean"], ref.mean)
    for i in range(n):
        sh = np.empty(65536, np.uint32)
        hip.check(L.tmh_stats_site_histogram(h, i, hip.ptr(sh)))
        assert np.array_equal(sh.astype(np.uint64), orc.histogram_u16(sites[i])), i
    assert np.array_equal(r["hist"], sum(orc.histogram_u16(s) for s in sites))
    assert np.array_equal(r["acc"], ref.percentile_sums)
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    for b in planes + [d_in, d_out]:
        b.free()
