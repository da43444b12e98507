"""The multi-job planes step (tmh_job_planes_multi_device) and batched
coefficients (tmh_corrector_update_multi_device) against the per-job calls.

A rank's channels (configs[2]/[3]; reference: one corilla job per channel,
tmlib/workflow/corilla/api.py:64-105) each finalize their statistics
(stats.py:94-112), smooth mean and std (image.py:1172-1193) and derive the
correction's coefficients (image.py:599-631).  The multi-job entry does all
jobs in one launch per kernel, finalizing std as the smoothing reads M2;
results must be BIT-identical to finalize + smooth2 + corrector update per
job -- unsmoothed and smoothed planes, the correctors' global means and the
corrected pixels -- for sigma 5 (one-pass smoothing) and another sigma
(finalize into scratch, two passes), and for a job of one site (std NaN).
The jobs' corrected passes share one fused launch
(tmh_correct_u16_hist_multi_device): per-site histograms, percentile sums and
corrected pixels bit-identical to one launch per job.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import corilla_oracle as orc
from test_gpu_parity import Dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from tmlibrary_amd import hip
    return hip.lib()


def _handle(L, H, W):
    from tmlibrary_amd import hip
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    lo, hi, gamma = quantile_table(H * W, np.linspace(0, 100, 1000))
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, len(lo), hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 4, 0, C.byref(h)))
    return h


@pytest.mark.parametrize("sigma,ns", [(5.0, (7, 5, 9)), (2.5, (6, 4)), (5.0, (1, 6))])
def test_job_planes_multi_bit_identical(L, sigma, ns):
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.synth import synth_exact_host
    H, W = 200, 264
    npx = H * W
    n = len(ns)
    sites = [np.stack([synth_exact_host(H, W, 70 + j, j, i, 0) for i in range(k)])
             for j, k in enumerate(ns)]
    d_in = [Dev(L, s.nbytes) for s in sites]
    d_out = [Dev(L, s.nbytes) for s in sites]
    for d, s in zip(d_in, sites):
        d.put(s)
    res = {}
    for mode in ("per-job", "multi"):
        hs = [_handle(L, H, W) for _ in range(n)]
        pl = [[Dev(L, npx * 8) for _ in range(6)] for _ in range(n)]  # mean std smean sstd t t2
        cs = []
        L.tmh_synchronize(None)
        for j in range(n):
            c = C.c_void_p()
            hip.check(L.tmh_corrector_create_device(pl[j][0].p, pl[j][1].p, H, W, 1, ZERO_LOG10,
                                                    None, C.byref(c)))
            cs.append(c)
        L.tmh_synchronize(None)
        for j in range(n):
            hip.check(L.tmh_stats_reset(hs[j]))
            hip.check(L.tmh_stats_update_welford_device(hs[j], d_in[j].p, ns[j], 1, None))
        if mode == "per-job":
            for j in range(n):
                m, sd, sm, ss, t, t2 = pl[j]
                hip.check(L.tmh_stats_finalize_device(hs[j], m.p, sd.p, None))
                L.tmh_synchronize(None)  # handle's stream -> null stream
                hip.check(L.tmh_smooth2_f64_device(m.p, sd.p, sm.p, ss.p, t.p, t2.p, H, W, sigma,
                                                   None))
                hip.check(L.tmh_corrector_update_device(cs[j], sm.p, ss.p, None))
        else:
            arr = lambda xs: (C.c_void_p * n)(*xs)  # noqa: E731
            hip.check(L.tmh_job_planes_multi_device(
                arr([h.value for h in hs]), arr([c.value for c in cs]), n,
                arr([pl[j][0].p for j in range(n)]), arr([pl[j][1].p for j in range(n)]),
                arr([pl[j][2].p for j in range(n)]), arr([pl[j][3].p for j in range(n)]),
                sigma, None))
        L.tmh_synchronize(None)
        out = []
        for j in range(n):
            ms, mm = C.c_double(), C.c_double()
            hip.check(L.tmh_corrector_means(cs[j], C.byref(ms), C.byref(mm)))
            hip.check(L.tmh_correct_u16_device(cs[j], d_in[j].p, d_out[j].p, ns[j], -1, -1, None))
            L.tmh_synchronize(None)
            out.append({"planes": [pl[j][k].get(np.float64, (H, W)) for k in range(4)],
                        "means": (ms.value, mm.value),
                        "corrected": d_out[j].get(np.uint16, sites[j].shape)})
        res[mode] = out
        for c in cs:
            L.tmh_corrector_destroy(c)
        for h in hs:
            L.tmh_stats_destroy(h)
        for p in pl:
            for d in p:
                d.free()
    for j in range(n):
        a, b = res["per-job"][j], res["multi"][j]
        for k in range(4):  # mean, std, smoothed mean, smoothed std: bit for bit (NaN too)
            assert np.array_equal(a["planes"][k], b["planes"][k], equal_nan=True), (j, k)
        assert np.array_equal(a["means"], b["means"], equal_nan=True), (a["means"], b["means"])
        assert np.array_equal(a["corrected"], b["corrected"]), j
    if ns[0] == 1:
        assert np.isnan(res["multi"][0]["planes"][1]).all()  # one site: std is NaN (stats.py:108)
    for d in d_in + d_out:
        d.free()


def test_corrector_update_multi_equals_single(L):
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    H, W, n = 120, 160, 3
    npx = H * W
    rng = np.random.default_rng(3)
    planes = [(rng.uniform(1, 3, npx), rng.uniform(0.05, 0.3, npx)) for _ in range(n)]
    dev = [(Dev(L, npx * 8), Dev(L, npx * 8)) for _ in range(n)]
    for (m, s), (dm, ds) in zip(planes, dev):
        dm.put(m)
        ds.put(s)
    site = rng.integers(0, 4000, (2, H, W)).astype(np.uint16)
    d_in, d_out = Dev(L, site.nbytes), Dev(L, site.nbytes)
    d_in.put(site)
    got = {}
    for mode in ("single", "multi"):
        cs = []
        for dm, ds in dev:
            c = C.c_void_p()
            hip.check(L.tmh_corrector_create_device(dm.p, ds.p, H, W, 1, ZERO_LOG10, None,
                                                    C.byref(c)))
            cs.append(c)
        # shift every job's planes, then recompute the coefficients
        for j, (dm, ds) in enumerate(dev):
            dm.put(planes[j][0] + 0.1 * (j + 1))
        if mode == "single":
            for c, (dm, ds) in zip(cs, dev):
                hip.check(L.tmh_corrector_update_device(c, dm.p, ds.p, None))
        else:
            arr = lambda xs: (C.c_void_p * n)(*xs)  # noqa: E731
            hip.check(L.tmh_corrector_update_multi_device(arr([c.value for c in cs]), n,
                                                          arr([d[0].p for d in dev]),
                                                          arr([d[1].p for d in dev]), None))
        L.tmh_synchronize(None)
        outs = []
        for c in cs:
            hip.check(L.tmh_correct_u16_device(c, d_in.p, d_out.p, 2, -1, -1, None))
            L.tmh_synchronize(None)
            outs.append(d_out.get(np.uint16, site.shape))
            L.tmh_corrector_destroy(c)
        for j, (dm, ds) in enumerate(dev):
            dm.put(planes[j][0])
        got[mode] = outs
    for a, b in zip(got["single"], got["multi"]):
        assert np.array_equal(a, b)
    for dm, ds in dev:
        dm.free()
        ds.free()
    d_in.free()
    d_out.free()


@pytest.mark.parametrize("layout,streams", [("contiguous", "cross"), ("blocks", "cross"),
                                            ("contiguous", "own"), ("contiguous", "mixed")])
def test_correct_hist_multi_equals_per_job(L, layout, streams):
    """tmh_correct_u16_hist_multi(_blocks)_device against one
    tmh_correct_u16_hist(_blocks)_device per job: corrected pixels, per-site
    histograms, pooled histogram, order statistics (percentile sums) and
    moments bit for bit.  Jobs 0 and 2 share the narrow configuration (one
    launch); job 1 is bright (packed configuration: its own launch); job 3 is
    forced to the very wide configuration (histograms from a second read, no
    finalize in the batched histogram tail).  streams: the call's stream is
    none of the handles' streams (cross: the tails batched on the first
    handle's tail stream), all of them (own: batched on the call's stream), or
    only the first's (mixed: per-job tails)."""
    import torch

    from tmlibrary_amd import hip, synth
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    H, W = 216, 256
    npx = H * W
    ns = (9, 8, 5, 6)
    n = len(ns)
    kinds = (synth.STANDARD, synth.BRIGHT, synth.STANDARD, synth.STANDARD)
    sites = [np.stack([synth.synth_exact_host(H, W, 500 + j, j, i, kinds[j]) for i in range(k)])
             for j, k in enumerate(ns)]
    sites[1][:, :3, :40] = 60000  # values beyond the packed slices (rare lists)
    lo, hi, gamma = quantile_table(npx, np.linspace(0, 100, 1000))
    lut = stats_log10_lut()
    d_in = [Dev(L, s.nbytes) for s in sites]
    for d, s in zip(d_in, sites):
        d.put(s)
    shift = 2  # blocks of 4 sites
    dev = torch.device("cuda", 0)
    res = {}
    for mode in ("per-job", "multi"):
        d_out = [Dev(L, s.nbytes) for s in sites]
        hs, cs, planes = [], [], []
        ps = torch.cuda.Stream(dev)
        sp = C.c_void_p(ps.cuda_stream)
        for j in range(n):
            h = C.c_void_p()
            hip.check(L.tmh_stats_create(H, W, len(lo), hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                         hip.ptr(lut), 1, hip.TMH_STATS_KEEP_SITE_HIST,
                                         C.byref(h)))
            if streams == "own" or (streams == "mixed" and j == 0):
                hip.check(L.tmh_stats_set_stream(h, sp))
            if j == 3:
                hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_FUSED_CONFIG, 100))
            hs.append(h)
            planes.append([Dev(L, npx * 8) for _ in range(6)])
        L.tmh_synchronize(None)
        for j in range(n):
            c = C.c_void_p()
            hip.check(L.tmh_corrector_create_device(planes[j][0].p, planes[j][1].p, H, W, 1,
                                                    ZERO_LOG10, None, C.byref(c)))
            cs.append(c)
        tabs = []
        if layout == "blocks":
            for j in range(n):
                nb = (ns[j] + 3) >> shift
                ti = torch.tensor([d_in[j].p.value + b * 4 * npx * 2 for b in range(nb)],
                                  dtype=torch.int64, device=dev)
                to = torch.tensor([d_out[j].p.value + b * 4 * npx * 2 for b in range(nb)],
                                  dtype=torch.int64, device=dev)
                tabs.append((ti, to))
        L.tmh_synchronize(None)
        torch.cuda.synchronize()
        for j in range(n):
            m, sd, sm, ss, t, t2 = planes[j]
            hip.check(L.tmh_stats_reset(hs[j]))
            hip.check(L.tmh_stats_update_welford_device(hs[j], d_in[j].p, ns[j], 1, None))
            hip.check(L.tmh_stats_finalize_device(hs[j], m.p, sd.p, None))
            # (the handle's stream, the null stream and the corrector's: one
            # device synchronisation between them; the stream contract of the
            # corrected passes is what is under test below)
            L.tmh_synchronize(None)
            hip.check(L.tmh_smooth2_f64_device(m.p, sd.p, sm.p, ss.p, t.p, t2.p, H, W, 5.0, None))
            hip.check(L.tmh_corrector_update_device(cs[j], sm.p, ss.p, None))
            L.tmh_synchronize(None)
        arr = lambda xs: (C.c_void_p * n)(*[C.c_void_p(x) for x in xs])  # noqa: E731
        if mode == "per-job":
            for j in range(n):
                if layout == "blocks":
                    hip.check(L.tmh_correct_u16_hist_blocks_device(
                        cs[j], hs[j], C.c_void_p(tabs[j][0].data_ptr()),
                        C.c_void_p(tabs[j][1].data_ptr()), shift, ns[j], -1, -1, sp))
                else:
                    hip.check(L.tmh_correct_u16_hist_device(cs[j], hs[j], d_in[j].p, d_out[j].p,
                                                            ns[j], -1, -1, sp))
        else:
            nn = (C.c_int64 * n)(*ns)
            if layout == "blocks":
                hip.check(L.tmh_correct_u16_hist_multi_blocks_device(
                    arr([c.value for c in cs]), arr([h.value for h in hs]), n,
                    arr([t[0].data_ptr() for t in tabs]), arr([t[1].data_ptr() for t in tabs]),
                    shift, nn, -1, -1, sp))
            else:
                hip.check(L.tmh_correct_u16_hist_multi_device(
                    arr([c.value for c in cs]), arr([h.value for h in hs]), n,
                    arr([d.p.value for d in d_in]), arr([d.p.value for d in d_out]), nn, -1, -1, sp))
        cfg = []
        for j in range(n):
            fc = C.c_int()
            hip.check(L.tmh_stats_job_choice(hs[j], None, None, C.byref(fc)))
            cfg.append(fc.value)
        assert cfg == [3, 5, 3, 100], cfg
        L.tmh_synchronize(None)
        torch.cuda.synchronize()
        out = []
        for j in range(n):
            nn_ = C.c_int64()
            mean, std = np.empty(npx), np.empty(npx)
            acc = np.empty(len(lo))
            hist = np.empty(65536, np.uint64)
            hip.check(L.tmh_stats_finalize(hs[j], C.byref(nn_), hip.ptr(mean), hip.ptr(std),
                                           hip.ptr(acc), hip.ptr(hist)))
            sh = []
            for i in range(ns[j]):
                x = np.empty(65536, np.uint32)
                hip.check(L.tmh_stats_site_histogram(hs[j], i, hip.ptr(x)))
                sh.append(x)
            out.append({"n": nn_.value, "mean": mean, "std": std, "acc": acc, "hist": hist,
                        "site_hist": np.stack(sh),
                        "corrected": d_out[j].get(np.uint16, sites[j].shape)})
        res[mode] = out
        for c in cs:
            L.tmh_corrector_destroy(c)
        for h in hs:
            L.tmh_stats_destroy(h)
        for p in planes:
            for d in p:
                d.free()
        for d in d_out:
            d.free()
    for j in range(n):
        a, b = res["per-job"][j], res["multi"][j]
        assert a["n"] == b["n"] == ns[j]
        for k in ("mean", "std", "acc", "hist", "site_hist", "corrected"):
            if not np.array_equal(a[k], b[k], equal_nan=True):
                bad = np.argwhere(a[k] != b[k])
                raise AssertionError("job %d %s: %d of %d differ, first at %s (%s vs %s)" % (
                    j, k, len(bad), a[k].size, bad[0].tolist(), a[k][tuple(bad[0])],
                    b[k][tuple(bad[0])]))
        assert np.array_equal(b["hist"], sum(orc.histogram_u16(x) for x in sites[j])), j
        for i in (0, ns[j] - 1):
            assert np.array_equal(b["site_hist"][i].astype(np.uint64),
                                  orc.histogram_u16(sites[j][i])), (j, i)
    for d in d_in:
        d.free()
