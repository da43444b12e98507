"""GPU: the blocked site layout gives the contiguous layout's results.

tmh_stats_update_welford_blocks_device / tmh_correct_u16_hist_blocks_device
take the sites (and the corrected outputs) as blocks of 2^shift consecutive
sites in separate allocations -- how sites arrive in the reference (one file
per site, tmlib/workflow/corilla/api.py:131-136) and how bench.py now lays a
job out in HBM (placement).  Every kernel that touches the
sites takes the block table: the Welford pass (and its bright-site probe and
site split), the fused correct + histogram pass in each configuration (narrow,
wide, the very-wide no-histogram form + the u16 LDS histogram pass) and the
f64 refinement.  The same job on the same pixels must give bit-identical
statistics, histograms, percentile sums and corrected pixels in both layouts,
and match the oracle (stats.py:64-121, image.py:599-631).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import corilla_oracle as orc
from util import assert_close_rel, dn_report

pytestmark = pytest.mark.gpu


def _job(L, torch, H, W, sites_np, shift, cfg=-1, order_seed=0):
    """Run one job (bench.py's call sequence) with the sites contiguous
    (shift None) or in blocks of 2^shift sites allocated in shuffled order;
    returns (results dict, corrected sites)."""
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    n = sites_np.shape[0]
    npx = H * W
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    src = torch.from_numpy(sites_np.view(np.int16)).to(dev)
    if shift is None:
        d_in, d_out = src, torch.empty_like(src)
    else:
        B = 1 << shift
        nb = (n + B - 1) // B
        rng = np.random.default_rng(order_seed)
        blocks_in, blocks_out = [None] * nb, [None] * nb
        for b in rng.permutation(nb):  # allocation order unrelated to site order
            m = min(B, n - b * B)
            blocks_in[b] = src[b * B:b * B + m].clone()
            blocks_out[b] = torch.empty((m, H, W), dtype=torch.int16, device=dev)
        t_in = torch.tensor([t.data_ptr() for t in blocks_in], dtype=torch.int64, device=dev)
        t_out = torch.tensor([t.data_ptr() for t in blocks_out], dtype=torch.int64, device=dev)
    lo, hi, gamma = quantile_table(npx, np.linspace(0, 100, 100000))
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, 100000, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 1, 0, C.byref(h)))
    hip.check(L.tmh_stats_set_stream(h, sp))
    hip.check(L.tmh_stats_set_option(h, hip.TMH_OPT_FUSED_CONFIG, cfg))
    planes = [torch.empty(npx, dtype=torch.float64, device=dev) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    c = C.c_void_p()
    torch.cuda.synchronize(dev)
    hip.check(L.tmh_corrector_create_device(p(mean), p(std), H, W, 1, ZERO_LOG10, sp, C.byref(c)))
    hip.check(L.tmh_stats_reset(h))
    if shift is None:
        hip.check(L.tmh_stats_update_welford_device(h, p(d_in), n, 1, sp))
    else:
        hip.check(L.tmh_stats_update_welford_blocks_device(h, p(t_in), shift, n, 1, sp))
    hip.check(L.tmh_stats_finalize_device(h, p(mean), p(std), sp))
    hip.check(L.tmh_smooth_f64_device(p(mean), p(smean), p(tmp), H, W, 5.0, sp))
    hip.check(L.tmh_smooth_f64_device(p(std), p(sstd), p(tmp), H, W, 5.0, sp))
    hip.check(L.tmh_corrector_update_device(c, p(smean), p(sstd), sp))
    if shift is None:
        hip.check(L.tmh_correct_u16_hist_device(c, h, p(d_in), p(d_out), n, -1, -1, sp))
    else:
        hip.check(L.tmh_correct_u16_hist_blocks_device(c, h, p(t_in), p(t_out), shift, n, -1, -1,
                                                       sp))
    nn = C.c_int64()
    r = {"mean": np.empty(npx), "std": np.empty(npx), "acc": np.empty(100000),
         "hist": np.empty(65536, np.uint64)}
    hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(r["mean"]), hip.ptr(r["std"]),
                                   hip.ptr(r["acc"]), hip.ptr(r["hist"])))
    r["n"] = nn.value
    r["smean"], r["sstd"] = smean.cpu().numpy(), sstd.cpu().numpy()
    out = d_out if shift is None else torch.cat(blocks_out)
    corrected = out.cpu().numpy().view(np.uint16).reshape(n, H, W)
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    return r, corrected


@pytest.mark.parametrize("kind,n,shift,cfg", [
    ("synthetic", 37, 2, -1),   # ragged last block (1 site), narrow configuration
    ("bright", 100, 2, -1),     # probe -> 3 Welford parts, wide configuration (2 sites/unit)
    ("synthetic", 100, 6, 1),   # 64-site blocks, a forced 4-site / 32,768-bin configuration
    ("uniform", 13, 3, -1),     # very wide: no-histogram fused pass + u16 LDS histograms
])
def test_blocked_equals_contiguous(kind, n, shift, cfg):
    import torch

    from tmlibrary_amd import hip, synth
    L = hip.lib()
    H, W = 96, 128
    dist = synth.DISTRIBUTIONS[kind]
    sites = np.stack([synth.synth_exact_host(H, W, 515, 3, i, dist) for i in range(n)])
    sites[n - 1, 0, :5] = 0          # zero pixels (the correction's log10(1e-10) floor)
    sites[0, -1, -3:] = 65535        # saturated pixels (f64 refinement candidates)
    rc, oc = _job(L, torch, H, W, sites, None, cfg)
    rb, ob = _job(L, torch, H, W, sites, shift, cfg, order_seed=n)
    for k in ("n", "mean", "std", "acc", "hist", "smean", "sstd"):
        assert np.array_equal(rc[k], rb[k]), "blocked layout differs in %s" % k
    assert np.array_equal(oc, ob), "blocked layout differs in the corrected sites"
    ref = orc.run_illumstats(list(sites))
    assert rb["n"] == n
    assert_close_rel(rb["mean"].reshape(H, W), ref.mean)
    assert_close_rel(rb["std"].reshape(H, W), ref.std)
    assert np.array_equal(rb["acc"], ref.percentile_sums)
    assert np.array_equal(rb["hist"], sum(orc.histogram_u16(s) for s in sites))
    sm, ss = orc.smooth_reflect(ref.mean, 5), orc.smooth_reflect(ref.std, 5)
    for i in (0, n // 2, n - 1):
        worst, flips, _ = dn_report(ob[i], orc.correct_illumination(sites[i], sm, ss))
        assert worst <= 1 and flips == 0, (kind, i, worst, flips)


def test_blocked_argument_checks():
    import torch

    from tmlibrary_amd import hip
    L = hip.lib()
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    H, W = 30, 30  # 900 pixels: not a multiple of 8
    lo, hi, gamma = quantile_table(H * W, np.linspace(0, 100, 1000))
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, 1000, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 1, 0, C.byref(h)))
    tab = torch.zeros(4, dtype=torch.int64, device="cuda")
    tp = C.c_void_p(tab.data_ptr())
    with pytest.raises(ValueError, match="divisible by 8"):
        hip.check(L.tmh_stats_update_welford_blocks_device(h, tp, 2, 4, 1, None))
    with pytest.raises(ValueError, match="block_shift"):
        hip.check(L.tmh_stats_update_welford_blocks_device(h, tp, 1, 4, 1, None))
    with pytest.raises(ValueError, match="NULL"):
        hip.check(L.tmh_stats_update_welford_blocks_device(h, None, 2, 4, 1, None))
    L.tmh_stats_destroy(h)
