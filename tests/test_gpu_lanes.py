"""The headline's default execution mode under -m gpu: two jobs in flight.

bench.py's default step alternates two job lanes -- each its
own statistics handle, corrector and stream -- and runs every corrected pass
on ONE stream shared by the lanes, so a job's histogram tail (order
statistics, ordered percentile sum) runs on its handle's tail stream while
the next job's Welford pass and corrected pass are already queued.  The
ordering that keeps the results exact (include/tmhip.h stream contract):
the corrected pass waits for everything queued on its handle's stream; the
handle's stream waits for the tail; a corrector whose previous tail is
still pending waits for it (``ev_tail``) before its next pass, because that
tail reads the corrector's round masks.

test_bench_two_lanes runs bench.py itself in that mode on 48 full-size sites
and requires every lane's last job to match the oracle fingerprint of the same
48 sites (tests/golden/make_bench_fingerprint.py).  test_corrector_tail_pending
drives the C-ABI directly: one corrector serves two statistics handles
back to back on a stream of its own, its second pass issued while the first
job's tail is still pending on another stream; both jobs' per-site histograms,
order statistics, pooled histograms and percentile sums must equal the
oracle's bit for bit (tmlib/workflow/corilla/stats.py:64-121).
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import corilla_oracle as orc
from test_gpu_parity import Dev, check_order_stats, site_order_stats
from util import assert_close_rel, dn_report

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from tmlibrary_amd import hip
    return hip.lib()


@pytest.mark.timeout(600)
def test_bench_two_lanes():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--sites", "48", "--steps",
                        "3", "--warmup", "1", "--no-extras", "--cpu-sample", "0"],
                       cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=540)
    assert r.returncode == 0, r.stderr.decode()[-4000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.strip()][-1])
    assert d["config"]["jobs_in_flight"] == 2 and d["config"]["jobs_order"] == "welford"
    chk = d["check"]
    assert d["check_vs_oracle"] is True, chk
    assert chk["vs_oracle"]["fingerprint"].endswith("s48_seed12345_c0_synthetic.npz")
    assert all(v for k, v in chk["vs_oracle"].items() if k != "fingerprint"), chk["vs_oracle"]
    lane = chk["lanes"]["lane1"]["vs_oracle"]
    assert all(v for k, v in lane.items() if k != "fingerprint"), lane
    for c in (chk, chk["lanes"]["lane1"]):
        assert c["n"] == 48
        assert c["corrected_vs_oracle"]["beyond_1DN"] == 0
        assert c["corrected_vs_oracle"]["wrap_flips"] == 0
    # one fused launch per job: the timed kernel is the configuration that ran
    assert d["kernels"]["correct_hist"]["launches"] == 3


def _handle(L, H, W):
    from tmlibrary_amd import hip
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    lo, hi, gamma = quantile_table(H * W, np.linspace(0, 100, 100000))
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, len(lo), hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 1, hip.TMH_STATS_KEEP_SITE_HIST, C.byref(h)))
    return h


@pytest.mark.timeout(600)
def test_corrector_tail_pending(L):
    import torch

    from tmlibrary_amd import hip, synth
    from tmlibrary_amd.image import ZERO_LOG10
    H, W, n = 540, 640, 24
    npx = H * W
    dev = torch.device("cuda", 0)
    s1, s2, sc = (torch.cuda.Stream(dev) for _ in range(3))
    sp1, sp2, spc = (C.c_void_p(s.cuda_stream) for s in (s1, s2, sc))
    # job 1 standard (narrow configuration), job 2 bright with high values in
    # other 1,024-bin rounds (packed configuration): a second pass that ran
    # before job 1's tail had read the corrector's round-mask union would
    # change job 1's pooled histogram or order statistics
    sites = [np.stack([synth.synth_exact_host(H, W, 910 + j, 0, i,
                                              synth.BRIGHT if j else synth.STANDARD)
                       for i in range(n)]) for j in range(2)]
    sites[1][0, :4, :50] = 61000
    sites[1][n - 1, -2, -30:] = 47000
    hs = [_handle(L, H, W), _handle(L, H, W)]
    for h, sp in zip(hs, (sp1, sp2)):
        hip.check(L.tmh_stats_set_stream(h, sp))
    d_in = [Dev(L, n * npx * 2) for _ in range(2)]
    d_out = [Dev(L, n * npx * 2) for _ in range(2)]
    for j in range(2):
        d_in[j].put(sites[j])
    planes = [[Dev(L, npx * 8) for _ in range(5)] for _ in range(2)]
    c = C.c_void_p()
    L.tmh_synchronize(None)
    hip.check(L.tmh_corrector_create_device(planes[0][0].p, planes[0][1].p, H, W, 1, ZERO_LOG10,
                                            spc, C.byref(c)))
    L.tmh_synchronize(None)
    cfgs = []
    for j, (h, sp) in enumerate(zip(hs, (sp1, sp2))):  # no host synchronisation in between
        mean, std, smean, sstd, tmp = planes[j]
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_device(h, d_in[j].p, n, 1, sp))
        hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, sp))
        hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, sp))
        hip.check(L.tmh_corrector_update_device(c, smean.p, sstd.p, sp))
        # the corrected pass on the corrector's own stream: cross-stream, so
        # this job's tail goes to h's tail stream and the pass of job 2 is
        # queued while job 1's tail is pending
        hip.check(L.tmh_correct_u16_hist_device(c, h, d_in[j].p, d_out[j].p, n, -1, -1, spc))
        fc = C.c_int()
        hip.check(L.tmh_stats_job_choice(h, None, None, C.byref(fc)))
        cfgs.append(fc.value)
    assert cfgs == [3, 5], cfgs
    for j, h in enumerate(hs):
        nn = C.c_int64()
        mean = np.empty((H, W))
        std = np.empty((H, W))
        acc = np.empty(100000)
        hist = np.empty(65536, np.uint64)
        hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(mean), hip.ptr(std), hip.ptr(acc),
                                       hip.ptr(hist)))
        ref = orc.run_illumstats(list(sites[j]))
        assert nn.value == n
        assert_close_rel(mean, ref.mean)
        assert_close_rel(std, ref.std)
        assert np.array_equal(acc, ref.percentile_sums), j
        assert np.array_equal(hist, sum(orc.histogram_u16(s) for s in sites[j])), j
        idx = (0, n // 2, n - 1)
        for i in idx:
            sh = np.empty(65536, np.uint32)
            hip.check(L.tmh_stats_site_histogram(h, i, hip.ptr(sh)))
            assert np.array_equal(sh.astype(np.uint64), orc.histogram_u16(sites[j][i])), (j, i)
        check_order_stats([sites[j][i] for i in idx], site_order_stats(L, h, idx, 100000))
        out = d_out[j].get(np.uint16, sites[j].shape)
        sm_ref, ss_ref = orc.smooth_reflect(ref.mean, 5), orc.smooth_reflect(ref.std, 5)
        for i in (0, n - 1):
            worst, flips, _ = dn_report(out[i], orc.correct_illumination(sites[j][i], sm_ref, ss_ref))
            assert worst <= 1 and flips == 0, (j, i, worst, flips)
    L.tmh_corrector_destroy(c)
    for h in hs:
        L.tmh_stats_destroy(h)
    for b in d_in + d_out + planes[0] + planes[1]:
        b.free()
