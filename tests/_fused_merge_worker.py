"""One rank of tests/test_gpu_two_process.py (not a test module itself).

Two processes share GPU 0 and form a gloo group; each runs bench.py's channel
job on its contiguous shard of the sites -- Channel.stats() / Channel.apply()
with the multi-GPU merges in between, i.e. a TMH_STATS_DEFERRED_PCT handle,
the site-split Welford pass, merge_welford (two all-reduces), finalize,
smoothing, coefficients, the FUSED correct + histogram pass, then
merge_counts (ordered percentile chain over quantile chunks + histogram
all-reduce) -- with the collectives staged through host memory
(sharded.HostStagedDist: RCCL needs one GPU per rank).  The job runs twice on
the same handles (bench warm-up, then the checked job) and the rank's results
go to <out_dir>/r<rank>.npz.

usage: python _fused_merge_worker.py OUT_DIR RANK WORLD PORT H W N SEED CHANNEL DIST
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(out_dir, rank, world, port, H, W, N, seed, channel, dist_id):
    import torch
    import torch.distributed as tdist

    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    from tmlibrary_amd.workflow.corilla.sharded import (HostStagedDist, StatsOps, merge_counts,
                                                         merge_welford, shard_bounds)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    sd = HostStagedDist(tdist)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)  # StatsOps and the staged copies order on it
    sp = C.c_void_p(stream.cuda_stream)
    L = hip.lib()
    npx, Q = H * W, 100000
    a, b = shard_bounds(N, world, rank)
    S = b - a
    sites = torch.empty((S, H, W), dtype=torch.int16, device=dev)
    out = torch.empty_like(sites)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    hip.check(L.tmh_synth_sites_device(p(sites), S, H, W, seed, channel, a, dist_id, sp))
    lo, hi, gamma = quantile_table(npx, np.linspace(0, 100, Q))
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, Q, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma), hip.ptr(lut),
                                 1, hip.TMH_STATS_DEFERRED_PCT, C.byref(h)))
    hip.check(L.tmh_stats_set_stream(h, sp))
    planes = [torch.empty(npx, dtype=torch.float64, device=dev) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    corr = C.c_void_p()
    torch.cuda.synchronize(dev)
    hip.check(L.tmh_corrector_create_device(p(mean), p(std), H, W, 1, ZERO_LOG10, sp,
                                            C.byref(corr)))
    ops = StatsOps(L, h, npx, Q, dev)
    for _ in range(2):  # bench.py step(): stats(), merge_welford, apply(), merge_counts
        hip.check(L.tmh_stats_reset(h))
        hip.check(L.tmh_stats_update_welford_device(h, p(sites), S, 1, sp))
        merge_welford(ops, sd, n_total=N)
        hip.check(L.tmh_stats_finalize_device(h, p(mean), p(std), sp))
        hip.check(L.tmh_smooth_f64_device(p(mean), p(smean), p(tmp), H, W, 5.0, sp))
        hip.check(L.tmh_smooth_f64_device(p(std), p(sstd), p(tmp), H, W, 5.0, sp))
        hip.check(L.tmh_corrector_update_device(corr, p(smean), p(sstd), sp))
        hip.check(L.tmh_correct_u16_hist_device(corr, h, p(sites), p(out), S, -1, -1, sp))
        merge_counts(ops, sd)
    torch.cuda.synchronize(dev)
    nn = C.c_int64()
    res = {"mean": np.empty(npx), "std": np.empty(npx), "acc": np.empty(Q),
           "hist": np.empty(65536, np.uint64)}
    hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(res["mean"]), hip.ptr(res["std"]),
                                   hip.ptr(res["acc"]), hip.ptr(res["hist"])))
    keep = sorted({0, S // 2, S - 1})  # local sites whose corrected planes are checked
    corrected = out[keep].cpu().numpy().view(np.uint16)
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), n=nn.value, first=a, count=S,
             keep=np.array(keep) + a, corrected=corrected, smean=smean.cpu().numpy(),
             sstd=sstd.cpu().numpy(), **res)
    L.tmh_corrector_destroy(corr)
    L.tmh_stats_destroy(h)
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    out_dir = sys.argv[1]
    rank, world, port, H, W, N, seed, channel, dist_id = (int(x) for x in sys.argv[2:11])
    main(out_dir, rank, world, port, H, W, N, seed, channel, dist_id)
