"""GPU diagnostic: per-site histogram / order statistics vs numpy."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
from util import load_golden
from oracle import corilla_oracle as orc
from tmlibrary_amd import hip
from tmlibrary_amd.image import ChannelImage
from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
from tmlibrary_amd.workflow.corilla.quantiles import quantile_table

L = hip.lib()
for name in ["stats_single", "stats_small", "stats_extremes", "stats_dec1"]:
    g = load_golden(name)
    Q = 10 ** (int(g["decimals"]) + 2)
    sites = list(g["sites"])
    st = OnlineStatistics(sites[0].shape, decimals=int(g["decimals"]), batch_size=64,
                          flags=hip.TMH_STATS_KEEP_SITE_HIST)
    for s in sites:
        st.update(ChannelImage(s))
    st._finalize()
    lo, hi, gamma = quantile_table(sites[0].size, np.linspace(0, 100, Q))
    for i, s in enumerate(sites):
        h = np.empty(65536, np.uint32)
        hip.check(L.tmh_stats_site_histogram(st._h, i, hip.ptr(h)))
        want = orc.histogram_u16(s)
        bad = np.nonzero(h.astype(np.uint64) != want)[0]
        vlo = np.empty(Q, np.uint16); vhi = np.empty(Q, np.uint16)
        hip.check(L.tmh_stats_site_order_stats(st._h, i, hip.ptr(vlo), hip.ptr(vhi)))
        srt = np.sort(s.ravel()).astype(np.uint16)
        blo = np.nonzero(vlo != srt[lo])[0]
        bhi = np.nonzero(vhi != srt[hi])[0]
        print(name, i, "hist bad bins", len(bad), bad[:8], h[bad[:8]], want[bad[:8]],
              "| vlo bad", len(blo), blo[:6], vlo[blo[:6]], srt[lo][blo[:6]],
              "| vhi bad", len(bhi), bhi[:6], vhi[bhi[:6]], srt[hi][bhi[:6]])
    acc = st.percentile_sums
    want = orc.run_illumstats(sites, decimals=int(g["decimals"])).percentile_sums
    bad = np.nonzero(acc != want)[0]
    print(name, "acc bad", len(bad), bad[:8], acc[bad[:8]] - want[bad[:8]], gamma[bad[:8]])
