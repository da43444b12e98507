"""GPU: configs[2]/[3]'s multi-channel sharded layout against the oracle, every channel.

VERDICT r3 item 2.  bench.py's own ``Channel`` pipeline -- four channels, each
its own job on its own stream, with the multi-GPU merges between the passes
(merge_welford's two all-reduces, the ordered percentile chain over quantile
chunks, the histogram all-reduce) -- run two ways on one GPU:

* forced-distributed in a one-rank RCCL group (the N > 1 code path: deferred
  percentiles, device-buffer RCCL collectives, per-channel streams);
* two rank processes sharing GPU 0 through ``bench.py --gpus 2 --share-gpu``
  (the launcher of VERDICT r3 item 1; gloo with host-staged collectives, so the
  chain's send/recv and the broadcast really cross ranks).

Every channel's results are compared with its committed oracle fingerprint
(tests/golden/make_bench_fingerprint.py --sites 48 --channel c): n, mean/std
and the smoothed planes within 1e-6 at 16,384 sampled pixels, the pooled
histogram and the percentile sums bit-exact, and the corrected values of three
sites at 65,536 sampled pixels within +-1 DN (non-modular) with zero wrap
flips.  Reference: tmlib/workflow/corilla/stats.py:64-121 (one job per
channel), tmlib/image.py:599-631.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from util import REPO

pytestmark = pytest.mark.gpu

BENCH = os.path.join(REPO, "bench.py")
ARGS = ["--layout", "sharded", "--channels", "4", "--sites", "48", "--steps", "2", "--warmup",
        "1", "--no-extras", "--cpu-sample", "0", "--no-same-workload"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(args, env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                       timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _assert_all_channels(d):
    chk = d["check"]
    assert chk["channels_checked"] == [0, 1, 2, 3], chk
    per = [chk] + [chk["channels"]["c%d" % c] for c in (1, 2, 3)]
    for c, cc in enumerate(per):
        v = cc["vs_oracle"]
        assert v["fingerprint"].endswith("_s48_seed12345_c%d_synthetic.npz" % c)
        for k in ("n", "pct_sums_bit_exact", "hist_bit_exact", "mean_1e-6", "std_1e-6",
                  "smoothed_1e-6", "corrected_within_1DN"):
            assert v[k] is True, (c, k, cc)
        cv = cc["corrected_vs_oracle"]
        assert cv["beyond_1DN"] == 0 and cv["wrap_flips"] == 0
        assert cv["sampled_pixels"] == 3 * 65536
    assert d["check_vs_oracle"] is True
    # consecutive jobs rotate over channel sets (jobs in flight, three in the
    # default deep order): every set's last job is checked
    lanes = chk.get("lanes", {})
    sets = d["config"]["jobs_in_flight"]
    assert sets == (3 if d["config"]["channel_order"] == "deep" else 2), d["config"]
    assert len(lanes) == 4 * (sets - 1), sorted(lanes)
    for name, cc in lanes.items():
        assert all(v for k, v in cc["vs_oracle"].items() if k != "fingerprint"), (name, cc)
        assert cc["corrected_vs_oracle"]["beyond_1DN"] == 0


@pytest.mark.timeout(600)
def test_four_channels_forced_distributed_rccl():
    d = _bench(ARGS, {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0",
                      "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_port()),
                      "TMH_BENCH_FORCE_DIST": "1"})
    assert d["config"]["rccl_world_size"] == 1
    assert d["config"]["channels"] == 4
    _assert_all_channels(d)


@pytest.mark.timeout(600)
def test_four_channels_two_ranks_share_gpu():
    d = _bench(["--gpus", "2", "--share-gpu"] + ARGS, {})
    assert d["ranks"] == 2 and d["config"]["collective_world_size"] == 2
    assert d["config"]["sites_per_gpu"] == 4 * 24  # rank 0's shard of every channel
    _assert_all_channels(d)
