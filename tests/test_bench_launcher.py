"""bench.py --gpus N starts its own N rank processes.

The driver runs ``python bench.py --gpus N`` as well as the torchrun form; a
rank per GPU must exist either way (each channel's sites are
sharded over one process per GPU; the reference's per-channel jobs,
tmlib/workflow/corilla/api.py:64-105).  On CPU the launcher is exercised with
``--dry-run``: every rank joins a gloo group and rank 0 prints the ranks'
launch environment as the one JSON line.
"""
import json
import os
import subprocess
import sys

import pytest

from util import REPO

BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_launcher_dry_run_two_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # exactly rank 0's JSON line
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 2 and d["world_size"] == 2
    ranks = d["ranks"]
    assert [e["RANK"] for e in ranks] == ["0", "1"]
    assert [e["LOCAL_RANK"] for e in ranks] == ["0", "1"]
    assert {e["WORLD_SIZE"] for e in ranks} == {"2"}
    assert {e["MASTER_ADDR"] for e in ranks} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in ranks}) == 1


def test_launcher_rank_failure_is_nonzero():
    # rank 1 exits before joining the group: rank 0 would wait in the
    # rendezvous forever, so the launcher must stop it and fail
    r = _run(["--gpus", "2", "--dry-run"], {"TMH_BENCH_DRY_FAIL_RANK": "1"})
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    assert r.stdout.strip() == ""


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") not in (None, ""),
                    reason="device visibility restricted")
def test_launcher_refuses_more_ranks_than_gpus():
    import torch
    have = torch.cuda.device_count()
    n = max(2, have + 1)
    r = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0"], timeout=120)
    assert r.returncode == 2
    assert "needs %d visible GPU(s), found %d" % (n, have) in r.stderr
    assert r.stdout.strip() == ""


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2
    assert "disagrees with WORLD_SIZE=2" in r.stderr


def test_launcher_stalled_collective_fails_loudly():
    """every rank stuck (rank 1 hangs before an all_reduce,
    rank 0 waits inside it) must not hang the run.  With no heartbeat from any
    rank for --stall-timeout seconds the launcher kills the ranks' process
    groups and exits 3, naming each rank's last stage -- the reference's
    failed job exits non-zero with its cause (tmlib/workflow/cli.py:287-293)."""
    import time
    t0 = time.time()
    r = _run(["--gpus", "2", "--dry-run", "--stall-timeout", "8", "--deadline", "120"],
             {"TMH_BENCH_DRY_STALL_RANK": "1"}, timeout=170)
    took = time.time() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    assert r.stdout.strip() == ""
    assert "no rank made progress" in r.stderr, r.stderr[-3000:]
    assert "rank 0 (running): all_reduce #1" in r.stderr, r.stderr[-3000:]
    assert "rank 1 (running): stalled on purpose" in r.stderr, r.stderr[-3000:]
    assert took < 150


def test_launcher_deadline():
    r = _run(["--gpus", "2", "--dry-run", "--stall-timeout", "600", "--deadline", "6"],
             {"TMH_BENCH_DRY_STALL_RANK": "1"}, timeout=170)
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    assert "deadline of 6 s passed" in r.stderr, r.stderr[-3000:]
    assert "rank 1 (running)" in r.stderr


def test_one_rank_output_unchanged():
    """--gpus 1 (and no WORLD_SIZE): no launcher, no heartbeat lines."""
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["world_size"] == 1
    assert "[rank" not in r.stderr


def test_launcher_dry_run_eight_ranks_rehearses_the_merges():
    """the N = 8 launch and its exchange before any 8-GPU
    run.  Eight ranks each take their contiguous 432-site share of four
    3,456-site channels (configs[2]) and run the bench's merges at that
    geometry -- per-channel Welford all-reduces, the 8-hop ordered chain in
    chain_chunks(100,000, 8) pieces, the histogram all-reduce (the default
    pipelined order), through the heartbeat-wrapped collectives -- on
    synthetic per-rank state; rank 0 checks every channel: the chained sums
    bit-equal to the site-order sum, the pooled Welford state and histograms
    (reference: corilla/api.py:64-105, stats.py:75-76).  Plane size reduced
    (216 x 256) to keep eight CPU ranks light; the chain carries the full Q."""
    r = _run(["--gpus", "8", "--dry-run", "--sites", "3456", "--height", "216", "--width", "256",
              "--deadline", "400", "--stall-timeout", "120"], timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["world_size"] == 8 and [e["RANK"] for e in d["ranks"]] == [str(i) for i in range(8)]
    m = d["merges"]
    assert m["ok"], m
    assert m["channels"] == 4 and m["chain_chunks"] == 8 and m["merge"] == "per-channel"
    for c in range(4):
        chk = m["check"]["c%d" % c]
        assert chk["sites_per_rank"] == [432] * 8
        assert chk["pct_sum_bit_exact"] and chk["welford_close"] and chk["hist_equal"]
    # every rank's heartbeat went through the collectives (the launcher's
    # watchdog read them against --deadline / --stall-timeout and let them run)
    for i in range(8):
        assert "[rank %d]" % i in r.stderr, r.stderr[-2000:]


def test_launcher_dry_run_eight_ranks_batched_merges():
    r = _run(["--gpus", "8", "--dry-run", "--sites", "100", "--height", "24", "--width", "32",
              "--merge", "batched", "--channel-order", "concurrent", "--deadline", "300"],
             timeout=320)
    assert r.returncode == 0, r.stderr[-3000:]
    m = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])["merges"]
    assert m["ok"] and m["merge"] == "batched", m
    assert m["check"]["c0"]["sites_per_rank"] == [13] * 4 + [12] * 4


def test_launcher_eight_ranks_one_stalled():
    r = _run(["--gpus", "8", "--dry-run", "--stall-timeout", "10", "--deadline", "200"],
             {"TMH_BENCH_DRY_STALL_RANK": "7"}, timeout=230)
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    assert r.stdout.strip() == ""
    assert "rank 7 (running): stalled on purpose" in r.stderr, r.stderr[-3000:]
