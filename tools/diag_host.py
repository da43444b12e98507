#!/usr/bin/env python3
"""Host staging diagnostics on the GPU box: pinned vs pageable H2D/D2H
bandwidth (torch copies), single-thread host memcpy bandwidth, and the
drop-in host-path rates of tmh_stats_update / tmh_correct_u16."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def bw(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t = min(t, time.perf_counter() - t0)
    return round(nbytes / t / 1e9, 1)


n = 354 << 20
res = {"cpus": os.cpu_count(), "sched_cpus": len(os.sched_getaffinity(0))}
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
pin = torch.empty(n, dtype=torch.uint8).pin_memory()
pag = torch.empty(n, dtype=torch.uint8)
pag.fill_(1)
pin.fill_(1)
res["h2d_pinned_GBs"] = bw(lambda: dev.copy_(pin, non_blocking=True), n)
res["h2d_pageable_GBs"] = bw(lambda: dev.copy_(pag), n)
res["d2h_pinned_GBs"] = bw(lambda: pin.copy_(dev, non_blocking=True), n)
a = np.ones(n, np.uint8)
b = np.empty(n, np.uint8)
b.fill(0)
res["host_memcpy_1t_GBs"] = bw(lambda: np.copyto(b, a), n)
pn = pin.numpy()
res["host_to_pinned_1t_GBs"] = bw(lambda: np.copyto(pn, a), n)
print(json.dumps(res), flush=True)
