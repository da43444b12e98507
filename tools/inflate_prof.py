#!/usr/bin/env python3
"""Per-chunk decode counters of the GPU inflate's phase 1 (a TMH_ZPROF=1 build
of libtmhip, tools/build_variant.sh; pass it as TMH_LIB): loop iterations,
cycles per iteration, canonical-search (slow path) codes, block headers and
their share of the cycles, literal iterations.  One JSON line.
    TMH_LIB=build_ab/zprof/libtmhip.so python tools/inflate_prof.py [--block 128] [--lanes 8]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--distinct", type=int, default=8)
    ap.add_argument("--block", type=int, default=128)
    ap.add_argument("--lanes", default="8")
    ap.add_argument("--level", type=int, default=4)
    a = ap.parse_args()
    import torch

    from tmlibrary_amd import hip
    from tmlibrary_amd.models.device_decode import DeviceChunkDecoder
    from tmlibrary_amd.models.file import write_channel_image
    from tmlibrary_amd.synth import synth_exact_host
    H, W = 2160, 2560
    d = tempfile.mkdtemp(prefix="tmh_zprof_")
    files = []
    for i in range(a.distinct):
        p = os.path.join(d, "channel_image_file_%d.h5" % i)
        write_channel_image(p, synth_exact_host(H, W, 12345, 0, i), a.level)
        files.append(p)
    paths = [files[i % a.distinct] for i in range(a.block)]
    dev = torch.device("cuda", 0)
    out = torch.empty((a.block, H, W), dtype=torch.int16, device=dev)
    dec = DeviceChunkDecoder(device=dev, slots=1)
    L = hip.lib()
    import ctypes as C
    res = {"block": a.block}
    for lanes in a.lanes.split(","):
        os.environ["TMH_INFLATE_LANES"] = lanes
        dec.decode(paths, out.data_ptr())
        try:
            dec.check()
        except IOError as e:  # a timing-only build (no output stores)
            res["check"] = str(e)[:120]
        L.tmh_profile_enable(1)
        L.tmh_profile_reset()
        dec.decode(paths, out.data_ptr())
        try:
            dec.check()
        except IOError:
            pass
        torch.cuda.synchronize()
        ms, k = C.c_double(), C.c_int64()
        hip.check(L.tmh_profile_read(b"inflate", C.byref(ms), C.byref(k)))
        L.tmh_profile_enable(0)
        slot = dec.slots[0]
        n = slot["n"] if slot.get("n") else 42 * a.block
        n = 42 * a.block
        raw_max = 52 * W * 2
        mw = (8 + 2 * (raw_max // 3 + 2) + 3) & ~3
        scr = slot["d_scratch"][:n * mw * 4].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, mw)
        head = scr[:, :8].astype(np.float64)
        it, cyc, slow, acyc, hcyc, lit = (head[:, i] for i in range(2, 8))
        cyc *= 256
        hcyc *= 256
        acyc *= 256
        r = {"kernel_ms": round(ms.value / max(k.value, 1), 3),
             "iterations_per_chunk": float(it.mean()), "matches_per_chunk": float(head[:, 0].mean()),
             "literal_iterations_per_chunk": float(lit.mean()),
             "slow_codes_per_chunk": float(slow.mean()),
             "code_cycle_share": float((acyc / np.maximum(cyc, 1)).mean()),
             "cycles_per_chunk_mean": float(cyc.mean()), "cycles_per_chunk_max": float(cyc.max()),
             "cycles_per_iteration": float((cyc / np.maximum(it, 1)).mean()),
             "header_cycle_share": float((hcyc / np.maximum(cyc, 1)).mean()),
             }
        r["clock_ghz_est"] = round(r["cycles_per_chunk_max"] / (r["kernel_ms"] * 1e6), 3)
        res[lanes] = r
        print(json.dumps({"lanes": lanes, **r}), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
