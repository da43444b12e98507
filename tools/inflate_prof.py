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
        torch.cuda.synchronize()
        n_chunks = dec.slots[0]["n"]
        try:
            dec.check()
        except IOError:
            pass
        ms, k = C.c_double(), C.c_int64()
        hip.check(L.tmh_profile_read(b"inflate", C.byref(ms), C.byref(k)))
        L.tmh_profile_enable(0)
        slot = dec.slots[0]
        from tmlibrary_amd.models.file import h5py_chunk_shape
        cr, cc = h5py_chunk_shape((H, W), 2)
        n = n_chunks
        raw_max = cr * cc * 2
        mw = (16 + 2 * (raw_max // 3 + 2) + 3) & ~3
        scr = slot["d_scratch"][:n * mw * 4].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, mw)
        head = scr[:, :16].astype(np.float64)
        sym, cyc, slow, dcyc, hcyc, runs, priv, tops, hdr = (head[:, i] for i in range(2, 11))
        cyc, dcyc, hcyc = cyc * 256, dcyc * 256, hcyc * 256
        r = {"kernel_ms": round(ms.value / max(k.value, 1), 3),
             "symbols_per_chunk": float(sym.mean()), "matches_per_chunk": float(head[:, 0].mean()),
             "slow_codes_per_chunk": float(slow.mean()),
             "data_loop_entries_per_chunk": float(runs.mean()),
             "headers_per_chunk": float(hdr.mean()),
             "private_unit_loads_per_chunk": float(priv.mean()),
             "top_ups_per_chunk": float(tops.mean()),
             "cycles_per_chunk_mean": float(cyc.mean()), "cycles_per_chunk_max": float(cyc.max()),
             "data_cycles_per_symbol": float((dcyc / np.maximum(sym, 1)).mean()),
             "data_cycle_share": float((dcyc / np.maximum(cyc, 1)).mean()),
             "header_cycle_share": float((hcyc / np.maximum(cyc, 1)).mean()),
             "cycles_per_header": float((hcyc / np.maximum(hdr, 1)).mean())}
        r["clock_ghz_est"] = round(r["cycles_per_chunk_max"] / (r["kernel_ms"] * 1e6), 3)
        res[lanes] = r
        print(json.dumps({"lanes": lanes, **r}), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
