#!/usr/bin/env python3
"""Site-image input path on the GPU box: host inflate vs GPU inflate.

Writes D distinct full-size synthetic sites as channel image files (gzip
level 4, h5py's default 135 x 160 chunks -- the reference's ChannelImageFile
layout, tmlib/models/file.py:353-363), then decodes a block of B files (the
D files cycled) R times each way:
  host:  read_channel_images (libhdf5 metadata + zlib inflate on the granted cores)
  raw:   read_raw_chunks only (the host half of the GPU path)
  gpu:   DeviceChunkDecoder (raw chunks -> H2D -> tmh_inflate_device -> place)
and checks the GPU result equals the host one.  One JSON line.
    python tools/bench_inflate.py [--distinct 16] [--block 128] [--reps 3] [--lanes 4,8,16,32,64]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--distinct", type=int, default=16)
    ap.add_argument("--block", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=2560)
    ap.add_argument("--level", type=int, default=4)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--lanes", default="", help="comma list of TMH_INFLATE_LANES to sweep")
    a = ap.parse_args()
    import torch

    from tmlibrary_amd import hip
    from tmlibrary_amd.models.device_decode import DeviceChunkDecoder
    from tmlibrary_amd.models.file import (default_decode_threads, read_channel_images,
                                           read_raw_chunks, write_channel_image)
    from tmlibrary_amd.synth import synth_exact_host
    H, W = a.height, a.width
    d = a.dir or tempfile.mkdtemp(prefix="tmh_inflate_")
    t0 = time.time()
    files = []
    for i in range(a.distinct):
        p = os.path.join(d, "channel_image_file_%d.h5" % i)
        write_channel_image(p, synth_exact_host(H, W, 12345, 0, i), a.level)
        files.append(p)
    print("wrote %d files in %.1f s" % (a.distinct, time.time() - t0), file=sys.stderr, flush=True)
    paths = [files[i % a.distinct] for i in range(a.block)]
    comp = sum(os.path.getsize(p) for p in paths)
    nt = default_decode_threads()
    res = {"sites": a.block, "distinct": a.distinct, "height": H, "width": W, "gzip_level": a.level,
           "compressed_bytes_per_site": comp / a.block, "host_threads": nt}
    # host decode
    host = np.empty((a.block, H, W), np.uint16)
    read_channel_images(paths, nt, out=host)
    tt = []
    for _ in range(a.reps):
        t = time.perf_counter()
        read_channel_images(paths, nt, out=host)
        tt.append(time.perf_counter() - t)
    res["host_sites_per_s"] = round(a.block / min(tt), 1)
    # raw chunk read alone
    blob, table, geom = read_raw_chunks(paths, nt)
    tt = []
    for _ in range(a.reps):
        t = time.perf_counter()
        blob, table, geom = read_raw_chunks(paths, nt, blob=blob, table=table)
        tt.append(time.perf_counter() - t)
    res["raw_read_sites_per_s"] = round(a.block / min(tt), 1)
    res["chunks_per_site"] = len(table) / a.block
    res["chunk_geometry"] = list(geom)
    # GPU decode
    L = hip.lib()
    dev = torch.device("cuda", 0)
    out = torch.empty((a.block, H, W), dtype=torch.int16, device=dev)
    dec = DeviceChunkDecoder(device=dev, n_threads=nt)
    dec.decode(paths, out.data_ptr())
    dec.check()
    torch.cuda.synchronize()
    ok = bool(np.array_equal(out.cpu().numpy().view(np.uint16), host))
    import ctypes as C

    def timed(lanes):
        if lanes:
            os.environ["TMH_INFLATE_LANES"] = str(lanes)
        else:
            os.environ.pop("TMH_INFLATE_LANES", None)
        dec.decode(paths, out.data_ptr())
        dec.check()
        torch.cuda.synchronize()
        good = bool(np.array_equal(out.cpu().numpy().view(np.uint16), host))
        L.tmh_profile_enable(1)
        L.tmh_profile_reset()
        tt = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            dec.decode(paths, out.data_ptr())
            dec.check()
            torch.cuda.synchronize()
            tt.append(time.perf_counter() - t)
        kern = {}
        for name in ("inflate", "inflate_matches", "place_chunks"):
            ms, k = C.c_double(), C.c_int64()
            hip.check(L.tmh_profile_read(name.encode(), C.byref(ms), C.byref(k)))
            if k.value:
                kern[name] = round(ms.value / k.value, 3)
        L.tmh_profile_enable(0)
        return good, round(a.block / min(tt), 1), kern

    ok2, sps, kern = timed(0)
    ok = ok and ok2
    res["gpu_sites_per_s"] = sps
    res["gpu_kernel_ms_per_block"] = kern
    if "inflate" in kern:
        tot = kern["inflate"] + kern.get("inflate_matches", 0.0)
        res["inflate_kernels_sites_per_s"] = round(a.block / (tot * 1e-3), 1)
        res["inflate_kernels_out_GBs"] = round(a.block * H * W * 2 / (tot * 1e-3) / 1e9, 1)
    if a.lanes:
        sweep = {}
        for w in [int(x) for x in a.lanes.split(",")]:
            g, sps, kern = timed(w)
            ok = ok and g
            sweep[str(w)] = {"gpu_sites_per_s": sps, "kernel_ms": kern, "equal": g}
            print(json.dumps({"lanes": w, **sweep[str(w)]}), file=sys.stderr, flush=True)
        res["lanes_sweep"] = sweep
        os.environ.pop("TMH_INFLATE_LANES", None)
    res["gpu_equals_host"] = ok
    print(json.dumps(res), flush=True)
    if a.dir is None:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
