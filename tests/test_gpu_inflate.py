"""GPU inflate of HDF5 gzip chunks (the site-image input path).

The reference reads sites through h5py, whose deflate filter is zlib's inflate
(tmlib/models/file.py:322-351, tmlib/readers.py:367-389).  Bar: every chunk
decoded by tmh_inflate_device is byte-identical to ``zlib.decompress`` of the
same stream -- zlib (Python's stdlib binding of the library libhdf5 links) is
the oracle -- over every deflate block kind (stored, fixed, dynamic; the
strategies and window sizes zlib can emit), and corrupt streams are reported
per chunk (TMH_Z_*) without touching other chunks.  Then whole channel image
files: DeviceChunkDecoder on files written through libtmh5 (whole-row and
2-D chunks with edge padding, uint8 and uint16, several levels) equals the
host read (libhdf5 + zlib), and at full size (2160x2560 synthetic sites).
"""
import ctypes as C
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from tmlibrary_amd import hip
    return hip.lib()


def _streams():
    """(name, raw bytes, zlib stream) for every block kind zlib produces."""
    rng = np.random.default_rng(5)
    from tmlibrary_amd.synth import synth_exact_host
    site = synth_exact_host(64, 512, 12345, 0, 3)  # microscopy-like u16 rows
    data = {
        "site_rows": site.tobytes(),
        "random": rng.integers(0, 256, 40000, dtype=np.uint8).tobytes(),
        "zeros": bytes(70000),
        "ramp": (np.arange(30000, dtype=np.uint16) // 7).tobytes(),
        "repeat3": b"abc" * 20000,  # overlapping back-references (distance < length)
        "one": b"\x07",
        "text": (b"corilla illumination statistics " * 900),
    }
    out = []
    for name, raw in data.items():
        for lvl in (0, 1, 4, 9):
            out.append(("%s_l%d" % (name, lvl), raw, zlib.compress(raw, lvl)))
        for strat, sname in ((zlib.Z_FILTERED, "filtered"), (zlib.Z_HUFFMAN_ONLY, "huffman"),
                             (zlib.Z_RLE, "rle"), (zlib.Z_FIXED, "fixed")):
            co = zlib.compressobj(6, zlib.DEFLATED, 15, 8, strat)
            out.append(("%s_%s" % (name, sname), raw, co.compress(raw) + co.flush()))
        for wbits in (9, 12):
            co = zlib.compressobj(6, zlib.DEFLATED, wbits, 1)
            out.append(("%s_w%d" % (name, wbits), raw, co.compress(raw) + co.flush()))
        # several blocks with sync / full flushes between them (empty stored blocks)
        co = zlib.compressobj(4)
        h = len(raw) // 3
        s = co.compress(raw[:h]) + co.flush(zlib.Z_SYNC_FLUSH)
        s += co.compress(raw[h:2 * h]) + co.flush(zlib.Z_FULL_FLUSH) + co.compress(raw[2 * h:])
        out.append(("%s_flushes" % name, raw, s + co.flush()))
    return out


def _run(L, streams, raw_lens=None):
    """tmh_inflate_device over the streams as one launch; returns (outputs, statuses)."""
    from tmlibrary_amd import hip
    from test_gpu_parity import Dev
    n = len(streams)
    blob = b"".join(s for _, _, s in streams)
    tab = np.zeros(n, hip.ZCHUNK_DTYPE)
    off = roff = 0
    for i, (_, raw, s) in enumerate(streams):
        rl = len(raw) if raw_lens is None else raw_lens[i]
        tab[i] = (off, len(s), roff, rl, i, 0, 0, 0, 0)
        off += len(s)
        roff += rl
    d_src, d_tab = Dev(L, max(len(blob), 1)), Dev(L, tab.nbytes)
    d_raw, d_st = Dev(L, max(roff, 1)), Dev(L, 4 * n)
    raw_max = int(tab["raw_len"].max())
    scr = int(L.tmh_inflate_scratch_bytes(n, raw_max))
    d_scr = Dev(L, scr)
    d_src.put(np.frombuffer(blob, np.uint8))
    d_tab.put(tab)
    hip.check(L.tmh_inflate_device(d_src.p, len(blob), d_tab.p, n, raw_max, d_raw.p, roff,
                                   d_scr.p, scr, d_st.p, None))
    assert L.tmh_synchronize(None) == 0
    rawout = d_raw.get(np.uint8, (max(roff, 1),))
    st = d_st.get(np.int32, (n,))
    outs = [rawout[t["raw_off"]:t["raw_off"] + t["raw_len"]].tobytes() for t in tab]
    for b in (d_src, d_tab, d_raw, d_st, d_scr):
        b.free()
    return outs, st


@pytest.mark.parametrize("lanes", [None, 4, 64])
def test_inflate_every_block_kind_bit_exact(L, monkeypatch, lanes):
    """Every workgroup width the phase-1 launch can pick decodes the same."""
    if lanes:
        monkeypatch.setenv("TMH_INFLATE_LANES", str(lanes))
    streams = _streams()
    outs, st = _run(L, streams)
    bad = [(name, int(s)) for (name, _, _), s in zip(streams, st) if s]
    assert not bad, bad
    for (name, raw, s), got in zip(streams, outs):
        assert got == zlib.decompress(s) == raw, name


def test_inflate_many_streams_one_launch(L):
    """More streams than one workgroup's lanes, each its own content."""
    rng = np.random.default_rng(8)
    streams = []
    for i in range(300):
        raw = (rng.integers(0, 600 + 40 * i, 900 + 37 * i, dtype=np.uint16)).tobytes()
        streams.append(("s%d" % i, raw, zlib.compress(raw, (i % 9) + 1)))
    outs, st = _run(L, streams)
    assert not np.any(st)
    for (name, raw, s), got in zip(streams, outs):
        assert got == raw, name


def test_inflate_corrupt_streams_reported(L):
    """Corrupt chunks get their own status; the good chunks of the same
    launch still decode exactly."""
    from tmlibrary_amd import hip
    raw = (np.arange(20000, dtype=np.uint16) % 1234).tobytes()
    good = zlib.compress(raw, 6)
    flipped = bytearray(good)
    flipped[len(good) // 2] ^= 0x5A
    bad_adler = good[:-1] + bytes([good[-1] ^ 1])
    streams = [
        ("good", raw, good),
        ("truncated", raw, good[: len(good) // 2]),
        ("bad_adler", raw, bad_adler),
        ("flipped", raw, bytes(flipped)),
        ("not_zlib", raw, b"\x1f\x8b" + good[2:]),
        ("good2", raw, good),
    ]
    raw_lens = [len(raw)] * 6
    outs, st = _run(L, streams, raw_lens)
    assert st[0] == 0 and st[5] == 0
    assert outs[0] == raw and outs[5] == raw
    assert st[1] != 0 and st[2] == 7 and st[3] != 0 and st[4] == 1
    # wrong expected sizes: too small -> overflow, too large -> size
    outs, st = _run(L, [("small", raw, good), ("large", raw, good)], [len(raw) - 10, len(raw) + 10])
    assert st[0] == 5 and st[1] == 8
    assert set(hip.Z_STATUS) >= set(int(x) for x in st)


def _files(tmp_path, n, H, W, dtype, chunks, level, seed=1):
    from tmlibrary_amd.models.file import write_channel_image
    from tmlibrary_amd.synth import synth_exact_host
    paths, imgs = [], []
    for i in range(n):
        a = synth_exact_host(H, W, seed, 0, i)
        if dtype == np.uint8:
            a = (a >> 4).astype(np.uint8)
        p = os.path.join(str(tmp_path), "channel_image_file_%d.h5" % i)
        write_channel_image(p, a, level, chunks=chunks)
        paths.append(p)
        imgs.append(a)
    return paths, np.stack(imgs)


@pytest.mark.parametrize("H,W,dtype,chunks,level", [
    (300, 500, np.uint16, None, 4),        # h5py's default chunks (38 x 125), last row padded
    (300, 500, np.uint16, (64, 96), 1),    # 2-D chunks, right and bottom edges padded
    (257, 333, np.uint8, (50, 50), 9),
    (128, 256, np.uint16, (128, 256), 6),  # one chunk per file
])
def test_device_decode_channel_image_files(L, tmp_path, H, W, dtype, chunks, level):
    import torch

    from tmlibrary_amd.models.device_decode import DeviceChunkDecoder
    from tmlibrary_amd.models.file import read_channel_image
    paths, want = _files(tmp_path, 5, H, W, dtype, chunks, level)
    for p, w in zip(paths, want):
        assert np.array_equal(read_channel_image(p), w)  # the host path reads what was written
    tdt = torch.int16 if dtype == np.uint16 else torch.uint8
    out = torch.empty((5, H, W), dtype=tdt, device="cuda")
    dec = DeviceChunkDecoder(n_threads=4)
    assert dec.decode(paths, out.data_ptr()) == (H, W, np.dtype(dtype).itemsize)
    dec.check()
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(dtype)
    assert np.array_equal(got, want)
    # the same decoder again (slot reuse), a different subset of the files
    out2 = torch.empty((3, H, W), dtype=tdt, device="cuda")
    dec.decode(paths[1:4], out2.data_ptr())
    dec.decode(paths[:3], out.data_ptr())
    dec.check()
    torch.cuda.synchronize()
    assert np.array_equal(out2.cpu().numpy().view(dtype), want[1:4])
    assert np.array_equal(out.cpu().numpy().view(dtype)[:3], want[:3])


@pytest.mark.timeout(300)
def test_device_decode_fullsize_sites(L, tmp_path):
    """Eight 2160x2560 synthetic sites, written as the reference-layout files
    (gzip level 4, h5py's default 135 x 160 chunks), decoded on the GPU = the host read."""
    import torch

    from tmlibrary_amd.models.device_decode import DeviceChunkDecoder
    paths, want = _files(tmp_path, 8, 2160, 2560, np.uint16, None, 4, seed=12345)
    out = torch.empty((8, 2160, 2560), dtype=torch.int16, device="cuda")
    dec = DeviceChunkDecoder()
    dec.decode(paths, out.data_ptr())
    dec.check()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)


def test_corrupt_file_raises(L, tmp_path):
    """A damaged chunk on disk: the decoder's check names the file and the
    reason (zlib would raise on the same bytes)."""
    import torch

    from tmlibrary_amd.models.device_decode import DeviceChunkDecoder
    from tmlibrary_amd.models.file import read_raw_chunks
    paths, _ = _files(tmp_path, 2, 200, 300, np.uint16, (50, 300), 4)
    blob, table, _ = read_raw_chunks(paths[1:])
    e = table[2]
    chunk = blob[e["src_off"]:e["src_off"] + e["src_len"]].tobytes()
    data = bytearray(open(paths[1], "rb").read())
    at = data.find(chunk)
    assert at > 0 and data.find(chunk, at + 1) < 0
    data[at + len(chunk) // 2] ^= 0xFF
    data[at + len(chunk) - 1] ^= 0x01  # the Adler-32 too
    open(paths[1], "wb").write(bytes(data))
    with pytest.raises(zlib.error):
        zlib.decompress(bytes(data[at:at + len(chunk)]))
    out = torch.empty((2, 200, 300), dtype=torch.int16, device="cuda")
    dec = DeviceChunkDecoder(n_threads=2)
    dec.decode(paths, out.data_ptr())
    with pytest.raises(IOError, match="channel_image_file_1.h5: chunk 6"):
        dec.check()
