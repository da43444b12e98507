"""CPU: the GPU inflate's decode core, built for the host, against zlib.

tmlibrary_amd/csrc/inflate_core.h is the exact code k_inflate runs per lane
(inflate_kernels.hip includes it); tests/inflate_host.cpp compiles it with g++
and runs the lanes one after another.  So every round's CPU suite checks the
decoder byte for byte against zlib -- the library behind the reference's h5py
deflate filter (tmlib/models/file.py:322-351) -- over every block kind and
the corrupt-stream statuses, without a GPU; tests/test_gpu_inflate.py runs the
same streams through the device kernel.
"""
import os
import subprocess
import zlib

import numpy as np
import pytest

from util import REPO

HARNESS = os.path.join(REPO, "tests", "inflate_host.cpp")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("inflate") / "inflate_host")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-o", out, HARNESS],
                   check=True, capture_output=True)
    return out


def _run(exe, tmp_path, streams, raw_lens=None):
    from tmlibrary_amd.hip import ZCHUNK_DTYPE
    n = len(streams)
    tab = np.zeros(n, ZCHUNK_DTYPE)
    off = roff = 0
    for i, (_, raw, s) in enumerate(streams):
        rl = len(raw) if raw_lens is None else raw_lens[i]
        tab[i] = (off, len(s), roff, rl, i, 0, 0, 0, 0)
        off += len(s)
        roff += rl
    p = lambda name: str(tmp_path / name)  # noqa: E731
    open(p("tab"), "wb").write(tab.tobytes())
    open(p("blob"), "wb").write(b"".join(s for _, _, s in streams))
    subprocess.run([exe, p("tab"), p("blob"), str(roff), p("out"), p("st")], check=True)
    out = open(p("out"), "rb").read()
    st = np.fromfile(p("st"), np.int32)
    return [out[t["raw_off"]:t["raw_off"] + t["raw_len"]] for t in tab], st


def test_every_block_kind(exe, tmp_path):
    from test_gpu_inflate import _streams
    streams = _streams()
    outs, st = _run(exe, tmp_path, streams)
    assert not [(s[0], int(c)) for s, c in zip(streams, st) if c]
    for (name, raw, s), got in zip(streams, outs):
        assert got == zlib.decompress(s) == raw, name


def test_random_streams(exe, tmp_path):
    rng = np.random.default_rng(2024)
    streams = []
    for i in range(200):
        kind = i % 4
        n = int(rng.integers(1, 30000))
        if kind == 0:
            raw = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            raw = (rng.integers(0, 40, n, dtype=np.uint16) + 900).tobytes()
        elif kind == 2:
            raw = bytes(rng.choice([0, 1, 2, 255], n).astype(np.uint8))
        else:
            raw = (np.cumsum(rng.integers(-2, 3, n)) % 5000).astype(np.uint16).tobytes()
        co = zlib.compressobj(int(rng.integers(0, 10)), zlib.DEFLATED, int(rng.integers(9, 16)),
                              int(rng.integers(1, 10)),
                              int(rng.choice([zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED,
                                              zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED])))
        streams.append(("r%d" % i, raw, co.compress(raw) + co.flush()))
    outs, st = _run(exe, tmp_path, streams)
    assert not np.any(st)
    for (name, raw, _), got in zip(streams, outs):
        assert got == raw, name


def test_corrupt_streams(exe, tmp_path):
    raw = (np.arange(20000, dtype=np.uint16) % 1234).tobytes()
    good = zlib.compress(raw, 6)
    flipped = bytearray(good)
    flipped[len(good) // 2] ^= 0x5A
    streams = [("good", raw, good), ("truncated", raw, good[: len(good) // 2]),
               ("bad_adler", raw, good[:-1] + bytes([good[-1] ^ 1])),
               ("flipped", raw, bytes(flipped)), ("not_zlib", raw, b"\x1f\x8b" + good[2:]),
               ("good2", raw, good)]
    outs, st = _run(exe, tmp_path, streams)
    assert st[0] == 0 and st[5] == 0 and outs[0] == raw and outs[5] == raw
    assert st[1] != 0 and st[2] == 7 and st[3] != 0 and st[4] == 1
    _, st = _run(exe, tmp_path, [("s", raw, good), ("l", raw, good)],
                 [len(raw) - 10, len(raw) + 10])
    assert st[0] == 5 and st[1] == 8
    # random garbage never escapes a status (and never crashes the harness)
    rng = np.random.default_rng(3)
    junk = [("j%d" % i, b"", bytes([0x78, 0x9C]) + rng.integers(0, 256, 300, dtype=np.uint8).tobytes())
            for i in range(100)]
    _, st = _run(exe, tmp_path, junk, [4096] * 100)
    assert np.all(st != 0)
