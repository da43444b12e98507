"""CPU: HDF5 layout of IllumstatsFile / ChannelImageFile (tmlib/models/file.py:420-456,
:322-363) written and read through libtmh5 (no h5py)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from util import load_golden

h5 = pytest.importorskip("tmlibrary_amd.models.file")
try:
    h5.h5lib()
except RuntimeError as e:  # libhdf5 absent on this host
    pytest.skip(str(e), allow_module_level=True)

H5DUMP = shutil.which("h5dump") or "/opt/conda/bin/h5dump"


def test_illumstats_roundtrip(tmp_path):
    g = load_golden("stats_small")
    pct = dict(zip(g["pct_keys"].tolist(), g["pct_values"].tolist()))
    path = str(tmp_path / "illumstats_file_3.h5")
    h5.write_illumstats(path, g["mean"], g["std"], pct)
    mean, std, keys, vals = h5.read_illumstats(path)
    assert np.array_equal(mean, g["mean"]) and np.array_equal(std, g["std"])
    assert dict(zip(keys.tolist(), vals.tolist())) == pct
    assert keys.dtype == np.float64 and vals.dtype == np.int64


@pytest.mark.skipif(not os.path.exists(H5DUMP), reason="h5dump not available")
def test_illumstats_layout_h5dump(tmp_path):
    path = str(tmp_path / "illumstats_file_1.h5")
    h5.write_illumstats(path, np.zeros((4, 6)), np.ones((4, 6)), {0.0: 1, 50.0: 2, 100.0: 3})
    out = subprocess.run([H5DUMP, "-H", path], capture_output=True, text=True, check=True).stdout
    for frag in ('DATASET "mean"', 'DATASET "std"', 'GROUP "percentiles"', 'DATASET "keys"',
                 'DATASET "values"', "H5T_IEEE_F64LE", "H5T_STD_I64LE", "( 4, 6 )", "( 3 )"):
        assert frag in out, frag


def test_channel_image_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    for dt in (np.uint16, np.uint8):
        a = rng.integers(0, np.iinfo(dt).max, (37, 53), dtype=dt)
        p = str(tmp_path / ("channel_image_file_%d.h5" % np.dtype(dt).itemsize))
        h5.write_channel_image(p, a)
        b = h5.read_channel_image(p)
        assert b.dtype == dt and np.array_equal(a, b)


@pytest.mark.skipif(not os.path.exists(H5DUMP), reason="h5dump not available")
def test_channel_image_is_gzip(tmp_path):
    p = str(tmp_path / "channel_image_file_9.h5")
    h5.write_channel_image(p, np.zeros((64, 80), np.uint16))
    out = subprocess.run([H5DUMP, "-p", "-H", p], capture_output=True, text=True, check=True).stdout
    assert "DEFLATE" in out and "H5T_STD_U16LE" in out


def test_h5py_chunk_shape():
    """h5py's guess_chunk as restated in models/file.py (h5py is not
    installed here: values from the algorithm, the site case worked by hand in
    the docstring).  The reference's sites are written this way
    (tmlib/writers.py:384-387: create_dataset(..., compression='gzip'))."""
    assert h5.h5py_chunk_shape((2160, 2560), 2) == (135, 160)
    assert h5.h5py_chunk_shape((2160, 2560), 1) == (135, 160)
    assert h5.h5py_chunk_shape((4, 4), 2) == (4, 4)          # below the 8 KiB floor: one chunk
    assert h5.h5py_chunk_shape((64, 80), 2) == (64, 80)
    r, c = h5.h5py_chunk_shape((101, 157), 2)
    assert r * c * 2 < 1024 * 1024 and r <= 101 and c <= 157


def test_missing_dataset_is_keyerror(tmp_path):
    p = str(tmp_path / "channel_image_file_1.h5")
    h5.write_channel_image(p, np.zeros((4, 4), np.uint16))
    with pytest.raises((KeyError, IOError)):
        h5.read_illumstats(p)


@pytest.mark.parametrize("dtype,chunks,gzip", [
    (np.uint16, None, 4),          # h5py's chunk choice (the default: the reference's layout)
    (np.uint16, "rows", 4),        # whole-row chunks
    (np.uint16, (37, 50), 4),      # 2-D chunks with partial edge chunks (h5py-style)
    (np.uint16, (64, 64), 1),
    (np.uint8, (30, 41), 6),
    (np.uint16, None, -1),         # contiguous, uncompressed: H5Dread fallback
])
def test_read_channel_images_parallel(tmp_path, dtype, chunks, gzip):
    """Parallel chunk inflate == the serial H5Dread path."""
    rng = np.random.default_rng(17)
    H, W = 101, 157
    hi = 256 if dtype == np.uint8 else 65536
    imgs = [rng.integers(0, hi, size=(H, W), dtype=dtype) for _ in range(9)]
    imgs[2][:] = 7  # highly compressible
    paths = []
    for i, a in enumerate(imgs):
        p = str(tmp_path / ("channel_image_file_%d.h5" % i))
        h5.write_channel_image(p, a, gzip_level=gzip, chunks=chunks)
        paths.append(p)
    for nt in (1, 3, 16):
        got = h5.read_channel_images(paths, n_threads=nt)
        assert got.dtype == dtype and got.shape == (9, H, W)
        assert np.array_equal(got, np.stack(imgs))
    for p, a in zip(paths, imgs):
        assert np.array_equal(h5.read_channel_image(p), a)


def test_read_channel_images_errors(tmp_path):
    a = np.zeros((10, 12), np.uint16)
    p0, p1, p2 = (str(tmp_path / ("f%d.h5" % i)) for i in range(3))
    h5.write_channel_image(p0, a)
    h5.write_channel_image(p1, np.zeros((10, 13), np.uint16))
    h5.write_channel_image(p2, a.astype(np.uint8))
    with pytest.raises(Exception, match="differs"):
        h5.read_channel_images([p0, p1], n_threads=2)
    with pytest.raises(Exception, match="differs"):
        h5.read_channel_images([p0, p2], n_threads=2)
    with pytest.raises(Exception):
        h5.read_channel_images([p0, str(tmp_path / "missing.h5")], n_threads=2)
    assert h5.read_channel_images([], n_threads=2).shape[0] == 0


@pytest.mark.parametrize("shape,dtype,chunks,level", [
    ((270, 320), np.uint16, None, 4),        # h5py's chunks (135 x 160 at full size)
    ((300, 500), np.uint16, (64, 96), 1),    # 2-D chunks, edges padded
    ((257, 333), np.uint8, (50, 50), 9),
    ((200, 300), np.uint16, "rows", 4),
    ((2160, 2560), np.uint16, None, 1),      # a full-size site: 256 chunks, a 2-level B-tree
])
def test_raw_chunk_index_parse_equals_libhdf5(tmp_path, monkeypatch, shape, dtype, chunks, level):
    """read_raw_chunks reads each file's chunk index itself (the version-1
    B-tree behind /array's layout message, outside the HDF5 lock): the table
    and bytes equal the ones libhdf5's H5Dget_chunk_info_by_coord gives."""
    rng = np.random.default_rng(3)
    paths = []
    for i in range(3):
        a = rng.integers(0, 4000, shape).astype(dtype)
        p = str(tmp_path / ("channel_image_file_%d.h5" % i))
        h5.write_channel_image(p, a, gzip_level=level, chunks=chunks)
        paths.append(p)
    monkeypatch.setenv("TMH5_CHUNK_INDEX", "parse")  # fail rather than fall back
    blob, tab, geom = h5.read_raw_chunks(paths, 3)
    blob, tab = blob.copy(), tab.copy()
    monkeypatch.setenv("TMH5_CHUNK_INDEX", "hdf5")
    blob2, tab2, geom2 = h5.read_raw_chunks(paths, 3)
    assert tuple(geom) == tuple(geom2)
    assert np.array_equal(tab, tab2)
    assert np.array_equal(blob, blob2)
