"""CPU: the bench's device generator and its numpy twin share their tables.

tmh_synth_sites_device (csrc/synth_kernels.hip) is integer arithmetic over
tables the library builds on the host; synth.synth_exact_host builds the same
tables in Python.  If the tables agree bit for bit, the GPU's sites equal the
host's (checked on the GPU in test_gpu_parity / test_gpu_fullsize), which is
what lets the bench's full-size result be compared with the CPU oracle."""
import numpy as np
import pytest

from tmlibrary_amd import hip, synth


@pytest.mark.parametrize("dist", [synth.STANDARD, synth.BRIGHT, synth.UNIFORM])
@pytest.mark.parametrize("shape", [(2160, 2560), (37, 53), (1, 1)])
def test_tables_bit_identical(dist, shape):
    L = hip.load_library()
    H, W = shape
    ln = np.empty(4096, np.int32)
    nz = np.empty(4096, np.int32)
    ey = np.empty(H, np.int32)
    ex = np.empty(W, np.int32)
    assert L.tmh_synth_tables(dist, H, W, hip.ptr(ln), hip.ptr(nz), hip.ptr(ey), hip.ptr(ex)) == 0
    for got, want in zip((ln, nz, ey, ex), synth.synth_tables(dist, H, W)):
        assert np.array_equal(got, want)


def test_tables_reject_bad_arguments():
    L = hip.load_library()
    a = np.empty(4096, np.int32)
    assert L.tmh_synth_tables(7, 4, 4, hip.ptr(a), hip.ptr(a), hip.ptr(a), hip.ptr(a)) == hip.TMH_EINVAL


def test_distribution_shape():
    """~0.01 % zeros and saturated pixels, a few thousand
    distinct values; 'bright' puts a large share at or above 4,096."""
    s = synth.synth_exact_host(540, 640, 12345, 0, 3)
    assert 2e-5 < np.mean(s == 0) < 3e-4 and 2e-5 < np.mean(s == 65535) < 3e-4
    assert 1000 < len(np.unique(s)) < 20000
    b = synth.synth_exact_host(540, 640, 12345, 0, 3, synth.BRIGHT)
    assert np.mean(b >= 4096) > 0.2
    u = synth.synth_exact_host(64, 64, 1, 0, 0, synth.UNIFORM)
    assert u.max() > 60000 and u.min() < 5000


def test_sites_differ_and_repeat():
    a = synth.synth_exact_host(32, 48, 5, 0, 10)
    assert np.array_equal(a, synth.synth_exact_host(32, 48, 5, 0, 10))
    assert not np.array_equal(a, synth.synth_exact_host(32, 48, 5, 0, 11))
    assert not np.array_equal(a, synth.synth_exact_host(32, 48, 5, 1, 10))


def test_bench_fingerprint_present():
    """bench.py's configs[1] input has a committed oracle fingerprint."""
    import os

    import bench
    name = bench.fingerprint_name(2160, 2560, 3456, bench.SEED, 0, "synthetic")
    path = os.path.join(os.path.dirname(bench.__file__), "tests", "golden", name)
    with np.load(path, allow_pickle=False) as z:
        assert int(z["n"]) == 3456 and z["hist"].sum() == 3456 * 2160 * 2560
        assert z["corr_samples"].shape[0] == len(z["corr_sites"])
