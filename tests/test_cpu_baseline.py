"""The CPU-baseline driver of bench.py (oracle/cpu_baseline.c, measurement infrastructure): a
pthread pool over the reference library (oracle/_ref/librs_ref.so, when built here) or the clean-room
port, coding resident stripes in place. Checked against the single-threaded oracle."""
import ctypes
import os

import numpy as np
import pytest

from _util import REPO, bench_pattern, gen_info, oracle_decode, oracle_encode

DRV = os.path.join(REPO, "oracle", "libcpu_baseline.so")
REF = os.path.join(REPO, "oracle", "_ref", "librs_ref.so")
PORT = os.path.join(REPO, "oracle", "librs_oracle.so")


def _drv():
    if not os.path.exists(DRV):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    d = ctypes.CDLL(DRV)
    d.cpub_run.restype = ctypes.c_int
    d.cpub_run.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p,
                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_double)]
    return d


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_cpu_baseline_driver_matches_oracle(kind, threads):
    lib = REF if kind == 0 else PORT
    if not os.path.exists(lib):
        pytest.skip("reference build absent (oracle/_ref is built only where /root/reference exists)")
    k, r, S, n = 20, 6, 512, 7
    er = np.zeros(k + r, np.bool_)
    er[bench_pattern(k, r)] = True
    stripes = np.zeros((n, k + r, S), np.uint8)
    for s in range(n):
        stripes[s, :k] = gen_info(0x5EED, s, k * S).reshape(k, S)
    want = stripes.copy()
    for s in range(n):
        assert oracle_encode(k, r, want[s]) == 0
    d, sec = _drv(), ctypes.c_double()
    assert d.cpub_run(lib.encode(), kind, k, r, S, stripes.ctypes.data, n, er.ctypes.data, int(er.sum()), 0, 2,
                      threads, ctypes.byref(sec)) == 0
    assert sec.value > 0
    assert np.array_equal(stripes, want)
    stripes[:, er] = 0xA5  # the driver zeroes erased slots before every decode pass
    assert d.cpub_run(lib.encode(), kind, k, r, S, stripes.ctypes.data, n, er.ctypes.data, int(er.sum()), 1, 2,
                      threads, ctypes.byref(sec)) == 0
    assert np.array_equal(stripes[:, :k], want[:, :k])
    ref = want[0].copy()
    ref[er] = 0
    assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
    assert np.array_equal(stripes[0], ref)


def test_cpu_baseline_driver_missing_library():
    d, sec = _drv(), ctypes.c_double()
    buf = np.zeros((1, 6, 8), np.uint8)
    er = np.zeros(6, np.bool_)
    assert d.cpub_run(b"/nonexistent/librs.so", 0, 4, 2, 8, buf.ctypes.data, 1, er.ctypes.data, 0, 0, 1, 1,
                      ctypes.byref(sec)) == -1
