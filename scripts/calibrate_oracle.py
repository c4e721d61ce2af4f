"""Calibration of the CPU baselines: the reference src/rs compiled from its
own sources (oracle/_ref/librs_ref.so) and the clean-room restatement (oracle/librs_oracle.so),
single-threaded on identical inputs; prints the time ratio per configuration and checks that both
produce the same bytes. TEST INFRASTRUCTURE (no GPU)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
from _util import bench_pattern, gen_info, oracle  # noqa: E402
from bench import _seq  # noqa: E402

ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "librs_ref.so"))
ref.rs_create.restype = ctypes.c_void_p
ref.rs_destroy.argtypes = [ctypes.c_void_p]
ref.rs_generate_repair_symbols.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
ref.rs_restore_symbols.argtypes = [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint16, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_uint16]
orc = oracle()

for k, r, S, n in ((4, 2, 256, 2000), (10, 4, 4096, 200), (128, 32, 65536, 2), (4096, 1024, 1024, 1)):
    er = np.zeros(k + r, np.bool_)
    er[bench_pattern(k, r)] = True
    t = int(er.sum())
    base = np.zeros((n, k + r, S), np.uint8)
    for s in range(n):
        base[s, :k] = gen_info(0x5EED, s, k * S).reshape(k, S)
    a, b = base.copy(), base.copy()
    rs = ref.rs_create()
    t0 = time.perf_counter()
    for s in range(n):
        inf, k1 = _seq(a[s], 0, k, S)
        rep, k2 = _seq(a[s], k, r, S)
        assert ref.rs_generate_repair_symbols(rs, ctypes.byref(inf), ctypes.byref(rep)) == 0
    t_ref_enc = time.perf_counter() - t0
    a[:, er] = 0
    t0 = time.perf_counter()
    for s in range(n):
        rcv, k3 = _seq(a[s], 0, k + r, S)
        assert ref.rs_restore_symbols(rs, k, r, ctypes.byref(rcv), er.ctypes.data, t) == 0
    t_ref_dec = time.perf_counter() - t0
    ref.rs_destroy(rs)
    t0 = time.perf_counter()
    assert orc.orc_encode_many(k, r, S, b.ctypes.data, n, 1) == 0
    t_orc_enc = time.perf_counter() - t0
    b[:, er] = 0
    t0 = time.perf_counter()
    assert orc.orc_decode_many(k, r, S, b.ctypes.data, n, er.ctypes.data, t, 1) == 0
    t_orc_dec = time.perf_counter() - t0
    print(json.dumps({"k": k, "r": r, "S": S, "stripes": n, "bitexact": bool(np.array_equal(a, b)),
                      "ref_ms_per_stripe": round((t_ref_enc + t_ref_dec) / n * 1e3, 3),
                      "oracle_ms_per_stripe": round((t_orc_enc + t_orc_dec) / n * 1e3, 3),
                      "oracle_over_ref": round((t_orc_enc + t_orc_dec) / (t_ref_enc + t_ref_dec), 3)}), flush=True)
