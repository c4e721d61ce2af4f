"""Calibration of the CPU baselines: the reference src/rs compiled from its own
sources (oracle/_ref/librs_ref.so) against the clean-room restatement (oracle/librs_oracle.so), timed by
the same C driver bench.py uses (oracle/cpu_baseline.c, cpub_run: views built before the clock), one
thread, identical inputs (encode + bench-pattern decode), median of 5 runs; checks that both produce
the same bytes. With --out FILE it writes the ratios bench.py reports beside a port-timed baseline on the
GPU box, where the reference never travels (oracle/calibration.json).

TEST INFRASTRUCTURE (no GPU): run here, where /root/reference is."""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "tests"))
from _util import bench_pattern, gen_info  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "librs_ref.so")
PORT = os.path.join(REPO, "oracle", "librs_oracle.so")
drv = ctypes.CDLL(os.path.join(REPO, "oracle", "libcpu_baseline.so"))
drv.cpub_run.restype = ctypes.c_int
drv.cpub_run.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p,
                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                         ctypes.POINTER(ctypes.c_double)]
out_path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None


def timed(lib, port, k, r, S, stripes, er, t, op, passes):
    sec = ctypes.c_double()
    rc = drv.cpub_run(lib.encode(), port, k, r, S, stripes.ctypes.data, stripes.shape[0], er.ctypes.data, t, op,
                      passes, 1, ctypes.byref(sec))
    assert rc == 0, rc
    return sec.value


def one(k, r, S, n, passes):
    er = np.zeros(k + r, np.bool_)
    er[bench_pattern(k, r)] = True
    t = int(er.sum())
    base = np.zeros((n, k + r, S), np.uint8)
    for s in range(n):
        base[s, :k] = gen_info(0x5EED, s, k * S).reshape(k, S)
    res = {}
    for name, lib, port in (("ref", REF, 0), ("port", PORT, 1)):
        a = base.copy()
        te = timed(lib, port, k, r, S, a, er, t, 0, passes)
        enc = a.copy()
        td = timed(lib, port, k, r, S, a, er, t, 1, passes)
        res[name] = (te + td) / (n * passes), enc, a
    same = np.array_equal(res["ref"][1], res["port"][1]) and np.array_equal(res["ref"][2], res["port"][2])
    return same, res["ref"][0], res["port"][0]


rows = []
for k, r, S, n, passes in ((4, 2, 256, 256, 200), (10, 4, 4096, 64, 20), (128, 32, 65536, 4, 1),
                           (4096, 1024, 1024, 1, 1)):
    runs = [one(k, r, S, n, passes) for _ in range(5)]
    ratio = sorted(p / f for _, f, p in runs)[2]
    row = {"k": k, "r": r, "S": S, "stripes": n, "passes": passes, "bitexact": all(b for b, _, _ in runs),
           "ref_ms_per_stripe": round(sorted(f for _, f, _ in runs)[2] * 1e3, 4),
           "port_ms_per_stripe": round(sorted(p for _, _, p in runs)[2] * 1e3, 4),
           "port_over_ref": round(ratio, 3)}
    rows.append(row)
    print(json.dumps(row), flush=True)
if out_path:
    with open(out_path, "w") as f:
        json.dump({"what": "time of the clean-room CPU port (oracle/librs_oracle.so) over the reference compiled from "
                           "its own sources (oracle/_ref/librs_ref.so): the same C driver (oracle/cpu_baseline.c), "
                           "one thread, identical inputs, encode + bench-pattern decode, median of 5 runs "
                           "(scripts/calibrate_oracle.py)",
                   "host": "build container (no GPU)", "measured": time.strftime("%Y-%m-%d"), "rows": rows}, f,
                  indent=1)
