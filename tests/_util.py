"""Shared test helpers: golden manifest access, the portable input generator, oracle bindings.

The oracle (oracle/librs_oracle.so) is TEST INFRASTRUCTURE: it is only loaded from tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
"""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_DIR = os.path.join(REPO, "oracle")

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)
_Q = np.uint64(0xC2B2AE3D27D4EB4F)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def gen_info(seed, stripe, nbytes, offset=0):
    """Bytes [offset, offset+nbytes) of the information region of `stripe`
    (same definition as oracle/gen_golden.c:gen_byte and the device generator)."""
    q0, q1 = offset // 8, (offset + nbytes + 7) // 8
    q = np.arange(q0, q1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ (np.uint64(stripe) * _G) ^ (q * _Q)
        v = _mix64(x + _G)
    b = v.astype("<u8").view(np.uint8)
    s = offset - q0 * 8
    return b[s:s + nbytes].copy()


def fingerprint_np(stripe_buf, sym0, nsym):
    """CPU port of the device fingerprint (rs_kernels.hip:k_fingerprint) of one stripe
    [k + r][S]: XOR over 8-byte words w at (sym, off) of mix64(w ^ mix64(sym << 40 | off))."""
    S = stripe_buf.shape[1]
    w = np.ascontiguousarray(stripe_buf[sym0:sym0 + nsym]).view("<u8").astype(np.uint64)
    sym = np.arange(sym0, sym0 + nsym, dtype=np.uint64)[:, None]
    off = (np.arange(S // 8, dtype=np.uint64) * np.uint64(8))[None, :]
    with np.errstate(over="ignore"):
        h = _mix64(w ^ _mix64((sym << np.uint64(40)) | off))
    return int(np.bitwise_xor.reduce(h.reshape(-1)).astype(np.int64))


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def case(name):
    for c in manifest()["cases"]:
        if c["name"] == name:
            return c
    raise KeyError(name)


def golden_bytes(c):
    if "file" in c:
        with open(os.path.join(GOLDEN, c["file"]), "rb") as f:
            return f.read()
    return None


def check_golden(c, out: bytes):
    """Compare produced raw output with the golden case (bytes if stored, else sha256)."""
    assert len(out) == c["nbytes"], (c["name"], len(out), c["nbytes"])
    ref = golden_bytes(c)
    if ref is not None:
        if out != ref:
            a = np.frombuffer(out, np.uint8)
            b = np.frombuffer(ref, np.uint8)
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{c['name']}: {bad.size} bytes differ, first at {bad[:8]}")
    else:
        assert hashlib.sha256(out).hexdigest() == c["sha256"], c["name"]


def case_inputs(c, stripe):
    """Stripe buffer [k+r][S] (uint8) holding the case's inputs for `stripe` and the erasure mask.

    encode*: info filled, repair zero.  decode: info filled, repair zero (caller encodes, erases).
    decode_noncw: every non-erased slot filled from the generator (not a codeword).
    gmatrix / dmatrix: unit words (see oracle/gen_golden.c)."""
    k, r, S = c["k"], c["r"], c["S"]
    n = k + r
    buf = np.zeros((n, S), np.uint8)
    er = np.zeros(n, bool)
    er[c["erased"]] = True
    op = c["op"]
    if op in ("encode", "decode"):
        buf[:k] = gen_info(c["seed"], stripe, k * S).reshape(k, S)
    elif op == "encode_iota":
        buf[:k] = (np.arange(k * S) & 0xFF).astype(np.uint8).reshape(k, S)
    elif op == "decode_noncw":
        buf[:] = gen_info(c["seed"], stripe, n * S).reshape(n, S)
        buf[er] = 0
    elif op == "gmatrix":
        for i in range(k):
            buf[i, 2 * i] = 1
    elif op == "dmatrix":
        for q in range(n):
            if not er[q]:
                buf[q, 2 * q] = 1
    return buf, er


def bench_pattern(k, r):
    step = k // r
    return [i * step for i in range(r)]


# ---------------------------------------------------------------- oracle bindings
_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        so = os.path.join(ORACLE_DIR, "librs_oracle.so")
        if not os.path.exists(so):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        lib = ctypes.CDLL(so)
        P, u16, sz = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_size_t
        lib.orc_init.restype = ctypes.c_int
        lib.orc_mul.argtypes = [u16, u16]
        lib.orc_mul.restype = u16
        lib.orc_div.argtypes = [u16, u16]
        lib.orc_div.restype = u16
        lib.orc_positions.argtypes = [u16, u16, P]
        lib.orc_cosets_upper.argtypes = [u16]
        lib.orc_cosets_upper.restype = u16
        lib.orc_select_cosets.argtypes = [u16, u16, P, P, P, P, P, P]
        lib.orc_encode_stripe.argtypes = [u16, u16, sz, P]
        lib.orc_decode_stripe.argtypes = [u16, u16, sz, P, P, u16]
        lib.orc_encode_many.argtypes = [u16, u16, sz, P, sz, ctypes.c_int]
        lib.orc_decode_many.argtypes = [u16, u16, sz, P, sz, P, u16, ctypes.c_int]
        lib.orc_init()
        _oracle = lib
    return _oracle


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def oracle_positions(k, r):
    out = np.zeros(k + r, np.uint16)
    oracle().orc_positions(k, r, ptr(out))
    return out


def oracle_encode(k, r, stripe_buf):
    S = stripe_buf.shape[1]
    rc = oracle().orc_encode_stripe(k, r, S, ptr(stripe_buf))
    return rc


def oracle_decode(k, r, stripe_buf, erased, t):
    S = stripe_buf.shape[1]
    er = np.ascontiguousarray(erased, dtype=np.bool_)
    return oracle().orc_decode_stripe(k, r, S, ptr(stripe_buf), ptr(er), t)


def run_case_oracle(c):
    """Run a golden case through the oracle, returning (rc, raw output bytes)."""
    k, r = c["k"], c["r"]
    outs, rc = [], 0
    for s in range(c["n"]):
        buf, er = case_inputs(c, s)
        if c["op"] in ("encode", "encode_iota", "gmatrix"):
            rc = oracle_encode(k, r, buf)
            outs.append(buf[k:].tobytes())
        else:
            if c["op"] == "decode":
                oracle_encode(k, r, buf)
                buf[er] = 0
            rc = oracle_decode(k, r, buf, er, c["t"])
            outs.append(buf.tobytes())
    return rc, b"".join(outs)


# ---------------------------------------------------------------- numpy GF(2^16) (test-side)
_GF = None


def gf_tables():
    """exp[2N], log[65536] for x^16 + x^5 + x^3 + x^2 + 1 (reference gf65536.c:59-88)."""
    global _GF
    if _GF is None:
        N = 65535
        exp = np.zeros(2 * N, np.int64)
        v = 1
        for i in range(N):
            exp[i] = v
            v <<= 1
            if v & 0x10000:
                v ^= 0x1002D
        exp[N:] = exp[:N]
        log = np.zeros(65536, np.int64)
        log[exp[:N]] = np.arange(N)
        _GF = (exp, log)
    return _GF


def gf_apply(M, X):
    """out[p] = sum_i M[p, i] * X[i] over GF(2^16); M [R, K] uint16, X [K, W] uint16 -> [R, W]."""
    exp, log = gf_tables()
    R, K = M.shape
    out = np.zeros((R, X.shape[1]), np.uint16)
    lm = log[M.astype(np.int64)]
    for i in range(K):
        x = X[i].astype(np.int64)
        nz = x != 0
        if not nz.any():
            continue
        lx = log[x]
        prod = exp[(lm[:, i:i + 1] + lx[None, :]) % 65535].astype(np.uint16)
        prod[:, ~nz] = 0
        prod[M[:, i] == 0] = 0
        out ^= prod
    return out
