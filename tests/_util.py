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
        # RS_ORACLE_LIB: another build of the same oracle (the sanitizer build, tests/test_sanitizers.py)
        so = os.environ.get("RS_ORACLE_LIB") or os.path.join(ORACLE_DIR, "librs_oracle.so")
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


# ---------------------------------------------------------------- symbol ops / transforms (fixtures)
EXTRA_OPS = ("gf_add", "gf_mul", "gf_madd", "fft_t", "fft_tc", "fft_p", "fft_pc")


def pos_gen(seed, i):
    """Position / component i of the fft cases (oracle/gen_golden.c:pos_gen)."""
    with np.errstate(over="ignore"):
        v = _mix64(np.uint64(seed) ^ (np.uint64(i + 1) * _G))
    return int(v % np.uint64(65535))


def _words(buf):
    """LE uint16 words of the first len // 2 * 2 bytes."""
    n = buf.size // 2
    return buf[:2 * n].view("<u2").astype(np.int64)


_REPR = {}


def normal_repr_table(m):
    """repr[d] = bits of alpha^d in the normal basis of GF(2^m) (oracle orc_normal_repr)."""
    if m not in _REPR:
        o = oracle()
        o.orc_normal_repr.restype = ctypes.c_uint16
        o.orc_normal_repr.argtypes = [ctypes.c_uint8, ctypes.c_uint16]
        _REPR[m] = np.array([o.orc_normal_repr(m, d) for d in range(65535)], np.int64)
    return _REPR[m]


def normal_basis(m):
    exp, _ = gf_tables()
    rep = normal_repr_table(m)
    return [int(exp[int(np.nonzero(rep == (1 << j))[0][0])]) for j in range(m)]


def extra_inputs(c):
    """Inputs of a symbol-op / transform case: (a, b) byte arrays, or (f [k][S], positions / cosets)."""
    S, seed = c["S"], c["seed"]
    if c["op"].startswith("gf_"):
        return gen_info(seed, 0, S), gen_info(seed, 1, S)
    f = gen_info(seed, 0, c["k"] * S).reshape(c["k"], S) if c["k"] else np.zeros((0, S), np.uint8)
    if c["op"] in ("fft_t", "fft_tc"):
        arg = [pos_gen(seed, i) for i in range(c["k"])]
    elif c["op"] == "fft_p":
        arg = [pos_gen(seed, j) for j in range(c["r"])]
    else:
        arg = [tuple(x) for x in c["cosets"]]
    return f, arg


def transform_matrix(c, arg):
    """The transform's GF(2^16) matrix [r][k] as the reference evaluates it (src/rs/fft.c)."""
    exp, _ = gf_tables()
    N = 65535
    k, r = c["k"], c["r"]
    i = np.arange(k, dtype=np.int64)
    if c["op"] in ("fft_t", "fft_tc"):
        return exp[(np.array(arg, np.int64)[None, :] * np.arange(r, dtype=np.int64)[:, None]) % N].astype(np.uint16)
    if c["op"] == "fft_p":
        j = (N - np.array(arg, np.int64)) % N
        return exp[(i[None, :] * j[:, None]) % N].astype(np.uint16)
    rows = []
    for leader, m in arg:  # fft.c:142-169
        nb = normal_basis(m)
        rep = normal_repr_table(m)[((N - leader) % 65536 * i) % N]
        for jj in range(m):
            v = np.zeros(k, np.int64)
            for t in range(m):
                v ^= np.where((rep >> t) & 1, nb[(jj + t) % m], 0)
            rows.append(v)
    return np.array(rows, np.int64).reshape(r, k).astype(np.uint16)


def run_extra_numpy(c):
    """CPU restatement of a symbol-op / transform case (numpy GF(2^16)); raw output bytes."""
    exp, log = gf_tables()
    S = c["S"]
    if c["op"].startswith("gf_"):
        a, b = extra_inputs(c)
        a = a.copy()
        wa, wb = _words(a), _words(b)
        coef = c["t"]
        if c["op"] == "gf_add":
            wa ^= wb
        elif c["op"] == "gf_mul":
            wa = np.zeros_like(wa) if coef == 0 else np.where(wa != 0, exp[(log[wa] + log[coef]) % 65535], 0)
            if coef == 0:
                a[:] = 0
        elif coef:
            wa ^= np.where(wb != 0, exp[(log[wb] + log[coef]) % 65535], 0)
        a[:2 * wa.size] = wa.astype("<u2").view(np.uint8)
        return a.tobytes()
    f, arg = extra_inputs(c)
    M = transform_matrix(c, arg)
    X = np.stack([_words(x) for x in f]).astype(np.uint16) if len(f) else np.zeros((0, S // 2), np.uint16)
    Y = gf_apply(M, X) if len(f) else np.zeros((c["r"], S // 2), np.uint16)
    out = np.zeros((c["r"], S), np.uint8)
    out[:, :2 * (S // 2)] = Y.astype("<u2").view(np.uint8).reshape(c["r"], -1)
    return out.tobytes()
