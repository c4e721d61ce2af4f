"""Bit-plane XOR kernels (reed-solomon_amd/csrc/rs_xj.cpp) on CPU: the generated program, run by the
instruction emulator tests/xj_emu.py over one 256-byte column, must reproduce the oracle's repair
and restored symbols bit for bit (encode and decode matrices, partial roles and input groups)."""
import ctypes

import numpy as np
import pytest

import rs_amd
from _util import bench_pattern, oracle_decode, oracle_encode
from xj_emu import Memory, run_block

_lib = rs_amd._lib
_lib.rsg_xj_source.argtypes = [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16, ctypes.c_char_p,
                               ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
_lib.rsg_xj_basis.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]

S = 256


def xj_source(k, r, er=None):
    n = ctypes.c_size_t()
    t = 0 if er is None else int(er.sum())
    p = None if er is None else er.ctypes.data
    assert _lib.rsg_xj_source(k, r, p, t, None, 0, ctypes.byref(n)) == 0
    buf = ctypes.create_string_buffer(n.value + 1)
    assert _lib.rsg_xj_source(k, r, p, t, buf, n.value + 1, ctypes.byref(n)) == 0
    return buf.value.decode()


def test_basis_reconstructs_gf256():
    piv = np.zeros(8, np.int32)
    beta = np.zeros(8, np.uint16)
    bits = np.zeros(256, np.uint8)
    assert _lib.rsg_xj_basis(piv.ctypes.data, beta.ctypes.data, bits.ctypes.data) == 0
    assert len(set(piv.tolist())) == 8
    # the 256 bit patterns are a bijection onto GF(256) (linear, so distinct <=> basis)
    assert len(set(bits.tolist())) == 256 and bits[0] == 0


def _random_stripe(k, r, seed):
    rng = np.random.default_rng(seed)
    buf = np.zeros((k + r, S), np.uint8)
    buf[:k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
    return buf


@pytest.mark.parametrize("k,r", [(4, 2), (10, 4), (13, 11), (128, 32), (30, 17), (200, 55 - 25)])
def test_xj_encode_matches_oracle(k, r):
    want = _random_stripe(k, r, k * 1000 + r)
    assert oracle_encode(k, r, want) == 0
    mem = Memory((k + r) * S)
    mem.b[:k * S] = want[:k].reshape(-1)
    run_block(xj_source(k, r), mem, 0, S, k * S, S)
    got = mem.b.reshape(k + r, S)
    assert np.array_equal(got[k:], want[k:])


@pytest.mark.parametrize("k,r,kind", [(10, 4, "bench"), (128, 32, "bench"), (128, 32, "rand17"), (37, 12, "mixed"),
                                      (4, 2, "info_rep")])
def test_xj_decode_matches_oracle(k, r, kind):
    full = _random_stripe(k, r, 7 + k + r)
    assert oracle_encode(k, r, full) == 0
    er = np.zeros(k + r, bool)
    rng = np.random.default_rng(k * r)
    if kind == "bench":
        er[bench_pattern(k, r)] = True
    elif kind == "rand17":
        er[rng.choice(k + r, 17, replace=False)] = True
    elif kind == "mixed":
        er[rng.choice(k, 5, replace=False)] = True
        er[k + rng.choice(r, 4, replace=False)] = True
    else:
        er[[1, 4]] = True
    if not er[:k].any():
        er[0] = True
        er[np.nonzero(er)[0][-1]] = False if er.sum() > r else er[np.nonzero(er)[0][-1]]
    rcv = full.copy()
    rcv[er] = 0
    mem = Memory((k + r) * S)
    mem.b[:] = rcv.reshape(-1)
    run_block(xj_source(k, r, er), mem, 0, S, 0, S)
    got = mem.b.reshape(k + r, S)
    assert np.array_equal(got[:k], full[:k])
    ref = rcv.copy()
    assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
    assert np.array_equal(got, ref)  # erased repair slots stay zero, as in the reference


@pytest.mark.parametrize("k,r", [(10, 4), (128, 32), (13, 11)])
def test_xj_lds_finish_matches_oracle(k, r, monkeypatch):
    """fin = 1 (gamma-basis bit-planes, Horner through the LDS table) reproduces the oracle too."""
    monkeypatch.setenv("RS_XJ_FIN", "1")
    src = xj_source(k, r)
    assert "ds_read_u16_d16_hi" in src and "fin1" in src
    want = _random_stripe(k, r, k * 77 + r)
    assert oracle_encode(k, r, want) == 0
    mem = Memory((k + r) * S)
    mem.b[:k * S] = want[:k].reshape(-1)
    run_block(src, mem, 0, S, k * S, S)
    assert np.array_equal(mem.b.reshape(k + r, S)[k:], want[k:])


@pytest.mark.parametrize("k,r,kind", [(128, 32, "enc"), (128, 32, "bench"), (40, 20, "enc"), (13, 30, "enc")])
def test_xj_shared_tables_match_oracle(k, r, kind, monkeypatch):
    """RS_XJ_SHARE=1 (two roles build one group's subset tables each and exchange them through LDS
    around an s_barrier; the emulator runs the roles in lockstep between barriers)."""
    monkeypatch.setenv("RS_XJ_SHARE", "1")
    full = _random_stripe(k, r, 99 + k + r)
    assert oracle_encode(k, r, full) == 0
    if kind == "enc":
        src = xj_source(k, r)
        assert "share1" in src and "s_barrier" in src
        mem = Memory((k + r) * S)
        mem.b[:k * S] = full[:k].reshape(-1)
        run_block(src, mem, 0, S, k * S, S)
        assert np.array_equal(mem.b.reshape(k + r, S)[k:], full[k:])
    else:
        er = np.zeros(k + r, bool)
        er[bench_pattern(k, r)] = True
        rcv = full.copy()
        rcv[er] = 0
        mem = Memory((k + r) * S)
        mem.b[:] = rcv.reshape(-1)
        src = xj_source(k, r, er)
        assert "share1" in src
        run_block(src, mem, 0, S, 0, S)
        assert np.array_equal(mem.b.reshape(k + r, S)[:k], full[:k])


KNOBS = [{"RS_XJ_OPR": "8"}, {"RS_XJ_OPR": "5"}, {"RS_XJ_RING": "3"}, {"RS_XJ_BUFFER": "1"}, {"RS_XJ_SPREAD": "1"},
         {"RS_XJ_HORNER": "1"}, {"RS_XJ_LDS": "3"}, {"RS_XJ_NT": "3"}, {"RS_XJ_RING": "4", "RS_XJ_SPREAD": "1"},
         {"RS_XJ_KREG": "0"}, {"RS_XJ_EARLY": "0"}, {"RS_XJ_EARLY": "0", "RS_XJ_OPR": "8"}, {"RS_XJ_EARLY": "2"}, {"RS_XJ_EARLY": "2", "RS_XJ_OPR": "5"}, {"RS_XJ_ENDWAIT": "1"}, {"RS_XJ_SPLITWAIT": "1"}, {"RS_XJ_SPLITWAIT": "1", "RS_XJ_EARLY": "0"}, {"RS_XJ_INLINEFIN": "1"}, {"RS_XJ_PRIO": "1"}, {"RS_XJ_PRIO": "2"}, {"RS_XJ_PRIO": "3"}]


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda d: ",".join(f"{k[6:]}={v}" for k, v in d.items()))
@pytest.mark.parametrize("k,r", [(128, 32), (30, 17)])
def test_xj_generation_knobs_match_oracle(k, r, knobs, monkeypatch):
    """Every generation knob of the XOR kernel (outputs per wave, ring depth, buffer addressing, load
    spreading, Horner element, LDS-DMA ring, cache policy) yields a program that reproduces the
    oracle's repair symbols in the emulator."""
    for name, value in knobs.items():
        monkeypatch.setenv(name, value)
    want = _random_stripe(k, r, 5 * k + r)
    assert oracle_encode(k, r, want) == 0
    mem = Memory((k + r) * S)
    mem.b[:k * S] = want[:k].reshape(-1)
    run_block(xj_source(k, r), mem, 0, S, k * S, S)
    assert np.array_equal(mem.b.reshape(k + r, S)[k:], want[k:])


def _run_grid(src, mem, S4, dst_base, ncols, cpb):
    """Every block of one stripe's grid: gx = ceil(ncols / cpb) blocks, block b walks columns b, b + gx, ..."""
    gx = -(-ncols // cpb)
    for b in range(gx):
        run_block(src, mem, 0, S4, dst_base, S4, chunk=b, ncols=min(cpb, -(-(ncols - b) // gx)), gx=gx)


@pytest.mark.parametrize("cpb,ncols", [(2, 4), (4, 4), (4, 3), (8, 1), (2, 5), (4, 6)])
@pytest.mark.parametrize("k,r,kind", [(128, 32, "enc"), (128, 32, "bench"), (30, 17, "enc"), (16, 4, "enc"),
                                      (24, 8, "enc")])
def test_xj_column_loop_matches_oracle(k, r, kind, cpb, ncols, monkeypatch):
    """RS_XJ_CPB (a block loops over cpb 256-byte columns gridDim.x apart; the next column's first input pair
    is loaded under the current column's last pair and finish, results stored per batch of 8): every
    column of the block is bit-exact vs the oracle, including a block with fewer columns than cpb and
    pair counts the loop does not take (K = 24: three pairs -> one column per block)."""
    monkeypatch.setenv("RS_XJ_CPB", str(cpb))
    S4 = 256 * ncols
    rng = np.random.default_rng(k * 31 + r + cpb)
    full = np.zeros((k + r, S4), np.uint8)
    full[:k] = rng.integers(0, 256, (k, S4), dtype=np.uint8)
    assert oracle_encode(k, r, full) == 0
    looped = ((k + 7) // 8) % 2 == 0
    if kind == "enc":
        src = xj_source(k, r)
        assert ("cpb%d" % cpb in src) == looped and ("L_xj_col0" in src) == looped
        mem = Memory((k + r) * S4)
        mem.b[:k * S4] = full[:k].reshape(-1)
        _run_grid(src, mem, S4, k * S4, ncols, cpb if looped else 1)
        assert np.array_equal(mem.b.reshape(k + r, S4)[k:], full[k:])
    else:
        er = np.zeros(k + r, bool)
        er[bench_pattern(k, r)] = True
        rcv = full.copy()
        rcv[er] = 0
        mem = Memory((k + r) * S4)
        mem.b[:] = rcv.reshape(-1)
        src = xj_source(k, r, er)
        assert "cpb%d" % cpb in src
        _run_grid(src, mem, S4, 0, ncols, cpb)
        assert np.array_equal(mem.b.reshape(k + r, S4)[:k], full[:k])


def xj_fixed_source(k, r, route, masked):
    n = ctypes.c_size_t()
    assert _lib.rsg_xj_fixed_source(k, r, route, masked, None, 0, ctypes.byref(n)) == 0
    buf = ctypes.create_string_buffer(n.value + 1)
    assert _lib.rsg_xj_fixed_source(k, r, route, masked, buf, n.value + 1, ctypes.byref(n)) == 0
    return buf.value.decode()


@pytest.mark.parametrize("route", [1, 2])
@pytest.mark.parametrize("k,r,kind", [(128, 32, "t32info"), (128, 32, "mixed"), (10, 4, "mixed"), (30, 17, "t32info"),
                                      (20, 9, "none")])
def test_xj_masked_fixed_pass(k, r, kind, route):
    """The per-stripe route's masked fixed pass (rsg_decode_batch, GF(256)): with garbage in the erased slots,
    the masked kernel equals the plain kernel run on the same stripe with those slots zeroed, for the
    syndrome (1) and re-encode (2) matrices; for route 2 that is [G | I] applied to the zeroed stripe, i.e.
    the oracle's repair of the zeroed information XOR the zeroed received repair."""
    n = k + r
    rng = np.random.default_rng(k * 7 + r + route)
    full = _random_stripe(k, r, k + 3 * r)
    assert oracle_encode(k, r, full) == 0
    er = np.zeros(n, bool)
    if kind == "t32info":
        er[rng.choice(k, min(k, r), replace=False)] = True
    elif kind == "mixed":
        er[rng.choice(n, r, replace=False)] = True
    rcv = full.copy()
    rcv[er] = rng.integers(0, 256, (int(er.sum()), S), dtype=np.uint8)  # garbage, not zeros
    zeroed = rcv.copy()
    zeroed[er] = 0
    words = [0] * ((n + 31) // 32)
    for i in np.nonzero(er)[0]:
        words[i // 32] |= 1 << (i % 32)
    src = xj_fixed_source(k, r, route, 1)
    assert "s_bitcmp1_b32" in src and "masked" in src
    zero = (n + r) * S
    mem = Memory(zero + S)  # the zero buffer is one symbol long
    mem.b[:n * S] = rcv.reshape(-1)
    run_block(src, mem, 0, S, n * S, S, masks=words, zero=zero)
    got = mem.b[n * S:(n + r) * S].reshape(r, S).copy()
    ref = Memory((n + r) * S)
    ref.b[:n * S] = zeroed.reshape(-1)
    plain = xj_fixed_source(k, r, route, 0)
    assert "s_bitcmp1_b32" not in plain
    run_block(plain, ref, 0, S, n * S, S)
    assert np.array_equal(got, ref.b[n * S:].reshape(r, S))
    if route == 2:
        info = zeroed.copy()
        info[k:] = 0
        assert oracle_encode(k, r, info) == 0
        assert np.array_equal(got, info[k:] ^ zeroed[k:])
    # masked form 2: the same outputs, each dword converted through the four byte tables at LDS 0 (the kernel's
    # prologue copies XJArgs::tab there; any table checks the conversion wiring)
    coord = xj_fixed_source(k, r, route, 2)
    assert "masked coord" in coord and "ds_read_b32" in coord
    tab = rng.integers(0, 1 << 32, 1024, dtype=np.uint64).astype(np.uint32)
    mem2 = Memory(zero + S)
    mem2.b[:n * S] = rcv.reshape(-1)
    run_block(coord, mem2, 0, S, n * S, S, masks=words, zero=zero, lds_init=tab.astype("<u4").view(np.uint8))
    x = got.reshape(r, S // 4, 4).copy().view("<u4").reshape(r, S // 4).astype(np.uint64)
    want = tab[x & 255] ^ tab[256 + ((x >> 8) & 255)] ^ tab[512 + ((x >> 16) & 255)] ^ tab[768 + (x >> 24)]
    got2 = mem2.b[n * S:(n + r) * S].reshape(r, S).copy().view("<u4").reshape(r, S // 4)
    assert np.array_equal(got2, want.astype(np.uint32))
