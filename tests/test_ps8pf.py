"""CPU checks of the prefetching per-stripe GF(256) solve loop (gen_asm.py ps8pf_kernel, k_apply_m8_pf).

The generated asm statement runs in the instruction emulator (tests/xj_emu.py) with scalar-memory and LDS
reads landing only at the waits that retire them, so a register named while its load is in flight fails
the test, as does a wrong wait count on the raw-input ring. The accumulators it leaves are compared with a
numpy model of the V = 1 step (coordinate lookup, gamma multiples, nibble tables, lookups), for input counts
that end the loop at every step position and past the slot-block and record-bank turnovers. The accumulators
start as garbage (the statement must zero them itself).
"""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from xj_emu import Memory, Wave  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "..", "reed-solomon_amd", "csrc", "gen_asm.py")


def gen_lines(variant, tmp):
    out = tmp / f"{variant}.inc"
    subprocess.check_call([sys.executable, GEN, str(out), variant])
    lines = []
    for ln in open(out):
        m = re.match(r'^"(.*)\\n\\t"$', ln.strip())
        if m:
            lines.append(m.group(1))
    return lines


@pytest.fixture(scope="module")
def pf_lines(tmp_path_factory):
    return gen_lines("ps8pf_kernel", tmp_path_factory.mktemp("pf"))


@pytest.fixture(scope="module")
def pf1_lines(tmp_path_factory):
    return gen_lines("ps8pf1_kernel", tmp_path_factory.mktemp("pf1"))


@pytest.fixture(scope="module")
def pf1c_lines(tmp_path_factory):
    return gen_lines("ps8pf1c_kernel", tmp_path_factory.mktemp("pf1c"))


@pytest.fixture(scope="module")
def pf2_lines(tmp_path_factory):
    return gen_lines("ps8pf2_kernel", tmp_path_factory.mktemp("pf2"))


def pf_byte(L):
    return 4 * (2 * (L >> 3) + (L & 1)) + ((L & 7) >> 1)


def xt8(m):
    return (((m << 1) & 0xFEFEFEFE) ^ (((m >> 7) & 0x01010101) * 0x1D)) & 0xFFFFFFFF


def model(raw, lt, lo, hi, one_table=False, preconverted=False):
    """raw [K][64] input dwords, lt [1024] coordinate tables, lo / hi [K][32] nibble indices -> acc [32][64]
    (one_table: [64][64], the low-nibble lookups of the table over y gamma^0..3, then the high-nibble ones)."""
    acc = np.zeros((64 if one_table else 32, 64), np.uint64)
    for i in range(raw.shape[0]):
        x = raw[i].astype(np.uint64)
        y = x if preconverted else lt[x & 255] ^ lt[256 + ((x >> 8) & 255)] ^ lt[512 + ((x >> 16) & 255)] ^ lt[768 + (x >> 24)]
        m = [y]
        for _ in range(7):
            m.append(xt8(m[-1]))
        tl = [np.zeros(64, np.uint64) for _ in range(16)]
        th = [np.zeros(64, np.uint64) for _ in range(16)]
        for e in range(16):
            for b in range(4):
                if (e >> b) & 1:
                    tl[e] = tl[e] ^ m[b]
                    th[e] = th[e] ^ m[4 + b]
        for p in range(32):
            if one_table:
                acc[p] ^= tl[lo[i, p]]
                acc[32 + p] ^= tl[hi[i, p]]
            else:
                acc[p] ^= tl[lo[i, p]] ^ th[hi[i, p]]
    return acc.astype(np.uint32)


KS = [1, 2, 3, 4, 5, 7, 8, 9, 12, 13, 16, 17, 31, 32, 40]


@pytest.mark.parametrize("K", KS)
def test_ps8pf_loop_matches_model(pf_lines, K):
    run_case(pf_lines, K, False)


@pytest.mark.parametrize("K", KS)
def test_ps8pf1_loop_matches_model(pf1_lines, K):
    run_case(pf1_lines, K, True)


@pytest.mark.parametrize("K", KS)
def test_ps8pf1c_loop_matches_model(pf1c_lines, K):
    """The one-table loop over inputs already in coordinates (the fixed pass's masked form 2): y = the raw dword."""
    run_case(pf1c_lines, K, True, preconverted=True)


@pytest.mark.parametrize("K", KS)
def test_ps8pf2_loop_matches_model(pf2_lines, K):
    """The one-table loop reading y gamma^1..3 from three more LDS tables (table j = xt8^j of table 0)."""
    run_case(pf2_lines, K, True, read_multiples=True)


def run_case(pf_lines, K, one_table, read_multiples=False, preconverted=False):
    rng = np.random.default_rng(1000 + K)
    S = 4096                 # input symbol stride (bytes)
    nslots = 48
    col = 1024 + 256         # chunk 1, wave 1
    src_base, rec_base, pin_base = 0, nslots * S, nslots * S + 64 * 1024
    mem = Memory(pin_base + 4 * (K + 64) + 64)
    mem.b[:nslots * S] = rng.integers(0, 256, nslots * S, dtype=np.uint8)
    slots = rng.permutation(nslots)[:K].astype(np.uint32)
    pin = np.zeros(K + 64, np.uint32)  # zero padding past K (the plan kernels write in_stride entries)
    pin[:K] = slots
    mem.b[pin_base:pin_base + 4 * pin.size] = pin.view(np.uint8)
    lo = rng.integers(0, 16, (K, 32))
    hi = rng.integers(0, 16, (K, 32))
    rec = np.zeros((K + 1) * 64, np.uint8)  # one record of padding: the loop prefetches record K
    for i in range(K):
        for p in range(32):
            rec[i * 64 + pf_byte(p)] = lo[i, p]
            rec[i * 64 + pf_byte(32 + p)] = hi[i, p]
    rec[K * 64:] = rng.integers(0, 256, 64, dtype=np.uint8)
    mem.b[rec_base:rec_base + rec.size] = rec
    lt = rng.integers(0, 1 << 32, 1024, dtype=np.uint64)
    lds = np.zeros(24576, np.uint8)
    tab = lt.copy()
    for j in range(4 if read_multiples else 1):  # table j at byte 4096 j: gamma^j times table 0's entries
        lds[4096 * j:4096 * (j + 1)] = tab.astype("<u4").view(np.uint8)
        tab = xt8(tab)
    ops = dict(col=(col + 4 * np.arange(64)).astype(np.uint32), rec=rec_base, pin=pin_base, nk=K, sym=S,
               rsrc=(src_base, nslots * S))
    w = Wave(mem, ops, lgkm=True)
    w.lds = lds
    # accumulators hold garbage on entry: the statement zeroes them first
    w.v[16:80] = rng.integers(0, 1 << 32, w.v[16:80].shape, dtype=np.uint64).astype(w.v.dtype)
    w.run(pf_lines, [])
    assert not w.vm and not w.lg, "loads left in flight at the end of the statement"
    raw = np.stack([mem.load32(np.uint64(src_base + int(s) * S + col) + 4 * np.arange(64, dtype=np.uint64))
                    for s in slots])
    want = model(raw, lt, lo, hi, one_table, preconverted)
    if read_multiples:
        assert not w.v[0].any(), "T[0] must stay zero"
    got = w.v[16:80] if one_table else w.v[32:64]
    assert np.array_equal(got, want)


def test_ps8pf_record_bytes_cover_each_lookup_once():
    pos = sorted(pf_byte(L) for L in range(64))
    assert pos == list(range(64))
