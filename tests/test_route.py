"""The GF(2^16) syndrome route (rs_api.cpp make_plan_cs, rs_kernels.hip k_cs16, gen_asm.py cs16), on
CPU through the host-only rsg_route_dump:

* second stage: M2 [R][D] times the syndrome matrix H [D][K] (H[j][q] = X_q^j over the sources) equals
  the engine's coding matrix for the same pattern (which the golden tests pin to the reference), so
  out = M2 * syndromes is the reference's map on every input;
* k_cs16's plan: a numpy model of the kernel (subset tables per group, one index per (coset, t') for
  four tables, finish S_(s 2^b) = sum_t nb_(t + b) u_t) reproduces H * X from the dumped records."""
import numpy as np
import pytest

import rs_amd
from _util import gf_apply, gf_tables, normal_basis, oracle_positions

CASES = [("enc", 300, 200, None), ("dec", 300, 200, 150), ("enc", 4096, 1024, None), ("dec_bench", 4096, 1024, 1024),
         ("dec", 4096, 1024, 700), ("dec_info32", 4096, 1024, 32)]


def _pattern(kind, k, r, t, seed=3):
    if kind == "enc":
        return None
    er = np.zeros(k + r, bool)
    rng = np.random.default_rng(seed)
    if kind == "dec_bench":
        er[[i * (k // r) for i in range(r)]] = True
    elif kind == "dec_info32":
        er[rng.choice(k, t, replace=False)] = True
    else:
        er[rng.choice(k + r, t, replace=False)] = True
    return er


def _lists(k, r, er):
    pos = oracle_positions(k, r).astype(np.int64)
    if er is None:
        return pos, list(range(k)), list(range(k, k + r))
    return pos, [i for i in range(k + r) if not er[i]], [i for i in range(k + r) if er[i]]


@pytest.mark.parametrize("kind,k,r,t", CASES)
def test_second_stage_times_syndromes_is_the_coding_matrix(kind, k, r, t):
    exp, _ = gf_tables()
    er = _pattern(kind, k, r, t)
    d = rs_amd.route_dump(k, r, er)
    pos, srcs, tgts = _lists(k, r, er)
    assert d["D"] == len(tgts)
    H = exp[(np.arange(d["D"], dtype=np.int64)[:, None] * pos[srcs][None, :]) % 65535].astype(np.uint16)
    M, ins, outs = rs_amd.coding_matrix(k, r, er)
    assert list(ins) == srcs
    rows = slice(0, 96) if M.shape[0] > 96 else slice(None)  # a sample of rows keeps numpy quick
    assert np.array_equal(gf_apply(d["m2"][rows], H), M[rows])


def _model_syndromes(d, X, nb):
    """k_cs16's arithmetic on CPU: X [n slots][W] words -> syndromes [D][W]."""
    exp, log = gf_tables()
    groups, rec, fin, fin_off = d["groups"], d["rec"], d["fin"], d["fin_off"]
    nt, W = rec.shape[0], X.shape[1]
    S = np.zeros((d["D"], W), np.int64)
    for tile in range(nt):
        acc = np.zeros((4, 16, W), np.int64)
        for g in range(groups.shape[0]):
            f = np.array([X[s] if s >= 0 else np.zeros(W, np.int64) for s in groups[g]])
            for q in range(4):
                tab = np.zeros((16, W), np.int64)
                for e in range(16):
                    for dd in range(4):
                        if e >> dd & 1:
                            tab[e] ^= f[4 * q + dd]
                idx = rec[tile, g]  # [4][16]: e(t') per local coset
                for tp in range(16):
                    acc[:, (tp + 4 * q) % 16] ^= tab[idx[:, tp]]
        for c in range(4):
            for e in range(fin_off[tile, c], fin_off[tile, c + 1]):
                ent = int(fin[tile, e])
                assert ent & 15 == c
                b, j = (ent >> 4) & 15, ent >> 8
                v = np.zeros(W, np.int64)
                for t in range(16):
                    u = acc[c, t]
                    nz = u != 0
                    v ^= np.where(nz, exp[(log[u] + log[nb[(t + b) % 16]]) % 65535], 0)
                S[j] = v
    return S


@pytest.mark.parametrize("kind,k,r,t", [CASES[0], CASES[1], ("dec", 60, 40, 40), ("enc", 1100, 250, None)])
def test_cs16_plan_model_gives_the_syndromes(kind, k, r, t):
    exp, _ = gf_tables()
    er = _pattern(kind, k, r, t, seed=5)
    d = rs_amd.route_dump(k, r, er)
    pos, srcs, _ = _lists(k, r, er)
    rng = np.random.default_rng(k + r)
    X = rng.integers(0, 65536, (k + r, 2)).astype(np.int64)
    nb = normal_basis(16)
    # every coset element's square is the next one: the normal basis is Frobenius-cyclic
    _, log = gf_tables()
    assert all(exp[(2 * log[nb[i]]) % 65535] == nb[(i + 1) % 16] for i in range(16))
    got = _model_syndromes(d, X, nb)
    H = exp[(np.arange(d["D"], dtype=np.int64)[:, None] * pos[srcs][None, :]) % 65535].astype(np.uint16)
    want = gf_apply(H, X[srcs].astype(np.uint16))
    assert np.array_equal(got.astype(np.uint16), want)
    assert sorted(set(np.concatenate([d["groups"].ravel(), [-1]]))) == [-1] + srcs  # each source in one group slot


def _model_syndromes_t(d, dt, X, nb):
    """k_cs16t's arithmetic on CPU: a step runs the chain of blocks its record names -- entry 0's block
    first, then after block (position q) the block entry q + 1 names, until the last position's -- and
    block (c, n, v) at position 4c + n XORs f_((t - 4n - dd) mod 16) for the set bits dd of v into
    accumulator t of local coset c (gen_asm.py cs16t; zero nibbles are skipped by the record); the finish
    as k_cs16's."""
    exp, log = gf_tables()
    cw, rec, fin, fin_off = dt["cw"], dt["rec"], dt["fin"], dt["fin_off"]
    where = {int(o): divmod(b, 16) for b, o in enumerate(dt["blocks"])}  # offset -> (p, v)
    assert len(where) == len(dt["blocks"])  # distinct offsets
    groups = d["groups"]
    nt, W = rec.shape[0], X.shape[1]
    S = np.zeros((d["D"], W), np.int64)
    for tile in range(nt):
        acc = np.zeros((cw, 16, W), np.int64)
        for g in range(groups.shape[0]):
            f = np.array([X[s] if s >= 0 else np.zeros(W, np.int64) for s in groups[g]])
            for p, v in _chain(rec[tile, g], where, 4 * cw):
                c, n = divmod(p, 4)
                for t in range(16):
                    for dd in range(4):
                        if v >> dd & 1:
                            acc[c, t] ^= f[(t - 4 * n - dd) % 16]
        for c in range(cw):
            for e in range(fin_off[tile, c], fin_off[tile, c + 1]):
                ent = int(fin[tile, e])
                assert ent & 15 == c
                b, j = (ent >> 4) & 15, ent >> 8
                v = np.zeros(W, np.int64)
                for t in range(16):
                    u = acc[c, t]
                    nz = u != 0
                    v ^= np.where(nz, exp[(log[u] + log[nb[(t + b) % 16]]) % 65535], 0)
                S[j] = v
    for tile in range(nt):  # the padding records (groups past the last, the two prefetched) are valid too
        for g in range(groups.shape[0], rec.shape[1]):
            assert all(v == 0 for _, v in _chain(rec[tile, g], where, 4 * cw))
    return S


def _chain(row, where, nb):
    """[(position, v)] of the blocks a step runs for record row: positions strictly increase and end at
    the last one (the block that returns)."""
    out, p = [], -1
    while True:
        q, v = where[int(row[p + 1])]
        assert q > p, (q, p)
        out.append((q, v))
        if q == nb - 1:
            return out
        p = q


@pytest.mark.parametrize("kind,k,r,t", [CASES[0], CASES[1], ("dec", 60, 40, 40), ("dec_bench", 512, 128, 128)])
def test_cs16t_plan_model_gives_the_syndromes(kind, k, r, t):
    """The threaded kernel's records (rsg_route_dump_t) reproduce H * X through a numpy model of its
    blocks, with its own tiling of cosets and finish lists."""
    exp, _ = gf_tables()
    er = _pattern(kind, k, r, t, seed=7)
    d = rs_amd.route_dump(k, r, er)
    dt = rs_amd.route_dump_t(k, r, er)
    pos, srcs, _ = _lists(k, r, er)
    X = np.random.default_rng(k * r).integers(0, 65536, (k + r, 2)).astype(np.int64)
    got = _model_syndromes_t(d, dt, X, normal_basis(16))
    H = exp[(np.arange(d["D"], dtype=np.int64)[:, None] * pos[srcs][None, :]) % 65535].astype(np.uint16)
    assert np.array_equal(got.astype(np.uint16), gf_apply(H, X[srcs].astype(np.uint16)))


def _model_bs16(d, Syn, nb):
    """k_bs16's arithmetic on CPU: syndromes Syn [D][W] -> {output slot: words}. Per (tile, group of 16
    syndromes) four subset tables over syndromes 4q .. 4q + 3; record byte 16q + t of a local coset is the
    table index added into accumulator u_t; finish out = sum_t nb_((t + b) mod 16) u_t."""
    exp, log = gf_tables()
    rec, fin, fin_off = d["rec"], d["fin"], d["fin_off"]
    nt, W, D = rec.shape[0], Syn.shape[1], d["D"]
    out = {}
    for tile in range(nt):
        acc = np.zeros((4, 16, W), np.int64)
        for g in range(d["ngroups"]):
            f = np.array([Syn[16 * g + i] if 16 * g + i < D else np.zeros(W, np.int64) for i in range(16)])
            for q in range(4):
                tab = np.zeros((16, W), np.int64)
                for e in range(16):
                    for dd in range(4):
                        if e >> dd & 1:
                            tab[e] ^= f[4 * q + dd]
                for c in range(4):
                    for tb in range(16):
                        acc[c, tb] ^= tab[rec[tile, g, c, 16 * q + tb]]
        for c in range(4):
            for e in range(fin_off[tile, c], fin_off[tile, c + 1]):
                ent = int(fin[tile, e])
                assert ent & 15 == c
                b, slot = (ent >> 4) & 15, ent >> 8
                v = np.zeros(W, np.int64)
                for t in range(16):
                    u = acc[c, t]
                    v ^= np.where(u != 0, exp[(log[u] + log[nb[(t + b) % 16]]) % 65535], 0)
                out[slot] = v
    return out


@pytest.mark.parametrize("kind,k,r,t,step", [("enc", 300, 200, None, 1), ("dec_bench", 4096, 1024, 1024, 4),
                                              ("dec_bench", 1024, 256, 256, 4), ("dec_cosets", 640, 128, 96, 1),
                                              ("dec", 600, 100, 80, None)])
def test_bs16_second_stage_model(kind, k, r, t, step):
    """k_bs16 as the route's second stage: the encode (repair cosets, Frobenius step 1) and decodes whose
    erased set is closed under a Frobenius power (the C5 bench pattern: every 4th slot of the 16-slot
    information cosets, closed under x -> x^16; whole information cosets: step 1). A numpy model of the
    kernel over the dumped records equals M2 * syndromes for every output; a random pattern has no such
    structure (None: the dense second stage)."""
    er = None
    if kind == "dec_bench":
        er = _pattern(kind, k, r, t)
    elif kind == "dec_cosets":  # whole 16-slot information cosets (slots 16 i .. 16 i + 15 of the first t / 16)
        er = np.zeros(k + r, bool)
        er[:t] = True
    elif kind == "dec":
        er = _pattern(kind, k, r, t, seed=9)
    d = rs_amd.bs16_dump(k, r, er)
    if step is None:
        assert d is None
        return
    assert d is not None and d["d"] == step
    route = rs_amd.route_dump(k, r, er)
    m2 = route["m2"]
    rng = np.random.default_rng(k + r)
    Syn = rng.integers(0, 65536, (d["D"], 2)).astype(np.int64)
    got = _model_bs16(d, Syn, normal_basis(16))
    _, _, tgts = _lists(k, r, er)
    outs = [s for s in (range(k, k + r) if er is None else tgts) if er is None or s < k]
    want = gf_apply(m2, Syn.astype(np.uint16))
    slots = [s - k for s in outs] if er is None else outs
    assert sorted(got) == sorted(slots)
    for i, sl in enumerate(slots):
        assert np.array_equal(got[sl].astype(np.uint16), want[i]), f"output slot {sl}"
