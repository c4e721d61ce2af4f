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
