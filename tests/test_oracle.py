"""Pins the CPU oracle (oracle/rs_oracle.c) to the reference: its own KATs and the golden vectors
generated from the compiled reference (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from _util import EXTRA_OPS, case, check_golden, manifest, oracle, oracle_positions, ptr, run_case_oracle, run_extra_numpy

# test/src/rs/gf65536/test_gf_mul_ee.c:36-42 and test_gf_div_ee.c:36-42 (SageMath vectors)
MUL_KAT = [(1, 645, 645), (46478, 0, 0), (31981, 38739, 42167), (2491, 54249, 5290),
           (60895, 36296, 21017), (62824, 46526, 6710), (58263, 29917, 33120)]
DIV_KAT = [(0, 45687, 0), (65512, 65512, 1), (12320, 29623, 11439), (31193, 63233, 27486),
           (21844, 54054, 49588), (38756, 35149, 10047), (5768, 15888, 24163)]


def test_gf_kats():
    o = oracle()
    for a, b, want in MUL_KAT:
        assert o.orc_mul(a, b) == want
    for a, b, want in DIV_KAT:
        assert o.orc_div(a, b) == want


def _select(k, r):
    o = oracle()
    ci, cr = o.orc_cosets_upper(k), o.orc_cosets_upper(r)
    il, rl = np.zeros(ci + 1, np.uint16), np.zeros(cr + 1, np.uint16)
    isz, rsz = np.zeros(ci + 1, np.uint8), np.zeros(cr + 1, np.uint8)
    ni, nr = np.zeros(1, np.uint16), np.zeros(1, np.uint16)
    o.orc_select_cosets(k, r, ptr(il), ptr(isz), ptr(ni), ptr(rl), ptr(rsz), ptr(nr))
    inf = list(zip(il[:ni[0]].tolist(), isz[:ni[0]].tolist()))
    rep = list(zip(rl[:nr[0]].tolist(), rsz[:nr[0]].tolist()))
    return inf, rep


# test/src/rs/cyclotomic_coset/test_cc_select_cosets.c:107-187
SELECT_KAT = [
    (16, 3, [(257, 8), (4369, 4), (13107, 4)], [(21845, 2), (0, 1)]),
    (11, 11, [(257, 8), (30583, 4)], [(4369, 4), (13107, 4), (21845, 2), (0, 1)]),
    (19, 18, [(771, 8), (1285, 8), (30583, 4)], [(257, 8), (4369, 4), (13107, 4), (21845, 2)]),
    (22, 17, [(771, 8), (1285, 8), (30583, 4), (21845, 2)], [(257, 8), (4369, 4), (13107, 4), (0, 1)]),
]


@pytest.mark.parametrize("k,r,inf,rep", SELECT_KAT)
def test_select_cosets_kat(k, r, inf, rep):
    gi, gr = _select(k, r)
    assert gi == inf and gr == rep


# test/src/rs/cyclotomic_coset/test_cc_estimate_cosets_cnt.c:36-45 (lower bounds)
@pytest.mark.parametrize("k,r,lbi,lbr", [(19, 0, 5, 0), (255, 0, 35, 0), (389, 0, 42, 0), (16, 3, 3, 2),
                                         (11, 11, 2, 4), (19, 18, 3, 4), (1034, 389, 66, 42)])
def test_estimate_cosets_kat(k, r, lbi, lbr):
    o = oracle()
    assert o.orc_cosets_upper(k) >= lbi and o.orc_cosets_upper(r) >= lbr


def test_positions_survey_fingerprints():
    # SURVEY.md section 8 a-7 (measured on the reference)
    p = oracle_positions(4, 2)
    assert p.tolist() == [4369, 8738, 17476, 34952, 21845, 43690]
    p = oracle_positions(10, 4)
    assert p[10:].tolist() == [4369, 8738, 17476, 34952]


# max_n_route_*: k + r = 65535 at 1 KiB symbols, a minute of CPU per case; pinned by the reference's
# own outputs (the golden) and checked on the GPU only
CASES = [c["name"] for c in manifest()["cases"] if c["op"] not in EXTRA_OPS and not c["name"].startswith("max_n_route")]
EXTRA = [c["name"] for c in manifest()["cases"] if c["op"] in EXTRA_OPS]
FAST = [n for n in CASES if not n.startswith(("gmat_4096", "c5_", "c3_dec_bench_64k"))]
SLOW = [n for n in CASES if n not in FAST]


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_golden(name):
    c = case(name)
    rc, out = run_case_oracle(c)
    assert rc == c["rc"]
    check_golden(c, out)


@pytest.mark.slow
@pytest.mark.parametrize("name", SLOW)
def test_oracle_matches_golden_slow(name):
    c = case(name)
    rc, out = run_case_oracle(c)
    assert rc == c["rc"]
    check_golden(c, out)


@pytest.mark.parametrize("name", EXTRA)
def test_transforms_and_symbol_ops_match_golden(name):
    """gf_add / gf_mul / gf_madd and the four fft_* transforms restated in numpy (the matrices the
    product forms, src/rs/fft.c entry by entry) against the reference's outputs."""
    c = case(name)
    check_golden(c, run_extra_numpy(c))
