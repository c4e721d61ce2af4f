"""GPU parity tests (MI355X) of the non-default kernel variants, run after the production suite
(tests/test_gpu.py) so that a failure in an option-only family cannot hide the production path.

Release-library variants: the forced XOR kernel (jit), the nibble-table rs_v1jit (xj=0: the library's
default for shapes the XOR kernel rejects), the generic V = 1 kernels with two / one nibble tables per
input (v1 / v1h), and the GF(2^16) route on the gpr-indexed k_cs16 (cs_idx). Diagnostic-library variants
(librs_amd_diag.so, loaded beside the release library by rs_amd.diag_module()): the LDS-DMA gpr-index
kernel (idx), the compiler-indexed reference kernels (table / mask), the per-stripe solve A/B kernels,
overlapped chunks, multi-chunk workgroups and the 1 KiB route block layout. Same checks as the production
tests: reference goldens, C2 every stripe vs the oracle, C3-shape round trips, non-codeword decodes."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import rs_amd  # noqa: E402
from test_gpu import (BATCH_CASES, SYN_ROUTE_SHAPES, VARIANTS, config2_case, config3_case,  # noqa: E402
                      cs16_overlapped_case, golden_batch_case, m16_shapes_case, noncodeword_case, syndrome_route_case)

pytestmark = pytest.mark.gpu

OTHER = [v for v in VARIANTS if v != "auto"]


@pytest.mark.parametrize("variant", OTHER)
@pytest.mark.parametrize("name", BATCH_CASES)
def test_golden_batch_api_variant(name, variant):
    golden_batch_case(name, variant)


@pytest.mark.parametrize("variant", [v for v in OTHER if v != "cs_idx"])
def test_config2_all_stripes_vs_oracle_variant(variant):
    config2_case(variant)


@pytest.mark.parametrize("variant", [v for v in OTHER if v != "cs_idx"])
def test_config3_shape_roundtrip_variant(variant):
    config3_case(variant)


def test_decode_matches_oracle_on_noncodewords_variants():
    noncodeword_case([v for v in OTHER if v != "cs_idx"])


# diagnostic-library settings of the GF(256) per-stripe decode: overlapped chunks (ovl), the A/B solve kernels
# 1 (k_apply_m8_ps_w), 2 (_w2), 4 / 5 (ring-kernel table variants), 9 / 11 (prefetching solves with two tables /
# read multiples), several column chunks per workgroup (cpb)
@pytest.mark.parametrize("route,ovl,kern,cpb", [(1, 1, 0, 1), (1, 0, 1, 1), (0, 0, 1, 1), (1, 0, 2, 1), (1, 1, 2, 1),
                                                (0, 0, 2, 1), (2, 1, 0, 1), (2, 0, 2, 1), (2, 1, 2, 1), (2, 0, 0, 3),
                                                (2, 1, 0, 4), (1, 0, 0, 64), (0, 0, 0, 2), (2, 0, 4, 1), (2, 0, 5, 1),
                                                (2, 0, 9, 1), (1, 0, 9, 1), (2, 0, 11, 1), (1, 0, 11, 1), (2, 1, 10, 1)])
@pytest.mark.parametrize("k,r,S,n", SYN_ROUTE_SHAPES)
def test_decode_batch_syndrome_route_diag(k, r, S, n, route, ovl, kern, cpb):
    syndrome_route_case(rs_amd.diag_module(), k, r, S, n, route, ovl, kern, cpb)


@pytest.mark.parametrize("route", [1, 2])
@pytest.mark.parametrize("k,r,S,n", SYN_ROUTE_SHAPES)
def test_decode_batch_syndrome_route_coord(k, r, S, n, route):
    """Option m8_syn_coord 1 (diagnostic library): the masked fixed pass stores GF(256)^2 coordinates and the
    prefetching solve reads them as they are (k_apply_m8_pf<4>)."""
    syndrome_route_case(rs_amd.diag_module(), k, r, S, n, route, 0, 10, 1, coord=1)


@pytest.mark.parametrize("k,r,S,n", [(1000, 200, 2048, 37), (300, 64, 3072, 16)])
def test_cs16_overlapped_chunks_match_serial(k, r, S, n):
    cs16_overlapped_case(k, r, S, n)


@pytest.mark.parametrize("k,r,S", [(250, 33, 1024), (300, 64, 2048 + 40), (200, 65, 1024 + 1000), (1000, 100, 2048),
                                   (400, 129, 3072 + 4), (2000, 100, 1024)])
@pytest.mark.parametrize("route", [0, 1])
def test_m16_kernel_shapes_route_layout_1k(k, r, S, route):
    """The GF(2^16) shapes with the route kernels' 1 KiB block layout (m16_cs_col 1024, diagnostic build)."""
    m16_shapes_case(rs_amd.diag_module(), k, r, S, route, 1024)


def test_failed_group_fences_scratch_for_next_stream():
    """rsg_decode_batch's host-plan grouping path (<= 16 distinct patterns) failing after some group kernels
    were launched (diagnostic option inject_fail_group: the n-th group's plan fails with RS_ERR_DEVICE): the
    call must still mark the codec scratch (the stripe-id list those kernels read) busy on its stream, so a
    following call on another stream waits for the orphaned kernels before it restages the list. Checks: the
    second call returns only after the first stream's kernels are done, the launched groups restored their
    stripes bit-exactly (their id list was not overwritten under them), the failed group's stripes are
    untouched, and the second batch is correct."""
    k, r, S, per = 128, 32, 65536, 512
    groups = 4
    n = groups * per
    diag = rs_amd.diag_module()
    codec = diag.Codec(k, r)
    codec.set_option("inject_fail_group", groups - 1)
    dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0x6A11)
    rs_amd.Codec(k, r).encode(dev)
    ref = torch.zeros(n, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(dev, 0, k, ref)
    rng = np.random.default_rng(61)
    pats = np.zeros((n, k + r), bool)
    for g in range(groups):  # stripes interleaved over the groups: every launch goes through the id list
        p = np.zeros(k + r, bool)
        p[rng.choice(k, r, replace=False)] = True
        pats[g::groups] = p
    mask = torch.from_numpy(pats).cuda()
    dev.masked_fill_(mask[:, :, None], 0)
    small = torch.empty((8, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(small, k, seed=0x6A12)
    rs_amd.Codec(k, r).encode(small)
    small_ref = torch.zeros(8, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(small, 0, k, small_ref)
    spats = np.zeros((8, k + r), bool)
    for s in range(8):
        spats[s, rng.choice(k, 3, replace=False)] = True
    small.masked_fill_(torch.from_numpy(spats).cuda()[:, :, None], 0)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    rc = codec.decode_batch(dev, pats, stream=sa, check=False)
    assert rc == rs_amd.RS_ERR_DEVICE, rc
    done_a = torch.cuda.Event()
    done_a.record(sa)
    codec.set_option("inject_fail_group", -1)
    assert codec.decode_batch(small, spats, stream=sb) == 0
    assert done_a.query(), "the call on the second stream returned before the failed call's kernels finished"
    torch.cuda.synchronize()
    fp = torch.zeros(n, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(dev, 0, k, fp)
    launched = np.array([s % groups != groups - 1 for s in range(n)])
    idx = torch.from_numpy(np.nonzero(launched)[0]).cuda()
    assert torch.equal(fp[idx], ref[idx]), "a launched group restored wrong bytes"
    lost = torch.from_numpy(np.nonzero(pats[groups - 1])[0]).cuda()
    assert int(dev[groups - 1::groups][:, lost].count_nonzero()) == 0, "the failed group's stripes were written"
    sfp = torch.zeros(8, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(small, 0, k, sfp)
    torch.cuda.synchronize()
    assert torch.equal(sfp, small_ref)
