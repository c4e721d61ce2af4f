"""GPU parity tests (MI355X) of the non-default kernel variants, run after the production suite
(tests/test_gpu.py) so that a failure in an option-only family cannot hide the production path.

Release-library variants: the forced XOR kernel (jit), the nibble-table rs_v1jit (xj=0: the library's
default for shapes the XOR kernel rejects), the generic V = 1 kernels with two / one nibble tables per
input (v1 / v1h), and the GF(2^16) route on the gpr-indexed k_cs16 (cs_idx). Diagnostic-library variants
(librs_amd_diag.so, loaded beside the release library by rs_amd.diag_module()): the LDS-DMA gpr-index
kernel (idx), the compiler-indexed reference kernels (table / mask), the per-stripe solve A/B kernels,
overlapped chunks, multi-chunk workgroups and the 1 KiB route block layout. Same checks as the production
tests: reference goldens, C2 every stripe vs the oracle, C3-shape round trips, non-codeword decodes."""
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
