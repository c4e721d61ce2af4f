"""CPU check of every gfx950 kernel the libraries carry, and of the hiprtc-specialised kernels, for the
fault class behind GPUTEST_r04's illegal memory access: a register read while a memory load into it
is still in flight (CDNA does not interlock memory results; inline asm whose outputs are not
early-clobber lets the compiler place an asm input inside an asm output).

Round 4's instance: `sload32` (csrc/rs_device.h) compiled in rs_v1jit to
    s_load_dwordx16 s[8:23], s[10:11], 0x0
    s_load_dwordx16 s[72:87], s[10:11], 0x40
The same helper put the same pattern into the production per-stripe solve k_apply_m8_v1<0>.
No GPU is used: the code objects are disassembled with the ROCm llvm-objdump."""
import ctypes
import os
import shutil
import sys

import numpy as np
import pytest

from _util import REPO

sys.path.insert(0, os.path.join(REPO, "scripts"))
import isa_hazards  # noqa: E402

import rs_amd  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(f"{isa_hazards.LLVM}/llvm-objdump"), reason="no ROCm llvm-objdump")
PKG = os.path.join(REPO, "reed-solomon_amd")


def _check(path):
    text = isa_hazards.disassemble(path)
    found = isa_hazards.hazards(text)
    assert not found, "\n".join(f"{f} @{a}: {i}  in flight {r}" for f, a, i, r in found)
    found = isa_hazards.valu_sgpr_hazards(text)
    assert not found, "\n".join(f"{f} @{a}: {i}  VALU-written SGPR {r}" for f, a, i, r in found)


def test_checker_flags_valu_written_sgpr_read_by_vmem():
    """The second check: an SGPR from v_readfirstlane used as a store's saddr two instructions later (gfx9
    needs 5 wait states; inline asm gets no s_nop from the compiler), and the same with an s_nop 4 between."""
    bad = """
0000000000000000 <k3>:
\tv_readfirstlane_b32 s4, v1                                  // 000000000000: 7E080501
\tv_xor_b32_e32 v5, v4, v5                                   // 000000000004: 2A0A0B04
\tglobal_store_dword v2, v3, s[4:5]                          // 000000000008: DC708000 00040302
"""
    found = isa_hazards.valu_sgpr_hazards(bad)
    assert len(found) == 1 and found[0][3] == [("s", 4)], found
    good = bad.replace("\tv_xor_b32_e32 v5, v4, v5                                   // 000000000004: 2A0A0B04",
                       "\ts_nop 4                                                   // 000000000004: BF800004")
    assert not isa_hazards.valu_sgpr_hazards(good)
    # a VALU compare into an SGPR pair, then a buffer load with that pair as its soffset's neighbour
    cmp = """
0000000000000000 <k4>:
\tv_cmp_eq_u32_e64 s[6:7], v1, v2                            // 000000000000: D0CA0006 00020501
\tbuffer_load_dword v3, v4, s[8:11], s6 offen                // 000000000008: E0501000 06020304
"""
    found = isa_hazards.valu_sgpr_hazards(cmp)
    assert len(found) == 1 and found[0][3] == [("s", 6)], found


def test_checker_flags_the_round4_pattern():
    """The checker itself: the two SMEM loads of round 4's rs_v1jit, and a clean variant."""
    bad = """
0000000000001800 <k>:
\ts_waitcnt lgkmcnt(0)                                       // 00000000321C: BF8CC07F
\ts_load_dwordx16 s[8:23], s[10:11], 0x0                     // 000000003224: C0120205 00000000
\ts_load_dwordx16 s[72:87], s[10:11], 0x40                   // 00000000322C: C0121205 00000040
\ts_waitcnt lgkmcnt(0)                                       // 000000003234: BF8CC07F
"""
    found = isa_hazards.hazards(bad)
    assert len(found) == 1 and found[0][3] == [("s", 10), ("s", 11)], found
    good = bad.replace("s[8:23], s[10:11], 0x0", "s[24:39], s[10:11], 0x0")
    assert not isa_hazards.hazards(good)
    # a VMEM result read before its vmcnt wait; then the same after the wait
    vm = """
0000000000000000 <k2>:
\tglobal_load_dword v4, v[2:3], off                          // 000000000000: DC508000 047F0002
\tv_xor_b32_e32 v5, v4, v5                                   // 000000000008: 2A0A0B04
\ts_waitcnt vmcnt(0)                                         // 00000000000C: BF8C0F70
\tv_xor_b32_e32 v5, v4, v5                                   // 000000000010: 2A0A0B04
"""
    found = isa_hazards.hazards(vm)
    assert [f[1] for f in found] == ["8"], found


@pytest.mark.parametrize("lib", ["librs_amd.so", "librs_amd_diag.so"])
def test_library_kernels_have_no_inflight_reads(lib):
    path = os.path.join(PKG, lib)
    if not os.path.exists(path):
        pytest.skip(f"{lib} not built")
    _check(path)


# matrix-specialised kernels: (k, r, erasure pattern or None). 128 x 64 is past the XOR kernel's work
# bound (K * R > 6144), so it compiles the nibble-table rs_v1jit -- the library's default for such shapes
JIT_SHAPES = [(10, 4, None), (128, 32, None), (128, 64, None), (128, 64, "bench")]


@pytest.mark.parametrize("k,r,pattern", JIT_SHAPES)
def test_jit_kernels_have_no_inflight_reads(k, r, pattern, tmp_path, monkeypatch):
    monkeypatch.setenv("RS_AMD_JIT_CACHE", str(tmp_path))
    er = rs_amd.bench_pattern(k, r) if pattern else None
    rs_amd.jit_precompile(k, r, er)  # raises on failure
    objs = [os.path.join(tmp_path, f) for f in os.listdir(tmp_path) if f.endswith(".co")]
    assert objs, "no specialised kernel compiled"
    if (k, r) == (128, 64):
        assert all(os.path.basename(o).startswith("v1_") for o in objs), objs  # the nibble-table rs_v1jit
    for o in objs:
        _check(o)


def _kernel_names(path):
    import re
    text = isa_hazards.disassemble(path)
    return {m.group(1) for m in re.finditer(r"^[0-9a-f]+ <([^>]+)>:", text, re.M) if not m.group(1).startswith(("L_", ".L"))}


# kernel families reachable only through A/B options, ablations or stamps: diagnostic build only
DIAG_ONLY = ("k_apply_m8ILi", "k_apply_m8_lds", "k_apply_m8_ps_w", "k_apply_m8_idxILi0ELi8E", "k_apply_m8_idxILi4E",
             "k_apply_m8_v1ILi1E", "k_apply_m8_v1ILi3E", "k_apply_m8_v1ILi4E", "k_apply_m8_v1ILi5E", "k_apply_m8_v1ILi6E",
             "k_apply_m16_v1ILi1E", "k_apply_m8_pfILi1E", "k_apply_m8_pfILi3E", "k_apply_m8_pfILi12E",
             "k_apply_m8_pfILi13E", "k_apply_m8_pfILi4E")
# every production kernel (the release library carries exactly these)
PRODUCTION = ("k_apply_m8_v1ILi0E", "k_apply_m8_v1ILi2E", "k_apply_m8_idxILi0ELi4E", "k_apply_m8_ps_tail", "k_apply_m8_pf", "k_xor_slices",
              "k_apply_m16ILi16E", "k_apply_m16ILi32E", "k_apply_m16ILi64E", "k_apply_m16_v1ILi0E", "k_cs16E", "k_cs16tE",
              "k_bs16E", "k_cs16_goff", "k_plan_m8", "k_plan_syn_m8", "k_plan_reenc_m8", "k_plan16_sums", "k_plan16_fill",
              "k_plan16_ps", "k_plan16_ps_rec", "k_plan16_reenc", "k_plan16_reenc_logs", "k_plan16_reenc_rec",
              "k_symbol_op", "k_gen_info", "k_fingerprint", "k_gather_rows", "k_put_rows", "k_xor_rows",
              "k_gather_ptrs", "k_scatter_ptrs", "k_symbol_chains", "k_symop_consts")


def test_release_build_has_no_ablation_kernels():
    """The release library's kernel set is the production set: no option-only A/B family, ablation or
    stamped kernel (those are in librs_amd_diag.so, whose kernel set is a superset)."""
    rel = _kernel_names(os.path.join(PKG, "librs_amd.so"))
    bad = sorted(n for n in rel if any(d in n for d in DIAG_ONLY))
    assert not bad, bad
    unknown = sorted(n for n in rel if not any(p in n for p in PRODUCTION))
    assert not unknown, unknown
    missing = [p for p in PRODUCTION if not any(p in n for n in rel)]
    assert not missing, missing
    diag = os.path.join(PKG, "librs_amd_diag.so")
    if os.path.exists(diag):
        d = _kernel_names(diag)
        assert rel <= d and any(any(x in n for x in DIAG_ONLY) for n in d)


@pytest.mark.parametrize("k,r,route", [(128, 32, 2), (128, 32, 1), (10, 4, 2)])
def test_masked_fixed_pass_compiles_without_inflight_reads(k, r, route, tmp_path, monkeypatch):
    """The GF(256) per-stripe route's masked fixed-pass kernel compiles with hiprtc and has no in-flight read."""
    monkeypatch.setenv("RS_AMD_JIT_CACHE", str(tmp_path))
    assert rs_amd._lib.rsg_xj_fixed_precompile(k, r, route) == 0
    objs = [os.path.join(tmp_path, f) for f in os.listdir(tmp_path) if f.endswith(".co")]
    assert len(objs) == 1, objs
    _check(objs[0])
