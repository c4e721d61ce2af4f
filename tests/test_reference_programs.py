"""The reference's own test programs, compiled from /root/reference against THIS repo's headers
and librs_amd.so (oracle/Makefile target `reftests`, outputs in oracle/_ref/reftests/, built by
__graft_entry__.build() where the reference is present; the binaries travel to the GPU box with the
tree). Exit status 0 = the reference's test passes with our library in place of src/rs:

  test_rs_gf_mul_ee / test_rs_gf_div_ee            GF(2^16) KATs (test/src/rs/gf65536/)
  test_rs_cc_*                                     coset selection (test/src/rs/cyclotomic_coset/)
  test_rs_random_data (GPU)                        100 random encode / erase / restore rounds,
                                                   k 100-199, r 50-99 (test/src/rs/test_random_data.c)
  example (GPU)                                    src/example.c end to end (checks itself with
                                                   assert(seq_eq(...)); built without NDEBUG)
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "..", "oracle", "_ref", "reftests")


def _run(name, timeout=120):
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not built (needs /root/reference at build time)")
    p = subprocess.run([path], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, f"{name} exit {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    return p.stdout


@pytest.mark.parametrize("name", ["test_rs_gf_mul_ee", "test_rs_gf_div_ee", "test_rs_cc_estimate_cosets_cnt",
                                  "test_rs_cc_select_cosets", "test_rs_cc_cosets_to_positions"])
def test_reference_host_programs(name):
    _run(name)


@pytest.mark.gpu
def test_reference_random_data_program():
    _run("test_rs_random_data", timeout=300)


@pytest.mark.gpu
def test_reference_example_program():
    _run("example")
