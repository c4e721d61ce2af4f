"""Sanitizer run of the host code.

The reference checks its C code with -fanalyzer (CMakeLists.txt:16), cppcheck (compile_debug.sh:26-33)
and valgrind over every test (compile_test.sh:23). Here the same role is played by AddressSanitizer +
UndefinedBehaviorSanitizer builds of every host translation unit of librs_amd.so (`make -C
reed-solomon_amd asan`: allocators and registries, plan builders, the route's host plans, the XOR-kernel
generator, the reference-API shims) and of the oracle (`make -C oracle asan`), loaded into a Python run of
the GPU-free tests with the clang ASan runtime preloaded. Covered there: rsg_coding_matrix, rsg_route_dump
/ _t, rsg_bs16_dump, rsg_xj_source (and the generated kernels' emulation), the scalar GF / coset API,
seq_create / symbol_create / symbol_destroy churn through the idle pool, the pool cap and many address
reservations (RS_AMD_SYM_VA_MB=1), and the oracle against the golden vectors. Any sanitizer report
fails the run (halt_on_error for both; UBSan checks are not recoverable in these builds).

The C5-sized cases (k = 4096) and the exhaustive knob / column-loop generator sweeps are left to the
plain suite: under the sanitizers they take minutes each and exercise no other code.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_RT = "/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so"

SKIP = ("not 4096 and not c5 and not knobs and not column_loop and not header_layouts and not no_compiler_code "
        "and not release_build and not max_n and not 1100")


@pytest.mark.timeout(1200)
def test_host_code_under_asan_and_ubsan():
    if not os.path.exists(ASAN_RT):
        pytest.skip("clang ASan runtime not found")
    subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(REPO, "reed-solomon_amd"), "asan"])
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"])
    env = dict(os.environ)
    env.update(
        LD_PRELOAD=ASAN_RT,
        ASAN_OPTIONS="halt_on_error=1:detect_leaks=0:abort_on_error=0",  # the HIP runtime keeps its state at exit
        UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
        RS_AMD_LIB=os.path.join(REPO, "reed-solomon_amd", "librs_amd_asan.so"),
        RS_ORACLE_LIB=os.path.join(REPO, "oracle", "librs_oracle_asan.so"),
        RS_AMD_SYM_VA_MB="1",
    )
    env.pop("PYTEST_XDIST_WORKER", None)
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-p", "no:xdist", "-m",
           "not gpu and not slow", "tests/test_oracle.py", "tests/test_route.py", "tests/test_host.py",
           "tests/test_xj.py", "-k", SKIP]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=1100)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert r.returncode == 0, out[-6000:]
    assert " passed" in r.stdout and " failed" not in r.stdout
