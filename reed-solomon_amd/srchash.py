"""Identity of a kernel build for measurements recorded under profiles/ (traffic.json): a hash of
the sources that generate the kernel family, so an edit elsewhere does not void a measurement of an
unchanged kernel."""
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# bit-plane XOR kernels are generated at run time from these (generator, hiprtc wrapper, matrices)
_JIT_XJ = ("csrc/rs_xj.cpp", "csrc/rs_xj.hpp", "csrc/rs_jit.cpp", "csrc/gf16.cpp", "csrc/gf16.hpp")
# everything compiled ahead of time into librs_amd.so
_AOT = ("csrc/rs_kernels.hip", "csrc/gen_asm.py", "csrc/rs_device.h", "csrc/rs_v1args.h", "csrc/rs_kernels.hpp")


def kernel_src_hash(kernel):
    h = hashlib.sha256()
    files = _JIT_XJ if str(kernel).startswith("rs_xj") else _AOT
    for f in files:
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
