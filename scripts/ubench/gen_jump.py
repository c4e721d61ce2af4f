#!/usr/bin/env python3
"""Generates jump_bench.hip: cost of computed jumps into fixed-register code blocks (the candidate
k_cs16 step without gpr indexing). Per step: for 4 cosets x 4 nibbles, a block index byte is extracted
from SGPRs (s_bfe_u32), turned into a trampoline address (s_lshl_b32, s_add_u32 / s_addc_u32), entered by
s_swappc_b64; the trampoline s_branches to its block of full-rate v_bitop3 (u_t ^= sources of the
circulant's nibble), which returns with s_setpc_b64. "inline" runs the same blocks' VALU straight-line.
Timed with s_memtime per wave; block = 256 * W threads (W waves per SIMD), one workgroup per CU.
Prints cycles per step per wave and VALU cycles per SIMD."""
import random
import sys

random.seed(7)
F, ACC = 8, 24  # inputs f_0..15 in v[8:23]; accumulators of coset c in v[24 + 16c ..]


def block_ops(c, n, v):
    ops = []
    for t in range(16):
        src = [F + (t - 4 * n - d) % 16 for d in range(4) if v >> d & 1]
        a = ACC + 16 * c + t
        while src:
            if len(src) >= 2:
                ops.append(f"v_bitop3_b32 v{a}, v{a}, v{src[0]}, v{src[1]} bitop3:0x96")
                src = src[2:]
            else:
                ops.append(f"v_xor_b32_e64 v{a}, v{a}, v{src[0]}")
                src = src[1:]
    return ops


STEPS = 8  # distinct steps per loop iteration (index patterns)
pattern = [[random.randrange(1, 16) for _ in range(16)] for _ in range(STEPS)]  # v per (c, n)


def kernel(name, jump):
    L = []
    # index bytes for every step in s[40 + 4 * step ...] (4 dwords per step: byte 4c + n)
    setup = []
    for st in range(STEPS):
        for w in range(4):
            val = 0
            for b in range(4):
                cn = 4 * w + b
                c, n = cn // 4, cn % 4
                val |= (c * 64 + n * 16 + pattern[st][cn]) << (8 * b)
            setup.append(f"s_mov_b32 s{40 + 4 * st + w}, 0x{val:08x}")
    L += setup
    L += [f"v_mov_b32 v{F + i}, {i * 7 + 1}" for i in range(16)]
    L += [f"v_mov_b32 v{ACC + i}, 0" for i in range(64)]
    L += ["s_getpc_b64 s[74:75]", "s_add_u32 s74, s74, L_tab%=-.", "s_addc_u32 s75, s75, 0"]
    L += ["s_memtime %[t0]", "s_mov_b32 s22, %[iters]", "s_waitcnt lgkmcnt(0)", "L_loop%=:"]
    for st in range(STEPS):
        for cn in range(16):
            c, n = cn // 4, cn % 4
            if jump:
                w, b = cn // 4, cn % 4
                L.append(f"s_bfe_u32 s72, s{40 + 4 * st + w}, 0x{(8 << 16) | (8 * b):x}")
                L.append("s_lshl_b32 s72, s72, 2")
                L.append("s_add_u32 s76, s74, s72")
                L.append("s_addc_u32 s77, s75, 0")
                L.append("s_swappc_b64 s[78:79], s[76:77]")
            else:
                L += block_ops(c, n, pattern[st][cn])
    L += ["s_sub_u32 s22, s22, 1", "s_cmp_lg_u32 s22, 0", "s_cbranch_scc1 L_loop%=", "s_memtime %[t1]",
          "s_waitcnt lgkmcnt(0)", "s_branch L_end%="]
    L.append("L_tab%=:")
    for c in range(4):
        for n in range(4):
            for v in range(16):
                L.append(f"s_branch L_b{c}_{n}_{v}%=")
    for c in range(4):
        for n in range(4):
            for v in range(16):
                L.append(f"L_b{c}_{n}_{v}%=:")
                L += block_ops(c, n, v)
                L.append("s_setpc_b64 s[78:79]")
    L.append("L_end%=:")
    nvalu = sum(len(block_ops(cn // 4, cn % 4, pattern[st][cn])) for st in range(STEPS) for cn in range(16))
    text = "".join(f'"{x}\\n\\t"' for x in L)
    vclob = ", ".join(f'"v{r}"' for r in range(8, 88))
    sclob = ", ".join(f'"s{r}"' for r in list(range(20, 24)) + list(range(40, 80)))
    return f'''__global__ void __launch_bounds__(1024) {name}(unsigned long long* out, int iters) {{
    unsigned long long t0, t1;
    asm volatile({text} : [t0] "=&s"(t0), [t1] "=&s"(t1) : [iters] "s"(iters) : {vclob}, {sclob}, "scc");
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}}
static const int nvalu_{name} = {nvalu};'''


out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <algorithm>',
       kernel("k_jump", True), kernel("k_inline", False),
       r'''typedef void (*kfn)(unsigned long long*, int);
int main() {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 200;
    unsigned long long* d; hipMalloc(&d, sizeof(unsigned long long) * cus * 32);
    std::vector<unsigned long long> h(cus * 32);
    kfn fns[2] = {k_jump, k_inline};
    const char* names[2] = {"jump", "inline"};
    const int nv[2] = {nvalu_k_jump, nvalu_k_inline};
    for (int k = 0; k < 2; ++k)
        for (int w = 1; w <= 4; ++w) {
            hipLaunchKernelGGL(fns[k], dim3(cus), dim3(256 * w), 0, 0, d, iters);  // warm
            hipLaunchKernelGGL(fns[k], dim3(cus), dim3(256 * w), 0, 0, d, iters);
            if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s\"}\n", names[k]); return 1; }
            hipMemcpy(h.data(), d, sizeof(unsigned long long) * cus * 4 * w, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.begin() + cus * 4 * w);
            const double med = double(h[cus * 2 * w]);
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_step_wave\": %.1f, \"cyc_per_valu_simd\": %.3f}\n",
                   names[k], w, med / (double(iters) * 8), med / (double(iters) * nv[k] * w));
            fflush(stdout);
        }
    return 0;
}''']
open(sys.argv[1] if len(sys.argv) > 1 else "jump_bench.hip", "w").write("\n".join(out) + "\n")
