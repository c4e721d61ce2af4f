#!/usr/bin/env python3
"""Generates thread_bench.hip: can a k_cs16 group step run without gpr-indexed VALU?

Today's step (variant "idx"): four 16-entry subset tables over the group's 16 inputs (44 XORs), then per
syndrome coset 16 gpr-index switches feeding 4 half-rate indexed XORs each (256 indexed XORs per step of
4 cosets). Candidate ("thread"): no tables; the circulant of (group, coset) is its z's four nibbles
v_n, and block (c, n, v) XORs the raw inputs straight into coset c's accumulators
    u_t ^= f_((t - 4n - d) mod 16)   for the set bits d of v
with fixed register names (full-rate v_bitop3). The blocks are threaded: each ends by jumping to the
next block of the step (its offset from the step's record, one SGPR per block, loaded by s_load), the
last back to the step driver -- one s_setpc per block. "inline" runs the same kind of blocks straight-line
(the VALU floor). Per step every variant also moves 16 inputs (v_mov), as the real step does.

Blocks at a fixed 512-byte stride (offset = (4c + n) * 16 + v, times 512). One workgroup of 256 * W
threads per CU (W waves per SIMD), timed with s_memtime per wave over NSTEPS random steps.
Prints cycles per step per wave and SIMD cycles per step (the figure to compare across variants)."""
import random
import sys

random.seed(11)
F, ACC, LD = 8, 24, 88  # inputs v[8:23], accumulators v[24 : 24 + 16C], load ring v[88:103]
STRIDE = 512
NSTEPS = 4096


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
                ops.append(f"v_xor_b32 v{a}, v{a}, v{src[0]}")
                src = src[1:]
    return ops


def q(lines):
    return "".join(f'"{x}\\n\\t"' for x in lines)


def wrap(name, body, nvgpr=104, extra_s=(), lb=1024):
    vclob = ", ".join(f'"v{r}"' for r in range(8, nvgpr))
    sclob = ", ".join(f'"s{r}"' for r in list(range(40, 80)) + list(range(96, 98)) + list(extra_s))
    return f'''__global__ void __launch_bounds__({lb}) {name}(unsigned long long* out, const unsigned* rec, int nsteps) {{
    unsigned long long t0, t1;
    asm volatile({q(body)} : [t0] "=&s"(t0), [t1] "=&s"(t1) : [rec] "s"(rec), [nsteps] "s"(nsteps) : {vclob}, {sclob}, "scc", "memory");
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}}'''


def init():
    return ([f"v_mov_b32 v{F + i}, {i * 7 + 1}" for i in range(16)] + [f"v_mov_b32 v{ACC + i}, 0" for i in range(64)]
            + [f"v_mov_b32 v{LD + i}, {i * 5 + 3}" for i in range(16)])


def thread_kernel(C):
    nb = 4 * C  # blocks per step; record = nb dwords
    ld = {4: "s_load_dwordx16", 2: "s_load_dwordx8"}[C]
    B = init()
    B += ["s_getpc_b64 s[96:97]", "s_add_u32 s96, s96, L_blocks%=-.", "s_addc_u32 s97, s97, 0",
          "s_mov_b64 s[72:73], %[rec]", f"{ld} s[56:{55 + nb}], s[72:73], 0x0",
          f"s_add_u32 s72, s72, {4 * nb}", "s_addc_u32 s73, s73, 0", "s_mov_b32 s74, %[nsteps]",
          "s_waitcnt lgkmcnt(0)", "s_memtime %[t0]", "s_waitcnt lgkmcnt(0)", "L_loop%=:"]
    B += ["s_waitcnt lgkmcnt(0)"] + [f"s_mov_b64 s[{40 + 2 * i}:{41 + 2 * i}], s[{56 + 2 * i}:{57 + 2 * i}]" for i in range(nb // 2)]
    B += [f"{ld} s[56:{55 + nb}], s[72:73], 0x0", f"s_add_u32 s72, s72, {4 * nb}", "s_addc_u32 s73, s73, 0"]
    B += [f"v_mov_b32 v{F + i}, v{LD + i}" for i in range(16)]
    B += ["s_getpc_b64 s[78:79]", "s_add_u32 s78, s78, L_ret%=-.", "s_addc_u32 s79, s79, 0",
          "s_add_u32 s76, s96, s40", "s_addc_u32 s77, s97, 0", "s_setpc_b64 s[76:77]", "L_ret%=:",
          "s_sub_u32 s74, s74, 1", "s_cmp_lg_u32 s74, 0", "s_cbranch_scc1 L_loop%=",
          "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)", "s_getpc_b64 s[76:77]", "s_add_u32 s76, s76, L_end%=-.",
          "s_addc_u32 s77, s77, 0", "s_setpc_b64 s[76:77]", ".p2align 9", "L_blocks%=:"]
    for c in range(C):
        for n in range(4):
            p = 4 * c + n
            for v in range(16):
                B.append(".p2align 9")
                B += block_ops(c, n, v)
                if p < nb - 1:
                    B += [f"s_add_u32 s76, s96, s{41 + p}", "s_addc_u32 s77, s97, 0", "s_setpc_b64 s[76:77]"]
                else:
                    B.append("s_setpc_b64 s[78:79]")
    B.append("L_end%=:")
    return wrap(f"k_thread{C}", B)


INL_STEPS = 8
inl_pat = [[random.randrange(0, 16) for _ in range(16)] for _ in range(INL_STEPS)]


def inline_kernel():
    B = init() + ["s_mov_b32 s74, %[nsteps]", "s_lshr_b32 s74, s74, 3", "s_memtime %[t0]", "s_waitcnt lgkmcnt(0)", "L_loop%=:"]
    for st in range(INL_STEPS):
        B += [f"v_mov_b32 v{F + i}, v{LD + i}" for i in range(16)]
        for p in range(16):
            B += block_ops(p // 4, p % 4, inl_pat[st][p])
    B += ["s_sub_u32 s74, s74, 1", "s_cmp_lg_u32 s74, 0", "s_cbranch_scc1 L_loop%=", "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)"]
    return wrap("k_inline", B)


def idx_kernel():
    # today's step without its loads: 44 table XORs, then per coset 16 switches x 4 indexed XORs.
    # Tables T_q in v[8 + 16q ..] (64 VGPRs), accumulators v[72:135]; index bytes from 16 SGPRs s[40:55]
    T, A = 8, 72
    B = [f"v_mov_b32 v{T + i}, {i * 3 + 1}" for i in range(64)] + [f"v_mov_b32 v{A + i}, 0" for i in range(64)]
    B += [f"v_mov_b32 v{136 + i}, {i}" for i in range(16)]
    B += [f"s_mov_b32 s{40 + i}, 0x{random.getrandbits(32) & 0x0f0f0f0f:08x}" for i in range(16)]
    B += ["s_mov_b32 s74, %[nsteps]", "s_memtime %[t0]", "s_waitcnt lgkmcnt(0)", "L_loop%=:"]
    for qq in range(4):
        for d, slot in enumerate((1, 2, 4, 8)):
            B.append(f"v_mov_b32 v{T + 16 * qq + slot}, v{136 + 4 * qq + d}")
    for row in [(3, 1, 2), (5, 4, 1), (6, 4, 2), (7, 4, 3)] + [(8 + k, 8, k) for k in range(1, 8)]:
        for qq in range(4):
            b = T + 16 * qq
            B.append(f"v_xor_b32 v{b + row[0]}, v{b + row[1]}, v{b + row[2]}")
    first = True
    for c in range(4):
        for pair in range(2):
            lo = 40 + 4 * c + 2 * pair
            for byte in range(4):
                if byte:
                    B.append(f"s_lshr_b64 s[72:73], s[{lo}:{lo + 1}], {8 * byte}")
                for h in range(2):
                    tp = 8 * pair + 4 * h + byte
                    sreg = f"s{lo + h}" if byte == 0 else f"s{72 + h}"
                    B.append(f"s_set_gpr_idx_on {sreg}, gpr_idx(SRC0)" if first else f"s_set_gpr_idx_idx {sreg}")
                    first = False
                    for qq in range(4):
                        acc = A + 16 * c + (tp + 4 * qq) % 16
                        B.append(f"v_xor_b32 v{acc}, v{T + 16 * qq}, v{acc}")
        # (the real step switches mode off only at its end)
    B += ["s_set_gpr_idx_off", "s_sub_u32 s74, s74, 1", "s_cmp_lg_u32 s74, 0", "s_cbranch_scc1 L_loop%=",
          "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)"]
    return wrap("k_idx", B, nvgpr=152, lb=768)


def records(C):
    nb = 4 * C
    vals, rec = 0, []
    for _ in range(NSTEPS):
        for p in range(nb):
            v = random.randrange(0, 16)
            vals += len(block_ops(p // 4, p % 4, v)) + 16 / nb
            rec.append((p * 16 + v) * STRIDE)
    return rec, vals / NSTEPS


rec4, valu4 = records(4)
rec2, valu2 = records(2)
valu_inl = sum(len(block_ops(p // 4, p % 4, inl_pat[s][p])) + 1 for s in range(INL_STEPS) for p in range(16)) / INL_STEPS
valu_idx = 16 + 44 + 256

arr = lambda xs: ", ".join(str(x) for x in xs)
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <algorithm>',
       thread_kernel(4), thread_kernel(2), inline_kernel(), idx_kernel(),
       f"static const unsigned rec4[] = {{{arr(rec4)}}};",
       f"static const unsigned rec2[] = {{{arr(rec2)}}};",
       r'''typedef void (*kfn)(unsigned long long*, const unsigned*, int);
int main() {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nsteps = ''' + str(NSTEPS) + r''';
    unsigned long long* d; hipMalloc(&d, sizeof(unsigned long long) * cus * 32);
    unsigned *r4, *r2;
    hipMalloc(&r4, sizeof(rec4) + 256); hipMalloc(&r2, sizeof(rec2) + 256);
    hipMemcpy(r4, rec4, sizeof(rec4), hipMemcpyHostToDevice);
    hipMemcpy(r2, rec2, sizeof(rec2), hipMemcpyHostToDevice);
    std::vector<unsigned long long> h(cus * 32);
    kfn fns[4] = {k_idx, k_inline, k_thread4, k_thread2};
    const unsigned* recs[4] = {r4, r4, r4, r2};
    const char* names[4] = {"idx (today, 4 cosets)", "inline (4 cosets)", "thread (4 cosets)", "thread (2 cosets)"};
    const double nv[4] = {''' + f"{valu_idx}, {valu_inl:.3f}, {valu4:.3f}, {valu2:.3f}" + r'''};
    const int cos[4] = {4, 4, 4, 2};
    const int wmax[4] = {3, 4, 4, 4};
    for (int k = 0; k < 4; ++k)
        for (int w = 1; w <= wmax[k]; ++w) {
            hipLaunchKernelGGL(fns[k], dim3(cus), dim3(256 * w), 0, 0, d, recs[k], nsteps);  // warm
            hipLaunchKernelGGL(fns[k], dim3(cus), dim3(256 * w), 0, 0, d, recs[k], nsteps);
            if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s\"}\n", names[k]); return 1; }
            hipMemcpy(h.data(), d, sizeof(unsigned long long) * cus * 4 * w, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.begin() + cus * 4 * w);
            const double med = double(h[cus * 2 * w]);
            const double per_step = med / nsteps;  // one wave's step, wall-clock
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"valu_per_step\": %.1f, \"cyc_per_step_wave\": %.1f, "
                   "\"simd_cyc_per_4coset_step\": %.1f, \"simd_cyc_per_valu\": %.3f}\n",
                   names[k], w, nv[k], per_step, per_step / w * 4.0 / cos[k], per_step / w / nv[k]);
            fflush(stdout);
        }
    return 0;
}''']
open(sys.argv[1] if len(sys.argv) > 1 else "thread_bench.hip", "w").write("\n".join(out) + "\n")
