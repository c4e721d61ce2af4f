#!/usr/bin/env python3
"""Generates bank_bench.hip: does a VALU op whose VGPR operands share a register bank (index mod 4)
issue slower on gfx950? Each kernel is ONE asm statement (counted loop of 64-instruction bodies,
timed with s_memtime), block = 256 * W threads, one block per CU, W = 1..3 waves per SIMD; prints
cycles per VALU per SIMD as gen_issue.py does. The XOR network of rs_xj issues
`v_bitop3 acc, acc, tabA, tabB`; this decides whether register assignment by bank pays."""
import sys


def regs(i, banks):
    """64 distinct-per-slot registers: operand k of instruction i in bank banks[k] (v8..v71)."""
    out = []
    for k, b in enumerate(banks):
        base = 8 + 16 * k  # operand k draws from v[8+16k .. 8+16k+15]
        off = (i // 4 + k) % 4  # with the bank rotation: 16 distinct registers per operand over 16 ops
        r = base + 4 * off + ((b - base) % 4)
        out.append(r)
    return out


def body(kind):
    L = []
    for i in range(64):
        # operand banks per kind: (d, a, b); rotate the whole pattern with i so every bank is used
        rot = i % 4
        pat = {
            "b3rmw_nc": (0, 1, 2), "b3rmw_ab": (0, 1, 1), "b3rmw_da": (0, 0, 1), "b3rmw_all": (0, 0, 0),
            "b3new_nc": (0, 1, 2, 3), "b3new_abc": (0, 1, 1, 1), "b3new_bc": (0, 1, 2, 2),
            "xorrmw_nc": (0, 1), "xorrmw_c": (0, 0), "xornew_nc": (0, 1, 2), "xornew_c": (0, 1, 1),
            "mul_lit": (0, 1), "and_lit": (0, 1), "lshr_imm": (0, 1), "add_vv": (0, 1, 2),
            "sub_vv": (0, 1, 2), "add_lit": (0, 1),
        }[kind]
        bk = [(p + rot) % 4 for p in pat]
        r = regs(i, bk)
        if kind.startswith("b3rmw"):
            L.append(f"v_bitop3_b32 v{r[0]}, v{r[0]}, v{r[1]}, v{r[2]} bitop3:0x96")
        elif kind.startswith("b3new"):
            L.append(f"v_bitop3_b32 v{r[0]}, v{r[1]}, v{r[2]}, v{r[3]} bitop3:0x96")
        elif kind.startswith("xorrmw"):
            L.append(f"v_xor_b32 v{r[0]}, v{r[1]}, v{r[0]}")
        elif kind.startswith("xornew"):
            L.append(f"v_xor_b32 v{r[0]}, v{r[1]}, v{r[2]}")
        elif kind == "mul_lit":
            L.append(f"v_mul_u32_u24 v{r[0]}, 0x8016, v{r[1]}")
        elif kind == "and_lit":
            L.append(f"v_and_b32 v{r[0]}, 0x10001, v{r[1]}")
        elif kind == "lshr_imm":
            L.append(f"v_lshrrev_b32 v{r[0]}, 1, v{r[1]}")
        elif kind == "add_vv":
            L.append(f"v_add_u32 v{r[0]}, v{r[1]}, v{r[2]}")
        elif kind == "sub_vv":
            L.append(f"v_sub_u32 v{r[0]}, v{r[1]}, v{r[2]}")
        elif kind == "add_lit":
            L.append(f"v_add_u32 v{r[0]}, 0x7fff7fff, v{r[1]}")
    return L


KINDS = ["b3rmw_nc", "b3rmw_ab", "b3rmw_da", "b3rmw_all", "b3new_nc", "b3new_abc", "b3new_bc", "xorrmw_nc",
         "xorrmw_c", "xornew_nc", "xornew_c", "mul_lit", "and_lit", "lshr_imm", "add_vv", "sub_vv", "add_lit"]
VCLOB = ", ".join(f'"v{r}"' for r in range(8, 72))
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <algorithm>',
       'static const char* kinds[] = {' + ", ".join(f'"{k}"' for k in KINDS) + '};']
for n, k in enumerate(KINDS):
    b = body(k)
    lines = ["s_memtime %[t0]", "s_mov_b32 s22, %[iters]", "s_waitcnt lgkmcnt(0)", "BB%=:"] + b + \
            ["s_sub_u32 s22, s22, 1", "s_cmp_lg_u32 s22, 0", "s_cbranch_scc1 BB%=", "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)"]
    text = "".join(f'"{x}\\n\\t"' for x in lines)
    out.append(f'''__global__ void __launch_bounds__(1024) k{n}(unsigned long long* out, int iters) {{
    unsigned long long t0, t1;
    asm volatile({text} : [t0] "=&s"(t0), [t1] "=&s"(t1) : [iters] "s"(iters) : {VCLOB}, "s22", "scc");
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}}''')
out.append('typedef void (*kfn)(unsigned long long*, int);')
out.append('static kfn fns[] = {' + ", ".join(f"k{n}" for n in range(len(KINDS))) + '};')
out.append(r'''int main() {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 500;
    unsigned long long* d; hipMalloc(&d, sizeof(unsigned long long) * cus * 16);
    std::vector<unsigned long long> h(cus * 16);
    for (int k = 0; k < (int)(sizeof(fns) / sizeof(fns[0])); ++k)
        for (int w = 1; w <= 3; ++w) {
            hipLaunchKernelGGL(fns[k], dim3(cus), dim3(256 * w), 0, 0, d, iters);  // warm
            hipLaunchKernelGGL(fns[k], dim3(cus), dim3(256 * w), 0, 0, d, iters);
            if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s\"}\n", kinds[k]); return 1; }
            hipMemcpy(h.data(), d, sizeof(unsigned long long) * cus * 4 * w, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.begin() + cus * 4 * w);
            const double med = double(h[cus * 2 * w]);
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_valu_simd\": %.2f}\n", kinds[k], w,
                   med / (double(iters) * 64 * w));
            fflush(stdout);
        }
    return 0;
}''')
open(sys.argv[1] if len(sys.argv) > 1 else "bank_bench.hip", "w").write("\n".join(out) + "\n")
