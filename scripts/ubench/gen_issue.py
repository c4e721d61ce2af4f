#!/usr/bin/env python3
"""Generates issue_bench.hip: VALU/SALU issue-rate microbenchmark for candidate instructions of the
m8 asm kernel. Each kernel is ONE asm statement (SGPR setup, counted loop of 64-instruction bodies)
timed with s_memtime; block = 256 * W threads (W waves on each of the CU's 4 SIMDs), one block per
CU. Prints cycles per instruction per wave and VALU cycles per SIMD."""
import sys

def body(kind):
    L = []
    for i in range(64):
        d, a, b, c = 8 + i % 32, 40 + (i * 7) % 32, 40 + (i * 13 + 5) % 32, 40 + (i * 5 + 3) % 32
        simple = {
            "xor": f"v_xor_b32 v{d}, v{a}, v{b}",
            "xor_sgpr": f"v_xor_b32 v{d}, s20, v{b}",
            "xor_e64": f"v_xor_b32_e64 v{d}, v{a}, v{b}",
            "and_lit": f"v_and_b32 v{d}, 0x1010101, v{a}",
            "and_sgpr": f"v_and_b32 v{d}, s21, v{a}",
            "lshl_imm": f"v_lshlrev_b32 v{d}, 1, v{a}",
            "lshr_imm": f"v_lshrrev_b32 v{d}, 7, v{a}",
            "lshl_v": f"v_lshlrev_b32 v{d}, v{b}, v{a}",
            "add_u32": f"v_add_u32 v{d}, v{a}, v{b}",
            "pk_lshl16": f"v_pk_lshlrev_b16 v{d}, 1, v{a} op_sel_hi:[0,1]",
            "lshl_add": f"v_lshl_add_u32 v{d}, v{a}, 1, v{b}",
            "lshl_or": f"v_lshl_or_b32 v{d}, v{a}, 1, v{b}",
            "and_or": f"v_and_or_b32 v{d}, v{a}, v{b}, v{c}",
            "or3": f"v_or3_b32 v{d}, v{a}, v{b}, v{c}",
            "bfi": f"v_bfi_b32 v{d}, v{a}, v{b}, v{c}",
            "bfe": f"v_bfe_u32 v{d}, v{a}, 7, 1",
            "perm_v": f"v_perm_b32 v{d}, v{a}, v{b}, v{c}",
            "perm_s": f"v_perm_b32 v{d}, s20, v{b}, v{c}",
            "alignbit": f"v_alignbit_b32 v{d}, v{a}, v{b}, 7",
            "pk_mul": f"v_pk_mul_lo_u16 v{d}, v{a}, 29 op_sel_hi:[1,0]",
            "pk_mul_v": f"v_pk_mul_lo_u16 v{d}, v{a}, v{b}",
            "mul_u24": f"v_mul_u32_u24 v{d}, v{a}, v{b}",
            "bitop3_s": f"v_bitop3_b32 v{d}, v{a}, v{b}, s20 bitop3:0x6c",
            "bitop3_v": f"v_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x6c",
            "cndmask": f"v_cndmask_b32 v{d}, v{a}, v{b}, vcc",
            "mov": f"v_mov_b32 v{d}, v{a}",
            "xor_sdwa": f"v_xor_b32_sdwa v{d}, v{a}, v{b} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD",
            "idx_noswitch": f"v_xor_b32 v{d}, v40, v{d}",
            # accumulate patterns of the XOR kernel's rows: destination also a source
            "b3_rmw0": f"v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0x96",
            "b3_rmw2": f"v_bitop3_b32 v{d}, v{a}, v{b}, v{d} bitop3:0x96",
            "b3_new": f"v_bitop3_b32 v{d}, v{c}, v{a}, v{b} bitop3:0x96",
            "xor_rmw": f"v_xor_b32 v{d}, v{a}, v{d}",
            "xor_c0": f"v_xor_b32 v{d}, v40, v{b}",
        }
        if kind.startswith("dep"):  # d interleaved self-dependent chains
            dd = int(kind[3:-1])
            r_ = 8 + i % dd
            L.append(f"v_xor_b32 v{r_}, v{40 + i % 8}, v{r_}" if kind.endswith("x") else
                     f"v_add_u32 v{r_}, v{r_}, v{r_}")
            continue
        if kind in simple:
            L.append(simple[kind])
        elif kind in ("idx_sw2", "nop_sw2", "sadd_2", "idx_sw4"):
            per = 4 if kind == "idx_sw4" else 2
            if i % per == 0:
                s = 24 + (i // per) % 8
                L.append({"idx_sw2": f"s_set_gpr_idx_idx s{s}", "idx_sw4": f"s_set_gpr_idx_idx s{s}", "nop_sw2": "s_nop 0",
                          "sadd_2": f"s_add_u32 s{36 + (i // 2) % 4}, s{36 + (i // 2) % 4}, 1"}[kind])
            L.append(f"v_xor_b32 v{d}, v40, v{d}")
        else:
            raise ValueError(kind)
    return L

OCC = "--occ" in sys.argv  # occupancy sweep: 1..8 waves per SIMD (two workgroups per CU above 4)
KINDS = ["idx_noswitch", "idx_sw4", "xor", "bitop3_v", "b3_rmw0"] if OCC else \
    ["b3_rmw0", "b3_rmw2", "b3_new", "xor_rmw", "xor_c0", "idx_noswitch", "xor", "bitop3_v"] if "--rmw" in sys.argv else ["dep1x", "dep2x", "dep3x", "dep4x", "dep6x", "dep8x", "dep1a", "dep2a", "dep4a", "xor", "xor_sgpr", "xor_e64", "and_lit", "and_sgpr", "lshl_imm", "lshr_imm", "lshl_v", "add_u32", "pk_lshl16",
         "lshl_add", "lshl_or", "and_or", "or3", "bfi", "bfe", "perm_v", "perm_s", "alignbit", "pk_mul", "pk_mul_v",
         "mul_u24", "bitop3_s", "bitop3_v", "cndmask", "mov", "xor_sdwa", "idx_noswitch", "idx_sw2",
         "idx_sw4", "nop_sw2", "sadd_2"]
VCLOB = ", ".join(f'"v{r}"' for r in range(8, 72))
SCLOB = ", ".join(f'"s{r}"' for r in list(range(20, 32)) + list(range(36, 40)))
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', '#include <vector>', '#include <algorithm>',
       'static const char* kinds[] = {' + ", ".join(f'"{k}"' for k in KINDS) + '};']
for n, k in enumerate(KINDS):
    b = body(k)
    nv = sum(1 for x in b if x.startswith("v_"))
    idx = k.startswith("idx")
    setup = ["s_mov_b32 s20, 0xfefefefe", "s_mov_b32 s21, 0x01010101", "s_mov_b32 vcc_lo, 0x55555555",
             "s_mov_b32 vcc_hi, 0x55555555"] + [f"s_mov_b32 s{24 + j}, {(j + 1) % 8}" for j in range(8)] + \
            [f"s_mov_b32 s{36 + j}, 0" for j in range(4)]
    pre = ["s_set_gpr_idx_on s24, gpr_idx(SRC0)"] if idx else []
    post = ["s_set_gpr_idx_off"] if idx else []
    lines = setup + ["s_memtime %[t0]", "s_mov_b32 s22, %[iters]", "s_waitcnt lgkmcnt(0)", "BB%=:"] + pre + b + post + \
            ["s_sub_u32 s22, s22, 1", "s_cmp_lg_u32 s22, 0", "s_cbranch_scc1 BB%=", "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)"]
    text = "".join(f'"{x}\\n\\t"' for x in lines)
    out.append(f'''__global__ void __launch_bounds__(1024) k{n}(unsigned long long* out, int iters) {{
    unsigned long long t0, t1;
    asm volatile({text} : [t0] "=&s"(t0), [t1] "=&s"(t1) : [iters] "s"(iters) : {VCLOB}, {SCLOB}, "vcc", "scc");
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}}
static const int nvalu{n} = {nv}, ninst{n} = {len(pre) + len(b) + len(post) + 3};''')
out.append(f'#define WMAX {6 if OCC else 3}')
out.append('typedef void (*kfn)(unsigned long long*, int);')
out.append('static kfn fns[] = {' + ", ".join(f"k{n}" for n in range(len(KINDS))) + '};')
out.append('static const int nvalu[] = {' + ", ".join(f"nvalu{n}" for n in range(len(KINDS))) + '};')
out.append('static const int ninst[] = {' + ", ".join(f"ninst{n}" for n in range(len(KINDS))) + '};')
out.append(r'''int main() {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 500;
    unsigned long long* d; hipMalloc(&d, sizeof(unsigned long long) * cus * 32);
    std::vector<unsigned long long> h(cus * 32);
    for (int k = 0; k < (int)(sizeof(fns) / sizeof(fns[0])); ++k)
        for (int w = 1; w <= WMAX; ++w) {
            if (w > 4 && (w & 1)) continue;  // above 4: two equal workgroups per CU
            const int nb = w > 4 ? 2 : 1, bs = 256 * w / nb;
            hipMemset(d, 0, sizeof(unsigned long long) * cus * 32); hipLaunchKernelGGL(fns[k], dim3(cus * nb), dim3(bs), 0, 0, d, iters);  // warm
            hipLaunchKernelGGL(fns[k], dim3(cus * nb), dim3(bs), 0, 0, d, iters);
            if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s\"}\n", kinds[k]); return 1; }
            hipMemcpy(h.data(), d, sizeof(unsigned long long) * cus * 4 * w, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.begin() + cus * 4 * w);
            const double med = double(h[cus * 2 * w]);
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_inst_wave\": %.2f, \"cyc_per_valu_simd\": %.2f}\n",
                   kinds[k], w, med / (double(iters) * ninst[k]), med / (double(iters) * nvalu[k] * w));
            fflush(stdout);
        }
    return 0;
}''')
open(sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "issue_bench.hip", "w").write("\n".join(out) + "\n")
