#!/usr/bin/env python3
"""Generates thread2_bench.hip: k_cs16 group-step designs with their input loads, at 1..10 waves per SIMD.

Variants (C syndrome cosets per wave; every step loads the next group's 16 inputs from an L2-resident
buffer with raw buffer loads, as the real kernel does):
  idx        today's k_cs16 step: four subset tables (44 XORs) + 256 gpr-indexed XORs (4 cosets),
             load ring (152 VGPRs: 3 waves)
  tC_ring    threaded blocks (gen_asm.py cs16t), inputs through a load ring (moved into F each step)
  tC_direct  threaded blocks, the next group's inputs loaded straight into F after the chain
  tC_r2      as direct, plus R2_j = f_j ^ f_(j-1) (16 XORs a step): every nibble pattern is at most two
             terms (a pair of consecutive bits is one R2), so each accumulator costs exactly one op
One workgroup = one wave per SIMD (256 threads); grid = CUs x W workgroups (W waves per SIMD where the
VGPRs allow). Timed with s_memtime per wave over NSTEPS steps with random records.
(at most 8 waves per SIMD.) Prints SIMD cycles per 4-coset step (lower is better)."""
import random
import sys

random.seed(13)
STRIDE = 512
NSTEPS = 2048


def regs(C, ring, r2):
    F = 8
    R = F + 16
    A = R + (16 if r2 else 0)
    LD = A + 16 * C
    top = LD + (16 if ring else 0)
    return F, R, A, LD, top


def block_ops(C, c, n, v, r2):
    F, R, A, _, _ = regs(C, False, r2)
    ops = []
    for t in range(16):
        terms, d = [], 0
        while d < 4:
            if v >> d & 1:
                a = (t - 4 * n - d) % 16
                if r2 and d < 3 and v >> (d + 1) & 1:
                    terms.append(R + a)  # f_a ^ f_(a-1)
                    d += 2
                    continue
                terms.append(F + a)
            d += 1
        acc = A + 16 * c + t
        while terms:
            if len(terms) >= 2:
                ops.append(f"v_bitop3_b32 v{acc}, v{acc}, v{terms[0]}, v{terms[1]} bitop3:0x96")
                terms = terms[2:]
            else:
                ops.append(f"v_xor_b32 v{acc}, v{acc}, v{terms[0]}")
                terms = terms[1:]
    return ops


def q(lines):
    return "".join(f'"{x}\\n\\t"' for x in lines)


def wrap(name, body, top):
    vclob = ", ".join(f'"v{r}"' for r in range(8, top))
    sclob = ", ".join(f'"s{r}"' for r in list(range(40, 96)))
    return f'''__global__ void __launch_bounds__(256) {name}(unsigned long long* out, const unsigned* rec, const unsigned* data, int nsteps) {{
    unsigned long long t0, t1;
    const unsigned lane = (threadIdx.x & 63) * 4;
    const unsigned long long b = (unsigned long long)data;
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 rsrc = {{unsigned(b), unsigned(b >> 32) & 0xFFFFu, 65536u, 0x20000u}};
    unsigned tv0, tv1;
    asm volatile({q(body)} : [t0] "=&s"(t0), [t1] "=&s"(t1), [a0] "=&v"(tv0), [a1] "=&v"(tv1) : [rec] "s"(rec), [nsteps] "s"(nsteps), [lane] "v"(lane), [rsrc] "s"(rsrc) : {vclob}, {sclob}, "scc", "memory");
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}}'''


def loads(base):
    L = []
    for a in range(16):
        t = "%[a0]" if a % 2 == 0 else "%[a1]"
        L += [f"v_add_u32 {t}, s{76 + a}, %[lane]", f"buffer_load_dword v{base + a}, {t}, %[rsrc], 0 offen"]
    return L


def setup(top):
    L = [f"v_mov_b32 v{r}, {r}" for r in range(8, top)]
    L += [f"s_mov_b32 s{76 + a}, {1024 * ((a * 7) % 16)}" for a in range(16)]
    return L


def thread_kernel(C, ring, r2):
    F, R, A, LD, top = regs(C, ring, r2)
    nb = 4 * C
    ld = {4: "s_load_dwordx16", 3: "s_load_dwordx16", 2: "s_load_dwordx8"}[C]
    wd = {4: 16, 3: 16, 2: 8}[C]  # record window dwords
    B = setup(top)
    B += ["s_getpc_b64 s[92:93]", "s_add_u32 s92, s92, L_blocks%=-.", "s_addc_u32 s93, s93, 0",
          "s_mov_b64 s[72:73], %[rec]", f"{ld} s[56:{55 + wd}], s[72:73], 0x0",
          f"s_add_u32 s72, s72, {4 * nb}", "s_addc_u32 s73, s73, 0", "s_mov_b32 s94, %[nsteps]"]
    B += loads(LD if ring else F)
    B += ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_memtime %[t0]", "s_waitcnt lgkmcnt(0)", "L_loop%=:"]
    B += ["s_waitcnt vmcnt(0)"]
    if ring:
        B += [f"v_mov_b32 v{F + i}, v{LD + i}" for i in range(16)]
    if r2:
        B += [f"v_xor_b32 v{R + j}, v{F + j}, v{F + (j - 1) % 16}" for j in range(16)]
    B += ["s_waitcnt lgkmcnt(0)"] + [f"s_mov_b64 s[{40 + 2 * i}:{41 + 2 * i}], s[{56 + 2 * i}:{57 + 2 * i}]" for i in range(nb // 2)]
    if ring:
        B += loads(LD)
    B += [f"{ld} s[56:{55 + wd}], s[72:73], 0x0", f"s_add_u32 s72, s72, {4 * nb}", "s_addc_u32 s73, s73, 0"]
    B += ["s_getpc_b64 s[74:75]", "s_add_u32 s74, s74, L_ret%=-.", "s_addc_u32 s75, s75, 0",
          "s_add_u32 s90, s92, s40", "s_addc_u32 s91, s93, 0", "s_setpc_b64 s[90:91]", "L_ret%=:"]
    if not ring:
        B += loads(F)
    B += ["s_sub_u32 s94, s94, 1", "s_cmp_lg_u32 s94, 0", "s_cbranch_scc1 L_loop%=",
          "s_waitcnt vmcnt(0)", "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)", "s_getpc_b64 s[90:91]",
          "s_add_u32 s90, s90, L_end%=-.", "s_addc_u32 s91, s91, 0", "s_setpc_b64 s[90:91]", ".p2align 9", "L_blocks%=:"]
    for c in range(C):
        for n in range(4):
            p = 4 * c + n
            for v in range(16):
                B.append(".p2align 9")
                B += block_ops(C, c, n, v, r2)
                if p < nb - 1:
                    B += [f"s_add_u32 s90, s92, s{41 + p}", "s_addc_u32 s91, s93, 0", "s_setpc_b64 s[90:91]"]
                else:
                    B.append("s_setpc_b64 s[74:75]")
    B.append("L_end%=:")
    name = f"k_t{C}_{'ring' if ring else ('r2' if r2 else 'direct')}"
    return name, wrap(name, B, top), top


def idx_kernel():
    T, A, LD = 8, 72, 136
    B = setup(152)
    B += [f"s_mov_b32 s{40 + i}, 0x{random.getrandbits(32) & 0x0f0f0f0f:08x}" for i in range(16)]
    B += ["s_mov_b32 s94, %[nsteps]"] + loads(LD) + ["s_waitcnt vmcnt(0)", "s_memtime %[t0]", "s_waitcnt lgkmcnt(0)", "L_loop%=:"]
    B += ["s_waitcnt vmcnt(0)"]
    for qq in range(4):
        for d, slot in enumerate((1, 2, 4, 8)):
            B.append(f"v_mov_b32 v{T + 16 * qq + slot}, v{LD + 4 * qq + d}")
    B += loads(LD)
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
    B += ["s_set_gpr_idx_off", "s_sub_u32 s94, s94, 1", "s_cmp_lg_u32 s94, 0", "s_cbranch_scc1 L_loop%=",
          "s_waitcnt vmcnt(0)", "s_memtime %[t1]", "s_waitcnt lgkmcnt(0)"]
    return "k_idx", wrap("k_idx", B, 152), 152


def records(C, r2):
    nb, vals, rec = 4 * C, 0, []
    for _ in range(NSTEPS + 4):
        for p in range(nb):
            v = random.randrange(0, 16)
            vals += len(block_ops(C, p // 4, p % 4, v, r2))
            rec.append((p * 16 + v) * STRIDE)
    return rec, vals / (NSTEPS + 4)


kernels = [idx_kernel()]
recs, meta = [], []
for C, ring, r2 in [(4, False, False), (3, False, False), (3, False, True), (2, False, False)]:
    kernels.append(thread_kernel(C, ring, r2))
    rc, blk = records(C, r2)
    recs.append(rc)
    meta.append((C, 32 + (16 if r2 else 0) + blk + (16 if ring else 0)))
arr = lambda xs: ", ".join(str(x) for x in xs)
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <algorithm>']
out += [k[1] for k in kernels]
out += [f"static const unsigned rec{i}[] = {{{arr(r)}}};" for i, r in enumerate(recs)]
ents = []
ents.append(f'{{k_idx, nullptr, 0, "idx (today)", 4, {16 + 44 + 256 + 32}, {512 // 152}}}')
for i, (name, _, top) in enumerate(kernels[1:]):
    C, valu = meta[i]
    alloc = (top + 3 + 7) // 8 * 8
    ents.append(f'{{{name}, rec{i}, sizeof(rec{i}), "{name}", {C}, {valu:.1f}, {min(8, 512 // alloc)}}}')
out.append(r'''typedef void (*kfn)(unsigned long long*, const unsigned*, const unsigned*, int);
struct Ent { kfn f; const unsigned* rec; size_t bytes; const char* name; int cosets; double valu; int wmax; };
int main() {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nsteps = ''' + str(NSTEPS) + r''';
    Ent ents[] = {''' + ", ".join(ents) + r'''};
    unsigned long long* d; hipMalloc(&d, sizeof(unsigned long long) * cus * 64);
    unsigned* data; hipMalloc(&data, 65536); hipMemset(data, 0x5a, 65536);
    std::vector<unsigned long long> h(cus * 64);
    for (auto& e : ents) {
        unsigned* r = nullptr;
        if (e.rec) { hipMalloc(&r, e.bytes); hipMemcpy(r, e.rec, e.bytes, hipMemcpyHostToDevice); }
        for (int w = 1; w <= e.wmax; ++w) {
            hipLaunchKernelGGL(e.f, dim3(cus * w), dim3(256), 0, 0, d, r, data, nsteps / 4);  // warm
            hipLaunchKernelGGL(e.f, dim3(cus * w), dim3(256), 0, 0, d, r, data, nsteps);
            if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s\"}\n", e.name); return 1; }
            hipMemcpy(h.data(), d, sizeof(unsigned long long) * cus * 4 * w, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.begin() + cus * 4 * w);
            const double med = double(h[cus * 2 * w]);
            const double per_step = med / nsteps;
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"valu_per_step\": %.1f, \"cyc_per_step_wave\": %.1f, "
                   "\"simd_cyc_per_4coset_step\": %.1f, \"simd_cyc_per_valu\": %.3f}\n",
                   e.name, w, e.valu, per_step, per_step / w * 4.0 / e.cosets, per_step / w / e.valu);
            fflush(stdout);
        }
        if (r) hipFree(r);
    }
    return 0;
}''')
open(sys.argv[1] if len(sys.argv) > 1 else "thread2_bench.hip", "w").write("\n".join(out) + "\n")
