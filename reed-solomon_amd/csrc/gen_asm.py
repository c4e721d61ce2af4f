#!/usr/bin/env python3
"""Emits csrc/gen/m8_idx_asm*.inc: one input step of the m <= 8 asm kernels (everything after the
LDS coordinate lookup), as a single hand-scheduled block.

Register contract (pinned by the asm constraints in rs_kernels.hip):
  Tl0 v[8:23]  Th0 v[24:39]   nibble tables of dword 0 (entry e in register base + e, e = 0..15)
  Tl1 v[40:55] Th1 v[56:71]   nibble tables of dword 1
  acc0 v[72:103]  acc1 v[104:135]   output p of dword 0 / 1 in register base + p
  s[40:71]  32 table indices (the 64-dword record of an input is loaded in two halves)
Inputs %[y0] %[y1]: the input dwords in GF(256)^2 coordinates; %[t0]..%[t3] scratch VGPRs; %[cp]
the index record of this input: dword p = low nibble, dword 32 + p = high nibble of the
coefficient of output p.

Multiples: m_0 = y, m_{j+1} = xtime(m_j) on 4 packed bytes (xtime_ops: six full-rate VALU ops, no
SGPR operand -- measured with scripts/ubench: SGPR operands, left shifts, v_pk_mul, v_perm and
3-input VOP3 ops issue at half rate), written straight into the table slots T[1], T[2], T[4], T[8];
the other 11 entries of each table are XORs. Lookups: s_set_gpr_idx_idx <nibble> retargets src0 of the
following v_xor to table register base + nibble.

Variants (all but "full", "split" and "split_mul" give wrong results; they are timing ablations):
  split      (production) all lo lookups, then all hi lookups; no accumulator is touched twice
             within a pass, and the high tables are built while the high-nibble indices load
  split_mul  split with the older multiply-based xtime
  full       per output: lo lookup (2 dwords), hi lookup (2 dwords); multiply-based xtime
  noidx      full with the index switches replaced by s_nop
  build      multiples + tables only       look  lookups only (tables not rebuilt)
  nop        consume the inputs only (memory-structure timing)
  plain      split without gpr-index mode (fixed table registers)
  v1         one dword per lane (k_apply_m8_v1): half the registers, so 5 waves per SIMD
  v1_plain   v1 without gpr-index mode (timing ablation)
  v1_jitcall input step of the matrix-specialised V = 1 kernel (multiples, tables, call into the
             input's generated lookup block)
  m16_v1     m = 16 input step (k_apply_m16_v1): 16 multiples x * alpha^j, four nibble tables, 256
             gpr-indexed lookups for 64 outputs (m16_v1_plain: fixed registers, timing only)
"""
import os
import sys

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "gen", "m8_idx_asm.inc")
variant = sys.argv[2] if len(sys.argv) > 2 else "split"
XT = "mul" if variant in ("full", "noidx", "split_mul") else "fast"  # xtime style
L = []
e = L.append

TL = {0: 8, 1: 40}   # low-nibble table base per dword
TH = {0: 24, 1: 56}  # high-nibble table base per dword
ACC = {0: 72, 1: 104}
slots = [1, 2, 4, 8]
tmp = {0: ("%[t0]", "%[t1]"), 1: ("%[t2]", "%[t3]")}


def mult_reg(v, j):
    return (TL[v] if j < 4 else TH[v]) + slots[j % 4]


def xtime_ops(j, style):
    """Multiple j of both dwords from multiple j - 1, interleaved op by op.
    style "fast" (all full-rate VALU): u = x & 0x80808080, v = u >> 7, w = u - v (0x7F in every byte
    whose top bit is set), s = x ^ u, x*gamma = (s + s) ^ (w & 0x1D1D1D1D)  [no carry crosses a byte:
    s has every top bit clear, u - v never borrows].
    style "mul": ((x << 1) & 0xFEFEFEFE) ^ ((x >> 7) & 0x01010101) * 0x1D (3 half-rate ops)."""
    ops = []
    if style == "fast":
        seq = ["v_and_b32 {ta}, 0x80808080, v{src}", "v_lshrrev_b32 {tb}, 7, {ta}", "v_xor_b32 v{dst}, v{src}, {ta}",
               "v_sub_u32 {tb}, {ta}, {tb}", "v_add_u32 v{dst}, v{dst}, v{dst}",
               "v_bitop3_b32 v{dst}, v{dst}, {tb}, %[k1d] bitop3:0x78"]
    else:
        seq = ["v_lshrrev_b32 {ta}, 7, v{src}", "v_lshlrev_b32 {tb}, 1, v{src}", "v_and_b32 {ta}, 0x1010101, {ta}",
               "v_pk_mul_lo_u16 {ta}, {ta}, 29 op_sel_hi:[1,0]", "v_bitop3_b32 v{dst}, {tb}, {ta}, %[kfe] bitop3:0x6c"]
    for op in seq:
        for v in (0, 1):
            ta, tb = tmp[v]
            ops.append(op.format(ta=ta, tb=tb, src=mult_reg(v, j - 1), dst=mult_reg(v, j)))
    return ops


def table_ops(bases):
    """T[0] = 0, T[3] = T1^T2, T[5] = T4^T1, T[6] = T4^T2, T[7] = T4^T3, T[8+k] = T8^T[k]; the
    tables in `bases` interleaved entry by entry."""
    ops = []
    rows = [lambda b: f"v_mov_b32 v{b}, 0", lambda b: f"v_xor_b32 v{b + 3}, v{b + 1}, v{b + 2}",
            lambda b: f"v_xor_b32 v{b + 5}, v{b + 4}, v{b + 1}", lambda b: f"v_xor_b32 v{b + 6}, v{b + 4}, v{b + 2}",
            lambda b: f"v_xor_b32 v{b + 7}, v{b + 4}, v{b + 3}"]
    rows += [(lambda k: lambda b: f"v_xor_b32 v{b + 8 + k}, v{b + 8}, v{b + k}")(k) for k in range(1, 8)]
    for row in rows:
        for b in bases:
            ops.append(row(b))
    return ops


def mix(a, b):
    """Interleave op lists: spread b evenly between the ops of a."""
    if not b:
        return list(a)
    res, k = [], 0
    for i, op in enumerate(a):
        res.append(op)
        want = (i + 1) * len(b) // len(a)
        while k < want:
            res.append(b[k])
            k += 1
    return res + b[k:]


def emit(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write("// generated by csrc/gen_asm.py -- do not edit\n")
        f.write("".join(f'"{ln}\\n\\t"\n' for ln in L))


if variant == "v1_jitcall":
    # one input step of the matrix-specialised V = 1 kernel (rs_jit.cpp, rs_v1jit): multiples and both
    # nibble tables, then s_swappc_b64 into this input's lookup block (fixed-register XORs,
    # generated per coding matrix) at L_rs_blk0 + %[off]; the block returns with s_setpc_b64 s[72:73].
    # L_rs_blk0 precedes every call site (the blocks are placed at the kernel entry), so the
    # 64-bit sign extension of the negative offset is -1.
    tl, th = 8, 24
    tv = ("%[t0]", "%[t1]")
    mreg = lambda j: (tl if j < 4 else th) + slots[j % 4]
    e("s_getpc_b64 s[74:75]")
    e("s_add_u32 s74, s74, L_rs_blk0-.")  # s_getpc returned the address of this instruction
    e("s_addc_u32 s75, s75, -1")
    e("s_add_u32 s74, s74, %[off]")
    e("s_addc_u32 s75, s75, 0")
    e(f"v_mov_b32 v{mreg(0)}, %[y0]")
    for j in range(1, 8):
        src, dst = mreg(j - 1), mreg(j)
        for op in ["v_and_b32 {ta}, 0x80808080, v{src}", "v_lshrrev_b32 {tb}, 7, {ta}",
                   "v_xor_b32 v{dst}, v{src}, {ta}", "v_sub_u32 {tb}, {ta}, {tb}", "v_add_u32 v{dst}, v{dst}, v{dst}",
                   "v_bitop3_b32 v{dst}, v{dst}, {tb}, %[k1d] bitop3:0x78"]:
            e(op.format(ta=tv[0], tb=tv[1], src=src, dst=dst))
        if j == 3:
            L.extend(table_ops((tl,)))
    L.extend(table_ops((th,)))
    e("s_swappc_b64 s[72:73], s[74:75]")
    emit(out)
    sys.exit(0)

if variant in ("m16_v1", "m16_v1_plain"):
    # m = 16, one dword (two GF(2^16) words) per lane per step (k_apply_m16_v1), 64 outputs per tile:
    #   T_n v[8 + 16n : 23 + 16n]  nibble table n: entry e = XOR of x * alpha^(4n + b) over the set bits b
    #   acc v[72:135]               output p in v[72 + p]
    #   s[40:55] / s[56:71]         two 16-dword buffers, one nibble plane of the record each;
    #   s[72:73] scratch pair, s74 = 0xFFFEFFFE
    # Record of (tile, input): 64 dwords, 16 per plane; lookup l of plane n (output l) takes its index
    # 16n + nibble n from byte (l % 8) // 2 of plane dword 2 (l // 8) + l % 2, so every lookup indexes
    # from v8; s_set_gpr_idx_idx takes bits [7:0] of its operand, and one s_lshr_b64 of a dword pair
    # brings the next byte of both dwords down (3 shifts per 8 lookups). Plane n + 1 (or the next input's plane 0: the record array is padded by one
    # input) loads while plane n is consumed; this input's plane 0 was requested by the previous step
    # (or by the kernel before the first one) and arrives in s[40:55].
    # Plane n reads only table T_n, so T_(n+1) is built while plane n's lookups run. In gpr-index mode
    # only VGPR src0 operands are offset, so every building op keeps src0 a constant or an SGPR:
    #   x * alpha on packed words: ((x << 1) & 0xFFFEFFFE) ^ (((x >> 15) & 0x10001) * 0x2D)
    #   table XORs as v_bitop3_b32 with a constant first operand (truth table 0x66 = src1 ^ src2).
    T, ACC = 8, 72
    ta, tb = "%[t0]", "%[t1]"
    mreg = lambda j: T + 16 * (j // 4) + slots[j % 4]

    def xt(j):  # multiple j from multiple j - 1
        src, dst = mreg(j - 1), mreg(j)
        return [f"v_lshrrev_b32 {ta}, 15, v{src}", f"v_and_b32 {ta}, 0x10001, {ta}", f"v_mul_u32_u24 {ta}, 45, {ta}",
                f"v_lshlrev_b32 {tb}, 1, v{src}", f"v_bitop3_b32 v{dst}, s74, {tb}, {ta} bitop3:0x6a"]

    def tab(b):
        ops = [f"v_mov_b32 v{b}, 0"]
        pairs = [(3, 1, 2), (5, 4, 1), (6, 4, 2), (7, 4, 3)] + [(8 + k, 8, k) for k in range(1, 8)]
        ops += [f"v_bitop3_b32 v{b + d}, 0, v{b + x}, v{b + y} bitop3:0x66" for d, x, y in pairs]
        return ops

    def build(n):  # table n from multiple 4n - 1 (or the input for n = 0)
        ops = [f"v_mov_b32 v{mreg(0)}, %[y0]"] if n == 0 else xt(4 * n)
        for j in range(4 * n + 1, 4 * n + 4):
            ops += xt(j)
        return ops + tab(T + 16 * n)

    e("s_mov_b32 s74, 0xfffefffe")
    L.extend(build(0))
    idx = variant == "m16_v1"
    for n in range(4):
        buf, nxt = (40, 56) if n % 2 == 0 else (56, 40)
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_load_dwordx16 s[{nxt}:{nxt + 15}], %[cp], {hex(64 * (n + 1))}")
        look = []
        for l in range(64):
            # lookup l of the plane: dword pair m = l // 8 of the buffer, byte b = (l % 8) // 2 of dword
            # 2m + (l % 2); one s_lshr_b64 of the pair brings byte b of both dwords down to bits [7:0]
            m, r8 = divmod(l, 8)
            b, h = divmod(r8, 2)
            grp = []
            if idx:
                if b == 0:
                    sreg = f"s{buf + 2 * m + h}"
                else:
                    if h == 0:
                        grp.append(f"s_lshr_b64 s[72:73], s[{buf + 2 * m}:{buf + 2 * m + 1}], {8 * b}")
                    sreg = f"s{72 + h}"
                grp.append(f"s_set_gpr_idx_on {sreg}, gpr_idx(SRC0)" if n == 0 and l == 0 else f"s_set_gpr_idx_idx {sreg}")
            src = T if idx else T + 16 * n + (l * 7 + 3) % 16
            grp.append(f"v_xor_b32 v{ACC + l}, v{src}, v{ACC + l}")
            look.append(grp)
        other = build(n + 1) if n < 3 else []
        # spread the next table's ops over the 64 lookups (after each lookup's v_xor)
        k = 0
        for l, grp in enumerate(look):
            L.extend(grp)
            want = (l + 1) * len(other) // 64
            while k < want:
                e(other[k])
                k += 1
        L.extend(other[k:])
    if idx:
        e("s_set_gpr_idx_off")
    emit(out)
    sys.exit(0)

if variant == "cs16_pro":
    # k_cs16 prologue: group 0's inputs in flight into v[136:151], group 1's slot offsets in s[76:91],
    # group 0's record in s[40:55] (operands %[g0] offsets array, %[r0] records, %[rsrc], %[lane])
    e("s_load_dwordx16 s[76:91], %[g0], 0x0")
    e("s_waitcnt lgkmcnt(0)")
    for a in range(16):
        e(f"v_add_u32 %[t0], s{76 + a}, %[lane]")
        e(f"buffer_load_dword v{136 + a}, %[t0], %[rsrc], 0 offen")
    e("s_load_dwordx16 s[76:91], %[g0], 0x40")
    e("s_load_dwordx16 s[40:55], %[r0], 0x0")
    emit(out)
    sys.exit(0)

if variant == "bs16":
    # m = 16 binary accumulation with per-accumulator indices (k_bs16): the GF(2^16) syndrome route's
    # encode second stage. Output coset c (16 accumulators u_t, normal-basis coordinates) accumulates
    #     u_t ^= sum_j bit_t(z_(c, j)) * S_j,   z = normal repr of the coefficient of S_j
    # over the step's 16 inputs (four subset tables T_q over inputs 4q .. 4q + 3 as in cs16); the
    # coefficients have no circulant structure here, so each (coset, table, t) has its own index: 64
    # gpr-index switches per coset. Registers as cs16a (tables, 4 cosets' accumulators, L ring,
    # s[76:91] slot offsets); the record of (tile, group) is 4 cosets x 64 byte indices (byte 16q + t
    # of coset c = index of (q, t)), read one coset at a time into s[40:55] / s[56:71] alternately
    # (coset c in buffer c % 2; the next step's coset 0 is requested while coset 3 runs).
    T, ACC, LD = 8, 72, 136
    e("s_waitcnt vmcnt(0)")
    for q in range(4):
        b = T + 16 * q
        for d, slot in enumerate((1, 2, 4, 8)):
            e(f"v_mov_b32 v{b + slot}, v{LD + 4 * q + d}")
    e("s_waitcnt lgkmcnt(0)")  # coset 0's record and the next group's slot offsets
    for a in range(16):
        t = "%[t0]" if a % 2 == 0 else "%[t1]"
        e(f"v_add_u32 {t}, s{76 + a}, %[lane]")
        e(f"buffer_load_dword v{LD + a}, {t}, %[rsrc], 0 offen")
    e("s_load_dwordx16 s[56:71], %[cp], 0x40")  # coset 1's record
    e("s_load_dwordx16 s[76:91], %[gp], 0x0")
    for row in [(3, 1, 2), (5, 4, 1), (6, 4, 2), (7, 4, 3)] + [(8 + k, 8, k) for k in range(1, 8)]:
        for q in range(4):
            b = T + 16 * q
            e(f"v_xor_b32 v{b + row[0]}, v{b + row[1]}, v{b + row[2]}")
    first = True
    for c in range(4):
        buf = 40 if c % 2 == 0 else 56
        if c:
            if first is False:
                e("s_set_gpr_idx_off")  # s_load / s_waitcnt outside gpr-index mode
                first = True
            e("s_waitcnt lgkmcnt(0)")
            nxt = 56 if c % 2 == 0 else 40
            e(f"s_load_dwordx16 s[{nxt}:{nxt + 15}], %[cp], {hex(64 * (c + 1))}")  # coset c + 1 / next step's 0
        for pair in range(8):  # dwords (2 pair, 2 pair + 1): bytes 8 pair + (0..3, 4..7)
            lo = buf + 2 * pair
            for byte in range(4):
                if byte:
                    e(f"s_lshr_b64 s[72:73], s[{lo}:{lo + 1}], {8 * byte}")
                for h in range(2):
                    bi = 8 * pair + 4 * h + byte
                    q, t = divmod(bi, 16)
                    sreg = f"s{lo + h}" if byte == 0 else f"s{72 + h}"
                    e(f"s_set_gpr_idx_on {sreg}, gpr_idx(SRC0)" if first else f"s_set_gpr_idx_idx {sreg}")
                    first = False
                    acc = ACC + 16 * c + t
                    e(f"v_xor_b32 v{acc}, v{T + 16 * q}, v{acc}")
    e("s_set_gpr_idx_off")
    emit(out)
    sys.exit(0)

if variant in ("cs16a", "cs16b"):
    # m = 16 cyclotomic syndromes (k_cs16), one dword (two GF(2^16) words) per lane per group step.
    # A group is 16 inputs f_a at positions L * 2^a (a cyclotomic coset, empty slots zero); a syndrome
    # coset s owns 16 accumulators u_t (normal-basis coordinates of GF(2^16)):
    #     u_t ^= sum_a f_a * bit_((t - a) mod 16)(z),   z = normal repr of alpha^(s * L)
    # (alpha^(s L 2^a) is z rotated by a: Frobenius permutes the normal basis cyclically). Four 16-entry
    # subset tables T_q over inputs 4q .. 4q + 3 make that 64 lookups per (group, coset): the index
    # for accumulator t from table q depends only on t - 4q, so ONE gpr-index switch e(t') feeds four
    # XORs, into accumulators t' + 4q (q = 0..3). A wave holds 4 cosets (152 VGPRs: 3 waves per SIMD).
    # Register contract:
    #   T_q   v[8 + 16q : 23 + 16q]   entry e = XOR of f_(4q + d) over the set bits d of e (entry 0 stays 0)
    #   acc   v[72 : 135]             coset c (of the wave's 4), accumulator t in v[72 + 16c + t]
    #   L     v[136 : 151]            the next group's inputs, loaded by this step (raw buffer loads at
    #                                 voffset = %[lane] + slot offset; an empty slot's offset 0x80000000 is
    #                                 out of range, so it loads 0)
    #   records                       4 cosets x 16 byte indices (byte t' of coset c = e(t')) per group:
    #                                 this step's in s[40:55] (cs16a) / s[56:71] (cs16b), the next group's
    #                                 loaded into the other buffer; the kernel alternates a, b
    #   s[72:73]                      shift scratch
    #   s[76:91]                      byte offsets of the next group's 16 slots (from the previous step)
    # Operands: %[cp] this record (the next group's at +64), %[gp] the group-offset record of the group
    # after next, %[rsrc] the stripe's V#, %[lane] the lane's byte column, %[t0] %[t1] address scratch.
    T, ACC, LD = 8, 72, 136
    cur, nxt = (40, 56) if variant == "cs16a" else (56, 40)
    e("s_waitcnt vmcnt(0)")  # this group's inputs (loaded by the previous step)
    for q in range(4):
        b = T + 16 * q
        for d, slot in enumerate((1, 2, 4, 8)):
            e(f"v_mov_b32 v{b + slot}, v{LD + 4 * q + d}")
    e("s_waitcnt lgkmcnt(0)")  # this record and the next group's slot offsets
    for a in range(16):  # the next group's inputs
        t = "%[t0]" if a % 2 == 0 else "%[t1]"
        e(f"v_add_u32 {t}, s{76 + a}, %[lane]")
        e(f"buffer_load_dword v{LD + a}, {t}, %[rsrc], 0 offen")
    e(f"s_load_dwordx16 s[{nxt}:{nxt + 15}], %[cp], 0x40")  # the next group's record
    e("s_load_dwordx16 s[76:91], %[gp], 0x0")  # slot offsets of the group after next
    for row in [(3, 1, 2), (5, 4, 1), (6, 4, 2), (7, 4, 3)] + [(8 + k, 8, k) for k in range(1, 8)]:
        for q in range(4):
            b = T + 16 * q
            e(f"v_xor_b32 v{b + row[0]}, v{b + row[1]}, v{b + row[2]}")
    first = True
    for c in range(4):
        for pair in range(2):  # dwords (4c + 2pair, 4c + 2pair + 1): indices t' = 8 pair + (0..3, 4..7)
            lo = cur + 4 * c + 2 * pair
            for byte in range(4):
                if byte:
                    e(f"s_lshr_b64 s[72:73], s[{lo}:{lo + 1}], {8 * byte}")
                for h in range(2):
                    tp = 8 * pair + 4 * h + byte
                    sreg = f"s{lo + h}" if byte == 0 else f"s{72 + h}"
                    e(f"s_set_gpr_idx_on {sreg}, gpr_idx(SRC0)" if first else f"s_set_gpr_idx_idx {sreg}")
                    first = False
                    for q in range(4):
                        acc = ACC + 16 * c + (tp + 4 * q) % 16
                        e(f"v_xor_b32 v{acc}, v{T + 16 * q}, v{acc}")
    e("s_set_gpr_idx_off")
    emit(out)
    sys.exit(0)

if variant in ("v1", "v1_plain"):
    # one dword per lane per step (k_apply_m8_v1): Tl v[8:23], Th v[24:39], acc v[40:71]; temps t0, t1
    tl, th, acc = 8, 24, 40
    tv = ("%[t0]", "%[t1]")
    mreg = lambda j: (tl if j < 4 else th) + slots[j % 4]
    e("s_load_dwordx16 s[40:55], %[cp], 0x0")
    e("s_load_dwordx16 s[56:71], %[cp], 0x40")
    e(f"v_mov_b32 v{mreg(0)}, %[y0]")
    for j in range(1, 8):
        src, dst = mreg(j - 1), mreg(j)
        for op in ["v_and_b32 {ta}, 0x80808080, v{src}", "v_lshrrev_b32 {tb}, 7, {ta}",
                   "v_xor_b32 v{dst}, v{src}, {ta}", "v_sub_u32 {tb}, {ta}, {tb}", "v_add_u32 v{dst}, v{dst}, v{dst}",
                   "v_bitop3_b32 v{dst}, v{dst}, {tb}, %[k1d] bitop3:0x78"]:
            e(op.format(ta=tv[0], tb=tv[1], src=src, dst=dst))
        if j == 3:
            L.extend(table_ops((tl,)))
    e("s_waitcnt lgkmcnt(0)")
    idx = variant == "v1"
    for p in range(32):
        if idx:
            e("s_set_gpr_idx_on s40, gpr_idx(SRC0)" if p == 0 else f"s_set_gpr_idx_idx s{40 + p}")
        e(f"v_xor_b32 v{acc + p}, v{tl + (0 if idx else p % 16)}, v{acc + p}")
    if idx:
        e("s_set_gpr_idx_off")
    e("s_load_dwordx16 s[40:55], %[cp], 0x80")
    e("s_load_dwordx16 s[56:71], %[cp], 0xc0")
    L.extend(table_ops((th,)))
    e("s_waitcnt lgkmcnt(0)")
    for p in range(32):
        if idx:
            e("s_set_gpr_idx_on s40, gpr_idx(SRC0)" if p == 0 else f"s_set_gpr_idx_idx s{40 + p}")
        e(f"v_xor_b32 v{acc + p}, v{th + (0 if idx else (p + 5) % 16)}, v{acc + p}")
    if idx:
        e("s_set_gpr_idx_off")
    emit(out)
    sys.exit(0)

if variant == "nop":
    e("v_xor_b32 v72, %[y0], v72")
    e("v_xor_b32 v104, %[y1], v104")
    emit(out)
    sys.exit(0)

if variant in ("split", "plain", "split_mul"):
    e("s_load_dwordx16 s[40:55], %[cp], 0x0")   # low nibbles of outputs 0..31
    e("s_load_dwordx16 s[56:71], %[cp], 0x40")
    e("v_mov_b32 v%d, %%[y0]" % mult_reg(0, 0))
    e("v_mov_b32 v%d, %%[y1]" % mult_reg(1, 0))
    for j in range(1, 4):
        L.extend(xtime_ops(j, XT))
    chain = []
    for j in range(4, 8):
        chain += xtime_ops(j, XT)
    L.extend(mix(chain, table_ops((TL[0], TL[1]))))
    e("s_waitcnt lgkmcnt(0)")
    idx = variant != "plain"
    for p in range(32):
        if idx:
            e("s_set_gpr_idx_on s40, gpr_idx(SRC0)" if p == 0 else f"s_set_gpr_idx_idx s{40 + p}")
        src = 0 if idx else p % 16
        e(f"v_xor_b32 v{ACC[0] + p}, v{TL[0] + src}, v{ACC[0] + p}")
        e(f"v_xor_b32 v{ACC[1] + p}, v{TL[1] + src}, v{ACC[1] + p}")
    if idx:
        e("s_set_gpr_idx_off")
    e("s_load_dwordx16 s[40:55], %[cp], 0x80")  # high nibbles
    e("s_load_dwordx16 s[56:71], %[cp], 0xc0")
    L.extend(table_ops((TH[0], TH[1])))
    e("s_waitcnt lgkmcnt(0)")
    for p in range(32):
        if idx:
            e("s_set_gpr_idx_on s40, gpr_idx(SRC0)" if p == 0 else f"s_set_gpr_idx_idx s{40 + p}")
        src = 0 if idx else (p + 5) % 16
        e(f"v_xor_b32 v{ACC[0] + p}, v{TH[0] + src}, v{ACC[0] + p}")
        e(f"v_xor_b32 v{ACC[1] + p}, v{TH[1] + src}, v{ACC[1] + p}")
    if idx:
        e("s_set_gpr_idx_off")
    emit(out)
    sys.exit(0)

# full / noidx / build / look: record halves = outputs 0-15 (lo at 0x0, hi at 0x80) and 16-31
e("s_load_dwordx16 s[40:55], %[cp], 0x0")
e("s_load_dwordx16 s[56:71], %[cp], 0x80")
if variant == "look":
    e("s_waitcnt lgkmcnt(0)")
e("v_mov_b32 v%d, %%[y0]" % mult_reg(0, 0))
e("v_mov_b32 v%d, %%[y1]" % mult_reg(1, 0))
if variant != "look":
    for j in range(1, 8):
        L.extend(xtime_ops(j, XT))
    L.extend(table_ops((TL[0], TL[1], TH[0], TH[1])))
    e("s_waitcnt lgkmcnt(0)")
for half in ((0, 1) if variant != "build" else ()):
    if half == 1:  # second half of the record into the same 32 SGPRs
        e("s_load_dwordx16 s[40:55], %[cp], 0x40")
        e("s_load_dwordx16 s[56:71], %[cp], 0xc0")
        e("s_waitcnt lgkmcnt(0)")
    for j in range(16):
        p = 16 * half + j
        lo, hi = 40 + j, 56 + j
        if variant == "noidx":
            e("s_set_gpr_idx_on s40, gpr_idx(SRC0)" if p == 0 else "s_nop 0")
        else:
            e(f"s_set_gpr_idx_on s{lo}, gpr_idx(SRC0)" if p == 0 else f"s_set_gpr_idx_idx s{lo}")
        e(f"v_xor_b32 v{72 + p}, v8, v{72 + p}")
        e(f"v_xor_b32 v{104 + p}, v40, v{104 + p}")
        e("s_nop 0" if variant == "noidx" else f"s_set_gpr_idx_idx s{hi}")
        e(f"v_xor_b32 v{72 + p}, v24, v{72 + p}")
        e(f"v_xor_b32 v{104 + p}, v56, v{104 + p}")
if variant != "build":
    e("s_set_gpr_idx_off")
emit(out)
