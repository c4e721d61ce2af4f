"""CPU emulator for the generated bit-plane XOR kernel (reed-solomon_amd/csrc/rs_xj.cpp).

TEST INFRASTRUCTURE: executes the instruction subset the generator emits (SALU address arithmetic,
global_load/store_dword, v_xor/v_and/v_lshrrev/v_mul_u32_u24/v_bitop3(0x96)/v_mov, the shared finish
block entered by s_swappc) for every role wave of one 256-byte column block, so the generator's
XOR network and finish map can be checked bit-exactly against the oracle without a GPU.
"""
import re

import numpy as np

_STR = re.compile(r'^"(.*)\\n"$')


def split_source(src):
    """-> (finish_lines, [role_lines...]) from the generated hiprtc source."""
    blocks, cur = [], None
    for line in src.splitlines():
        line = line.strip()
        if line.startswith("asm volatile(") or line.endswith("asm volatile("):
            cur = []
            blocks.append(cur)
            continue
        m = _STR.match(line)
        if m and cur is not None:
            cur.append(m.group(1))
    return blocks[0], blocks[1:]


def _vreg(tok):
    assert tok[0] == "v", tok
    return int(tok[1:])


class Wave:
    def __init__(self, mem, operands, lgkm=False):
        self.v = np.zeros((256, 64), np.uint32)
        # lgkm=True: scalar-memory and LDS reads land only when an s_waitcnt lgkmcnt retires them (SMEM returns
        # out of order, so only lgkmcnt(0) retires it; LDS reads retire in order when no SMEM is pending); an
        # instruction that names a register with a read still in flight raises
        self.lgkm = lgkm
        self.lg = []  # [("s", first sgpr, words) | ("v", vgpr, data)]
        self.s = np.zeros(128, np.uint64)
        self.scc = 0
        self.m0 = 0
        self.lds = None  # np.uint8 array shared by the block's waves
        # vector-memory counter model: loads land in their VGPRs only when an s_waitcnt vmcnt(N) retires
        # them (in issue order, stores counted too); touching a VGPR whose load has not been retired is
        # a missing or too-loose wait and raises
        self.vm = []  # [(vgpr or None, data)]
        self.mem = mem
        self.ops = operands  # name -> int or np.ndarray (VGPR operand)

    def val(self, tok):
        tok = tok.strip()
        if tok.startswith("%["):
            return self.ops[tok[2:-1]]
        if tok == "m0":
            return self.m0
        if tok[0] == "v" and tok[1:].isdigit():
            return self.v[int(tok[1:])]
        if tok[0] == "s" and tok[1:].isdigit():
            return int(self.s[int(tok[1:])])
        return int(tok, 0) & 0xFFFFFFFF

    def sset(self, tok, x):
        if tok == "m0":
            self.m0 = x & 0xFFFFFFFF
            return
        self.s[int(tok[1:])] = np.uint64(x & 0xFFFFFFFF)

    def vset(self, tok, x):
        if tok.startswith("%["):  # a read-write VGPR operand ("+v"), e.g. the column offset of the loop
            self.ops[tok[2:-1]] = np.asarray(x, dtype=np.uint64).astype(np.uint32)
            return
        self.v[_vreg(tok)] = np.asarray(x, dtype=np.uint64).astype(np.uint32) if np.ndim(x) else np.uint32(x)

    def pair(self, tok):
        if tok.startswith("%["):  # a 64-bit SGPR-pair operand
            return int(self.ops[tok[2:-1]])
        m = re.match(r"s\[(\d+):(\d+)\]", tok)
        lo, hi = int(m.group(1)), int(m.group(2))
        return int(self.s[lo]) | (int(self.s[hi]) << 32)

    def vsharp(self, tok):
        if tok.startswith("%["):  # a V# operand: (base, num_records)
            return int(self.ops[tok[2:-1]][0])
        m = re.match(r"s\[(\d+):(\d+)\]", tok)
        lo = int(m.group(1))
        return int(self.s[lo]) | ((int(self.s[lo + 1]) & 0xFFFF) << 32)

    def retire(self, n):
        """s_waitcnt vmcnt(n): retire the oldest vector-memory operations until at most n are left."""
        while len(self.vm) > n:
            r, data = self.vm.pop(0)
            if isinstance(r, tuple):  # LDS DMA
                self.lds[r[1]] = data
            elif r is not None:
                self.v[r] = data

    def drain(self):
        """Every load in flight lands (the wait a following step or the kernel end performs)."""
        self.retire(0)
        self.retire_lgkm(0)

    def retire_lgkm(self, n):
        """s_waitcnt lgkmcnt(n) under the lgkm model."""
        if n == 0 or not any(k == "s" for k, _, _ in self.lg):
            while len(self.lg) > n:
                kind, r, data = self.lg.pop(0)
                if kind == "s":
                    for w, x in enumerate(data):
                        self.s[r + w] = np.uint64(int(x))
                else:
                    self.v[r] = data

    def check_lgkm(self, ln):
        if not self.lg:
            return
        busy_v = {r for k, r, _ in self.lg if k == "v"}
        busy_s = set()
        for k, r, data in self.lg:
            if k == "s":
                busy_s.update(range(r, r + len(data)))
        for tok in re.findall(r"\bv(\d+)\b", ln):
            assert int(tok) not in busy_v, f"v{tok} named while its LDS read is in flight: {ln}"
        names = {int(t) for t in re.findall(r"\bs(\d+)\b", ln)}
        for lo, hi in re.findall(r"s\[(\d+):(\d+)\]", ln):
            names.update(range(int(lo), int(hi) + 1))
        hit = names & busy_s
        assert not hit, f"s{sorted(hit)[0]} named while its scalar load is in flight: {ln}"

    def check_vgprs(self, ln):
        busy = {r for r, _ in self.vm if isinstance(r, int)}
        if busy:
            for tok in re.findall(r"\bv(\d+)\b", ln):
                assert int(tok) not in busy, f"v{tok} used before its load was waited for: {ln}"

    def run(self, lines, finish, entry=None):
        """Executes `lines` from label `entry` (or the top) until its end or an s_setpc_b64 (the finish
        blocks' return); labels, s_branch / s_cbranch_scc0/1 jumps within `lines`."""
        labels = {ln[:-1]: i for i, ln in enumerate(lines) if ln.endswith(":")}
        pc = labels[entry] if entry else 0
        self.setpc = None  # the target pair of the s_setpc_b64 that ended this run, if one did
        while pc < len(lines):
            ln = lines[pc]
            pc += 1
            if ln.endswith(":"):
                continue
            op, _, rest = ln.partition(" ")
            a = [x.strip() for x in re.split(r",\s*(?![^\[]*\])", rest)] if rest else []
            if op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", rest)
                if m:
                    self.retire(int(m.group(1)))
                m = re.search(r"lgkmcnt\((\d+)\)", rest)
                if m and self.lgkm:
                    self.retire_lgkm(int(m.group(1)))
                continue
            self.check_vgprs(ln)
            if self.lgkm:
                self.check_lgkm(ln)
            if op == "s_setpc_b64":
                self.setpc = a[0]
                return
            if op == "s_branch":
                if entry is None and a[0] in labels:  # the role code's own jumps (the finish is entered by call)
                    pc = labels[a[0]]
                continue
            if op in ("s_cbranch_scc0", "s_cbranch_scc1"):
                if (self.scc != 0) == (op == "s_cbranch_scc1"):
                    pc = labels[a[0]]
                continue
            if op in ("s_cmp_gt_u32", "s_cmp_lg_u32", "s_cmp_eq_u32"):
                x, y = self.val(a[0]), self.val(a[1])
                self.scc = int(x > y) if op == "s_cmp_gt_u32" else int(x != y) if op == "s_cmp_lg_u32" else int(x == y)
                continue
            if op == "s_sub_u32":
                t = self.val(a[1]) - self.val(a[2])
                self.scc = int(t < 0)
                self.sset(a[0], t)
                continue
            if op in ("s_nop", "s_getpc_b64", "s_barrier", "s_setprio"):
                continue
            if op == "s_bitcmp1_b32":  # masked loads: SCC = bit a[1] of a[0]
                self.scc = (self.val(a[0]) >> (self.val(a[1]) & 31)) & 1
                continue
            if op == "s_cselect_b64":  # dst pair = SCC ? src0 : src1 (a "%[name]" source is a 64-bit operand)
                lo = int(re.match(r"s\[(\d+):", a[0]).group(1))
                pick = a[1] if self.scc else a[2]
                v = self.ops[pick[2:-1]] if pick.startswith("%[") else self.pair(pick)
                self.s[lo], self.s[lo + 1] = np.uint64(v & 0xFFFFFFFF), np.uint64((v >> 32) & 0xFFFFFFFF)
                continue
            # gpr-index mode (s_set_gpr_idx_on ..., gpr_idx(SRC0)): src0 of VALU ops is offset by the index
            if op == "s_set_gpr_idx_on":
                assert a[1] == "gpr_idx(SRC0)", ln
                self.gpr_idx = self.val(a[0]) & 0xFF
                continue
            if op == "s_set_gpr_idx_idx":
                self.gpr_idx = self.val(a[0]) & 0xFF
                continue
            if op == "s_set_gpr_idx_off":
                self.gpr_idx = None
                continue
            if getattr(self, "gpr_idx", None) is not None and op.startswith("v_") and len(a) > 1:
                # only a VGPR src0 is offset; constants and SGPRs in src0 are not
                if re.fullmatch(r"v\d+", a[1]):
                    a[1] = f"v{_vreg(a[1]) + self.gpr_idx}"
            if op in ("s_load_dwordx16", "s_load_dwordx8", "s_load_dwordx4"):
                m = re.match(r"s\[(\d+):(\d+)\]", a[0])
                lo, cnt = int(m.group(1)), int(op[len("s_load_dwordx"):])
                assert int(m.group(2)) - lo + 1 == cnt, ln
                addr = self.pair(a[1]) + int(a[2], 0)
                words = self.mem.load32(np.uint64(addr) + 4 * np.arange(cnt, dtype=np.uint64))
                if self.lgkm:
                    self.lg.append(("s", lo, words))
                    continue
                for w in range(cnt):
                    self.s[lo + w] = np.uint64(int(words[w]))
                continue
            if op == "v_sub_u32":
                self.vset(a[0], (self.val(a[1]).astype(np.int64) - self.val(a[2])) & 0xFFFFFFFF)
                continue
            if op == "s_swappc_b64":
                self.run(finish, finish, self.call)
            elif op == "s_mov_b32":
                self.sset(a[0], self.val(a[1]))
            elif op == "s_mov_b64":
                lo = int(re.match(r"s\[(\d+):", a[0]).group(1))
                v = self.pair(a[1])
                self.s[lo], self.s[lo + 1] = np.uint64(v & 0xFFFFFFFF), np.uint64(v >> 32)
            elif op == "s_lshr_b64":
                lo = int(re.match(r"s\[(\d+):", a[0]).group(1))
                v = self.pair(a[1]) >> (self.val(a[2]) & 63)
                self.s[lo], self.s[lo + 1] = np.uint64(v & 0xFFFFFFFF), np.uint64((v >> 32) & 0xFFFFFFFF)
            elif op == "s_lshr_b32":
                self.sset(a[0], self.val(a[1]) >> (self.val(a[2]) & 31))
            elif op == "s_and_b32":
                self.sset(a[0], self.val(a[1]) & self.val(a[2]))
            elif op == "s_mul_i32":
                self.sset(a[0], self.val(a[1]) * self.val(a[2]))
            elif op == "s_add_u32":
                if "L_" in a[2]:
                    self.call = a[2].split("-")[0]  # call-target arithmetic: the finish entry label
                    continue
                t = self.val(a[1]) + self.val(a[2])
                self.scc = t >> 32
                self.sset(a[0], t)
            elif op == "s_addc_u32":
                if a[0] == "s57":
                    continue
                t = self.val(a[1]) + (self.val(a[2]) & 0xFFFFFFFF) + self.scc
                self.scc = t >> 32
                self.sset(a[0], t)
            elif op == "v_mov_b32":
                self.vset(a[0], self.val(a[1]))
            elif op in ("v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32"):  # with an all-ones mask: lane id parts
                assert self.val(a[1]) == 0xFFFFFFFF, ln
                lanes = np.arange(64, dtype=np.uint64)
                part = np.minimum(lanes, 32) if op == "v_mbcnt_lo_u32_b32" else np.maximum(lanes, 32) - 32
                self.vset(a[0], (part + np.asarray(self.val(a[2]), np.uint64)) & np.uint64(0xFFFFFFFF))
            elif op == "v_lshl_add_u32":
                x = np.asarray(self.val(a[1]), np.uint64) << np.uint64(self.val(a[2]) & 31)
                self.vset(a[0], (x + np.asarray(self.val(a[3]), np.uint64)) & np.uint64(0xFFFFFFFF))
            elif op == "v_add_u32":
                self.vset(a[0], (np.asarray(self.val(a[1]), np.uint64) + np.asarray(self.val(a[2]), np.uint64))
                          & np.uint64(0xFFFFFFFF))
            elif op == "v_xor_b32":
                self.vset(a[0], self.val(a[1]) ^ self.val(a[2]))
            elif op == "v_and_b32":
                self.vset(a[0], np.uint32(self.val(a[1])) & self.val(a[2]))
            elif op == "v_lshlrev_b32":
                self.vset(a[0], (self.val(a[2]).astype(np.uint64) << np.uint64(self.val(a[1]) & 31)) & np.uint64(0xFFFFFFFF))
            elif op == "v_lshrrev_b32":
                self.vset(a[0], self.val(a[2]) >> np.uint32(self.val(a[1])))
            elif op == "v_mul_u32_u24":
                x = self.val(a[2]).astype(np.uint64) & np.uint64(0xFFFFFF)
                self.vset(a[0], (np.uint64(self.val(a[1]) & 0xFFFFFF) * x) & np.uint64(0xFFFFFFFF))
            elif op == "v_bitop3_b32":
                a3, mod = a[3].split()
                tt = int(mod.split(":")[1], 0)
                x, y, z = (np.broadcast_to(np.uint32(self.val(t)), (64,)) for t in (a[1], a[2], a3))
                r = np.zeros(64, np.uint32)
                for idx in range(8):  # truth table index = src0 << 2 | src1 << 1 | src2
                    if (tt >> idx) & 1:
                        m0 = x if idx & 4 else ~x
                        m1 = y if idx & 2 else ~y
                        m2 = z if idx & 1 else ~z
                        r |= m0 & m1 & m2
                self.vset(a[0], r)
            elif op == "v_pk_add_u16":
                x, y = self.val(a[1]), self.val(a[2])
                lo = ((x & 0xFFFF) + (y & 0xFFFF)) & 0xFFFF
                hi = ((x >> 16) + (y >> 16)) & 0xFFFF
                self.vset(a[0], lo | (hi << np.uint32(16)))
            elif op == "v_pk_mul_lo_u16":
                src1, mod = a[2].split()
                assert mod == "op_sel_hi:[0,1]", ln  # src0's low half for both lanes
                c = self.val(a[1]) & 0xFFFF
                x = self.val(src1)
                lo = ((x & 0xFFFF).astype(np.uint64) * c) & 0xFFFF
                hi = ((x >> 16).astype(np.uint64) * c) & 0xFFFF
                self.vset(a[0], (lo | (hi << np.uint64(16))).astype(np.uint32))
            elif op == "v_pk_ashrrev_i16":
                src, mod = a[2].split()
                assert mod == "op_sel_hi:[0,1]", ln  # shift count from the low half for both lanes
                sh = self.val(a[1]) & 0xF
                x = self.val(src)
                lo = ((x & 0xFFFF).astype(np.uint16).view(np.int16) >> sh).view(np.uint16).astype(np.uint32)
                hi = ((x >> 16).astype(np.uint16).view(np.int16) >> sh).view(np.uint16).astype(np.uint32)
                self.vset(a[0], lo | (hi << np.uint32(16)))
            elif op == "global_load_dword":
                mods = a[2].split()[1:]
                off = sum(int(m.split(":")[1], 0) for m in mods if m.startswith("offset:"))
                addr = self.pair(a[2].split()[0]) + self.val(a[1]).astype(np.uint64) + np.uint64(off)
                self.vm.append((_vreg(a[0]), self.mem.load32(addr)))
            elif op == "global_store_dword":
                addr = self.pair(a[2].split()[0]) + self.val(a[0]).astype(np.uint64)
                self.mem.store32(addr, self.val(a[1]))
                self.vm.append((None, None))
            elif op == "buffer_load_dword" and ln.endswith(" lds"):
                # LDS DMA: a[0] = voffset, a[1] = V#, a[2] = "soffset offen lds"; raw buffer range check
                # on the VGPR offset as for VGPR loads (out of range: zero written to LDS)
                voff = np.asarray(self.val(a[0]), np.uint64)
                addr = self.vsharp(a[1]) + self.val(a[2].split()[0]) + voff
                nrec = int(self.s[int(re.match(r"s\[(\d+):", a[1]).group(1)) + 2])
                inb = voff < np.uint64(nrec)
                data = np.where(inb, self.mem.load32(np.where(inb, addr, np.uint64(0))), np.uint32(0)).astype(np.uint32)
                dst = self.m0 + 4 * np.arange(64)
                idx = dst[:, None] + np.arange(4)[None, :]
                self.vm.append((("lds", idx.reshape(-1)), data.astype("<u4").view(np.uint8)))  # lands at retire
            elif op == "ds_write_b32":
                base, off = a[0], 0
                if " " in a[1]:
                    a1, o = a[1].split()
                    off = int(o.split(":")[1])
                else:
                    a1 = a[1]
                addr = self.val(base).astype(np.int64) + off
                idx = addr[:, None] + np.arange(4)[None, :]
                self.lds[idx.reshape(-1)] = np.ascontiguousarray(self.val(a1), dtype="<u4").view(np.uint8)
            elif op == "ds_read_b32":
                base, _, off = a[1].partition(" ")
                assert not off or off.startswith("offset:"), ln
                addr = self.val(base).astype(np.int64) + (int(off.split(":")[1]) if off else 0)
                idx = addr[:, None] + np.arange(4)[None, :]
                data = self.lds[idx].copy().view("<u4").reshape(-1)
                if self.lgkm:
                    self.lg.append(("v", _vreg(a[0]), data))
                else:
                    self.vset(a[0], data)
            elif op in ("ds_read_u16", "ds_read_u16_d16_hi"):
                # gfx950 (SRAM-ECC): d16 loads do not preserve the other half -- it is zeroed
                addr = self.val(a[1]).astype(np.int64)
                h = (self.lds[addr].astype(np.uint32) | (self.lds[addr + 1].astype(np.uint32) << np.uint32(8)))
                self.vset(a[0], h << np.uint32(16) if op.endswith("_hi") else h)
            elif op == "buffer_load_dword":
                assert a[3].endswith("offen"), ln
                voff = self.val(a[1]).astype(np.uint64)
                addr = self.vsharp(a[2]) + self.val(a[3].split()[0]) + voff
                # raw buffer (stride 0) range check on the VGPR offset: out of range loads return 0
                nrec = (int(self.ops[a[2][2:-1]][1]) if a[2].startswith("%[")
                        else int(self.s[int(re.match(r"s\[(\d+):", a[2]).group(1)) + 2]))
                inb = voff < np.uint64(nrec)
                data = self.mem.load32(np.where(inb, addr, np.uint64(0)))
                self.vm.append((_vreg(a[0]), np.where(inb, data, np.uint32(0)).astype(np.uint32)))
            elif op == "buffer_store_dword":
                addr = self.vsharp(a[2]) + self.val(a[3].split()[0]) + self.val(a[1]).astype(np.uint64)
                self.mem.store32(addr, self.val(a[0]))
                self.vm.append((None, None))
            else:
                raise NotImplementedError(ln)


def gamma_table():
    """T[w] = gamma * w in GF(2^16) (poly 0x1002D, gamma = alpha^257): the LDS table of the fin = 1
    kernels, as little-endian bytes."""
    exp = np.zeros(2 * 65535, np.uint32)
    x = 1
    for i in range(65535):
        exp[i] = x
        x <<= 1
        if x & 0x10000:
            x ^= 0x1002D
    exp[65535:] = exp[:65535]
    log = np.zeros(65536, np.int64)
    log[exp[:65535]] = np.arange(65535)
    t = np.zeros(65536, np.uint16)
    t[1:] = exp[log[1:] + 257]
    return t.astype("<u2").view(np.uint8)


class Memory:
    """Flat little-endian byte space for emulated loads/stores."""

    def __init__(self, nbytes):
        self.b = np.zeros(nbytes, np.uint8)

    def load32(self, addr):
        idx = addr.astype(np.int64)[:, None] + np.arange(4)[None, :]
        return self.b[idx].copy().view("<u4").reshape(-1)

    def store32(self, addr, val):
        idx = addr.astype(np.int64)[:, None] + np.arange(4)[None, :]
        self.b[idx.reshape(-1)] = np.ascontiguousarray(val, dtype="<u4").view(np.uint8)


def run_block(src, mem, src_base, src_sym, dst_base, dst_sym, chunk=0, ncols=1, gx=1, masks=None, zero=None,
              lds_init=None):
    """Runs every role wave of block (chunk, stripe 0) of the generated kernel over `mem`
    (LDS base address 0; each role's ring region at role * region bytes). Column-loop kernels (cpb > 1)
    process `ncols` columns from `chunk`, `gx` (the grid's x size) columns apart. Masked kernels take the
    stripe's mask words (`masks`, list of ints) and the byte address of a zero buffer in `mem` (`zero`)."""
    finish, roles = split_source(src)
    m = re.search(r"\(uint32_t\)role \* (\d+)u", src)
    region = int(m.group(1)) if m else 0
    lds = np.zeros(max(1, region * len(roles)) + 64, np.uint8)
    if "ds_read_u16_d16_hi" in src:  # LDS finish: the gamma table at LDS address 0
        lds = gamma_table().copy()
    if "ds_write_b32" in src:  # shared table exchange between the roles
        lds = np.zeros(1 << 16, np.uint8)
    if lds_init is not None:  # LDS contents the kernel's C prologue copies in (coordinate tables at 0)
        lds = np.zeros(max(lds.size, lds_init.size), np.uint8)
        lds[:lds_init.size] = lds_init
    col = (chunk * 256 + np.arange(64) * 4).astype(np.uint32)
    waves, segments = [], []
    for w, lines in enumerate(roles):
        lb = w * region
        ops = dict(col=col, sl=src_base & 0xFFFFFFFF, sh=src_base >> 32, dl=dst_base & 0xFFFFFFFF,
                   dh=dst_base >> 32, ss=src_sym, ds=dst_sym, lb=lb, nc=ncols, cs=gx * 256,
                   la=(lb + np.arange(64) * 4).astype(np.uint32))
        ops["col"] = col.copy()
        if masks is not None:  # the kernel's C prologue: mask words and the zero base of this column
            for i, w in enumerate(masks):
                ops[f"mw{i}"] = int(w)
            ops["zb"] = int(zero)
        wave = Wave(mem, ops, lgkm=True)
        wave.lds = lds
        waves.append(wave)
        seg = [[]]  # the block's waves run in lockstep between s_barriers
        for ln in lines:
            if ln == "s_barrier" and "L_xj_col" not in src:  # column-loop roles share nothing: barrier = no-op
                seg.append([])
            else:
                seg[-1].append(ln)
        segments.append(seg)
    assert len({len(sg) for sg in segments}) == 1, "roles reach different numbers of barriers"
    for i in range(len(segments[0])):
        for wave, seg in zip(waves, segments):
            wave.run(seg[i], finish)
