"""The hand-scheduled m = 16 input step (reed-solomon_amd/csrc/gen_asm.py variant m16_v1, used by
k_apply_m16_v1) run by the instruction emulator on CPU: after one step every accumulator must hold
acc ^ c_p * x for both packed GF(2^16) words of every lane, with c_p taken from the step's index
record exactly as rs_api.cpp:build_plan lays it out."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from xj_emu import Memory, Wave

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "..", "reed-solomon_amd", "csrc", "gen_asm.py")


def gf_mul(a, b):
    """GF(2^16) product, poly 0x1002D (numpy, elementwise)."""
    a = np.asarray(a, np.uint32).copy()
    b = np.asarray(b, np.uint32).copy()
    r = np.zeros(np.broadcast(a, b).shape, np.uint32)
    for _ in range(16):
        r ^= np.where(b & 1, a, 0).astype(np.uint32)
        b >>= 1
        a = ((a << 1) ^ np.where(a & 0x8000, 0x1002D, 0)).astype(np.uint32) & 0xFFFF
    return r


def step_lines(tmp_path):
    out = os.path.join(tmp_path, "m16.inc")
    subprocess.check_call([sys.executable, GEN, out, "m16_v1"])
    lines = []
    for ln in open(out):
        m = re.match(r'^"(.*)\\n\\t"$', ln.strip())
        if m:
            lines.append(m.group(1))
    return lines


def test_m16_v1_step_matches_gf_multiply(tmp_path):
    rng = np.random.default_rng(16)
    coef = rng.integers(0, 65536, 64, dtype=np.uint32)
    coef[:4] = [0, 1, 2, 0xFFFF]
    rec = np.zeros(256, np.uint8)  # packed as rs_api.cpp:build_plan
    for n in range(4):
        for j in range(64):
            rec[4 * (16 * n + 2 * (j // 8) + j % 2) + (j % 8) // 2] = 16 * n + ((coef[j] >> (4 * n)) & 15)
    mem = Memory(4096)
    mem.b[1024:1280] = rec
    x = rng.integers(0, 2 ** 32, 64, dtype=np.uint64).astype(np.uint32)
    acc0 = rng.integers(0, 2 ** 32, (64, 64), dtype=np.uint64).astype(np.uint32)
    text = "\n".join(step_lines(str(tmp_path)))
    text = (text.replace("%[t0]", "v200").replace("%[t1]", "v201").replace("%[y0]", "v202")
            .replace("%[k2d]", "v203").replace("%[cp]", "s[90:91]"))
    w = Wave(mem, {}, lgkm=True)
    w.v[202] = x
    w.v[203] = 0x002D002D
    w.v[72:136] = acc0
    w.s[90], w.s[91] = 1024, 0
    w.run(["s_load_dwordx16 s[40:55], s[90:91], 0x0"] + text.splitlines(), [])  # the kernel's first-plane load
    w.drain()  # the next step (or the kernel) waits for these loads before use
    lo, hi = x & 0xFFFF, x >> 16
    for p in range(64):
        want = (gf_mul(lo, coef[p]) | (gf_mul(hi, coef[p]) << 16)) ^ acc0[p]
        assert np.array_equal(w.v[72 + p], want), p


def gf256_mul_bytes(x, c):
    """Each byte of the uint32 array x times c in GF(256) with gamma's minimal polynomial 0x11D."""
    out = np.zeros_like(x)
    for b in range(4):
        v = (x >> np.uint32(8 * b)) & np.uint32(0xFF)
        r = np.zeros_like(v)
        cc = int(c)
        for _ in range(8):
            if cc & 1:
                r ^= v
            cc >>= 1
            v = ((v << np.uint32(1)) ^ np.where(v & 0x80, 0x11D, 0).astype(np.uint32)) & np.uint32(0xFF)
        out |= r << np.uint32(8 * b)
    return out


def test_m8_v1_step_matches_gf256_multiply(tmp_path):
    """k_apply_m8_v1's input step (gen_asm.py variant v1): acc_p ^= c_p * y byte-wise in GF(256),
    c_p from the (lo, hi) nibble record of rs_api.cpp:build_plan."""
    out = os.path.join(str(tmp_path), "v1.inc")
    subprocess.check_call([sys.executable, GEN, out, "v1"])
    lines = [re.match(r'^"(.*)\\n\\t"$', ln.strip()).group(1) for ln in open(out) if ln.startswith('"')]
    rng = np.random.default_rng(8)
    coef = rng.integers(0, 256, 32, dtype=np.uint32)
    coef[:3] = [0, 1, 255]
    rec = np.zeros(64, np.uint32)
    rec[:32], rec[32:] = coef & 15, coef >> 4
    mem = Memory(4096)
    mem.b[1024:1280] = rec.astype("<u4").view(np.uint8)
    y = rng.integers(0, 2 ** 32, 64, dtype=np.uint64).astype(np.uint32)
    acc0 = rng.integers(0, 2 ** 32, (32, 64), dtype=np.uint64).astype(np.uint32)
    text = "\n".join(lines)
    text = (text.replace("%[t0]", "v200").replace("%[t1]", "v201").replace("%[y0]", "v202")
            .replace("%[k1d]", "v203").replace("%[cp]", "s[90:91]"))
    w = Wave(mem, {}, lgkm=True)
    w.v[202] = y
    w.v[203] = 0x1D1D1D1D
    w.v[40:72] = acc0
    w.s[90], w.s[91] = 1024, 0
    w.run(text.splitlines(), [])
    w.drain()  # the next step (or the kernel) waits for these loads before use
    for p in range(32):
        assert np.array_equal(w.v[40 + p], gf256_mul_bytes(y, coef[p]) ^ acc0[p]), p


def cs16_record(z):
    """Byte t' of coset c = e(t'), bit d of e(t') = bit (t' - d) mod 16 of z_c (gen_asm.py cs16a/b)."""
    rec = np.zeros((len(z), 16), np.uint8)
    for c in range(len(z)):
        for tp in range(16):
            rec[c, tp] = sum(((int(z[c]) >> ((tp - d) % 16)) & 1) << d for d in range(4))
    return rec.reshape(-1)


@pytest.mark.parametrize("variant", ["cs16a", "cs16b"])
def test_cs16_step_circulant_xor(tmp_path, variant):
    """k_cs16's group step (gen_asm.py variants cs16a / cs16b): for each of the wave's 4 syndrome cosets
    and each accumulator t, acc_t ^= XOR_a f_a * bit_((t - a) mod 16)(z_c) from the current inputs in
    v[136:151], both words of every lane; meanwhile the next group's inputs load into v[136:151] at lane
    + slot offset (an offset of 0x80000000 is out of the V#'s range: zero), the next record loads into
    the other record buffer and the slot offsets of the group after next into s[76:91]."""
    out = os.path.join(str(tmp_path), "cs16.inc")
    subprocess.check_call([sys.executable, GEN, out, variant])
    lines = [re.match(r'^"(.*)\\n\\t"$', ln.strip()).group(1) for ln in open(out) if ln.startswith('"')]
    cur, nxt = (40, 56) if variant == "cs16a" else (56, 40)
    rng = np.random.default_rng(1616)
    for trial in range(3):
        z = rng.integers(0, 65536, 4)
        z[:3] = [0, 0xFFFF, 1]
        mem = Memory(1 << 16)
        mem.b[1024:1088] = cs16_record(z)
        mem.b[1088:1152] = cs16_record(rng.integers(0, 65536, 4))  # the next group's record
        data = rng.integers(0, 256, 16384, dtype=np.uint8)
        mem.b[32768:32768 + 16384] = data  # stripe inputs: 16 symbols of 1 KiB at the V# base
        offs = np.array([1024 * ((a * 7) % 16) for a in range(16)], np.uint32)
        offs[3] = 0x80000000  # an empty slot
        mem.b[4160:4224] = rng.integers(0, 2 ** 31, 16).astype("<u4").view(np.uint8)  # the group after next
        f = rng.integers(0, 2 ** 32, (16, 64), dtype=np.uint64).astype(np.uint32)
        f[5] = 0  # an empty slot of the current group
        acc0 = rng.integers(0, 2 ** 32, (64, 64), dtype=np.uint64).astype(np.uint32)
        text = "\n".join(lines)
        text = (text.replace("%[cp]", "s[100:101]").replace("%[gp]", "s[92:93]").replace("%[rsrc]", "s[96:99]")
                .replace("%[lane]", "v230").replace("%[t0]", "v231").replace("%[t1]", "v232"))
        w = Wave(mem, {}, lgkm=True)
        w.v[136:152] = f
        w.v[72:136] = acc0
        lane = (np.arange(64) * 4 + 256).astype(np.uint32)
        w.v[230] = lane
        w.s[100], w.s[101] = 1024, 0
        w.s[92], w.s[93] = 4160, 0
        w.s[96], w.s[97], w.s[98], w.s[99] = 32768, 0, 16384, 0x20000
        w.s[76:92] = offs.astype(np.uint64)
        w.run([f"s_load_dwordx16 s[{cur}:{cur + 15}], s[100:101], 0x0"] + text.splitlines(), [])
        w.drain()  # the next step (or the kernel) waits for these loads before use
        for c in range(4):
            for t in range(16):
                want = acc0[16 * c + t].copy()
                for a in range(16):
                    if (int(z[c]) >> ((t - a) % 16)) & 1:
                        want ^= f[a]
                assert np.array_equal(w.v[72 + 16 * c + t], want), (trial, c, t)
        assert not w.v[8:72:16].any()  # table entry 0 stays zero
        words = data.view("<u4")
        for a in range(16):
            want = np.zeros(64, np.uint32) if offs[a] == 0x80000000 else words[(offs[a] + lane) // 4]
            assert np.array_equal(w.v[136 + a], want), (trial, a)
        assert list(w.s[76:92]) == list(mem.load32(np.uint64(4160) + 4 * np.arange(16, dtype=np.uint64)))
        assert list(w.s[nxt:nxt + 16]) == list(mem.load32(np.uint64(1088) + 4 * np.arange(16, dtype=np.uint64)))


def test_bs16_step_binary_accumulation(tmp_path):
    """k_bs16's group step (gen_asm.py bs16): for each of the wave's 4 output cosets and accumulator t,
    acc_t ^= XOR_j bit_t(z_(c, j)) * f_j over the step's 16 inputs (one gpr-index switch per (coset,
    table, t)); the coset records load one at a time, the next step's first one last."""
    out = os.path.join(str(tmp_path), "bs16.inc")
    subprocess.check_call([sys.executable, GEN, out, "bs16"])
    lines = [re.match(r'^"(.*)\\n\\t"$', ln.strip()).group(1) for ln in open(out) if ln.startswith('"')]
    rng = np.random.default_rng(1717)
    z = rng.integers(0, 65536, (4, 16))
    z[0, :] = 0
    z[1, 3] = 0xFFFF
    rec = np.zeros((4, 64), np.uint8)
    for c in range(4):
        for q in range(4):
            for t in range(16):
                rec[c, 16 * q + t] = sum(((int(z[c, 4 * q + d]) >> t) & 1) << d for d in range(4))
    mem = Memory(1 << 16)
    mem.b[1024:1280] = rec.reshape(-1)
    nxt = rng.integers(0, 256, 64, dtype=np.uint8)
    mem.b[1280:1344] = nxt  # the next step's coset-0 record
    mem.b[4160:4224] = rng.integers(0, 2 ** 31, 16).astype("<u4").view(np.uint8)
    data = rng.integers(0, 256, 16384, dtype=np.uint8)
    mem.b[32768:32768 + 16384] = data
    offs = np.array([1024 * a for a in range(16)], np.uint32)
    f = rng.integers(0, 2 ** 32, (16, 64), dtype=np.uint64).astype(np.uint32)
    acc0 = rng.integers(0, 2 ** 32, (64, 64), dtype=np.uint64).astype(np.uint32)
    text = "\n".join(lines)
    text = (text.replace("%[cp]", "s[100:101]").replace("%[gp]", "s[92:93]").replace("%[rsrc]", "s[96:99]")
            .replace("%[lane]", "v230").replace("%[t0]", "v231").replace("%[t1]", "v232"))
    w = Wave(mem, {}, lgkm=True)
    w.v[136:152] = f
    w.v[72:136] = acc0
    w.v[230] = (np.arange(64) * 4).astype(np.uint32)
    w.s[100], w.s[101] = 1024, 0
    w.s[92], w.s[93] = 4160, 0
    w.s[96], w.s[97], w.s[98], w.s[99] = 32768, 0, 16384, 0x20000
    w.s[76:92] = offs.astype(np.uint64)
    w.run(["s_load_dwordx16 s[40:55], s[100:101], 0x0"] + text.splitlines(), [])
    w.drain()  # the next step (or the kernel) waits for these loads before use
    for c in range(4):
        for t in range(16):
            want = acc0[16 * c + t].copy()
            for j in range(16):
                if (int(z[c, j]) >> t) & 1:
                    want ^= f[j]
            assert np.array_equal(w.v[72 + 16 * c + t], want), (c, t)
    assert list(w.s[40:56]) == list(nxt.view("<u4"))


def cs16t_parts(tmp_path):
    """(step lines, prologue lines before the blocks, {offset: block lines}, offset table, register bases
    {cw, F, R, acc}, the whole kernel loop without its blocks) of k_cs16t (gen_asm.py)."""
    d = str(tmp_path)
    for v, f in (("cs16t", "t.inc"), ("cs16t_kernel", "k.inc"), ("cs16t_off", "off.h")):
        subprocess.check_call([sys.executable, GEN, os.path.join(d, f), v])
    rd = lambda f: [re.match(r'^"(.*)\\n\\t"$', ln.strip()).group(1) for ln in open(os.path.join(d, f))
                    if ln.startswith('"')]
    step, kern = rd("t.inc"), rd("k.inc")
    head = kern[:kern.index("L_cst_blk%=:")]
    blocks, cur = {}, None
    for ln in kern[kern.index("L_cst_blk%=:") + 1:kern.index("L_cst_over%=:")]:
        m = re.match(r"\.if \. - L_cst_blk%= - (\d+)$", ln)
        if m:
            cur = blocks.setdefault(int(m.group(1)), [])
        elif not ln.startswith((".error", ".endif", "s_nop", ".p2align")):  # padding between blocks never runs
            cur.append(ln)
    txt = open(os.path.join(d, "off.h")).read()
    regs = {k: int(v) for k, v in re.findall(r"kCs16t(Cw|F|R|Acc) = (-?\d+)", txt)}
    off = [int(x) for x in re.search(r"kCs16tOff\[\d+\] = \{([^}]*)\}", txt).group(1).split(",")]
    assert len(off) == 64 * regs["Cw"]
    return step, head, blocks, off, regs, head + kern[kern.index("L_cst_over%=:"):]


def _circulant(acc0, f, z, cw):
    want = acc0.copy()
    for c in range(cw):
        for t in range(16):
            for a in range(16):
                if (int(z[c]) >> ((t - a) % 16)) & 1:
                    want[16 * c + t] ^= f[a]
    return want


def test_cs16t_threaded_step_circulant_xor(tmp_path):
    """k_cs16t's group step (gen_asm.py cs16t): R2_j = f_j ^ f_(j-1), then the 4 cw threaded blocks
    p = 4c + n named by the record (offsets kCs16tOff[(p, nibble n of z_c)]) give acc_t ^= XOR_a f_a *
    bit_((t - a) mod 16)(z_c) for each of the wave's cw syndrome cosets, exactly as cs16a; every block ends
    in the next record entry's block and the last returns. After the blocks the next group's inputs load
    into F at the lane's column + slot offset (an offset of 0x80000000 reads zero), the next record into
    s[40:] and the group after next's offsets into s[76:91]. Every block's code offset is also checked by
    the assembler at build time."""
    step, head, blocks, off, regs, _ = cs16t_parts(tmp_path)
    cw, F, A = regs["Cw"], regs["F"], regs["Acc"]
    nb = 4 * cw
    assert sorted(blocks) == sorted(off)
    for b, o in enumerate(off):  # every block ends in a jump to its successor position, or returns
        assert blocks[o][-1] == ("s_setpc_b64 s[74:75]" if b // 16 == nb - 1 else "s_setpc_b64 s[72:73]"), b
        if b // 16 < nb - 1:  # the successor's address is formed first, under the block's VALU
            assert blocks[o][:2] == [f"s_add_u32 s72, s92, s{41 + b // 16}", "s_addc_u32 s73, s93, 0"], b
        nv = sum(1 for ln in blocks[o] if ln.startswith("v_"))
        if b % 16 == 0:
            assert nv == 0, b
        else:  # one op per accumulator with pair sums, one or two from raw inputs
            assert nv == 16 if regs["R"] >= 0 else 16 <= nv <= 32, (b, nv)
    rng = np.random.default_rng(1618)
    text = "\n".join(step)
    text = (text.replace("%[cp]", "s[100:101]").replace("%[gp]", "s[94:95]").replace("%[rsrc]", "s[96:99]")
            .replace("%[colbase]", "s108"))
    for trial in range(4):
        z = rng.integers(0, 65536, cw)
        if trial == 0:
            z[:2] = [0, 0xFFFF]
        if trial == 1:
            z[:2] = [1, 0x8000]
        rec = np.array([off[(4 * c + n) * 16 + ((int(z[c]) >> (4 * n)) & 15)] for c in range(cw) for n in range(4)],
                       np.uint32)
        mem = Memory(1 << 16)
        nxt_rec = rng.integers(0, 2 ** 32, nb, dtype=np.uint64).astype(np.uint32)
        mem.b[1024 + 4 * nb:1024 + 8 * nb] = nxt_rec.astype("<u4").view(np.uint8)  # the next group's record
        data = rng.integers(0, 256, 16384, dtype=np.uint8)
        mem.b[32768:32768 + 16384] = data
        offs = np.array([1024 * ((a * 5) % 16) for a in range(16)], np.uint32)
        offs[7] = 0x80000000  # an empty slot
        mem.b[4160:4224] = rng.integers(0, 2 ** 31, 16).astype("<u4").view(np.uint8)  # the group after next
        f = rng.integers(0, 2 ** 32, (16, 64), dtype=np.uint64).astype(np.uint32)
        acc0 = rng.integers(0, 2 ** 32, (16 * cw, 64), dtype=np.uint64).astype(np.uint32)
        w = Wave(mem, {}, lgkm=True)
        w.v[F:F + 16] = f  # this group's inputs, loaded by the previous step
        w.v[A:A + 16 * cw] = acc0
        w.s[108] = 512  # the wave's byte column
        w.s[40:40 + nb] = rec.astype(np.uint64)  # this record, loaded by the previous step
        w.s[100], w.s[101] = 1024, 0
        w.s[94], w.s[95] = 4160, 0
        w.s[96], w.s[97], w.s[98], w.s[99] = 32768, 0, 16384, 0x20000
        w.s[92], w.s[93] = 0, 0  # block base: offsets address the blocks directly
        w.s[76:92] = offs.astype(np.uint64)
        lines = text.splitlines()
        w.run(lines, [])  # up to the jump into block 0
        visited = []
        while True:
            target = int(w.s[72]) | (int(w.s[73]) << 32)
            visited.append(target)
            assert target in blocks and len(visited) <= nb, visited
            w.run(blocks[target], [])
            if blocks[target][-1] == "s_setpc_b64 s[74:75]":
                break
        assert visited == list(rec), (visited, list(rec))
        w.run(lines, [], entry="L_cst_ret%=")  # back in the step: the next group's loads
        w.drain()
        assert np.array_equal(w.v[A:A + 16 * cw], _circulant(acc0, f, z, cw)), trial
        words = data.view("<u4")
        lane = (np.arange(64) * 4 + 512).astype(np.uint32)
        for a in range(16):
            want = np.zeros(64, np.uint32) if offs[a] == 0x80000000 else words[(offs[a] + lane) // 4]
            assert np.array_equal(w.v[F + a], want), (trial, a)
        assert list(w.s[76:92]) == list(mem.load32(np.uint64(4160) + 4 * np.arange(16, dtype=np.uint64)))
        assert list(w.s[40:40 + nb]) == list(nxt_rec)


def test_cs16t_prologue_loads_and_base(tmp_path):
    """k_cs16t's prologue issues group 0's 16 input loads into F, loads group 1's slot offsets and
    group 0's record, and holds all 64 cw blocks behind a jump (nothing but the base address is executed).
    The blocks read F and R2 and write the accumulators only: no block touches another register."""
    step, head, blocks, off, regs, _ = cs16t_parts(tmp_path)
    cw, F, R, A = regs["Cw"], regs["F"], regs["R"], regs["Acc"]
    assert "s_branch L_cst_over%=" in head and head.index("s_getpc_b64 s[92:93]") < head.index("s_branch L_cst_over%=")
    assert sum(1 for ln in head if ln.startswith("buffer_load_dword v")) == 16
    assert {int(re.match(r"buffer_load_dword v(\d+)", ln).group(1)) for ln in head if ln.startswith("buffer_load")} \
        == set(range(F, F + 16))
    for blk in blocks.values():
        for ln in blk:
            if ln.startswith("v_"):
                regs_ = [int(x) for x in re.findall(r"\bv(\d+)\b", ln)]
                assert A <= regs_[0] < A + 16 * cw and regs_[1] == regs_[0], ln
                assert all(F <= x < F + 16 or (R >= 0 and R <= x < R + 16) for x in regs_[2:]), ln
    assert off == sorted(off) and off[0] == 0


def test_cs16t_kernel_loop_over_groups(tmp_path):
    """The whole k_cs16t group loop (gen_asm.py cs16t_kernel, one asm statement) in the emulator over
    several groups: the prologue's loads, every step's R2, threaded blocks, record / slot-offset loads,
    the loop count and the final wait. The accumulators equal the circulant sums over all groups' inputs
    (empty slots read zero); a zero group count runs no step."""
    step, head, blocks, off, regs, main = cs16t_parts(tmp_path)
    cw, F, A = regs["Cw"], regs["F"], regs["Acc"]
    nb = 4 * cw
    rng = np.random.default_rng(16016)
    text = "\n".join(main)
    text = (text.replace("%[g0]", "s[102:103]").replace("%[g2]", "s[104:105]").replace("%[r0]", "s[100:101]")
            .replace("%[ng]", "s109").replace("%[rsrc]", "s[112:115]").replace("%[colbase]", "s108"))
    lines = text.splitlines()
    for ng in (5, 0):
        z = rng.integers(0, 65536, (ng, cw))
        mem = Memory(1 << 17)
        G0, R0, DATA = 4096, 8192, 65536
        offs = (1024 * rng.integers(0, 32, (ng + 3, 16))).astype(np.uint32)
        offs[rng.random((ng + 3, 16)) < 0.2] = 0x80000000  # empty slots
        mem.b[G0:G0 + offs.size * 4] = offs.astype("<u4").view(np.uint8).reshape(-1)
        rec = np.array([[off[(4 * c + n) * 16 + ((int(z[g, c]) >> (4 * n)) & 15)] for c in range(cw) for n in range(4)]
                        for g in range(ng)] + [[off[p * 16] for p in range(nb)]] * 2, np.uint32)
        mem.b[R0:R0 + rec.size * 4] = rec.astype("<u4").view(np.uint8).reshape(-1)
        data = rng.integers(0, 256, 32768, dtype=np.uint8)
        mem.b[DATA:DATA + 32768] = data
        w = Wave(mem, {}, lgkm=True)
        acc0 = rng.integers(0, 2 ** 32, (16 * cw, 64), dtype=np.uint64).astype(np.uint32)
        w.v[A:A + 16 * cw] = acc0
        w.s[102], w.s[103] = G0, 0
        w.s[104], w.s[105] = G0 + 128, 0
        w.s[100], w.s[101] = R0, 0
        w.s[109] = ng
        w.s[108] = 256
        w.s[112], w.s[113], w.s[114], w.s[115] = DATA, 0, 32768, 0x20000
        w.run(lines, [])
        steps = 0
        while w.setpc == "s[72:73]":  # into a step's blocks
            visited = 0
            while True:
                target = int(w.s[72]) - (int(w.s[92]) | (int(w.s[93]) << 32))
                w.run(blocks[target], [])
                visited += 1
                if w.setpc == "s[74:75]":
                    break
                assert w.setpc == "s[72:73]" and visited < nb
            assert visited == nb
            steps += 1
            w.run(lines, [], entry="L_cst_ret%=")
        assert w.setpc is None and steps == ng
        words = data.view("<u4")
        lane = (np.arange(64) * 4 + 256).astype(np.uint32)
        want = acc0.copy()
        for g in range(ng):
            f = [np.zeros(64, np.uint32) if offs[g, a] == 0x80000000 else words[(offs[g, a] + lane) // 4] for a in range(16)]
            want = _circulant(want, f, z[g], cw)
        assert np.array_equal(w.v[A:A + 16 * cw], want), ng
