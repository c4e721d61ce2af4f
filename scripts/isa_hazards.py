#!/usr/bin/env python3
"""Static check of gfx950 disassembly for registers used while a memory load into them is in flight.

CDNA does not interlock memory results: a load's destination registers must not be read (or written)
until the matching s_waitcnt has retired the load. The compiler's waitcnt pass guarantees this for code
it generates; hand-written inline asm has to get it right itself, and an operand constraint that lets
the compiler place an asm input inside an asm output (no early clobber) breaks it silently. Round 4's
illegal-address fault was exactly that: `sload32` (csrc/rs_device.h) issued

    s_load_dwordx16 s[8:23], s[10:11], 0x0
    s_load_dwordx16 s[72:87], s[10:11], 0x40

so the second load's base could be overwritten by the first load's data before it issued.

Model (each function in address order; the state at a branch target is the union of every path that
jumps there, back edges included -- a few passes to a fixed point; after an unconditional branch the
next instruction is reached only by jumps):
  * SMEM loads (s_load_* / s_buffer_load_*): destinations in flight until s_waitcnt lgkmcnt(0) (SMEM
    returns out of order, so only lgkmcnt(0) retires them);
  * LDS loads (ds_read* / ds_load*): in flight until an lgkmcnt(N) leaves at most N newer lgkm ops;
  * vector memory loads (global_/buffer_/flat_/scratch_load*, not the LDS-DMA forms): in issue order,
    retired by vmcnt(N) (N = ops allowed outstanding, stores included in the count).
Any operand of a later instruction that overlaps an in-flight destination is reported.

Second check (`valu_sgpr_hazards`): an SGPR written by a VALU instruction (v_readfirstlane / v_readlane, a
VALU compare or carry-out into an SGPR) and read by a vector memory instruction (its saddr, srsrc or
soffset) fewer than 5 wait states later. gfx9 does not interlock this; the compiler inserts s_nop for its
own code, but not inside inline asm (the SGPR-addressed stores of m8_v1h_store, the s_cselect-chosen load
bases of the masked rs_xj pass). Wait states are counted per instruction (s_nop N counts N + 1), in
address order; a branch, s_endpgm or a branch target ends the window (conservative at joins only by
restarting, which the kernels here never need).

Usage: isa_hazards.py <code object or .so or disassembly .s> [...]; exit 1 if anything is found.
Importable: hazards(text) -> list of (function, address, instruction, registers).
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
_REG = re.compile(r"\b([sv])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")
_FUNC = re.compile(r"^[0-9a-fA-F]+ <([^>]+)>:")
_INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*//\s*([0-9A-Fa-f]+):\s*([0-9A-Fa-f]{8})")


def _regs(text):
    out = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _split_ops(args):
    # operands are comma separated; modifiers (offset:, glc, ...) follow the last comma-less token
    return [a.strip() for a in args.split(",")] if args else []


def _counts(args):
    c = {}
    for name in ("vmcnt", "lgkmcnt", "expcnt"):
        m = re.search(name + r"\((\d+)\)", args or "")
        if m:
            c[name] = int(m.group(1))
    return c


def disassemble(path):
    """Disassembly text of a gfx950 code object, of a .s file, or of the device code inside a host .so
    (its .hip_fatbin section, unbundled)."""
    if path.endswith(".s"):
        with open(path) as f:
            return f.read()
    with open(path, "rb") as f:
        elf = f.read(20)
    if elf[18:20] == b"\xe0\x00":  # an AMDGPU ELF
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", path], text=True)
    # a host library carrying a fat binary: one offload bundle per translation unit with device code
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin.bin")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb])
        with open(fb, "rb") as f:
            blob = f.read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts, i = [], blob.find(magic)
        while i >= 0:
            starts.append(i)
            i = blob.find(magic, i + 1)
        texts = []
        for n, (a, b) in enumerate(zip(starts, starts[1:] + [len(blob)])):
            part, obj = os.path.join(d, f"b{n}.bin"), os.path.join(d, f"dev{n}.co")
            with open(part, "wb") as f:
                f.write(blob[a:b])
            subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                   "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                                   f"--output={obj}"])
            texts.append(subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", obj], text=True))
        return "\n".join(texts)


_BRANCH = re.compile(r"^s_(c?branch)")


class _State:
    """Loads in flight: SMEM destinations, lgkm ops in order (is_smem, regs), VMEM ops in order (regs)."""

    def __init__(self, smem=(), lgkm=(), vmem=()):
        self.smem, self.lgkm, self.vmem = list(smem), list(lgkm), list(vmem)

    def copy(self):
        return _State(self.smem, self.lgkm, self.vmem)

    def merge(self, o):
        # union: an op in flight on either path is in flight here; order by the longer queue
        self.smem = self.smem + [r for r in o.smem if r not in self.smem]
        if len(o.lgkm) > len(self.lgkm):
            self.lgkm, extra = list(o.lgkm), self.lgkm
        else:
            extra = o.lgkm
        self.lgkm += [x for x in extra if x not in self.lgkm]
        if len(o.vmem) > len(self.vmem):
            self.vmem, extra = list(o.vmem), self.vmem
        else:
            extra = o.vmem
        self.vmem += [x for x in extra if x not in self.vmem]

    def key(self):
        f = lambda rs: tuple(sorted(rs))
        return (tuple(f(r) for r in self.smem), tuple((s, f(r)) for s, r in self.lgkm), tuple(f(r) for r in self.vmem))

    def busy(self):
        b = set()
        for r in self.smem:
            b |= r
        for s, r in self.lgkm:
            if not s:
                b |= r
        for r in self.vmem:
            b |= r
        return b


def _step(st, op, args):
    """Apply one instruction to the in-flight state (after its operands were checked)."""
    ops = _split_ops(args)
    if op == "s_waitcnt":
        c = _counts(args)
        if "lgkmcnt" in c:
            n = c["lgkmcnt"]
            st.lgkm = st.lgkm[len(st.lgkm) - n:] if n else []
            st.smem = [r for s, r in st.lgkm if s] if n else []
        if "vmcnt" in c:
            n = c["vmcnt"]
            st.vmem = st.vmem[len(st.vmem) - n:] if n else []
    elif op.startswith(("s_load_", "s_buffer_load_", "s_memtime", "s_memrealtime")) and ops:
        d = _regs(ops[0])
        st.smem.append(d)
        st.lgkm.append((True, d))
    elif op.startswith(("ds_read", "ds_load")) and ops:
        st.lgkm.append((False, _regs(ops[0])))
    elif op.startswith("ds_"):
        st.lgkm.append((False, set()))
    elif re.match(r"(global|buffer|flat|scratch)_load", op):
        lds = "_lds_" in op or op.endswith("_lds") or " lds" in args
        st.vmem.append(set() if lds else _regs(ops[0]))
    elif re.match(r"(global|buffer|flat|scratch)_(store|atomic)", op):
        st.vmem.append(_regs(ops[0]) if ("glc" in args and "atomic" in op) else set())


def _functions(text):
    funcs, cur = [], None
    for line in text.splitlines():
        fm = _FUNC.match(line)
        if fm:
            cur = (fm.group(1), [])
            funcs.append(cur)
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            cur[1].append((int(m.group(3), 16), m.group(1), m.group(2) or "", int(m.group(4), 16)))
    # local labels inside a function (the JIT kernel's lookup blocks) continue it
    merged = []
    for name, body in funcs:
        if merged and (name.startswith("L_") or name.startswith(".L")):
            merged[-1][1].extend(body)
        else:
            merged.append((name, body))
    return merged


def hazards(text):
    found = []
    for func, body in _functions(text):
        at = {}  # address -> merged state of the branches that jump there
        seen = set()
        for _ in range(4):  # forward pass; back-edge states feed the next pass
            changed = False
            st = _State()
            for addr, op, args, word in body:
                if addr in at:
                    st.merge(at[addr])
                used = _regs(args)
                if re.match(r"(global|buffer|flat|scratch)_load", op) and "_lds" not in op:
                    # VMEM returns in order: a newer load into a register an older one still targets wins
                    vm = set()
                    for r in st.vmem:
                        vm |= r
                    used -= _regs(_split_ops(args)[0]) & vm - (st.busy() - vm)
                hit = used & st.busy()
                if hit and (addr, op) not in seen:
                    seen.add((addr, op))
                    found.append((func, f"{addr:X}", f"{op} {args}".strip(), sorted(hit)))
                _step(st, op, args)
                bm = _BRANCH.match(op)
                if bm:
                    simm = word & 0xFFFF  # SOPP: the branch offset in dwords past the next instruction
                    tgt = addr + 4 + 4 * (simm - 0x10000 if simm & 0x8000 else simm)
                    old = at.get(tgt)
                    new = st.copy() if old is None else old.copy()
                    if old is not None:
                        new.merge(st)
                    if old is None or new.key() != old.key():
                        at[tgt] = new
                        changed = changed or tgt <= addr
                if op in ("s_branch", "s_endpgm", "s_setpc_b64") or op.startswith("s_endpgm"):
                    st = _State()  # the next instruction is reached only by a jump
            if not changed:
                break
    return found


_VMEM = re.compile(r"(global|buffer|flat|scratch)_(load|store|atomic)")


def _sregs(text):
    return {i for kind, i in _regs(text) if kind == "s"}


def valu_sgpr_hazards(text, window=5):
    """(function, address, instruction, sgprs) for every VMEM instruction that reads an SGPR a VALU
    instruction wrote fewer than `window` wait states before it."""
    found = []
    for func, body in _functions(text):
        targets = set()
        for addr, op, args, word in body:
            if _BRANCH.match(op):
                simm = word & 0xFFFF
                targets.add(addr + 4 + 4 * (simm - 0x10000 if simm & 0x8000 else simm))
        recent = []  # [sgprs, wait states still needed]
        for addr, op, args, word in body:
            if addr in targets:
                recent = []
            if _VMEM.match(op):
                ops = _split_ops(args)
                reads = set()
                for o in ops:
                    reads |= _sregs(o)
                hit = set()
                for regs, left in recent:
                    if left > 0:
                        hit |= regs & reads
                if hit:
                    found.append((func, f"{addr:X}", f"{op} {args}".strip(), sorted(("s", r) for r in hit)))
            cost = 1
            if op == "s_nop":
                m = re.match(r"\s*(0x[0-9a-fA-F]+|\d+)", args or "0")
                cost = int(m.group(1), 0) + 1 if m else 1
            recent = [[regs, left - cost] for regs, left in recent if left - cost > 0]
            if op.startswith("v_"):
                ops = _split_ops(args)
                dst = _sregs(ops[0]) if ops else set()
                if len(ops) > 1 and ("_co_" in op or op.startswith(("v_div_scale", "v_add_co", "v_sub_co"))):
                    dst |= _sregs(ops[1])
                if dst:
                    recent.append([dst, window])
            if op in ("s_branch", "s_setpc_b64") or op.startswith("s_endpgm"):
                recent = []
    return found


def main(argv):
    bad = 0
    for p in argv[1:]:
        text = disassemble(p)
        for func, addr, insn, regs in hazards(text):
            bad += 1
            print(f"{p}: {func} @{addr}: {insn}   in flight: {regs}")
        for func, addr, insn, regs in valu_sgpr_hazards(text):
            bad += 1
            print(f"{p}: {func} @{addr}: {insn}   VALU-written SGPR within 5 wait states: {regs}")
    print(f"{bad} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
