"""rs_amd -- Python host side of the MI355X Reed-Solomon engine (ctypes over librs_amd.so).

Two layers, both thin wrappers over the C ABI (include/rs/reed_solomon.h, include/rs_amd/rsg.h):

* ``RS``     -- mirror of the reference codec API (reference include/rs/reed_solomon.h:44-74):
               ``generate_repair_symbols(inf, rep)`` and ``restore_symbols(k, r, rcv, is_erased, t)``
               over lists of host symbols (numpy uint8 arrays), same return codes.
* ``Codec``  -- the batched device-resident engine over torch tensors already in HBM
               (shape [n_stripes, k + r, symbol_size] uint8 or explicit strides).

There is no CPU fallback: if librs_amd.so is missing this module raises on import, and a codec
cannot be created without a GPU.
"""
import atexit
import ctypes
import weakref
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RS_AMD_LIB selects another build of the library (the diagnostic librs_amd_diag.so of the sweep
# scripts); the default is the product build
LIB_PATH = os.environ.get("RS_AMD_LIB") or os.path.join(HERE, "librs_amd.so")

RS_OK = 0
RS_ERR_ALLOC = 1
RS_ERR_INVALID = 2
RS_ERR_DEVICE = 3
RS_ERR_CANNOT_RESTORE = 100


class RSError(RuntimeError):
    def __init__(self, rc, what):
        super().__init__(f"{what} failed with code {rc}")
        self.rc = rc


DIAG_LIB_PATH = os.path.join(HERE, "librs_amd_diag.so")


def diag_module():
    """A second instance of this module bound to the diagnostic library (librs_amd_diag.so: the option-only
    A/B kernel families, ablations and stamps the release library does not carry), loaded beside the
    release library in the same process. Raises ImportError when that library is not built."""
    import importlib.util
    import sys
    name = "rs_amd_diag"
    if name in sys.modules:
        return sys.modules[name]
    if not os.path.exists(DIAG_LIB_PATH):
        raise ImportError(f"{DIAG_LIB_PATH} is missing: build it with `make -C {HERE} diag`")
    spec = importlib.util.spec_from_file_location(name, os.path.abspath(__file__))
    mod = importlib.util.module_from_spec(spec)
    old = os.environ.get("RS_AMD_LIB")
    os.environ["RS_AMD_LIB"] = DIAG_LIB_PATH
    try:
        spec.loader.exec_module(mod)
    finally:
        if old is None:
            os.environ.pop("RS_AMD_LIB", None)
        else:
            os.environ["RS_AMD_LIB"] = old
    sys.modules[name] = mod
    return mod


def build(force=False):
    """Compile librs_amd.so in-tree (hipcc --offload-arch=gfx950)."""
    import subprocess
    if force:
        subprocess.check_call(["make", "-s", "-C", HERE, "clean"])
    subprocess.check_call(["make", "-s", "-j8", "-C", HERE])


if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {HERE}` (no CPU fallback exists)")

_lib = ctypes.CDLL(LIB_PATH)

P = ctypes.c_void_p
u8, u16, u32, u64, i32, i64 = (ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_int32, ctypes.c_int64)


class SymbolT(ctypes.Structure):  # include/memory/symbol.h
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8))]


class SymbolSeqT(ctypes.Structure):  # include/memory/seq.h
    _fields_ = [("length", ctypes.c_size_t), ("symbol_size", ctypes.c_size_t),
                ("symbols", ctypes.POINTER(ctypes.POINTER(SymbolT)))]


def _sig(name, restype, *argtypes):
    f = getattr(_lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


_sig("rs_create", P)
_sig("rs_destroy", None, P)
_sig("seq_create", ctypes.POINTER(SymbolSeqT), ctypes.c_size_t, ctypes.c_size_t)
_sig("seq_destroy", None, ctypes.POINTER(SymbolSeqT))
_sig("rs_generate_repair_symbols", ctypes.c_int, P, ctypes.POINTER(SymbolSeqT), ctypes.POINTER(SymbolSeqT))
_sig("rs_restore_symbols", ctypes.c_int, P, u16, u16, ctypes.POINTER(SymbolSeqT), P, u16)
_sig("rsg_codec_create", ctypes.c_int, ctypes.c_int, u16, u16, ctypes.POINTER(P))
_sig("rsg_codec_destroy", None, P)
_sig("rsg_codec_subfield", ctypes.c_int, P)
_sig("rsg_codec_trim", ctypes.c_int, P)
_sig("rsg_set_option", ctypes.c_int, P, ctypes.c_char_p, i64)
_sig("rsg_last_kernel", ctypes.c_char_p, P)
_sig("rsg_last_work", ctypes.c_int, P, P, P)
_sig("rsg_encode", ctypes.c_int, P, P, u64, u64, P, u64, u64, u64, u64, P)
_sig("rsg_decode", ctypes.c_int, P, P, u64, u64, u64, u64, P, u16, P)
_sig("rsg_decode_batch", ctypes.c_int, P, P, u64, u64, u64, u64, P, P)
_sig("rsg_encode_host", ctypes.c_int, P, P, u64, u64, P, u64, u64, u64, u64)
_sig("rsg_decode_host", ctypes.c_int, P, P, u64, u64, u64, u64, P, u16)
_sig("rsg_fill_info", ctypes.c_int, P, u64, u64, u64, u16, u64, u64, u64, P)
_sig("rsg_fingerprint", ctypes.c_int, P, u64, u64, u64, u32, u32, u64, P, P)
_sig("rsg_coding_matrix", ctypes.c_int, u16, u16, P, u16, P, P, P, P, P)
_sig("rsg_jit_precompile", ctypes.c_int, u16, u16, P, u16)
_sig("rsg_gamma_tables", ctypes.c_int, P, P, P)
_sig("rsg_route_dump", ctypes.c_int, u16, u16, P, u16, P, P, P, P, P, P)
_sig("rsg_route_dump_t", ctypes.c_int, u16, u16, P, u16, P, P, P, P, P)
_sig("rsg_bs16_dump", ctypes.c_int, u16, u16, P, u16, P, P, P, P)
_sig("rsg_symbol_registered", ctypes.c_int, P)


class SymbolStatsT(ctypes.Structure):  # include/rs_amd/rsg.h rsg_symbol_stats_t
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "live", "live_registered", "idle_blocks", "idle_bytes", "idle_reuses", "registrations",
        "register_failures", "unregistrations", "unregister_failures", "retired_blocks", "stuck_blocks",
        "stuck_bytes", "pinned_bytes")]


class SymbolOpT(ctypes.Structure):  # include/rs_amd/rsg.h rsg_symbol_op_t
    _fields_ = [("a", P), ("b", P), ("coef", u16), ("op", u16), ("reserved", u32)]


OP_ADD, OP_MUL, OP_MADD = 0, 1, 2  # RSG_OP_*

_sig("rsg_symbol_stats", ctypes.c_int, ctypes.POINTER(SymbolStatsT))
_sig("rsg_symbol_ops", ctypes.c_int, ctypes.c_int, ctypes.POINTER(SymbolOpT), u64, u64, P)
_sig("rsg_symbol_pool_cap", i64, i64)
_sig("rsg_version", ctypes.c_char_p)
_sig("rsg_check_enabled", ctypes.c_int)
_sig("rsg_xj_fixed_precompile", ctypes.c_int, u16, u16, ctypes.c_int)
_sig("rsg_xj_fixed_source", ctypes.c_int, u16, u16, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
     ctypes.POINTER(ctypes.c_size_t))
_sig("gf_create", P)
_sig("gf_destroy", None, P)
_sig("gf_mul_ee", u16, P, u16, u16)
_sig("gf_div_ee", u16, P, u16, u16)
_sig("gf_get_normal_repr", u16, P, u8, u16)
_sig("gf_get_normal_basis_element", u16, P, u8, u8)
_sig("gf_add", None, P, P, ctypes.c_size_t)
_sig("gf_mul", None, P, P, u16, ctypes.c_size_t)
_sig("gf_madd", None, P, P, u16, P, ctypes.c_size_t)
_sig("fft_transform", None, P, ctypes.POINTER(SymbolSeqT), P, ctypes.POINTER(SymbolSeqT))
_sig("fft_transform_cycl", ctypes.c_int, P, ctypes.POINTER(SymbolSeqT), P, ctypes.POINTER(SymbolSeqT))
_sig("fft_partial_transform", None, P, ctypes.POINTER(SymbolSeqT), P, ctypes.POINTER(SymbolSeqT))
_sig("fft_partial_transform_cycl", ctypes.c_int, P, ctypes.POINTER(SymbolSeqT), P, u16, ctypes.POINTER(SymbolSeqT))
_sig("cc_create", P)
_sig("cc_destroy", None, P)
_sig("cc_get_coset_size", u8, u16)
_sig("cc_estimate_cosets_cnt", None, u16, u16, P, P)
_sig("cc_select_cosets", None, P, u16, u16, P, u16, P, P, u16, P)
_sig("cc_cosets_to_positions", None, P, u16, P, u16)

lib = _lib


def _np_ptr(a):
    return a.ctypes.data_as(P) if a is not None else None


def version():
    return _lib.rsg_version().decode()


# ------------------------------------------------------------------------------ host-only helpers
def coding_matrix(k, r, is_erased=None):
    """(matrix[rows, cols] uint16, in_slots, out_slots) exactly as the GPU engine applies them."""
    er = None if is_erased is None else np.ascontiguousarray(is_erased, dtype=np.bool_)
    t = 0 if er is None else int(er.sum())
    rows, cols = u32(), u32()
    rc = _lib.rsg_coding_matrix(k, r, _np_ptr(er), t, None, ctypes.byref(rows), ctypes.byref(cols), None, None)
    if rc:
        raise RSError(rc, "rsg_coding_matrix")
    M = np.zeros((rows.value, cols.value), np.uint16)
    ins = np.zeros(cols.value, np.int32)
    outs = np.zeros(rows.value, np.int32)
    rc = _lib.rsg_coding_matrix(k, r, _np_ptr(er), t, _np_ptr(M), None, None, _np_ptr(ins), _np_ptr(outs))
    if rc:
        raise RSError(rc, "rsg_coding_matrix")
    return M, ins, outs


def route_dump(k, r, is_erased=None):
    """The GF(2^16) syndrome route of the encode / decode matrix (host only): dict with D, groups
    [ngroups][16] (ngroups even), rec [ntiles][ngroups + 2][4][16] (bytes), fin [ntiles][fin_stride],
    fin_off [ntiles][5], m2 [R][D]."""
    er = None if is_erased is None else np.ascontiguousarray(is_erased, dtype=np.bool_)
    t = 0 if er is None else int(er.sum())
    info = np.zeros(5, np.int32)
    rc = _lib.rsg_route_dump(k, r, _np_ptr(er), t, _np_ptr(info), None, None, None, None, None)
    if rc:
        raise RSError(rc, "rsg_route_dump")
    D, ng, nt, fs, R = (int(v) for v in info)
    groups = np.zeros((ng, 16), np.int32)
    rec = np.zeros((nt, ng + 2, 4, 16), np.uint8)
    fin = np.zeros((nt, fs), np.int32)
    fin_off = np.zeros((nt, 5), np.int32)
    m2 = np.zeros((R, D), np.uint16)
    rc = _lib.rsg_route_dump(k, r, _np_ptr(er), t, None, _np_ptr(groups), _np_ptr(rec), _np_ptr(fin), _np_ptr(fin_off),
                             _np_ptr(m2))
    if rc:
        raise RSError(rc, "rsg_route_dump")
    return dict(D=D, groups=groups, rec=rec, fin=fin, fin_off=fin_off, m2=m2)


def route_dump_t(k, r, is_erased=None):
    """k_cs16t's side of the syndrome route plan (host only): dict with cw, rec [ntiles][ngroups + 2][4 cw]
    block offsets, fin [ntiles][fin_stride], fin_off [ntiles][cw + 1], blocks [(4c + n) * 16 + v] offsets."""
    er = None if is_erased is None else np.ascontiguousarray(is_erased, dtype=np.bool_)
    t = 0 if er is None else int(er.sum())
    info = np.zeros(4, np.int32)
    rc = _lib.rsg_route_dump_t(k, r, _np_ptr(er), t, _np_ptr(info), None, None, None, None)
    if rc:
        raise RSError(rc, "rsg_route_dump_t")
    cw, nt, fs, nblk = (int(v) for v in info)
    ng = route_dump(k, r, is_erased)["groups"].shape[0]
    rec = np.zeros((nt, ng + 2, 4 * cw), np.uint32)
    fin = np.zeros((nt, fs), np.int32)
    fin_off = np.zeros((nt, cw + 1), np.int32)
    blocks = np.zeros(nblk, np.uint32)
    rc = _lib.rsg_route_dump_t(k, r, _np_ptr(er), t, None, _np_ptr(rec), _np_ptr(fin), _np_ptr(fin_off), _np_ptr(blocks))
    if rc:
        raise RSError(rc, "rsg_route_dump_t")
    return dict(cw=cw, rec=rec, fin=fin, fin_off=fin_off, blocks=blocks)


def symbol_registered(arr):
    """1 / 0: a symbol_create buffer (>= 16 KiB) is / is not yet page-locked for the per-call path; -1: other."""
    return int(_lib.rsg_symbol_registered(ctypes.c_void_p(arr.ctypes.data)))


def symbol_stats():
    """Counters of the library-allocated symbol pages (rsg_symbol_stats) as a dict."""
    st = SymbolStatsT()
    rc = _lib.rsg_symbol_stats(ctypes.byref(st))
    if rc:
        raise RSError(rc, "rsg_symbol_stats")
    return {n: int(getattr(st, n)) for n, _ in SymbolStatsT._fields_}


def symbol_pool_cap(nbytes=-1):
    """Sets the idle pool's cap (bytes; < 0 queries) and returns the previous one."""
    return int(_lib.rsg_symbol_pool_cap(int(nbytes)))


def bs16_dump(k, r, is_erased=None):
    """The k_bs16 second stage of the GF(2^16) route (host only), or None when it does not apply: dict
    with D, d (Frobenius step of the row orbits), rec [ntiles][ngroups + 2][4][64] (bytes), fin
    [ntiles][fin_stride], fin_off [ntiles][5]."""
    er = None if is_erased is None else np.ascontiguousarray(is_erased, dtype=np.bool_)
    t = 0 if er is None else int(er.sum())
    info = np.zeros(6, np.int32)
    rc = _lib.rsg_bs16_dump(k, r, _np_ptr(er), t, _np_ptr(info), None, None, None)
    if rc:
        raise RSError(rc, "rsg_bs16_dump")
    ok, D, ng, nt, fs, d = (int(v) for v in info)
    if not ok:
        return None
    rec = np.zeros((nt, ng + 2, 4, 64), np.uint8)
    fin = np.zeros((nt, fs), np.int32)
    fin_off = np.zeros((nt, 5), np.int32)
    rc = _lib.rsg_bs16_dump(k, r, _np_ptr(er), t, None, _np_ptr(rec), _np_ptr(fin), _np_ptr(fin_off))
    if rc:
        raise RSError(rc, "rsg_bs16_dump")
    return dict(D=D, d=d, ngroups=ng, rec=rec, fin=fin, fin_off=fin_off)


def gamma_tables():
    lbyte = np.zeros((2, 256), np.uint16)
    ibyte = np.zeros((2, 256), np.uint16)
    red = np.zeros(1, np.uint8)
    _lib.rsg_gamma_tables(_np_ptr(lbyte), _np_ptr(ibyte), _np_ptr(red))
    return lbyte, ibyte, int(red[0])


def jit_precompile(k, r, is_erased=None):
    er = None if is_erased is None else np.ascontiguousarray(is_erased, dtype=np.bool_)
    t = 0 if er is None else int(er.sum())
    rc = _lib.rsg_jit_precompile(k, r, _np_ptr(er), t)
    if rc:
        raise RSError(rc, "rsg_jit_precompile")


def bench_pattern(k, r):
    """t = r erasures of information symbols at i * (k // r)."""
    er = np.zeros(k + r, np.bool_)
    step = max(k // r, 1) if r else 1
    er[[i * step for i in range(r)]] = True
    return er


# ------------------------------------------------------------------------------ drop-in mirror
class _SeqBuf:
    """symbol_seq_t view over a list of numpy uint8 arrays (kept alive by this object)."""

    def __init__(self, arrays, symbol_size):
        self.arrays = arrays
        self.syms = (SymbolT * max(len(arrays), 1))()
        for i, a in enumerate(arrays):
            assert a.dtype == np.uint8 and a.flags.c_contiguous and a.size >= symbol_size
            self.syms[i].data = a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        self.ptrs = (ctypes.POINTER(SymbolT) * max(len(arrays), 1))()
        for i in range(len(arrays)):
            self.ptrs[i] = ctypes.pointer(self.syms[i])
        self.seq = SymbolSeqT(len(arrays), symbol_size, self.ptrs)


_live_seqs = weakref.WeakSet()


@atexit.register
def _close_live_seqs():
    # page-locked sequences must be released while the HIP runtime is still up (before its static
    # destructors run at process exit), not whenever the garbage collector reaches them
    for q in list(_live_seqs):
        q.close()


class Seq:
    """A library-allocated symbol_seq_t (seq_create, reference include/memory/seq.h). The symbols
    live in page-locked memory (own block from 1 MiB, slab share below), which
    rs_generate_repair_symbols / rs_restore_symbols use in place (zero-copy launches or DMA).
    symbols[i] is a numpy view of symbol i."""

    def __init__(self, length, symbol_size):
        self._p = _lib.seq_create(length, symbol_size)
        if not self._p:
            raise MemoryError("seq_create")
        _live_seqs.add(self)
        self.length, self.symbol_size = length, symbol_size
        q = self._p.contents
        self.symbols = [np.ctypeslib.as_array(q.symbols[i].contents.data, (symbol_size,)) for i in range(length)]

    def view(self, start, count):
        """symbol_seq_t over symbols [start, start + count) (shares the symbol pointers)."""
        q = self._p.contents
        base = ctypes.cast(q.symbols, ctypes.c_void_p).value + start * ctypes.sizeof(ctypes.c_void_p)
        return SymbolSeqT(count, self.symbol_size, ctypes.cast(base, ctypes.POINTER(ctypes.POINTER(SymbolT))))

    def close(self):
        if self._p:
            self.symbols = []
            _lib.seq_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()


class RS:
    """Mirror of the reference context API (reference include/rs/reed_solomon.h:44-74)."""

    def __init__(self):
        self._h = _lib.rs_create()
        if not self._h:
            raise RSError(RS_ERR_DEVICE, "rs_create (no usable GPU?)")

    def close(self):
        if self._h:
            _lib.rs_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def generate_repair_symbols(self, inf_symbols, rep_symbols):
        """inf_symbols: k host symbols, rep_symbols: r host symbols (written); or a Seq of k + r
        symbols as inf_symbols with rep_symbols = r. Returns the C rc."""
        if isinstance(inf_symbols, Seq):
            q, r = inf_symbols, int(rep_symbols)
            a, b = q.view(0, q.length - r), q.view(q.length - r, r)
            return _lib.rs_generate_repair_symbols(self._h, ctypes.byref(a), ctypes.byref(b))
        S = inf_symbols[0].size if len(inf_symbols) else rep_symbols[0].size
        a, b = _SeqBuf(list(inf_symbols), S), _SeqBuf(list(rep_symbols), S)
        return _lib.rs_generate_repair_symbols(self._h, ctypes.byref(a.seq), ctypes.byref(b.seq))

    def restore_symbols(self, k, r, rcv_symbols, is_erased, t):
        """rcv_symbols: k + r host symbols (or a Seq), erased ones zero; restored in place. Returns the C rc."""
        if isinstance(rcv_symbols, Seq):
            er = np.ascontiguousarray(is_erased, dtype=np.bool_)
            a = rcv_symbols.view(0, rcv_symbols.length)
            return _lib.rs_restore_symbols(self._h, k, r, ctypes.byref(a), _np_ptr(er), t)
        S = rcv_symbols[0].size
        a = _SeqBuf(list(rcv_symbols), S)
        er = np.ascontiguousarray(is_erased, dtype=np.bool_)
        return _lib.rs_restore_symbols(self._h, k, r, ctypes.byref(a.seq), _np_ptr(er), t)


# ------------------------------------------------------------------------------ symbol ops, transforms
class CosetT(ctypes.Structure):  # include/rs/cyclotomic_coset.h coset_t
    _fields_ = [("leader", ctypes.c_uint16), ("size", ctypes.c_uint8)]


def _u8(a):
    assert a.dtype == np.uint8 and a.flags.c_contiguous, "symbols must be C-contiguous uint8 arrays"
    return a


def symbol_add(a, b):
    """a ^= b in place (gf_add, reference include/rs/gf65536.h:146); numpy uint8 arrays of equal size."""
    _lib.gf_add(_np_ptr(_u8(a)), _np_ptr(_u8(b)), a.size)


def symbol_mul(a, coef, gf=None):
    """a = coef * a in place (gf_mul, reference :156)."""
    _lib.gf_mul(gf, _np_ptr(_u8(a)), coef, a.size)


def symbol_madd(a, coef, b, gf=None):
    """a ^= coef * b in place (gf_madd, reference :167)."""
    _lib.gf_madd(gf, _np_ptr(_u8(a)), coef, _np_ptr(_u8(b)), a.size)


def fft(kind, f, res, arg, gf=None):
    """Reference rs/fft.h transforms on lists of host symbols (numpy uint8). kind: "transform" /
    "transform_cycl" (arg = positions, uint16), "partial" (arg = components, uint16),
    "partial_cycl" (arg = [(leader, size), ...]). Writes res in place; returns the C rc (0 for the void
    entry points)."""
    S = (f[0] if len(f) else res[0]).size
    a, b = _SeqBuf([_u8(x) for x in f], S), _SeqBuf([_u8(x) for x in res], S)
    if kind == "partial_cycl":
        cs = (CosetT * max(len(arg), 1))(*[CosetT(int(l), int(m)) for l, m in arg])
        return _lib.fft_partial_transform_cycl(gf, ctypes.byref(a.seq), cs, len(arg), ctypes.byref(b.seq))
    v = np.ascontiguousarray(arg, dtype=np.uint16)
    fn = {"transform": _lib.fft_transform, "transform_cycl": _lib.fft_transform_cycl,
          "partial": _lib.fft_partial_transform}[kind]
    rc = fn(gf, ctypes.byref(a.seq), _np_ptr(v), ctypes.byref(b.seq))
    return 0 if rc is None else rc


# numpy layout of rsg_symbol_op_t (a, b, coef, op, reserved: 24 bytes)
SYMBOL_OP_DTYPE = np.dtype([("a", "<u8"), ("b", "<u8"), ("coef", "<u2"), ("op", "<u2"), ("reserved", "<u4")])
assert SYMBOL_OP_DTYPE.itemsize == ctypes.sizeof(SymbolOpT)


def symbol_op_array(ops):
    """rsg_symbol_op_t array from a sequence of (op, a, b, coef) tuples (a / b device addresses as ints, b
    ignored for OP_MUL), or a SYMBOL_OP_DTYPE array as it is."""
    if isinstance(ops, np.ndarray) and ops.dtype == SYMBOL_OP_DTYPE:
        return np.ascontiguousarray(ops)
    t = np.array([(int(o), int(a), int(b or 0), int(c)) for o, a, b, c in ops], dtype=np.uint64).reshape(-1, 4)
    arr = np.zeros(len(t), SYMBOL_OP_DTYPE)
    arr["op"], arr["a"], arr["b"], arr["coef"] = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    return arr


def symbol_ops(ops, symbol_size, device=0, stream=None, check=True):
    """Batched gf_add / gf_mul / gf_madd on device-accessible symbols (rsg_symbol_ops): `ops` is a sequence
    of (op, a, b, coef) with op in OP_ADD / OP_MUL / OP_MADD, or a SYMBOL_OP_DTYPE array. Ops on one target
    apply in order; asynchronous on `stream`. Returns the C rc."""
    arr = symbol_op_array(ops)
    rc = _lib.rsg_symbol_ops(device, arr.ctypes.data_as(ctypes.POINTER(SymbolOpT)), len(arr), symbol_size,
                             _stream_ptr(stream))
    if check and rc:
        raise RSError(rc, "rsg_symbol_ops")
    return rc


# ------------------------------------------------------------------------------ device engine
def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return P(stream.cuda_stream) if hasattr(stream, "cuda_stream") else P(stream)


class Codec:
    """Batched (k, r) engine on one GPU. Buffers are torch uint8 CUDA tensors (or raw pointers)."""

    def __init__(self, k, r, device=0, jit=None, m8_mode=None, xj=None, batch_plans=None):
        """jit: None = library default (2), 0/False = generic kernels only, 1/True = specialise every
        eligible matrix, 2 = encode matrix + decode matrices from their second use.
        xj: specialised kernel family, None = library default (1 = bit-plane XOR kernels, rs_xj.hpp),
        0 = nibble-table rs_v1jit kernels.
        batch_plans (decode_batch): None = library default (2 = decode matrices built on the device
        when a batch has more than 16 distinct patterns), 0 = host plans per pattern, 1 = device."""
        self.k, self.r, self.device = k, r, device
        h = P()
        rc = _lib.rsg_codec_create(device, k, r, ctypes.byref(h))
        if rc:
            raise RSError(rc, f"rsg_codec_create({k}, {r})")
        self._h = h
        if jit is not None:
            self.set_option("jit", int(jit))
        if batch_plans is not None:
            self.set_option("batch_plans", int(batch_plans))
        if m8_mode is not None:
            self.set_option("m8_mode", m8_mode)
        if xj is not None:
            self.set_option("xj", int(xj))

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:  # _lib is None during interpreter shutdown
            _lib.rsg_codec_destroy(self._h)
        self._h = None

    def __del__(self):
        self.close()

    @property
    def subfield(self):
        return _lib.rsg_codec_subfield(self._h)

    @property
    def last_kernel(self):
        return _lib.rsg_last_kernel(self._h).decode()

    @property
    def last_work(self):
        """(VALU, SALU) wave-instructions of the hand-scheduled GF(2^16) kernels in the last call."""
        v, s_ = u64(), u64()
        _lib.rsg_last_work(self._h, ctypes.byref(v), ctypes.byref(s_))
        return v.value, s_.value

    def set_option(self, name, value):
        rc = _lib.rsg_set_option(self._h, name.encode(), int(value))
        if rc:
            raise RSError(rc, f"rsg_set_option({name})")

    def trim(self):
        """Frees the codec's grow-only device scratch after its outstanding work (rsg_codec_trim)."""
        rc = _lib.rsg_codec_trim(self._h)
        if rc:
            raise RSError(rc, "rsg_codec_trim")

    def encode(self, stripes, n_stripes=None, symbol_size=None, stream=None, check=True):
        """Repair symbols of `stripes` ([n, k + r, S] uint8, contiguous, on this device), in place."""
        n, nsym, S = stripes.shape
        assert nsym == self.k + self.r and stripes.is_contiguous()
        base = stripes.data_ptr()
        rc = _lib.rsg_encode(self._h, P(base), nsym * S, S, P(base + self.k * S), nsym * S, S,
                             n if n_stripes is None else n_stripes, S if symbol_size is None else symbol_size,
                             _stream_ptr(stream))
        if check and rc:
            raise RSError(rc, "rsg_encode")
        return rc

    def decode(self, stripes, is_erased, stream=None, check=True):
        """Restore erased information symbols of `stripes` ([n, k + r, S]) in place."""
        n, nsym, S = stripes.shape
        assert nsym == self.k + self.r and stripes.is_contiguous()
        er = np.ascontiguousarray(is_erased, dtype=np.bool_)
        rc = _lib.rsg_decode(self._h, P(stripes.data_ptr()), nsym * S, S, n, S, _np_ptr(er), int(er.sum()),
                             _stream_ptr(stream))
        if check and rc not in (0,):
            raise RSError(rc, "rsg_decode")
        return rc

    def decode_batch(self, stripes, patterns, stream=None, check=True):
        """Per-stripe erasure patterns: patterns [n, k + r] bool (host); restores in place."""
        n, nsym, S = stripes.shape
        assert nsym == self.k + self.r and stripes.is_contiguous()
        er = np.ascontiguousarray(patterns, dtype=np.bool_)
        assert er.shape == (n, nsym)
        rc = _lib.rsg_decode_batch(self._h, P(stripes.data_ptr()), nsym * S, S, n, S, _np_ptr(er),
                                   _stream_ptr(stream))
        if check and rc:
            raise RSError(rc, "rsg_decode_batch")
        return rc

    @staticmethod
    def _host_ptr(stripes):
        """Address of a C-contiguous uint8 host array (numpy or CPU tensor): the host batch calls derive
        their byte strides from the shape alone."""
        if hasattr(stripes, "data_ptr"):
            import torch
            assert stripes.dtype == torch.uint8 and stripes.is_contiguous() and not stripes.is_cuda
            return stripes.data_ptr()
        assert stripes.dtype == np.uint8 and stripes.flags.c_contiguous
        return stripes.ctypes.data

    def encode_host(self, stripes, check=True):
        """Stripes in HOST memory: a [n, k + r, S] uint8 array (numpy or a CPU tensor, pinned for PCIe
        rate); writes the repair symbols in place (rsg_encode_host, pipelined, synchronous)."""
        n, nsym, S = stripes.shape
        assert nsym == self.k + self.r
        ptr = self._host_ptr(stripes)
        rc = _lib.rsg_encode_host(self._h, P(ptr), nsym * S, S, P(ptr + self.k * S), nsym * S, S, n, S)
        if check and rc:
            raise RSError(rc, "rsg_encode_host")
        return rc

    def decode_host(self, stripes, is_erased, check=True):
        """Restores erased information symbols of host-memory stripes in place (rsg_decode_host)."""
        n, nsym, S = stripes.shape
        er = np.ascontiguousarray(is_erased, dtype=np.bool_)
        assert nsym == self.k + self.r
        ptr = self._host_ptr(stripes)
        rc = _lib.rsg_decode_host(self._h, P(ptr), nsym * S, S, n, S, _np_ptr(er), int(er.sum()))
        if check and rc:
            raise RSError(rc, "rsg_decode_host")
        return rc

    def encode_raw(self, d_info, info_stripe, info_sym, d_rep, rep_stripe, rep_sym, n, S, stream):
        return _lib.rsg_encode(self._h, P(d_info), info_stripe, info_sym, P(d_rep), rep_stripe, rep_sym, n, S,
                               _stream_ptr(stream))

    def decode_raw(self, d_rcv, stripe_stride, sym_stride, n, S, is_erased, stream):
        er = np.ascontiguousarray(is_erased, dtype=np.bool_)
        return _lib.rsg_decode(self._h, P(d_rcv), stripe_stride, sym_stride, n, S, _np_ptr(er), int(er.sum()),
                               _stream_ptr(stream))


def fill_info(stripes, k, seed, stripe0=0, stream=None):
    """Counter-based synthetic information symbols (same bytes as tests/_util.py:gen_info)."""
    n, nsym, S = stripes.shape
    rc = _lib.rsg_fill_info(P(stripes.data_ptr()), nsym * S, S, S, k, stripe0, n, seed, _stream_ptr(stream))
    if rc:
        raise RSError(rc, "rsg_fill_info")


def fingerprint(stripes, sym0, nsym, out, stream=None):
    """Per-stripe 64-bit fingerprint of symbols [sym0, sym0 + nsym) into `out` (int64 CUDA tensor [n])."""
    n, total, S = stripes.shape
    rc = _lib.rsg_fingerprint(P(stripes.data_ptr()), total * S, S, S, sym0, nsym, n, P(out.data_ptr()),
                              _stream_ptr(stream))
    if rc:
        raise RSError(rc, "rsg_fingerprint")
