#!/usr/bin/env python3
"""Device-resident Reed-Solomon encode + decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2] at N=1, configs[3] across N GPUs): k=128, r=32, 64 KiB symbols,
8192 stripes per GPU resident in HBM ([stripe][symbol][bytes], 80 GiB per GPU). One step = encode
every stripe (read k, write r symbols) + decode every stripe with t = r erased information symbols
(read the k survivors, write the t restored symbols), in place through the C ABI.
Byte accounting: encode (k + r) * S, decode (k + t) * S per stripe.

Multi-GPU: one process per GPU (torchrun), stripes partitioned, no data-path collective; the timed
region is bracketed by barriers and the max time over ranks is reported (weak scaling).

Also reported: the dominant kernel's roofline fraction (HIP-event timing of each launch on the
stream it runs on), and the CPU baseline -- the reference src/rs built from source
(oracle/_ref/librs_ref.so) or, if absent, the clean-room oracle -- timed on this host's cores on a
bounded sample of the same workload.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "reed-solomon_amd"))
import rs_amd  # noqa: E402  (raises if librs_amd.so is missing: no fallback)
import rs_dist  # noqa: E402
from srchash import kernel_src_hash  # noqa: E402


HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TRAFFIC_JSON = os.path.join(REPO, "profiles", "traffic.json")  # scripts/traffic.py output


def measured_traffic(kernel, cfg):
    """HBM bytes per launch of `kernel` measured with rocprofv3 PMC counters on this configuration
    (profiles/traffic.json, written by scripts/traffic.py), or None when no measurement matches: the
    exact kernel name for JIT kernels (content-addressed), name + source hash for compiled ones."""
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("config") != cfg:
        return None
    if "[" in str(kernel):  # JIT kernel: its name carries the hash of its generated source
        if t.get("bench_kernel") != kernel:
            return None
    elif t.get("bench_kernel") != kernel or t.get("src_hash") != kernel_src_hash(kernel):
        return None
    return int(t["traffic_bytes"])
SEED = 0x5EED


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--r", type=int, default=32)
    ap.add_argument("--symbol", type=int, default=65536)
    ap.add_argument("--stripes", type=int, default=8192, help="stripes per GPU")
    ap.add_argument("--kernel", default="auto", choices=["auto", "jit", "v1jit", "v1", "idx", "table", "mask", "m16c", "m16p"],
                    help="auto = library default policy (matrix-specialised kernels, generic fallback)")
    ap.add_argument("--cpu-stripes", type=int, default=128, help="CPU-baseline sample (stripes, resident)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget (passes repeat)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-only", action="store_true", help="skip verification/CPU legs (profilers)")
    ap.add_argument("--scatter", type=int, default=0, metavar="STRIPES",
                    help="N>1: also time an RCCL scatter of STRIPES stripes per rank from rank 0 (and the gather of "
                         "their repair symbols back), outside the timed region; reported as 'scatter'")
    return ap.parse_args()


# ------------------------------------------------------------------------------ CPU baseline
class _Sym(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8))]


class _Seq(ctypes.Structure):
    _fields_ = [("length", ctypes.c_size_t), ("symbol_size", ctypes.c_size_t),
                ("symbols", ctypes.POINTER(ctypes.POINTER(_Sym)))]


def _seq(buf, first, count, S):
    syms = (_Sym * count)()
    ptrs = (ctypes.POINTER(_Sym) * count)()
    for i in range(count):
        syms[i].data = buf[first + i].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        ptrs[i] = ctypes.pointer(syms[i])
    return _Seq(count, S, ptrs), (syms, ptrs)


def cpu_baseline(args, erased, gpu_sample):
    """Times encode + decode of `cpu_stripes` stripes on `cpu_threads` host threads.
    Returns (baseline dict, parity ok)."""
    k, r, S = args.k, args.r, args.symbol
    t = int(erased.sum())
    n = args.cpu_stripes
    ref_so = os.path.join(REPO, "oracle", "_ref", "librs_ref.so")
    kind = "reference" if os.path.exists(ref_so) else "port"
    stripes = np.zeros((n, k + r, S), np.uint8)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _util import gen_info, oracle
    for s in range(n):
        stripes[s, :k] = gen_info(SEED, s, k * S).reshape(k, S)

    if kind == "reference":
        lib = ctypes.CDLL(ref_so)
        lib.rs_create.restype = ctypes.c_void_p
        lib.rs_destroy.argtypes = [ctypes.c_void_p]
        lib.rs_generate_repair_symbols.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Seq), ctypes.POINTER(_Seq)]
        lib.rs_restore_symbols.argtypes = [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint16, ctypes.POINTER(_Seq),
                                           ctypes.c_void_p, ctypes.c_uint16]
        er = np.ascontiguousarray(erased, np.bool_)

        def work(lo, hi, dec, errs):
            rs = lib.rs_create()
            for s in range(lo, hi):
                buf = stripes[s]
                if not dec:
                    inf, keep1 = _seq(buf, 0, k, S)
                    rep, keep2 = _seq(buf, k, r, S)
                    errs.append(lib.rs_generate_repair_symbols(rs, ctypes.byref(inf), ctypes.byref(rep)))
                else:
                    rcv, keep = _seq(buf, 0, k + r, S)
                    errs.append(lib.rs_restore_symbols(rs, k, r, ctypes.byref(rcv), er.ctypes.data, t))
            lib.rs_destroy(rs)

        def run(dec, nt=None, cnt=n):
            nt = min(args.cpu_threads if nt is None else nt, cnt)
            errs, ths = [], []
            for i in range(nt):
                th = threading.Thread(target=work, args=(cnt * i // nt, cnt * (i + 1) // nt, dec, errs))
                ths.append(th)
            t0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            dt = time.perf_counter() - t0
            assert not any(errs), errs
            return dt
    else:
        o = oracle()
        er = np.ascontiguousarray(erased, np.bool_)

        def run(dec, nt=None, cnt=n):
            nt = args.cpu_threads if nt is None else nt
            t0 = time.perf_counter()
            if dec:
                rc = o.orc_decode_many(k, r, S, stripes.ctypes.data, cnt, er.ctypes.data, t, nt)
            else:
                rc = o.orc_encode_many(k, r, S, stripes.ctypes.data, cnt, nt)
            assert rc == 0
            return time.perf_counter() - t0

    # bounded sample: passes over the resident stripes repeat until the time budget is spent
    t_enc, p_enc = run(False), 1
    parity = all(np.array_equal(stripes[s], gpu_sample[s]) for s in range(min(len(gpu_sample), n)))
    while t_enc < args.cpu_seconds / 2:
        t_enc += run(False)
        p_enc += 1
    info = stripes[:, :k].copy()
    t_dec, p_dec = 0.0, 0
    while p_dec == 0 or t_dec < args.cpu_seconds / 2:
        stripes[:, erased] = 0  # the reference requires erased slots to be zero (untimed)
        t_dec += run(True)
        p_dec += 1
    parity = parity and np.array_equal(stripes[:, :k], info)
    bytes_total = n * ((k + r) * p_enc + (k + t) * p_dec) * S
    gbs = bytes_total / (t_enc + t_dec) / 1e9
    threads = min(args.cpu_threads, n)
    # single core, same code, a few stripes (all-core and single-core rates)
    c1 = min(n, 4)
    t1e, t1d = run(False, 1, c1), 0.0
    stripes[:c1, erased] = 0
    t1d = run(True, 1, c1)
    gbs1 = c1 * ((k + r) + (k + t)) * S / (t1e + t1d) / 1e9
    return dict(value=round(gbs, 4), unit="GB/s", cores=threads, kind=kind, single_core=round(gbs1, 4),
                sample=f"{n} resident stripes of k={k} r={r} S={S}: {p_enc} encode + {p_dec} decode (t={t}) "
                       f"passes, {threads} threads, {t_enc + t_dec:.1f} s; single_core: {c1} stripes, "
                       f"1 thread, {t1e + t1d:.1f} s"), parity


# ------------------------------------------------------------------- stripes from one rank
def scatter_leg(args, rank, world, dev):
    """Stripes that originate on rank 0 (--scatter STRIPES per rank): RCCL scatter of the information
    symbols to their owners (rs_dist.scatter_stripes, one P2P group, one xGMI link per peer) and the
    gather of the repair symbols back. Timed on its own (barrier-bracketed, max over ranks); never
    part of `value`."""
    k, r, S, m = args.k, args.r, args.symbol, args.scatter
    src = torch.empty((world * m if rank == 0 else 1, k, S), dtype=torch.uint8, device=dev)
    if rank == 0:
        src.random_(0, 256)
    info = torch.empty((m, k, S), dtype=torch.uint8, device=dev)
    rep = torch.randint(0, 256, (m, r, S), dtype=torch.uint8, device=dev)
    back = torch.empty((world * m if rank == 0 else 1, r, S), dtype=torch.uint8, device=dev)
    rs_dist.scatter_stripes(src, info)  # warm-up (communicator and P2P channel setup)
    with rs_dist.TimedRegion(dev) as t_sc:
        rs_dist.scatter_stripes(src, info)
    with rs_dist.TimedRegion(dev) as t_ga:
        rs_dist.gather_stripes(rep, back)
    moved_sc = (world - 1) * m * k * S
    moved_ga = (world - 1) * m * r * S
    ok = rank != 0 or torch.equal(info, src[:m])
    ok = rs_dist.max_over_ranks(0.0 if ok else 1.0, dev) == 0.0
    return {"stripes_per_rank": m, "scatter_GBps": round(moved_sc / t_sc.max_elapsed / 1e9, 1),
            "gather_GBps": round(moved_ga / t_ga.max_elapsed / 1e9, 1), "scatter_ms": round(t_sc.max_elapsed * 1e3, 3),
            "gather_ms": round(t_ga.max_elapsed * 1e3, 3), "check": "ok" if ok else "MISMATCH"}


# ------------------------------------------------------------------------------ main
def main():
    args = parse()
    rank, world, local = rs_dist.env()
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    k, r, S, n = args.k, args.r, args.symbol, args.stripes
    erased = rs_amd.bench_pattern(k, r)
    t = int(erased.sum())
    opts = {"auto": {}, "jit": dict(jit=1), "v1jit": dict(jit=1, xj=0), "v1": dict(jit=0, m8_mode=18), "idx": dict(jit=0, m8_mode=2),
            "table": dict(jit=0, m8_mode=0), "mask": dict(jit=0, m8_mode=1), "m16c": {}, "m16p": {}}[args.kernel]
    codec = rs_amd.Codec(k, r, device=local, **opts)
    if args.kernel in ("m16c", "m16p"):  # GF(2^16) codes: compiled kernel / asm timing ablation (wrong results)
        codec.set_option("m16_mode", 2 if args.kernel == "m16c" else 1)
    stripes = torch.empty((n, k + r, S), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    stripe0, _ = rs_dist.weak_shard(n, rank)  # this rank's global stripe ids: [stripe0, stripe0 + n)
    rs_amd.fill_info(stripes, k, SEED, stripe0=stripe0, stream=stream)
    # reference fingerprint of the generated information symbols (the timed loop must preserve them)
    fp_ref = torch.zeros(n, dtype=torch.int64, device=dev)
    if not args.profile_only:
        rs_amd.fingerprint(stripes, 0, k, fp_ref, stream=stream)

    # warmup (also compiles / loads the specialised kernels)
    for _ in range(args.warmup):
        codec.encode(stripes, stream=stream)
        codec.decode(stripes, erased, stream=stream)
    torch.cuda.synchronize()
    kern_enc = kern_dec = None

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    with rs_dist.TimedRegion(dev) as region:
        for i in range(args.steps):
            ev[i][0].record(stream)
            codec.encode(stripes, stream=stream)
            kern_enc = codec.last_kernel
            ev[i][1].record(stream)
            codec.decode(stripes, erased, stream=stream)
            kern_dec = codec.last_kernel
            ev[i][2].record(stream)
    elapsed = region.max_elapsed

    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    enc_bytes = n * (k + r) * S
    dec_bytes = n * (k + t) * S
    total_bytes = (enc_bytes + dec_bytes) * world * args.steps
    value = total_bytes / elapsed / 1e9

    # verification: restored information == generated information (fingerprints), sampled repair
    parity = "skipped"
    gpu_sample = np.zeros((0,), np.uint8)
    if not args.profile_only:
        # every timed step encoded and restored in place, so the information symbols must still be the
        # generated ones; then poison the erased slots, decode once more and check again
        fp0 = torch.zeros(n, dtype=torch.int64, device=dev)
        rs_amd.fingerprint(stripes, 0, k, fp0, stream=stream)
        stripes[:, torch.from_numpy(erased).to(dev)] = 0xA5  # poison the erased slots
        codec.decode(stripes, erased, stream=stream)
        fp1 = torch.zeros(n, dtype=torch.int64, device=dev)
        rs_amd.fingerprint(stripes, 0, k, fp1, stream=stream)
        torch.cuda.synchronize()
        good = torch.equal(fp0, fp_ref) and torch.equal(fp1, fp_ref)
        ok = rs_dist.max_over_ranks(0.0 if good else 1.0, dev) == 0.0  # any rank
        if rank == 0:
            gpu_sample = stripes[: args.cpu_stripes].cpu().numpy()
        parity = "roundtrip-ok" if ok else "ROUNDTRIP-MISMATCH"

    scatter = scatter_leg(args, rank, world, dev) if args.scatter > 0 and world > 1 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.profile_only:
        cpu, cpu_ok = cpu_baseline(args, erased, gpu_sample)
        parity += ",cpu-bitexact-ok" if cpu_ok else ",CPU-MISMATCH"

    # roofline of the dominant kernel (encode and decode move the same algorithmic bytes here)
    dom_ms, dom_bytes, dom_name = (enc_ms, enc_bytes, kern_enc) if enc_ms >= dec_ms else (dec_ms, dec_bytes, kern_dec)
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9
    traffic = measured_traffic(dom_name, f"k{k}_r{r}_S{S}_n{n}_t{t}")
    line = {
        "metric": "encode+decode GB/s (device-resident) at k/r/symbol_len; % HBM roofline",  # BASELINE.json
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16 (GF(2^16) words)",
        "data": "synthetic (counter-based splitmix64 stripes generated in HBM)",
        "config": {"workload": f"k={k} r={r} symbol={S}B stripes/gpu={n} decode t={t} (info erasures "
                               f"at i*{k // r})", "stripes_total": n * world, "parallelism": f"stripes x{world}",
                   "kernel": {"encode": kern_enc, "decode": kern_dec}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": dom_name, "kernel_ms": round(dom_ms, 3), "bytes_per_launch": dom_bytes},
        "encode_ms": round(enc_ms, 3),
        "decode_ms": round(dec_ms, 3),
        "cpu_baseline": cpu,
        "parity": parity,
    }
    if scatter is not None:
        line["scatter"] = scatter
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    if "MISMATCH" in parity:
        sys.exit(1)


if __name__ == "__main__":
    main()
