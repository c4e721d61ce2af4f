#!/usr/bin/env python3
"""Device-resident Reed-Solomon encode + decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2] at N=1, configs[3] across N GPUs): k=128, r=32, 64 KiB symbols,
8192 stripes per GPU resident in HBM ([stripe][symbol][bytes], 80 GiB per GPU). One step = encode
every stripe (read k, write r symbols) + decode every stripe with t = r erased information symbols
(read the k survivors, write the t restored symbols), in place through the C ABI.
Byte accounting: encode (k + r) * S, decode (k + t) * S per stripe.

Multi-GPU: one process per GPU, stripes partitioned, no data-path collective; the timed region is
bracketed by barriers and the max time over ranks is reported (weak scaling). `--gpus N` without a
torchrun environment spawns the N rank processes itself (before anything touches a GPU) and relays
rank 0's line; under torchrun, --gpus must equal WORLD_SIZE.

Also reported: the dominant kernel's roofline fraction (HIP-event timing of each launch on the
stream it runs on), and the CPU baseline -- the reference src/rs built from source
(oracle/_ref/librs_ref.so) on a pthread pool of this host's cores (oracle/cpu_baseline.c), or, if
that build is absent, the clean-room port, labelled as such -- on a bounded sample of the workload.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "reed-solomon_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TRAFFIC_JSON = os.path.join(REPO, "profiles", "traffic.json")  # scripts/traffic.py output
SEED = 0x5EED
METRIC = "encode+decode GB/s (device-resident) at k/r/symbol_len; % HBM roofline"  # BASELINE.json


def measured_traffic(kernel, cfg, with_source=False, leg=None):
    """HBM bytes per launch of `kernel` measured with rocprofv3 PMC counters on this configuration
    (profiles/traffic.json, written by scripts/traffic.py), or None when no measurement matches: the
    exact kernel name for JIT kernels (content-addressed), name + source hash for compiled ones.
    traffic.json holds one record per (kernel, config). The value is a lookup of an EARLIER rocprofv3
    run of the same kernel bytes, not a counter read in this run; `with_source` also returns where it
    came from. `leg` ("encode" / "decode") picks that leg's record when both legs run kernels of the same
    name (the GF(2^16) route: "cs16t+bs16" for both); the newest matching record wins."""
    from srchash import kernel_src_hash
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return (None, None) if with_source else None
    for rec in reversed(t.get("records", [t])):
        if rec.get("config") != cfg or rec.get("bench_kernel") != kernel:
            continue
        if leg is not None and rec.get("leg", leg) != leg:
            continue
        if "[" not in str(kernel) and rec.get("src_hash") != kernel_src_hash(kernel):
            continue
        src = (f"profiles/traffic.json (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE, separate passes, "
               f"{rec.get('measured', 'undated')}; earlier run of this exact kernel, not this run)")
        return (int(rec["traffic_bytes"]), src) if with_source else int(rec["traffic_bytes"])
    return (None, None) if with_source else None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps (default 100: ~4.4 s of back-to-back GPU work at C3, so utilisation samplers see it)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--r", type=int, default=32)
    ap.add_argument("--symbol", type=int, default=65536)
    ap.add_argument("--stripes", type=int, default=8192, help="stripes per GPU")
    ap.add_argument("--t", type=int, default=0,
                    help="decode erasures (information symbols at i * (k // t)); 0 = r, the bench pattern")
    ap.add_argument("--kernel", default="auto", choices=["auto", "jit", "v1jit", "v1", "idx", "table", "mask", "m16c"],
                    help="auto = library default policy (matrix-specialised kernels, generic fallback)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="codec option (rsg_set_option), e.g. m16_route=0; repeatable")
    ap.add_argument("--cpu-stripes", type=int, default=128, help="CPU-baseline sample (stripes, resident)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget (passes repeat)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra legs (N=1 only: host-memory path, per-stripe patterns, C2 / C5 configs)")
    ap.add_argument("--extras", default="end_to_end,per_stripe_decode,configs,symbol_ops",
                    help="comma list of extra legs to run after the headline (N=1, never part of `value`)")
    ap.add_argument("--ps-stripes", type=int, default=4096, help="per_stripe_decode leg: stripes, each its own pattern")
    ap.add_argument("--host-stripes", type=int, default=256, help="end_to_end leg: pinned host stripes")
    ap.add_argument("--cfg-stripes", type=int, default=1024, help="configs leg: stripes of C2 and C5")
    ap.add_argument("--profile-only", action="store_true", help="skip verification/CPU legs (profilers)")
    ap.add_argument("--scatter", type=int, default=0, metavar="STRIPES",
                    help="N>1: also time an RCCL scatter of STRIPES stripes per rank from rank 0 (and the gather of "
                         "their repair symbols back), outside the timed region; reported as 'scatter'")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks run the launch / barrier / max-over-ranks protocol with no coding work "
                         "(tests the multi-rank harness on CPU); the line says dry_run")
    ap.add_argument("--dry-fail-rank", type=int, default=-1,
                    help="dry run only: this rank exits with status 3 inside the timed region (launcher tests)")
    ap.add_argument("--dry-same-device", action="store_true",
                    help="dry run only: every rank reports the same device (duplicate-device check tests)")
    a = ap.parse_args(argv)
    if (a.dry_fail_rank >= 0 or a.dry_same_device) and not a.dry_run:
        ap.error("--dry-fail-rank / --dry-same-device need --dry-run")
    return a


# ------------------------------------------------------------------------------ rank launcher
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count(environ=None, kfd_nodes="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs a rank process started from here will see, counted WITHOUT loading HIP in this process:
    the GPU nodes of the KFD topology (nodes whose gpu_id is non-zero; CPU nodes have 0), cut down by
    ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (comma lists; an empty value
    hides every device). None when nothing is known (no topology and no visibility variable)."""
    environ = os.environ if environ is None else environ
    count = None
    try:
        ids = []
        for node in os.listdir(kfd_nodes):
            try:
                with open(os.path.join(kfd_nodes, node, "gpu_id")) as f:
                    ids.append(int(f.read().strip() or "0"))
            except (OSError, ValueError):
                continue
        count = sum(1 for g in ids if g != 0)
    except OSError:
        pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if var in environ:
            listed = [e for e in environ[var].split(",") if e.strip()]
            count = len(listed) if count is None else min(count, len(listed))
    return count


def spawn_ranks(args):
    """`--gpus N` outside torchrun: start N rank processes (this script, RANK/LOCAL_RANK/WORLD_SIZE set,
    rendezvous on 127.0.0.1) and wait for them. This process never loads HIP (the device count comes
    from the KFD topology, `visible_gpu_count`) and never replaces itself: the ranks are fresh child
    processes, each of which dies with this one (PR_SET_PDEATHSIG). Rank 0 prints the JSON line. A
    rank that fails stops the others; every child is reaped before this returns. Returns the exit code
    (the first failing rank's, else 0)."""
    import signal
    n = args.gpus
    if not args.dry_run:
        ndev = visible_gpu_count()
        if ndev is not None and n > ndev:
            print(f"bench.py: --gpus {n} but only {ndev} GPU(s) are visible", file=sys.stderr)
            return 2
    port = _free_port()

    def die_with_parent():  # runs in the child before exec (the parent holds no GPU state)
        try:
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except (OSError, AttributeError):
            pass

    procs = []
    for rank in range(n):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      preexec_fn=die_with_parent))
        print(f"bench.py: rank {rank} pid {procs[-1].pid}", file=sys.stderr, flush=True)

    def stop(live):
        for j in live:
            if procs[j].poll() is None:
                procs[j].terminate()
        deadline = time.time() + 20
        for j in live:
            try:
                procs[j].wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                procs[j].kill()
                procs[j].wait()

    def on_signal(signum, _frame):
        stop(range(n))
        sys.exit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    live = set(range(n))
    try:
        while live:
            for i in sorted(live):
                c = procs[i].poll()
                if c is None:
                    continue
                live.discard(i)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 1
                    print(f"bench.py: rank {i} exited with {c}; stopping the other ranks", file=sys.stderr)
                    stop(sorted(live))
                    live.clear()
            time.sleep(0.05)
    finally:
        stop(range(n))
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def device_identity(dev):
    """PCI address (domain:bus:device) and UUID of the rank's GPU (torch device properties)."""
    import torch
    p = torch.cuda.get_device_properties(dev)
    pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}"
    uuid = str(getattr(p, "uuid", ""))
    return {"pci_bus_id": pci, "uuid": uuid}


def check_distinct_devices(idents):
    """Fatal if two ranks run on the same device (same PCI address): a weak-scaling number would then
    count one GPU twice. Every rank calls this on the same gathered list, so all of them stop."""
    seen = {}
    for rank, ident in enumerate(idents):
        key = ident["pci_bus_id"]
        if key in seen:
            print(f"bench.py: ranks {seen[key]} and {rank} share device {key}", file=sys.stderr, flush=True)
            return False
        seen[key] = rank
    return True


# ------------------------------------------------------------------------------ CPU baseline
def cpu_cores():
    """(cores this process may run on, cgroup CPU quota in cores or None)."""
    avail = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2: "<quota> <period>" or "max <period>"
            q, p = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f1, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f2:
                q, p = int(f1.read()), int(f2.read())
                if q > 0:
                    quota = max(1, q // p)
        except (OSError, ValueError):
            pass
    return avail, quota


def port_calibration(k, r, S, gbs):
    """The port's speed relative to the reference (oracle/calibration.json, measured in the build container
    by scripts/calibrate_oracle.py: same C driver, one thread, identical inputs) and the reference-equivalent
    rate of this run's port baseline; None when the configuration was not calibrated."""
    try:
        with open(os.path.join(REPO, "oracle", "calibration.json")) as f:
            cal = json.load(f)
    except (OSError, ValueError):
        return None
    for row in cal.get("rows", []):
        if (row["k"], row["r"], row["S"]) == (k, r, S):
            x = float(row["port_over_ref"])
            # the port restates the reference's cost structure (64-bit XOR loop, word-wise madd through the
            # shifted pow table, per-symbol temporaries; oracle/rs_oracle.c), so it runs at the reference's
            # speed: within 1.0 +- 0.1 the timed port IS the reference-speed baseline; outside that band the
            # scaled value is only an estimate (the ratio was measured on another CPU, the build container)
            est = not 0.9 <= x <= 1.1
            return dict(port_over_reference=x, reference_equivalent_value=round(gbs * x, 4), estimate=est,
                        calibration_host=cal.get("host"),
                        source=f"oracle/calibration.json ({cal.get('measured')}, {cal.get('host')}): port "
                               f"{row['port_ms_per_stripe']} ms vs reference {row['ref_ms_per_stripe']} ms per stripe, "
                               f"bit-exact {row['bitexact']}")
    return None


def cpu_baseline(args, erased, gpu_sample):
    """Times encode + decode of `cpu_stripes` resident stripes with the reference CPU path on a pthread
    pool (oracle/cpu_baseline.c: one context per thread, views built before the clock). Returns
    (baseline dict, parity ok); `gpu_sample` None (dry run) skips the comparison with GPU output."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _util import gen_info
    k, r, S = args.k, args.r, args.symbol
    t = int(erased.sum())
    n = args.cpu_stripes
    ref_so = os.path.join(REPO, "oracle", "_ref", "librs_ref.so")
    port_so = os.path.join(REPO, "oracle", "librs_oracle.so")
    drv_so = os.path.join(REPO, "oracle", "libcpu_baseline.so")
    kind = "reference" if os.path.exists(ref_so) else "port"
    drv = ctypes.CDLL(drv_so)
    drv.cpub_run.restype = ctypes.c_int
    drv.cpub_run.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    avail, quota = cpu_cores()
    threads = args.cpu_threads or (min(avail, quota) if quota else avail)
    threads = max(1, min(threads, n))
    stripes = np.zeros((n, k + r, S), np.uint8)
    for s in range(n):
        stripes[s, :k] = gen_info(SEED, s, k * S).reshape(k, S)
    er = np.ascontiguousarray(erased, np.bool_)

    def run(op, passes, nt, cnt):
        sec = ctypes.c_double()
        rc = drv.cpub_run((ref_so if kind == "reference" else port_so).encode(), 0 if kind == "reference" else 1,
                          k, r, S, stripes.ctypes.data, cnt, er.ctypes.data, t, op, passes, nt, ctypes.byref(sec))
        if rc:
            raise RuntimeError(f"cpu baseline ({kind}) failed with {rc}")
        return sec.value

    # bounded sample: passes over the resident stripes, sized from the first pass to the time budget
    t_enc, p_enc = run(0, 1, threads, n), 1
    parity = gpu_sample is None or all(np.array_equal(stripes[s], gpu_sample[s])
                                       for s in range(min(len(gpu_sample), n)))
    more = int(max(0.0, args.cpu_seconds / 2 - t_enc) / max(t_enc, 1e-9))
    if more:
        t_enc += run(0, more, threads, n)
        p_enc += more
    info = stripes[:, :k].copy()
    t_dec, p_dec = run(1, 1, threads, n), 1
    more = int(max(0.0, args.cpu_seconds / 2 - t_dec) / max(t_dec, 1e-9))
    if more:
        t_dec += run(1, more, threads, n)
        p_dec += more
    parity = parity and np.array_equal(stripes[:, :k], info)
    gbs = n * ((k + r) * p_enc + (k + t) * p_dec) * S / (t_enc + t_dec) / 1e9
    # single core, same driver, a few stripes (all-core and single-core rates)
    c1 = min(n, 4)
    t1 = run(0, 1, 1, c1) + run(1, 1, 1, c1)
    gbs1 = c1 * ((k + r) + (k + t)) * S / t1 / 1e9
    label = kind if kind == "reference" else "port (oracle/_ref/librs_ref.so absent: clean-room restatement timed)"
    out = dict(value=round(gbs, 4), unit="GB/s", cores=threads, kind=kind, cores_available=avail, cpu_quota=quota,
               single_core=round(gbs1, 4))
    if kind == "port":
        out["calibration"] = port_calibration(k, r, S, gbs)
    return dict(out,
                sample=f"{label}: {n} resident stripes of k={k} r={r} S={S}, {p_enc} encode + {p_dec} decode (t={t}) "
                       f"passes on {threads} pthreads ({avail} cores available, quota {quota}), "
                       f"{t_enc + t_dec:.1f} s; single_core: {c1} stripes, 1 thread, {t1:.2f} s"), parity


def oracle_check_decode(k, r, restored, erased):
    """Checker for the extra legs (after their timed regions): the CPU oracle restores the erased
    information slots of `restored` (a host stripe [k + r][S] as the GPU left it) from its survivors;
    True when it writes exactly the GPU's bytes."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _util import oracle_decode
    inp = restored.copy()
    inp[erased] = 0  # the reference's contract: erased slots zero on entry (reed_solomon.h:64)
    return oracle_decode(k, r, inp, erased, int(erased.sum())) == 0 and np.array_equal(inp[:k], restored[:k])


def oracle_check_batch(k, r, host, erased, threads, decode=True):
    """Checker: re-encode every stripe of `host` ([n][k + r][S], as the GPU left it) with the CPU oracle
    and compare the repair symbols; with `decode`, also erase `erased` and restore with the oracle."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _util import oracle, ptr
    n, _, S = host.shape
    a = host.copy()
    a[:, k:] = 0
    ok = oracle().orc_encode_many(k, r, S, ptr(a), n, threads) == 0 and np.array_equal(a, host)
    if decode and ok:
        er = np.ascontiguousarray(erased, np.bool_)
        a[:, er] = 0
        ok = (oracle().orc_decode_many(k, r, S, ptr(a), n, ptr(er), int(er.sum()), threads) == 0
              and np.array_equal(a[:, :k], host[:, :k]))
    return ok


# ------------------------------------------------------------------ extra legs (N = 1; never `value`)
def per_stripe_leg(args, stripes, fp_ref, stream, dev):
    """Per-stripe erasure patterns (ref reed_solomon.c:443-559 decodes any pattern per call):
    the first `ps_stripes` resident headline stripes, each with its own t = r information-erasure pattern
    (all distinct), restored by ONE rsg_decode_batch call (device-built plans: masked fixed pass + per-stripe
    solve). Times calls with HIP events on the launch stream. Checks: every stripe's information symbols
    against the generated ones (fingerprints) and two sampled stripes bit for bit against the CPU oracle."""
    import torch
    import rs_amd
    k, r, S = args.k, args.r, args.symbol
    n = min(args.ps_stripes, stripes.shape[0])
    rng = np.random.default_rng(SEED)
    pats = np.zeros((n, k + r), np.bool_)
    pats[np.arange(n)[:, None], np.argsort(rng.random((n, k)), axis=1)[:, :r]] = True
    distinct = int(len(np.unique(pats, axis=0)))
    sub = stripes[:n]
    flat = sub.view(n * (k + r), S)
    erased_rows = torch.from_numpy(np.nonzero(pats.reshape(-1))[0]).to(dev)
    codec = rs_amd.Codec(k, r, device=dev.index)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    wall = []
    for i in range(1 + len(ev)):  # call 0: warm-up (plans scratch, masked fixed-pass kernel load)
        flat.index_fill_(0, erased_rows, 0)  # the reference's contract: erased slots zero on entry
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if i:
            ev[i - 1][0].record(stream)
        codec.decode_batch(sub, pats, stream=stream)
        if i:
            ev[i - 1][1].record(stream)
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    fp = torch.zeros(n, dtype=torch.int64, device=dev)
    rs_amd.fingerprint(sub, 0, k, fp, stream=stream)
    torch.cuda.synchronize()
    ok = bool(torch.equal(fp, fp_ref[:n]))
    sampled = [0, n - 1]
    for s in sampled:
        ok = ok and oracle_check_decode(k, r, sub[s].cpu().numpy(), pats[s])
    alg = n * (k + r) * S  # per stripe: k + r - t survivors read + t information symbols written
    return {"stripes": n, "distinct_patterns": distinct, "t": r, "pattern": "t = r information erasures per stripe, "
            "uniform random without replacement, a different set per stripe", "ms": round(ms, 3),
            "GBps": round(alg / ms / 1e6, 1), "wall_ms": round(float(np.median(wall[1:])) * 1e3, 3),
            "kernel": codec.last_kernel, "bytes": alg, "timing": f"HIP events on the launch stream, median of {len(ev)}",
            "parity": "ok" if ok else "MISMATCH",
            "check": f"all {n} stripes' information fingerprints + stripes {sampled} bit-exact vs the CPU oracle"}


def host_path_leg(args, stripes, erased, dev):
    """The path the reference's callers take (north star: starts and ends in host memory; PCIe-inclusive,
    never `value`): (a) rsg_encode_host / rsg_decode_host over `host_stripes` page-locked C3 stripes
    (pipelined H2D -> kernel -> D2H; decode moves survivors in and restored symbols out), synchronous calls
    timed by wall clock; (b) the reference API per call (rs_generate_repair_symbols / rs_restore_symbols,
    ref include/rs/reed_solomon.h:61,74, src/example.c:138,151) on seq_create stripes (page-locked arena).
    Checks: repair symbols equal the device-resident encode's, restored symbols equal the originals."""
    import torch
    import rs_amd
    k, r, S = args.k, args.r, args.symbol
    t = int(erased.sum())
    er_idx = torch.from_numpy(np.nonzero(erased)[0])
    n = min(args.host_stripes, stripes.shape[0])
    h = torch.empty((n, k + r, S), dtype=torch.uint8, pin_memory=True)
    h.copy_(stripes[:n])  # headline stripes: generated information + device-computed repair
    rep_ref = h[:, k:].clone()
    codec = rs_amd.Codec(k, r, device=dev.index)
    out = {}
    enc, dec = [], []
    for i in range(4):  # call 0 warms up (staging buffers, streams)
        h[:, k:] = 0
        t0 = time.perf_counter()
        codec.encode_host(h)
        enc.append(time.perf_counter() - t0)
    ok = bool(torch.equal(h[:, k:], rep_ref))
    saved = h[:, er_idx].clone()
    for i in range(4):
        h[:, er_idx] = 0
        t0 = time.perf_counter()
        codec.decode_host(h, erased)
        dec.append(time.perf_counter() - t0)
    ok = ok and bool(torch.equal(h[:, er_idx], saved))
    te, td = float(np.median(enc[1:])), float(np.median(dec[1:]))
    out["batch_host"] = {"stripes": n, "encode_GBps": round(n * (k + r) * S / te / 1e9, 2),
                         "decode_GBps": round(n * (k + t) * S / td / 1e9, 2), "encode_ms": round(te * 1e3, 3),
                         "decode_ms": round(td * 1e3, 3), "calls": "rsg_encode_host / rsg_decode_host, synchronous, "
                         "wall clock, median of 3 after a warm-up call", "parity": "ok" if ok else "MISMATCH"}
    # (b) reference API, one stripe per call, on seq_create sequences
    rs = rs_amd.RS()
    hn = h.numpy()
    seqs = []
    try:
        for j in range(8):
            q = rs_amd.Seq(k + r, S)
            for i in range(k):
                q.symbols[i][:] = hn[j, i]
            seqs.append(q)
        calls = 48
        for q in seqs:  # warm-up
            assert rs.generate_repair_symbols(q, r) == 0
        te = 0.0
        for c in range(calls):
            q = seqs[c % len(seqs)]
            t0 = time.perf_counter()
            rc = rs.generate_repair_symbols(q, r)
            te += time.perf_counter() - t0
            ok2 = rc == 0
        ok2 = ok2 and all(np.array_equal(seqs[j].symbols[k + i], hn[j, k + i]) for j in range(len(seqs))
                          for i in range(r))
        eidx = np.nonzero(erased)[0]
        td = 0.0
        for c in range(3 + calls):  # 3 warm-up calls: the pattern's plan and its specialised kernel
            q = seqs[c % len(seqs)]
            for i in eidx:
                q.symbols[i][:] = 0
            t0 = time.perf_counter()
            rc = rs.restore_symbols(k, r, q, erased, t)
            if c >= 3:
                td += time.perf_counter() - t0
            ok2 = ok2 and rc == 0
        ok2 = ok2 and all(np.array_equal(seqs[j].symbols[i], hn[j, i]) for j in range(len(seqs)) for i in eidx)
    finally:
        for q in seqs:
            q.close()
        rs.close()
    out["reference_api"] = {"calls": calls, "encode_GBps": round(calls * (k + r) * S / te / 1e9, 2),
                            "decode_GBps": round(calls * (k + t) * S / td / 1e9, 2),
                            "encode_ms_per_call": round(te / calls * 1e3, 4),
                            "decode_ms_per_call": round(td / calls * 1e3, 4),
                            "buffers": f"{len(seqs)} seq_create stripes (page-locked arena), one stripe per call, "
                                       "wall clock summed over the calls (Python ctypes caller)",
                            "parity": "ok" if ok2 else "MISMATCH"}
    return out


def config_leg(k, r, S, n, steps, warmup, dev, stream, oracle_decode_check):
    """Another BASELINE config on this GPU (a few steps, same step definition and byte accounting as the
    headline): encode + decode of `n` resident stripes, t = r information erasures. Reports the whole-step
    rate, each leg's per-launch HIP-event time, the dominant launch's HBM roofline fraction and the
    PMC-measured traffic from profiles/traffic.json (null when no record matches this build). Checks: round
    trip (fingerprints) on every stripe; repair (and, with `oracle_decode_check`, restored) symbols of the
    first stripes bit-exact vs the CPU oracle."""
    import torch
    import rs_amd
    import rs_dist
    erased = rs_amd.bench_pattern(k, r)
    t = int(erased.sum())
    codec = rs_amd.Codec(k, r, device=dev.index)
    buf = torch.empty((n, k + r, S), dtype=torch.uint8, device=dev)
    rs_amd.fill_info(buf, k, SEED, stream=stream)
    fp_ref = torch.zeros(n, dtype=torch.int64, device=dev)
    rs_amd.fingerprint(buf, 0, k, fp_ref, stream=stream)
    for _ in range(warmup):
        codec.encode(buf, stream=stream)
        kern_enc, work_enc = codec.last_kernel, codec.last_work
        codec.decode(buf, erased, stream=stream)
        kern_dec, work_dec = codec.last_kernel, codec.last_work
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(steps)]
    with rs_dist.TimedRegion(dev) as region:
        for e in ev:
            e[0].record(stream)
            codec.encode(buf, stream=stream)
            e[1].record(stream)
            codec.decode(buf, erased, stream=stream)
            e[2].record(stream)
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    enc_bytes, dec_bytes = n * (k + r) * S, n * (k + t) * S
    cfg_key = f"k{k}_r{r}_S{S}_n{n}_t{t}"
    dom = max((enc_ms, enc_bytes, kern_enc, "encode"), (dec_ms, dec_bytes, kern_dec, "decode"))
    achieved = dom[1] / (dom[0] / 1e3) / 1e9
    traffic = {leg: measured_traffic(kern, cfg_key, leg=leg) for leg, kern in (("encode", kern_enc),
                                                                              ("decode", kern_dec))}
    # parity: the information symbols survived every step; poisoned erased slots are restored
    fp = torch.zeros(n, dtype=torch.int64, device=dev)
    rs_amd.fingerprint(buf, 0, k, fp, stream=stream)
    buf[:, torch.from_numpy(erased).to(dev)] = 0xA5
    codec.decode(buf, erased, stream=stream)
    fp1 = torch.zeros(n, dtype=torch.int64, device=dev)
    rs_amd.fingerprint(buf, 0, k, fp1, stream=stream)
    torch.cuda.synchronize()
    ok = bool(torch.equal(fp, fp_ref) and torch.equal(fp1, fp_ref))
    n_chk = n if oracle_decode_check else 1
    avail, quota = cpu_cores()
    ok = ok and oracle_check_batch(k, r, buf[:n_chk].cpu().numpy(), erased, max(1, min(avail, quota or avail)),
                                   decode=oracle_decode_check)
    line = {"workload": f"k={k} r={r} symbol={S}B stripes={n} decode t={t} (info erasures at i*{max(k // t, 1)})",
            "value": round((enc_bytes + dec_bytes) * steps / region.elapsed / 1e9, 2), "unit": "GB/s",
            "steps": steps, "warmup": warmup, "ms_per_step": round(region.elapsed / steps * 1e3, 3),
            "kernel": {"encode": kern_enc, "decode": kern_dec},
            "per_launch": {"encode": {"ms": round(enc_ms, 4), "bytes": enc_bytes, "traffic": traffic["encode"]},
                           "decode": {"ms": round(dec_ms, 4), "bytes": dec_bytes, "traffic": traffic["decode"]}},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic[dom[3]], "kernel": dom[2],
                         "leg": dom[3], "traffic_key": cfg_key},
            "parity": "ok" if ok else "MISMATCH",
            "check": f"round trip on all {n} stripes; " + (f"all {n_chk} stripes encode + decode" if oracle_decode_check
                                                         else "stripe 0 encode") + " bit-exact vs the CPU oracle"}
    if work_enc[0] + work_dec[0] > 0:
        line["roofline"]["compute"] = compute_roofline(work_enc, enc_ms, work_dec, dec_ms)
    del buf
    codec.close()
    torch.cuda.empty_cache()
    return line


def symbol_ops_leg(dev, stream):
    """The secondary surface batched (rsg_symbol_ops; ref src/rs/gf65536.c:155-219, one synchronous GPU round
    trip per gf_* call otherwise): chains of gf_madd accumulating into targets, as the reference's evaluator /
    restore loops do, ONE call per batch. Per-op device time (HIP events on the stream, median of 5 calls) and
    the call's host time. Check: every target against the ops applied one after another with numpy."""
    import torch
    import rs_amd
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _util import gf_tables
    exp, log = gf_tables()
    out = {}
    rng = np.random.default_rng(SEED)
    for S, n_t, per_t in ((1024, 128, 32), (65536, 32, 32)):
        src = torch.from_numpy(rng.integers(0, 256, (per_t, S), dtype=np.uint8)).to(dev)
        tgt = torch.zeros((n_t, S), dtype=torch.uint8, device=dev)
        coefs = rng.integers(2, 65536, (n_t, per_t))
        ops = np.zeros(n_t * per_t, rs_amd.SYMBOL_OP_DTYPE)
        ops["op"] = rs_amd.OP_MADD
        ops["a"] = tgt.data_ptr() + np.repeat(np.arange(n_t, dtype=np.uint64), per_t) * S
        ops["b"] = src.data_ptr() + np.tile(np.arange(per_t, dtype=np.uint64), n_t) * S
        ops["coef"] = coefs.reshape(-1)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(9)]
        host = []
        for e0, e1 in ev:  # calls 0-3 fill the library's 4 op-list staging slots: not counted
            tgt.zero_()
            torch.cuda.synchronize()
            torch.cuda._sleep(2_000_000)  # the stream waits ~1 ms: the events bracket the op-list copy + kernel only
            e0.record(stream)
            t0 = time.perf_counter()
            rs_amd.symbol_ops(ops, S, device=dev.index, stream=stream)
            host.append(time.perf_counter() - t0)
            e1.record(stream)
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev[4:]]))
        got = tgt.cpu().numpy().view("<u2").astype(np.int64)
        ws = src.cpu().numpy().view("<u2").astype(np.int64)
        want = np.zeros_like(got)
        for j in range(per_t):
            lw = np.where(ws[j] != 0, log[ws[j]], -1)
            prod = np.where(lw[None, :] >= 0, exp[(lw[None, :] + log[coefs[:, j]][:, None]) % 65535], 0)
            want ^= prod
        n_ops = n_t * per_t
        out[f"S{S}"] = {"ops": n_ops, "targets": n_t, "ops_per_target": per_t, "call_ms": round(ms, 4),
                        "us_per_op": round(ms * 1e3 / n_ops, 4), "host_us_per_call": round(float(np.median(host[4:])) * 1e6, 1),
                        "host_us_per_op": round(float(np.median(host[4:])) * 1e6 / n_ops, 4),
                        "source_GBps": round(n_ops * S / ms / 1e6, 1), "parity": "ok" if np.array_equal(got, want) else "MISMATCH"}
    out["note"] = ("gf_madd chains in one rsg_symbol_ops call (SYMBOL_OP_DTYPE array); call_ms = HIP events around the "
                   "op-list copy + kernel (stream held by a spin kernel while the call is queued), median of 5 calls after 4 "
                   "warm-up calls; host_us = the C call's "
                   "host time (validation, chains, staging). The per-call gf_madd on host symbols is a synchronous round "
                   "trip of ~16-23 us (DESIGN.md section 9)")
    return out


def extra_legs(args, stripes, fp_ref, erased, stream, dev):
    """The legs VERDICT r5 asked the driver to measure beside the headline (N = 1, after its timed region and
    checks; never part of `value`). A leg that raises is reported as such; the headline line still prints."""
    wanted = {x.strip() for x in args.extras.split(",") if x.strip()}
    out = {}
    t_all = time.perf_counter()
    for name, fn in (("per_stripe_decode", lambda: per_stripe_leg(args, stripes, fp_ref, stream, dev)),
                     ("end_to_end", lambda: host_path_leg(args, stripes, erased, dev)),
                     ("symbol_ops", lambda: symbol_ops_leg(dev, stream))):
        if name in wanted:
            t0 = time.perf_counter()
            try:
                out[name] = fn()
            except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
                out[name] = {"error": f"{type(e).__name__}: {e}", "parity": "ERROR"}
            out[name]["leg_s"] = round(time.perf_counter() - t0, 2)
    if "configs" in wanted:
        out["configs"] = {}
        for label, (k, r, S, steps, warmup, dec_chk) in (("C2", (10, 4, 4096, 50, 5, True)),
                                                         ("C5", (4096, 1024, 1024, 3, 2, False))):
            t0 = time.perf_counter()
            try:
                out["configs"][label] = config_leg(k, r, S, args.cfg_stripes, steps, warmup, dev, stream, dec_chk)
            except Exception as e:  # noqa: BLE001
                out["configs"][label] = {"error": f"{type(e).__name__}: {e}", "parity": "ERROR"}
            out["configs"][label]["leg_s"] = round(time.perf_counter() - t0, 2)
    out["extras_s"] = round(time.perf_counter() - t_all, 2)
    return out


# ------------------------------------------------------------------- stripes from one rank
def scatter_leg(args, rank, world, dev):
    """Stripes that originate on rank 0 (--scatter STRIPES per rank): RCCL scatter of the information
    symbols to their owners (rs_dist.scatter_stripes, one P2P group, one xGMI link per peer) and the
    gather of the repair symbols back. Timed on its own (barrier-bracketed, max over ranks); never
    part of `value`."""
    import torch
    import rs_dist
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


VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions / s: 256 CUs x 4 SIMD-32, 2 cycles each, 2.4 GHz


def compute_roofline(work_enc, enc_ms, work_dec, dec_ms):
    """Issue rate of the generated kernels (their asm's VALU + SALU counts per launch, rsg_last_work:
    XOR kernels per 256-byte column, GF(2^16) steps per step) against the chip's VALU issue peak
    (2 cycles per wave64 op per SIMD at 2.4 GHz). The chip holds ~1.4-1.5 GHz under these loads, and
    gpr-indexed VALU (the GF(2^16) table lookups) issue at half rate on gfx950
    (profiles/r1/r1_issue_bench.log), so frac ~0.6 (XOR kernels) / ~0.5 (GF(2^16)) are practical ceilings."""
    v = work_enc[0] + work_dec[0]
    sa = work_enc[1] + work_dec[1]
    t = (enc_ms + dec_ms) / 1e3
    return {"bound": "valu-issue", "valu_insts": v, "salu_insts": sa, "achieved": round(v / t / 1e12, 4),
            "peak": round(VALU_PEAK / 1e12, 4), "unit": "T wave-VALU/s", "frac": round(v / t / VALU_PEAK, 4)}


def gather_objects(obj, group):
    """`obj` of every rank, in rank order (over the CPU-side gloo group; one entry without one)."""
    import torch.distributed as dist
    if group is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=group)
    return out


def per_rank_times(enc_ms, dec_ms, ident, group):
    """[{rank, encode_ms, decode_ms, pci_bus_id, uuid}] of every rank."""
    mine = {"encode_ms": round(float(enc_ms), 3), "decode_ms": round(float(dec_ms), 3), **ident}
    return [dict(rank=i, **p) for i, p in enumerate(gather_objects(mine, group))]


def cpu_group_barrier(group):
    """Barrier over the gloo side group: ranks waiting here (e.g. while rank 0 runs the CPU baseline)
    block in a socket read instead of spinning on a device collective."""
    import torch.distributed as dist
    if group is not None:
        dist.barrier(group=group)


def start_group(backend, local):
    """Joins the job's process group (`backend`: "nccl" = RCCL, or "gloo" for a dry run) when launched as
    a rank, plus a gloo side group for host-side exchanges (device identities, per-rank times, waits
    while rank 0 runs the CPU baseline). Returns the side group, or None for a single process."""
    import torch
    import torch.distributed as dist
    if "WORLD_SIZE" not in os.environ:
        return None
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist.new_group(backend="gloo") if dist.get_world_size() > 1 else None


def base_line(args, world, n, k, r, S, t, elapsed):
    total_bytes = n * ((k + r) * S + (k + t) * S) * world * args.steps
    return {
        "metric": METRIC,
        "value": round(total_bytes / elapsed / 1e9, 2),
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
                               f"at i*{max(k // max(t, 1), 1)})", "stripes_total": n * world,
                   "parallelism": f"stripes x{world}"},
    }


# ------------------------------------------------------------------------------ dry run (CPU)
def dry_run_main(args, rank, world):
    """The multi-rank protocol without a GPU: gloo process group, the same barrier-bracketed timed
    region and max-over-ranks reduction, per-rank times gathered, no coding work (step = a no-op)."""
    import torch.distributed as dist
    import rs_dist
    group = start_group("gloo", local=rank)
    n, k, r, S = args.stripes, args.k, args.r, args.symbol
    ident = {"pci_bus_id": "dry-run" if args.dry_same_device else f"dry-run:{rank}", "uuid": ""}
    if not check_distinct_devices(gather_objects(ident, group)):
        sys.exit(3)
    with rs_dist.TimedRegion(None) as region:
        for _ in range(args.steps):
            time.sleep(0.001 * (1 + rank))
            if rank == args.dry_fail_rank:
                print(f"bench.py: rank {rank}: injected failure (--dry-fail-rank)", file=sys.stderr, flush=True)
                os._exit(3)
    erased = np.zeros(k + r, np.bool_)
    erased[[i * max(k // r, 1) for i in range(r)]] = True
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:  # N = 1 only, as on the GPU
        cpu, _ = cpu_baseline(args, erased, None)
    cpu_group_barrier(group)
    line = base_line(args, world, n, k, r, S, r, region.max_elapsed)
    line["dry_run"] = True
    line["value"] = None  # no coding work ran: there is no throughput to report
    line["data"] = "dry run: no GPU work, harness protocol only"
    line["rccl_world"] = dist.get_world_size() if dist.is_initialized() else 1
    line["per_rank"] = per_rank_times(region.elapsed * 1e3, 0.0, ident, group)
    line["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


# ------------------------------------------------------------------------------ main
def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))  # parent: no GPU touched, children do the work
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} does not match WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    import rs_dist
    rank, world, local = rs_dist.env()
    if args.dry_run:
        return dry_run_main(args, rank, world)

    import torch
    if world > torch.cuda.device_count():
        print(f"bench.py: WORLD_SIZE {world} exceeds the {torch.cuda.device_count()} visible GPU(s)", file=sys.stderr)
        sys.exit(2)
    import rs_amd  # raises if librs_amd.so is missing: no fallback
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # launched as ranks (torchrun or --gpus N): RCCL process group, even at N=1, + a gloo side group
    group = start_group("nccl", local)
    ident = device_identity(dev)
    if not check_distinct_devices(gather_objects(ident, group)):  # before any HBM is committed
        sys.exit(3)

    k, r, S, n = args.k, args.r, args.symbol, args.stripes
    erased = rs_amd.bench_pattern(k, r)
    if args.t:  # t information erasures at i * (k // t), no repair erasure
        erased = np.concatenate([rs_amd.bench_pattern(k, args.t)[:k], np.zeros(r, np.bool_)])
    t = int(erased.sum())
    opts = {"auto": {}, "jit": dict(jit=1), "v1jit": dict(jit=1, xj=0), "v1": dict(jit=0, m8_mode=18),
            "idx": dict(jit=0, m8_mode=2), "table": dict(jit=0, m8_mode=0), "mask": dict(jit=0, m8_mode=1),
            "m16c": {}}[args.kernel]
    # the A/B families idx / table / mask live in the diagnostic library (never a reported value's default)
    lib = rs_amd.diag_module() if args.kernel in ("idx", "table", "mask") else rs_amd
    codec = lib.Codec(k, r, device=local, **opts)
    if args.kernel == "m16c":  # GF(2^16) codes: the compiled kernel
        codec.set_option("m16_mode", 2)
    for o in args.opt:
        name, _, value = o.partition("=")
        codec.set_option(name, int(value))
    stripes = torch.empty((n, k + r, S), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    stripe0, _ = rs_dist.weak_shard(n, rank)  # this rank's global stripe ids: [stripe0, stripe0 + n)
    rs_amd.fill_info(stripes, k, SEED, stripe0=stripe0, stream=stream)
    # reference fingerprint of the generated information symbols (the timed loop must preserve them)
    fp_ref = torch.zeros(n, dtype=torch.int64, device=dev)
    if not args.profile_only:
        rs_amd.fingerprint(stripes, 0, k, fp_ref, stream=stream)

    # warmup (also compiles / loads the specialised kernels); the kernels and their instruction counts
    # are read here, outside the timed loop (at small sizes the extra library calls per launch would
    # show as host time between launches), and checked again after it
    kern_enc = kern_dec = None
    work_enc = work_dec = (0, 0)
    for _ in range(args.warmup):
        codec.encode(stripes, stream=stream)
        kern_enc, work_enc = codec.last_kernel, codec.last_work
        codec.decode(stripes, erased, stream=stream)
        kern_dec, work_dec = codec.last_kernel, codec.last_work
    torch.cuda.synchronize()

    # HIP events on the launch stream around both launches of every `stride`-th step (about 32 sampled
    # steps spread over the timed region): each record costs ~5 us of host time, which at small
    # configurations (C2: 14 us kernels) would otherwise starve the GPU between launches
    stride = max(1, args.steps // 32)
    sampled = range(0, args.steps, stride)
    ev = {i: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
              torch.cuda.Event(enable_timing=True)) for i in sampled}
    with rs_dist.TimedRegion(dev) as region:
        for i in range(args.steps):
            e = ev.get(i)
            if e:
                e[0].record(stream)
            codec.encode(stripes, stream=stream)
            if kern_enc is None:  # --warmup 0: read them on the first timed step
                kern_enc, work_enc = codec.last_kernel, codec.last_work
            if e:
                e[1].record(stream)
            codec.decode(stripes, erased, stream=stream)
            if kern_dec is None:
                kern_dec, work_dec = codec.last_kernel, codec.last_work
            if e:
                e[2].record(stream)
    elapsed = region.max_elapsed
    if args.steps and codec.last_kernel != kern_dec:  # the decode plan changed kernels inside the timed loop
        print(f"bench.py: decode kernel changed after warmup ({kern_dec} -> {codec.last_kernel}); use more "
              f"--warmup", file=sys.stderr)
        kern_dec, work_dec = codec.last_kernel, codec.last_work

    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev.values()]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev.values()]))
    enc_bytes = n * (k + r) * S
    dec_bytes = n * (k + t) * S
    per_rank = per_rank_times(enc_ms, dec_ms, ident, group)
    # N = 1 only (rank 0, after the timed region): the baseline is one host's CPU path, not a per-N figure,
    # and the scaling runs (N = 2, 4, 8) stay free of ~15 s of CPU work each
    run_cpu = rank == 0 and world == 1 and not args.no_cpu and not args.profile_only

    # verification: restored information == generated information (fingerprints), sampled repair
    parity = "skipped"
    gpu_sample = None
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
        if run_cpu:  # the CPU leg compares these stripes (global ids 0.. on rank 0) bit for bit
            gpu_sample = stripes[: args.cpu_stripes].cpu().numpy()
        parity = "roundtrip-ok" if ok else "ROUNDTRIP-MISMATCH"

    scatter = scatter_leg(args, rank, world, dev) if args.scatter > 0 and world > 1 else None

    cpu = None
    if run_cpu:  # the other ranks wait at the gloo barrier below (no device spin)
        cpu, cpu_ok = cpu_baseline(args, erased, gpu_sample)
        gpu_sample = None
        if not args.profile_only:
            parity += ",cpu-bitexact-ok" if cpu_ok else ",CPU-MISMATCH"
    cpu_group_barrier(group)

    extras = None
    if world == 1 and not args.no_extras and not args.profile_only and "MISMATCH" not in parity:
        extras = extra_legs(args, stripes, fp_ref, erased, stream, dev)

    # roofline of the dominant kernel (encode and decode move the same algorithmic bytes here)
    dom_ms, dom_bytes, dom_name, dom_leg = ((enc_ms, enc_bytes, kern_enc, "encode") if enc_ms >= dec_ms
                                            else (dec_ms, dec_bytes, kern_dec, "decode"))
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9
    cfg_key = f"k{k}_r{r}_S{S}_n{n}_t{t}"
    traffic, traffic_src = measured_traffic(dom_name, cfg_key, with_source=True, leg=dom_leg)
    line = base_line(args, world, n, k, r, S, t, elapsed)
    line["config"]["kernel"] = {"encode": kern_enc, "decode": kern_dec}
    line["rccl_world"] = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "kernel": dom_name, "kernel_ms": round(dom_ms, 3), "bytes_per_launch": dom_bytes,
                        "traffic_key": cfg_key, "traffic_source": traffic_src}
    if work_enc[0] + work_dec[0] > 0:  # compute roofline (the kernels are VALU-issue bound)
        line["roofline"]["compute"] = compute_roofline(work_enc, enc_ms, work_dec, dec_ms)
    # both legs: algorithmic bytes and PMC-measured HBM bytes per launch (null when unmeasured)
    line["per_launch"] = {"encode": {"kernel": kern_enc, "ms": round(enc_ms, 3), "bytes": enc_bytes,
                                     "traffic": measured_traffic(kern_enc, cfg_key, leg="encode")},
                          "decode": {"kernel": kern_dec, "ms": round(dec_ms, 3), "bytes": dec_bytes,
                                     "traffic": measured_traffic(kern_dec, cfg_key, leg="decode")}}
    line["event_steps"] = {"sampled": len(ev), "stride": stride}  # steps carrying the per-launch HIP events
    line["encode_ms"] = round(enc_ms, 3)
    line["decode_ms"] = round(dec_ms, 3)
    line["per_rank"] = per_rank
    line["cpu_baseline"] = cpu
    line["parity"] = parity
    if scatter is not None:
        line["scatter"] = scatter
    if extras is not None:
        line.update(extras)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    if "MISMATCH" in parity:
        sys.exit(1)


if __name__ == "__main__":
    main()
