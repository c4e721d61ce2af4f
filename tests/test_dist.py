"""Multi-process stripe sharding (the N>1 path of bench.py) on CPU with gloo, world_size 2.

Each rank owns a contiguous stripe range (rs_dist.weak_shard / shard), builds its stripes from the
global stripe ids, encodes, erases and decodes them with the CPU oracle (the GPU engine is not
available here), and fingerprints them; the XOR of the per-rank fingerprints must equal the
single-process fingerprint of the whole job, and TimedRegion must report the max over ranks."""
import os
import socket
import sys
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "reed-solomon_amd"))
import rs_dist  # noqa: E402
from _util import bench_pattern, fingerprint_np, gen_info, oracle_decode, oracle_encode  # noqa: E402

K, R, S, PER_RANK, SEED = 10, 4, 512, 3, 0x5EED


def _job_stripes(first, count):
    """Encoded + round-tripped stripes [first, first + count) and their fingerprints."""
    er = np.zeros(K + R, np.bool_)
    er[bench_pattern(K, R)] = True
    fps = []
    for s in range(first, first + count):
        buf = np.zeros((K + R, S), np.uint8)
        buf[:K] = gen_info(SEED, s, K * S).reshape(K, S)
        assert oracle_encode(K, R, buf) == 0
        fp = fingerprint_np(buf, 0, K + R)
        lost = buf.copy()
        lost[er] = 0
        assert oracle_decode(K, R, lost, er, int(er.sum())) == 0
        assert np.array_equal(lost[:K], buf[:K])
        fps.append(fp)
    return fps


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, w, _ = rs_dist.env()
        first, count = rs_dist.weak_shard(PER_RANK, r)
        fps = _job_stripes(first, count)
        mine = np.bitwise_xor.reduce(np.array(fps, np.int64))
        job = rs_dist.xor_over_ranks(torch.tensor([int(mine)], dtype=torch.int64))
        with rs_dist.TimedRegion() as region:
            time.sleep(0.05 + 0.25 * r)  # rank 1 is the slow one
        q.put((r, first, count, int(job.item()), region.elapsed, region.max_elapsed))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partitions():
    for n in (0, 1, 7, 8192, 65536):
        for world in (1, 2, 3, 8):
            ranges = [rs_dist.shard(n, world, g) for g in range(world)]
            assert sum(c for _, c in ranges) == n
            assert all(ranges[g][0] + ranges[g][1] == ranges[g + 1][0] for g in range(world - 1))
            assert max(c for _, c in ranges) - min(c for _, c in ranges) <= 1
    assert [rs_dist.weak_shard(8192, g) for g in range(3)] == [(0, 8192), (8192, 8192), (16384, 8192)]


def test_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(g, 2, port, q)) for g in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0, 0]
    res = sorted(q.get(timeout=10) for _ in procs)
    want = np.bitwise_xor.reduce(np.array(_job_stripes(0, 2 * PER_RANK), np.int64))
    assert [(r[1], r[2]) for r in res] == [(0, PER_RANK), (PER_RANK, PER_RANK)]
    assert all(r[3] == int(want) for r in res), "XOR of shard fingerprints != whole-job fingerprint"
    assert res[0][4] < res[1][4]
    assert all(abs(r[5] - res[1][4]) < 1e-9 for r in res), "TimedRegion must report the max over ranks"
    assert res[0][5] >= 0.3


def _scatter_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = PER_RANK
        src = torch.zeros((world * n, K + R, S), dtype=torch.uint8)
        if rank == 0:  # the stripes originate on rank 0
            for s in range(world * n):
                src[s, :K] = torch.from_numpy(gen_info(SEED, s, K * S).reshape(K, S))
        mine = torch.empty((n, K + R, S), dtype=torch.uint8)
        rs_dist.scatter_stripes(src, mine, root=0)
        first, _ = rs_dist.weak_shard(n, rank)
        ok = all(np.array_equal(mine[i, :K].numpy(), gen_info(SEED, first + i, K * S).reshape(K, S))
                 for i in range(n))
        buf = mine.numpy()
        for i in range(n):  # encode the shard, results go back to rank 0
            assert oracle_encode(K, R, buf[i]) == 0
        back = torch.zeros((world * n, K + R, S), dtype=torch.uint8)
        rs_dist.gather_stripes(torch.from_numpy(buf), back, root=0)
        q.put((rank, ok, back.numpy()[:, K:].tobytes() if rank == 0 else b""))
    finally:
        dist.destroy_process_group()


def test_scatter_gather_from_rank0_gloo():
    """Stripes that originate on rank 0 reach their owners (scatter_stripes), are encoded there and
    the repair symbols come back to rank 0 (gather_stripes) equal to a single-process encode."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(g, 2, port, q)) for g in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0, 0]
    res = sorted((q.get(timeout=10) for _ in procs), key=lambda t: t[0])
    assert all(r[1] for r in res), "a rank received the wrong shard"
    want = []
    for s in range(2 * PER_RANK):
        buf = np.zeros((K + R, S), np.uint8)
        buf[:K] = gen_info(SEED, s, K * S).reshape(K, S)
        assert oracle_encode(K, R, buf) == 0
        want.append(buf[K:])
    assert res[0][2] == np.stack(want).tobytes()


def _bench_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return __import__("json").loads(lines[0])


def test_bench_launcher_spawns_ranks_dry_run():
    """`bench.py --gpus 2` outside torchrun starts two rank processes itself (gloo dry run here): the
    line reports both ranks, the whole-job stripe count and per-rank times; a --gpus / WORLD_SIZE
    mismatch is fatal."""
    import subprocess
    bench = os.path.join(HERE, "..", "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, bench, "--gpus", "2", "--dry-run", "--steps", "2", "--stripes", "64"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr
    line = _bench_line(p.stdout)
    assert line["n_gpus"] == 2 and line["rccl_world"] == 2
    assert line["config"]["stripes_total"] == 2 * 64
    assert [e["rank"] for e in line["per_rank"]] == [0, 1]
    assert line["dry_run"] is True and line["value"] is None
    bad = subprocess.run([sys.executable, bench, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                         timeout=120, env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert bad.returncode == 2 and "does not match" in bad.stderr


def _run_bench(*argv, timeout=300):
    import subprocess
    bench = os.path.join(HERE, "..", "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    return subprocess.run([sys.executable, bench, *argv], capture_output=True, text=True, timeout=timeout, env=env)


def _rank_pids(stderr):
    import re
    return {int(m.group(1)): int(m.group(2)) for m in re.finditer(r"rank (\d+) pid (\d+)", stderr)}


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    try:  # a zombie is not alive (it would only mean the parent did not reap it)
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


def test_bench_launcher_eight_ranks_dry_run():
    """The C4 shape (BASELINE.json configs[3]): `bench.py --gpus 8` at the default 8192 stripes per rank
    reports 65536 stripes, 8 distinct ranks on 8 distinct devices and per-rank times; the CPU baseline
    belongs to the N = 1 line only (rank 0 of a single-rank run times it after the timed region)."""
    p = _run_bench("--gpus", "8", "--dry-run", "--steps", "2", "--cpu-stripes", "2", "--cpu-seconds", "0.1")
    assert p.returncode == 0, p.stderr[-2000:]
    line = _bench_line(p.stdout)
    assert line["n_gpus"] == 8 and line["rccl_world"] == 8
    assert line["config"]["stripes_total"] == 65536
    assert [e["rank"] for e in line["per_rank"]] == list(range(8))
    assert len({e["pci_bus_id"] for e in line["per_rank"]}) == 8
    assert line["cpu_baseline"] is None
    pids = _rank_pids(p.stderr)
    assert sorted(pids) == list(range(8)) and not any(_alive(q) for q in pids.values())
    # N = 1 through the same launcher: the line carries the baseline
    p1 = _run_bench("--gpus", "1", "--dry-run", "--steps", "2", "--cpu-stripes", "2", "--cpu-seconds", "0.1")
    assert p1.returncode == 0, p1.stderr[-2000:]
    cpu = _bench_line(p1.stdout)["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1


def test_bench_launcher_rank_failure_stops_everyone():
    """A rank that exits non-zero (here inside the timed region, while the others block in a barrier)
    makes the launcher exit with that status, and no rank process outlives it."""
    p = _run_bench("--gpus", "8", "--dry-run", "--steps", "200", "--no-cpu", "--dry-fail-rank", "3")
    assert p.returncode == 3, p.stderr[-2000:]
    assert "rank 3 exited with 3" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    pids = _rank_pids(p.stderr)
    assert sorted(pids) == list(range(8))
    time.sleep(0.5)
    assert not any(_alive(q) for q in pids.values()), "orphaned rank processes"


def test_bench_duplicate_device_is_fatal():
    """Two ranks on one device would count one GPU twice: every rank stops before any work."""
    p = _run_bench("--gpus", "2", "--dry-run", "--no-cpu", "--dry-same-device")
    assert p.returncode == 3 and "share device" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_visible_gpu_count_without_hip(tmp_path):
    """The launcher counts GPUs from the KFD topology and the visibility variables, never through HIP."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(HERE, "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    nodes = tmp_path / "nodes"
    for i, gid in enumerate([0, 0, 4242, 4243, 4244, 4245, 4246, 4247, 4248, 4249]):  # 2 CPU nodes, 8 GPUs
        (nodes / str(i)).mkdir(parents=True)
        (nodes / str(i) / "gpu_id").write_text(f"{gid}\n")
    assert bench.visible_gpu_count({}, str(nodes)) == 8
    assert bench.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,1,2"}, str(nodes)) == 3
    assert bench.visible_gpu_count({"ROCR_VISIBLE_DEVICES": "3"}, str(nodes)) == 1
    assert bench.visible_gpu_count({"CUDA_VISIBLE_DEVICES": ""}, str(nodes)) == 0
    assert bench.visible_gpu_count({}, str(tmp_path / "absent")) is None
    assert bench.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,1"}, str(tmp_path / "absent")) == 2


def test_launcher_parent_never_loads_hip():
    """The `--gpus N` parent counts devices and spawns ranks without importing torch or the HIP library
    (checked in a fresh interpreter, with the rank processes replaced by no-ops)."""
    import subprocess
    code = f"""
import os, subprocess, sys
sys.path.insert(0, {os.path.join(HERE, "..")!r})
for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
    os.environ.pop(v, None)
os.environ["HIP_VISIBLE_DEVICES"] = "0,1,2,3,4,5,6,7"
import bench
class Done:
    pid = 0
    def poll(self): return 0
    def wait(self, timeout=None): return 0
started = []
subprocess.Popen = lambda *a, **k: started.append(a) or Done()
sys.argv = ["bench.py", "--gpus", "8"]
rc = bench.spawn_ranks(bench.parse(sys.argv[1:]))
loaded = [m for m in ("torch", "rs_amd") if m in sys.modules]
hip = [ln for ln in open("/proc/self/maps") if "amdhip" in ln]
print(rc, len(started), loaded, len(hip))
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split("\n")[-2] == "0 8 [] 0"
