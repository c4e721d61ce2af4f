"""Multi-GPU plumbing for the stripe-parallel path.

Stripes are independent (no exchange step in encode or decode), so N GPUs run as N processes
(torchrun: RANK / LOCAL_RANK / WORLD_SIZE), each owning a contiguous range of stripes; no collective
touches the data path. The only collectives are the barriers that bracket a timed region and one
MAX reduction of the elapsed time (the job is as slow as its slowest rank), plus an optional XOR
combination of per-stripe fingerprints for verification. Backend "nccl" (RCCL over xGMI) on GPUs,
"gloo" for the CPU tests.

When the stripes originate on one rank (shards arriving from a file or socket on one host process),
`scatter_stripes` moves every rank's contiguous shard with one batch of point-to-point sends from
the root -- RCCL runs the batch as one group, so each peer's shard travels on its own xGMI link --
and `gather_stripes` brings results back the same way. bench.py times this separately (--scatter);
it is never part of the device-resident number.
"""
import os
import time

import torch
import torch.distributed as dist


def env():
    """(rank, world_size, local_rank) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_total, world, rank):
    """Contiguous stripe range [first, first + count) of `rank` when n_total stripes are split over
    `world` ranks (sizes differ by at most one)."""
    first = n_total * rank // world
    return first, n_total * (rank + 1) // world - first


def weak_shard(per_rank, rank):
    """Weak scaling: every rank owns `per_rank` stripes; global stripe ids start at rank * per_rank."""
    return rank * per_rank, per_rank


def _active():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def barrier():
    if _active():
        dist.barrier()


def _sync(device):
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


class TimedRegion:
    """barrier + device sync on entry and exit; `.elapsed` is this rank's wall time and
    `.max_elapsed` the maximum over ranks (what a multi-GPU job is charged)."""

    def __init__(self, device=None):
        self.device = device

    def __enter__(self):
        barrier()
        _sync(self.device)
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        _sync(self.device)
        self.elapsed = time.perf_counter() - self.t0
        barrier()
        self.max_elapsed = max_over_ranks(self.elapsed, self.device)
        return False


def max_over_ranks(value, device=None):
    if not _active():
        return float(value)
    on_gpu = dist.get_backend() == "nccl"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def xor_over_ranks(fp):
    """XOR-combines an int64 tensor (e.g. whole-job fingerprint) across ranks."""
    if not _active():
        return fp
    parts = [torch.empty_like(fp) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, fp)
    out = parts[0].clone()
    for p in parts[1:]:
        out ^= p
    return out


def scatter_stripes(src, dst, root=0):
    """Root's `src` [world * n, ...] -> every rank's `dst` [n, ...] (rank g gets rows [g*n, (g+1)*n)).
    One batch of isend (root) / irecv (others); `src` is ignored on non-root ranks."""
    if not _active():
        dst.copy_(src[: dst.shape[0]])
        return
    rank, world = dist.get_rank(), dist.get_world_size()
    n = dst.shape[0]
    if rank == root:
        ops = [dist.P2POp(dist.isend, src[g * n:(g + 1) * n].contiguous(), g) for g in range(world) if g != root]
        reqs = dist.batch_isend_irecv(ops)
        dst.copy_(src[root * n:(root + 1) * n])
    else:
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.irecv, dst, root)])
    for q in reqs:
        q.wait()


def gather_stripes(src, dst, root=0):
    """Every rank's `src` [n, ...] -> root's `dst` [world * n, ...] (inverse of scatter_stripes)."""
    if not _active():
        dst[: src.shape[0]].copy_(src)
        return
    rank, world = dist.get_rank(), dist.get_world_size()
    n = src.shape[0]
    if rank == root:
        views = {g: dst[g * n:(g + 1) * n] for g in range(world) if g != root}
        bufs = {g: (v if v.is_contiguous() else torch.empty_like(v)) for g, v in views.items()}
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.irecv, bufs[g], g) for g in bufs])
        dst[root * n:(root + 1) * n].copy_(src)
        for q in reqs:
            q.wait()
        for g, b in bufs.items():
            if b is not views[g]:
                views[g].copy_(b)
    else:
        for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, src.contiguous(), root)]):
            q.wait()
