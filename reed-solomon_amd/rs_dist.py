"""Multi-GPU plumbing for the stripe-parallel path.

Stripes are independent (no exchange step in encode or decode), so N GPUs run as N processes
(torchrun: RANK / LOCAL_RANK / WORLD_SIZE), each owning a contiguous range of stripes; no collective
touches the data path. The only collectives are the barriers that bracket a timed region and one
MAX reduction of the elapsed time (the job is as slow as its slowest rank), plus an optional XOR
combination of per-stripe fingerprints for verification. Backend "nccl" (RCCL over xGMI) on GPUs,
"gloo" for the CPU tests.
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
