"""One process per GPU, torch.distributed over RCCL ("nccl" on ROCm) or gloo on CPU.

find_direction shards naturally: the seeds of a batch are independent images.  Every rank holds the
frozen networks, the full S table and an identical direction; rank r takes a contiguous slice of the
batch, and ONE all_reduce(SUM) per step combines the [8*512] direction gradient with the 4 loss
scalars (16.4 KB -- latency-bound over xGMI, so one fused buffer).  The reference has no distributed
code on this path; this is the build's single exchange step (section 8(e)).
"""
import os

import torch
import torch.distributed as dist


class World:
    def __init__(self, rank=0, world_size=1, local_rank=0, backend=None, device_index=None):
        self.rank, self.world_size, self.local_rank, self.backend = rank, world_size, local_rank, backend
        self.device_index = local_rank if device_index is None else device_index

    @property
    def distributed(self):
        return self.world_size > 1

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device_index])
            else:
                dist.barrier()

    def all_reduce_(self, t):
        if self.distributed:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def all_max(self, v, device):
        if not self.distributed:
            return float(v)
        t = torch.tensor([float(v)], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def init_from_env(use_cuda=True):
    """Read RANK / WORLD_SIZE / LOCAL_RANK (torch.distributed.run) and initialise the process group."""
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size <= 1:
        return World()
    # rehearsal knobs for a one-GPU box: SMC_DIST_BACKEND=gloo (RCCL refuses two ranks on one GPU) and
    # SMC_SHARE_GPU=1 (every rank on device 0); the production path is RCCL with one GPU per rank
    backend = os.environ.get("SMC_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    device_index = 0 if os.environ.get("SMC_SHARE_GPU") == "1" else local_rank
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if use_cuda:
        torch.cuda.set_device(device_index)
    if not dist.is_initialized():
        kw = {"device_id": torch.device("cuda", device_index)} if use_cuda and backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world_size, **kw)
    return World(rank, world_size, local_rank, backend, device_index)


def shard_rows(lo, hi, rank, world_size):
    """Contiguous slice [a, b) of rows [lo, hi) owned by `rank` (sizes differ by at most one)."""
    n = hi - lo
    base, extra = divmod(n, world_size)
    a = lo + rank * base + min(rank, extra)
    b = a + base + (1 if rank < extra else 0)
    return a, b
