"""One process per GPU, torch.distributed over RCCL ("nccl" on ROCm) or gloo on CPU.

find_direction shards naturally: the seeds of a batch are independent images.  Every rank holds the
frozen networks, the full S table and an identical direction; rank r takes a contiguous slice of the
batch.  The step's single exchange (the reference has no distributed code on this
path, section 2.3) is ONE all_gather of per-image rows -- each image's [8*512] direction gradient and its
4 loss terms, 16.4 KB a row, 4 rows per rank at batch 4: latency-bound over xGMI either way -- after which
every rank sums the global batch's rows in the same fixed order.  An all_reduce(SUM) would add the ranks'
partial sums in the collective's own order (ring chunks start at different ranks), so its result would
depend on the number of ranks; the gathered rows make the N-rank direction equal the 1-rank one bit for bit.
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

    def gather_rows(self, rows, lo, hi):
        """Every rank's rows of the global batch [lo, hi) (rank r holds shard_rows(lo, hi, r, N)) as one contiguous
        [hi - lo, F] tensor in global order, on every rank.  One all_gather of equal-size blocks (shards differ by at
        most one row: zero-padded).  Gloo has no device-tensor all_gather on every build: its rows go by the host."""
        if not self.distributed:
            return rows.contiguous()
        N = self.world_size
        cap = -(-(hi - lo) // N)
        feat = rows.shape[1]
        dev = rows.device
        host = self.backend != "nccl" and rows.is_cuda
        block = torch.zeros(cap, feat, dtype=rows.dtype, device="cpu" if host else dev)
        block[:rows.shape[0]] = rows.cpu() if host else rows
        parts = [torch.empty_like(block) for _ in range(N)]
        dist.all_gather(parts, block)
        out = torch.cat([parts[r][:b - a] for r, (a, b) in ((r, shard_rows(lo, hi, r, N)) for r in range(N))])
        return out.to(dev) if host else out

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
