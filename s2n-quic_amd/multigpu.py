"""Multi-GPU driver pieces: one process per GPU, packets sharded by contiguous ranges, no data-path collective.

Packets are independent, so a batch shards across the node's GPUs with a per-GPU split only:
rank r owns packets [r*n, (r+1)*n) of the job, its own key table replica and its own HIP stream.  The only
inter-process traffic is control: a barrier before and after the timed region and a max over ranks of the
elapsed time, carried by torch.distributed over gloo on CPU tensors (RCCL is never needed: there is no
exchange step in the data path).
"""
import os


def env_rank():
    """(rank, world, local_rank) from torchrun's environment (single process: 0, 1, 0)."""
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def shard(rank, world, n_per_rank, seed_base):
    """The contiguous packet range of one rank (weak scaling: n_per_rank fixed as world grows) and the seed of
    its synthetic data.  PN ranges never overlap, so no (key, nonce) pair repeats across GPUs."""
    first = rank * n_per_rank
    return {"first": first, "count": n_per_rank, "pn_base": first, "seed": seed_base + 7919 * rank}


class Control:
    """Barrier + max-over-ranks for the timed region; a no-op for one process."""

    def __init__(self, world, backend="gloo"):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist

            if not dist.is_initialized():
                dist.init_process_group(backend)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return float(x)
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if not self.dist:
            return float(x)
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()
