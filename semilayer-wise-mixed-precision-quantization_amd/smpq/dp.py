"""Data-parallel inference over the GPUs of one node.

Images are independent units: rank r owns images [r*B/k, (r+1)*B/k) of a global batch, runs the
whole model on them, and the logits are all-gathered once (RCCL over xGMI on the GPU box; gloo in
the CPU tests). There is no other collective — batched ImageNet inference has no exchange step.
"""
import torch
import torch.distributed as dist


def shard_range(global_batch, rank, world):
    """[start, end) of this rank's images; the remainder goes to the lowest ranks."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_logits(local, world, out=None):
    """All-gather equal-size per-rank logits [b, C] into [world*b, C] in rank order."""
    if world == 1:
        return local
    local = local.contiguous()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
    dist.all_gather_into_tensor(out, local)
    return out


def sharded_forward(fn, x_global, rank, world):
    """Run ``fn`` on this rank's shard of ``x_global`` and return the gathered result."""
    s, e = shard_range(x_global.shape[0], rank, world)
    assert (e - s) * world == x_global.shape[0], "equal shards required for all_gather_into_tensor"
    return gather_logits(fn(x_global[s:e]), world)
