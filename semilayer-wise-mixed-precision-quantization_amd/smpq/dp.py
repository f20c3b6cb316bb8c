"""Data-parallel inference over the GPUs of one node.

Images are independent units: rank r owns images [r*B/k, (r+1)*B/k) of a global batch, runs the
whole model on them, and the logits are all-gathered once (RCCL over xGMI on the GPU box; gloo in
the CPU tests). The data path has no other collective — batched ImageNet inference has no exchange
step. The static-range engine adds two control collectives of a few bytes while the ranks run in
``lockstep``: the MAX of the per-layer calibration maxima (so every rank uses the ranges of the
whole global batch and the gathered logits equal the single-GPU logits bit for bit) and the MAX of
the per-forward overflow / staleness flags (so the ranks recalibrate together).
"""
import contextlib

import torch
import torch.distributed as dist


def shard_range(global_batch, rank, world):
    """[start, end) of this rank's images; the remainder goes to the lowest ranks."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_logits(local, world, out=None, group=None):
    """All-gather equal-size per-rank logits [b, C] into [world*b, C] in rank order (RCCL over
    xGMI; a gloo group — the multi-process tests that share one GPU — gathers through the host)."""
    if world == 1:
        return local
    local = local.contiguous()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, local.cpu(), group=group)
        out.copy_(h)
        return out
    dist.all_gather_into_tensor(out, local, group=group)
    return out


@contextlib.contextmanager
def lockstep(group=None):
    """Within this block every rank of ``group`` (default: the whole world) runs the same
    sequence of static-range forwards on its shard of each global batch (smpq.engine
    set_dp_group); outside it each process calibrates on its own inputs."""
    from smpq import engine
    old = engine.get_dp_group()
    use = group if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    engine.set_dp_group(use if (use is not None and dist.get_world_size(use) > 1) else None)
    try:
        yield
    finally:
        engine.set_dp_group(old)


def sharded_forward(fn, x_global, rank, world):
    """Run ``fn`` on this rank's shard of ``x_global`` and return the gathered result."""
    s, e = shard_range(x_global.shape[0], rank, world)
    assert (e - s) * world == x_global.shape[0], "equal shards required for all_gather_into_tensor"
    return gather_logits(fn(x_global[s:e]), world)


def all_reduce_stats(stats, world):
    """Sum per-rank evaluation accumulators (smpq_softmax_xent's [loss_sum, correct, seen,
    batches] or smpq_kl_rows' [kl_sum, rows], float64) over ranks: the only collective the
    sharded evaluation needs (SURVEY.md 8(f) rank 1 — a few scalars instead of the logits)."""
    if world > 1:
        if stats.is_cuda and dist.get_backend() == "gloo":
            h = stats.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            stats.copy_(h)
        else:
            dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    return stats


def sharded_eval(net, loader, rank, world, device=None, keep_probs=True):
    """functions.evaluate_acc_loss_softmax (functions.py:84-129) with every global batch split
    over the ranks (equal shards): each rank forwards its images, the fused softmax / CE / top-1
    kernel accumulates on its device, and one all-reduce of 4 doubles combines the ranks.
    Returns (acc, loss, this rank's softmax shards) — the shards stay where they were made and
    feed sharded_kldiv, so no logits or probabilities cross xGMI."""
    from smpq import engine, ops
    from smpq.batches import DeviceBatches
    from smpq.models import ResNet
    dev = device or torch.device("cuda", torch.cuda.current_device())
    stats = torch.zeros(4, dtype=torch.float64, device=dev)
    probs = []
    if isinstance(net, ResNet):
        engine.new_evaluation(net)  # as functions.evaluate_acc_loss_softmax (history-independent)

    def shards():
        for x, y in loader:
            s, e = shard_range(x.shape[0], rank, world)
            assert (e - s) * world == x.shape[0], "equal shards required (the batch mean of shard means)"
            yield x[s:e], y[s:e]
    with torch.no_grad(), lockstep():
        # this rank's shards reach the device as functions.evaluate_acc_loss_softmax's batches do:
        # the next one's copy on a side stream while this one runs
        for x, y in DeviceBatches(shards(), dev):
            out = net(x).float().contiguous()
            p = ops.softmax_xent(out, y, stats, want_probs=keep_probs)
            if keep_probs:
                probs.append(p)
    loss_sum, correct, seen, count = all_reduce_stats(stats, world).tolist()
    return correct / seen, loss_sum / count, probs


def sharded_kldiv(n_out_local, out_local, world):
    """functions.KLdiv (functions.py:131-149) over softmax shards held per rank: per-rank
    smpq_kl_rows sums, then one all-reduce of 2 doubles."""
    from smpq import ops
    stats = None
    for p, q in zip(n_out_local, out_local):
        if stats is None:
            stats = torch.zeros(2, dtype=torch.float64, device=q.device)
        ops.kl_rows(p, q, stats)
    s, n = all_reduce_stats(stats, world).tolist()
    return s / n
