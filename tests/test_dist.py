"""World-size-2 gloo tests of the data-parallel sharding + logits all-gather (CPU). The real model
path with two live processes on the GPU is tests/test_gpu_mp.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(x):
    """The reference's CPU forward of a seeded ResNet-18 (oracle.torch_ref: the torch operators of
    resnet.py:204-220), in float64 so that every image's logits are the same bits in any batch."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (repo, os.path.join(repo, "semilayer-wise-mixed-precision-quantization_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import resnet
    from oracle import torch_ref
    torch.manual_seed(0)
    sd = {k: v.double() for k, v in resnet.resnet18().state_dict().items() if v.is_floating_point()}
    return torch_ref.resnet_forward("resnet18", sd, x.double())


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "semilayer-wise-mixed-precision-quantization_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from smpq import dp
        x = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(1))
        y = dp.sharded_forward(_model, x, rank, world)
        q.put((rank, y))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_forward_equals_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    ref = _model(x)
    assert ref.shape == (8, 1000)
    for r in range(world):
        assert torch.equal(res[r], ref)


def test_shard_range_covers_batch():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "semilayer-wise-mixed-precision-quantization_amd"))
    from smpq import dp
    for b in (1, 7, 256, 2048):
        for w in (1, 2, 3, 8):
            spans = [dp.shard_range(b, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == b
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def _stats_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "semilayer-wise-mixed-precision-quantization_amd"))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np
        from oracle import eval_ref
        from smpq import dp
        # each rank holds its shard of every global batch; per-rank accumulators as the kernel
        # (smpq_softmax_xent) forms them: [sum of shard-mean CE, correct, rows, batches]
        g = torch.Generator().manual_seed(5)
        st = torch.zeros(4, dtype=torch.float64)
        for _ in range(3):
            x = torch.randn(8, 50, generator=g).numpy()
            y = torch.randint(0, 50, (8,), generator=g).numpy()
            s, e = dp.shard_range(8, rank, world)
            acc, loss, _ = eval_ref.evaluate_acc_loss_softmax([(x[s:e], y[s:e])])
            st += torch.tensor([loss, acc * (e - s), e - s, 1.0], dtype=torch.float64)
        q.put((rank, dp.all_reduce_stats(st, world).tolist()))
        del np
    finally:
        dist.destroy_process_group()


def test_sharded_eval_stats_all_reduce_equals_single_process():
    """The sharded evaluation's only collective: 4 doubles summed over ranks reproduce the
    single-process accuracy and mean batch loss of functions.py:84-129 (equal shards)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import eval_ref
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(3):
        x = torch.randn(8, 50, generator=g).numpy()
        y = torch.randint(0, 50, (8,), generator=g).numpy()
        batches.append((x, y))
    acc, loss, _ = eval_ref.evaluate_acc_loss_softmax(batches)
    for r in range(world):
        loss_sum, correct, seen, count = res[r]
        assert res[r] == res[0]
        assert abs(correct / seen - acc) < 1e-12
        assert abs(loss_sum / count - loss) < 1e-9


def _calib_worker(rank, world, port, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "semilayer-wise-mixed-precision-quantization_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import resnet
        from smpq import dp, engine
        from smpq.qconv import QConv2d
        torch.manual_seed(0)
        net = resnet.resnet18()
        convs = [m for m in net.modules() if isinstance(m, QConv2d)]
        # this rank's per-layer calibration maxima (its shard of the global batch)
        g = torch.Generator().manual_seed(100 + rank)
        c = engine.Calibration()
        c.keys = [id(m) for m in convs]
        c.maxima = torch.rand(len(convs), generator=g) * (1 + rank)
        c.logits, c.fp, c.changed, c.sig0 = None, None, True, None
        local = c.maxima.clone()
        with dp.lockstep():
            assert engine.get_dp_group() is not None
            engine._dp_max_(c.maxima)
            # the collective decision: one rank's flag makes every rank recalibrate
            need = torch.tensor([1 if rank == world - 1 else 0], dtype=torch.int32)
            engine._dp_max_(need)
        assert engine.get_dp_group() is None
        engine.set_calibration(net, c)
        ranges = [net._smpq_ranges[0][k] for k in c.keys]
        q.put((rank, local, ranges, int(need.item())))
    finally:
        dist.destroy_process_group()


def test_calibration_maxima_all_reduced_across_ranks():
    """Data-parallel static ranges (engine.set_dp_group / dp.lockstep): every rank ends with the
    ranges HEADROOM * (max over ranks of its per-layer maxima) = the single-process calibration of
    the global batch, and a recalibration decision on any rank is taken by all."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calib_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (loc, rng, need)) for r, loc, rng, need in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "semilayer-wise-mixed-precision-quantization_amd"))
    from smpq import engine
    gmax = torch.maximum(res[0][0], res[1][0])
    want = [max(v, 1e-30) * engine.HEADROOM for v in gmax.tolist()]
    for r in range(world):
        assert res[r][1] == want
        assert res[r][2] == 1
