"""GPU parity of the evaluation reductions (smpq_softmax_xent / smpq_kl_rows) against the
reference's own outputs (tests/golden/eval_golden.npz: functions.py:84-149 run by the reference)
and the float64 oracle (oracle/eval_ref.py). Tolerances: softmax rtol 2e-6 (fp32 exp / division,
a few ulp), loss / KL rel 2e-6, top-1 accuracy exact."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import eval_ref

pytestmark = pytest.mark.gpu


def _golden():
    z = np.load(os.path.join(GOLDEN, "eval_golden.npz"), allow_pickle=False)
    cuts = np.cumsum([0] + list(z["sizes"]))
    split = lambda a: [torch.from_numpy(a[cuts[i]:cuts[i + 1]].copy()) for i in range(len(cuts) - 1)]  # noqa
    return z, split


def test_evaluate_acc_loss_softmax_vs_reference(gpu):
    import functions
    z, split = _golden()
    net = torch.nn.Identity()  # the 'images' of the loader are the logits (make_golden.py)
    for tag in ("a", "b"):
        loader = list(zip(split(z["logits_" + tag]), split(z["labels"])))
        acc, loss, outs = functions.evaluate_acc_loss_softmax(net, gpu, loader)
        assert abs(acc - float(z["acc_" + tag])) < 1e-7
        assert abs(loss - float(z["loss_" + tag])) <= 2e-6 * abs(float(z["loss_" + tag]))
        got = torch.cat(outs).cpu().numpy()
        np.testing.assert_allclose(got, z["softmax_" + tag], rtol=2e-6, atol=1e-12)
        assert all(o.is_cuda for o in outs)
        assert abs(functions.evaluate_loss(net, gpu, loader) - loss) == 0.0


def test_kldiv_vs_reference(gpu):
    import functions
    z, split = _golden()
    p = [t.to(gpu) for t in split(z["softmax_a"])]
    q = [t.to(gpu) for t in split(z["softmax_b"])]
    kl = functions.KLdiv(p, q)
    assert abs(kl - float(z["kl"])) <= 2e-6 * abs(float(z["kl"]))


@pytest.mark.parametrize("rows,cols", [(256, 1000), (1, 1000), (3, 7), (65, 129)])
def test_softmax_xent_vs_oracle(gpu, rows, cols):
    from smpq import ops
    g = torch.Generator().manual_seed(rows * 1000 + cols)
    x = torch.randn(rows, cols, generator=g) * 4
    y = torch.randint(0, cols, (rows,), generator=g)
    y[: rows // 3] = x[: rows // 3].argmax(1)  # some correct rows
    stats = torch.zeros(4, dtype=torch.float64, device=gpu)
    p = ops.softmax_xent(x.to(gpu), y, stats)
    acc, loss, outs = eval_ref.evaluate_acc_loss_softmax([(x.numpy(), y.numpy())])
    loss_sum, correct, seen, count = stats.tolist()
    assert seen == rows and count == 1 and correct / seen == acc
    assert abs(loss_sum - loss) <= 2e-6 * abs(loss)
    np.testing.assert_allclose(p.cpu().numpy(), outs[0], rtol=3e-6, atol=1e-12)
    # accumulation over calls, bitwise reproducible
    stats2 = torch.zeros(4, dtype=torch.float64, device=gpu)
    for _ in range(2):
        ops.softmax_xent(x.to(gpu), y, stats2, want_probs=False)
    assert stats2.tolist() == [2 * v for v in stats.tolist()]


def test_kl_rows_vs_oracle_and_deterministic(gpu):
    from smpq import ops
    g = torch.Generator().manual_seed(3)
    a = torch.softmax(torch.randn(300, 1000, generator=g), 1)
    b = torch.softmax(torch.randn(300, 1000, generator=g), 1)
    ref = eval_ref.kldiv([a.numpy()], [b.numpy()])
    s1 = torch.zeros(2, dtype=torch.float64, device=gpu)
    s2 = torch.zeros(2, dtype=torch.float64, device=gpu)
    ops.kl_rows(a.to(gpu), b.to(gpu), s1)
    ops.kl_rows(a.to(gpu), b.to(gpu), s2)
    assert s1.tolist() == s2.tolist() and s1[1].item() == 300
    assert abs(s1[0].item() / 300 - ref) <= 2e-6 * abs(ref)


def test_sharded_eval_world1_equals_functions(gpu):
    import functions
    from smpq import dp
    z, split = _golden()
    loader = [(x[:4], y[:4]) for x, y in zip(split(z["logits_a"]), split(z["labels"]))]
    acc, loss, outs = functions.evaluate_acc_loss_softmax(torch.nn.Identity(), gpu, loader)
    acc2, loss2, outs2 = dp.sharded_eval(torch.nn.Identity(), loader, 0, 1, device=gpu)
    assert (acc, loss) == (acc2, loss2)
    assert dp.sharded_kldiv(outs, outs2, 1) == functions.KLdiv(outs, outs2) == 0.0


def test_eval_kernels_reject_bad_input(gpu):
    from smpq import _lib, ops
    stats = torch.zeros(4, dtype=torch.float64, device=gpu)
    with pytest.raises(ValueError):
        ops.softmax_xent(torch.randn(4, 10, device=gpu).double(), torch.zeros(4, dtype=torch.long), stats)
    with pytest.raises(_lib.SmpqError):
        _lib.check(_lib.load().smpq_softmax_xent(None, None, 4, 10, None, None, None, _lib.stream_ptr()), "x")


def test_repeated_evaluations_keep_graphs_and_host_batches_match(gpu):
    """The reference calls net.to(device) on every evaluation (functions.py:97): a no-op .to() keeps
    the engine's packed weights, calibration and graphs, so a second evaluation of the same loader
    captures and repacks nothing (it recalibrates on its first batch, engine.new_evaluation).
    Host batches (pageable and pinned: DeviceBatches copies them on a side stream) give the same
    results bit for bit as device batches, and a .to() that really moves the model drops the caches
    and still gives the same results."""
    import functions
    from smpq import stats
    from test_gpu import build_model
    net = build_model(gpu, "resnet18", "r18_u8")
    g = torch.Generator().manual_seed(12)
    host = [(torch.randn(6, 3, 224, 224, generator=g), torch.randint(0, 1000, (6,), generator=g)) for _ in range(4)]
    on_dev = [(x.to(gpu), y.to(gpu)) for x, y in host]
    pinned = [(x.pin_memory(), y.pin_memory()) for x, y in host]

    def same(r, ref):
        return r[0] == ref[0] and r[1] == ref[1] and all(torch.equal(a, b) for a, b in zip(r[2], ref[2]))
    ref = functions.evaluate_acc_loss_softmax(net, gpu, on_dev)
    keys = ("graph_captures", "repack", "calibrations", "graph_replays")
    s0 = {k: stats[k] for k in keys}
    again = functions.evaluate_acc_loss_softmax(net, gpu, on_dev)
    d = {k: stats[k] - s0[k] for k in keys}
    assert d["graph_captures"] == 0 and d["repack"] == 0 and d["calibrations"] == 1 and d["graph_replays"] == 3, d
    assert same(again, ref)
    for loader in (host, pinned):
        assert same(functions.evaluate_acc_loss_softmax(net, gpu, loader), ref)
    net.cpu()
    net.to(gpu)
    r0 = stats["repack"]
    assert same(functions.evaluate_acc_loss_softmax(net, gpu, on_dev), ref)
    assert stats["repack"] > r0


def test_host_batches_staged_during_graph_capture(gpu):
    """DeviceBatches stages batch i+1 on a worker thread while batch i runs, and a
    forward on a new input address captures a HIP graph. A loader that is slow in __next__ makes the
    worker's device work (pinned copy, side-stream allocation and copy, event) fall inside the
    capture window; engine.CAPTURE_LOCK makes it wait for the capture. Results equal the
    device-resident loader's bit for bit, and graphs were captured meanwhile."""
    import time

    import functions
    from smpq import stats
    from test_gpu import build_model
    net = build_model(gpu, "resnet18", "r18_u8")
    g = torch.Generator().manual_seed(13)
    host = [(torch.randn(6, 3, 224, 224, generator=g), torch.randint(0, 1000, (6,), generator=g)) for _ in range(6)]
    on_dev = [(x.to(gpu), y.to(gpu)) for x, y in host]

    class Slow:
        def __iter__(self):
            for i, b in enumerate(host):
                if i:
                    time.sleep(0.02 * i)  # staggered: some stagings land inside a capture
                yield b
    c0 = stats["graph_captures"]
    runs = [functions.evaluate_acc_loss_softmax(net, gpu, Slow()) for _ in range(2)]
    assert stats["graph_captures"] > c0  # the first slow evaluation captured its graphs
    ref = functions.evaluate_acc_loss_softmax(net, gpu, on_dev)
    for r in runs:
        assert r[0] == ref[0] and r[1] == ref[1] and all(torch.equal(a, b) for a, b in zip(r[2], ref[2]))


def test_pinned_dataloader_batches_during_graph_capture(gpu):
    """the reference's loader (imagenet.py:36-40: num_workers=16, pin_memory=True) pins
    each batch on torch's pin-memory THREAD, which allocates pinned host memory while the main
    thread may be capturing a HIP graph. engine._capture uses capture_error_mode='thread_local',
    so those calls stay legal; the results equal the device-resident loader's bit for bit and
    graphs were captured meanwhile."""
    import functions
    from smpq import stats
    from test_gpu import build_model
    net = build_model(gpu, "resnet18", "r18_u8")
    g = torch.Generator().manual_seed(17)
    xs = torch.randn(36, 3, 224, 224, generator=g)
    ys = torch.randint(0, 1000, (36,), generator=g)
    ds = torch.utils.data.TensorDataset(xs, ys)
    loader = torch.utils.data.DataLoader(ds, batch_size=6, shuffle=False, num_workers=2, pin_memory=True,
                                         multiprocessing_context="fork")
    on_dev = [(xs[i:i + 6].to(gpu), ys[i:i + 6].to(gpu)) for i in range(0, 36, 6)]
    c0 = stats["graph_captures"]
    runs = [functions.evaluate_acc_loss_softmax(net, gpu, loader) for _ in range(2)]
    assert stats["graph_captures"] > c0
    ref = functions.evaluate_acc_loss_softmax(net, gpu, on_dev)
    for r in runs:
        assert r[0] == ref[0] and r[1] == ref[1] and all(torch.equal(a, b) for a, b in zip(r[2], ref[2]))
