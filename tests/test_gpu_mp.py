"""The data-parallel path with two live processes: two ranks of a gloo group
share cuda:0 (tests/dp_worker.py), each forwards its shard of every global batch in dp.lockstep —
the first forward calibrates with the per-layer maxima MAX-all-reduced across the processes, the
later ones replay HIP graphs and MAX-reduce their overflow / staleness flags — and the logits are
all-gathered. The gathered logits must equal this process's single-GPU forward of the global batch
bit for bit, in static and dynamic range mode, for ResNet-18 u8 and ResNet-50 mixed."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(gpu, tmp_path, cfg=None):
    """Start the two ranks (tests/dp_worker.py, optional SMPQ_DPW_CFG) and return the worker module
    configured the same way."""
    import importlib
    import json
    sys.path.insert(0, HERE)
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    if cfg is not None:
        env["SMPQ_DPW_CFG"] = os.environ["SMPQ_DPW_CFG"] = json.dumps(cfg)
    else:
        env.pop("SMPQ_DPW_CFG", None)
        os.environ.pop("SMPQ_DPW_CFG", None)
    import dp_worker
    dp_worker = importlib.reload(dp_worker)
    world, port = 2, _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), str(r), str(world), str(port),
                               str(tmp_path)], env=env) for r in range(world)]
    try:
        rcs = [p.wait(timeout=600) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    return dp_worker


def _check(gpu, tmp_path, dp_worker):
    from smpq import engine
    xs = dp_worker.global_batches(gpu)
    try:
        for arch, assign in dp_worker.CASES:
            for mode in dp_worker.MODES:
                engine.set_range_mode(mode)
                net = dp_worker.model(arch, assign, gpu)
                got = torch.load(os.path.join(tmp_path, "%s_%s.pt" % (arch, mode)), weights_only=True)
                assert len(got) == dp_worker.STEPS
                with torch.no_grad():
                    for step in range(dp_worker.STEPS):
                        ref = net(xs[step % dp_worker.BATCHES]).cpu()
                        assert torch.equal(got[step], ref), (arch, mode, step, (got[step] - ref).abs().max().item())
    finally:
        engine.set_range_mode("static")


def test_two_process_dp_equals_single_gpu_bitwise(gpu, tmp_path):
    _check(gpu, tmp_path, _run(gpu, tmp_path))


def test_two_process_dp_full_per_rank_size(gpu, tmp_path):
    """the data-parallel path at BASELINE configs[3]'s per-rank size — 2 ranks x 256
    images of ResNet-50 mixed, static ranges, 4 distinct global batches (calibrate on the first,
    capture one graph per batch, replay): the gathered logits equal the one-process forward of
    each 512-image global batch bit for bit, and no rank recalibrates after the first forward."""
    cfg = {"global_batch": 512, "steps": 7, "batches": 4, "cases": [["resnet50", "r50_mixed"]], "modes": ["static"]}
    try:
        w = _run(gpu, tmp_path, cfg)
        info = torch.load(os.path.join(tmp_path, "resnet50_static_info.pt"), weights_only=True)
        assert info["rows_per_rank"] == 256 and info["recalibrations_after_first"] == 0, info
        assert info["graph_replays"] >= 2, info
        _check(gpu, tmp_path, w)
    finally:
        os.environ.pop("SMPQ_DPW_CFG", None)
