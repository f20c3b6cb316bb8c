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


def test_two_process_dp_equals_single_gpu_bitwise(gpu, tmp_path):
    sys.path.insert(0, HERE)
    import dp_worker
    from smpq import engine
    world, port = 2, _free_port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), str(r), str(world), str(port),
                               str(tmp_path)], env=env) for r in range(world)]
    try:
        rcs = [p.wait(timeout=600) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    xs = dp_worker.global_batches(gpu)
    try:
        for arch, assign in dp_worker.CASES:
            for mode in ("static", "dynamic"):
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
