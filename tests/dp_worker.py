"""One rank of tests/test_gpu_mp.py (not a test module): a process of a world-size-2 gloo group on
cuda:0 that runs the real data-parallel path — dp.lockstep, the engine's MAX-all-reduced
calibration and flags, HIP-graph replay of the static-range forward, dp.gather_logits — on its
shard of every global batch, and saves the gathered logits (rank 0).

    python tests/dp_worker.py RANK WORLD PORT OUTDIR
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CASES = [("resnet18", "r18_u8"), ("resnet50", "r50_mixed")]
MODES = ("static", "dynamic")
GLOBAL_BATCH, STEPS, BATCHES = 8, 6, 3  # step 0 calibrates, 1-3 capture a graph per batch, 4-5 replay
# SMPQ_DPW_CFG (json) overrides these: the full per-rank size of BASELINE configs[3] is
# {"global_batch": 512, "steps": 7, "batches": 4, "cases": [["resnet50", "r50_mixed"]], "modes": ["static"]}
if os.environ.get("SMPQ_DPW_CFG"):
    import json
    _c = json.loads(os.environ["SMPQ_DPW_CFG"])
    GLOBAL_BATCH, STEPS, BATCHES = _c["global_batch"], _c["steps"], _c["batches"]
    CASES = [tuple(c) for c in _c["cases"]]
    MODES = tuple(_c["modes"])


def global_batches(dev):
    """The global batches every process (and the single-GPU reference) generates identically."""
    return [torch.randn(GLOBAL_BATCH, 3, 224, 224, generator=torch.Generator(device=dev).manual_seed(300 + b),
                        device=dev) for b in range(BATCHES)]


def model(arch, assign, dev):
    import resnet
    from smpq import assignments
    torch.manual_seed(0)
    net = getattr(resnet, arch)().to(dev).eval()
    assignments.apply_assignment(net, assign)
    return net


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from smpq import dp, engine, stats
    try:
        s, e = dp.shard_range(GLOBAL_BATCH, rank, world)
        shards = [x[s:e].contiguous() for x in global_batches(dev)]  # this rank's, resident
        for arch, assign in CASES:
            for mode in MODES:
                engine.set_range_mode(mode)
                net = model(arch, assign, dev)
                outs = []
                r0 = stats["graph_replays"]
                with torch.no_grad(), dp.lockstep():
                    for step in range(STEPS):
                        if step == 1:
                            c1 = stats["calibrations"]
                        y = net(shards[step % BATCHES])
                        outs.append(dp.gather_logits(y, world).cpu())
                if mode == "static":
                    assert stats["graph_replays"] > r0, "the static forward never replayed a graph"
                info = {"recalibrations_after_first": stats["calibrations"] - c1,
                        "graph_replays": stats["graph_replays"] - r0, "rows_per_rank": e - s}
                if rank == 0:
                    torch.save(outs, os.path.join(outdir, "%s_%s.pt" % (arch, mode)))
                    torch.save(info, os.path.join(outdir, "%s_%s_info.pt" % (arch, mode)))
        engine.set_range_mode("static")
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
