#!/usr/bin/env python3
"""Headline benchmark: images/s of the ResNet-50 mixed 8/6/4-bit quantized forward
(BASELINE.json metric; configs[2] at N=1: batch 256 on one MI355X; configs[3] at N=8:
batch 2048 = 8 x 256, weak scaling, RCCL all-gather of logits).

python bench.py --gpus N --steps K --warmup W       (N > 1: launched by torch.distributed.run)

One step = one fused forward of 256 synthetic 224x224 images per GPU (inputs generated on
device, resident in HBM before the timed region) + the all-gather of the logits. Prints ONE
JSON line on rank 0 with the roofline of the dominant kernel (qconv_kernel, timed with HIP
events on its launch stream over the timed region) and the CPU baseline (the reference's
fp32 torch-CPU forward restated in oracle/torch_ref.py, timed on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd")
for _p in (PKG_DIR, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec ResNet-50 mixed 8/6/4b @224×224, 1/2/4/8 MI355X; % int8 roofline"
# MI355X dense int8 MFMA peak: v_mfma_i32_16x16x64_i8 = 2x the bf16 rate (MI355X_MICROARCH.md
# 'Matrix cores': I8 row), bf16 dense ~2.5 PF  ->  ~5.0 POPS dense (no sparsity).
INT8_DENSE_PEAK_TOPS = 5000.0
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    "r50_mixed": ("resnet50", "r50_mixed", "ResNet-50 mixed 8/6/4-bit (published semilayer assignment), 224x224"),
    "r18_u8": ("resnet18", "r18_u8", "ResNet-18 uniform int8 addressable convs, 224x224"),
    "r34_4bit": ("resnet34", "r34_4bit", "ResNet-34 4-bit-dominant semilayer mix, 224x224"),
}


class ConvTimer:
    """Events around every quantized-conv launch, on the stream it is launched on."""

    def __init__(self):
        self.recs = []
        self.active = False
        self._ev = None

    def begin(self):
        if self.active:
            self._ev = torch.cuda.Event(enable_timing=True)
            self._ev.record(torch.cuda.current_stream())

    def end(self, alg_ops, shape):
        if self.active:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(torch.cuda.current_stream())
            self.recs.append((self._ev, e1, alg_ops, shape))

    def summary(self):
        torch.cuda.synchronize()
        total_ms = sum(a.elapsed_time(b) for a, b, _, _ in self.recs)
        ops = sum(o for _, _, o, _ in self.recs)
        return len(self.recs), total_ms, ops


def cpu_baseline(arch, assign_name, budget_s=12.0):
    """The reference CPU path (fp32 torch forward on the fake-quantized weights) on host cores."""
    import numpy as np
    from oracle import quant_ref, torch_ref
    import resnet
    from smpq import assignments
    torch.manual_seed(0)
    net = getattr(resnet, arch)()
    sd = {k: v.clone() for k, v in net.state_dict().items() if not k.endswith(("qbits", "qstep"))}
    asg = assignments.load_assignment(assign_name)
    names = {id(m): n for n, m in net.named_modules()}
    for ln, cn, ch in zip(asg["lnum"], asg["cnum"], asg["chain"]):
        key = names[id(assignments.conv_for_lnum(net, int(ln)))] + ".weight"
        sd[key][cn] = torch.from_numpy(quant_ref.apply_chain(sd[key][cn].numpy(), [int(b) for b in ch if b]))
    threads = torch.get_num_threads()
    bs = 16
    x = torch.randn(bs, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    torch_ref.resnet_forward(arch, sd, x[:2])  # warm-up
    n_img, t0 = 0, time.perf_counter()
    while True:
        torch_ref.resnet_forward(arch, sd, x)
        n_img += bs
        el = time.perf_counter() - t0
        if el >= budget_s or n_img >= 4096:
            break
    del np
    return {"value": round(n_img / el, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": "%d images (batches of %d) of the fp32 torch-CPU reference forward on the same "
                      "fake-quantized %s, %.1f s" % (n_img, bs, arch, el)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step")
    ap.add_argument("--config", default="r50_mixed", choices=sorted(CONFIGS))
    ap.add_argument("--limbs", type=int, default=2, help="activation int8 limbs (2 = int16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--chunk", type=int, default=None, help="images per pass (Infinity-Cache blocking)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import __graft_entry__
    if rank == 0 or world == 1:
        __graft_entry__.build()
    if world > 1:
        dist.barrier()
        __graft_entry__.build()
    import resnet
    from smpq import assignments, dp, ops, stats

    arch, assign, desc = CONFIGS[args.config]
    ops.set_act_limbs(args.limbs)
    from smpq import engine
    if args.chunk:
        engine.set_chunk(args.chunk)
    torch.manual_seed(0)
    net = getattr(resnet, arch)().to(dev).eval()
    assignments.apply_assignment(net, assign)

    # this rank's shard of the global batch (dp.shard_range), generated on device
    s0, s1 = dp.shard_range(args.batch * world, rank, world)
    g = torch.Generator(device=dev).manual_seed(1000 + s0)
    x = torch.randn(s1 - s0, 3, 224, 224, generator=g, device=dev)
    gathered = torch.empty(world * args.batch, 1000, device=dev) if world > 1 else None

    def step():
        with torch.no_grad():
            y = net(x)
            return dp.gather_logits(y, world, out=gathered)

    for _ in range(args.warmup):
        step()
    if rank == 0:
        print("autotuned tiles:", {"x".join(map(str, k[:8])): v for k, v in ops._TUNED.items()},
              file=sys.stderr, flush=True)
    timer = ConvTimer()
    ops.set_conv_hook(timer)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    h0 = stats["hip_conv"]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    timer.active = False
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    hip_convs = stats["hip_conv"] - h0
    n_launch, kern_ms, alg_ops = timer.summary()
    ops.set_conv_hook(None)

    images = args.batch * world * args.steps
    value = images / elapsed
    per_launch_ops = alg_ops / max(n_launch, 1)
    avg_ms = kern_ms / max(n_launch, 1)
    achieved_tops = per_launch_ops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "i8",
            "data": "synthetic (N(0,1) 224x224 on device; seeded random-init weights, reference init)",
            "config": {"workload": desc, "assignment": assign, "batch_per_gpu": args.batch,
                       "global_batch": args.batch * world, "act_limbs": args.limbs,
                       "act_code": {1: "int8", 2: "int16 (2 int8 limbs)", 3: "int24 (3 int8 limbs)"}[args.limbs],
                       "parallelism": "dp%d" % world, "quantized_convs_per_step": hip_convs // max(args.steps, 1),
                       "range_mode": engine.get_range_mode(), "chunk": engine.CHUNK[0]},
            "roofline": {"bound": "mfma", "kernel": "qconv_kernel", "achieved": round(achieved_tops, 2),
                         "peak": INT8_DENSE_PEAK_TOPS, "unit": "TFLOP/s",
                         "frac": round(achieved_tops / INT8_DENSE_PEAK_TOPS, 4), "traffic": None,
                         "alg_ops_per_launch": per_launch_ops, "avg_launch_ms": round(avg_ms, 5),
                         "launches": n_launch, "mfma_passes_per_alg_op": args.limbs,
                         "kernel_share_of_step": round(kern_ms / (elapsed * 1e3), 4)},
        }
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(arch, assign, args.cpu_budget)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
