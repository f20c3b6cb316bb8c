#!/usr/bin/env python3
"""What the drop-in quantizer costs under the unmodified search driver.

resnet50_main.py:176-197 quantizes one channel per call — functions.channel_wise_quantizationperchan
(conv.weight.data, w_bit, cnum) — for every channel of a semilayer, then evaluates the model on the
validation loader (functions.evaluate_acc_loss_softmax, resnet50_main.py:201; imagenet.py:38-39:
batch 256, 50,000 images). This replays one such step on the GPU with the drop-in modules:

  * the per-channel calls for the largest R50 semilayer shape the driver meets (layer4's last conv3,
    2048 channels; a semilayer is the channels of one conv with one Δloss sign, so up to all of
    them), timed as the driver issues them (each call ends in a host sync: the reference raises
    ZeroDivisionError synchronously on a constant channel);
  * the evaluation that follows, on a synthetic loader of pinned host batches (256 images each),
    timed over a bounded number of batches and scaled to the 196 batches of ImageNet val.

usage: python tools/driver_quant_cost.py [--channels 1024] [--eval-batches 12] [--out F.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=1024, help="channels quantized in the semilayer")
    ap.add_argument("--eval-batches", type=int, default=12)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    import functions
    import resnet
    from smpq import assignments
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = resnet.resnet50().to(dev).eval()
    assignments.apply_assignment(net, "r50_mixed")
    conv = net.layer4[2].conv3
    g = torch.Generator().manual_seed(5)
    batches = [(torch.randn(256, 3, 224, 224, generator=g).pin_memory(), torch.randint(0, 1000, (256,), generator=g))
               for _ in range(2)]
    loader = [batches[i % 2] for i in range(args.eval_batches)]
    functions.evaluate_acc_loss_softmax(net, dev, loader[:3])  # warm: pack, calibrate, graphs
    res = {"semilayer_channels": args.channels, "conv": "layer4[2].conv3 (2048 x 512)"}
    for bits, name in ((6, "per_channel_calls"), (4, "per_channel_calls_repeat")):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for c in range(args.channels):  # resnet50_main.py:189-197, one channel per call
            conv.weight.data = functions.channel_wise_quantizationperchan(conv.weight.data, bits, c)
        torch.cuda.synchronize()
        res[name + "_s"] = round(time.perf_counter() - t0, 5)
    res["per_call_us"] = round(res["per_channel_calls_repeat_s"] / args.channels * 1e6, 2)
    # the evaluation after the semilayer: the weights changed, so it repacks and recalibrates once
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    functions.evaluate_acc_loss_softmax(net, dev, loader)
    torch.cuda.synchronize()
    t_eval = time.perf_counter() - t0
    res["eval_batches_timed"] = args.eval_batches
    res["eval_s_timed"] = round(t_eval, 4)
    per_batch = t_eval / args.eval_batches
    res["eval_s_imagenet_val_scaled"] = round(per_batch * 50000 / 256, 3)
    q = res["per_channel_calls_repeat_s"]
    res["quant_share_of_step"] = round(q / (q + res["eval_s_imagenet_val_scaled"]), 4)
    res["note"] = ("step = the semilayer's per-channel quantize calls + one evaluation over ImageNet val "
                   "(50,000 images, batch 256), the latter scaled from the timed host batches")
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
