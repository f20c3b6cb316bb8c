#!/usr/bin/env python3
"""Throughput of the drop-in evaluation loop (functions.evaluate_acc_loss_softmax, the reference's
functions.py:84-129) when the batches come from the host, as the reference's DataLoader delivers
them (pin_memory=True, imagenet.py), against the same loop on device-resident batches.

    python tools/eval_host_batches.py [--batches 8] [--batch 256] [--config r50_mixed] [--out PATH]

Prints one JSON object: images/s for pinned host batches, pageable host batches and device batches
(each the second of two evaluations of the same loader: the first calibrates and captures graphs),
and the host/device ratios.
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

import __graft_entry__  # noqa: E402

ARCH = {"r50_mixed": "resnet50", "r18_u8": "resnet18", "r34_4bit": "resnet34"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--config", default="r50_mixed")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    __graft_entry__.build()
    import functions
    import resnet
    from smpq import assignments, stats
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = getattr(resnet, ARCH[args.config])().to(dev).eval()
    assignments.apply_assignment(net, args.config)
    g = torch.Generator().manual_seed(5)
    host = [(torch.randn(args.batch, 3, 224, 224, generator=g), torch.randint(0, 1000, (args.batch,), generator=g))
            for _ in range(args.batches)]
    pinned = [(x.pin_memory(), y.pin_memory()) for x, y in host]
    device = [(x.to(dev), y.to(dev)) for x, y in host]
    res = {"workload": "%s, %d batches of %d images, functions.evaluate_acc_loss_softmax" % (
        args.config, args.batches, args.batch)}
    accs = {}
    keys = ("calibrations", "overflow_reruns", "stale_reruns", "graph_captures", "graph_replays")

    class Stamped:
        """The loader, with the host time at which each batch is handed out."""
        def __init__(self, items):
            self.items, self.t = items, []

        def __iter__(self):
            for it in self.items:
                self.t.append(time.perf_counter())
                yield it
    for name, loader in (("device", device), ("pinned_host", pinned), ("pageable_host", host)):
        functions.evaluate_acc_loss_softmax(net, dev, loader)  # calibration + graph captures
        best = None
        for _ in range(args.reps):
            st = Stamped(loader)
            s0 = {k: stats[k] for k in keys}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            acc, loss, _ = functions.evaluate_acc_loss_softmax(net, dev, st)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            if best is None or el < best:
                best = el
                res[name + "_engine_events"] = {k: stats[k] - s0[k] for k in keys}
                res[name + "_batch_ms"] = [round((b - a) * 1e3, 2) for a, b in zip([t0] + st.t, st.t + [t0 + el])]
        accs[name] = (acc, loss)
        res[name + "_img_s"] = round(args.batches * args.batch / best, 1)
        print(name, res[name + "_img_s"], "img/s", res[name + "_engine_events"], res[name + "_batch_ms"], flush=True)
    assert accs["pinned_host"] == accs["device"] == accs["pageable_host"], accs  # same results bit for bit
    res["pinned_over_device"] = round(res["pinned_host_img_s"] / res["device_img_s"], 4)
    res["pageable_over_device"] = round(res["pageable_host_img_s"] / res["device_img_s"], 4)
    res["timing"] = "best of %d evaluations after one warm-up evaluation per loader" % args.reps
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
