#!/usr/bin/env python3
"""Host cost of replaying the captured R50 forward graph, and the step time, for several batch-slice counts.

For each slice count: the host wall time of CUDAGraph.replay() itself (the call
returns once every node is enqueued) and the GPU step time (replay + sync) over a few replays.
A second slice can only start once its first node has been enqueued, so a replay() that takes
milliseconds on the host delays the second slice by about the first slice's share of it.

usage: python tools/graph_launch_probe.py [--reps 10]
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--settings", default="1,2,3,4")
    args = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    import resnet
    from smpq import assignments, engine
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = resnet.resnet50().to(dev).eval()
    assignments.apply_assignment(net, "r50_mixed")
    x = torch.randn(256, 3, 224, 224, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    out = []
    with torch.no_grad():
        net(x)  # calibrate
        for st in args.settings.split(","):
            nst = int(st)
            engine.STREAMS[0] = nst
            for _ in range(3):
                net(x)  # eager + capture for this layout
            per = net._smpq_graphs
            g = [v for k, v in per.items() if k != "base"][0][0]
            host, step = [], []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.replay()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                host.append((t1 - t0) * 1e3)
                step.append((t2 - t0) * 1e3)
            host.sort()
            step.sort()
            r = {"slices": nst, "replay_host_ms": round(host[len(host) // 2], 3),
                 "step_ms": round(step[len(step) // 2], 3)}
            out.append(r)
            print(json.dumps(r), flush=True)
    return out


if __name__ == "__main__":
    main()
