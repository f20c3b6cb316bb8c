#!/usr/bin/env python3
"""Diagnostics: which multi-stream capture sequence crashes (prints each step before it runs)."""
import faulthandler
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
faulthandler.enable()
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
import resnet  # noqa: E402
from smpq import assignments, engine  # noqa: E402

mode = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 7
dev = torch.device("cuda")
torch.manual_seed(0)
net = resnet.resnet50().to(dev).eval()
assignments.apply_assignment(net, "r50_mixed")
x = torch.randn(n, 3, 224, 224, device=dev)


def say(m):
    print(m, flush=True)


with torch.no_grad():
    engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0] = False, False, 1
    say("calibrate")
    net(x)
    say("serial eager")
    a = net(x)
    if mode == "ds_graph":  # bench-like: fork only inside _graph_forward (eager warm + capture)
        engine.CONCURRENT_DS[0], engine.USE_GRAPH[0] = True, True
    elif mode == "ds_eager_graph":
        engine.CONCURRENT_DS[0] = True
        say("ds eager")
        b = net(x)
        say("eq %s" % torch.equal(a, b))
        engine.USE_GRAPH[0] = True
    elif mode == "nods_graph":
        engine.USE_GRAPH[0] = True
    elif mode == "test_seq":
        x2 = torch.randn(n, 3, 224, 224, device=dev)
        for streams in (1, 2, 3):
            engine.STREAMS[0] = streams
            engine.CONCURRENT_DS[0], engine.USE_GRAPH[0] = True, False
            say("streams %d eager x" % streams)
            net(x)
            say("streams %d eager x2" % streams)
            net(x2)
            engine.USE_GRAPH[0] = True
            say("streams %d graph x (capture)" % streams)
            net(x)
            say("streams %d graph x2" % streams)
            net(x2)
            say("streams %d graph x" % streams)
            net(x)
        torch.cuda.synchronize()
    elif mode.startswith("recap"):
        # capture, then force a recapture (graph key change) in the same configuration
        engine.CONCURRENT_DS[0], engine.USE_GRAPH[0] = ("ds" in mode), True
        engine.STREAMS[0] = 2 if "sl" in mode else 1
        say("capture 1")
        net(x)
        net(x)
        for i in range(3):
            engine.FUSED_STEM[0] = not engine.FUSED_STEM[0]
            if "empty" in mode:
                import gc
                torch.cuda.synchronize()
                net._smpq_graph = None
                gc.collect()
                torch.cuda.empty_cache()
            say("recapture %d" % i)
            net(x)
            net(x)
        torch.cuda.synchronize()
    elif mode == "slices_graph":
        engine.STREAMS[0] = 2
        engine.USE_GRAPH[0] = True
    say("graph forward 1 (warm + capture)")
    c = net(x)
    say("eq %s" % torch.equal(a, c))
    say("graph forward 2 (replay)")
    d = net(x)
    torch.cuda.synchronize()
    say("eq %s" % torch.equal(a, d))
say("done")
