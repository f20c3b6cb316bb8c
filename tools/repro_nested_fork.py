#!/usr/bin/env python3
"""Minimal torch-only reproduction of the host segfault in hipStreamEndCapture seen when a
batch-slice stream forks a downsample side stream inside a graph capture (gpurun_out/dsin_tests.log,
round 2). No smpq code: plain torch ops on the same stream topology as engine._forward with
CONCURRENT_DS inside slices — capture-stream -> slice streams -> side streams (nested fork), the
side stream's allocation consumed on the slice stream after the join, then a RECAPTURE.

    python tools/repro_nested_fork.py            # runs every mode in its own child process
    python tools/repro_nested_fork.py <mode>     # one mode

Modes: flat (one fork level), nested (slice -> side), nested_recapture (capture twice),
nested_recapture_rs (record_stream on the side allocation), nested_recapture_del (free the first
graph before the second capture)."""
import faulthandler
import subprocess
import sys

MODES = ["flat", "flat_recapture", "nested", "nested_recapture", "nested_recapture_rs", "nested_recapture_del"]


def run(mode):
    import torch
    faulthandler.enable()
    dev = torch.device("cuda")
    x = torch.randn(2, 1 << 20, device=dev)
    slices = [torch.cuda.Stream() for _ in range(2)]
    sides = [torch.cuda.Stream() for _ in range(2)]
    nested = mode.startswith("nested")

    def body(x):
        main = torch.cuda.current_stream()
        outs = []
        for s in slices:
            s.wait_stream(main)
        for i, sl in enumerate(slices):
            with torch.cuda.stream(sl):
                a = x[i] * 2.0
                if nested:
                    sd = sides[i]
                    sd.wait_stream(sl)
                    with torch.cuda.stream(sd):
                        b = a + 1.0  # allocated on the side stream
                    c = a * 3.0
                    sl.wait_stream(sd)  # join before the consumer
                    if mode.endswith("_rs"):
                        b.record_stream(sl)
                    outs.append(b + c)
                else:
                    outs.append(a + 1.0)
        for s in slices:
            main.wait_stream(s)
        return torch.stack(outs)

    want = body(x)
    torch.cuda.synchronize()
    graphs = []
    for k in range(2 if "recapture" in mode else 1):
        if mode.endswith("_del") and graphs:
            graphs.clear()
            torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        print("%s: capture %d" % (mode, k), flush=True)
        with torch.cuda.graph(g):
            y = body(x)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, want), mode
        graphs.append((g, y))
    print("%s: ok" % mode, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for m in MODES:
            rc = subprocess.call([sys.executable, __file__, m], timeout=120)
            print("mode %-24s exit %d%s" % (m, rc, "  (SIGSEGV)" if rc == -11 else ""), flush=True)
