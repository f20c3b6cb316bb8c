#!/usr/bin/env python3
"""Timeline of the graph-replayed R50 forward WITHOUT a profiler (rocprofv3's per-dispatch
overhead distorts when the second batch slice starts): a one-lane stamp kernel
(tools/stamp_kernel.hip, built into tools/bin/libstamp.so) stores s_memrealtime (100 MHz) before
and after every quantized conv; the stamps are captured into the graph like the convs.

usage: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/stamp_kernel.hip -o tools/bin/libstamp.so
       python tools/timeline_probe.py [--streams 2] [--reps 5]
Prints per slice: first/last stamp, busy time (sum of conv spans), and the layer timeline.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


class StampHook:
    def __init__(self, lib, buf):
        self.lib, self.buf, self.n, self.rec = lib, buf, 0, []
        self.active = False

    def _stamp(self):
        s = torch.cuda.current_stream()
        i = self.n
        self.n += 1
        self.lib.stamp_launch(ctypes.c_void_p(self.buf.data_ptr()), i, ctypes.c_void_p(s.cuda_stream))
        return i, s.cuda_stream

    def begin(self):
        if self.active:
            self._b = self._stamp()

    def end(self, work):
        if self.active:
            e = self._stamp()
            self.rec.append((self._b[0], e[0], self._b[1], work.get("shape", "?")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    import resnet
    from smpq import assignments, engine, ops
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "bin", "libstamp.so"))
    lib.stamp_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    engine.STREAMS[0] = args.streams
    torch.manual_seed(0)
    net = resnet.resnet50().to(dev).eval()
    assignments.apply_assignment(net, "r50_mixed")
    x = torch.randn(args.batch, 3, 224, 224, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    buf = torch.zeros(4096, dtype=torch.int64, device=dev)
    hook = StampHook(lib, buf)
    ops.set_conv_hook(hook)
    with torch.no_grad():
        net(x)  # calibrate (no stamps)
        hook.active = True
        net(x)  # eager pass + capture: the capture records stamp nodes with their own indices
        rec = hook.rec[len(hook.rec) // 2:]  # the captured half (the eager half came first)
        hook.active = False
        import time
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            net(x)  # replay
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
    st = buf.cpu().tolist()
    t0 = min(st[b] for b, e, s, sh in rec)
    lanes = {}
    for b, e, s, sh in rec:
        lanes.setdefault(s, []).append((b, e, sh))
    print("replay wall (host) %.3f ms; stamps %d; slices %d" % (wall, hook.n, len(lanes)))
    for k, (s, lst) in enumerate(lanes.items()):
        t_first = (st[lst[0][0]] - t0) / 100.0
        t_last = (st[lst[-1][1]] - t0) / 100.0
        busy = sum(st[e] - st[b] for b, e, _ in lst) / 100.0
        print("slice %d: %d convs, first start %.1f us, last end %.1f us, busy %.1f us" % (k, len(lst), t_first * 1e3 / 1e3,
                                                                                       t_last, busy))
    for k, (s, lst) in enumerate(lanes.items()):
        print("slice %d timeline (us): " % k + " ".join("%.0f-%.0f" % ((st[b] - t0) / 100.0, (st[e] - t0) / 100.0)
                                                        for b, e, _ in lst))


if __name__ == "__main__":
    main()
