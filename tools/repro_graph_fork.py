#!/usr/bin/env python3
"""Root-cause probe for the two HIP-graph crashes of rounds 2-5 (verdict r5 item 2).

  A. round 5: a host segfault inside CUDAGraph.replay() (gpurun_out/r05z_gputests.log) after commit
     a082ca2 put the weights' content check on a stream of its own, forked from the capture stream
     beside the downsample side-stream forks (test_gpu.py::test_concurrent_streams_bitwise);
  B. rounds 2-3: a host segfault in hipStreamEndCapture when a batch-slice stream forks a side
     stream (nested fork; tools/repro_nested_fork.py).

Every case runs in a child process (a crash ends only that child) and prints its exit status.
Cases (mode = topology):
  torch_flat      torch ops only: capture stream forks a 'check' stream, then forks and joins a
                  'ds' side stream four times, joins 'check'; two graphs captured on two inputs in
                  ONE shared memory pool, replayed A, B, A (the test's order)
  torch_flat_own  the same, each graph with its own pool
  torch_nested    capture stream -> 2 slice streams -> a side stream each (tools/repro_nested_fork.py)
  torch_nested_join  the same, each side stream ALSO joined straight into the capture stream at the end
  torch_prefork   the side streams forked from the capture stream together with the slice streams,
                  then slice -> side and side -> slice edges (the round-2 variant)
  torch_prefork_join  the same, each side stream also joined straight into the capture stream
  smpq_check      the real engine with a082ca2's capture (check on its own forked stream), the
                  test's call sequence (R18 u8, 7 images, STREAMS 1/2/3, CONCURRENT_DS)
  smpq_head       the engine as shipped (check on slice 0's stream), the same sequence
  smpq_check50 / smpq_head50  the same with R50 mixed (the test's first parametrization)
Variants (environment of the child): base; nopc = DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (the runtime
records kernel nodes as plain dispatches instead of pre-built AQL packets); q1 =
DEBUG_HIP_FORCE_GRAPH_QUEUES=1 (graph branches not spread over parallel internal streams); log =
AMD_LOG_LEVEL=4 with the [hipGraph] lines kept (the last lines before a crash name the step).

    python tools/repro_graph_fork.py [--cases a,b] [--variants base,nopc] [--out DIR]
"""
import argparse
import faulthandler
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd")
CASES = ["torch_flat", "torch_flat_own", "torch_nested", "torch_nested_join", "torch_prefork",
         "torch_prefork_join", "smpq_check", "smpq_head", "smpq_check50", "smpq_head50"]
VARIANTS = {
    "base": {},
    "nopc": {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0"},
    "q1": {"DEBUG_HIP_FORCE_GRAPH_QUEUES": "1"},
    "log": {"AMD_LOG_LEVEL": "4"},
}


def torch_case(mode):
    import torch
    dev = torch.device("cuda")
    main_s = torch.cuda.current_stream()
    chk = torch.cuda.Stream()
    ds = torch.cuda.Stream()
    slices = [torch.cuda.Stream() for _ in range(2)]
    sides = [torch.cuda.Stream() for _ in range(2)]
    w = torch.randn(1 << 16, device=dev)
    flag = torch.zeros(2, dtype=torch.int32, device=dev)

    def check():
        # reads only w, writes only flag[1] (the fingerprint check's footprint)
        flag[1:].copy_((w.sum() != w.sum()).to(torch.int32).reshape(1))

    def flat(x):
        main = torch.cuda.current_stream()
        chk.wait_stream(main)
        with torch.cuda.stream(chk):
            check()
        h = x * 2.0
        for _ in range(4):
            ds.wait_stream(main)
            with torch.cuda.stream(ds):
                d = h * 0.5 + 1.0  # allocated on the side stream, consumed after the join
            h = torch.relu(h * 1.5)
            main.wait_stream(ds)
            h = h + d
        main.wait_stream(chk)
        return h

    def nested(x):
        main = torch.cuda.current_stream()
        outs = []
        pre = mode.startswith("torch_prefork")
        for s in slices + (sides if pre else []):
            s.wait_stream(main)
        for i, sl in enumerate(slices):
            with torch.cuda.stream(sl):
                a = x[i] * 2.0
                sd = sides[i]
                sd.wait_stream(sl)
                with torch.cuda.stream(sd):
                    b = a + 1.0
                c = a * 3.0
                sl.wait_stream(sd)
                outs.append(b + c)
        for s in slices + (sides if mode.endswith("_join") else []):
            main.wait_stream(s)
        return torch.stack(outs)

    body = flat if mode.startswith("torch_flat") else nested
    xa = torch.randn(2, 1 << 20, device=dev)
    xb = torch.randn(2, 1 << 20, device=dev)
    want_a, want_b = body(xa), body(xb)
    torch.cuda.synchronize()
    shared = torch.cuda.graph_pool_handle()
    graphs = {}
    for name, x in (("A", xa), ("B", xb)):
        g = torch.cuda.CUDAGraph()
        print("%s: capture %s" % (mode, name), flush=True)
        pool = shared if mode != "torch_flat_own" else torch.cuda.graph_pool_handle()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, pool=pool):
            y = body(x)
        graphs[name] = (g, y)
    for name in ("A", "B", "A", "B", "A"):
        print("%s: replay %s" % (mode, name), flush=True)
        g, y = graphs[name]
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, want_a if name == "A" else want_b), (mode, name)
    print("%s: ok" % mode, flush=True)


def smpq_case(mode):
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import resnet
    from smpq import assignments, engine
    if mode.startswith("smpq_check"):
        # commit a082ca2's capture: the content check on a stream forked only for it
        def capture_locked(model, x_in, cal):
            g = torch.cuda.CUDAGraph()
            ctx = engine.Ctx(x_in.shape[0], x_in.device, ranges=cal[0], cache=cal[2])
            pool = getattr(model, "_smpq_pool", None)
            if pool is None or pool[0] != x_in.device:
                pool = model._smpq_pool = (x_in.device, torch.cuda.graph_pool_handle())
            torch.cuda.synchronize()
            with torch.cuda.graph(g, pool=pool[1]):
                ctx.overflow = torch.zeros(2, dtype=torch.int32, device=x_in.device)
                main = torch.cuda.current_stream()
                chk = engine._stream((x_in.device, "check"))
                chk.wait_stream(main)
                with torch.cuda.stream(chk):
                    cal[3].check(ctx.overflow[1:])
                y_static = engine._forward(model, x_in, ctx)
                main.wait_stream(chk)
            engine.stats["graph_captures"] += 1
            return g, ctx, y_static
        engine._capture_locked = capture_locked
    dev = torch.device("cuda")
    torch.manual_seed(0)
    r50 = mode.endswith("50")
    net = (resnet.resnet50() if r50 else resnet.resnet18()).to(dev).eval()
    assignments.apply_assignment(net, "r50_mixed" if r50 else "r18_u8", semantics="cpu")
    x = torch.randn(7, 3, 224, 224, generator=torch.Generator().manual_seed(23)).to(dev)
    x2 = torch.randn(7, 3, 224, 224, generator=torch.Generator().manual_seed(24)).to(dev)
    with torch.no_grad():
        engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0] = False, False, 1
        net(x)
        a, a2 = net(x), net(x2)
        for streams in (1, 2, 3):
            engine.STREAMS[0] = streams
            engine.CONCURRENT_DS[0], engine.USE_GRAPH[0] = True, False
            assert torch.equal(net(x), a) and torch.equal(net(x2), a2)
            engine.USE_GRAPH[0] = True
            for i, (xi, want) in enumerate(((x, a), (x2, a2), (x, a), (x2, a2), (x, a))):
                print("%s: streams %d call %d (%s)" % (mode, streams, i, "capture" if i < 2 else "replay"),
                      flush=True)
                y = net(xi)
                torch.cuda.synchronize()
                assert torch.equal(y, want), (mode, streams, i)
    print("%s: ok" % mode, flush=True)


def child(mode):
    faulthandler.enable()
    if mode.startswith("torch"):
        torch_case(mode)
    else:
        smpq_case(mode)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--variants", default="base,nopc,q1")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "graph_fork"))
    ap.add_argument("--child", default=None)
    args = ap.parse_args()
    if args.child:
        child(args.child)
        return
    os.makedirs(args.out, exist_ok=True)
    for case in args.cases.split(","):
        for var in args.variants.split(","):
            env = dict(os.environ)
            env.update(VARIANTS[var])
            log = os.path.join(args.out, "%s_%s.log" % (case, var))
            t0 = time.time()
            with open(log, "w") as f:
                try:
                    rc = subprocess.call([sys.executable, "-u", os.path.abspath(__file__), "--child", case],
                                         stdout=f, stderr=subprocess.STDOUT, env=env, timeout=150)
                except subprocess.TimeoutExpired:
                    rc = "timeout"
            tail = ""
            if var == "log" or rc != 0:
                # the last runtime / Python lines before the end (full log in the file)
                with open(log, "rb") as f:
                    lines = f.read().decode(errors="replace").splitlines()
                keep = [ln for ln in lines if "hipGraph" in ln or not ln.startswith(":")]
                tail = "\n    " + "\n    ".join(keep[-12:])
                if var == "log":
                    # the full AMD_LOG_LEVEL=4 log is large: keep the graph lines and the tail only
                    with open(log, "w") as f:
                        f.write("\n".join([ln for ln in lines if "hipGraph" in ln or "Graph" in ln][-4000:] +
                                          ["---- last 200 lines ----"] + lines[-200:]) + "\n")
            print("%-16s %-5s exit %-8s %5.1f s%s" % (case, var, rc, time.time() - t0,
                                                      "  (SIGSEGV)" if rc == -11 else ""), flush=True)
            if tail:
                print(tail, flush=True)


if __name__ == "__main__":
    main()
