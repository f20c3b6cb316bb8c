#!/usr/bin/env python3
"""Time the chained Bottleneck tails against the launches they replace (each on its table /
autotuned tile), at the R50 layer1 shapes, and check bitwise equality: the pair (ops.conv_pair_q:
conv3 + identity + ReLU -> next conv1 + ReLU) and conv3 with its fused downsample
(ops.conv_chain_q ds=...). Diagnostics only.

    TB_BATCH=128 python tools/pair_bench.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402

B = int(os.environ.get("TB_BATCH", "128"))
# output ranges wide enough that nothing overflows (an overflowing launch times its flag atomics)
RNG = 1000.0
dev = torch.device("cuda")


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e3


for cin, c1, c2, h in ((64, 256, 64, 56),):
    g = torch.Generator(device=dev).manual_seed(0)

    def codes(co, ci):
        w = torch.randn(co, ci, 1, 1, device=dev, generator=g) * 0.05
        step = ops.quantize_channels_(w.reshape(co, -1), [6] * co)
        return ops.pack_weights_ex(w, step, 1)[0]
    k1, k2 = codes(c1, cin), codes(c2, c1)
    x = torch.relu(torch.randn(B, h, h, cin, device=dev, generator=g))
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    rq = ops.act_quantize(torch.relu(torch.randn(B, h, h, c1, device=dev, generator=g)),
                          torch.full((B,), 4.0, device=dev), 3)
    cs1, sh1 = torch.full((c1,), 0.02, device=dev), torch.linspace(-0.1, 0.1, c1, device=dev)
    cs2, sh2 = torch.full((c2,), 0.02, device=dev), torch.linspace(-0.1, 0.1, c2, device=dev)
    am1 = torch.full((B,), RNG, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    out = {}

    def two():
        _, y1 = ops.tuned_conv2d_q(xq, am, k1, None, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=RNG, overflow=ovf,
                                   want_f32=False, residual_q=rq, residual_range=4.0)
        _, y2 = ops.tuned_conv2d_q(y1, am1, k2, None, 1, 1, 1, 0, cs2, sh2, relu=True, emit_range=RNG, overflow=ovf,
                                   want_f32=False)
        out["two"] = (y1, y2)

    def pair():
        out["pair"] = ops.conv_pair_q(xq, am, k1, cs1, sh1, rq, 4.0, RNG, am1, k2, cs2, sh2, RNG, ovf)

    def first():
        ops.tuned_conv2d_q(xq, am, k1, None, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=RNG, overflow=ovf,
                           want_f32=False, residual_q=rq, residual_range=4.0)
    def second():
        ops.tuned_conv2d_q(out["two"][0], am1, k2, None, 1, 1, 1, 0, cs2, sh2, relu=True, emit_range=RNG,
                           overflow=ovf, want_f32=False)
    t_two, t_pair, t_first = timed(two), timed(pair), timed(first)
    t_second = timed(second)
    same = all(torch.equal(a, b) for a, b in zip(out["two"], out["pair"]))
    print("B=%d %4d->%4d->%4d @%d: two launches %.1f us (conv3 alone %.1f, conv1 alone %.1f), pair %.1f us (%.2fx)%s"
          % (B, cin, c1, c2, h, t_two, t_first, t_second, t_pair, t_two / t_pair, "" if same else "  MISMATCH"),
          flush=True)

    # conv3 + the fused downsample vs the downsample launch + conv3 with the limb-plane identity
    wds = torch.randn(c1, cin, 1, 1, device=dev, generator=g) * 0.05
    dcodes, _, dscale, _ = ops.pack_weights_ex(wds, None, 3)
    dsh = torch.linspace(-0.1, 0.1, c1, device=dev)
    xb = torch.relu(torch.randn(B, h, h, cin, device=dev, generator=g))
    amb = ops.act_absmax(xb)
    xbq = ops.act_quantize(xb, amb, 3)

    def sep():
        _, yd = ops.tuned_conv2d_q(xbq, amb, dcodes, None, 1, 1, 1, 0, dscale, dsh, emit_range=RNG, overflow=ovf,
                                   want_f32=False)
        _, y1 = ops.tuned_conv2d_q(xq, am, k1, None, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=RNG, overflow=ovf,
                                   want_f32=False, residual_q=yd, residual_range=RNG)
        out["sep"] = y1

    def dsonly():
        ops.tuned_conv2d_q(xbq, amb, dcodes, None, 1, 1, 1, 0, dscale, dsh, emit_range=RNG, overflow=ovf,
                           want_f32=False)

    def chain():
        out["chain"] = ops.conv_chain_q(xq, am, k1, None, cs1, sh1, RNG, None, ovf,
                                        ds=(xbq, amb, dcodes, dscale, dsh, RNG))[0]
    t_sep, t_ds, t_chain = timed(sep), timed(dsonly), timed(chain)
    print("B=%d ds %d->%d + conv3 %d->%d @%d: two launches %.1f us (downsample alone %.1f), chain %.1f us (%.2fx)%s"
          % (B, cin, c1, cin, c1, h, t_sep, t_ds, t_chain, t_sep / t_chain,
             "" if torch.equal(out["sep"], out["chain"]) else "  MISMATCH"), flush=True)
