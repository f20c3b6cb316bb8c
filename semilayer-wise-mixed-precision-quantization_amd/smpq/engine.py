"""Fused eval-mode ResNet forward, every conv on the HIP path (NHWC end to end).

Restates ``ResNet._forward_impl`` (resnet.py:204-220), ``BasicBlock.forward`` (resnet.py:55-68)
and ``Bottleneck.forward`` (resnet.py:97-116):

  * input: per-image range + quantization of the NCHW image into space-to-depth limb planes
    (``image_quantize_s2d``; 16-channel pixels = 2x2 blocks of RGB + 0);
  * stem conv 7x7/2 + BN + ReLU + MaxPool 3x3/2 (resnet.py:143-147): static mode, ONE launch
    (``stem_pool_s2d``: only the pooled limb planes leave the CU); dynamic mode, the stem conv
    (fp32 weights as 24-bit fixed point) then the pool fused with its output's quantization;
  * every block conv + its BN (+ residual add) (+ ReLU) = one ``conv2d_q`` launch; static mode:
    its epilogue writes the NEXT conv's limb planes, dynamic mode: fp32 + the per-image max|y| the
    next conv's quantizer needs;
  * the downsample 1x1 conv + BN (resnet.py:188-192) reads the block input's limb planes
    (already quantized for conv1) and writes the identity (static mode: as limb planes) consumed
    by conv3's epilogue;
  * avgpool + fc (resnet.py:216-218): ``ops.avgpool_fc``, summed in an order that does not depend
    on the batch, so an image's logits are the same bits in any batch, slice or data-parallel shard.

Static mode runs the batch as ``STREAMS`` slices on their own streams (or, unsliced, each
downsample branch on a side stream), fork/join inside the captured HIP graph; every launch computes
what it computes serially, so the logits are bitwise those of the serial forward.

An activation is carried as ``Act`` = fp32 NHWC tensor and/or its int8 limb planes plus its
per-image range; limb planes are produced at most once per activation.

Range modes (``set_range_mode``):
  * "dynamic": every activation's range is its per-image max|x| (from the producer's epilogue),
    the producer writes fp32 and ``act_quantize`` makes the limb planes — each image's result is
    independent of the batch;
  * "static" (default): per-layer ranges calibrated by a dynamic forward (max over the batch x
    ``HEADROOM``); each conv's epilogue writes the NEXT conv's limb planes directly (no fp32 for
    block-internal tensors, no quantize pass). A value beyond its range sets an overflow flag
    and the forward is recomputed in dynamic mode, widening the ranges, so results are never
    silently clamped. Calibration is redone whenever a weight, BN buffer or the limb count changes.

Cache validity: every cache (packed codes, folded BN, ranges, the captured graph) is keyed on the
identity, data_ptr and ``_version`` of every parameter and buffer of the model (a replaced
Parameter, ``load_state_dict(assign=True)`` or a swapped submodule is seen), and on device-side
content fingerprints of the conv weights / metadata / BN tensors (smpq/fingerprint.py), checked
after every forward: a write through ``.data`` (no version bump) is detected, the result is
discarded and recomputed from freshly packed weights.
"""
import threading

import torch
import torch.nn.functional as F

from . import ops
from .fingerprint import Fingerprinter
from .qconv import QConv2d, stats
from .quant import check_pending

import os as _os
# "dynamic" is the deterministic mode for search runs (each image's logits depend on nothing but
# the weights and that image); "static" (default) is the fast mode (range modes)
_MODE = [_os.environ.get("SMPQ_RANGE_MODE", "static")]
HEADROOM = 2.0
# images per pass through the network: a chunk's inter-layer activations (int8 limb planes) stay
# resident in the 256 MiB Infinity Cache between producer and consumer instead of round-tripping
# HBM; every image is independent, so chunking changes no result (fc runs once on all features)
CHUNK = [int(_os.environ.get("SMPQ_CHUNK", "256"))]
# replay the static-range forward from a captured HIP graph (one launch instead of ~60 kernels
# with their Python/ctypes host cost); recaptured when weights, BN, ranges or shapes change
USE_GRAPH = [_os.environ.get("SMPQ_GRAPH", "1") != "0"]
# static range: conv1 + bn1 + relu + maxpool as ONE launch (ops.stem_pool_s2d; bitwise identical to
# the stem conv followed by maxpool_limbs, without the 112x112 conv output round trip)
FUSED_STEM = [_os.environ.get("SMPQ_FUSED_STEM", "1") != "0"]
# static range: the downsample branch of a block runs on a side stream beside conv1 / conv2
CONCURRENT_DS = [_os.environ.get("SMPQ_CONCURRENT_DS", "1") != "0"]
# static range: the batch split into this many slices, each on its own stream (concurrent kernels)
STREAMS = [int(_os.environ.get("SMPQ_STREAMS", "2"))]
# static range: a Bottleneck's conv3 and the next block's conv1 as ONE launch where the pair kernel
# is built (ops.conv_pair_q: conv1 reads conv3's output tile from LDS; bitwise the two launches)
PAIR_1X1 = [_os.environ.get("SMPQ_PAIR_1X1", "1") != "0"]
# ... also onto the conv1 of the next stage's first block (which has a downsample)
PAIR_STAGE_ENTRY = [_os.environ.get("SMPQ_PAIR_STAGE_ENTRY", "1") != "0"]
# static range: a stage's first Bottleneck computes its 1x1 / stride-1 downsample inside conv3's
# tiles (ops.conv_chain_q; its output limb planes are never written) where that is built
FUSE_DS = [_os.environ.get("SMPQ_FUSE_DS", "1") != "0"]
# ... for the blocks whose conv3 has at most this many input channels (64: layer1, 128: + layer2)
FUSE_DS_MAX_CIN = [int(_os.environ.get("SMPQ_FUSE_DS_MAX_CIN", "256"))]
stats.setdefault("graph_captures", 0)
stats.setdefault("graph_replays", 0)


def set_chunk(n):
    CHUNK[0] = max(1, int(n))
stats.setdefault("calibrations", 0)
stats.setdefault("overflow_reruns", 0)
stats.setdefault("stale_reruns", 0)


def set_range_mode(mode):
    if mode not in ("static", "dynamic"):
        raise ValueError("range mode must be 'static' or 'dynamic'")
    _MODE[0] = mode


def get_range_mode():
    return _MODE[0]


class Act:
    __slots__ = ("f32", "q", "amax", "rng")

    def __init__(self, f32=None, q=None, amax=None, rng=None):
        self.f32, self.q, self.amax, self.rng = f32, q, amax, rng  # rng: static range (float) or None

    def limbs(self):
        if self.q is None:
            self.q = ops.act_quantize(self.f32, self.amax)
        return self.q


def _bn_fold(bn):
    inv = torch.rsqrt(bn.running_var.float() + bn.eps)
    a = bn.weight.float() * inv if bn.affine else inv
    b = (bn.bias.float() if bn.affine else torch.zeros_like(a)) - bn.running_mean.float() * a
    return a, b


def _bn_key(bn):
    if bn is None:
        return None
    ts = [bn.running_mean, bn.running_var]
    if bn.affine:
        ts += [bn.weight, bn.bias]
    return tuple((id(t), t.data_ptr(), t._version) for t in ts) + (bn.eps,)


def conv_plan(conv, bn):
    """(codes, offset, col_scale, col_shift, kind) for the fused kernel, or None."""
    if not isinstance(conv, QConv2d):
        return None
    pk = conv.packed()
    if pk is None:
        return None
    key = (conv._pack_key(), _bn_key(bn), None if conv.bias is None else (conv.bias.data_ptr(), conv.bias._version))
    cache = getattr(conv, "_fold_cache", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    codes, _, offset, wscale, kind = pk
    with torch.no_grad():
        if bn is not None:
            a, b = _bn_fold(bn)
        else:
            a = torch.ones_like(wscale)
            b = torch.zeros_like(wscale)
        if conv.bias is not None:
            b = b + conv.bias.float() * a
        plan = (codes, offset, (wscale * a).contiguous(), b.contiguous(), kind)
    conv._fold_cache = (key, plan)
    return plan


def _to_nchw(x_nhwc):
    return x_nhwc.permute(0, 3, 1, 2)


def _to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


class Ctx:
    """Per-forward state: range mode, calibrated ranges, recorded maxima, overflow flag."""

    def __init__(self, n, device, ranges=None, record=False, cache=None):
        self.n, self.device = n, device
        self.ranges = ranges            # {id(conv): range} (static mode) or None
        self.record = {} if record else None
        # [0] a value exceeded its static range, [1] cached weight content is stale (fingerprint)
        self.overflow = torch.zeros(2, dtype=torch.int32, device=device) if ranges else None
        self._rt = cache if cache is not None else {}
        self.lane = None                # batch slice being enqueued (its own streams)
        # (graph capture) the weights' content check, enqueued by _forward on the last batch
        # slice's stream ahead of its work, or by the caller after the forward
        self.pending_check = None

    def range_tensor(self, conv):
        key = (id(conv), self.n)
        t = self._rt.get(key)
        if t is None:
            t = torch.full((self.n,), self.ranges[id(conv)], dtype=torch.float32, device=self.device)
            self._rt[key] = t
        return t


def run_conv(conv, bn, act, relu, residual=None, want_amax=True, ctx=None, want_f32=True):
    """y = act(bn(conv(x)) [+ residual]) -> Act (NHWC fp32 and/or the next conv's limb planes).
    ``residual``: an fp32 NHWC tensor, or an Act carrying limb planes + static range."""
    res_q = res_rng = None
    if isinstance(residual, Act):
        if residual.f32 is not None:
            residual = residual.f32
        else:
            res_q, res_rng, residual = residual.q, residual.rng, None
    n = act.amax.shape[0] if act.amax is not None else act.f32.shape[0]
    plan = conv_plan(conv, bn)
    static = ctx is not None and ctx.ranges is not None and want_amax and plan is not None \
        and id(conv) in ctx.ranges and conv.out_channels % 4 == 0
    yam = torch.zeros(n, dtype=torch.float32, device=conv.weight.device) if (want_amax and not static) else None
    if plan is not None:
        codes, offset, col_scale, col_shift, kind = plan
        stats["hip_conv"] += 1
        if kind == "fixed":
            stats["fixed_conv"] += 1
        conv.last_path = "hip-" + kind
        if static:
            rng = ctx.ranges[id(conv)]
            y, yq = ops.tuned_conv2d_q(act.limbs(), act.amax, codes, offset, conv.kernel_size[0],
                                       conv.kernel_size[1], conv.stride[0], conv.padding[0], col_scale, col_shift,
                                       residual=residual, relu=relu, emit_range=rng, overflow=ctx.overflow,
                                       want_f32=want_f32, residual_q=res_q, residual_range=res_rng)
            return Act(f32=y, q=yq, amax=ctx.range_tensor(conv), rng=rng)
        y = ops.tuned_conv2d_q(act.limbs(), act.amax, codes, offset, conv.kernel_size[0], conv.kernel_size[1],
                               conv.stride[0], conv.padding[0], col_scale, col_shift,
                               residual=residual, relu=relu, y_absmax=yam, residual_q=res_q,
                               residual_range=res_rng)
        if ctx is not None and ctx.record is not None and yam is not None:
            prev = ctx.record.get(id(conv))
            m = yam.amax().reshape(1)
            ctx.record[id(conv)] = m if prev is None else torch.maximum(prev, m)
        return Act(f32=y, amax=yam)
    yam = torch.zeros(n, dtype=torch.float32, device=conv.weight.device) if want_amax else None
    # geometry the kernel does not cover: the reference's fp32 arithmetic on MIOpen
    stats["fp32_conv"] += 1
    conv.last_path = "fp32"
    y = F.conv2d(_to_nchw(act.f32), conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)
    if bn is not None:
        y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
    if residual is not None:
        y = y + _to_nchw(residual)
    elif res_q is not None:
        raise RuntimeError("smpq: limb-plane residual on the fp32 fallback path")
    if relu:
        y = F.relu(y)
    y = _to_nhwc(y)
    if want_amax:
        ops.act_absmax(y, out=yam)
    return Act(f32=y, amax=yam)


_STREAMS = {}


# measurement (bench.py): run the batch slices one after another on the current stream
SERIAL_SLICES = [False]
# diagnostics: the first batch slice's stream at high priority (the others at normal priority)
SLICE_PRIORITY = [_os.environ.get("SMPQ_SLICE_PRIORITY", "0") != "0"]


def _stream(key):
    """A side stream per key (created once; reused by every forward and graph capture)."""
    s = _STREAMS.get(key)
    if s is None:
        prio = -1 if (SLICE_PRIORITY[0] and key[1] == "slice" and key[2] == 0) else 0
        s = _STREAMS[key] = torch.cuda.Stream(device=key[0], priority=prio)
    return s


def _side_stream(device, lane):
    """The downsample branch's stream of batch slice ``lane`` (None: the unsliced forward)."""
    return _stream((device, "ds", lane))


def _1x1(c):
    return c.kernel_size == (1, 1) and c.stride == (1, 1) and c.padding == (0, 0) and c.groups == 1


def _exact(plan):
    return plan is not None and (plan[0].dim() == 2 or plan[0].shape[0] == 1)


def _pair_plan(blk, nxt, ctx):
    """The next block's conv1 plan when it can be chained onto blk.conv3 (static ranges, exact
    codes without offsets, 1x1 / stride 1 / pad 0 both, a built shape), else None."""
    # (the next block may have a downsample: it reads the block input, which conv3 writes anyway)
    if not (PAIR_1X1[0] and nxt is not None and ctx is not None and ctx.ranges is not None
            and hasattr(blk, "conv3") and hasattr(nxt, "conv3")
            and (nxt.downsample is None or PAIR_STAGE_ENTRY[0])):
        return None
    c3, c1 = blk.conv3, nxt.conv1
    if id(c3) not in ctx.ranges or id(c1) not in ctx.ranges or not (_1x1(c3) and _1x1(c1)):
        return None
    p3, p1 = conv_plan(c3, blk.bn3), conv_plan(c1, nxt.bn1)
    if not (_exact(p3) and _exact(p1)) or p1[1] is not None:
        return None
    if not ops.conv_chain_supported(c3.in_channels, c3.out_channels, c1.out_channels):
        return None
    return p1


def _ds_fuse_plan(blk, x, ctx):
    """The downsample's plan when it can run inside blk.conv3's tiles (ops.conv_chain_q): a
    Bottleneck whose downsample (1x1 conv + BN, 24-bit fixed point) has the stride of its conv2
    (so its output pixels are conv3's), static ranges for both, a built shape
    (ops.conv_chain_ds_supported)."""
    if not (FUSE_DS[0] and ctx is not None and ctx.ranges is not None and hasattr(blk, "conv3")
            and isinstance(blk.downsample, torch.nn.Sequential) and len(blk.downsample) == 2
            and x.q is not None and x.amax is not None and x.q.shape[0] == 3):
        return None
    dc, dbn, c3 = blk.downsample[0], blk.downsample[1], blk.conv3
    st = dc.stride[0]
    if not (isinstance(dbn, torch.nn.BatchNorm2d) and dc.kernel_size == (1, 1) and dc.padding == (0, 0)
            and dc.groups == 1 and dc.stride == (st, st) and _1x1(c3) and blk.conv1.stride == (1, 1)
            and c3.in_channels <= FUSE_DS_MAX_CIN[0]
            and blk.conv2.stride == (st, st) and dc.out_channels == c3.out_channels
            and id(dc) in ctx.ranges and id(c3) in ctx.ranges):
        return None
    pd, p3 = conv_plan(dc, dbn), conv_plan(c3, blk.bn3)
    if pd is None or not _exact(p3) or pd[1] is not None or pd[0].dim() != 3 or pd[0].shape[0] != 3:
        return None
    if not ops.conv_chain_ds_supported(c3.in_channels, c3.out_channels, dc.in_channels, st):
        return None
    return pd


def block_forward(blk, x, ctx=None, last=False, t1=None, nxt=None):
    """One BasicBlock / Bottleneck on an Act; returns (output Act, the next block's conv1 output
    Act or None). ``t1``: this block's conv1 output when the previous block already computed it
    (chain launch); ``nxt``: the next block, whose conv1 is chained onto this block's conv3 when
    _pair_plan allows. In static mode no
    activation is stored in fp32 except the downsample's identity and the last block's output
    (avgpool): the identity of a block without downsample is read from its input's limb planes.

    Static mode: the downsample branch (resnet.py:188-192) depends only on the block input, so it
    runs beside conv1: outside batch slices on a side stream that joins before the conv that adds
    it (fork/join inside the captured graph); a single launch holding both convs was measured
    slower than the two launches (profiles/r03_pair_bench.txt). Where _ds_fuse_plan allows, it
    runs inside conv3's own tiles instead (ops.conv_chain_q) and its output is never written. Every
    conv computes exactly what it computes serially, so the result is bitwise the same
    (tests/test_gpu.py, tests/test_gpu_pair.py)."""
    side = None
    dsplan = None if last else _ds_fuse_plan(blk, x, ctx)

    def downsample():
        return run_conv(blk.downsample[0], blk.downsample[1], x, relu=False, ctx=ctx, want_f32=False)

    def as_identity(ds):
        # static mode: the identity as calibrated-range limb planes (3 B/element instead of fp32)
        return ds if (ds.f32 is None and ds.q is not None and ds.rng is not None) else ds.f32

    # (not inside a batch slice: a fork nested in a slice's fork crashes hipStreamEndCapture on
    # ROCm 7.2 / torch 2.10 — reproduced with torch alone by tools/repro_nested_fork.py)
    identity = None
    if dsplan is not None:
        pass  # computed in conv3's tiles
    elif blk.downsample is not None and CONCURRENT_DS[0] and ctx is not None and ctx.ranges is not None \
            and ctx.lane is None and x.q is not None:  # both branches read the input's limb planes
        main = torch.cuda.current_stream()
        side = _side_stream(x.q.device, ctx.lane)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            # allocated on the side stream, consumed on main after the join; freed blocks are
            # reused by the side stream only after its next wait on main (the next fork), which
            # is ordered after every consumer, so no record_stream is needed (none in a capture)
            identity = as_identity(downsample())
    elif blk.downsample is not None:
        identity = as_identity(downsample())
    elif x.f32 is not None or x.q is None or x.rng is None:
        identity = x.f32
    else:
        identity = x
    out_amax = not last  # the last block feeds only avgpool

    def join():
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)

    if t1 is None:
        t1 = run_conv(blk.conv1, blk.bn1, x, True, ctx=ctx, want_f32=False)
    if hasattr(blk, "conv3"):  # Bottleneck (resnet.py:97-116)
        t2 = run_conv(blk.conv2, blk.bn2, t1, True, ctx=ctx, want_f32=False)
        join()
        # (a fused downsample runs without a chained conv1: smpq_conv2d_chain_fwd)
        p1 = None if (last or dsplan is not None) else _pair_plan(blk, nxt, ctx)
        ident_q = dsplan is not None or (isinstance(identity, Act) and identity.f32 is None
                                         and identity.q is not None and identity.rng is not None)
        st = blk.downsample[0].stride[0] if dsplan is not None else 1
        chain = (dsplan is not None or p1 is not None) and ident_q and t2.q is not None and t2.amax is not None \
            and t2.q.shape[0] == 3 and (dsplan is None or t2.q.shape[2:4] == tuple((d - 1) // st + 1
                                                                                    for d in x.q.shape[2:4]))
        if dsplan is not None and not chain:
            identity = as_identity(downsample())  # (not expected: conv2 ran outside the static path)
        if chain:
            # conv3 (+ identity, ReLU) with its downsample and / or the next block's conv1, one launch
            c3 = blk.conv3
            codes3, off3, cs3, sh3, kind3 = conv_plan(c3, blk.bn3)
            rng3, am3 = ctx.ranges[id(c3)], ctx.range_tensor(c3)
            dsarg = nxtarg = None
            if dsplan is not None:
                dcodes, _, dcs, dsh, dkind = dsplan
                dsarg = (x.q, x.amax, dcodes, dcs, dsh, ctx.ranges[id(blk.downsample[0])], st)
            if p1 is not None:
                nxtarg = (p1[0], p1[2], p1[3], ctx.ranges[id(nxt.conv1)])
            yq3, yq1 = ops.conv_chain_q(t2.q, t2.amax, codes3, off3, cs3, sh3, rng3, am3, ctx.overflow,
                                        residual_q=None if dsarg else identity.q,
                                        residual_range=None if dsarg else identity.rng, ds=dsarg, nxt=nxtarg)
            stats["hip_conv"] += 1 + (dsarg is not None) + (nxtarg is not None)
            stats["fixed_conv"] += dsarg is not None
            stats["chain_conv"] = stats.get("chain_conv", 0) + 1
            stats["pair_conv"] = stats.get("pair_conv", 0) + (nxtarg is not None)
            stats["fused_ds"] = stats.get("fused_ds", 0) + (dsarg is not None)
            c3.last_path = "hip-%s-chain" % kind3
            if dsarg is not None:
                blk.downsample[0].last_path = "hip-%s-chain" % dkind
            nt1 = None
            if nxtarg is not None:
                nxt.conv1.last_path = "hip-%s-chain" % p1[4]
                nt1 = Act(q=yq1, amax=ctx.range_tensor(nxt.conv1), rng=nxtarg[3])
            return Act(q=yq3, amax=am3, rng=rng3), nt1
        return run_conv(blk.conv3, blk.bn3, t2, True, residual=identity, ctx=ctx, want_amax=out_amax,
                        want_f32=last), None
    # BasicBlock (resnet.py:55-68)
    join()
    return run_conv(blk.conv2, blk.bn2, t1, True, residual=identity, ctx=ctx, want_amax=out_amax,
                    want_f32=last), None


def stem_s2d_plan(conv, bn):
    """(codes, col_scale, col_shift, kind) of the stem in space-to-depth form (ops.stem_conv_s2d), or
    None when conv1 is not the 7x7/2/3 stem on <= 4 channels. Its fp32 weights become per-channel
    fixed point with max(2, L) limbs (quantized channels, if any: exact codes), as in
    QConv2d.packed_s2d."""
    if not (isinstance(conv, QConv2d) and conv.s2d_stem()):
        return None
    key = (conv._pack_key(), _bn_key(bn), None if conv.bias is None else (conv.bias.data_ptr(), conv.bias._version))
    cache = getattr(conv, "_s2d_cache", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    with torch.no_grad():
        codes, wscale, kind = conv.packed_s2d()
        if bn is not None:
            a, b = _bn_fold(bn)
        else:
            a, b = torch.ones_like(wscale), torch.zeros_like(wscale)
        if conv.bias is not None:
            b = b + conv.bias.float() * a
        plan = (codes, (wscale * a).contiguous(), b.contiguous(), kind)
    conv._s2d_cache = (key, plan)
    return plan


def stem_forward(model, x, ctx=None):
    """conv1 7x7/2 + bn1 + relu + maxpool 3x3/2 (resnet.py:206-209) -> Act of the pooled output.
    Static-range mode: the stem writes its calibrated-range limb planes and the max pool works on
    the codes (exact: the quantizer is monotone); no fp32 tensor is written. A stem the kernel does
    not cover (not 7x7/2/3, or other input channels than the conv's) runs on torch, counted in
    stats['fp32_conv'] like every such conv."""
    x = x.float().contiguous()
    n = x.shape[0]
    pool_ok = isinstance(model.maxpool, torch.nn.MaxPool2d) and model.maxpool.kernel_size in (3, (3, 3)) \
        and model.maxpool.stride in (2, (2, 2)) and model.maxpool.padding in (1, (1, 1))
    s2d = stem_s2d_plan(model.conv1, model.bn1) if (pool_ok and x.shape[1] == model.conv1.in_channels
                                                    and x.shape[2] >= 2 and x.shape[3] >= 2) else None
    if s2d is not None:
        # space-to-depth stem: 16-channel pixels, K steps of whole tap rows (an odd h or w gets a
        # zero row / column: the conv's own padding)
        codes, col_scale, col_shift, kind = s2d
        amax_in = ops.act_absmax(x)
        xq = ops.image_quantize_s2d(x, amax_in)
        stats["hip_conv"] += 1
        if kind == "fixed":
            stats["fixed_conv"] += 1
        model.conv1.last_path = "hip-%s-s2d" % kind
        conv = model.conv1
        if ctx is not None and ctx.ranges is not None and id(conv) in ctx.ranges and conv.out_channels % 16 == 0:
            rng = ctx.ranges[id(conv)]
            if FUSED_STEM[0] and conv.out_channels == 64 and ops.stem_pool_supported(xq, codes, x.shape[2], x.shape[3]):
                model.conv1.last_path = "hip-%s-s2d-pool" % kind
                yq = ops.stem_pool_s2d(xq, amax_in, codes, x.shape[2], x.shape[3], col_scale, col_shift,
                                       emit_range=rng, overflow=ctx.overflow)
                return Act(q=yq, amax=ctx.range_tensor(conv), rng=rng)
            _, yq = ops.tuned_stem_conv_s2d(xq, amax_in, codes, x.shape[2], x.shape[3], col_scale, col_shift,
                                            relu=True, emit_range=rng, overflow=ctx.overflow, want_f32=False)
            return Act(q=ops.maxpool_limbs(yq), amax=ctx.range_tensor(conv), rng=rng)
        yam = torch.zeros(n, dtype=torch.float32, device=x.device)
        y = ops.tuned_stem_conv_s2d(xq, amax_in, codes, x.shape[2], x.shape[3], col_scale, col_shift,
                                    relu=True, y_absmax=yam)
        if ctx is not None and ctx.record is not None:
            prev = ctx.record.get(id(conv))
            m = yam.amax().reshape(1)
            ctx.record[id(conv)] = m if prev is None else torch.maximum(prev, m)
        q, f = ops.maxpool_quantize(y, yam, want_f32=True)
        return Act(f32=f, q=q, amax=yam)
    # a stem the kernel does not cover: the reference's fp32 arithmetic (MIOpen), then quantized
    stats["fp32_conv"] += 1
    model.conv1.last_path = "fp32"
    h = model.maxpool(model.relu(model.bn1(model.conv1(x.contiguous(memory_format=torch.channels_last)))))
    h = _to_nhwc(h)
    amax = ops.act_absmax(h)
    return Act(f32=h, amax=amax)


def _blocks(model):
    return [b for layer in (model.layer1, model.layer2, model.layer3, model.layer4) for b in layer]


def _head(model, feat, out=None):
    """avgpool + flatten + fc (resnet.py:216-218) on the last block's NHWC fp32 output: the
    batch-invariant HIP kernel for the reference's modules, torch for anything else. ``out``: the
    rows of the batch's logits this slice fills (None: a new tensor)."""
    ap = model.avgpool
    if isinstance(model.fc, torch.nn.Linear) and isinstance(ap, torch.nn.AdaptiveAvgPool2d) \
            and ap.output_size in (1, (1, 1)) and feat.is_cuda and feat.shape[-1] % 4 == 0:
        return ops.avgpool_fc(feat, model.fc.weight, model.fc.bias, out=out)
    y = model.fc(feat.mean(dim=(1, 2)))
    if out is not None:
        out.copy_(y)
        return out
    return y


def _features(model, x, ctx):
    act = stem_forward(model, x, ctx)
    blocks = _blocks(model)
    t1 = None
    for i, blk in enumerate(blocks):
        nxt = blocks[i + 1] if i + 1 < len(blocks) else None
        act, t1 = block_forward(blk, act, ctx, last=nxt is None, t1=t1, nxt=nxt)
    return act.f32


def _forward(model, x, ctx):
    n = x.shape[0]
    c = CHUNK[0]
    parts = [(s, min(n, s + c)) for s in range(0, n, c)]
    nst = STREAMS[0] if (ctx is not None and ctx.ranges is not None) else 1
    if nst > 1 and n >= 2 * nst:
        # static mode: the batch as nst concurrent slices, each on its own stream, so that one
        # slice's bandwidth-bound convs overlap another's MFMA/L2-bound ones; every image's result
        # is the same as in the serial forward (per-layer ranges are fixed, kernels exact, the head
        # batch-invariant). With chunking (CHUNK < n) the chunks go round-robin over the streams.
        if len(parts) == 1:
            step = (n + nst - 1) // nst
            parts = [(s, min(n, s + step)) for s in range(0, n, step)]
        main = torch.cuda.current_stream()
        for s0, s1 in parts:  # shared per-layer range tensors exist before the fork
            ctx.n = s1 - s0
            for m in model.modules():
                if id(m) in ctx.ranges:
                    ctx.range_tensor(m)
        logits = []
        lanes = min(nst, len(parts))
        # every slice writes its rows of the batch's logits (allocated before the fork: no
        # concatenation after the join)
        y = torch.empty(n, model.fc.out_features, dtype=torch.float32, device=x.device) \
            if isinstance(model.fc, torch.nn.Linear) else None
        for i in range(lanes):
            _stream((x.device, "slice", i)).wait_stream(main)
        for i, (s0, s1) in enumerate(parts):
            # SERIAL_SLICES (bench.py's roofline region): the same slices and launches, one after
            # another on the current stream, so that per-launch events time each kernel alone
            with torch.cuda.stream(main if SERIAL_SLICES[0] else _stream((x.device, "slice", i % lanes))):
                ctx.n, ctx.lane = s1 - s0, i % lanes
                logits.append(_head(model, _features(model, x[s0:s1], ctx), out=None if y is None else y[s0:s1]))
                if i == 0 and lanes > 1 and ctx.pending_check is not None and not SERIAL_SLICES[0]:
                    # the weights' content check (reads only the weights, writes only overflow[1])
                    # after the first slice, which ends while the last one runs its narrow layer-4
                    # convs: off the step's critical path. (Ahead of the last slice's work it
                    # delayed that slice, -0.5 %; a stream forked only for it crashed a graph
                    # replay beside the downsample forks on ROCm 7.2.)
                    ctx.pending_check()
                    ctx.pending_check = None
        for i in range(lanes):
            main.wait_stream(_stream((x.device, "slice", i)))
        ctx.n, ctx.lane = n, None
        if y is not None:
            return y
        return torch.cat(logits) if len(logits) > 1 else logits[0]
    if len(parts) == 1:
        return _head(model, _features(model, x, ctx))
    logits = []
    for s0, s1 in parts:
        if ctx is not None:
            ctx.n = s1 - s0
        logits.append(_head(model, _features(model, x[s0:s1], ctx)))
    if ctx is not None:
        ctx.n = n
    return torch.cat(logits)


# ---- data-parallel group ------------------------------------------------------------------------
# When set, every rank of this process group runs the same sequence of static-range forwards on
# its own shard of each global batch (smpq.dp / bench.py). The per-layer maxima of a calibration
# are MAX-all-reduced, so every rank holds the ranges a single process would calibrate on the
# whole global batch; and every decision that starts a calibration (first use, a weight change,
# an overflow, stale weights) is taken collectively, so the ranks never diverge. Static-range
# logits of an image then depend only on the weights, the global batch's ranges and the image:
# the gathered logits equal the single-GPU forward of the global batch bit for bit.
_DP = [None]


def set_dp_group(group):
    """Process group (torch.distributed) of the ranks that forward shards of the same global
    batches in lockstep, or None (default: this process calibrates on its own inputs)."""
    _DP[0] = group


def get_dp_group():
    return _DP[0]


def _dp_max_(t):
    """In-place MAX all-reduce of ``t`` over the data-parallel group (a no-op without one)."""
    g = _DP[0]
    if g is None:
        return t
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(g) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=g)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
    return t


# ---- cache validity -----------------------------------------------------------------------------
def _fp_tensors(model):
    """Tensors whose CONTENT the caches are built from: conv weights (+ bias) and quantization
    metadata (packed codes, folded scales), BN buffers / affine parameters (folded shift)."""
    out = []
    for m in model.modules():
        if isinstance(m, QConv2d):
            out += [m.weight, m.qstep, m.qbits] + ([m.bias] if m.bias is not None else [])
        elif isinstance(m, torch.nn.BatchNorm2d):
            out += [m.running_mean, m.running_var] + ([m.weight, m.bias] if m.affine else [])
    return [t.detach() for t in out]


def _signature(model):
    """Host key of everything the calibrated ranges and the captured graph depend on: identity,
    data_ptr and version of every parameter and buffer (walked afresh each call, so replaced
    Parameters, load_state_dict(assign=True) and swapped submodules are seen), each conv's
    metadata and content generations and the limb count."""
    ts = tuple((id(t), t.data_ptr(), t._version) for t in model.parameters()) + \
        tuple((id(t), t.data_ptr(), t._version) for t in model.buffers())
    convs = tuple((id(m), m._meta_gen, m._content_gen) for m in model.modules() if isinstance(m, QConv2d))
    return (ops.get_act_limbs(), HEADROOM, ts, convs)


def _bump_content(model):
    """Invalidate the content-keyed caches (packed codes, folded BN): rebuilt on next use."""
    for m in model.modules():
        if isinstance(m, QConv2d):
            m._content_gen += 1


def _refresh_fingerprint(model, device, stale=False):
    """Fingerprint the current content. The content-keyed caches are invalidated only when they
    may hold other content: ``stale`` (a fingerprint check failed) or the content differs from
    the last fingerprint taken (model._smpq_fp, shared by both range modes; one host sync).
    Returns (fingerprinter, whether the caches were invalidated)."""
    fp = Fingerprinter(_fp_tensors(model), device)
    old = getattr(model, "_smpq_fp", None)
    changed = stale or old is None or not fp.same_content(old)
    if changed:
        _bump_content(model)
    model._smpq_fp = fp
    return fp, changed


class Calibration:
    """Per-layer maxima of one calibration forward (a dynamic-range forward): ``keys`` (conv ids in
    module order), ``maxima`` (device fp32 tensor), the logits, the content fingerprint taken
    before it and whether that forward's content differs from the previous calibration's."""
    __slots__ = ("keys", "maxima", "logits", "fp", "changed", "sig0")


def calibration_maxima(model, x, stale=False):
    """Run the calibration forward of ``x`` (dynamic ranges) and return its Calibration."""
    c = Calibration()
    c.sig0 = _signature(model)
    c.fp, c.changed = _refresh_fingerprint(model, x.device, stale)
    ctx = Ctx(x.shape[0], x.device, record=True)
    c.logits = _forward(model, x, ctx)
    c.keys = [id(m) for m in model.modules() if id(m) in ctx.record]
    c.maxima = torch.cat([ctx.record[k] for k in c.keys]) if c.keys else torch.zeros(0, device=x.device)
    return c


def set_calibration(model, c, widen=True):
    """Install the static ranges range_l = HEADROOM * max_l of Calibration ``c``. With ``widen``
    and unchanged weights (same signature, same content as the previous calibration, e.g. an
    overflow rerun) each range stays at least its previous value, so ranges only grow. Ranges
    equal to the installed ones (same weights, same calibration batch) keep the installed
    calibration object, and with it the graphs captured for it."""
    maxima = c.maxima.cpu().tolist()
    old = getattr(model, "_smpq_ranges", None)
    keep = widen and old is not None and not c.changed and old[1] == c.sig0
    ranges = {}
    for k, v in zip(c.keys, maxima):
        r = max(v, 1e-30) * HEADROOM
        if keep and k in old[0]:
            r = max(r, old[0][k])
        ranges[k] = r
    sig = _signature(model)
    if old is not None and not c.changed and old[1] == sig and old[0] == ranges:
        return
    model._smpq_ranges = (ranges, sig, {}, c.fp)


def calibrate(model, x, stale=False, fresh=False):
    """Dynamic forward of ``x`` that (re)sets the per-layer static ranges; returns its logits.
    In a data-parallel group the maxima are MAX-all-reduced over the ranks first. ``fresh``: the
    ranges come from this batch alone (no widening by earlier ranges: new_evaluation)."""
    c = calibration_maxima(model, x, stale)
    _dp_max_(c.maxima)
    set_calibration(model, c, widen=not fresh)
    stats["calibrations"] += 1
    return c.logits


def new_evaluation(model):
    """Start of an evaluation pass over a loader (functions.evaluate_acc_loss_softmax /
    evaluate_loss, dp.sharded_eval): the next static-range forward recalibrates on its own batch,
    so every evaluation's ranges are a function of the weights and of that evaluation's first
    batch only — two evaluations of the same weights on the same loader give the same results
    bit for bit, whatever ran before (an overflow rerun widens the ranges for the rest of the
    pass only). Identical ranges keep the captured graphs."""
    model._smpq_recal = True


def _static_eager(model, x, cal):
    ctx = Ctx(x.shape[0], x.device, ranges=cal[0], cache=cal[2])
    y = _forward(model, x, ctx)
    cal[3].check(ctx.overflow[1:])
    return y, ctx.overflow


def _graph_base(cal):
    """What every captured graph of a model depends on besides its input's shape and address:
    the calibration (ranges, signature) and the forward's structure knobs."""
    return (cal[1], CHUNK[0], ops.get_act_limbs(), id(cal[0]), FUSED_STEM[0], CONCURRENT_DS[0], STREAMS[0],
            ops.KMAJOR[0], PAIR_1X1[0], FUSE_DS[0], FUSE_DS_MAX_CIN[0], PAIR_STAGE_ENTRY[0])


def _graph_key(model, x, cal):
    return (tuple(x.shape), x.dtype, x.device) + _graph_base(cal)


def _addr_key(x):
    """Per-address graph key of an input: its shape, dtype, device and address. A graph captured on
    an input reads it as a contiguous NCHW tensor, so only contiguous inputs ever match one."""
    return (tuple(x.shape), x.dtype, x.device, x.data_ptr()) if x.is_contiguous() else None


def _graphs(model, cal):
    """The model's per-address graphs for calibration ``cal`` (dropped when it changes; graphs of
    other input shapes are kept, so a short last batch does not evict the full-batch graphs)."""
    per = getattr(model, "_smpq_graphs", None)
    base = _graph_base(cal)
    if per is None or per.get("base") != base:
        per = model._smpq_graphs = {"base": base}
    return per


def _graph_ready(model, x, cal):
    ak = _addr_key(x)
    if ak is not None and ak in _graphs(model, cal):
        return True
    entry = getattr(model, "_smpq_graph", None)
    return entry is not None and entry[0] == _graph_key(model, x, cal)


# HIP graphs captured on an input tensor's own memory (no copy of the input into the graph's static
# buffer): up to this many distinct input addresses per model (an evaluation loop's input buffers
# recycle a few addresses); further inputs are copied into the fallback graph's static buffer.
GRAPHS_PER_MODEL = [int(_os.environ.get("SMPQ_GRAPHS", "4"))]


# Held while a HIP graph is being captured. torch captures in the default "global" mode, in which
# device allocations and synchronising calls made by ANY thread during the capture are errors (or
# end up in the graph); smpq.batches' staging worker takes this lock around its device work
# (pinned-buffer waits, the side-stream copies and their allocations), so a batch staged while
# the evaluation loop captures waits for the capture to end instead of breaking it.
CAPTURE_LOCK = threading.Lock()


def _capture(model, x_in, cal):
    with CAPTURE_LOCK:
        return _capture_locked(model, x_in, cal)


def _capture_locked(model, x_in, cal):
    g = torch.cuda.CUDAGraph()
    ctx = Ctx(x_in.shape[0], x_in.device, ranges=cal[0], cache=cal[2])
    # one memory pool for all of the model's graphs: they are replayed one at a time on one stream
    # and each replay's outputs are copied out before the next, so they may share blocks
    pool = getattr(model, "_smpq_pool", None)
    if pool is None or pool[0] != x_in.device:
        pool = model._smpq_pool = (x_in.device, torch.cuda.graph_pool_handle())
    torch.cuda.synchronize()
    # thread_local: only THIS thread's unsafe calls break the capture; other threads' CUDA calls
    # (a DataLoader's pin-memory thread allocating pinned host memory) stay legal
    with torch.cuda.graph(g, pool=pool[1], capture_error_mode="thread_local"):
        ctx.overflow = torch.zeros(2, dtype=torch.int32, device=x_in.device)
        ctx.pending_check = lambda: cal[3].check(ctx.overflow[1:])
        y_static = _forward(model, x_in, ctx)
        if ctx.pending_check is not None:  # (not enqueued inside a batch slice)
            ctx.pending_check()
            ctx.pending_check = None
    stats["graph_captures"] += 1
    return g, ctx, y_static


def _capture_graph_for(model, x, cal):
    """Capture the static forward of ``x`` (every cache already warm: an eager forward of the same
    calibration ran first): on the input's own memory when it has a per-address slot left,
    otherwise as the fallback graph reading a static copy of the input."""
    per_ptr = _graphs(model, cal)
    ak = _addr_key(x)
    same_shape = sum(1 for k in per_ptr if k != "base" and k[:3] == ak[:3]) if ak is not None else 0
    if ak is not None and same_shape < GRAPHS_PER_MODEL[0]:
        per_ptr[ak] = _capture(model, x, cal)
        return
    static_x = x.contiguous().clone()
    g, ctx, y_static = _capture(model, static_x, cal)
    model._smpq_graph = (_graph_key(model, x, cal), g, static_x, ctx, y_static)


def _graph_forward(model, x, cal, capture=True):
    """Static forward through a captured HIP graph; returns (logits, overflow flag tensor). The
    graph reads the input where it lies when its (contiguous) input's address has a graph of its
    own (captured on first sight, up to GRAPHS_PER_MODEL addresses per input shape, dropped with
    the calibration); otherwise the input is copied into the fallback graph's static buffer.
    Without a graph for ``x`` the forward runs eagerly, and the graph is captured right after it
    (``capture``) or left to the caller (``_capture_graph_for``, once a data-parallel group has
    agreed that this calibration stays)."""
    key = _graph_key(model, x, cal)
    per_ptr = _graphs(model, cal)
    ak = _addr_key(x)
    hit = per_ptr.get(ak) if ak is not None else None
    if hit is not None:
        g, ctx, y_static = hit
        g.replay()
        stats["graph_replays"] += 1
        return y_static.clone(), ctx.overflow
    same_shape = sum(1 for k in per_ptr if k != "base" and k[:3] == ak[:3]) if ak is not None else 0
    entry = getattr(model, "_smpq_graph", None)
    if (ak is not None and same_shape < GRAPHS_PER_MODEL[0]) or entry is None or entry[0] != key:
        if not (ak is not None and same_shape < GRAPHS_PER_MODEL[0]):
            model._smpq_graph = None
        y, ovf = _static_eager(model, x, cal)  # warm every cache outside the capture
        if capture and not any(ovf.tolist()):
            _capture_graph_for(model, x, cal)
        return y, ovf
    _, g, static_x, ctx, y_static = entry
    static_x.copy_(x)
    g.replay()
    stats["graph_replays"] += 1
    return y_static.clone(), ctx.overflow


def _dynamic_forward(model, x):
    """Dynamic-range forward (batch-independent results); one host sync for the content check.
    A content change seen after the forward is recomputed once from freshly packed weights; a
    change seen again after that (weights written concurrently with the forward) raises."""
    for attempt in range(2):
        sig = _signature(model)
        st = getattr(model, "_smpq_dyn", None)
        if st is None or st[0] != sig or attempt:
            fp, _ = _refresh_fingerprint(model, x.device, stale=attempt > 0)
            model._smpq_dyn = st = (_signature(model), fp)
        y = _forward(model, x, None)
        flag = torch.zeros(1, dtype=torch.int32, device=x.device)
        st[1].check(flag)
        if int(flag.item()) == 0:
            return y
        stats["stale_reruns"] += 1
        model._smpq_dyn = None
    raise RuntimeError("smpq: the model's weights changed while its forward ran (twice); no stale result returned")


def forward_fused(model, x):
    """Eval-mode forward of an smpq ResNet on the GPU; returns logits [n, num_classes]."""
    check_pending()  # a deferred per-channel quantization that met a constant channel raises here
    if _MODE[0] == "dynamic":
        return _dynamic_forward(model, x)
    if torch.cuda.is_current_stream_capturing():
        # the overflow / staleness flags need a host read after the forward
        raise RuntimeError("smpq: the static-range forward cannot run inside a caller's graph capture "
                           "(it replays its own HIP graph); use dynamic range mode to capture it")
    cal = getattr(model, "_smpq_ranges", None)
    fresh = model.__dict__.pop("_smpq_recal", False)
    if _DP[0] is not None:
        # collective decision: every rank calibrates, or none does; and if any rank starts a new
        # evaluation, all of them calibrate afresh (the same widening rule on every rank). One MAX
        # all-reduce and one host sync per forward carry all four flags — [overflow, stale, this
        # rank needs a calibration, this rank starts a new evaluation] — after the forward, which
        # runs optimistically (its result is dropped when any rank calibrates); as on one GPU,
        # the graph replay is enqueued before the host's signature walk.
        y = ovf = None
        need_local = True
        deferred_capture = False
        if cal is not None and not fresh:
            if USE_GRAPH[0] and _graph_ready(model, x, cal):
                y, ovf = _graph_forward(model, x, cal)
                need_local = _signature(model) != cal[1]
            elif cal[1] == _signature(model):
                # no graph for this input yet: an eager forward only; the capture waits until the
                # ranks have agreed below that this calibration stays (a capture that
                # another rank's calibration would discard is not paid for)
                need_local = False
                y, ovf = _graph_forward(model, x, cal, capture=False) if USE_GRAPH[0] else \
                    _static_eager(model, x, cal)
                deferred_capture = USE_GRAPH[0] and not _graph_ready(model, x, cal)
        flags = torch.zeros(4, dtype=torch.int32, device=x.device)
        if ovf is not None:
            flags[:2].copy_(ovf)
        if need_local:
            flags[2] = 1
        if fresh:
            flags[3] = 1
        overflow, stale, need, fresh_any = _dp_max_(flags).tolist()
        if need or fresh_any:
            return calibrate(model, x, stale=bool(stale), fresh=bool(fresh_any))
        if not overflow and not stale:
            if deferred_capture:
                _capture_graph_for(model, x, cal)
            return y
        stats["stale_reruns" if stale else "overflow_reruns"] += 1
        return calibrate(model, x, stale=bool(stale))
    else:
        if cal is None or fresh:
            return calibrate(model, x, fresh=fresh)
        if USE_GRAPH[0] and _graph_ready(model, x, cal):
            # fast path: replay first, then validate on the host while the GPU runs; a changed
            # weight or BN buffer discards the result (recalibrate + recapture): nothing stale
            y, ovf = _graph_forward(model, x, cal)
            if _signature(model) != cal[1]:
                return calibrate(model, x)
        else:
            if cal[1] != _signature(model):
                return calibrate(model, x)
            y, ovf = _graph_forward(model, x, cal) if USE_GRAPH[0] else _static_eager(model, x, cal)
    overflow, stale = ovf.tolist()  # one sync: results are never silently clamped or stale
    if not overflow and not stale:
        return y
    stats["stale_reruns" if stale else "overflow_reruns"] += 1
    return calibrate(model, x, stale=bool(stale))
