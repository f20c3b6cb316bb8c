""".pth checkpoints + bit-assignment sidecar.

The reference's drivers checkpoint and roll back with plain state dicts
(resnet50_main.py:212 ``torch.save(net.state_dict(), pthname)``, :233-234 / :426-427
``net.load_state_dict(torch.load(pthname))``). Those files carry fake-quantized fp32 weights
only: the bit-widths are implicit in the values. Our QConv2d keeps ``qbits``/``qstep`` buffers
(qconv.py), so a state dict written by this package reloads with its metadata. This module covers
the other two cases:

* ``save_checkpoint`` writes the state dict plus ``<path>.bits.json``, the per-channel bit
  assignment in the reference's own vocabulary (lnum -> per-channel bits, 0 = never quantized)
  and the exact fp32 step of every channel (its IEEE bit pattern in hex), readable without torch
  by the search drivers' bookkeeping. By default (``plain=True``) the ``.pth`` holds exactly the
  reference's keys (no ``qbits``/``qstep``), so the reference's and torchvision's
  ``load_state_dict(strict=True)`` accept it; the sidecar restores the metadata bitwise;
* ``load_checkpoint`` / ``infer_quant_`` recover the metadata of a reference-written ``.pth``
  (no ``qbits``/``qstep`` keys): per channel, the smallest bit-width b whose re-quantization
  (functions.py:25-43 restated on the native library) leaves the channel bitwise unchanged is
  recorded with its step. A sidecar, when present, restricts the search to the recorded bit.
  The packer still verifies every code bitwise (smpq_pack_weights), so a wrong inference can
  only send a channel to the fixed-point path, never change a result.
"""
import json
import os

import numpy as np
import torch

from . import ops
from .assignments import addressable_convs

SIDECAR_SUFFIX = ".bits.json"
CANDIDATE_BITS = (2, 3, 4, 5, 6, 7, 8)


def sidecar_path(path):
    return str(path) + SIDECAR_SUFFIX


def bit_assignment(net):
    """{lnum: [bits per output channel]} over the addressable convs (lnum from 1, the drivers'
    numbering: resnet50_main.py:81-136, resnet18_main.py:86-115)."""
    out = {}
    for ln, conv in enumerate(addressable_convs(net), start=1):
        out[ln] = [int(b) for b in conv.qbits.detach().cpu().tolist()]
    return out


META_KEYS = (".qbits", ".qstep")


def plain_state_dict(net):
    """``net.state_dict()`` without the quantization metadata buffers: the reference's keys only."""
    return {k: v for k, v in net.state_dict().items() if not k.endswith(META_KEYS)}


def step_assignment(net):
    """{lnum: [fp32 step per output channel as its IEEE bit pattern, 8 hex digits]}."""
    out = {}
    for ln, conv in enumerate(addressable_convs(net), start=1):
        bits = conv.qstep.detach().cpu().contiguous().view(torch.int32).numpy().astype(np.uint32)
        out[ln] = ["%08x" % int(b) for b in bits]
    return out


def save_checkpoint(net, path, plain=True):
    """``torch.save(net.state_dict(), path)`` + ``<path>.bits.json`` (bits + exact steps). With
    ``plain`` the .pth carries the reference's keys only (loadable with strict=True by the
    reference's / torchvision's ResNet); otherwise it also keeps the qbits/qstep buffers."""
    from .quant import check_pending
    check_pending()
    torch.save(plain_state_dict(net) if plain else net.state_dict(), path)
    side = {"format": "smpq-bits/2", "convs": {str(k): v for k, v in bit_assignment(net).items()},
            "steps": {str(k): v for k, v in step_assignment(net).items()}}
    with open(sidecar_path(path), "w") as f:
        json.dump(side, f)


def _read_sidecar_full(path):
    p = sidecar_path(path)
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        side = json.load(f)
    fmt = side.get("format")
    if fmt not in ("smpq-bits/1", "smpq-bits/2"):
        raise ValueError("%s: unknown sidecar format %r" % (p, fmt))
    bits = {int(k): np.asarray(v, dtype=np.int64) for k, v in side["convs"].items()}
    steps = None
    if fmt == "smpq-bits/2":
        steps = {int(k): np.array([int(h, 16) for h in v], dtype=np.uint32).view(np.float32)
                 for k, v in side["steps"].items()}
    return bits, steps


def read_sidecar(path):
    """{lnum: int array of bits per channel} from ``<path>.bits.json``, or None."""
    return _read_sidecar_full(path)[0]


def read_sidecar_steps(path):
    """{lnum: fp32 array of exact steps per channel} (format smpq-bits/2), or None."""
    return _read_sidecar_full(path)[1]


def infer_quant_(conv, allowed=None):
    """Record (bit, step) for channels of ``conv`` that carry no metadata but whose weights lie on
    the reference quantizer's grid. ``allowed``: optional int array [cout] restricting channel c to
    bit allowed[c] (0 = leave). Returns the number of channels recorded."""
    w2d = conv.weight.detach().reshape(conv.out_channels, -1).to(torch.float32).contiguous()
    cout = conv.out_channels
    # channels already carrying metadata, and constant channels (the reference quantizer divides
    # by zero on them, functions.py:40), are left alone
    known = conv.qbits.detach().cpu().numpy() > 0
    known |= (w2d.amax(dim=1) == w2d.amin(dim=1)).cpu().numpy()
    found = np.zeros(cout, dtype=np.int64)
    steps = torch.zeros(cout, dtype=torch.float32, device=w2d.device)
    cands = CANDIDATE_BITS if allowed is None else sorted({int(b) for b in np.asarray(allowed) if b > 0})
    for b in cands:
        todo = ~known & (found == 0)
        if allowed is not None:
            todo &= np.asarray(allowed) == b
        if not todo.any():
            continue
        # the channel may have been written by torch on the CPU or on the GPU (functions.py:41
        # rounds differently there, ops.QSEM): either re-quantization that is a fixed point counts
        for sem in ("cpu", "device"):
            todo_s = todo & (found == 0)
            if not todo_s.any():
                break
            work = w2d.clone()
            step = ops.quantize_channels_(work, np.where(todo_s, b, 0), semantics=sem)
            same = (work == w2d).all(dim=1).cpu().numpy() & todo_s
            found[same] = b
            sel = torch.from_numpy(np.nonzero(same)[0]).to(steps.device)
            steps[sel] = step.reshape(-1).to(steps.device)[sel]
    # Re-quantization is not always idempotent (the min/max of a quantized channel round to a
    # grid shifted by an ulp): the rest get a direct grid search on the values
    lo_b = None if allowed is None else np.asarray(allowed)
    for c in np.nonzero(~known & (found == 0))[0]:
        if lo_b is not None and lo_b[c] <= 0:
            continue
        hit = _grid_search(w2d[c].detach().cpu().numpy(),
                           CANDIDATE_BITS if lo_b is None else (int(lo_b[c]),))
        if hit is not None:
            found[c] = hit[0]
            steps[int(c)] = float(hit[1])
    if (found > 0).any():
        conv.record_quant_all(found, steps)
    return int((found > 0).sum())


def _grid_search(v, bits):
    """(b, fp32 step) such that every value is fl32(m * step) for an integer m, with the code span
    of a b-bit reference quantization (2^b - 1, +-1 from rounding); None if no candidate fits."""
    nlev = np.unique(v).size
    if nlev > (1 << max(bits)) + 1:
        return None
    lo, hi = np.float64(v.min()), np.float64(v.max())
    for b in bits:
        if nlev > (1 << b) + 1:
            continue
        for n in ((1 << b) - 1, 1 << b, (1 << b) - 2):
            s = np.float32((hi - lo) / n)
            for k in (0, -1, 1, -2, 2, -3, 3, -4, 4):  # the nearest fp32 steps first
                cand = s
                for _ in range(abs(k)):
                    cand = np.nextafter(cand, np.float32(np.inf if k > 0 else 0), dtype=np.float32)
                m = np.rint(v.astype(np.float64) / np.float64(cand)).astype(np.float32)
                if np.array_equal(m * cand, v):
                    return b, cand
    return None


def _strict_ok(net, state):
    """strict=True for a plain (reference-format) state dict: only the metadata buffers, which the
    QConv2d loader tolerates as missing, may be absent."""
    want = set(net.state_dict())
    missing = {k for k in want - set(state) if not k.endswith(META_KEYS)}
    unexpected = set(state) - want
    if missing or unexpected:
        raise RuntimeError("Error(s) in loading state_dict: missing keys %s, unexpected keys %s"
                           % (sorted(missing)[:8], sorted(unexpected)[:8]))


def load_checkpoint(net, path, map_location="cpu", strict=True):
    """``net.load_state_dict(torch.load(path))`` with a safe loader, then restore the quantization
    metadata: exactly from a smpq-bits/2 sidecar (bits + fp32 steps), else recovered from the
    values (sidecar-guided when a smpq-bits/1 ``<path>.bits.json`` exists). Returns
    {lnum: bits per channel} after loading."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    if strict:
        _strict_ok(net, state)
    net.load_state_dict(state, strict=False)
    side, side_steps = _read_sidecar_full(path)
    has_meta = any(k.endswith(".qbits") for k in state)
    for ln, conv in enumerate(addressable_convs(net), start=1):
        allowed = None
        if side is not None:
            allowed = side.get(ln)
            if allowed is None or not (allowed > 0).any():
                continue
            if len(allowed) != conv.out_channels:
                raise ValueError("sidecar lnum %d: %d channels, conv has %d"
                                 % (ln, len(allowed), conv.out_channels))
            if side_steps is not None and not has_meta:
                st = side_steps.get(ln)
                if st is None or len(st) != conv.out_channels:
                    raise ValueError("sidecar lnum %d: steps missing or of the wrong length" % ln)
                conv.clear_quant()
                conv.record_quant_all(np.asarray(allowed), torch.from_numpy(st.copy()))
                continue
        infer_quant_(conv, allowed)
    return bit_assignment(net)
