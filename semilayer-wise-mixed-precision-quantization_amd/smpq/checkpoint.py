""".pth checkpoints + bit-assignment sidecar.

The reference's drivers checkpoint and roll back with plain state dicts
(resnet50_main.py:212 ``torch.save(net.state_dict(), pthname)``, :233-234 / :426-427
``net.load_state_dict(torch.load(pthname))``). Those files carry fake-quantized fp32 weights
only: the bit-widths are implicit in the values. Our QConv2d keeps ``qbits``/``qstep`` buffers
(qconv.py), so a state dict written by this package reloads with its metadata. This module covers
the other two cases:

* ``save_checkpoint`` writes the state dict plus ``<path>.bits.json``, the per-channel bit
  assignment in the reference's own vocabulary (lnum -> per-channel bits, 0 = never quantized),
  readable without torch by the search drivers' bookkeeping;
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


def save_checkpoint(net, path):
    """``torch.save(net.state_dict(), path)`` + ``<path>.bits.json``."""
    torch.save(net.state_dict(), path)
    side = {"format": "smpq-bits/1", "convs": {str(k): v for k, v in bit_assignment(net).items()}}
    with open(sidecar_path(path), "w") as f:
        json.dump(side, f)


def read_sidecar(path):
    p = sidecar_path(path)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        side = json.load(f)
    if side.get("format") != "smpq-bits/1":
        raise ValueError("%s: unknown sidecar format %r" % (p, side.get("format")))
    return {int(k): np.asarray(v, dtype=np.int64) for k, v in side["convs"].items()}


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
        work = w2d.clone()
        step = ops.quantize_channels_(work, np.where(todo, b, 0))
        same = (work == w2d).all(dim=1).cpu().numpy() & todo
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


def load_checkpoint(net, path, map_location="cpu", strict=True):
    """``net.load_state_dict(torch.load(path))`` with a safe loader, then recover missing
    quantization metadata (sidecar-guided when ``<path>.bits.json`` exists). Returns
    {lnum: bits per channel} after loading."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    net.load_state_dict(state, strict=strict)
    side = read_sidecar(path)
    for ln, conv in enumerate(addressable_convs(net), start=1):
        allowed = None
        if side is not None:
            allowed = side.get(ln)
            if allowed is None or not (allowed > 0).any():
                continue
            if len(allowed) != conv.out_channels:
                raise ValueError("sidecar lnum %d: %d channels, conv has %d"
                                 % (ln, len(allowed), conv.out_channels))
        infer_quant_(conv, allowed)
    return bit_assignment(net)
