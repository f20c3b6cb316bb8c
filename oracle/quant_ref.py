"""ORACLE — test infrastructure only (see oracle/__init__.py).

Bit-exact numpy restatement of the reference weight fake-quantizer.

Reference: ``functions.py:25-43`` (``quantize_wgt``) and ``functions.py:9-23``
(``channel_wise_quantizationperchan``).

Arithmetic, step by step, as the reference executes it on CPU torch:
  * ``min_value = torch.min(t).item()`` / ``max`` (functions.py:35-36): exact fp32 values,
    promoted to Python doubles.
  * ``scale = (max - min) / (2**bit - 1)`` (functions.py:39): IEEE double.
  * ``z = round(min / scale)`` (functions.py:40): Python banker's rounding of a double;
    ``ZeroDivisionError`` when max == min.
  * ``(((t / scale) + z).round() - z) * scale`` (functions.py:41): fp32 tensor ops with the
    Python scalars wrapped to fp32, i.e. ``t / fp32(scale)`` (true IEEE division, not a
    reciprocal multiply), ``+ fp32(z)``, round-half-even, ``- fp32(z)``, ``* fp32(scale)``.
  * ``semantics="device"``: the same line executed by torch on a GPU tensor (the reference's
    drivers quantize a model already on the GPU, functions.py:97 before resnet50_main.py:189-197):
    ``t / scale`` becomes ``t * fp32(1.0 / scale)`` (reciprocal of the double scale, rounded once).
    Pinned by tests/golden/quant_kat_device.npz (torch's own output on an MI355X).
"""
import numpy as np


def _quotient(t, scale, semantics):
    if semantics == "device":
        return t * np.float32(1.0 / scale)
    if semantics != "cpu":
        raise ValueError("semantics must be 'cpu' or 'device'")
    return t / np.float32(scale)


def quantize_wgt(tensor, bit, semantics="cpu"):
    """functions.py:25-43 — returns a new float32 array."""
    t = np.asarray(tensor, dtype=np.float32)
    min_value = float(t.min())
    max_value = float(t.max())
    scale = (max_value - min_value) / (2 ** bit - 1)
    z = round(min_value / scale)  # raises ZeroDivisionError for a constant channel
    s32 = np.float32(scale)
    z32 = np.float32(z)
    with np.errstate(all="ignore"):
        q = np.rint(_quotient(t, scale, semantics) + z32) - z32
        return (q * s32).astype(np.float32)


def quantize_codes(tensor, bit):
    """Integer codes m and fp32 step s32 such that quantize_wgt(t) == fl32(m * s32)."""
    t = np.asarray(tensor, dtype=np.float32)
    min_value = float(t.min())
    max_value = float(t.max())
    scale = (max_value - min_value) / (2 ** bit - 1)
    z = round(min_value / scale)
    s32 = np.float32(scale)
    z32 = np.float32(z)
    m = np.rint((t / s32) + z32) - z32
    return m.astype(np.int32), s32


def channel_wise_quantizationperchan(tensor, bit, i):
    """functions.py:9-23 — quantizes row ``i`` in place and returns the same array."""
    tensor[i] = quantize_wgt(tensor[i], bit)
    return tensor


def apply_chain(w, chain, semantics="cpu"):
    """Apply the quantizer once per chain element, in order (Q4(Q8(w)) etc.)."""
    out = np.asarray(w, dtype=np.float32).copy()
    for b in chain:
        if b:
            out = quantize_wgt(out, int(b), semantics)
    return out
