"""Device-side content fingerprints of the tensors the engine's caches are built from.

The engine keys its caches (packed weight codes, folded BatchNorm, calibrated ranges, the captured
HIP graph) on what the host can see: tensor identity, data_ptr and ``_version``. Writes through
``.data`` — the reference's own idiom, functions.py:22 and resnet50_main.py:191 — do not bump
``_version``. ``Fingerprinter`` hashes the bytes of those tensors on the GPU
(``smpq_fingerprint``, csrc/fingerprint.hip) when the caches are built and again after every
forward, raising a device flag on any difference, which the engine reads with the overflow flag
(no extra host sync in static mode).
"""
import ctypes

import numpy as np
import torch

from . import _lib


class Fingerprinter:
    """Fingerprints of a fixed list of device tensors (any dtype; contiguous, 4-B aligned). Every
    byte of every tensor is covered (a partial last word is hashed zero-padded); a tensor that
    cannot be covered raises instead of being skipped, so the staleness guarantee has no holes."""

    def __init__(self, tensors, device):
        lib = _lib.load()
        cw = int(lib.smpq_fingerprint_chunk_words())
        self.tensors = [t for t in tensors if t.numel() > 0]
        for t in self.tensors:
            if not (t.is_cuda and t.is_contiguous() and t.data_ptr() % 4 == 0):
                raise ValueError("smpq fingerprint: tensors must be contiguous, 4-B aligned and on the GPU "
                                 "(got %s %s on %s)" % (tuple(t.shape), t.dtype, t.device))
        self.device = device
        ptrs, nbytes, ct, cwd = [], [], [], []
        for i, t in enumerate(self.tensors):
            nb = t.numel() * t.element_size()
            n = (nb + 3) // 4
            ptrs.append(t.data_ptr())
            nbytes.append(nb)
            for w0 in range(0, n, cw):
                ct.append(i)
                cwd.append(w0)
        self.n = len(self.tensors)
        self.enabled = self.n > 0
        if not self.enabled:
            return
        self._ptrs = torch.tensor(np.array(ptrs, dtype=np.uint64).view(np.int64), device=device)
        self._nbytes = torch.tensor(nbytes, dtype=torch.int64, device=device)
        self._layout = tuple(zip(ptrs, nbytes))
        self._ct = torch.tensor(ct, dtype=torch.int32, device=device)
        self._cw = torch.tensor(cwd, dtype=torch.int64, device=device)
        self.ref = torch.empty(self.n, dtype=torch.int64, device=device)
        self.now = torch.empty(self.n, dtype=torch.int64, device=device)
        self.compute(self.ref)

    def compute(self, out):
        lib = _lib.load()
        with torch.cuda.device(self.device):
            _lib.check(lib.smpq_fingerprint(_lib.ptr(self._ptrs), _lib.ptr(self._nbytes), self.n, _lib.ptr(self._ct),
                                            _lib.ptr(self._cw), int(self._ct.numel()), _lib.ptr(out),
                                            _lib.stream_ptr()), "smpq_fingerprint")
        return out

    def same_content(self, other):
        """True when ``other`` fingerprints the same tensors (addresses and sizes) and their
        content was the same then as now (one host sync)."""
        if not self.enabled or not other.enabled:
            return self.enabled == other.enabled
        return self._layout == other._layout and bool(torch.equal(self.ref, other.ref))

    def check(self, flag):
        """Enqueue: flag (device int32 [1]) |= 1 if any tensor's bytes differ from the reference."""
        if not self.enabled:
            return
        self.compute(self.now)
        with torch.cuda.device(self.device):
            _lib.check(_lib.load().smpq_fingerprint_compare(_lib.ptr(self.now), _lib.ptr(self.ref), self.n,
                                                            _lib.ptr(flag), _lib.stream_ptr()),
                       "smpq_fingerprint_compare")


def host_fingerprint(t):
    """The same fingerprint of a host tensor (tests)."""
    t = t.contiguous()
    return int(_lib.load().smpq_fingerprint_host(ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size()))
