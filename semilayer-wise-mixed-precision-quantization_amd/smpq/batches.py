"""Host batches to the device for the evaluation loops (functions.evaluate_acc_loss_softmax /
evaluate_loss, smpq.dp.sharded_eval), with the copy of the next batch overlapping the evaluation of
the current one (the reference copies each batch on the compute stream, functions.py:109-111)."""
import threading

import torch


class DeviceBatches:
    """The batches of ``loader`` on ``dev``, with batch i+1's host-to-device copy in flight on a
    side stream while batch i is being evaluated (the reference copies each batch on the compute
    stream, functions.py:109-111, so copy and forward alternate). Host batches are copied from
    pinned memory: a pinned batch (the reference's DataLoader uses pin_memory=True) directly, any
    other one after a copy into one of two reusable pinned buffers, made on a worker thread while
    the GPU runs. Device batches pass through untouched."""

    def __init__(self, loader, dev):
        self.loader, self.dev = loader, dev
        self.stream = torch.cuda.Stream(device=dev)
        self._pinned = {}    # (shape, dtype) -> [buffer 0, buffer 1]
        self._done = [None, None]  # copy-finished event of each pinned slot
        self._slot = 0

    def _pin(self, t):
        if t.is_pinned():
            return t, None
        key = (tuple(t.shape), t.dtype)
        bufs = self._pinned.get(key)
        if bufs is None:
            bufs = self._pinned[key] = [torch.empty(t.shape, dtype=t.dtype).pin_memory() for _ in range(2)]
        k = self._slot
        self._slot ^= 1
        if self._done[k] is not None:
            self._done[k].synchronize()  # the slot's previous copy has left the buffer
        bufs[k].copy_(t)
        return bufs[k], k

    def _stage(self, x, y):
        """(x, y) -> device tensors + the event that marks their copy done (None: nothing to wait)."""
        if x.is_cuda:
            return x, y, None
        xp, kx = self._pin(x)
        yp = y if (not torch.is_tensor(y) or y.is_pinned()) else y.pin_memory()
        with torch.cuda.stream(self.stream):
            xd = xp.to(self.dev, non_blocking=True)
            yd = yp.to(self.dev, non_blocking=True) if torch.is_tensor(yp) else yp
            ev = torch.cuda.Event()
            ev.record(self.stream)
        if kx is not None:
            self._done[kx] = ev
        return xd, yd, ev

    def __iter__(self):
        it = iter(self.loader)
        nxt = [None]

        from .engine import CAPTURE_LOCK

        def fetch():
            try:
                x, y = next(it)  # the loader's own work (host only) runs beside anything
                # device work waits for a graph capture on the main thread to end (engine.CAPTURE_LOCK)
                with CAPTURE_LOCK, torch.cuda.device(self.dev):
                    nxt[0] = self._stage(x, y)
            except StopIteration:
                nxt[0] = StopIteration
            except BaseException as e:  # noqa: BLE001 -- re-raised in the consuming thread
                nxt[0] = e
        fetch()
        while nxt[0] is not StopIteration:
            if isinstance(nxt[0], BaseException):
                raise nxt[0]
            xd, yd, ev = nxt[0]
            worker = threading.Thread(target=fetch)  # stage batch i+1 while batch i runs
            worker.start()
            main = torch.cuda.current_stream(self.dev)
            if ev is not None:
                main.wait_event(ev)
                xd.record_stream(main)  # allocated on the copy stream, used on this one
                if torch.is_tensor(yd):
                    yd.record_stream(main)
            try:
                yield xd, yd
            finally:
                worker.join()
