"""ORACLE — test infrastructure only (see oracle/__init__.py).

numpy restatement of the evaluation reductions that follow each forward of the search:

  * ``evaluate_acc_loss_softmax`` (functions.py:84-129): per batch ``output.max(1)`` (the first
    maximal class), ``CrossEntropyLoss`` (mean over the batch, :116), ``Softmax(dim=1)`` (:117);
    ``acc = #(y == y_pred) / N`` (:125), ``loss = sum of batch losses / #batches`` (:126-128).
  * ``KLdiv`` (functions.py:131-149): per image ``sum_c n * log(n / o)``, mean over images.

The reference computes in fp32 torch; this restatement computes in float64 (the checker's
reference values), fp32 rounding differences are inside the tolerances the tests state.
Pinned against the reference's own outputs on the same logits: tests/golden/eval_golden.npz
(tests/golden/make_golden.py imports the reference and runs these two functions).
"""
import numpy as np


def softmax(x):
    x = np.asarray(x, np.float64)
    e = np.exp(x - x.max(axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def evaluate_acc_loss_softmax(batches):
    """batches: list of (logits [B, C], labels [B]) -> (acc, loss, [softmax per batch])."""
    correct, seen, losses, outs = 0, 0, [], []
    for x, y in batches:
        x = np.asarray(x, np.float64)
        y = np.asarray(y, np.int64)
        pred = x.argmax(axis=1)  # numpy: first maximal index
        m = x.max(axis=1)
        lse = m + np.log(np.exp(x - m[:, None]).sum(axis=1))
        losses.append(float(np.mean(lse - x[np.arange(len(y)), y])))
        correct += int((pred == y).sum())
        seen += len(y)
        outs.append(softmax(x))
    return correct / seen, sum(losses) / len(losses), outs


def kldiv(n_out, out):
    """functions.py:131-149 over lists of per-batch softmax arrays."""
    kls = []
    for a, b in zip(n_out, out):
        a = np.asarray(a, np.float64)
        b = np.asarray(b, np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            kls.extend((a * np.log(a / b)).sum(axis=1))
    return float(sum(kls) / len(kls))
