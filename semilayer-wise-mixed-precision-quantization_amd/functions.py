"""Drop-in for the reference's ``functions`` module (functions.py:1-612).

Same names, signatures and return values:
  quantize_wgt, channel_wise_quantizationperchan      -> smpq.quant (libsmpq, bit-exact)
  evaluate_loss, evaluate_acc_loss_softmax             -> GPU eval loop over net(x) + the fused
                                                          softmax / CE / top-1 kernel, one host
                                                          sync per call instead of per batch
  KLdiv                                                -> smpq_kl_rows on device (same formula)
  make_divide_minusplusmodels, make_quantizedlists,
  make_semilayers_resnet18/34/50                       -> the search bookkeeping, restated
The reference's quirks that change results are kept on purpose (they are what a drop-in must
reproduce): the dummy sentinel rows appended to the caller's lists, the semilayer split on
``dlists[i][index] <= 0`` indexed by list position (functions.py:171-173), and the sensitivity
pass quantizing the caller's net for its first semilayer before switching to fresh models.
"""
import torch

from smpq import engine, ops
from smpq.batches import DeviceBatches
from smpq.models import ResNet
from smpq.quant import channel_wise_quantizationperchan, quantize_wgt  # noqa: F401

_SENTINEL = [0, 0, 100, 0, 0, 0, 0, 0]


def _run_eval(net, device, data_loader, want_probs):
    """Forward every batch, then the fused softmax / cross-entropy / top-1 kernel
    (smpq_softmax_xent) accumulates [loss_sum, correct, seen, batches] on the device: one host
    sync per evaluation. Host batches reach the device through DeviceBatches (the copy of the
    next batch overlaps this batch's forward). Returns (stats float64 [4] on the device, list of
    softmax outputs)."""
    net.to(device)
    net.eval()
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    stats = torch.zeros(4, dtype=torch.float64, device=dev)
    outputs = []
    if isinstance(net, ResNet):
        engine.new_evaluation(net)  # ranges from this pass's own first batch: history-independent
    batches = DeviceBatches(data_loader, dev) if dev.type == "cuda" else data_loader
    with torch.no_grad():
        for x, y in batches:
            x = x.to(device, non_blocking=True)
            out = net(x).float().contiguous()
            p = ops.softmax_xent(out, y, stats, want_probs=want_probs)
            if want_probs:
                outputs.append(p)
    return stats, outputs


def _finish(stats):
    loss_sum, correct, seen, count = stats.tolist()  # the one host sync
    return correct / seen, loss_sum / count


def evaluate_loss(net, device, data_loader):
    """functions.py:45-82: mean over batches of the batch CE loss (the reference's second,
    redundant forward per batch at :71 only recomputed the prediction, so it is not repeated)."""
    stats, _ = _run_eval(net, device, data_loader, want_probs=False)
    return _finish(stats)[1]


def evaluate_acc_loss_softmax(net, device, data_loader):
    """functions.py:84-129: (top-1 accuracy, mean batch loss, list of per-batch softmax)."""
    stats, outs = _run_eval(net, device, data_loader, want_probs=True)
    acc, loss = _finish(stats)
    return acc, loss, outs


def KLdiv(n_out, out):
    """functions.py:131-149: mean over images of sum_c p_c * log(p_c / q_c) (smpq_kl_rows per
    batch pair, accumulated on the device, one host sync)."""
    stats = None
    for p, q in zip(n_out, out):
        if stats is None:
            stats = torch.zeros(2, dtype=torch.float64, device=q.device)
        ops.kl_rows(p.to(q.device), q, stats)
    s, n = stats.tolist()
    return s / n


def make_divide_minusplusmodels(paramlists, dlists, index):
    """functions.py:151-184: split rows into (delta <= 0, delta > 0) semilayer lists; flag
    counters move by one whenever the layer number changes between consecutive rows."""
    minus, plus = [], []
    mflag, pflag = 0, 1
    last = len(paramlists) - 1
    for i, row in enumerate(paramlists):
        base = [row[0], row[1], row[2], row[3], row[4]]
        tail = [row[6], row[7]]
        if dlists[i][index] <= 0:
            minus.append(base + [mflag] + tail)
        else:
            plus.append(base + [pflag] + tail)
        if i == last:
            print('function debug:number of total channels=', len(minus) + len(plus),
                  'No.1:', len(minus), 'No.2:', len(plus))
            break
        if row[2] != paramlists[i + 1][2]:
            mflag -= 1
            pflag += 1
    return minus, plus


def _target_conv(layers, arch, layer_index, block_index, lnum):
    blk = layers[layer_index][block_index]
    if arch == "resnet50":
        return (blk.conv3, blk.conv1, blk.conv2)[lnum % 3]
    return blk.conv1 if lnum % 2 != 0 else blk.conv2


def _make_semilayers(net, device, originaloutputs, listminus, listplus, arch):
    import imagenet
    import resnet
    semilayers, orders = [], []
    index = 0
    for lst in (listminus, listplus):
        lst.append(list(_SENTINEL))
    layers = [net.layer1, net.layer2, net.layer3, net.layer4]
    for lst in (listminus, listplus):
        group, param, counta = [], 0.0, 0
        for i, row in enumerate(lst):
            layer_index, block_index, lnum, cnum, w_bit = row[0], row[1], row[2], row[3], row[4]
            if lnum == 100:
                break
            group.append(list(row))
            conv = _target_conv(layers, arch, layer_index, block_index, lnum)
            conv.weight.data = channel_wise_quantizationperchan(conv.weight.data, w_bit, cnum)
            param += conv.weight[cnum].data.numel() * ((32 - w_bit) / 32)
            counta += 1
            if lnum != lst[i + 1][2]:
                semilayers.append(group)
                _, _, afteroutputs = evaluate_acc_loss_softmax(net, device, imagenet.val_loader)
                kldiv = KLdiv(originaloutputs, afteroutputs) / param
                print(w_bit, 'bit', 'semilayer-No.', index, 'layernumber=', lnum, 'channels=', counta,
                      'total KL divergence=', kldiv)
                orders.append([index, kldiv])
                net = getattr(resnet, arch)(num_classes=1000, pretrained='imagenet')
                layers = [net.layer1, net.layer2, net.layer3, net.layer4]
                group, param, counta = [], 0.0, 0
                index += 1
    return semilayers, orders


def make_semilayers_resnet18(net, device, originaloutputs, listminus, listplus):
    """functions.py:186-319."""
    return _make_semilayers(net, device, originaloutputs, listminus, listplus, "resnet18")


def make_semilayers_resnet34(net, device, originaloutputs, listminus, listplus):
    """functions.py:321-454."""
    return _make_semilayers(net, device, originaloutputs, listminus, listplus, "resnet34")


def make_semilayers_resnet50(net, device, originaloutputs, listminus, listplus):
    """functions.py:456-588."""
    return _make_semilayers(net, device, originaloutputs, listminus, listplus, "resnet50")


def make_quantizedlists(semilayers, orders):
    """functions.py:590-612: concatenate semilayers in ascending sensitivity + sentinel row."""
    orders.sort(key=lambda x: x[1])
    flat = []
    for inum, _ in orders:
        flat.extend(list(r) for r in semilayers[inum])
        print('debug layernum=', semilayers[inum][-1][2], 'number of channels=', len(semilayers[inum]))
    print('number of valuationfirsts list=', len(flat))
    flat.append(list(_SENTINEL))
    return flat
