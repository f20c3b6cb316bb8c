"""One semilayer step of the reference's search drivers, replayed through the drop-in modules on
the GPU (resnet50_main.py:176-243; resnet18_main.py / resnet34_main.py run the same loop):

  quantize a semilayer channel by channel with ``conv.weight.data =
  functions.channel_wise_quantizationperchan(conv.weight.data, w_bit, cnum)`` (:189-197), then
  ``acc, loss, afteroutputs = functions.evaluate_acc_loss_softmax(net, device, val_loader)`` and
  ``functions.KLdiv(originaloutputs, afteroutputs)`` (:204-205); on ``acc >= preacc``
  ``torch.save(net.state_dict(), pthname)`` (:212), otherwise ``net.load_state_dict(torch.load(
  pthname))`` and a re-evaluation (:233-236).

Checked against the oracle (the reference's CPU forward on the same fake-quantized weights,
oracle/torch_ref.py, and functions.py:84-149 restated in oracle/eval_ref.py) on the same images:
top-1 accuracy exact, loss within 1e-3 relative, KL within 1 % relative (the KL of a semilayer
step is a difference of two nearby softmaxes, so the 2e-4 logit tolerance of DESIGN.md 1 shows
up amplified in it). The rejected step's restore must give the accepted step's evaluation back
bit for bit (every cache — packed codes, folded BN, static ranges, graphs — follows
``load_state_dict``)."""
import os

import pytest
import torch

from test_gpu import build_model

pytestmark = pytest.mark.gpu


def _oracle_eval(arch, net, loader):
    from oracle import eval_ref, torch_ref
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items() if not k.endswith(("qbits", "qstep"))}
    batches = [(torch_ref.resnet_forward(arch, sd, x).numpy(), y.numpy()) for x, y in loader]
    return eval_ref.evaluate_acc_loss_softmax(batches)


def _quantize_semilayer(conv, w_bit, channels):
    import functions
    for cnum in channels:  # resnet50_main.py:189-197, one channel per call
        conv.weight.data = functions.channel_wise_quantizationperchan(conv.weight.data, w_bit, cnum)


@pytest.mark.parametrize("mode", ["static", "dynamic"])
def test_semilayer_step_through_dropin(gpu, tmp_path, monkeypatch, mode):
    import functions
    from oracle import eval_ref
    from smpq import engine
    monkeypatch.setenv("SMPQ_SYNTHETIC", "1")
    import imagenet
    arch = "resnet18"
    net = build_model(gpu, arch, None, "r18_u8_cal")  # BN-recalibrated parity model, fp32 weights
    loader = list(imagenet.SyntheticImageNet(n_images=32, batch_size=16, seed=5))
    # labels the network gets mostly right, so that the accuracy moves with the quantization
    from oracle import torch_ref
    sd0 = {k: v.detach().cpu() for k, v in net.state_dict().items() if not k.endswith(("qbits", "qstep"))}
    loader = [(x, torch.where(torch.arange(len(y)) % 4 == 0, y, torch_ref.resnet_forward(arch, sd0, x).argmax(1)))
              for x, y in loader]
    old_mode = engine.get_range_mode()
    engine.set_range_mode(mode)
    try:
        preacc, preloss, originaloutputs = functions.evaluate_acc_loss_softmax(net, gpu, loader)
        r_acc, r_loss, r_orig = _oracle_eval(arch, net, loader)
        assert preacc == r_acc and abs(preloss - r_loss) <= 1e-3 * abs(r_loss)

        # semilayer 1: every channel of layer2.0.conv1 at 4 bits, accepted
        conv = net.layer2[0].conv1
        _quantize_semilayer(conv, 4, range(conv.out_channels))
        assert conv.fully_quantized()
        acc, loss, afteroutputs = functions.evaluate_acc_loss_softmax(net, gpu, loader)
        kldiv = functions.KLdiv(originaloutputs, afteroutputs)
        r_acc, r_loss, r_after = _oracle_eval(arch, net, loader)
        r_kl = eval_ref.kldiv(r_orig, r_after)
        print("%s step 1: acc %.4f (oracle %.4f) loss %.6f (oracle %.6f) KL %.4e (oracle %.4e)"
              % (mode, acc, r_acc, loss, r_loss, kldiv, r_kl))
        assert acc == r_acc
        assert abs(loss - r_loss) <= 1e-3 * abs(r_loss)
        assert abs(kldiv - r_kl) <= 0.01 * r_kl
        pth = os.path.join(tmp_path, "step.pth")
        torch.save(net.state_dict(), pth)  # resnet50_main.py:212 (acc >= preacc branch)
        accepted = (acc, loss, [o.clone() for o in afteroutputs])

        # semilayer 2: the first half of layer3.1.conv2 at 4 bits, then rejected and restored
        conv2 = net.layer3[1].conv2
        _quantize_semilayer(conv2, 4, range(conv2.out_channels // 2))
        acc2, loss2, out2 = functions.evaluate_acc_loss_softmax(net, gpu, loader)
        r_acc2, r_loss2, r_out2 = _oracle_eval(arch, net, loader)
        assert acc2 == r_acc2 and abs(loss2 - r_loss2) <= 1e-3 * abs(r_loss2)
        net.load_state_dict(torch.load(pth, weights_only=True))  # resnet50_main.py:233-234
        assert not conv2.fully_quantized() and conv2._bits_host.max() == 0  # metadata restored too
        debugacc, debugloss, debugoutputs = functions.evaluate_acc_loss_softmax(net, gpu, loader)  # :236
        assert debugacc == accepted[0] and debugloss == accepted[1]
        for a, b in zip(debugoutputs, accepted[2]):
            assert torch.equal(a, b)
    finally:
        engine.set_range_mode(old_mode)


def test_evaluation_history_independent(gpu):
    """Each evaluation pass calibrates its static ranges on its own first batch
    (engine.new_evaluation): the same weights on the same loader give the same accuracy, loss and
    softmax bit for bit whatever ran before — here a first pass whose second batch overflows (its
    ranges widen) and a pass on a different loader in between."""
    import functions
    from smpq import engine, stats
    net = build_model(gpu, "resnet18", "r18_u8", "r18_u8_cal")
    g = torch.Generator().manual_seed(41)
    xa = torch.randn(8, 3, 224, 224, generator=g)
    ya = torch.randint(0, 1000, (8,), generator=g)
    loader = [(xa, ya), (xa * 4.0, ya), (xa, ya)]  # the x4 batch exceeds ranges calibrated on xa
    assert engine.get_range_mode() == "static"
    o0 = stats["overflow_reruns"]
    r1 = functions.evaluate_acc_loss_softmax(net, gpu, loader)
    assert stats["overflow_reruns"] > o0
    r2 = functions.evaluate_acc_loss_softmax(net, gpu, loader)
    functions.evaluate_acc_loss_softmax(net, gpu, [(xa * 8.0, ya)])  # another history
    r3 = functions.evaluate_acc_loss_softmax(net, gpu, loader)
    for r in (r2, r3):
        assert r[0] == r1[0] and r[1] == r1[1]
        for a, b in zip(r[2], r1[2]):
            assert torch.equal(a, b)


def test_deferred_channel_quantizer(gpu):
    """The drop-in per-channel quantizer on device weights runs without a host sync per call
    (smpq.quant.DEFER): each call gives the same weight bits, recorded step and bit-width as the
    synchronous quantizer, and a constant channel leaves its weights untouched and raises the
    reference's ZeroDivisionError (functions.py:40) at the next forward instead of in the call."""
    import functions
    from smpq import ops, quant
    net = build_model(gpu, "resnet18", None)
    conv = net.layer3[1].conv1
    w0 = conv.weight.detach().clone()
    chans = list(range(0, conv.out_channels, 3))
    for c in chans:
        conv.weight.data = functions.channel_wise_quantizationperchan(conv.weight.data, 6 if c % 2 else 4, c)
    ref = w0.reshape(conv.out_channels, -1).clone()
    bits = [0] * conv.out_channels
    for c in chans:
        bits[c] = 6 if c % 2 else 4
    step = ops.quantize_channels_(ref, bits, semantics="device")
    assert torch.equal(conv.weight.detach().reshape(conv.out_channels, -1), ref)
    assert torch.equal(conv.qstep, step) and conv.qbits.tolist() == bits
    assert int(conv._bits_host.sum()) == sum(bits)
    quant.check_pending()  # nothing to report
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(4)).to(gpu)
    with torch.no_grad():
        net(x)
    # a constant channel: no error in the call, the channel untouched, the error at the next forward
    conv2 = net.layer4[0].conv2
    with torch.no_grad():
        conv2.weight.data[7] = 0.25
    before = conv2.weight.detach().clone()
    # channel 3 quantized before and after (applied), channel 7 constant (its metadata restored)
    functions.channel_wise_quantizationperchan(conv2.weight.data, 6, 3)
    functions.channel_wise_quantizationperchan(conv2.weight.data, 4, 5)
    meta = (conv2.qbits.clone(), conv2.qstep.clone(), conv2._bits_host.copy())
    functions.channel_wise_quantizationperchan(conv2.weight.data, 8, 7)
    functions.channel_wise_quantizationperchan(conv2.weight.data, 4, 3)
    with pytest.raises(ZeroDivisionError):
        with torch.no_grad():
            net(x)
    assert torch.equal(conv2.weight.detach()[7], before[7])
    # the failed channel is not reported as quantized; the later call stays applied
    assert conv2.qbits[7].item() == meta[0][7].item() == 0 and conv2._bits_host[7] == 0
    assert torch.equal(conv2.qstep[7], meta[1][7]) and not conv2.fully_quantized()
    assert conv2.qbits[3].item() == 4 and conv2.qbits[5].item() == 4
    quant.check_pending()  # cleared by the raise
    # the synchronous path (DEFER off) raises in the call, as the reference does
    quant.DEFER[0] = False
    try:
        with pytest.raises(ZeroDivisionError):
            functions.channel_wise_quantizationperchan(conv2.weight.data, 8, 7)
    finally:
        quant.DEFER[0] = True
