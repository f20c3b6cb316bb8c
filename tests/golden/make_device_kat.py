"""Device quantizer KAT: the reference's quantize_wgt formula (functions.py:25-43) evaluated by
torch itself on GPU tensors, over the inputs of quant_kat.npz.

The reference's drivers quantize weights that already live on the GPU (evaluate_acc_loss_softmax
moves the net with net.to(device), functions.py:97, before the search loop quantizes channels of
it, e.g. resnet50_main.py:189-197). On a device tensor torch evaluates ``t / scale`` (scale a
Python float) as ``t * fl32(1.0 / scale)`` — a multiply by the reciprocal of the DOUBLE scale,
rounded to fp32 once (not ``1.0f / fl32(scale)``: over this file's 71 cases the former matches
all of them and the latter misses 4) — which can differ from the CPU's IEEE division by one ulp
and flip rint() at a .5 boundary. This script records what torch
produces there, so the device kernel's semantics are pinned by torch's own device arithmetic.

Run on the GPU box (the reference itself does not travel; the formula below is functions.py:35-41
with the same torch operators, on device tensors):
    python tests/golden/make_device_kat.py gpurun_out/quant_kat_device.npz
then copy the file to tests/golden/.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def quantize_wgt_torch(tensor, bit):
    """functions.py:25-43, the same torch operators on whatever device ``tensor`` lives on."""
    min_weight = torch.min(tensor).item()
    max_weight = torch.max(tensor).item()
    scale = (max_weight - min_weight) / (2 ** bit - 1)
    zero_point = round(min_weight / scale)
    return (((tensor / scale) + zero_point).round() - zero_point) * scale


def main(out):
    assert torch.cuda.is_available(), "run on the GPU box"
    d = np.load(os.path.join(HERE, "quant_kat.npz"))
    x, offs, chains = d["x"], d["offsets"], d["chain"]
    ys = []
    nd_cases = 0
    for i in range(len(chains)):
        t = torch.from_numpy(x[offs[i]:offs[i + 1]].copy()).cuda()
        for b in chains[i]:
            if b:
                t = quantize_wgt_torch(t, int(b))
        y = t.cpu().numpy()
        if not np.array_equal(y.view(np.uint32), d["y"][offs[i]:offs[i + 1]].view(np.uint32)):
            nd_cases += 1
        ys.append(y)
    # extra cases where reciprocal multiply and IEEE division disagree after rint: random
    # channels, kept only if the device result differs from the CPU result
    g = torch.Generator().manual_seed(4321)
    ex_in, ex_out, ex_cpu, ex_bits, ex_offs = [], [], [], [], [0]
    tries = 0
    while len(ex_bits) < 24 and tries < 20000:
        tries += 1
        size = (9, 64, 576, 1152)[tries % 4]
        b = (8, 6, 4, 2)[(tries // 4) % 4]
        t = torch.randn(size, generator=g) * 0.05
        yc = quantize_wgt_torch(t, b)
        yd = quantize_wgt_torch(t.cuda(), b).cpu()
        if not torch.equal(yc, yd):
            ex_in.append(t.numpy())
            ex_out.append(yd.numpy())
            ex_cpu.append(yc.numpy())
            ex_bits.append(b)
            ex_offs.append(ex_offs[-1] + size)
    np.savez_compressed(out, y_device=np.concatenate(ys), differs_from_cpu_cases=np.array(nd_cases),
                        ex_x=np.concatenate(ex_in) if ex_in else np.zeros(0, np.float32),
                        ex_y_device=np.concatenate(ex_out) if ex_out else np.zeros(0, np.float32),
                        ex_y_cpu=np.concatenate(ex_cpu) if ex_cpu else np.zeros(0, np.float32),
                        ex_bits=np.array(ex_bits, dtype=np.int8), ex_offsets=np.array(ex_offs, dtype=np.int64),
                        ex_tries=np.array(tries), torch_version=np.array(torch.__version__))
    print("device KAT: %d of %d KAT cases differ from the CPU goldens; %d extra differing cases in %d tries"
          % (nd_cases, len(chains), len(ex_bits), tries))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "quant_kat_device.npz"))
