"""Which fp32 semantics does torch use on the GPU for the ops of functions.py:41?
(tensor / python float, + python int, .round(), * python float). Writes gpurun_out/torch_ops.json."""
import json
import os

import numpy as np
import torch

out = {}
r = torch.tensor([-52.5, -90.5, 0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 3.5], dtype=torch.float32)
out["round_cpu"] = r.round().tolist()
out["round_dev"] = r.cuda().round().tolist()
g = torch.Generator().manual_seed(7)
t = torch.randn(1 << 22, generator=g) * 0.05
s = 0.0007541168261976804
s32 = np.float32(s)
tn = t.numpy()
dev = (t.cuda() / s).cpu().numpy()
out["div_dev_eq_ieee"] = int((dev == (tn / s32)).sum())
# the two candidate reciprocals: of the fp32 scale (1.0f / fl32(s)) and of the double scale
# rounded once (fl32(1.0 / s), what smpq implements as SMPQ_QSEM_DEVICE)
out["div_dev_eq_recip_of_fl32_scale"] = int((dev == (tn * (np.float32(1) / s32))).sum())
out["div_dev_eq_fl32_recip_of_double_scale"] = int((dev == (tn * np.float32(1.0 / s))).sum())
out["div_n"] = int(tn.size)
q = (t / s).round()
out["add_dev_eq_cpu"] = bool(torch.equal((q.cuda() + (-107)).cpu(), q + (-107)))
out["mul_dev_eq_cpu"] = bool(torch.equal((q.cuda() * s).cpu(), q * s))
x = (torch.arange(-400, 400, dtype=torch.float32) + 0.5)
out["round_half_dev_eq_rne"] = bool(torch.equal(x.cuda().round().cpu(), torch.from_numpy(np.rint(x.numpy()))))
out["round_half_dev_eq_away"] = bool(torch.equal(x.cuda().round().cpu(),
                                                 torch.from_numpy(np.sign(x.numpy()) * np.floor(np.abs(x.numpy()) + 0.5))))
os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/torch_ops.json", "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out))
