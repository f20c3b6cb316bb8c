import torch
"""Diagnostics: do timing events recorded during HIP graph capture time kernels on replay?"""
x = torch.randn(4096, 4096, device="cuda")
y = x @ x  # initialise the GEMM library outside the capture
evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
s = torch.cuda.Stream()
with torch.cuda.graph(g):
    evs[0].record(); y = x @ x; evs[1].record(); z = y @ y; z2 = z @ z; evs[2].record()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("graph events ms:", evs[0].elapsed_time(evs[1]), evs[1].elapsed_time(evs[2]))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); y = x @ x; e1.record(); torch.cuda.synchronize()
print("eager one matmul ms:", e0.elapsed_time(e1))
