import torch, time, sys, os
sys.path.insert(0, os.getcwd())
n = 16384*16384*3
x = torch.randint(0, 255, (n,), dtype=torch.uint8, device='cuda')
y = torch.empty_like(x)
for _ in range(5): y.copy_(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): y.copy_(x)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1)/50
print(f"torch copy_ {n/2**20:.0f} MiB: {ms:.4f} ms  {2*n/ms/1e9:.1f} TB/s")
