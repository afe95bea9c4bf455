import time, torch, sys
sys.path.insert(0, '.')
from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine, to_nhwc_input
net = CPnet().randomize_(0).eval()
dev = torch.device('cuda')
eng = CPnetEngine(net, dev)
for B in (8, 32):
    x = torch.randn(B, 2, 512, 512, device=dev)
    xin = to_nhwc_input(x, 8)
    y, s = eng(xin); torch.cuda.synchronize()
    t = time.time(); n = 10
    for _ in range(n): y, s = eng(xin)
    torch.cuda.synchronize(); dt = (time.time() - t) / n
    print(f"fused engine B={B}: {dt*1e3:.2f} ms -> {B/dt:.1f} img/s", flush=True)
    netg = net.to(dev).to(memory_format=torch.channels_last)
    xb = x.to(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        yr = netg(xb)[0]; torch.cuda.synchronize(); t = time.time()
        for _ in range(n): yr = netg(xb)[0]
        torch.cuda.synchronize(); dt = (time.time() - t) / n
    print(f"torch eager bf16 autocast channels_last B={B}: {dt*1e3:.2f} ms -> {B/dt:.1f} img/s", flush=True)
    print("max diff", (y.float() - yr.float()).abs().max().item(), yr.abs().max().item())
    net = net.cpu()
