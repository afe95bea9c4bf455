import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, synthetic_cells
dev = torch.device("cuda", 0)
r = CellposeRunner(device=dev, seed=1)
batches = [torch.from_numpy(synthetic_cells(3, 256, 256, ncells=25, seed=s)).to(dev) for s in range(4)]
a = [r.eval(b) for b in batches]
b2 = [r.eval(b) for b in batches]
for i, ((m1, f1, s1), (m2, f2, s2)) in enumerate(zip(a, b2)):
    print("eval vs eval", i, (f1 - f2).abs().max().item(), (s1 - s2).abs().max().item(), (m1 != m2).float().mean().item())
st = r.stream()
got = [st.submit(b) for b in batches] + [st.flush()]
for i, ((m, f, s), (mr, fr, sr)) in enumerate(zip(got[1:], a)):
    print("stream vs eval", i, (f - fr).abs().max().item(), (s - sr).abs().max().item(), (m != mr).float().mean().item())
# stream with a sync after each submit
st = r.stream()
got2 = []
for b in batches:
    got2.append(st.submit(b)); torch.cuda.synchronize()
got2.append(st.flush())
for i, ((m, f, s), (mr, fr, sr)) in enumerate(zip(got2[1:], a)):
    print("stream+sync vs eval", i, (f - fr).abs().max().item(), (s - sr).abs().max().item())
# flows straight from _net_stage
for i, bt in enumerate(batches):
    from bioengine_worker_amd.cellpose.pipeline import EvalParams, as_batch
    y, style, rescale = r._net_stage(as_batch(bt, r.nchan, dev), EvalParams())
    print("net_stage vs eval", i, (y - a[i][1]).abs().max().item())
