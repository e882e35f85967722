"""Training experiment: C2 train_step ms/step and per-kernel timer averages for
a list of edge-slab counts (Trainer nslab: the edge / edge-encoder backward
grid), e.g.  python tools/exp_train.py 256 512"""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from sgnn_amd.train import Trainer

dev = torch.device("cuda", 0)
dims, radius, H, L = bench.WORKLOADS["c2"]
g, s = bench._train_graph(dims, 2000)
pos = torch.from_numpy(g[:, :bench.T_SEQ]).to(dev)
nxt = torch.from_numpy(g[:, bench.T_SEQ]).to(dev)
strain = torch.from_numpy(s).to(dev)
n = pos.shape[0]
from sgnn_amd._hip import lib
for arg in sys.argv[1:] or ["256"]:
    ns, _, ab = arg.partition(":")
    ns = int(ns)
    if ab:   # experiment builds only (kernel ablation mask)
        lib().sgnn_set_ablate(int(ab))
    sim = bench.make_sim(H, L, radius, 2, dev, 0)
    tr = Trainer(sim, lr_init=1e-3, nslab=ns)
    kw = dict(n_global=n, particle_offset=0)
    for _ in range(5):
        tr.train_step(pos, nxt, strain, [n], **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        out = tr.train_step(pos, nxt, strain, [n], **kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20
    timers = {}
    for _ in range(10):
        tr.train_step(pos, nxt, strain, [n], timers=timers, **kw)
    torch.cuda.synchronize()
    ks = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e3 for k, v in timers.items()}
    print(f"nslab={ns} ablate={ab or 0}: {dt * 1e3:.3f} ms/step loss={float(out['loss']):.5f} "
          + " ".join(f"{k}={v:.1f}us" for k, v in ks.items()), flush=True)
