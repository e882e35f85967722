"""Is the C2 training step host-bound?  Host time to issue K steps (no sync)
vs the wall time until the GPU is done."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from sgnn_amd.train import Trainer
dev = torch.device("cuda:0")
dims, radius, H, L = bench.WORKLOADS["c2"]
sim = bench.make_sim(H, L, radius, 2, dev, 0)
g, st = bench._train_graph(dims, 2000)
pos = torch.from_numpy(g[:, :bench.T_SEQ]).to(dev); nxt = torch.from_numpy(g[:, bench.T_SEQ]).to(dev)
strain = torch.from_numpy(st).to(dev)
tr = Trainer(sim, lr_init=1e-3)
for _ in range(3): tr.train_step(pos, nxt, strain, [pos.shape[0]], n_global=pos.shape[0], particle_offset=0)
torch.cuda.synchronize()
K = 20
t0 = time.perf_counter()
for _ in range(K): tr.train_step(pos, nxt, strain, [pos.shape[0]], n_global=pos.shape[0], particle_offset=0)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host issue {1e3 * (t1 - t0) / K:.3f} ms/step, wall {1e3 * (t2 - t0) / K:.3f} ms/step")
