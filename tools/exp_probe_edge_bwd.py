"""Edge-backward phase timing (experiment builds with per-wave s_memtime marks
in k_edge_bwd, `sgnn_set_probe`): one C2 training step, then the per-phase
cycle averages over waves and chunks of the last edge-backward launch."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from sgnn_amd.train import Trainer
from sgnn_amd._hip import lib

dev = torch.device("cuda", 0)
dims, radius, H, L = bench.WORKLOADS["c2"]
g, s = bench._train_graph(dims, 2000)
pos = torch.from_numpy(g[:, :bench.T_SEQ]).to(dev)
nxt = torch.from_numpy(g[:, bench.T_SEQ]).to(dev)
strain = torch.from_numpy(s).to(dev)
n = pos.shape[0]
ns = int(sys.argv[1]) if len(sys.argv) > 1 else 512
sim = bench.make_sim(H, L, radius, 2, dev, 0)
tr = Trainer(sim, lr_init=1e-3, nslab=ns)
kw = dict(n_global=n, particle_offset=0)
for _ in range(5):
    tr.train_step(pos, nxt, strain, [n], **kw)
torch.cuda.synchronize()
buf = torch.zeros(ns * 4 * 32, dtype=torch.int64, device=dev)
import ctypes
lib().sgnn_set_probe(ctypes.c_void_p(buf.data_ptr()))
tr.train_step(pos, nxt, strain, [n], **kw)
torch.cuda.synchronize()
lib().sgnn_set_probe(ctypes.c_void_p(0))
t = buf.view(ns * 4, 32).cpu().numpy().astype(np.float64)
t0 = t[:, 0].min()
print(f"nslab={ns}: kernel span {t[:, 31].max() - t0:.0f} cycles; wave start spread "
      f"{np.percentile(t[:, 0] - t0, [0, 50, 90, 100]).round()} ; end spread "
      f"{np.percentile(t[:, 31] - t0, [0, 50, 90, 100]).round()}")
print(f"prologue {np.mean(t[:, 1] - t[:, 0]):.0f}")
names = ["loads+LN", "LN sums", "dy img+sync", "outer+sync", "matvec", "dh st+segsum"]
rows = []
for ci in range(4):
    sl = 2 + 7 * ci
    ok = (t[:, sl] > 0) & (t[:, sl + 6] > 0)
    if not ok.any():
        break
    d = [np.mean(t[ok, sl + k + 1] - t[ok, sl + k]) for k in range(6)]
    rows.append(d)
    print(f"chunk {ci} ({ok.sum()} waves): " + "  ".join(f"{nm}={v:.0f}" for nm, v in zip(names, d))
          + f"  total={sum(d):.0f}")
last = np.array([t[w, 2 + 7 * np.max(np.nonzero(t[w, 2:30:7] > 0)) + 6] for w in range(ns * 4)])
print(f"epilogue {np.mean(t[:, 31] - last):.0f}")
