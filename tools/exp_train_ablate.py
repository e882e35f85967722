"""Training experiment: C2 train_step ms/step with chosen library calls replaced
by no-ops (results are wrong; the time each call's removal saves bounds what
speeding it up can gain).  python tools/exp_train_ablate.py [name ...]"""
import os, sys, time
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
L_ = lib()
orig = {}


def run(tag):
    sim = bench.make_sim(H, L, radius, 2, dev, 0)
    tr = Trainer(sim, lr_init=1e-3)
    kw = dict(n_global=n, particle_offset=0)
    for _ in range(5):
        tr.train_step(pos, nxt, strain, [n], **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        tr.train_step(pos, nxt, strain, [n], **kw)
    torch.cuda.synchronize()
    print(f"{tag:40s} {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step", flush=True)


run("baseline")
for spec in sys.argv[1:]:
    names = spec.split("+")
    for nm in names:
        orig[nm] = getattr(L_, nm)
        setattr(L_, nm, lambda *a, **k: 0)
    run("without " + spec)
    for nm in names:
        setattr(L_, nm, orig[nm])
