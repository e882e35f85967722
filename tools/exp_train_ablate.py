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
def noop_when(fn, which):
    """sgnn_edge_latent_grad@dw: only the per-layer dW1e launches (de0t = NULL);
    @de0: only the dE0 pass (de0t set)."""
    def f(*a):
        is_dw = a[8] is None
        if (which == "dw") == is_dw:
            return 0
        return fn(*a)
    return f


from sgnn_amd import training as _training


for spec in sys.argv[1:]:
    if spec.startswith("flag:"):   # flag:NAME=0|1 toggles a module switch of sgnn_amd.training
        name, _, val = spec[5:].partition("=")
        old = getattr(_training, name)
        setattr(_training, name, bool(int(val)))
        run(spec)
        setattr(_training, name, old)
        continue
    names = spec.split("+")
    for nm in names:
        base, _, which = nm.partition("@")
        orig[nm] = getattr(L_, base)
        setattr(L_, base, noop_when(orig[nm], which) if which else (lambda *a, **k: 0))
    run("without " + spec)
    for nm in names:
        setattr(L_, nm.partition("@")[0], orig[nm])
