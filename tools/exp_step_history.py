import sys, os
sys.path.insert(0, "/root/repo"); os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from sgnn_amd import synthetic
from sgnn_amd.multi_scale import build_static_multi_scale_graph
from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
from tests.test_gpu_configs import _ms_sim
dims = tuple(int(v) for v in sys.argv[1:4])
base = synthetic.lattice_3d(*dims); base[:, 0] -= 2.0
seq = synthetic.trajectory(base, 12, seed=3000); n = seq.shape[0]
g = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), 2, 2, 2.0)
sim = _ms_sim().cuda(); sim.set_static_graph(g)
pos = torch.from_numpy(seq[:, :11]).cuda(); nxt = torch.from_numpy(seq[:, 11]).cuda()
strain = torch.zeros(n, device="cuda"); noise = torch.zeros_like(pos)
tr = MultiScaleTrainer(sim, lr_init=0.0)
def L():
    out = tr.train_step(pos, nxt, strain, noise=noise); torch.cuda.synchronize(); return float(out["loss"]), tr.flat.grad.clone()
la, ga = L()
flat = tr.flat.param; w0 = flat.clone()
u = ga / ga.norm()
for eps in (2e-2, 1e-2):
    flat.copy_(w0).add_(u, alpha=eps); lp, _ = L()
    flat.copy_(w0); lb, gb = L()
    print(f"n={n} eps={eps}: L(w0) first {la:.9e}, L(w0+eps u) {lp:.9e}, L(w0) again {lb:.9e}; grad equal: {torch.equal(ga, gb)}  max|dg| {float((ga-gb).abs().max()):.3e}", flush=True)
    # the reverse order: a second L(w0) after L(w0) again
    lc, gc = L()
    print(f"   L(w0) third {lc:.9e}  grad equal to second: {torch.equal(gb, gc)}", flush=True)
