"""Round-6 check of the full-size C5 finite-difference test's yardstick (tests/test_gpu_configs.py::
test_c5_full_1m...): on the 9,600-particle C5-width case, where the float64 multi-scale oracle runs, compare
  |g_fused| (the product's gradient, one MultiScaleTrainer step at lr 0),
  u . g64   (the float64 oracle's gradient along u = g_fused / |g_fused|),
  central differences of the PRODUCT's loss along u at several step sizes,
  central differences of the float64 ORACLE's loss along u at the same step sizes.
If the product's differences fall short of |g_fused| by the same fraction as the oracle's fall short of
u . g64, the gap is the finite-difference yardstick's (ReLU kinks / curvature), not the gradient's."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from oracle import multi_scale_oracle as MO
from oracle import sgnn_oracle as O
from sgnn_amd import synthetic
from sgnn_amd.multi_scale import build_static_multi_scale_graph
from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
from tests.test_gpu_configs import _ms_sim, _stats


def main():
    seq = synthetic.trajectory(synthetic.lattice_3d(24, 20, 20, x0=-1.75), 12, seed=13)
    n = seq.shape[0]
    sim = _ms_sim()
    names = [k for k, _ in sim.named_parameters()]
    state0 = {k: v.detach().clone() for k, v in sim.state_dict().items()}
    g_ref = MO.create_all_edges(torch.from_numpy(seq[:, 0]), 2, 2, 2.0)
    pos, nxt = torch.from_numpy(seq[:, :11]), torch.from_numpy(seq[:, 11])
    strain = torch.zeros(n)
    noise = torch.zeros_like(pos)
    sim = sim.cuda()
    g = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), 2, 2, 2.0)
    sim.set_static_graph(g)
    tr = MultiScaleTrainer(sim, lr_init=0.0)
    P, N, S, Z = pos.cuda(), nxt.cuda(), strain.cuda(), noise.cuda()
    tr.train_step(P, N, S, noise=Z)
    torch.cuda.synchronize()
    grad = tr.flat.grad.clone()
    gnorm = float(grad.norm())
    u = grad / gnorm
    flat = tr.flat.param
    # u per parameter tensor (the flat buffer holds parameters() in order)
    u_p = {}
    for k, (off, numel, shape) in zip(names, tr.flat.order):
        u_p[k] = u[off:off + numel].view(shape).cpu().double()

    def oracle_loss(t):
        st = {k: (v.detach().double() + (t * u_p[k] if k in u_p else 0.0)) for k, v in state0.items()}
        o = MO.MultiScaleOracle(st, 3, 10, _stats(3, torch.float64), g_ref, 2, 2.0, 1, 2)
        a, b, c = o.predict_accelerations(nxt.double(), noise.double(), pos.double())
        return O.training_loss(a, b, c, strain.double())

    st64 = {k: v.detach().double().clone().requires_grad_(True) for k, v in state0.items()}
    o = MO.MultiScaleOracle(st64, 3, 10, _stats(3, torch.float64), g_ref, 2, 2.0, 1, 2)
    a, b, c = o.predict_accelerations(nxt.double(), noise.double(), pos.double())
    O.training_loss(a, b, c, strain.double()).backward()
    ug64 = sum(float((st64[k].grad * u_p[k]).sum()) for k in u_p if st64[k].grad is not None)
    print(f"|g_fused| = {gnorm:.6e}   u.g64 = {ug64:.6e}   (rel {abs(gnorm - ug64) / ug64:.2e})")
    for eps in (2e-2, 1e-2, 5e-3, 2.5e-3, 1.25e-3):
        w0 = flat.clone()
        flat.add_(u, alpha=eps)
        lp = float(tr.train_step(P, N, S, noise=Z)["loss"])
        flat.copy_(w0).add_(u, alpha=-eps)
        lm = float(tr.train_step(P, N, S, noise=Z)["loss"])
        flat.copy_(w0)
        fd32 = (lp - lm) / (2 * eps)
        fd64 = (float(oracle_loss(eps)) - float(oracle_loss(-eps))) / (2 * eps)
        print(f"eps {eps:.2e}: product FD {fd32:.6e} ({(fd32 - gnorm) / gnorm:+.2e} of |g|)   "
              f"oracle fp64 FD {fd64:.6e} ({(fd64 - ug64) / ug64:+.2e} of u.g64)", flush=True)


if __name__ == "__main__":
    main()
