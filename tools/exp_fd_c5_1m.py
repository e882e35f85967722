"""Round-6 localisation experiment: per-parameter-tensor central differences of the C5 training loss at the
full 1M-particle size (100^3 lattice at the wall, as tests/test_gpu_configs.py::test_c5_full_1m...), each
tensor's gradient direction u_k = g_k / |g_k| against (L(w + eps u_k) - L(w - eps u_k)) / (2 eps).  On the
9.6k case both the product's and the float64 oracle's differences converge to |g| (tools/exp_fd_c5.py).
Usage: python tools/exp_fd_c5_1m.py [nx ny nz] [eps ...]"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

from sgnn_amd import synthetic
from sgnn_amd.multi_scale import build_static_multi_scale_graph
from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
from tests.test_gpu_configs import _ms_sim


def main():
    dims = tuple(int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (100, 100, 100)
    epss = [float(v) for v in sys.argv[4:]] or [5e-3, 2.5e-3]
    base = synthetic.lattice_3d(*dims)
    base[:, 0] -= 2.0
    seq = synthetic.trajectory(base, 12, seed=3000)
    n = seq.shape[0]
    g = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), 2, 2, 2.0)
    print(f"n = {n}; edges: " + ", ".join(f"{k} {g[k].shape[1]}" for k in ("grid2mesh_edges", "mesh2mesh_edges",
                                                                        "mesh2grid_edges")), flush=True)
    sim = _ms_sim().cuda()
    names = [k for k, _ in sim.named_parameters()]
    sim.set_static_graph(g)
    pos = torch.from_numpy(seq[:, :11]).cuda()
    nxt = torch.from_numpy(seq[:, 11]).cuda()
    strain = torch.zeros(n, device="cuda")
    noise = torch.zeros_like(pos)
    tr = MultiScaleTrainer(sim, lr_init=0.0)
    L0 = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
    grad = tr.flat.grad.clone()
    flat = tr.flat.param
    w0 = flat.clone()
    gn_all = float(grad.norm())
    u_all = grad / gn_all
    for eps in (1e-2, 5e-3, 2.5e-3, 1.25e-3, 6.25e-4, 3.125e-4):   # the whole gradient's direction first
        flat.copy_(w0).add_(u_all, alpha=eps)
        lp = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
        flat.copy_(w0).add_(u_all, alpha=-eps)
        lm = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
        f = (lp - lm) / (2 * eps)
        print(f"whole gradient: |g| {gn_all:.6e}  eps {eps:.3e}  FD {f:.6e}  rel {(f - gn_all) / gn_all:+.3e}", flush=True)
    flat.copy_(w0)
    if os.environ.get("FD_WHOLE_ONLY"):
        return
    rows = []
    for k, (off, numel, shape) in zip(names, tr.flat.order):
        gk = grad[off:off + numel]
        gn = float(gk.norm())
        if gn == 0.0:
            continue
        u = torch.zeros_like(grad)
        u[off:off + numel] = gk / gn
        fds = []
        for eps in epss:
            flat.copy_(w0).add_(u, alpha=eps)
            lp = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
            flat.copy_(w0).add_(u, alpha=-eps)
            lm = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
            fds.append((lp - lm) / (2 * eps))
        flat.copy_(w0)
        rel = [(f - gn) / gn for f in fds]
        rows.append((abs(rel[-1]), k, gn, fds, rel))
        print(f"{k:70s} |g| {gn:.4e}  FD " + " ".join(f"{f:.4e}" for f in fds) + "  rel " +
              " ".join(f"{r:+.2e}" for r in rel), flush=True)
    print(f"L0 = {L0:.6e}")
    print("worst tensors:")
    for r in sorted(rows, reverse=True)[:15]:
        print(f"  {r[1]:70s} rel {r[4][-1]:+.3e} |g| {r[2]:.4e}")


if __name__ == "__main__":
    main()
