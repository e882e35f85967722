"""GPU parity of the multi-scale training step (SURVEY.md §8 C5 path): HIP
forward-with-saves + fused backward over the three static graphs + slab
reduction + Adam, against the reference's own step (golden ms_train2d) and
oracle autograd at H = 128 in 3D.  Tolerances as tests/test_gpu_training.py."""
import numpy as np
import pytest
import torch

from tests.helpers import golden, hparams, ms_graph_of, state_of, stats_of
from tests.test_gpu_training import _grad_close

pytestmark = pytest.mark.gpu


def _sim(z, prefix="w0/"):
    from sgnn_amd.multi_scale import MultiScaleSimulator
    hp = hparams(z)
    d, T, H = hp["dim"], hp["T"], hp["H"]
    sim = MultiScaleSimulator(d, (T - 1) * d + 1, d + 1, H, H, hp["L"], hp["nmlp"], stats_of(z, "cuda"), 1, 9,
                              hp["num_scales"], hp["window"], hp["mult"])
    sim.load_state_dict(state_of(z, prefix))
    sim = sim.cuda()
    sim.set_static_graph(ms_graph_of(z, "cuda"))
    return sim


def _inputs(z):
    T = hparams(z)["T"]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t(z["positions"][:, :T]), t(z["next_position"]), t(z["next_strain"]), t(z["noise"])


def test_multi_scale_trainer_step_matches_reference():
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    z = golden("ms_train2d")
    sim = _sim(z)
    tr = MultiScaleTrainer(sim, lr_init=float(z["lr"]))
    pos, nxt, strain, noise = _inputs(z)
    out = tr.train_step(pos, nxt, strain, noise=noise)
    torch.cuda.synchronize()
    loss = float(out["loss"])
    print(f"loss {loss:.7f} ref {float(z['loss']):.7f}")
    assert abs(loss - float(z["loss"])) <= 1e-5 * abs(float(z["loss"]))
    grads = {k: p.grad for k, p in sim.named_parameters()}
    worst = 0.0
    for k in z.files:
        if k.startswith("g/"):
            worst = max(worst, _grad_close(grads[k[2:]].cpu().numpy(), z[k], k))
    print(f"worst relative grad error {worst:.3e}")
    sd = sim.state_dict()
    for k in z.files:
        if k.startswith("w1/") and ("g/" + k[3:]) in z.files:
            np.testing.assert_allclose(sd[k[3:]].cpu().numpy(), z[k], rtol=1e-5, atol=2e-5, err_msg=k)


def test_multi_scale_autograd_matches_reference():
    z = golden("ms_train2d")
    sim = _sim(z)
    pos, nxt, strain, noise = _inputs(z)
    pa, ta, ps = sim.predict_accelerations(nxt, noise, pos, [pos.shape[0]], None)
    np.testing.assert_allclose(ta.detach().cpu().numpy(), z["target_acc"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(pa.detach().cpu().numpy(), z["pred_acc"], rtol=1e-4, atol=2e-5)
    loss = ((((pa - ta) ** 2).sum(-1)) + (ps - strain) ** 2).mean()   # multi_scale_train.py:162-173
    loss.backward()
    for k, p in sim.named_parameters():
        if ("g/" + k) in z.files:
            _grad_close(p.grad.cpu().numpy(), z["g/" + k], k)


def test_multi_scale_backward_deterministic():
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    z = golden("ms_train2d")
    pos, nxt, strain, noise = _inputs(z)
    outs = []
    for _ in range(2):
        tr = MultiScaleTrainer(_sim(z), lr_init=1e-3)
        tr.train_step(pos, nxt, strain, noise=noise)
        torch.cuda.synchronize()
        outs.append(tr.flat.grad.cpu().clone())
    assert torch.equal(outs[0], outs[1])


def test_multi_scale_3d_h128_gradients_against_oracle():
    """Config-5 widths (3D, H = 128, nmlp_layers 2, 2 scales) on a lattice the
    oracle differentiates in seconds; graph built on the GPU."""
    from oracle import multi_scale_oracle as MO
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import MultiScaleSimulator, build_static_multi_scale_graph
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    dim, T, H, L = 3, 6, 128, 2
    seq = synthetic.trajectory(synthetic.lattice_3d(12, 8, 6, x0=-1.75), T + 1, seed=13)
    n = seq.shape[0]
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(21)
    sim = MultiScaleSimulator(dim, (T - 1) * dim + 1, dim + 1, H, H, L, 2, stats, 1, 9, 2, 2, 2.0)
    state = {k: v.detach().clone().requires_grad_(True) for k, v in sim.state_dict().items()}
    g_ref = MO.create_all_edges(torch.from_numpy(seq[:, 0]), 2, 2, 2.0)
    osim = MO.MultiScaleOracle(state, dim, L, stats, g_ref, 2, 2.0, 1, 2)
    pos, nxt = torch.from_numpy(seq[:, :T]), torch.from_numpy(seq[:, T])
    strain = torch.from_numpy(np.random.default_rng(4).normal(0, 1, n).astype(np.float32))
    noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(5))
    pa, ta, ps = osim.predict_accelerations(nxt, noise, pos)
    ref_loss = O.training_loss(pa, ta, ps, strain)
    ref_loss.backward()
    sim = sim.cuda()
    sim.set_static_graph(build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), 2, 2, 2.0))
    tr = MultiScaleTrainer(sim, lr_init=1e-3)
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), noise=noise.cuda())
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - ref_loss.item()) <= 2e-5 * abs(ref_loss.item())
    worst = 0.0
    for k, p in sim.named_parameters():
        if state[k].grad is not None:
            worst = max(worst, _grad_close(p.grad.cpu().numpy(), state[k].grad.numpy(), k, rel=5e-4))
    print(f"multi-scale 3D H=128: worst relative grad error {worst:.3e}")
