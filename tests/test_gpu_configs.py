"""GPU parity at the BASELINE configurations themselves (BASELINE.json
`configs`), not only at fixture sizes.

  C2  2D 50k, L = 5, H = 64: a full training step (noise injected) against
      oracle autograd in float64 — loss, every parameter gradient, and the
      fused Adam update against torch.optim.Adam applied to the same gradient.
  C4  3D, L = 10, H = 128: forward and a full training step on a 9,600-particle
      lattice against the float64 oracle; at the full 200k size the radius
      graph is bit-exact against the oracle's cell-list search and every
      prediction of an interior corner block equals the oracle run on that
      block alone (the L-hop locality of message passing: nodes more than L
      hops from the cut see identical neighbourhoods).
  C5  multi-scale 3D, L = 10, H = 128, nmlp_layers = 2: forward and gradients
      on 9,600 particles against the float64 multi-scale oracle; at 1M
      particles the hierarchy and the three static edge lists are bit-exact
      against the oracle, the training step is finite and bitwise
      deterministic, its gradient agrees with central differences of its own
      loss (to 5e-4 of |g|), and the fused forward equals the width-generic
      autograd path's on every particle.

Why float64 oracles: at L = 10 the edge latent enters the last block scaled
by 2^9 and the fp32 oracle's own rounding error grows with depth (measured
1.2e-3 of max|g| at L = 7 in round 1), so the fp32 product is compared
against the exact (float64) evaluation of the same reference ops, on the same
fp32 graph (positions and noise are fp32 sums, so the fp64 noisy window
rounds back to the identical fp32 search input).

Tolerances (stated per test): forward |got - ref| <= ATOL + RTOL |ref|
(ATOL = 2e-4, RTOL = 1e-4 on normalised outputs; x acc_std on positions);
gradients |g - g_ref| <= max(rel * max|g_ref|, 4 |g_fp32oracle - g_ref|) per tensor
(the fp32 oracle = the reference's own precision, as the yardstick).
"""
import numpy as np
import pytest
import torch

from tests.test_gpu_parity import ATOL, _close

pytestmark = pytest.mark.gpu


def _acc_std_max():
    from sgnn_amd import synthetic
    return float(max(synthetic.normalization_stats(3, noise_std=0.02)["acceleration"]["std"]))


ACC_STD = _acc_std_max()      # positions = prediction x acc_std: the forward bound scales with it


def _grad_close(got, ref, name, rel, ref32=None):
    """|got - ref| <= max(rel * max|ref|, 4 * |ref32 - ref|) + 1e-7, where ref32
    is the same oracle evaluated in fp32 (the reference's own precision): deep
    first-layer gradients (sums over every particle through L blocks) carry
    fp32 rounding of that size in the reference itself."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = np.abs(ref).max()
    err = np.abs(got - ref).max()
    yard = 0.0 if ref32 is None else float(np.abs(np.asarray(ref32, np.float64) - ref).max())
    bound = max(rel * scale, 4.0 * yard) + 1e-7
    assert err <= bound, f"{name}: max err {err:.3e} vs scale {scale:.3e} (fp32 oracle err {yard:.3e})"
    return err / max(scale, 1e-30)


def _f32_grads(make_oracle, run):
    """Gradients of the fp32 oracle (the yardstick of _grad_close)."""
    st32 = {k: v.detach().float().clone().requires_grad_(True) for k, v in make_oracle.items()}
    run(st32).backward()
    return {k: (v.grad.numpy() if v.grad is not None else None) for k, v in st32.items()}


def _stats(dim, dtype=torch.float32):
    from sgnn_amd import synthetic
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    return {k: {kk: torch.from_numpy(vv).to(dtype) for kk, vv in v.items()} for k, v in st.items()}


def _f64(state):
    return {k: v.detach().double().clone().requires_grad_(True) for k, v in state.items()}


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


# --------------------------------------------------------------------------- C2
def test_c2_training_step_50k_against_float64_oracle():
    """C2 (BASELINE configs[1]): 250 x 200 = 50,000 particles, r = 0.6, L = 5,
    H = 64, one Trainer step with injected noise.  Gradients rel 5e-4 of
    max|g| per tensor (as at C4/C5: the first encoder layer's bias gradient is
    a sum over 50k particles, measured 2.1e-4 off the float64 sum); Adam-updated weights vs torch.optim.Adam on the
    product's own gradient: |dp| <= 1e-7 + 1e-6 |p|."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.learned_simulator import LearnedSimulator
    from sgnn_amd.train import Trainer
    seq = synthetic.trajectory(synthetic.lattice_2d(250, 200), 12, seed=2000)
    n = seq.shape[0]
    stats = _stats(2)
    torch.manual_seed(0)
    sim = LearnedSimulator(2, 21, 3, 64, 5, 1, 64, 0.6, stats, 1, 9)
    state0 = {k: v.detach().clone() for k, v in sim.state_dict().items()}
    pos, nxt = torch.from_numpy(seq[:, :11]), torch.from_numpy(seq[:, 11])
    strain = torch.from_numpy(np.random.default_rng(1).normal(0, 1, n).astype(np.float32))
    noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(3))
    # float64 oracle autograd
    st64 = _f64(state0)
    osim = O.OracleSimulator(st64, 2, 5, 0.6, _stats(2, torch.float64))
    osim.p = st64
    pa, ta, ps = osim.predict_accelerations(nxt.double(), noise.double(), pos.double(), [n],
                                            torch.zeros(n, dtype=torch.long))
    ref_loss = O.training_loss(pa, ta, ps, strain.double())
    ref_loss.backward()

    def run32(p):
        o = O.OracleSimulator(p, 2, 5, 0.6, _stats(2))
        o.p = p
        a, b, c = o.predict_accelerations(nxt, noise, pos, [n], torch.zeros(n, dtype=torch.long))
        return O.training_loss(a, b, c, strain)
    g32 = _f32_grads(state0, run32)
    # product
    sim = sim.cuda()
    tr = Trainer(sim, lr_init=1e-3)
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), [n], noise=noise.cuda())
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - ref_loss.item()) <= 2e-5 * abs(ref_loss.item())
    worst = 0.0
    grads = {k: p.grad.detach().cpu().clone() for k, p in sim.named_parameters()}
    for k in grads:
        if st64[k].grad is not None:
            worst = max(worst, _grad_close(grads[k].numpy(), st64[k].grad.numpy(), k, rel=5e-4, ref32=g32[k]))
    print(f"C2 50k: E={tr.workspace(n, 11, 'cuda').f.num_edges()} worst relative grad error {worst:.3e}")
    # fused Adam == torch.optim.Adam on the same gradient (train.py:199, :271-273)
    ref_p = {k: state0[k].clone().requires_grad_(True) for k in grads}
    opt = torch.optim.Adam([ref_p[k] for k in grads], lr=1e-3)
    for k in grads:
        ref_p[k].grad = grads[k]
    opt.step()
    sd = sim.state_dict()
    for k in grads:
        np.testing.assert_allclose(sd[k].cpu().numpy(), ref_p[k].detach().numpy(), rtol=1e-6, atol=1e-7,
                                   err_msg=k)
    _free()


# --------------------------------------------------------------------------- C4
def _c4_sim(L=10, H=128, seed=4):
    from sgnn_amd.learned_simulator import LearnedSimulator
    torch.manual_seed(seed)
    return LearnedSimulator(3, 31, 4, H, L, 1, H, 0.75, _stats(3), 1, 9)


def test_c4_shapes_l10_h128_forward_and_gradients_against_float64_oracle():
    """C4 widths (3D, r = 0.75, L = 10, H = 128) on a 24 x 20 x 20 lattice:
    predict_positions (strain, next positions) and one training step's
    gradients vs the float64 oracle.  Gradients rel 5e-4 of max|g|."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.train import Trainer
    seq = synthetic.trajectory(synthetic.lattice_3d(24, 20, 20), 12, seed=31)
    n = seq.shape[0]
    sim = _c4_sim()
    state0 = {k: v.detach().clone() for k, v in sim.state_dict().items()}
    pos, nxt = torch.from_numpy(seq[:, :11]), torch.from_numpy(seq[:, 11])
    types_ = torch.zeros(n, dtype=torch.long)
    st64 = _f64(state0)
    osim = O.OracleSimulator(st64, 3, 10, 0.75, _stats(3, torch.float64))
    osim.p = st64
    with torch.no_grad():
        ref_next, ref_strain = osim.predict_positions(pos.double(), [n], types_)
    sim = sim.cuda()
    with torch.no_grad():
        got_next, got_strain = sim.predict_positions(pos.cuda(), [n], types_.cuda())
    _close(got_strain.cpu().numpy(), ref_strain.numpy(), what="C4 L10 strain")
    _close(got_next.cpu().numpy(), ref_next.numpy(), atol=ATOL * ACC_STD, rtol=1e-6, what="C4 L10 next_pos")
    # training step
    strain = torch.from_numpy(np.random.default_rng(2).normal(0, 1, n).astype(np.float32))
    noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(5))
    pa, ta, ps = osim.predict_accelerations(nxt.double(), noise.double(), pos.double(), [n], types_)
    ref_loss = O.training_loss(pa, ta, ps, strain.double())
    ref_loss.backward()

    def run32(p):
        o = O.OracleSimulator(p, 3, 10, 0.75, _stats(3))
        o.p = p
        a, b, c = o.predict_accelerations(nxt, noise, pos, [n], types_)
        return O.training_loss(a, b, c, strain)
    g32 = _f32_grads(state0, run32)
    tr = Trainer(sim, lr_init=1e-3)
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), [n], noise=noise.cuda())
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - ref_loss.item()) <= 2e-5 * abs(ref_loss.item())
    worst = 0.0
    for k, p in sim.named_parameters():
        if st64[k].grad is not None:
            worst = max(worst, _grad_close(p.grad.cpu().numpy(), st64[k].grad.numpy(), k, rel=5e-4, ref32=g32[k]))
    print(f"C4 L=10 H=128 9.6k: worst relative grad error {worst:.3e}")
    _free()


def test_c4_full_200k_graph_bit_exact_and_interior_block_matches_oracle():
    """C4 at its full size (100 x 50 x 40 = 200,000 particles): the radius
    graph equals the oracle's cell-list search bit for bit; the prediction of
    every particle of the 13^3 interior corner block equals the oracle run on
    the 24^3 corner block alone (those particles are >= 11 hops from the cut,
    L = 10); the full output is finite."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    dims = (100, 50, 40)
    seq = synthetic.trajectory(synthetic.lattice_3d(*dims), 11, seed=1000)
    n = seq.shape[0]
    sim = _c4_sim().cuda()
    pos = torch.from_numpy(seq)
    ei_ref = O.radius_graph(pos[:, -1], [n], 0.75)
    r, s = sim._compute_graph_connectivity(pos[:, -1].cuda(), [n], 0.75)
    assert r.shape[0] == ei_ref.shape[1] > 17 * n
    np.testing.assert_array_equal(torch.stack([r, s]).cpu().numpy(), ei_ref.numpy())
    del r, s
    types_ = torch.zeros(n, dtype=torch.long)
    with torch.no_grad():
        got_next, got_strain = sim.predict_positions(pos.cuda(), [n], types_.cuda())
    got_next, got_strain = got_next.cpu(), got_strain.cpu()
    assert torch.isfinite(got_next).all() and torch.isfinite(got_strain).all()
    # lattice index (i, j, k) -> particle i*ny*nz + j*nz + k (synthetic.lattice_3d, z fastest)
    B, I = 24, 13
    ii, jj, kk = np.meshgrid(np.arange(B), np.arange(B), np.arange(B), indexing="ij")
    block = (ii * dims[1] * dims[2] + jj * dims[2] + kk).ravel()
    inner = ((ii < I) & (jj < I) & (kk < I)).ravel()
    st = {k: v.detach().cpu() for k, v in sim.state_dict().items()}
    osim = O.OracleSimulator(st, 3, 10, 0.75, _stats(3))
    with torch.no_grad():
        ref_next, ref_strain = osim.predict_positions(pos[block], [block.size], types_[:block.size])
    sel = block[inner]
    _close(got_strain[sel].numpy(), ref_strain[inner].numpy(), what="C4 200k interior strain")
    _close(got_next[sel].numpy(), ref_next[inner].numpy(), atol=ATOL * ACC_STD, rtol=1e-6,
           what="C4 200k interior next_pos")
    _free()


# --------------------------------------------------------------------------- C5
def _ms_sim(dim=3, H=128, L=10, nmlp=2, seed=21):
    from sgnn_amd.multi_scale import MultiScaleSimulator
    torch.manual_seed(seed)
    return MultiScaleSimulator(dim, 10 * dim + 1, dim + 1, H, H, L, nmlp, _stats(dim), 1, 9, 2, 2, 2.0)


def test_c5_shapes_l10_h128_forward_and_gradients_against_float64_oracle():
    """C5 widths (multi-scale, 2 scales, window 2, radius multiplier 2, L = 10
    M2M blocks, H = 128, nmlp_layers = 2) on a 24 x 20 x 20 lattice at the
    wall: prediction and one training step's gradients vs the float64
    multi-scale oracle on the same static graph.  Gradients rel 5e-4."""
    from oracle import multi_scale_oracle as MO
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import build_static_multi_scale_graph
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    seq = synthetic.trajectory(synthetic.lattice_3d(24, 20, 20, x0=-1.75), 12, seed=13)
    n = seq.shape[0]
    sim = _ms_sim()
    state0 = {k: v.detach().clone() for k, v in sim.state_dict().items()}
    g_ref = MO.create_all_edges(torch.from_numpy(seq[:, 0]), 2, 2, 2.0)
    st64 = _f64(state0)
    osim = MO.MultiScaleOracle(st64, 3, 10, _stats(3, torch.float64), g_ref, 2, 2.0, 1, 2)
    pos, nxt = torch.from_numpy(seq[:, :11]), torch.from_numpy(seq[:, 11])
    with torch.no_grad():
        ref_next, ref_strain = osim.predict_positions(pos.double())
    sim = sim.cuda()
    g = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), 2, 2, 2.0)
    for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
        np.testing.assert_array_equal(g[key].cpu().numpy(), g_ref[key].numpy(), err_msg=key)
    sim.set_static_graph(g)
    with torch.no_grad():
        got_next, got_strain = sim.predict_positions(pos.cuda(), [n], None)
    _close(got_strain.cpu().numpy(), ref_strain.numpy(), what="C5 L10 strain")
    _close(got_next.cpu().numpy(), ref_next.numpy(), atol=ATOL * ACC_STD, rtol=1e-6, what="C5 L10 next_pos")
    strain = torch.from_numpy(np.random.default_rng(4).normal(0, 1, n).astype(np.float32))
    noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(5))
    pa, ta, ps = osim.predict_accelerations(nxt.double(), noise.double(), pos.double())
    ref_loss = O.training_loss(pa, ta, ps, strain.double())
    ref_loss.backward()

    def run32(p):
        o = MO.MultiScaleOracle(p, 3, 10, _stats(3), g_ref, 2, 2.0, 1, 2)
        a, b, c = o.predict_accelerations(nxt, noise, pos)
        return O.training_loss(a, b, c, strain)
    g32 = _f32_grads(state0, run32)
    tr = MultiScaleTrainer(sim, lr_init=1e-3)
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), noise=noise.cuda())
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - ref_loss.item()) <= 2e-5 * abs(ref_loss.item())
    worst = 0.0
    for k, p in sim.named_parameters():
        if st64[k].grad is not None:
            worst = max(worst, _grad_close(p.grad.cpu().numpy(), st64[k].grad.numpy(), k, rel=5e-4, ref32=g32[k]))
    print(f"C5 L=10 H=128 nmlp=2 9.6k: worst relative grad error {worst:.3e}")
    _free()


def test_c5_full_1m_hierarchy_bit_exact_and_training_deterministic():
    """C5 at its full per-GPU size (100^3 = 1,000,000 particles): the GPU
    hierarchy and g2m/m2m/m2g edge lists equal the oracle's bit for bit; two
    training steps on the same inputs (lr = 0) give bitwise-identical finite
    gradients and losses; the gradient against central differences of the
    step's own loss along it; the fused forward against the width-generic
    path (independent kernels) on the same window."""
    from oracle import multi_scale_oracle as MO
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import build_static_multi_scale_graph
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    base = synthetic.lattice_3d(100, 100, 100)
    base[:, 0] -= 2.0
    seq = synthetic.trajectory(base, 12, seed=3000)
    n = seq.shape[0]
    g_ref = MO.create_all_edges(torch.from_numpy(seq[:, 0]), 2, 2, 2.0)
    g = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), 2, 2, 2.0)
    for s in range(2):
        np.testing.assert_array_equal(g["graph_hierarchy"][s]["sampling_indices"].cpu().numpy(),
                                      g_ref["graph_hierarchy"][s]["sampling_indices"].numpy())
    for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
        np.testing.assert_array_equal(g[key].cpu().numpy(), g_ref[key].numpy(), err_msg=key)
    assert g["grid2mesh_edges"].shape[1] > 5 * n // 1      # ~5.9 edges per particle
    del g_ref
    sim = _ms_sim().cuda()
    sim.set_static_graph(g)
    pos = torch.from_numpy(seq[:, :11]).cuda()
    nxt = torch.from_numpy(seq[:, 11]).cuda()
    strain = torch.zeros(n, device="cuda")
    noise = torch.zeros_like(pos)
    tr = MultiScaleTrainer(sim, lr_init=0.0)
    w_init = tr.flat.param.clone()   # the schedule's + 1e-6 (train.py:276-278) moves the weights after step 2
    res = []
    for _ in range(2):
        out = tr.train_step(pos, nxt, strain, noise=noise)
        torch.cuda.synchronize()
        res.append((float(out["loss"]), tr.flat.grad.clone()))
    assert np.isfinite(res[0][0]) and torch.isfinite(res[0][1]).all()
    assert res[0][0] == res[1][0] and torch.equal(res[0][1], res[1][1])
    # Full-size checks of the fused chain against independent arithmetic (no CPU oracle finishes at 1M):
    # (1) the gradient along its own direction u = g / |g| against central differences of the step's loss at
    #     the SAME weights (restored first: the LR schedule's + 1e-6 floor, train.py:276-278, moved them after
    #     the second step), L(w + eps u) - L(w - eps u) over 2 eps.  Each step's loss is formed before its Adam
    #     update, and the weights are reset before every evaluation.  Measured at 1M (tools/exp_fd_c5_1m.py):
    #     -4.8e-4 of |g| at eps 5e-3, -1.2e-4 at 2.5e-3, converging as eps^2 (-4.8e-6 at 3.1e-4); per tensor
    #     the same (the largest, the late M2M edge-MLP first Linears under the 2^k latent, -8e-3 -> 2e-3).
    loss0, grad = res[0]
    gnorm = float(grad.norm())
    assert gnorm > 0.0
    u = grad / gnorm
    flat = tr.flat.param
    fd = []
    for eps in (5e-3, 2.5e-3):
        flat.copy_(w_init).add_(u, alpha=eps)
        lp = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
        flat.copy_(w_init).add_(u, alpha=-eps)
        lm = float(tr.train_step(pos, nxt, strain, noise=noise)["loss"])
        fd.append((lp - lm) / (2 * eps))
    flat.copy_(w_init)
    print(f"C5 1M: |g| = {gnorm:.6e}, central differences " + " / ".join(f"{v:.6e}" for v in fd))
    assert abs(fd[0] - gnorm) <= 2e-3 * gnorm and abs(fd[1] - gnorm) <= 5e-4 * gnorm, (gnorm, fd)
    # (2) the fused forward (k_encode_*, k_edge_layer, k_node_layer at H = 128, nmlp 2) against the
    #     width-generic path (autograd.hip: MFMA GEMMs, gathers, LayerNorm and CSR sums of their own) on the
    #     same 1M-particle window: every predicted acceleration and strain.
    with torch.no_grad():
        _, pred_fused, _ = sim._run(pos, None)
        inp, use_emb = sim._step_inputs(pos, None)
        pred_gen = sim._generic_pred(inp, use_emb)
    torch.cuda.synchronize()
    scale = float(pred_gen.abs().max())
    err = float((pred_fused - pred_gen).abs().max())
    print(f"C5 1M forward: fused vs generic max|d| = {err:.3e} (max|pred| {scale:.3e})")
    assert torch.isfinite(pred_fused).all() and err <= 1e-3 * scale + 1e-5, (err, scale)
    del tr, sim, res, grad, u
    _free()
