"""Autograd through the reference's module forwards and training at every
shape: Encoder / InteractionNetwork / Processor /
Decoder / EncodeProcessDecode.forward and MultiScaleGNN.forward are
differentiable (graph_network.py:98, :150, :276, :324, :388;
multi_scale_gnn.py:84, :132, :179, :262) at any latent / hidden / edge widths
and any nmlp_layers, with forward and backward in libsgnn_hip.so
(sgnn_amd/autograd.py over autograd.hip).  Checked against oracle autograd
(test infrastructure) per parameter and per input; and the module forwards at
the fast widths run the fused edge / node kernels in inference.

Tolerances (fp32, different summation order than CPU autograd):
  outputs |got - ref| <= 2e-4 + 1e-4 |ref|; gradients |g - g_ref| <= 5e-4 max|g_ref|
  per tensor; loss rel 2e-5; Adam-updated parameters as test_gpu_training.py."""
import numpy as np
import pytest
import torch

from tests.test_gpu_parity import _close
from tests.test_gpu_training import _grad_close

pytestmark = pytest.mark.gpu


def _setup(latent, hidden, nmlp, dim, L=3, ntypes=1, emb=9, seed=3, dims=None):
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.learned_simulator import LearnedSimulator
    lat = synthetic.lattice_2d(*(dims or (24, 16))) if dim == 2 else synthetic.lattice_3d(*(dims or (8, 6, 5)))
    seq = synthetic.trajectory(lat, 12, seed=5)
    n = seq.shape[0]
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(seed)
    nin = 10 * dim + 1 + (emb if ntypes > 1 else 0)
    sim = LearnedSimulator(dim, nin, dim + 1, latent, L, nmlp, hidden, 1.1, stats, ntypes, emb)
    state = {k: v.detach().clone().requires_grad_(True) for k, v in sim.state_dict().items()}
    osim = O.OracleSimulator(state, dim, L, 1.1, stats, ntypes, nmlp_layers=nmlp)
    types_ = torch.from_numpy(np.random.default_rng(2).integers(0, ntypes, n))
    return sim.cuda(), osim, state, seq, types_, st


def _check_grads(sim_named, state, rel=5e-4, prefix=""):
    worst, checked = 0.0, 0
    for k, p in sim_named:
        ref = state[prefix + k].grad
        if ref is None:
            continue
        assert p.grad is not None, f"{k}: no gradient"
        worst = max(worst, _grad_close(p.grad.cpu().numpy(), ref.numpy(), k, rel=rel))
        checked += 1
    assert checked > 0
    return worst


@pytest.mark.parametrize("latent,hidden,nmlp,dim", [
    (64, 64, 1, 2),     # the fused widths, under autograd (the differentiable path)
    (48, 80, 3, 2),     # latent != mlp_hidden_dim, nmlp_layers 3 (4 Linears per MLP)
    (128, 128, 2, 3),   # H = 128, 3D
])
def test_epd_forward_backward_matches_oracle(latent, hidden, nmlp, dim, monkeypatch):
    """gnn(x, ei, e).backward() == oracle autograd (float64) per parameter and per input.
    At the fused widths (64/64/1, 128/128/2) every InteractionNetwork of the
    Processor runs its forward and backward on the training step's fused layer
    kernels (sgnn_amd/fused_block.py; counted), elsewhere the GEMM chain."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import fused_block
    calls = []
    real = fused_block.block_backward
    monkeypatch.setattr(fused_block, "block_backward", lambda *a: calls.append(1) or real(*a))
    sim, osim, state, seq, types_, _ = _setup(latent, hidden, nmlp, dim)
    pos = torch.from_numpy(seq[:, :11])
    n = pos.shape[0]
    nf, ei, ef = osim.preprocess(pos, [n], types_)
    # the reference gradient in float64 (the fp32 oracle's own error through a 3-Linear stack is
    # of the order of the tolerance); the HIP path computes in fp32
    state = {k: v.detach().double().requires_grad_(True) for k, v in state.items()}
    nf, ef = nf.detach().double().requires_grad_(True), ef.detach().double().requires_grad_(True)
    w = torch.from_numpy(np.random.default_rng(7).normal(0, 1, (n, dim + 1)).astype(np.float32))
    ref = O.encode_process_decode(state, nf, ei, ef, 3, nmlp)
    (ref * w.double()).sum().backward()
    nf_g, ef_g = nf.detach().float().cuda().requires_grad_(True), ef.detach().float().cuda().requires_grad_(True)
    epd = sim._encode_process_decode
    got = epd(nf_g, ei.cuda(), ef_g)
    assert got.grad_fn is not None
    _close(got.detach().cpu().numpy(), ref.detach().numpy(), what=f"EPD L{latent} H{hidden} nmlp{nmlp}")
    (got * w.cuda()).sum().backward()
    assert len(calls) == (3 if latent == hidden and latent in (64, 128) else 0), calls
    worst = _check_grads(epd.named_parameters(prefix="_encode_process_decode"), state)
    _grad_close(nf_g.grad.cpu().numpy(), nf.grad.numpy(), "d node_features", rel=5e-4)
    _grad_close(ef_g.grad.cpu().numpy(), ef.grad.numpy(), "d edge_features", rel=5e-4)
    print(f"L{latent} H{hidden} nmlp{nmlp}: worst relative grad error {worst:.3e}")


def test_module_forwards_backward_match_oracle(monkeypatch):
    """Encoder / InteractionNetwork / Processor / Decoder each on their own under
    autograd, with the input latents' gradients (x, e) and a shuffled edge order
    (the fused block's COO -> CSR permutation both ways)."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import fused_block
    calls = []
    real = fused_block.block_backward
    monkeypatch.setattr(fused_block, "block_backward", lambda *a: calls.append(1) or real(*a))
    fused_block_calls = lambda: len(calls)
    sim, osim, state, seq, types_, _ = _setup(64, 64, 1, 2)
    pos = torch.from_numpy(seq[:, :11])
    n = pos.shape[0]
    nf, ei, ef = osim.preprocess(pos, [n], types_)
    perm = torch.randperm(ei.shape[1], generator=torch.Generator().manual_seed(1))
    ei, ef = ei[:, perm], ef[perm]
    epd = sim._encode_process_decode
    pre = "_encode_process_decode."
    x0 = O.mlp_ln(nf, state, pre + "_encoder.node_fn.", 2).detach()
    e0 = O.mlp_ln(ef, state, pre + "_encoder.edge_fn.", 2).detach()
    rng = np.random.default_rng(3)
    wx = torch.from_numpy(rng.normal(0, 1, x0.shape).astype(np.float32))
    we = torch.from_numpy(rng.normal(0, 1, e0.shape).astype(np.float32))
    # InteractionNetwork 1
    xr, er = x0.clone().requires_grad_(True), e0.clone().requires_grad_(True)
    rx, re = O.interaction_network(xr, ei, er, state, pre + "_processor.gnn_stacks.1.", 2)
    ((rx * wx).sum() + (re * we).sum()).backward()
    xg, eg = x0.cuda().requires_grad_(True), e0.cuda().requires_grad_(True)
    gx, ge = epd._processor.gnn_stacks[1](xg, ei.cuda(), eg)
    _close(gx.detach().cpu().numpy(), rx.detach().numpy(), what="InteractionNetwork")
    ((gx * wx.cuda()).sum() + (ge * we.cuda()).sum()).backward()
    _check_grads(epd._processor.gnn_stacks[1].named_parameters(prefix=pre + "_processor.gnn_stacks.1"), state)
    _grad_close(xg.grad.cpu().numpy(), xr.grad.numpy(), "InteractionNetwork dx", rel=5e-4)
    _grad_close(eg.grad.cpu().numpy(), er.grad.numpy(), "InteractionNetwork de", rel=5e-4)
    assert fused_block_calls(), "the InteractionNetwork backward did not run the fused kernels"
    # Processor, Encoder, Decoder
    for v in state.values():
        v.grad = None
    sim.zero_grad(set_to_none=True)
    xr = x0.clone().requires_grad_(True)
    x, e = xr, e0
    for k in range(3):
        x, e = O.interaction_network(x, ei, e, state, f"{pre}_processor.gnn_stacks.{k}.", 2)
    (x * wx).sum().backward()
    xg = x0.cuda().requires_grad_(True)
    px, pe = epd._processor(xg, ei.cuda(), e0.cuda())
    (px * wx.cuda()).sum().backward()
    _close(px.detach().cpu().numpy(), x.detach().numpy(), what="Processor")
    _check_grads(epd._processor.named_parameters(prefix=pre + "_processor"), state)
    _grad_close(xg.grad.cpu().numpy(), xr.grad.numpy(), "Processor dx", rel=5e-4)
    # random output weights: the plain sum of a LayerNorm's outputs has a zero gradient
    ex, ee = epd._encoder(nf.cuda(), ef.cuda())
    ((ex * wx.cuda()).sum() + (ee * we.cuda()).sum()).backward()
    ((O.mlp_ln(nf, state, pre + "_encoder.node_fn.", 2) * wx).sum()
     + (O.mlp_ln(ef, state, pre + "_encoder.edge_fn.", 2) * we).sum()).backward()
    _check_grads(epd._encoder.named_parameters(prefix=pre + "_encoder"), state)
    d = epd._decoder(x0.cuda())
    (d * 3.0).sum().backward()
    (O.mlp(x0, state, pre + "_decoder.node_fn.", 2) * 3.0).sum().backward()
    _check_grads(epd._decoder.named_parameters(prefix=pre + "_decoder"), state)


def test_row_strided_views_through_layernorm():
    """torch.cat's backward hands each input a narrow() view (row
    stride > width), and a column slice used as an input is row-strided too.
    The LayerNorm kernels index rows as r * width, so those views must reach
    them dense: Encoder outputs concatenated with another tensor, and an
    InteractionNetwork whose x (its residual) is a column slice."""
    from oracle import sgnn_oracle as O
    sim, osim, state, seq, types_, _ = _setup(64, 64, 1, 2)
    pos = torch.from_numpy(seq[:, :11])
    n = pos.shape[0]
    nf, ei, ef = osim.preprocess(pos, [n], types_)
    epd = sim._encode_process_decode
    pre = "_encode_process_decode."
    rng = np.random.default_rng(5)
    # Encoder outputs inside a cat: the node / edge latents' gradients arrive as narrow() views
    ex, ee = epd._encoder(nf.cuda(), ef.cuda())
    ox = torch.from_numpy(rng.normal(0, 1, (n, 7)).astype(np.float32)).cuda()
    oe = torch.from_numpy(rng.normal(0, 1, (ef.shape[0], 5)).astype(np.float32)).cuda()
    wx = torch.from_numpy(rng.normal(0, 1, (n, 64 + 7)).astype(np.float32))
    we = torch.from_numpy(rng.normal(0, 1, (ef.shape[0], 64 + 5)).astype(np.float32))
    ((torch.cat([ex, ox], 1) * wx.cuda()).sum() + (torch.cat([ee, oe], 1) * we.cuda()).sum()).backward()
    ((O.mlp_ln(nf, state, pre + "_encoder.node_fn.", 2) * wx[:, :64]).sum()
     + (O.mlp_ln(ef, state, pre + "_encoder.edge_fn.", 2) * we[:, :64]).sum()).backward()
    _check_grads(epd._encoder.named_parameters(prefix=pre + "_encoder"), state)
    # InteractionNetwork on a column slice of a wider tensor (row-strided x and residual)
    for v in state.values():
        v.grad = None
    sim.zero_grad(set_to_none=True)
    x0 = O.mlp_ln(nf, state, pre + "_encoder.node_fn.", 2).detach()
    e0 = O.mlp_ln(ef, state, pre + "_encoder.edge_fn.", 2).detach()
    xr = x0.clone().requires_grad_(True)
    rx, _ = O.interaction_network(xr, ei, e0, state, pre + "_processor.gnn_stacks.0.", 2)
    w2 = torch.from_numpy(rng.normal(0, 1, x0.shape).astype(np.float32))
    (rx * w2).sum().backward()
    wide = torch.cat([x0, torch.zeros(n, 3)], 1).cuda().requires_grad_(True)
    gx, _ = epd._processor.gnn_stacks[0](wide[:, :64], ei.cuda(), e0.cuda())
    _close(gx.detach().cpu().numpy(), rx.detach().numpy(), what="InteractionNetwork on a column slice")
    (gx * w2.cuda()).sum().backward()
    _check_grads(epd._processor.gnn_stacks[0].named_parameters(prefix=pre + "_processor.gnn_stacks.0"), state)
    _grad_close(wide.grad[:, :64].cpu().numpy(), xr.grad.numpy(), "column-slice dx", rel=5e-4)
    assert float(wide.grad[:, 64:].abs().max()) == 0.0


@pytest.mark.parametrize("H", [64, 128])
def test_interaction_network_inference_runs_fused_kernels(H, monkeypatch):
    """InteractionNetwork.forward in inference at the fast widths goes through
    engine.interaction_forward (k_edge_layer + k_node_layer), matching the oracle
    and the differentiable path."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import autograd, engine
    sim, osim, state, seq, types_, _ = _setup(H, H, 1, 2)
    pos = torch.from_numpy(seq[:, :11])
    n = pos.shape[0]
    nf, ei, ef = osim.preprocess(pos, [n], types_)
    pre = "_encode_process_decode."
    x0 = O.mlp_ln(nf, state, pre + "_encoder.node_fn.", 2).detach()
    e0 = O.mlp_ln(ef, state, pre + "_encoder.edge_fn.", 2).detach()
    ref_x, ref_e = O.interaction_network(x0, ei, e0, state, pre + "_processor.gnn_stacks.0.", 2)
    calls = []
    real = engine.interaction_forward
    monkeypatch.setattr(engine, "interaction_forward", lambda *a, **k: calls.append(1) or real(*a, **k))
    blk = sim._encode_process_decode._processor.gnn_stacks[0]
    with torch.no_grad():
        gx, ge = blk(x0.cuda(), ei.cuda(), e0.cuda())
        ax, ae = autograd.message_passing(blk, x0.cuda(), autograd.EdgeGraph(ei.cuda(), n), e0.cuda())
    assert calls, "the fused path was not taken"
    _close(gx.cpu().numpy(), ref_x.detach().numpy(), what=f"fused InteractionNetwork H{H}")
    _close(gx.cpu().numpy(), ax.cpu().numpy(), atol=1e-5, rtol=1e-5, what="fused vs differentiable path")
    np.testing.assert_array_equal(ge.cpu().numpy(), ref_e.detach().numpy())


@pytest.mark.parametrize("latent,hidden,nmlp,dim,ntypes", [
    (48, 80, 3, 2, 1),    # latent != hidden, nmlp_layers 3
    (96, 96, 1, 2, 3),    # hidden 96 with particle-type embeddings (their gradient: per-type sums)
])
def test_generic_trainer_step_matches_oracle(latent, hidden, nmlp, dim, ntypes):
    """Trainer at shapes the fused kernels are not built for: loss, every
    gradient (embedding included) and the Adam update vs oracle autograd +
    torch.optim.Adam."""
    from oracle import sgnn_oracle as O
    from sgnn_amd.train import Trainer
    sim, osim, state, seq, types_, _ = _setup(latent, hidden, nmlp, dim, ntypes=ntypes)
    pos, nxt = torch.from_numpy(seq[:, :11]), torch.from_numpy(seq[:, 11])
    n = pos.shape[0]
    strain = torch.from_numpy(np.random.default_rng(1).normal(0, 1, n).astype(np.float32))
    noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(7))
    pa, ta, ps = osim.predict_accelerations(nxt, noise, pos, [n], types_)
    ref_loss = O.training_loss(pa, ta, ps, strain)
    ref_loss.backward()
    params = [state[k] for k, _ in sim.named_parameters()]
    opt = torch.optim.Adam([p for p in params if p.grad is not None], lr=1e-3)
    opt.step()
    tr = Trainer(sim, lr_init=1e-3)
    assert not tr.fused
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), [n], types_.cuda(), noise=noise.cuda())
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - ref_loss.item()) <= 2e-5 * abs(ref_loss.item())
    worst = _check_grads(sim.named_parameters(), state)
    print(f"generic L{latent} H{hidden} nmlp{nmlp} types{ntypes}: worst relative grad error {worst:.3e}")
    # Adam's first step moves a weight by ~lr g / (|g| + eps): where |g| is near zero a relative gradient
    # error of the order of the tolerance moves it by up to 2 lr, so the bound scales with it per element
    sd = sim.state_dict()
    for k, p in sim.named_parameters():
        ref = state[k]
        if ref.grad is None:
            continue
        g = ref.grad.abs().numpy()
        bound = 2e-5 + 2e-3 * np.minimum(1.0, 1e-5 * g.max() / np.maximum(g, 1e-30))
        dw = np.abs(sd[k].cpu().numpy() - ref.detach().numpy())
        assert (dw <= bound).all(), f"{k}: max |dw| {dw.max():.3e}, worst |dw|/bound {(dw / bound).max():.3f}"


def test_multi_scale_generic_training_and_block_autograd():
    """MultiScaleGNN with nedge_out != latent_dim (multi_scale_gnn.py:225-272):
    MultiScaleTrainer step (loss, every gradient) vs oracle autograd; the fused
    widths' MultiScaleGNN.forward under autograd vs the reference golden output."""
    from oracle import multi_scale_oracle as MO
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import MultiScaleSimulator, build_static_multi_scale_graph
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    dim, T, L = 2, 6, 2
    seq = synthetic.trajectory(synthetic.lattice_2d(30, 12, x0=-1.75), T + 1, seed=13)
    n = seq.shape[0]
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(21)
    sim = MultiScaleSimulator(dim, (T - 1) * dim + 1, dim + 1, 48, 64, L, 2, stats, 1, 9, 2, 2, 2.0)
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
    assert not tr.fused
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), noise=noise.cuda())
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - ref_loss.item()) <= 2e-5 * abs(ref_loss.item())
    worst = _check_grads(sim.named_parameters(), state)
    print(f"multi-scale nedge_out 48: worst relative grad error {worst:.3e}")
