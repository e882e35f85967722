"""The reference's per-module forwards and width-generic models on the HIP
kernels (fused edge / node kernels in inference, the differentiable path of
sgnn_amd/autograd.py otherwise), against the reference's own per-layer latents
(tiny2d_r06: Encoder / InteractionNetwork x 5 / Decoder outputs recorded by
running the reference modules) and against the oracle for widths the fused
kernels are not built for.  Tolerance as test_gpu_parity.py (fp32:
|got - ref| <= 2e-4 + 1e-4 |ref|); the edge latents double exactly."""
import numpy as np
import pytest
import torch

from tests.helpers import golden, hparams, ms_graph_of, product_sim, state_of, stats_of
from tests.test_gpu_parity import ATOL, _close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("grad", [False, True])
def test_module_forwards_match_reference_latents(grad):
    """grad False: inference (InteractionNetwork / Processor on the fused edge / node kernels at
    these widths); grad True: the differentiable path (outputs carry a grad_fn)."""
    z = golden("tiny2d_r06")
    sim = product_sim(z)
    epd = sim._encode_process_decode
    t = lambda k: torch.from_numpy(z[k]).cuda()
    ei = t("edge_index")
    with torch.set_grad_enabled(grad):
        x, e = epd._encoder(t("node_features"), t("edge_features"))            # graph_network.py:98-111
        assert (x.grad_fn is not None) == grad
        _close(x.detach().cpu().numpy(), z["lat_x_enc"], what="Encoder.node_fn")
        _close(e.detach().cpu().numpy(), z["lat_e_enc"], what="Encoder.edge_fn")
        xk, ek = t("lat_x_enc"), t("lat_e_enc")
        for k, gnn in enumerate(epd._processor.gnn_stacks):                   # graph_network.py:150-176
            x1, e1 = gnn(xk, ei, ek)
            _close(x1.detach().cpu().numpy(), z[f"lat_x_{k}"], what=f"InteractionNetwork {k}")
            assert torch.equal(e1.detach(), ek + ek)
            xk, ek = t(f"lat_x_{k}"), e1.detach()
        xp, ep = epd._processor(t("lat_x_enc"), ei, t("lat_e_enc"))            # graph_network.py:276-293
        _close(xp.detach().cpu().numpy(), z["lat_x_4"], what="Processor")
        _close(ep.detach().cpu().numpy(), z["lat_e_final"], what="Processor edge latent")
        out = epd._decoder(t("lat_x_4"))                                       # graph_network.py:324-333
        _close(out.detach().cpu().numpy(), z["pred"], what="Decoder")


def test_interaction_network_edge_cases():
    """No edges (aggregates zero, node_fn still applies) and a shuffled COO order."""
    from oracle import sgnn_oracle as O
    z = golden("tiny2d_r06")
    sim = product_sim(z)
    gnn = sim._encode_process_decode._processor.gnn_stacks[2]
    p = {k: v for k, v in state_of(z).items()}
    pre = "_encode_process_decode._processor.gnn_stacks.2."
    x, e, ei = (torch.from_numpy(z[k]) for k in ("lat_x_1", "lat_e_enc", "edge_index"))
    perm = torch.randperm(ei.shape[1], generator=torch.Generator().manual_seed(1))
    for case, (ei_c, e_c) in {"edgeless": (ei[:, :0], e[:0]), "shuffled": (ei[:, perm], e[perm])}.items():
        ref_x, ref_e = O.interaction_network(x, ei_c, e_c, p, pre, 2)
        for grad in (False, True):   # the fused kernels (inference) and the differentiable path
            with torch.set_grad_enabled(grad):
                got_x, got_e = gnn(x.cuda(), ei_c.cuda(), e_c.cuda())
            _close(got_x.detach().cpu().numpy(), ref_x.numpy(), what=f"InteractionNetwork {case} grad={grad}")
            np.testing.assert_array_equal(got_e.detach().cpu().numpy(), ref_e.numpy())


@pytest.mark.parametrize("latent,hidden,nmlp,dim", [(96, 96, 1, 2), (32, 80, 2, 2), (256, 128, 1, 3)])
def test_generic_widths_predict_positions(latent, hidden, nmlp, dim):
    """Widths the fused kernels are not built for (hidden 96 / 256, latent !=
    mlp_hidden_dim): LearnedSimulator.predict_positions, EncodeProcessDecode.forward
    and the device rollout's fallback vs the oracle."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import evaluate, synthetic
    from sgnn_amd.learned_simulator import LearnedSimulator
    lat = synthetic.lattice_2d(30, 20) if dim == 2 else synthetic.lattice_3d(10, 8, 6)
    seq = synthetic.trajectory(lat, 14, seed=5)
    n = seq.shape[0]
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(3)
    sim = LearnedSimulator(dim, 10 * dim + 1, dim + 1, latent, 3, nmlp, hidden, 1.1, stats, 1, 9)
    state = {k: v.detach().clone() for k, v in sim.state_dict().items()}
    osim = O.OracleSimulator(state, dim, 3, 1.1, stats, 1, nmlp_layers=nmlp)
    pos = torch.from_numpy(seq[:, :11])
    types_ = torch.zeros(n, dtype=torch.long)
    ref_next, ref_strain = osim.predict_positions(pos, [n], types_)
    sim = sim.cuda()
    assert not sim._fast_path()
    with torch.no_grad():
        nxt, strain = sim.predict_positions(pos.cuda(), [n], types_.cuda())
    _close(strain.cpu().numpy(), ref_strain.numpy(), what=f"L{latent} H{hidden} strain")
    scale = float(np.max(st["acceleration"]["std"]))
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * scale, rtol=1e-6, what=f"L{latent} H{hidden} next")
    nf, ei, ef = osim.preprocess(pos, [n], types_)
    got = sim._encode_process_decode(nf.cuda(), ei.cuda(), ef.cuda())
    _close(got.detach().cpu().numpy(), osim.epd(nf, ei, ef).numpy(), what=f"L{latent} H{hidden} EPD.forward")
    full = torch.from_numpy(seq).cuda()
    out = evaluate.rollout(sim, full, types_.cuda(), torch.tensor(n), torch.zeros(14, n, device="cuda"), nsteps=3,
                           particle_dim=dim, device="cuda", input_sequence_length=11)
    ref_pos, _ = O.rollout(osim, torch.from_numpy(seq), types_, n, 3, 11)
    _close(out["predicted_rollout"], ref_pos.numpy(), atol=6 * ATOL * scale, rtol=1e-6, what="generic rollout")


def test_multi_scale_blocks_and_generic_forward_match_reference():
    """G2M / M2M / M2G blocks called on their own and MultiScaleGNN.forward
    block by block on the width-generic kernels reproduce the reference's
    output (ms2d_s3), and nedge_out != latent_dim runs (vs the oracle)."""
    from oracle import multi_scale_oracle as MO
    from sgnn_amd import generic
    from sgnn_amd.multi_scale import MultiScaleSimulator
    from tests.helpers import ms_product_sim
    z = golden("ms2d_s3")
    sim = ms_product_sim(z)
    gnn = sim._multi_scale_gnn
    t = lambda k: torch.from_numpy(z[k]).cuda()
    from sgnn_amd import autograd
    pred = autograd.ms_gnn_forward(gnn, t("node_features"), t("g2m"), t("ef_g2m"), t("m2m"), t("ef_m2m"), t("m2g"),
                                   t("ef_m2g"))
    assert pred.grad_fn is not None
    _close(pred.detach().cpu().numpy(), z["pred"], what="MultiScaleGNN block by block")
    # nedge_out != latent_dim (the fused chain needs them equal): inference on the generic kernels
    hp = hparams(z)
    d, T = hp["dim"], hp["T"]
    torch.manual_seed(9)
    sim2 = MultiScaleSimulator(d, (T - 1) * d + 1, d + 1, 48, 64, 2, hp["nmlp"], stats_of(z, "cuda"), 1, 9,
                               hp["num_scales"], hp["window"], hp["mult"]).cuda()
    sim2.set_static_graph(ms_graph_of(z, "cuda"))
    assert not sim2._fast_path()
    pos = t("positions")[:, :T]
    with torch.no_grad():
        nxt, strain = sim2.predict_positions(pos, [pos.shape[0]], None)
    state = {k: v.detach().cpu() for k, v in sim2.state_dict().items()}
    osim = MO.MultiScaleOracle(state, d, 2, stats_of(z), ms_graph_of(z), hp["num_scales"], hp["mult"], 1,
                               hp["nmlp"])
    ref_next, ref_strain = osim.predict_positions(pos.cpu())
    _close(strain.cpu().numpy(), ref_strain.numpy(), what="ms nedge_out 48 strain")
    scale = float(np.max(z["acc_std"]))
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * scale, rtol=1e-6, what="ms nedge_out 48 next")
