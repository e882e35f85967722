"""GPU parity for the multi-scale path: the HIP
chain through the C-ABI against the reference's golden outputs and the
multi-scale oracle.  Tolerances as tests/test_gpu_parity.py (fp32, different
summation order than MKL / PyG): |got - ref| <= 2e-4 + 1e-4 |ref| on the
normalised prediction, the same bound x acc_std on positions; graphs and
CSR conversions bit-exact."""
import numpy as np
import pytest
import torch

from tests.helpers import MS_CASES, golden, hparams, ms_graph_of, ms_oracle_sim, ms_product_sim
from tests.test_gpu_parity import ATOL, _close

pytestmark = pytest.mark.gpu


def _stable_csr(ei: np.ndarray, n: int):
    order = np.argsort(ei[1], kind="stable")
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, ei[1] + 1, 1)
    return np.cumsum(rowptr), ei[0][order], ei[1][order]


def test_coo_to_csr_stable_bit_exact():
    from sgnn_amd import engine
    rng = np.random.default_rng(0)
    for n, E in [(1, 0), (7, 1), (300, 5000), (1000, 37), (64, 4000)]:
        ei = np.stack([rng.integers(0, n, E), rng.integers(0, n, E)]).astype(np.int64)
        g = engine.coo_to_csr(torch.from_numpy(ei).cuda(), n)
        rp, s, r = _stable_csr(ei, n)
        assert g.num_edges == E
        np.testing.assert_array_equal(g.rowptr.cpu().numpy(), rp)
        np.testing.assert_array_equal(g.send[:E].cpu().numpy(), s)
        np.testing.assert_array_equal(g.recv[:E].cpu().numpy(), r)
    with pytest.raises(ValueError):
        engine.coo_to_csr(torch.tensor([[0, 5], [1, 2]]).cuda(), 3)


@pytest.mark.parametrize("case", MS_CASES)
def test_static_graph_on_gpu_bit_exact(case):
    from sgnn_amd.multi_scale import build_static_multi_scale_graph
    z = golden(case)
    hp = hparams(z)
    g = build_static_multi_scale_graph(torch.from_numpy(z["positions"][:, 0]).cuda(), hp["num_scales"],
                                       hp["window"], hp["mult"])
    for s in range(hp["num_scales"]):
        np.testing.assert_array_equal(g["graph_hierarchy"][s]["sampling_indices"].cpu().numpy(),
                                      z[f"scale{s}_indices"])
    for k, key in [("g2m", "grid2mesh_edges"), ("m2m", "mesh2mesh_edges"), ("m2g", "mesh2grid_edges")]:
        np.testing.assert_array_equal(g[key].cpu().numpy(), z[k], err_msg=k)


@pytest.mark.parametrize("case", MS_CASES)
def test_predict_positions_matches_reference(case):
    z = golden(case)
    hp = hparams(z)
    sim = ms_product_sim(z)
    pos = torch.from_numpy(z["positions"][:, :hp["T"]]).cuda()
    types_ = torch.from_numpy(z["particle_types"]).cuda()
    nxt, strain = sim.predict_positions(pos, [pos.shape[0]], types_)
    torch.cuda.synchronize()
    _close(strain.cpu().numpy(), z["strain"], what=f"{case} strain")
    scale = float(np.max(z["acc_std"]))
    _close(nxt.cpu().numpy(), z["next_position"], atol=ATOL * scale, rtol=1e-6, what=f"{case} next_pos")
    with torch.no_grad():
        pa, ta, ps = sim.predict_accelerations(pos[:, -1], torch.zeros_like(pos), pos, [pos.shape[0]], types_)
    _close(pa.cpu().numpy(), z["pred"][:, :hp["dim"]], what=f"{case} pred_acc")


def test_rollout_matches_reference():
    from sgnn_amd.multi_scale.multi_scale_evaluate import evaluate_multi_scale_rollout
    z = golden("ms2d_s3")
    hp = hparams(z)
    sim = ms_product_sim(z)
    pos = torch.from_numpy(z["positions"]).cuda()
    n = pos.shape[0]
    out = evaluate_multi_scale_rollout(sim, pos, torch.zeros(n, dtype=torch.long).cuda(), [n],
                                       torch.zeros(pos.shape[1], n).cuda(), 3, hp["dim"], "cuda", hp["T"])
    scale = float(np.max(z["acc_std"]))
    _close(out["predicted_rollout"], z["rollout_predicted"], atol=3 * ATOL * scale, rtol=1e-6,
           what="ms rollout positions")
    _close(out["predicted_strain"], z["rollout_strain"], atol=3 * ATOL, what="ms rollout strain")


@pytest.mark.parametrize("dims,case", [((60, 40), "ms2d_s3"), ((20, 16, 12), "ms3d_h128")])
def test_larger_against_oracle(dims, case):
    """Bigger lattices than the fixtures (graph built on the GPU, checked against
    the oracle's graph first), prediction vs the oracle."""
    from oracle import multi_scale_oracle as MO
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import build_static_multi_scale_graph
    z = golden(case)
    hp = hparams(z)
    base = (synthetic.lattice_2d(*dims, x0=-1.75) if len(dims) == 2
            else synthetic.lattice_3d(*dims, x0=-1.75))
    seq = synthetic.trajectory(base, hp["T"], seed=41)
    g_ref = MO.create_all_edges(torch.from_numpy(seq[:, 0]), hp["num_scales"], hp["window"], hp["mult"])
    g = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).cuda(), hp["num_scales"], hp["window"],
                                       hp["mult"])
    for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
        np.testing.assert_array_equal(g[key].cpu().numpy(), g_ref[key].numpy(), err_msg=key)
    n = seq.shape[0]
    types_ = torch.from_numpy(np.random.default_rng(2).integers(0, hp["ntypes"], n))
    sim = ms_product_sim(z)
    sim.set_static_graph(g)
    osim = ms_oracle_sim(z, g_ref)
    pos = torch.from_numpy(seq)
    ref_next, ref_strain = osim.predict_positions(pos, types_)
    nxt, strain = sim.predict_positions(pos.cuda(), [n], types_.cuda())
    _close(strain.cpu().numpy(), ref_strain.numpy(), what=f"{dims} strain")
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * float(np.max(z["acc_std"])), rtol=1e-6,
           what=f"{dims} next_pos")


def test_high_degree_user_graph_against_oracle():
    """A user-supplied static graph whose receivers have up to 100 incoming
    edges (segments spanning several 32-edge tiles) and nodes with none."""
    z = golden("ms2d_s3")
    hp = hparams(z)
    n = z["positions"].shape[0]
    rng = np.random.default_rng(9)
    graph = ms_graph_of(z)
    hubs = np.repeat(np.arange(0, 40, 4), 100)          # 10 receivers x 100 edges
    extra = np.stack([rng.integers(0, n, hubs.size), hubs]).astype(np.int64)
    m2m = np.concatenate([z["m2m"], extra], 1)
    m2m = m2m[:, rng.permutation(m2m.shape[1])]
    graph["mesh2mesh_edges"] = torch.from_numpy(m2m)
    osim = ms_oracle_sim(z, graph)
    sim = ms_product_sim(z)
    sim.set_static_graph({k: (v.cuda() if isinstance(v, torch.Tensor) else v) for k, v in graph.items()})
    pos = torch.from_numpy(z["positions"][:, :hp["T"]])
    ref_next, ref_strain = osim.predict_positions(pos, None)
    nxt, strain = sim.predict_positions(pos.cuda(), [n], None)
    _close(strain.cpu().numpy(), ref_strain.numpy(), what="high-degree strain")
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * float(np.max(z["acc_std"])), rtol=1e-6,
           what="high-degree next_pos")


@pytest.mark.parametrize("case", MS_CASES)
def test_multi_scale_gnn_on_explicit_features(case):
    """MultiScaleGNN.forward(x, g2m_ei, g2m_e, m2m_ei, m2m_e, m2g_ei, m2g_e, h)
    (multi_scale_gnn.py:262-326) on the reference's own features."""
    z = golden(case)
    sim = ms_product_sim(z)
    t = lambda k: torch.from_numpy(z[k]).cuda()
    with torch.no_grad():   # inference: the fused chain (ms_engine.gnn_forward)
        pred = sim._multi_scale_gnn(t("node_features"), t("g2m"), t("ef_g2m"), t("m2m"), t("ef_m2m"), t("m2g"),
                                    t("ef_m2g"), None)
    torch.cuda.synchronize()
    _close(pred.cpu().numpy(), z["pred"], what=f"{case} MultiScaleGNN.forward")


def test_batched_static_graphs_per_sample(tmp_path):
    """f4: the multi-scale dataset on the GPU graph builder, two trajectories
    of different sizes in one batch with per_sample_graphs=True: the HIP
    simulator on the merged block-diagonal graph reproduces each sample run
    alone (fp32 summation order aside), and each sample's graph equals the
    oracle's hierarchy build of its first frame."""
    import json
    from oracle import multi_scale_oracle as MO
    from sgnn_amd import data as D
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import MultiScaleSimulator
    from sgnn_amd.multi_scale import static_graph_data_loader as S
    trajs = {}
    for k, (nx, ny, x0) in enumerate([(20, 12, -1.75), (24, 10, -1.25)]):
        seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny, x0=x0), 10, seed=30 + k)
        pos = np.transpose(seq, (1, 0, 2)).copy()
        trajs[f"t{k}"] = (pos, np.zeros(pos.shape[1], np.int64), np.zeros(pos.shape[:2]))
    path = str(tmp_path / "train.npz")
    D.save_trajectories(path, trajs, reference_format=True)
    (tmp_path / "metadata.json").write_text(json.dumps({"stress_mean": 0.0, "stress_std": 1.0}))
    ds = S.MultiScaleTaylorImpactSamplesDataset(path, input_length_sequence=6, num_scales=2, window_size=2,
                                                radius_multiplier=2.0)
    items = [ds[0], ds[len(ds) - 1]]
    for it, (pos, _, _) in zip(items, trajs.values()):
        ref = MO.create_all_edges(torch.tensor(pos[0]), 2, 2, 2.0)
        for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
            np.testing.assert_array_equal(it["graph"][key].cpu().numpy(), ref[key].numpy(), err_msg=key)
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(5)
    sim = MultiScaleSimulator(2, 11, 3, 64, 64, 3, 2, stats, 1, 9, 2, 2, 2.0).cuda()
    outs = []
    for it in items:
        sim.set_static_graph(it["graph"])
        p = torch.from_numpy(it["input"]["positions"]).cuda()
        outs.append(sim.predict_positions(p, [p.shape[0]], None))
    merged = S.multi_scale_collate_fn(items, per_sample_graphs=True)
    sim.set_static_graph(merged["graph"])
    p = merged["input"]["positions"].cuda()
    nxt, strain = sim.predict_positions(p, merged["input"]["n_particles_per_example"].tolist(), None)
    torch.cuda.synchronize()
    np.testing.assert_allclose(nxt.cpu().numpy(), torch.cat([o[0] for o in outs]).cpu().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(strain.cpu().numpy(), torch.cat([o[1] for o in outs]).cpu().numpy(), rtol=0,
                               atol=2e-4)


def test_multi_scale_loaders_default_arguments(tmp_path):
    """Both multi-scale loaders with their default arguments (GPU graph builder,
    pin_memory=True as in the reference): the static graphs live in host memory,
    so the DataLoader can pin every batch; a batch drives the simulator."""
    import json
    from sgnn_amd import data as D
    from sgnn_amd import synthetic
    from sgnn_amd.multi_scale import MultiScaleSimulator
    from sgnn_amd.multi_scale import static_graph_data_loader as S
    trajs = {}
    for k, (nx, ny) in enumerate([(16, 10), (18, 8)]):
        seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny, x0=-1.75), 9, seed=50 + k)
        pos = np.transpose(seq, (1, 0, 2)).copy()
        trajs[f"t{k}"] = (pos, np.zeros(pos.shape[1], np.int64), np.zeros(pos.shape[:2]))
    path = str(tmp_path / "train.npz")
    D.save_trajectories(path, trajs, reference_format=True)
    (tmp_path / "metadata.json").write_text(json.dumps({"stress_mean": 0.0, "stress_std": 1.0}))
    batches = list(S.get_multi_scale_data_loader_by_samples(path, input_length_sequence=6, batch_size=1,
                                                            num_scales=2, window_size=2))
    trajectories = list(S.get_multi_scale_data_loader_by_trajectories(path, num_scales=2, window_size=2))
    assert len(batches) == sum(t[0].shape[0] - 6 for t in trajs.values())
    assert len(trajectories) == 2
    for b in batches[:2] + trajectories:
        assert all(not v.is_cuda for v in (b["graph"]["grid2mesh_edges"], b["graph"]["mesh2mesh_edges"]))
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(6)
    sim = MultiScaleSimulator(2, 11, 3, 64, 64, 3, 2, stats, 1, 9, 2, 2, 2.0).cuda()
    b = batches[0]
    sim.set_static_graph(b["graph"])
    p = b["input"]["positions"].cuda()
    nxt, strain = sim.predict_positions(p, b["input"]["n_particles_per_example"].tolist(), None)
    torch.cuda.synchronize()
    assert torch.isfinite(nxt).all() and torch.isfinite(strain).all()
