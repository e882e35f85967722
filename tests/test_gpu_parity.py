"""GPU parity: the HIP path (through the C-ABI) against the reference's own
golden outputs and the oracle.  Tolerances (fp32):
  * graph (edge_index): bit-exact;
  * decoder output / next position / strain: |got - ref| <= ATOL + RTOL*|ref|
    with ATOL = 2e-4, RTOL = 1e-4 on the normalised decoder output (O(1)
    values; the HIP path sums in a different order than MKL/PyG), and the
    same bound scaled by acc_std on positions.
"""
import numpy as np
import pytest
import torch

from tests.helpers import golden, hparams, oracle_sim, product_sim

pytestmark = pytest.mark.gpu

ATOL, RTOL = 2e-4, 1e-4
FWD_H64 = ["tiny2d_r06", "batch2d_r06", "c1_r15", "c1_r06", "types2d_r06"]


def _close(got, ref, atol=ATOL, rtol=RTOL, what=""):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    bound = atol + rtol * np.abs(ref)
    worst = float((err / bound).max()) if err.size else 0.0
    print(f"{what}: max|err|={err.max() if err.size else 0:.3e} worst err/bound={worst:.3f}")
    assert worst <= 1.0, f"{what}: max abs err {err.max():.3e}"


@pytest.mark.parametrize("case", FWD_H64 + ["tiny3d_h128"])
def test_radius_graph_bit_exact(case):
    z = golden(case)
    hp = hparams(z)
    sim = product_sim(z)
    pos = torch.from_numpy(z["positions"][:, hp["T"] - 1]).cuda()
    recv_name, send_name = sim._compute_graph_connectivity(pos, z["nparticles_per_example"], hp["R"])
    ei = torch.stack([recv_name, send_name]).cpu().numpy()
    np.testing.assert_array_equal(ei, z["edge_index"])


@pytest.mark.parametrize("case", FWD_H64 + ["tiny3d_h128"])
def test_predict_positions_matches_reference(case):
    z = golden(case)
    hp = hparams(z)
    sim = product_sim(z)
    pos = torch.from_numpy(z["positions"][:, :hp["T"]]).cuda()
    types_ = torch.from_numpy(z["particle_types"]).cuda()
    nxt, strain = sim.predict_positions(pos, z["nparticles_per_example"], types_)
    torch.cuda.synchronize()
    _close(strain.cpu().numpy(), z["strain"], what=f"{case} strain")
    scale = float(np.max(z["acc_std"]))
    _close(nxt.cpu().numpy(), z["next_position"], atol=ATOL * scale, rtol=1e-6, what=f"{case} next_pos")


def test_rollout_matches_reference():
    from sgnn_amd import evaluate
    z = golden("tiny2d_r06")
    hp = hparams(z)
    sim = product_sim(z)
    pos = torch.from_numpy(z["positions"]).cuda()
    n = pos.shape[0]
    strains = torch.zeros(pos.shape[1], n, device="cuda")
    out = evaluate.rollout(sim, pos, torch.zeros(n, dtype=torch.long, device="cuda"), torch.tensor(n),
                           strains, nsteps=pos.shape[1] - hp["T"], particle_dim=hp["dim"], device="cuda",
                           input_sequence_length=hp["T"])
    scale = float(np.max(z["acc_std"]))
    _close(out["predicted_rollout"], z["rollout_predicted"], atol=4 * ATOL * scale, rtol=1e-6,
           what="rollout positions")
    _close(out["predicted_strain"], z["rollout_strain"], atol=4 * ATOL, what="rollout strain")


def test_one_step_rollout_matches_reference():
    """evaluate.rollout(..., inference_mode='one_step') -- ONE sgnn_rollout_one_step call -- against the
    reference's own teacher-forced rollout (evaluate.py:140-143; golden onestep_* arrays)."""
    from sgnn_amd import evaluate
    z = golden("tiny2d_r06")
    hp = hparams(z)
    sim = product_sim(z)
    pos = torch.from_numpy(z["positions"]).cuda()
    n = pos.shape[0]
    strains = torch.zeros(pos.shape[1], n, device="cuda")
    out = evaluate.rollout(sim, pos, torch.zeros(n, dtype=torch.long, device="cuda"), torch.tensor(n),
                           strains, nsteps=pos.shape[1] - hp["T"], particle_dim=hp["dim"], device="cuda",
                           input_sequence_length=hp["T"], inference_mode="one_step")
    scale = float(np.max(z["acc_std"]))
    _close(out["predicted_rollout"], z["onestep_predicted"], atol=4 * ATOL * scale, rtol=1e-6,
           what="one_step rollout positions")
    _close(out["predicted_strain"], z["onestep_strain"], atol=4 * ATOL, what="one_step rollout strain")
    np.testing.assert_allclose(out["rmse_position"], z["onestep_rmse_position"], rtol=1e-3, atol=1e-7)


def _lattice_case(nx, ny, radius, seed, n_ex=1):
    from sgnn_amd import synthetic
    seqs = [synthetic.trajectory(synthetic.lattice_2d(nx, ny, x0=0.25 + 0.1 * k), 11, seed=seed + k)
            for k in range(n_ex)]
    return np.concatenate(seqs, 0), [s.shape[0] for s in seqs]


@pytest.mark.parametrize("nx,ny,radius,n_ex", [(250, 200, 0.6, 1), (60, 40, 1.1, 3), (50, 40, 15.0, 2)])
def test_large_against_oracle(nx, ny, radius, n_ex):
    """C2-sized (50k) and multi-example graphs vs the oracle (same weights)."""
    z = golden("c1_r06")
    from oracle import sgnn_oracle as O
    from tests.helpers import state_of, stats_of
    seq, counts = _lattice_case(nx, ny, radius, 21, n_ex)
    sim = product_sim(z)
    sim._connectivity_radius = radius
    osim = O.OracleSimulator(state_of(z), 2, 5, radius, stats_of(z))
    pos = torch.from_numpy(seq)
    types_ = torch.zeros(seq.shape[0], dtype=torch.long)
    ref_next, ref_strain = osim.predict_positions(pos, counts, types_)
    ei_ref = O.radius_graph(pos[:, -1], counts, radius)
    r, s = sim._compute_graph_connectivity(pos[:, -1].cuda(), counts, radius)
    np.testing.assert_array_equal(torch.stack([r, s]).cpu().numpy(), ei_ref.numpy())
    nxt, strain = sim.predict_positions(pos.cuda(), counts, types_.cuda())
    _close(strain.cpu().numpy(), ref_strain.numpy(), what=f"{nx}x{ny} r={radius} strain")
    # the acceleration channels through the Euler integrator (positions: the normalised-output bound x acc_std)
    scale = float(np.max(z["acc_std"]))
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * scale, rtol=1e-6, what=f"{nx}x{ny} r={radius} next_pos")


def test_radius_graph_random_vs_bruteforce():
    """Random clouds, several examples, loop on/off, cap binding, a NaN particle;
    sizes on both sides of the small-graph path's limit (n <= 8192: LDS brute
    force in index order; above: the cell-list pipeline)."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import engine
    g = torch.Generator().manual_seed(3)
    for trial, (n, dim, r, loop) in enumerate([(700, 2, 0.9, True), (500, 3, 1.3, True),
                                               (600, 2, 3.0, False), (400, 3, 0.5, False),
                                               (8192, 3, 0.9, False), (9000, 2, 0.25, True),
                                               (12000, 3, 1.2, False)]):
        pos = torch.rand(n, dim, generator=g) * 10.0
        pos[5] = float("nan")
        counts = [n // 3, n // 3, n - 2 * (n // 3)]
        ref = O.radius_graph(pos, counts, r, loop=loop, method="bruteforce")
        ws = engine.StepWorkspace(n, 2, dim, 64, 20, loop, torch.device("cuda"))
        engine.radius_graph(ws, pos.cuda(), 0, dim, engine.ex_ptr_tensor(counts, "cuda"), 3, r)
        e = ws.num_edges()
        got = torch.stack([ws.send[:e], ws.recv[:e]]).cpu().to(torch.int64)
        np.testing.assert_array_equal(got.numpy(), ref.numpy(), err_msg=f"trial {trial}")


@pytest.mark.parametrize("K,loop", [(32, False), (48, True), (63, False)])
def test_radius_graph_caps_above_32(K, loop):
    """Neighbour caps past 32: torch_cluster's default max_num_neighbors = 32
    with loop = False asks for 33 candidates (INTEGRATION.md's stub), up to 64
    here.  Dense random clouds so the cap binds, both paths (n <= 8192: LDS
    brute force; above: the cell-list pipeline with the 64-slot register
    list), several examples, bit-exact against the brute-force oracle."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import engine
    g = torch.Generator().manual_seed(11 + K)
    for trial, (n, dim, r) in enumerate([(3000, 2, 1.2), (2500, 3, 1.6), (12000, 2, 0.7), (10000, 3, 0.9)]):
        side = 10.0 if dim == 2 else 6.0
        pos = torch.rand(n, dim, generator=g) * side
        counts = [n // 2, n - n // 2]
        ref = O.radius_graph(pos, counts, r, loop=loop, max_num_neighbors=K, method="bruteforce")
        deg = torch.bincount(ref[1], minlength=n)
        # the cap binds (loop = False: K + 1 candidates, then the self edge dropped, so rows whose
        # self is not among them keep K + 1, as torch_cluster's radius_graph does)
        assert int(deg.max()) == (K if loop else K + 1), "the cap should bind in this cloud"
        ws = engine.StepWorkspace(n, 2, dim, 64, K, loop, torch.device("cuda"))
        engine.radius_graph(ws, pos.cuda(), 0, dim, engine.ex_ptr_tensor(counts, "cuda"), 2, r)
        e = ws.num_edges()
        got = torch.stack([ws.send[:e], ws.recv[:e]]).cpu().to(torch.int64)
        np.testing.assert_array_equal(got.numpy(), ref.numpy(), err_msg=f"K={K} loop={loop} trial {trial}")
    # the static-graph entry (torch_cluster.radius_graph(pos, r, max_num_neighbors=K, loop=...))
    pos = torch.rand(4000, 2, generator=g) * 10.0
    csr = engine.radius_graph_csr(pos.cuda(), 1.0, K, loop)
    ref = O.radius_graph(pos, [4000], 1.0, loop=loop, max_num_neighbors=K, method="bruteforce")
    e = csr.num_edges
    np.testing.assert_array_equal(torch.stack([csr.send[:e], csr.recv[:e]]).cpu().to(torch.int64).numpy(), ref.numpy())


def test_3d_h128_against_oracle():
    """Config-4 shapes (3D, H=128) at a size the oracle finishes quickly."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from tests.helpers import state_of, stats_of
    z = golden("tiny3d_h128")
    hp = hparams(z)
    seq = synthetic.trajectory(synthetic.lattice_3d(16, 10, 8), hp["T"], seed=31)
    sim = product_sim(z)
    osim = O.OracleSimulator(state_of(z), 3, hp["L"], hp["R"], stats_of(z))
    pos = torch.from_numpy(seq)
    types_ = torch.zeros(seq.shape[0], dtype=torch.long)
    ref_next, ref_strain = osim.predict_positions(pos, [seq.shape[0]], types_)
    nxt, strain = sim.predict_positions(pos.cuda(), [seq.shape[0]], types_.cuda())
    _close(strain.cpu().numpy(), ref_strain.numpy(), what="3d h128 strain")
    scale = float(np.max(z["acc_std"]))
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * scale, rtol=1e-6, what="3d h128 next_pos")


@pytest.mark.parametrize("case", FWD_H64 + ["tiny3d_h128"])
def test_encode_process_decode_on_explicit_features(case):
    """The operator boundary EncodeProcessDecode.forward(x, edge_index, e)
    (graph_network.py:388-406) on the reference's own features."""
    z = golden(case)
    sim = product_sim(z)
    t = lambda k: torch.from_numpy(z[k]).cuda()
    with torch.no_grad():   # inference: the fused chain (engine.epd_forward)
        pred = sim._encode_process_decode(t("node_features"), t("edge_index"), t("edge_features"))
    torch.cuda.synchronize()
    _close(pred.cpu().numpy(), z["pred"], what=f"{case} EPD.forward")


def test_encode_process_decode_edgeless_and_shuffled():
    """No edges at all (aggregates are zero) and a shuffled COO edge order
    (the CSR conversion restores receiver order; sums are order-independent
    up to fp32 rounding) against the oracle."""
    from oracle import sgnn_oracle as O
    from tests.helpers import state_of
    z = golden("tiny2d_r06")
    sim = product_sim(z)
    state = state_of(z)
    nf = torch.from_numpy(z["node_features"])
    ei = torch.from_numpy(z["edge_index"])
    ef = torch.from_numpy(z["edge_features"])
    ref = O.encode_process_decode(state, nf, ei[:, :0], ef[:0], 5)
    perm = torch.randperm(ei.shape[1], generator=torch.Generator().manual_seed(0))
    for grad in (False, True):   # the fused chain, then the differentiable path
        with torch.set_grad_enabled(grad):
            got = sim._encode_process_decode(nf.cuda(), ei[:, :0].cuda(), ef[:0].cuda())
            _close(got.detach().cpu().numpy(), ref.numpy(), what=f"edgeless EPD.forward grad={grad}")
            got = sim._encode_process_decode(nf.cuda(), ei[:, perm].cuda(), ef[perm].cuda())
            _close(got.detach().cpu().numpy(), z["pred"], what=f"shuffled EPD.forward grad={grad}")


@pytest.mark.parametrize("nsteps", [8, 9])
def test_device_rollout_runner(nsteps):
    """evaluate.rollout's device path (fused window shift, predictions written
    into device slots) matches the oracle rollout."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    z = golden("tiny2d_r06")
    hp = hparams(z)
    T = hp["T"]
    seq = synthetic.trajectory(synthetic.lattice_2d(24, 16), T + nsteps, seed=17)
    n = seq.shape[0]
    sim = product_sim(z)
    types_ = torch.zeros(n, dtype=torch.long, device="cuda")
    win = torch.from_numpy(seq[:, :T]).cuda()
    pos, strain = sim.rollout_runner(win, [n], types_, nsteps).run()
    torch.cuda.synchronize()
    osim = oracle_sim(z)
    ref_pos, ref_str = O.rollout(osim, torch.from_numpy(seq), torch.zeros(n, dtype=torch.long), n, nsteps, T)
    scale = float(np.max(z["acc_std"]))
    _close(pos.cpu().numpy(), ref_pos.numpy(), atol=2 * nsteps * ATOL * scale, rtol=1e-6,
           what=f"device rollout {nsteps} positions")


@pytest.mark.parametrize("dim,nmlp,dims,radius,n_ex,ntypes", [
    (2, 2, (40, 30), 1.1, 3, 1),      # nmlp_layers = 2 (3-Linear MLPs), several examples
    (3, 1, (16, 14, 12), 0.75, 1, 1),  # 3D at hidden 64
    (2, 1, (60, 40), 15.0, 2, 3),     # cap binds, particle-type embeddings
    (2, 1, (100, 82), 0.6, 1, 1),     # n = 8200 > 8192: the edge / node kernel pair
])
def test_inference_paths_against_oracle(dim, nmlp, dims, radius, n_ex, ntypes):
    """predict_positions at hidden 64 on both inference paths (the fused
    per-layer kernel for n <= 8192, the edge / node pair above) vs the oracle:
    strain and next positions within the module's forward bound."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    from sgnn_amd.learned_simulator import LearnedSimulator
    lat = synthetic.lattice_2d if dim == 2 else synthetic.lattice_3d
    seqs = [synthetic.trajectory(lat(*dims), 11, seed=40 + k) for k in range(n_ex)]
    for k, sq in enumerate(seqs):
        sq[..., 0] += 0.13 * k
    seq = np.concatenate(seqs, 0)
    counts = [s.shape[0] for s in seqs]
    n = seq.shape[0]
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(7)
    emb = 16 if ntypes > 1 else 0
    sim = LearnedSimulator(dim, 10 * dim + 1 + emb, dim + 1, 64, 5, nmlp, 64, radius, stats, ntypes, emb or 9)
    state = {k: v.detach().clone() for k, v in sim.state_dict().items()}
    types_ = torch.from_numpy(np.random.default_rng(1).integers(0, ntypes, n))
    pos = torch.from_numpy(seq)
    osim = O.OracleSimulator(state, dim, 5, radius, stats, ntypes, nmlp_layers=nmlp)
    ref_next, ref_strain = osim.predict_positions(pos, counts, types_)
    sim = sim.cuda()
    nxt, strain = sim.predict_positions(pos.cuda(), counts, types_.cuda())
    torch.cuda.synchronize()
    _close(strain.cpu().numpy(), ref_strain.numpy(), what=f"n={n} dim={dim} nmlp={nmlp} strain")
    scale = float(np.max(st["acceleration"]["std"]))
    _close(nxt.cpu().numpy(), ref_next.numpy(), atol=ATOL * scale, rtol=1e-6, what=f"n={n} next_pos")
