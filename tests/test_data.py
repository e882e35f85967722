"""Real-data ingestion on CPU: the Taylor-impact npz
format (the reference's pickled `trajectories` dict, read without executing
code, and the flat pickle-free layout), the samples / trajectories datasets and
collate with the reference's indexing (taylor_impact_data_loader.py:96-284),
device-side window batching equal to the host collate in the DataLoader's
order, and checkpoint / optimizer-state interchange with torch.optim.Adam.

Parity: pinned to the reference's own loader (test_loaders_match_reference_
loader_outputs: tests/golden/loader_taylor.npz was produced by running
datasets/taylor_impact_2d/taylor_impact_data_loader.py on a synthetic split,
tests/golden/make_golden_data.py); the other tests restate its semantics for
the edge cases (no dataset file ships with the reference)."""
import io
import json
import os
import pickle
import zipfile

import numpy as np
import pytest
import torch

from sgnn_amd import data as D


def _trajs(seed=0, sizes=(12, 20, 9), T=14, dim=2):
    rng = np.random.default_rng(seed)
    return {f"case_{i}": (rng.normal(size=(T, n, dim)).astype(np.float32),
                          np.full(n, 0, dtype=np.int64),
                          rng.normal(size=(T, n)).astype(np.float64))
            for i, n in enumerate(sizes)}


@pytest.fixture()
def split(tmp_path):
    tr = _trajs()
    path = tmp_path / "train.npz"
    D.save_trajectories(str(path), tr, reference_format=True)
    md = {"sequence_length": 14, "vel_mean": [0.0, 0.0], "vel_std": [1.0, 1.0], "acc_mean": [0.0, 0.0],
          "acc_std": [1.0, 1.0], "stress_mean": 2.5, "stress_std": 4.0, "num_particle_types": 1}
    (tmp_path / "metadata.json").write_text(json.dumps(md))
    return tr, str(path), md


def test_both_layouts_round_trip(tmp_path):
    tr = _trajs()
    for ref in (True, False):
        p = str(tmp_path / f"s{int(ref)}.npz")
        D.save_trajectories(p, tr, reference_format=ref)
        got = D.load_trajectories(p)
        assert list(got) == list(tr)
        for k in tr:
            for a, b in zip(tr[k], got[k]):
                assert a.dtype == b.dtype and np.array_equal(a, b)


def test_reference_pickle_cannot_run_code(tmp_path):
    """A `trajectories` member naming anything but numpy's array reconstructors is refused."""
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    buf = io.BytesIO()
    np.lib.format.write_array(buf, np.array(Evil(), dtype=object), allow_pickle=True)
    p = tmp_path / "evil.npz"
    with zipfile.ZipFile(p, "w") as zf:
        zf.writestr("trajectories.npy", buf.getvalue())
    with pytest.raises(pickle.UnpicklingError, match="refusing"):
        D.load_trajectories(str(p))
    with pytest.raises(FileNotFoundError):
        D.load_trajectories(str(tmp_path / "missing.npz"))


def test_samples_dataset_indexing(split):
    tr, path, md = split
    T_in = 6
    ds = D.TaylorImpactSamplesDataset(path, T_in)
    lens = [v[0].shape[0] - T_in for v in tr.values()]
    assert len(ds) == sum(lens)
    # restated reference semantics: trajectory k owns samples [start_k, start_k + len_k)
    idx = 0
    for k, (pos, types, stress) in enumerate(tr.values()):
        for t in range(T_in, pos.shape[0]):
            item = ds[idx]
            assert item["meta"] == {"trajectory_idx": k, "time_idx": t}
            assert np.array_equal(item["input"]["positions"], np.transpose(pos[t - T_in:t], (1, 0, 2)))
            assert np.array_equal(item["output"]["next_position"], pos[t])
            assert np.array_equal(item["output"]["next_strain"], stress[t].astype(np.float32))
            assert item["input"]["n_particles_per_example"] == pos.shape[1]
            idx += 1
    assert ds._stress_stats == {"mean": 2.5, "std": 4.0}
    np.testing.assert_allclose(ds.denormalize_stress(np.array([1.0])), [6.5])


def test_device_batches_equal_host_collate_in_dataloader_order(split):
    tr, path, md = split
    ds = D.TaylorImpactSamplesDataset(path, 5)
    dev = D.DeviceSamples(ds, "cpu")
    torch.manual_seed(3)
    host = list(D.get_data_loader_by_samples(path, 5, batch_size=4, shuffle=True, pin_memory=False))
    torch.manual_seed(3)
    mine = list(dev.loader(batch_size=4, shuffle=True))
    assert len(host) == len(mine) == (len(ds) + 3) // 4
    for h, m in zip(host, mine):
        for grp in ("input", "output", "meta"):
            for key in h[grp]:
                a, b = h[grp][key], m[grp][key]
                assert torch.equal(a.to(b.dtype), b), (grp, key)
    torch.manual_seed(3)
    idx = next(iter(dev.index_batches(4)))
    assert dev.count(idx) == int(host[0]["input"]["n_particles_per_example"].sum())


def test_trajectories_dataset_and_info(split):
    tr, path, md = split
    ds = D.TaylorImpactTrajectoriesDataset(path)
    assert len(ds) == 3
    item = ds[1]
    pos = list(tr.values())[1][0]
    assert torch.equal(item["positions"], torch.from_numpy(np.transpose(pos, (1, 0, 2))))
    assert int(item["n_particles_per_example"]) == pos.shape[1]
    assert item["strains"].dtype == torch.float32
    info = D.get_dataset_info(path)
    assert info["num_trajectories"] == 3 and info["num_particles"] == 12 and info["max_timesteps"] == 14
    assert D.read_metadata(os.path.dirname(path))["stress_std"] == 4.0


def _small_sim():
    from sgnn_amd import synthetic
    from sgnn_amd.learned_simulator import LearnedSimulator
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(0)
    return LearnedSimulator(2, 21, 3, 16, 2, 1, 16, 0.6, stats, 1, 9)


def test_adam_state_interchanges_with_torch_adam():
    from sgnn_amd import training
    ref = _small_sim()
    opt = torch.optim.Adam(ref.parameters(), lr=3e-4)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        for p in ref.parameters():
            p.grad = torch.randn(p.shape, generator=g)
        opt.step()
    mine_sim = _small_sim()
    flat = training.FlatParams(mine_sim)
    adam = training.Adam(flat, 1e-3)
    adam.load_state_dict(opt.state_dict())
    assert adam.step_count == 3 and adam.lr == 3e-4
    for (off, n, shape), p in zip(flat.order, ref.parameters()):
        st = opt.state[p]
        assert torch.equal(adam.exp_avg[off:off + n].view(shape), st["exp_avg"])
        assert torch.equal(adam.exp_avg_sq[off:off + n].view(shape), st["exp_avg_sq"])
    # and back: a torch Adam accepts ours
    opt2 = torch.optim.Adam(_small_sim().parameters(), lr=1.0)
    opt2.load_state_dict(adam.state_dict())
    for a, b in zip(opt.state_dict()["state"].values(), opt2.state_dict()["state"].values()):
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a[k], b[k])
    assert opt2.param_groups[0]["lr"] == 3e-4


def test_checkpoint_files_load_weights_only(tmp_path):
    from sgnn_amd import checkpoint_utils
    sim = _small_sim()
    sim.save(str(tmp_path / "model-best-000010.pt"))
    opt = torch.optim.Adam(sim.parameters())
    checkpoint_utils.save_train_state(str(tmp_path / "train_state-best-000010.pt"), opt.state_dict(), 10,
                                      lowest_eval_loss=0.5)
    other = _small_sim()
    with torch.no_grad():
        for p in other.parameters():
            p.zero_()
    _, step, ost = checkpoint_utils.load_model(other, str(tmp_path) + "/", "model-best-000010.pt",
                                               "train_state-best-000010.pt", "cpu")
    assert step == 10 and "param_groups" in ost
    for a, b in zip(sim.state_dict().values(), other.state_dict().values()):
        assert torch.equal(a, b)
    with pytest.raises(FileNotFoundError):
        checkpoint_utils.load_model(other, str(tmp_path) + "/", "nope.pt", "nope.pt", "cpu")


def test_simulator_factory_stats_and_features():
    from sgnn_amd.train import _get_simulator
    md = {"vel_mean": [0.1, 0.2], "vel_std": [0.3, 0.4], "acc_mean": [0.0, 0.01], "acc_std": [0.05, 0.06],
          "num_particle_types": 3}
    cfg = {"dim": 2, "input_sequence_length": 11, "particle_type_embedding_size": 9, "hidden_dim": 16,
           "layers": 2, "connection_radius": 0.6}
    sim = _get_simulator(md, 0.02, 0.02, "cpu", cfg)
    st = sim._normalization_stats
    np.testing.assert_allclose(st["velocity"]["std"].numpy(), np.sqrt(np.array([0.3, 0.4]) ** 2 + 0.02 ** 2),
                               rtol=1e-6)
    np.testing.assert_allclose(st["acceleration"]["std"].numpy(),
                               np.sqrt(np.array([0.05, 0.06]) ** 2 + 0.02 ** 2), rtol=1e-6)
    enc = sim._encode_process_decode._encoder.node_fn[0][0]
    assert enc.in_features == 10 * 2 + 1 + 9
    assert sim._particle_type_embedding.weight.shape == (3, 9)


def test_loaders_match_reference_loader_outputs(tmp_path):
    """f1 pinned to the reference itself: tests/golden/loader_taylor.npz holds
    what datasets/taylor_impact_2d/taylor_impact_data_loader.py returned on a
    synthetic split (tests/golden/make_golden_data.py); the same split through
    sgnn_amd.data must give identical items, collate, loader batches,
    trajectories, dataset info and stress denormalisation."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "loader_taylor.npz"))
    k = 0
    trajs = {}
    while f"in{k}_positions" in z.files:
        trajs[f"traj_{k}"] = (z[f"in{k}_positions"], z[f"in{k}_types"], z[f"in{k}_stresses"])
        k += 1
    path = tmp_path / "train.npz"
    D.save_trajectories(str(path), trajs, reference_format=True)
    (tmp_path / "metadata.json").write_text(json.dumps({"stress_mean": float(z["stress_mean"]),
                                                        "stress_std": float(z["stress_std"]),
                                                        "sequence_length": 14}))
    L = int(z["input_len"])
    ds = D.TaylorImpactSamplesDataset(str(path), input_length_sequence=L)
    assert len(ds) == int(z["samples_len"])

    def same(a, b):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
        np.testing.assert_array_equal(a, b)

    for i in z["sample_idx"]:
        it = ds[int(i)]
        same(it["input"]["positions"], z[f"s{i}_positions"])
        same(it["input"]["particle_type"], z[f"s{i}_particle_type"])
        assert int(it["input"]["n_particles_per_example"]) == int(z[f"s{i}_n"])
        same(it["output"]["next_position"], z[f"s{i}_next_position"])
        same(it["output"]["next_strain"], z[f"s{i}_next_strain"])
        assert int(it["meta"]["trajectory_idx"]) == int(z[f"s{i}_traj"])
        assert int(it["meta"]["time_idx"]) == int(z[f"s{i}_time"])
    b = D.collate_fn([ds[i] for i in (1, 9, 21)])
    same(b["input"]["positions"].numpy(), z["c_positions"])
    same(b["input"]["particle_type"].numpy(), z["c_particle_type"])
    same(b["input"]["n_particles_per_example"].numpy(), z["c_n"])
    same(b["output"]["next_position"].numpy(), z["c_next_position"])
    same(b["output"]["next_strain"].numpy(), z["c_next_strain"])
    same(b["meta"]["trajectory_idx"].numpy(), z["c_traj"])
    same(b["meta"]["time_idx"].numpy(), z["c_time"])
    batches = list(D.get_data_loader_by_samples(str(path), input_length_sequence=L, batch_size=4,
                                                shuffle=False, pin_memory=False))
    assert len(batches) == int(z["dl_nbatches"])
    for kb in (0, int(z["dl_last"])):
        same(batches[kb]["input"]["positions"].numpy(), z[f"dl{kb}_positions"])
        same(batches[kb]["input"]["n_particles_per_example"].numpy(), z[f"dl{kb}_n"])
        same(batches[kb]["meta"]["time_idx"].numpy(), z[f"dl{kb}_time"])
        same(batches[kb]["output"]["next_strain"].numpy(), z[f"dl{kb}_next_strain"])
    tds = D.TaylorImpactTrajectoriesDataset(str(path))
    assert len(tds) == int(z["traj_len"])
    for kt in range(len(tds)):
        it = tds[kt]
        same(it["positions"].numpy(), z[f"t{kt}_positions"])
        same(it["particle_type"].numpy(), z[f"t{kt}_particle_type"])
        assert int(it["n_particles_per_example"]) == int(z[f"t{kt}_n"])
        same(it["strains"].numpy(), z[f"t{kt}_strains"])
    info = D.get_dataset_info(str(path))
    ref_info = json.loads(str(z["info_json"]))
    got = {kk: (v if not isinstance(v, list) else [float(x) for x in v]) for kk, v in info.items()}
    assert got == ref_info
    np.testing.assert_array_equal(ds.denormalize_stress(z["denorm_in"]), z["denorm_out"])
