"""Multi-scale datasets / collate on CPU.

The GPU graph builder needs a device, so here the datasets take the oracle's
graph builder (test infrastructure) through `graph_builder`; the GPU builder
itself is pinned bit-exactly against the same oracle in
tests/test_gpu_multi_scale.py / test_gpu_configs.py.

* default collate = the reference's behaviour (static_graph_data_loader.py:
  228-229): the whole batch carries sample 0's graph;
* per_sample_graphs=True: the block-diagonal union -- each sample's edges and
  hierarchy restricted to its node range equal its own graph, nothing crosses
  samples, and the multi-scale oracle run on the merged batch equals the
  oracle run on every sample alone (while the reference's collate gives the
  second sample the wrong neighbourhoods).
"""
import json

import numpy as np
import torch

from oracle import multi_scale_oracle as MO
from sgnn_amd import data as D
from sgnn_amd import synthetic
from sgnn_amd.multi_scale import static_graph_data_loader as S

NS, WIN, MULT = 2, 2, 2.0


def _builder(pos, num_scales, window_size, radius_multiplier):
    return MO.create_all_edges(pos, num_scales, window_size, radius_multiplier)


def _split(tmp_path):
    trajs = {}
    for k, (nx, ny, x0) in enumerate([(10, 8, -1.75), (12, 6, -1.25)]):
        seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny, x0=x0), 10, seed=20 + k)   # [N, T, 2]
        pos = np.transpose(seq, (1, 0, 2)).copy()
        trajs[f"t{k}"] = (pos, np.zeros(pos.shape[1], np.int64), np.zeros(pos.shape[:2]))
    path = tmp_path / "train.npz"
    D.save_trajectories(str(path), trajs, reference_format=True)
    (tmp_path / "metadata.json").write_text(json.dumps({"stress_mean": 0.0, "stress_std": 1.0}))
    return str(path), trajs


def test_default_collate_is_the_references_and_merge_is_block_diagonal(tmp_path):
    path, trajs = _split(tmp_path)
    ds = S.MultiScaleTaylorImpactSamplesDataset(path, input_length_sequence=6, num_scales=NS, window_size=WIN,
                                                radius_multiplier=MULT, graph_builder=_builder)
    a, b = ds[0], ds[len(ds) - 1]            # first sample of trajectory 0, last of trajectory 1
    assert int(a["meta"]["trajectory_idx"]) == 0 and int(b["meta"]["trajectory_idx"]) == 1
    ref = S.multi_scale_collate_fn([a, b])
    assert ref["graph"] is a["graph"]        # static_graph_data_loader.py:228-229
    m = S.multi_scale_collate_fn([a, b], per_sample_graphs=True)["graph"]
    na, nb = a["input"]["n_particles_per_example"], b["input"]["n_particles_per_example"]
    for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
        e = m[key]
        in_a = (e < na).all(0)
        in_b = (e >= na).all(0)
        assert bool((in_a | in_b).all()), f"{key}: an edge crosses samples"
        np.testing.assert_array_equal(e[:, in_a].numpy(), a["graph"][key].numpy())
        np.testing.assert_array_equal((e[:, in_b] - na).numpy(), b["graph"][key].numpy())
    for s in range(NS):
        h, ha, hb = m["graph_hierarchy"][s], a["graph"]["graph_hierarchy"][s], b["graph"]["graph_hierarchy"][s]
        np.testing.assert_array_equal(h["sampling_indices"].numpy(),
                                      np.concatenate([ha["sampling_indices"].numpy(),
                                                      hb["sampling_indices"].numpy() + na]))
        assert h["num_particles"] == ha["num_particles"] + hb["num_particles"]
        assert h["spacing"] == ha["spacing"]
    assert na + nb == m["graph_hierarchy"][0]["num_particles"]


def test_merged_batch_equals_per_sample_oracle(tmp_path):
    """The oracle (CPU restatement of sgnn/multi_scale) on the collated batch
    with the merged graph reproduces each sample run alone; with the
    reference's sample-0 graph it does not."""
    from sgnn_amd.multi_scale import MultiScaleSimulator
    path, _ = _split(tmp_path)
    ds = S.MultiScaleTaylorImpactSamplesDataset(path, input_length_sequence=6, num_scales=NS, window_size=WIN,
                                                radius_multiplier=MULT, graph_builder=_builder)
    items = [ds[0], ds[len(ds) - 1]]
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(3)
    sim = MultiScaleSimulator(2, 5 * 2 + 1, 3, 32, 32, 2, 2, stats, 1, 9, NS, WIN, MULT)
    state = {k: v.detach() for k, v in sim.state_dict().items()}

    def run(graph, pos):
        with torch.no_grad():
            return MO.MultiScaleOracle(state, 2, 2, stats, graph, NS, MULT, 1, 2).predict_positions(pos)

    alone = [run(it["graph"], torch.from_numpy(it["input"]["positions"])) for it in items]
    merged = S.multi_scale_collate_fn(items, per_sample_graphs=True)
    nxt, strain = run(merged["graph"], merged["input"]["positions"])
    np.testing.assert_allclose(nxt.numpy(), torch.cat([a[0] for a in alone]).numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(strain.numpy(), torch.cat([a[1] for a in alone]).numpy(), rtol=0, atol=1e-4)
    ref = S.multi_scale_collate_fn(items)
    n0 = items[0]["input"]["n_particles_per_example"]
    assert ref["graph"]["graph_hierarchy"][0]["num_particles"] == n0 < ref["input"]["positions"].shape[0]


def test_trajectories_dataset_and_loaders(tmp_path):
    path, trajs = _split(tmp_path)
    tds = S.MultiScaleTaylorImpactTrajectoriesDataset(path, num_scales=NS, window_size=WIN, radius_multiplier=MULT,
                                                      graph_builder=_builder)
    assert len(tds) == 2
    g1 = tds[1]["graph"]
    ref = _builder(torch.tensor(trajs["t1"][0][0], dtype=torch.float32), NS, WIN, MULT)
    for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
        np.testing.assert_array_equal(g1[key].numpy(), ref[key].numpy())
    dl = S.get_multi_scale_data_loader_by_samples(path, input_length_sequence=6, batch_size=3, shuffle=False,
                                                  pin_memory=False, num_scales=NS, window_size=WIN,
                                                  radius_multiplier=MULT, per_sample_graphs=True,
                                                  graph_builder=_builder)
    for batch in dl:
        n = batch["input"]["positions"].shape[0]
        assert batch["graph"]["graph_hierarchy"][0]["num_particles"] == n
        assert int(batch["graph"]["grid2mesh_edges"].max()) < n
