#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run here (the build container), never on the GPU box: it imports the
reference's own Python from /root/reference (`sgnn/single_scale/
learned_simulator.py`, `graph_network.py`, `evaluate.py`, `sgnn/noise_utils.py`)
and records inputs + outputs as .npz data.  Nothing of the reference's source
is stored; only arrays.

`torch_geometric` / `torch_cluster` are not installed, so
this script registers a small stand-in module that restates the two pieces of
PyG behaviour the reference uses:

* `MessagePassing.propagate` (PyG >= 2.3, flow='source_to_target'):
  `x_i = x.index_select(-2, edge_index[1])`, `x_j = x.index_select(-2,
  edge_index[0])`, message -> `zeros(N, H).scatter_add_(0, edge_index[1], m)`
  (aggr='add'), then `update(aggr_out, **kwargs)` receives the propagate
  keyword arguments it names (which is why the reference's edge latent
  doubles every layer, graph_network.py:176,222).
* `radius_graph(x, r, batch, loop, max_num_neighbors)` with torch_cluster's
  CUDA-kernel semantics: for each query i (ascending) scan candidates j of the
  same example in ascending index, keep ||x_j - x_i||^2 < r^2 (strict, fp32,
  dims summed in order), stop after max_num_neighbors; output rows
  `[neighbour j; query i]`.  **Truncation rule when the cap binds is the CUDA
  rule and is unverified against a real torch_cluster build** (none exists
  offline); uncapped cases are implementation-independent.

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import importlib.machinery
import inspect
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from sgnn_amd import synthetic  # noqa: E402  (input generation only)


# ----------------------------------------------------------------------------
# PyG / torch_cluster stand-in (restated semantics, see module docstring)
# ----------------------------------------------------------------------------
class _MessagePassing(torch.nn.Module):
    def __init__(self, aggr: str = "add", flow: str = "source_to_target", node_dim: int = -2):
        super().__init__()
        assert flow == "source_to_target"
        self.aggr = aggr
        self.node_dim = node_dim

    def propagate(self, edge_index, size=None, **kwargs):
        assert self.aggr == "add", "only aggr='add' is reached by the reference"
        msg_args = list(inspect.signature(self.message).parameters)
        coll = {}
        n_target = None
        for a in msg_args:
            if a.endswith("_i") or a.endswith("_j"):
                t = kwargs[a[:-2]]
                idx = edge_index[1] if a.endswith("_i") else edge_index[0]
                coll[a] = t.index_select(self.node_dim, idx)
                n_target = t.size(self.node_dim)
            else:
                coll[a] = kwargs[a]
        out = self.message(**coll)
        index = edge_index[1]
        agg = out.new_zeros((n_target,) + tuple(out.shape[1:]))
        agg.scatter_add_(0, index.view(-1, *([1] * (out.dim() - 1))).expand_as(out), out)
        upd_args = list(inspect.signature(self.update).parameters)[1:]
        return self.update(agg, **{a: kwargs[a] for a in upd_args})

    def message(self, x_j):  # pragma: no cover - overridden
        return x_j

    def update(self, inputs):  # pragma: no cover - overridden
        return inputs


def _radius_graph(x, r, batch=None, loop=False, max_num_neighbors=32, flow="source_to_target", **_):
    assert flow == "source_to_target"
    x = x.detach().to(torch.float32).cpu().numpy()
    n = x.shape[0]
    b = np.zeros(n, np.int64) if batch is None else batch.cpu().numpy()
    r2 = np.float32(r) * np.float32(r)
    cap = max_num_neighbors if loop else max_num_neighbors + 1
    rows, cols = [], []
    for i in range(n):
        cand = np.nonzero(b == b[i])[0]  # ascending index
        diff = x[cand] - x[i]
        d2 = np.zeros(len(cand), np.float32)
        for d in range(x.shape[1]):  # fp32, dims summed in order
            d2 = (d2 + diff[:, d] * diff[:, d]).astype(np.float32)
        hit = cand[d2 < r2][:cap]
        if not loop:
            hit = hit[hit != i]
        rows.extend(hit.tolist())
        cols.extend([i] * len(hit))
    return torch.tensor(np.stack([np.asarray(rows, np.int64), np.asarray(cols, np.int64)]))


def _module(name):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    return m


def _install_standins():
    pyg = _module("torch_geometric")
    pyg_nn = _module("torch_geometric.nn")
    pyg_nn.MessagePassing = _MessagePassing
    pyg_nn.radius_graph = _radius_graph
    pyg.nn = pyg_nn
    sys.modules["torch_geometric"] = pyg
    sys.modules["torch_geometric.nn"] = pyg_nn
    # evaluate.py imports these but never uses them (evaluate.py:4-7)
    for name in ("tree", "absl", "absl.flags", "absl.app"):
        sys.modules.setdefault(name, _module(name))
    sys.modules["absl"].flags = sys.modules["absl.flags"]
    sys.modules["absl"].app = sys.modules["absl.app"]
    # HF `datasets` shadows the reference's namespace package
    ds = _module("datasets")
    ds.__path__ = [os.path.join(REF, "datasets")]
    sys.modules["datasets"] = ds
    sys.path.insert(0, REF)


_install_standins()
from sgnn.single_scale import learned_simulator as ref_ls  # noqa: E402
from sgnn.single_scale import evaluate as ref_eval  # noqa: E402


# ----------------------------------------------------------------------------
def make_sim(dim, T, H, L, R, ntypes=1, emb=9, seed=0, stats=None):
    torch.manual_seed(seed)
    st = stats or synthetic.normalization_stats(dim)
    norm = {k: {kk: torch.tensor(vv) for kk, vv in v.items()} for k, v in st.items()}
    nnode_in = (T - 1) * dim + 1 + (emb if ntypes > 1 else 0)
    sim = ref_ls.LearnedSimulator(
        particle_dimensions=dim, nnode_in=nnode_in, nedge_in=dim + 1, latent_dim=H,
        nmessage_passing_steps=L, nmlp_layers=1, mlp_hidden_dim=H, connectivity_radius=R,
        normalization_stats=norm, nparticle_types=ntypes, particle_type_embedding_size=emb,
        device="cpu")
    return sim, st


def sd_arrays(sim, prefix="w/"):
    return {prefix + k: v.detach().cpu().numpy().astype(np.float32) for k, v in sim.state_dict().items()}


def hparams(dim, T, H, L, R, ntypes, emb):
    return {"hp_dim": np.int64(dim), "hp_T": np.int64(T), "hp_H": np.int64(H), "hp_L": np.int64(L),
            "hp_R": np.float32(R), "hp_ntypes": np.int64(ntypes), "hp_emb": np.int64(emb)}


def stats_arrays(st):
    return {"acc_mean": st["acceleration"]["mean"], "acc_std": st["acceleration"]["std"],
            "vel_mean": st["velocity"]["mean"], "vel_std": st["velocity"]["std"]}


def forward_case(name, pos_seq, npe, types_, dim, T, H, L, R, ntypes=1, emb=9, seed=0,
                 latents=False, rollout_frames=None):
    sim, st = make_sim(dim, T, H, L, R, ntypes, emb, seed)
    sim.eval()
    pos = torch.tensor(pos_seq[:, :T])
    pt = torch.tensor(types_, dtype=torch.long)
    out = {**hparams(dim, T, H, L, R, ntypes, emb), **stats_arrays(st), **sd_arrays(sim),
           "positions": pos_seq, "particle_types": types_.astype(np.int64),
           "nparticles_per_example": np.asarray(npe, np.int64)}
    with torch.no_grad():
        nf, ei, ef = sim._encoder_preprocessor(pos, torch.tensor(npe), pt)
        out["edge_index"] = ei.numpy()
        out["node_features"] = nf.numpy()
        out["edge_features"] = ef.numpy()
        epd = sim._encode_process_decode
        if latents:
            x, e = epd._encoder(nf, ef)
            out["lat_x_enc"], out["lat_e_enc"] = x.numpy(), e.numpy()
            for k, g in enumerate(epd._processor.gnn_stacks):
                x, e = g(x, ei, e)
                out[f"lat_x_{k}"] = x.numpy()
            out["lat_e_final"] = e.numpy()
        nxt, strain = sim.predict_positions(pos, torch.tensor(npe), pt)
        out["pred"] = epd(nf, ei, ef).numpy()
        out["next_position"] = nxt.numpy()
        out["strain"] = strain.numpy()
        if rollout_frames is not None:
            n = pos_seq.shape[0]
            strains = torch.zeros(pos_seq.shape[1], n)
            ro = ref_eval.rollout(sim, torch.tensor(pos_seq), pt, torch.tensor(n), strains,
                                  nsteps=pos_seq.shape[1] - T, particle_dim=dim, device="cpu",
                                  input_sequence_length=T)
            out["rollout_predicted"] = ro["predicted_rollout"]
            out["rollout_strain"] = ro["predicted_strain"]
            out["rollout_rmse_position"] = ro["rmse_position"]
            # teacher-forced rollout (evaluate.py:140-143): every step's window ends with ground truth
            ro1 = ref_eval.rollout(sim, torch.tensor(pos_seq), pt, torch.tensor(n), strains,
                                   nsteps=pos_seq.shape[1] - T, particle_dim=dim, device="cpu",
                                   input_sequence_length=T, inference_mode="one_step")
            out["onestep_predicted"] = ro1["predicted_rollout"]
            out["onestep_strain"] = ro1["predicted_strain"]
            out["onestep_rmse_position"] = ro1["rmse_position"]
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: N={pos_seq.shape[0]} E={out['edge_index'].shape[1]} -> {os.path.getsize(path)/1e3:.0f} KB")


def train_case(name, seed=0, ntypes=1, L=5):
    """One training step exactly as train.py:231-278 (noise passed in, lr_init=1e-3)."""
    dim, T, H, R = 2, 11, 64, 0.6
    noise_std = 0.02
    st = synthetic.normalization_stats(dim, noise_std=noise_std)
    sim, _ = make_sim(dim, T, H, L, R, ntypes=ntypes, seed=seed, stats=st)
    sim.train()
    a = synthetic.trajectory(synthetic.lattice_2d(10, 8), T + 1, seed=11)
    b = synthetic.trajectory(synthetic.lattice_2d(9, 8, x0=0.5, y0=-9.5), T + 1, seed=12)
    seq = np.concatenate([a, b], 0)
    npe = np.array([a.shape[0], b.shape[0]], np.int64)
    pos = torch.tensor(seq[:, :T])
    next_pos = torch.tensor(seq[:, T])
    next_strain = torch.tensor(np.random.default_rng(5).normal(0, 1, seq.shape[0]).astype(np.float32))
    types_ = torch.from_numpy(np.random.default_rng(seed + 7).integers(0, ntypes, seq.shape[0]))
    torch.manual_seed(123)
    noise = ref_noise.get_random_walk_noise_for_position_sequence(pos, noise_std_last_step=noise_std)
    init = sd_arrays(sim, "w0/")
    opt = torch.optim.Adam(sim.parameters(), lr=1e-3)
    pred_acc, target_acc, pred_strain = sim.predict_accelerations(
        next_positions=next_pos, position_sequence_noise=noise, position_sequence=pos,
        nparticles_per_example=torch.tensor(npe), particle_types=types_)
    loss_pos = ((pred_acc - target_acc) ** 2).sum(dim=-1)
    loss_strain = (pred_strain - next_strain) ** 2
    loss = (1.0 * loss_pos + 1.0 * loss_strain).mean()
    opt.zero_grad()
    loss.backward()
    grads = {"g/" + k: p.grad.detach().numpy().copy() for k, p in sim.named_parameters() if p.grad is not None}
    opt.step()
    out = {**hparams(dim, T, H, L, R, ntypes, 9), **stats_arrays(st), **init, **grads, **sd_arrays(sim, "w1/"),
           "positions": seq[:, :T], "next_position": seq[:, T], "next_strain": next_strain.numpy(),
           "noise": noise.numpy(), "nparticles_per_example": npe, "particle_types": types_.numpy(),
           "pred_acc": pred_acc.detach().numpy(), "target_acc": target_acc.detach().numpy(),
           "pred_strain": pred_strain.detach().numpy(), "loss": np.float32(loss.item()),
           "lr": np.float32(1e-3)}
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: loss={loss.item():.6f} -> {os.path.getsize(path)/1e3:.0f} KB")


from sgnn import noise_utils as ref_noise  # noqa: E402
from sgnn.multi_scale.multi_scale_graph import MultiScaleConfig as RefMSConfig  # noqa: E402
from sgnn.multi_scale.multi_scale_graph import MultiScaleGraph as RefMSGraph  # noqa: E402
from sgnn.multi_scale.multi_scale_simulator import MultiScaleSimulator as RefMSSim  # noqa: E402
from sgnn.multi_scale import multi_scale_evaluate as ref_ms_eval  # noqa: E402


def multi_scale_case(name, base, nframes, T, H, L, num_scales, window, mult, ntypes=1, emb=9,
                     nmlp=2, seed=0, traj_seed=0, rollout_steps=0):
    """MultiScaleSimulator forward (+ rollout) exactly as the reference runs it:
    static graph from the exact initial lattice (static_graph_data_loader.py:96-106),
    then predict_positions on the trajectory window (multi_scale_simulator.py:281-326)."""
    dim = base.shape[1]
    seq = synthetic.trajectory(base, nframes, seed=traj_seed)
    st = synthetic.normalization_stats(dim)
    norm = {k: {kk: torch.tensor(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(seed)
    nnode_in = (T - 1) * dim + 1 + (emb if ntypes > 1 else 0)
    sim = RefMSSim(kinematic_dimensions=dim, nnode_in=nnode_in, nedge_in=dim + 1, nedge_out=H,
                   latent_dim=H, nmessage_passing_steps=L, nmlp_layers=nmlp, normalization_stats=norm,
                   nparticle_types=ntypes, particle_type_embedding_size=emb, num_scales=num_scales,
                   window_size=window, radius_multiplier=mult, device="cpu")
    sim.eval()
    graph = RefMSGraph(RefMSConfig(num_scales=num_scales, window_size=window, radius_multiplier=mult)
                       ).create_all_edges(torch.tensor(seq[:, 0]))
    sim.set_static_graph(graph)
    types_ = np.random.default_rng(seed + 1).integers(0, ntypes, seq.shape[0]).astype(np.int64)
    pt = torch.tensor(types_)
    pos = torch.tensor(seq[:, :T])
    out = {"hp_dim": np.int64(dim), "hp_T": np.int64(T), "hp_H": np.int64(H), "hp_L": np.int64(L),
           "hp_ntypes": np.int64(ntypes), "hp_emb": np.int64(emb), "hp_nmlp": np.int64(nmlp),
           "hp_num_scales": np.int64(num_scales), "hp_window": np.int64(window),
           "hp_mult": np.float32(mult), **stats_arrays(st), **sd_arrays(sim),
           "positions": seq, "particle_types": types_,
           "g2m": graph["grid2mesh_edges"].numpy(), "m2m": graph["mesh2mesh_edges"].numpy(),
           "m2g": graph["mesh2grid_edges"].numpy()}
    for s_, d_ in graph["graph_hierarchy"].items():
        out[f"scale{s_}_indices"] = d_["sampling_indices"].numpy()
        out[f"scale{s_}_spacing"] = np.float32(d_["spacing"])
    with torch.no_grad():
        nf, ei, ef = sim._encoder_preprocessor(pos, torch.tensor([seq.shape[0]]), pt)
        out["node_features"] = nf.numpy()
        for k in ("g2m", "m2m", "m2g"):
            out[f"ef_{k}"] = ef[k].numpy()
        gnn = sim._multi_scale_gnn
        out["pred"] = gnn(nf, ei["g2m"], ef["g2m"], ei["m2m"], ef["m2m"], ei["m2g"], ef["m2g"],
                          graph["graph_hierarchy"]).numpy()
        nxt, strain = sim.predict_positions(pos, torch.tensor([seq.shape[0]]), pt)
        out["next_position"], out["strain"] = nxt.numpy(), strain.numpy()
        if rollout_steps:
            strains = torch.zeros(nframes, seq.shape[0])
            ro = ref_ms_eval.evaluate_multi_scale_rollout(
                sim, torch.tensor(seq), pt, torch.tensor([seq.shape[0]]), strains, nsteps=rollout_steps,
                dim=dim, device="cpu", input_sequence_length=T)
            out["rollout_predicted"] = ro["predicted_rollout"]
            out["rollout_strain"] = ro["predicted_strain"]
            out["rollout_rmse_position"] = ro["rmse_position"]
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: N={seq.shape[0]} g2m={out['g2m'].shape[1]} m2m={out['m2m'].shape[1]} "
          f"m2g={out['m2g'].shape[1]} -> {os.path.getsize(path)/1e3:.0f} KB")


def main(only=None):
    if only == "ms":
        return main_ms()
    if only == "train_types":
        return train_case("train2d_types", seed=2, ntypes=3, L=2)
    if only == "ms_train":
        return multi_scale_train_case("ms_train2d", synthetic.lattice_2d(16, 12, x0=-1.75), 6, 64, 2, 3, 2,
                                      2.0, seed=6)
    T = 11
    # 1) tiny 2D, reference default radius 0.6, per-layer latents + 3-step rollout (autoregressive and
    #    one_step)
    seq = synthetic.trajectory(synthetic.lattice_2d(10, 8), T + 3, seed=1)
    forward_case("tiny2d_r06", seq, [seq.shape[0]], np.zeros(seq.shape[0]), 2, T, 64, 5, 0.6,
                 latents=True, rollout_frames=3)
    if only == "tiny2d":
        return
    # 2) two examples overlapping in space: edges must never cross examples
    a = synthetic.trajectory(synthetic.lattice_2d(10, 8), T, seed=2)
    b = synthetic.trajectory(synthetic.lattice_2d(12, 6, x0=0.5, y0=-9.5), T, seed=3)
    seq = np.concatenate([a, b], 0)
    forward_case("batch2d_r06", seq, [a.shape[0], b.shape[0]], np.zeros(seq.shape[0]), 2, T, 64, 5, 0.6)
    # 3) C1 shape (50x40 = 2000 particles) at the BASELINE radius 15: cap of 20 binds
    seq = synthetic.trajectory(synthetic.lattice_2d(50, 40), T, seed=4)
    forward_case("c1_r15", seq, [seq.shape[0]], np.zeros(seq.shape[0]), 2, T, 64, 5, 15.0)
    # 4) C1 shape at the reference default radius 0.6
    forward_case("c1_r06", seq, [seq.shape[0]], np.zeros(seq.shape[0]), 2, T, 64, 5, 0.6)
    # 5) three particle types -> embedding concatenated to node features
    seq = synthetic.trajectory(synthetic.lattice_2d(10, 8), T, seed=6)
    types_ = np.random.default_rng(6).integers(0, 3, seq.shape[0])
    forward_case("types2d_r06", seq, [seq.shape[0]], types_, 2, T, 64, 2, 0.6, ntypes=3, emb=9)
    # 6) 3D, H=128 (C4 widths), shorter history, 3 layers to keep the fixture small
    seq = synthetic.trajectory(synthetic.lattice_3d(6, 5, 4), 6, seed=7)
    forward_case("tiny3d_h128", seq, [seq.shape[0]], np.zeros(seq.shape[0]), 3, 6, 128, 3, 0.75)
    # 7) one training step (loss, grads, Adam update)
    train_case("train2d_r06")
    # 8) training step with three particle types (embedding gradient)
    train_case("train2d_types", seed=2, ntypes=3, L=2)
    # 9-10) multi-scale cases
    main_ms()


def multi_scale_train_case(name, base, T, H, L, num_scales, window, mult, nmlp=2, seed=0):
    """One step of the multi_scale_train.py:140-186 loop body (noise passed in,
    lr_init 1e-3): loss, every gradient, Adam-updated weights."""
    dim = base.shape[1]
    noise_std = 0.02
    seq = synthetic.trajectory(base, T + 1, seed=seed + 20)
    st = synthetic.normalization_stats(dim, noise_std=noise_std)
    norm = {k: {kk: torch.tensor(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(seed)
    sim = RefMSSim(kinematic_dimensions=dim, nnode_in=(T - 1) * dim + 1, nedge_in=dim + 1, nedge_out=H,
                   latent_dim=H, nmessage_passing_steps=L, nmlp_layers=nmlp, normalization_stats=norm,
                   nparticle_types=1, particle_type_embedding_size=9, num_scales=num_scales,
                   window_size=window, radius_multiplier=mult, device="cpu")
    sim.train()
    graph = RefMSGraph(RefMSConfig(num_scales=num_scales, window_size=window, radius_multiplier=mult)
                       ).create_all_edges(torch.tensor(seq[:, 0]))
    sim.set_static_graph(graph)
    n = seq.shape[0]
    pos, next_pos = torch.tensor(seq[:, :T]), torch.tensor(seq[:, T])
    next_strain = torch.tensor(np.random.default_rng(seed + 5).normal(0, 1, n).astype(np.float32))
    types_ = torch.zeros(n, dtype=torch.long)
    torch.manual_seed(seed + 100)
    noise = ref_noise.get_random_walk_noise_for_position_sequence(pos, noise_std_last_step=noise_std)
    init = sd_arrays(sim, "w0/")
    opt = torch.optim.Adam(sim.parameters(), lr=1e-3)
    opt.zero_grad()
    pred_acc, target_acc, pred_strain = sim.predict_accelerations(
        next_positions=next_pos, position_sequence_noise=noise, position_sequence=pos,
        nparticles_per_example=torch.tensor([n]), particle_types=types_)
    loss_pos = ((pred_acc - target_acc) ** 2).sum(dim=-1)          # multi_scale_train.py:162-166
    loss_strain = (pred_strain - next_strain) ** 2                  # :169
    loss = (1.0 * loss_pos + 1.0 * loss_strain).mean()              # :172-173
    loss.backward()
    grads = {"g/" + k: p.grad.detach().numpy().copy() for k, p in sim.named_parameters() if p.grad is not None}
    opt.step()
    out = {"hp_dim": np.int64(dim), "hp_T": np.int64(T), "hp_H": np.int64(H), "hp_L": np.int64(L),
           "hp_ntypes": np.int64(1), "hp_emb": np.int64(9), "hp_nmlp": np.int64(nmlp),
           "hp_num_scales": np.int64(num_scales), "hp_window": np.int64(window), "hp_mult": np.float32(mult),
           **stats_arrays(st), **init, **grads, **sd_arrays(sim, "w1/"),
           "positions": seq, "next_position": seq[:, T], "next_strain": next_strain.numpy(),
           "noise": noise.numpy(), "particle_types": types_.numpy(),
           "pred_acc": pred_acc.detach().numpy(), "target_acc": target_acc.detach().numpy(),
           "pred_strain": pred_strain.detach().numpy(), "loss": np.float32(loss.item()),
           "lr": np.float32(1e-3),
           "g2m": graph["grid2mesh_edges"].numpy(), "m2m": graph["mesh2mesh_edges"].numpy(),
           "m2g": graph["mesh2grid_edges"].numpy()}
    for s_, d_ in graph["graph_hierarchy"].items():
        out[f"scale{s_}_indices"] = d_["sampling_indices"].numpy()
        out[f"scale{s_}_spacing"] = np.float32(d_["spacing"])
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: loss={loss.item():.6f} -> {os.path.getsize(path)/1e3:.0f} KB")


def main_ms():
    # multi-scale 2D: 3 scales (grid + 2 meshes), nmlp_layers 2, wall feature active
    # (x starts at -1.75 so x+2 spans the clamp range)
    multi_scale_case("ms2d_s3", synthetic.lattice_2d(20, 14, x0=-1.75), 9, 6, 64, 3, 3, 2, 2.0,
                     seed=3, traj_seed=8, rollout_steps=3)
    # multi-scale 3D, H=128 (config-5 widths), 2 scales, particle types (embedding);
    # 27 lattice neighbours inside r, so the max_neighbors=24 truncation binds
    multi_scale_case("ms3d_h128", synthetic.lattice_3d(8, 6, 5, x0=-1.75), 6, 6, 128, 2, 2, 2, 2.0,
                     ntypes=2, seed=4, traj_seed=9)
    # one multi-scale training step (2D, 3 scales, H=64, nmlp_layers 2)
    multi_scale_train_case("ms_train2d", synthetic.lattice_2d(16, 12, x0=-1.75), 6, 64, 2, 3, 2, 2.0, seed=6)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
