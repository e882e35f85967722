"""Drop-in `MultiScaleSimulator` (sgnn/multi_scale/multi_scale_simulator.py:20-388).

Same constructor, attributes, methods and state_dict keys as the reference;
one step runs as the fused HIP chain of `ms_engine` on the MI355X.  Inputs
must be CUDA tensors (no CPU path).  The static graph dict set by
`set_static_graph` may come from the reference's CPU builder or from
`build_static_multi_scale_graph` here; it is converted once per (graph,
device) into receiver-sorted CSR graphs by `sgnn_coo_to_csr`.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn as nn

from .. import engine, generic
from .._hip import require_gpu_tensor
from . import ms_engine
from .multi_scale_gnn import MultiScaleGNN
from .multi_scale_graph import MultiScaleConfig

_KEYS = {"g2m": "grid2mesh_edges", "m2m": "mesh2mesh_edges", "m2g": "mesh2grid_edges"}


class _TrainedGNN(torch.autograd.Function):
    """pred = MultiScaleGNN(features(noisy window)) with the HIP backward
    (multi_scale_train.py:176 loss.backward()).  One forward may be in flight
    per workspace: a second forward before backward invalidates the first."""

    @staticmethod
    def forward(ctx, sim, inp, tw, emb, *params):
        from . import ms_training
        ms_training.train_forward(sim._multi_scale_gnn, inp, tw, sim._grid_radius(), sim._mesh_radius(),
                                  emb_weight=emb)
        tw.generation = getattr(tw, "generation", 0) + 1
        ctx.sim, ctx.inp, ctx.tw, ctx.gen, ctx.emb = sim, inp, tw, tw.generation, emb
        return tw.pred.clone()

    @staticmethod
    def backward(ctx, dpred):
        from . import ms_training
        sim, tw = ctx.sim, ctx.tw
        if tw.generation != ctx.gen:
            raise RuntimeError("sgnn_amd: a newer predict_accelerations overwrote the saved "
                               "activations of this graph before backward")
        gnn = sim._multi_scale_gnn
        scratch = getattr(tw, "grad_scratch", None)
        if scratch is None:
            scratch = {k: torch.zeros_like(p) for k, p in gnn.named_parameters(prefix="_multi_scale_gnn")}
            tw.grad_scratch = scratch
        demb = torch.zeros_like(ctx.emb) if ctx.emb is not None else None
        ms_training.train_backward(gnn, ctx.inp, tw, scratch, sim._grid_radius(), sim._mesh_radius(),
                                   dpred=dpred.to(torch.float32).contiguous(), emb_weight=ctx.emb,
                                   emb_grad=demb)
        return (None, None, None, demb, *[g.clone() for g in scratch.values()])


class MultiScaleSimulator(nn.Module):
    """multi_scale_simulator.py:20-92"""

    def __init__(self, kinematic_dimensions: int, nnode_in: int, nedge_in: int, nedge_out: int,
                 latent_dim: int, nmessage_passing_steps: int, nmlp_layers: int,
                 normalization_stats: Dict, nparticle_types: int, particle_type_embedding_size: int,
                 num_scales: int = 3, window_size: int = 3, radius_multiplier: float = 2.0,
                 device: str = "cpu"):
        super().__init__()
        self._kinematic_dimensions = kinematic_dimensions
        self._normalization_stats = normalization_stats
        self._nparticle_types = nparticle_types
        self._num_scales = num_scales
        self._window_size = window_size
        self._device = device
        self._particle_type_embedding = nn.Embedding(nparticle_types, particle_type_embedding_size)
        self._multi_scale_config = MultiScaleConfig(num_scales=num_scales, window_size=window_size,
                                                    radius_multiplier=radius_multiplier)
        self._multi_scale_gnn = MultiScaleGNN(
            nnode_in_features=nnode_in, nnode_out_features=kinematic_dimensions + 1,
            nedge_in_features=nedge_in, nedge_out_features=nedge_out, latent_dim=latent_dim,
            nmessage_passing_steps=nmessage_passing_steps, nmlp_layers=nmlp_layers,
            num_scales=num_scales)
        self._static_graph_data = None
        self._csr_cache: Dict[tuple, Dict[str, engine.CsrGraph]] = {}
        self._ws_cache: Dict[tuple, ms_engine.MSWorkspace] = {}
        self._stats_cache: Dict[str, tuple] = {}

    def forward(self):
        """Forward hook runs on class instantiation (:94-96)."""
        pass

    # ------------------------------------------------------------ static graph
    def set_static_graph(self, graph_data: Dict[str, Any]):
        """:98-109"""
        self._static_graph_data = graph_data
        self._csr_cache.clear()
        self._ws_cache.clear()
        self.__dict__.get("_tw_cache", {}).clear()

    def _validate_static_graph(self):
        """:111-119"""
        if self._static_graph_data is None:
            raise ValueError("Static graph data not set. Call set_static_graph() first.")
        for key in ["graph_hierarchy", "grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"]:
            if key not in self._static_graph_data:
                raise ValueError(f"Missing required graph data key: {key}")

    def get_static_graph_data(self) -> Optional[Dict[str, Any]]:
        """:375-382"""
        return self._static_graph_data

    def _grid_radius(self) -> float:
        c = self._multi_scale_config
        return c.grid_spacing * c.radius_multiplier

    def _mesh_radius(self) -> float:
        """Coarsest mesh radius normalising m2m features (:226-233)."""
        c = self._multi_scale_config
        gh = self._static_graph_data["graph_hierarchy"]
        coarsest = c.num_scales - 1
        if coarsest in gh:
            return gh[coarsest]["spacing"] * c.radius_multiplier
        return self._grid_radius()

    def _csr(self, n: int, device) -> Dict[str, engine.CsrGraph]:
        self._validate_static_graph()
        key = (n, str(device))
        graphs = self._csr_cache.get(key)
        if graphs is None:
            graphs = {k: engine.coo_to_csr(torch.as_tensor(self._static_graph_data[v]).to(device), n)
                      for k, v in _KEYS.items()}
            self._csr_cache[key] = graphs
        return graphs

    # ----------------------------------------------------------------- helpers
    def _stats(self, device):
        key = str(device)
        st = self._stats_cache.get(key)
        if st is None:
            f = lambda v: torch.as_tensor(v, dtype=torch.float32).to(device).reshape(-1).contiguous()
            a, v = self._normalization_stats["acceleration"], self._normalization_stats["velocity"]
            st = (f(v["mean"]), f(v["std"]), f(a["mean"]), f(a["std"]))
            self._stats_cache[key] = st
        return st

    def _step_inputs(self, position_sequence, particle_types):
        require_gpu_tensor(position_sequence, "position_sequence")
        if position_sequence.dim() != 3 or position_sequence.shape[1] < 2:
            raise ValueError(f"Expected position_sequence (nparticles, T>=2, dim), got "
                             f"{tuple(position_sequence.shape)}")
        pos = position_sequence.to(torch.float32).contiguous()
        n, T, d = pos.shape
        if d != self._kinematic_dimensions:
            raise ValueError(f"positions have dim {d}, simulator has {self._kinematic_dimensions}")
        gnn = self._multi_scale_gnn
        use_emb = self._nparticle_types > 1
        feat = (T - 1) * d + 1 + (self._particle_type_embedding.embedding_dim if use_emb else 0)
        if feat != gnn.nnode_in:
            raise ValueError(f"position window gives {feat} node features, encoder expects {gnn.nnode_in}")
        if gnn.nedge_in != d + 1:
            raise ValueError(f"nedge_in must be dim + 1 = {d + 1}, got {gnn.nedge_in}")
        types = torch.as_tensor(particle_types).to(pos.device, torch.int64).contiguous() if use_emb else None
        vm, vs, am, as_ = self._stats(pos.device)
        return engine.StepInputs(pos, None, 1, types, vm, vs, am, as_), use_emb

    def _workspace(self, n: int, T: int, device, graphs) -> ms_engine.MSWorkspace:
        key = (n, T, str(device))
        ws = self._ws_cache.get(key)
        if ws is None:
            if len(self._ws_cache) > 4:
                self._ws_cache.clear()
            ws = ms_engine.MSWorkspace(n, T, self._kinematic_dimensions, self._multi_scale_gnn.latent_dim,
                                       graphs, device)
            self._ws_cache[key] = ws
        return ws

    def _fast_path(self) -> bool:
        """The fused MFMA chain implements this model's widths (else generic.py)."""
        return generic.ms_fast_shapes(self._multi_scale_gnn)

    def _run(self, position_sequence, particle_types, window_out=None):
        inp, use_emb = self._step_inputs(position_sequence, particle_types)
        n, T, d = inp.pos_seq.shape
        if not self._fast_path():   # e.g. nedge_out != latent_dim: block by block, width-generic path
            if window_out is not None:
                raise NotImplementedError("window_out needs the fused chain")
            pred = self._generic_pred(inp, use_emb)
            return inp, pred, self._decoder_postprocessor(pred[:, :d], inp.pos_seq)
        dev = inp.pos_seq.device
        graphs = self._csr(n, dev)
        ws = self._workspace(n, T, dev, graphs)
        pred = torch.empty(n, d + 1, dtype=torch.float32, device=dev)
        nxt = torch.empty(n, d, dtype=torch.float32, device=dev)
        ms_engine.forward_step(self._multi_scale_gnn, self._particle_type_embedding.weight, use_emb, inp,
                               graphs, self._grid_radius(), self._mesh_radius(), ws, pred, nxt,
                               window_out)
        return inp, pred, nxt

    def _generic_pred(self, inp: engine.StepInputs, use_emb: bool) -> torch.Tensor:
        """MultiScaleGNN(features) on the differentiable width-generic path
        (sgnn_amd.autograd): node features from sgnn_node_features (wall
        clamp(x + 2, 0, R_g) / R_g, :190-193) with the type embedding as a
        differentiable gather, edge features of the three static graphs in their
        receiver-CSR order (sgnn_edge_features; g2m / m2g over R_g, m2m over the
        coarsest mesh radius, :206-250), then block by block."""
        from .. import autograd
        pos = inp.pos_seq
        n, T, d = pos.shape
        dev = pos.device
        graphs = self._csr(n, dev)
        key = (n, str(dev), "autograd")
        egs = self._csr_cache.get(key)
        if egs is None:
            egs = {k: autograd.EdgeGraph(torch.stack([g.send[:g.num_edges], g.recv[:g.num_edges]]), n)
                   for k, g in graphs.items()}
            self._csr_cache[key] = egs
        rg, rm = self._grid_radius(), self._mesh_radius()
        nf = autograd.node_features(pos, inp.types, self._particle_type_embedding.weight, use_emb, inp.vel_mean,
                                    inp.vel_std, rg, rg, self._nparticle_types)
        ef = {k: generic.edge_features(graphs[k], pos, (T - 1) * d, T * d, d, r)
              for k, r in (("g2m", rg), ("m2m", rm), ("m2g", rg))}
        return autograd.ms_gnn_forward(self._multi_scale_gnn, nf, None, ef["g2m"], None, ef["m2m"], None, ef["m2g"],
                                       graphs=egs)

    def rollout_runner(self, window: torch.Tensor, particle_types, nsteps: int):
        """Device-resident rollout of `nsteps` predict_positions steps from
        `window` (multi_scale_evaluate.py:163-214): every step's prediction is
        written by the decoder kernel straight into its output slot and the
        window shifts on the device, so the loop never waits for the host."""
        inp, _ = self._step_inputs(window, particle_types)
        return _MSRollout(self, inp.pos_seq, particle_types, nsteps)

    # ------------------------------------------------------------ reference API
    def _time_diff(self, position_sequence: torch.Tensor) -> torch.Tensor:
        """:384-388"""
        return (position_sequence[:, 1:] - position_sequence[:, :-1]).contiguous()

    def _encoder_preprocessor(self, position_sequence, nparticles_per_example, particle_types):
        """:121-167 materialised (API parity / debugging only: predict_* compute
        the features inside the encoder kernels)."""
        self._validate_static_graph()
        inp, use_emb = self._step_inputs(position_sequence, particle_types)
        pos = inp.pos_seq
        n = pos.shape[0]
        recent = pos[:, -1].contiguous()
        nf = self._build_node_features(self._time_diff(pos), recent, inp.types, n)
        idx = {k: torch.as_tensor(self._static_graph_data[v]).to(pos.device) for k, v in _KEYS.items()}
        ef = self._build_edge_features(idx["g2m"], idx["m2m"], idx["m2g"], recent)
        return nf, idx, ef

    def _build_node_features(self, velocity_sequence, most_recent_position, particle_types, nparticles):
        """:169-204"""
        vs = self._normalization_stats["velocity"]
        mean = torch.as_tensor(vs["mean"]).to(velocity_sequence.device)
        std = torch.as_tensor(vs["std"]).to(velocity_sequence.device)
        feats = [((velocity_sequence - mean) / std).contiguous().reshape(nparticles, -1)]
        rg = self._grid_radius()
        feats.append(torch.clamp(most_recent_position[:, 0:1] + 2.0, min=0.0, max=rg) / rg)
        if self._nparticle_types > 1:
            feats.append(self._particle_type_embedding(particle_types))
        return torch.cat(feats, dim=-1)

    def _build_edge_features(self, g2m_edge_index, m2m_edge_index, m2g_edge_index, most_recent_position):
        """:206-250"""
        def one(ei, r):
            if ei.shape[1] == 0:
                return torch.empty((0, 3), device=most_recent_position.device)
            disp = (most_recent_position[ei[0], :] - most_recent_position[ei[1], :]) / r
            return torch.cat([disp, torch.norm(disp, dim=-1, keepdim=True)], dim=-1)
        rg, rm = self._grid_radius(), self._mesh_radius()
        return {"g2m": one(g2m_edge_index, rg), "m2m": one(m2m_edge_index, rm),
                "m2g": one(m2g_edge_index, rg)}

    def _decoder_postprocessor(self, normalized_acceleration, position_sequence):
        """:253-279"""
        st = self._normalization_stats["acceleration"]
        dev = normalized_acceleration.device
        acc = normalized_acceleration * torch.as_tensor(st["std"]).to(dev) + torch.as_tensor(st["mean"]).to(dev)
        recent = position_sequence[:, -1]
        return recent + ((recent - position_sequence[:, -2]) + acc)

    def predict_positions(self, current_positions: torch.Tensor, nparticles_per_example,
                          particle_types: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """:281-326 -> (next_positions [N, d], predicted_strain [N])."""
        _, pred, nxt = self._run(current_positions, particle_types)
        return nxt, pred[:, -1]

    def predict_accelerations(self, next_positions: torch.Tensor, position_sequence_noise: torch.Tensor,
                              position_sequence: torch.Tensor, nparticles_per_example,
                              particle_types: torch.Tensor):
        """:328-360 -> (predicted_normalized_acceleration, target_normalized_acceleration,
        predicted_strain)."""
        noisy = position_sequence + position_sequence_noise
        params = list(self._multi_scale_gnn.parameters())
        d = self._kinematic_dimensions
        from . import ms_training
        need_grad = torch.is_grad_enabled() and (any(p.requires_grad for p in params) or (
            self._nparticle_types > 1 and self._particle_type_embedding.weight.requires_grad))
        if need_grad and not ms_training.fused_trainable(self):   # differentiable width-generic path
            inp, use_emb = self._step_inputs(noisy, particle_types)
            pred = self._generic_pred(inp, use_emb)
        elif need_grad:
            inp, _ = self._step_inputs(noisy, particle_types)
            n, T, _ = inp.pos_seq.shape
            tw = self._train_workspace(n, T, inp.pos_seq.device)
            emb = self._particle_type_embedding.weight if self._nparticle_types > 1 else None
            pred = _TrainedGNN.apply(self, inp, tw, emb, *params)
        else:
            inp, pred, _ = self._run(noisy, particle_types)
        target = self._inverse_decoder_postprocessor(next_positions + position_sequence_noise[:, -1],
                                                     inp.pos_seq)
        return pred[:, :d], target, pred[:, -1]

    def _train_workspace(self, n: int, T: int, device):
        from . import ms_training
        graphs = self._csr(n, device)
        cache = self.__dict__.setdefault("_tw_cache", {})
        key = (n, T, str(device), id(graphs))
        tw = cache.get(key)
        if tw is None:
            cache.clear()
            tw = ms_training.MSTrainWorkspace(self._multi_scale_gnn, n, T, self._kinematic_dimensions, graphs,
                                              device)
            cache[key] = tw
        return tw

    def _inverse_decoder_postprocessor(self, next_position, position_sequence):
        """:362-373"""
        prev = position_sequence[:, -1]
        acc = (next_position - prev) - (prev - position_sequence[:, -2])
        st = self._normalization_stats["acceleration"]
        mean = torch.as_tensor(st["mean"]).to(acc.device)
        std = torch.as_tensor(st["std"]).to(acc.device)
        return (acc - mean) / std

    def save(self, path: str = "multi_scale_model.pt"):
        """:362-368"""
        torch.save(self.state_dict(), path)

    def load(self, path: str):
        """:370-376 (weights_only: never unpickles code)."""
        self.load_state_dict(torch.load(path, map_location=torch.device("cpu"), weights_only=True))


class _MSRollout:
    """Autoregressive / one-step rollout buffers for MultiScaleSimulator
    (two ping-pong windows, [nsteps, n, d] positions, [nsteps, n, d+1] raw
    predictions).  No .item()/.cpu() inside the loop."""

    def __init__(self, sim, window: torch.Tensor, particle_types, nsteps: int):
        self.sim, self.types, self.nsteps = sim, particle_types, nsteps
        n, T, d = window.shape
        dev = window.device
        self.win = [window.to(torch.float32).contiguous().clone(), torch.empty(n, T, d, device=dev)]
        self.out_pos = torch.empty(max(nsteps, 1), n, d, dtype=torch.float32, device=dev)
        self.out_pred = torch.empty(max(nsteps, 1), n, d + 1, dtype=torch.float32, device=dev)

    def run(self, window: torch.Tensor = None, ground_truth: torch.Tensor = None):
        """ground_truth [n, >= nsteps, d] switches to one_step mode: the window
        is shifted with the true next position instead of the prediction
        (multi_scale_evaluate.py:203-214).  Returns (positions [nsteps, n, d],
        strain [nsteps, n]) on the device."""
        sim = self.sim
        if window is not None:
            self.win[0].copy_(window)
        n, T, d = self.win[0].shape
        dev = self.win[0].device
        gnn = sim._multi_scale_gnn
        if not sim._fast_path():   # widths the fused chain is not built for: step by step
            cur = self.win[0]
            for k in range(self.nsteps):
                _, pred, nxt_pos = sim._run(cur, self.types)
                self.out_pred[k].copy_(pred)
                self.out_pos[k].copy_(nxt_pos)
                src = nxt_pos if ground_truth is None else ground_truth[:, k]
                cur = torch.cat([cur[:, 1:], src[:, None, :]], dim=1)
            return self.out_pos[:self.nsteps], self.out_pred[:self.nsteps, :, -1]
        graphs = sim._csr(n, dev)
        ws = sim._workspace(n, T, dev, graphs)
        cur, nxt = self.win
        for k in range(self.nsteps):
            inp, use_emb = sim._step_inputs(cur, self.types)
            ms_engine.forward_step(gnn, sim._particle_type_embedding.weight, use_emb, inp, graphs,
                                   sim._grid_radius(), sim._mesh_radius(), ws, self.out_pred[k],
                                   self.out_pos[k], nxt if ground_truth is None else None)
            if ground_truth is not None:
                nxt[:, :-1].copy_(cur[:, 1:])
                nxt[:, -1].copy_(ground_truth[:, k])
            cur, nxt = nxt, cur
        return self.out_pos[:self.nsteps], self.out_pred[:self.nsteps, :, -1]
