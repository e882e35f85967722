"""Drop-in `LearnedSimulator` (sgnn/single_scale/learned_simulator.py:9-550).

Same constructor, attribute names, methods, exceptions and state_dict keys as
the reference; the arithmetic runs in libsgnn_hip.so on the MI355X.  Inputs
must be CUDA tensors: there is no CPU path.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn

from . import engine, generic, graph_network, training
from ._hip import require_gpu_tensor


class _TrainedEPD(torch.autograd.Function):
    """pred = EncodeProcessDecode(features(noisy window)) with a HIP backward
    (graph_network.py:388-406 under autograd).  One forward may be in flight
    per workspace: a second forward before backward invalidates the first."""

    @staticmethod
    def forward(ctx, sim, inp, tw, emb, *params):
        training.train_forward(sim._encode_process_decode, sim._connectivity_radius, inp, tw, emb_weight=emb)
        tw.generation = getattr(tw, "generation", 0) + 1
        ctx.sim, ctx.inp, ctx.tw, ctx.gen, ctx.emb = sim, inp, tw, tw.generation, emb
        return tw.pred[:tw.n].clone()

    @staticmethod
    def backward(ctx, dpred):
        sim, tw = ctx.sim, ctx.tw
        if tw.generation != ctx.gen:
            raise RuntimeError("sgnn_amd: a newer predict_accelerations overwrote the saved "
                               "activations of this graph before backward")
        epd = sim._encode_process_decode
        scratch = getattr(tw, "grad_scratch", None)
        if scratch is None:
            scratch = {k: torch.zeros_like(p) for k, p in epd.named_parameters(prefix="_encode_process_decode")}
            tw.grad_scratch = scratch
        demb = None
        if ctx.emb is not None:
            demb = getattr(tw, "emb_grad_scratch", None)
            if demb is None or demb.shape != ctx.emb.shape:
                demb = torch.zeros_like(ctx.emb)
                tw.emb_grad_scratch = demb
        training.train_backward(epd, sim._connectivity_radius, ctx.inp, tw, scratch,
                                dpred=dpred.to(torch.float32).contiguous(), emb_weight=ctx.emb, emb_grad=demb)
        return (None, None, None, demb.clone() if demb is not None else None,
                *[g.clone() for g in scratch.values()])


class LearnedSimulator(nn.Module):
    """Learned simulator from https://arxiv.org/pdf/2002.09405.pdf
    (learned_simulator.py:9-64)."""

    def __init__(self, particle_dimensions: int, nnode_in: int, nedge_in: int, latent_dim: int,
                 nmessage_passing_steps: int, nmlp_layers: int, mlp_hidden_dim: int,
                 connectivity_radius: float, normalization_stats: Dict, nparticle_types: int,
                 particle_type_embedding_size, device="cpu"):
        super().__init__()
        self._connectivity_radius = connectivity_radius
        self._normalization_stats = normalization_stats
        self._nparticle_types = nparticle_types
        self._particle_dimensions = particle_dimensions
        self._particle_type_embedding = nn.Embedding(nparticle_types, particle_type_embedding_size)
        self._encode_process_decode = graph_network.EncodeProcessDecode(
            nnode_in_features=nnode_in, nnode_out_features=particle_dimensions + 1,
            nedge_in_features=nedge_in, latent_dim=latent_dim,
            nmessage_passing_steps=nmessage_passing_steps, nmlp_layers=nmlp_layers,
            mlp_hidden_dim=mlp_hidden_dim)
        self._device = device
        self._max_num_neighbors = engine.MAX_NUM_NEIGHBORS
        self._ws_cache: Dict[tuple, engine.StepWorkspace] = {}
        self._ptr_cache: Dict[tuple, torch.Tensor] = {}
        self._stats_cache: Dict[tuple, tuple] = {}

    def forward(self):
        """Forward hook runs on class instantiation (a no-op, :66-68)."""
        pass

    # ------------------------------------------------------------------ helpers
    def _workspace(self, n: int, T: int, device, loop: bool = True) -> engine.StepWorkspace:
        key = (n, T, str(device), loop)
        ws = self._ws_cache.get(key)
        if ws is None:
            if len(self._ws_cache) > 8:
                self._ws_cache.clear()
            ws = engine.StepWorkspace(n, T, self._particle_dimensions,
                                      self._encode_process_decode.latent_dim,
                                      self._max_num_neighbors, loop, device)
            self._ws_cache[key] = ws
        return ws

    def _ex_ptr(self, nparticles_per_example, n: int, device) -> Tuple[torch.Tensor, int]:
        counts = engine.counts_of(nparticles_per_example)
        if sum(counts) != n:  # learned_simulator.py:97-101 warns, the search then fails
            raise ValueError(f"Total particles mismatch: {sum(counts)} vs {n}")
        key = (tuple(counts), str(device))
        t = self._ptr_cache.get(key)
        if t is None:
            if len(self._ptr_cache) > 64:
                self._ptr_cache.clear()
            t = engine.ex_ptr_tensor(counts, device)
            self._ptr_cache[key] = t
        return t, len(counts)

    def _stats(self, device):
        key = str(device)
        st = self._stats_cache.get(key)
        if st is None:
            f = lambda v: torch.as_tensor(v, dtype=torch.float32).to(device).reshape(-1).contiguous()
            a, v = self._normalization_stats["acceleration"], self._normalization_stats["velocity"]
            st = (f(v["mean"]), f(v["std"]), f(a["mean"]), f(a["std"]))
            self._stats_cache[key] = st
        return st

    def _step_inputs(self, position_sequence, nparticles_per_example, particle_types):
        if len(position_sequence.shape) != 3:  # :251-254
            raise ValueError(f"Expected position_sequence to have 3 dimensions, got {len(position_sequence.shape)}")
        if position_sequence.shape[1] < 2:
            raise ValueError(f"Expected at least 2 timesteps, got {position_sequence.shape[1]}")
        require_gpu_tensor(position_sequence, "position_sequence")
        pos = position_sequence.to(torch.float32).contiguous()
        n, T, d = pos.shape
        if d != self._particle_dimensions:
            raise ValueError(f"positions have dim {d}, simulator has {self._particle_dimensions}")
        use_emb = self._nparticle_types > 1
        feat = (T - 1) * d + 1 + (self._particle_type_embedding.embedding_dim if use_emb else 0)
        if feat != self._encode_process_decode.nnode_in:
            raise ValueError(f"position window gives {feat} node features, encoder expects "
                             f"{self._encode_process_decode.nnode_in}")
        ex_ptr, n_ex = self._ex_ptr(nparticles_per_example, n, pos.device)
        types = None
        if use_emb:
            types = torch.as_tensor(particle_types).to(pos.device, torch.int64).contiguous()
        vm, vs, am, as_ = self._stats(pos.device)
        return engine.StepInputs(pos, ex_ptr, n_ex, types, vm, vs, am, as_), use_emb

    # ------------------------------------------------------------ reference API
    def _compute_graph_connectivity(self, positions: torch.Tensor, nparticles_per_example,
                                    radius: float, add_self_edges: bool = True):
        """learned_simulator.py:70-124 -> (edge_index[0], edge_index[1]) under the
        reference's names (receivers, senders); the caller swaps them (:261)."""
        if len(positions.shape) != 2:
            raise ValueError(f"Expected 2D positions tensor, got shape {positions.shape}")
        require_gpu_tensor(positions, "positions")
        pos = positions.to(torch.float32).contiguous()
        n, d = pos.shape
        ex_ptr, n_ex = self._ex_ptr(nparticles_per_example, n, pos.device)
        ws = engine.StepWorkspace(n, 2, d, self._encode_process_decode.latent_dim,
                                  self._max_num_neighbors, add_self_edges, pos.device)
        engine.radius_graph(ws, pos, 0, d, ex_ptr, n_ex, radius)
        e = ws.num_edges()
        return ws.send[:e].to(torch.int64), ws.recv[:e].to(torch.int64)

    def _encoder_preprocessor(self, position_sequence, nparticles_per_example, particle_types):
        """learned_simulator.py:231-316 materialised (API parity / debugging only:
        predict_* never build these tensors; the encoder kernels compute the
        features on the fly)."""
        inp, use_emb = self._step_inputs(position_sequence, nparticles_per_example, particle_types)
        pos = inp.pos_seq
        most_recent = pos[:, -1]
        senders, receivers = self._compute_graph_connectivity(
            most_recent, nparticles_per_example, self._connectivity_radius)
        vel = time_diff(pos)
        feats = [((vel - inp.vel_mean) / inp.vel_std).reshape(pos.shape[0], -1),
                 torch.clamp(most_recent[:, 0:1] + 2.0, min=0.0, max=self._connectivity_radius)]
        if use_emb:
            feats.append(self._particle_type_embedding(inp.types))
        disp = (most_recent[senders, :] - most_recent[receivers, :]) / self._connectivity_radius
        dist = torch.norm(disp, dim=-1, keepdim=True)
        return torch.cat(feats, -1), torch.stack([senders, receivers]), torch.cat([disp, dist], -1)

    def _decoder_postprocessor(self, normalized_acceleration, position_sequence):
        """learned_simulator.py:381-411 (used only on materialised tensors)."""
        st = self._normalization_stats["acceleration"]
        dev = normalized_acceleration.device
        acc = normalized_acceleration * torch.as_tensor(st["std"]).to(dev) + torch.as_tensor(st["mean"]).to(dev)
        most_recent = position_sequence[:, -1]
        return most_recent + ((most_recent - position_sequence[:, -2]) + acc)

    def predict_positions(self, current_positions: torch.Tensor, nparticles_per_example,
                          particle_types: torch.Tensor):
        """learned_simulator.py:413-438 -> (next_positions [N,d], predicted_strain [N])."""
        inp, use_emb = self._step_inputs(current_positions, nparticles_per_example, particle_types)
        n, T, d = inp.pos_seq.shape
        if not self._fast_path():   # widths the fused kernels are not built for
            pred = generic.predict_step(self, inp, use_emb)
            return self._decoder_postprocessor(pred[:, :d], inp.pos_seq), pred[:, -1]
        ws = self._workspace(n, T, inp.pos_seq.device)
        pred = torch.empty(n, d + 1, dtype=torch.float32, device=inp.pos_seq.device)
        next_pos = torch.empty(n, d, dtype=torch.float32, device=inp.pos_seq.device)
        engine.forward_step(self._encode_process_decode, self._particle_type_embedding.weight, use_emb,
                            self._connectivity_radius, inp, ws, pred, next_pos)
        return next_pos, pred[:, -1]

    def _fast_path(self) -> bool:
        """The fused MFMA kernels implement this model's widths (else generic.py)."""
        return generic.fast_shapes(self._encode_process_decode)

    def rollout_runner(self, window: torch.Tensor, nparticles_per_example, particle_types, nsteps: int):
        """Device-resident autoregressive rollout of `nsteps` predict_positions
        steps from `window` (evaluate.py:117-145): one sgnn_rollout call."""
        if not self._fast_path():
            raise NotImplementedError("the device rollout needs the fused kernels' widths (hidden = latent "
                                      "in {64, 128}); evaluate.rollout steps predict_positions instead")
        inp, use_emb = self._step_inputs(window, nparticles_per_example, particle_types)
        n, T, d = inp.pos_seq.shape
        ws = self._workspace(n, T, inp.pos_seq.device)
        pk = engine.ParamPack.get(self._encode_process_decode)
        sin = engine.step_in(inp, ws, self._connectivity_radius, self._particle_type_embedding.weight, use_emb)
        return engine.DeviceRollout(pk.epd, sin, ws, inp.pos_seq, n, d, nsteps, keep=(pk, inp))

    def predict_accelerations(self, next_positions: torch.Tensor, position_sequence_noise: torch.Tensor,
                              position_sequence: torch.Tensor, nparticles_per_example,
                              particle_types: torch.Tensor):
        """learned_simulator.py:440-491 -> (predicted_normalized_acceleration,
        target_normalized_acceleration, predicted_strain); differentiable with
        respect to the EncodeProcessDecode parameters and the type embedding: the
        fused HIP backward at the widths it is built for, the width-generic
        autograd path (sgnn_amd.autograd) at every other shape."""
        noisy = position_sequence + position_sequence_noise
        epd = self._encode_process_decode
        params = list(epd.parameters())
        need_grad = torch.is_grad_enabled() and (any(p.requires_grad for p in params) or (
            self._nparticle_types > 1 and self._particle_type_embedding.weight.requires_grad))
        inp, use_emb = self._step_inputs(noisy, nparticles_per_example, particle_types)
        n, T, d = inp.pos_seq.shape
        if need_grad and training.fused_trainable(epd, self._nparticle_types):
            tw = self._train_workspace(n, T, inp.pos_seq.device)
            emb = self._particle_type_embedding.weight if use_emb else None
            pred = _TrainedEPD.apply(self, inp, tw, emb, *params)
        elif need_grad or not self._fast_path():   # differentiable width-generic path (any widths / depth)
            pred = generic.predict_step(self, inp, use_emb)
        else:
            ws = self._workspace(n, T, inp.pos_seq.device)
            pred = torch.empty(n, d + 1, dtype=torch.float32, device=inp.pos_seq.device)
            nxt = torch.empty(n, d, dtype=torch.float32, device=inp.pos_seq.device)
            engine.forward_step(epd, self._particle_type_embedding.weight, use_emb,
                                self._connectivity_radius, inp, ws, pred, nxt)
        next_position_adjusted = next_positions + position_sequence_noise[:, -1]
        target = self._inverse_decoder_postprocessor(next_position_adjusted, inp.pos_seq)
        return pred[:, :d], target, pred[:, -1]

    def _train_workspace(self, n: int, T: int, device) -> training.TrainWorkspace:
        cache = self.__dict__.setdefault("_tw_cache", {})
        cap = training.capacity(n)
        key = (cap, T, str(device))
        tw = cache.get(key)
        if tw is None:
            if len(cache) > 4:
                cache.clear()
            tw = training.TrainWorkspace(self._encode_process_decode, cap, T, self._particle_dimensions,
                                         self._max_num_neighbors, True, device)
            cache[key] = tw
        return tw.activate(n)

    def _inverse_decoder_postprocessor(self, next_position, position_sequence):
        """learned_simulator.py:493-517"""
        prev = position_sequence[:, -1]
        prev_vel = prev - position_sequence[:, -2]
        acc = (next_position - prev) - prev_vel
        st = self._normalization_stats["acceleration"]
        mean = torch.as_tensor(st["mean"]).to(acc.device)
        std = torch.as_tensor(st["std"]).to(acc.device)
        return (acc - mean) / std

    def save(self, path: str = "model.pt"):
        """learned_simulator.py:519-527"""
        torch.save(self.state_dict(), path)

    def load(self, path: str):
        """learned_simulator.py:529-537 (weights_only: never unpickles code)."""
        self.load_state_dict(torch.load(path, map_location=torch.device("cpu"), weights_only=True))


def time_diff(position_sequence: torch.Tensor) -> torch.Tensor:
    """learned_simulator.py:540-550"""
    return (position_sequence[:, 1:] - position_sequence[:, :-1]).contiguous()
