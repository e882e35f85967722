"""Dispatch between the fused MFMA kernels and the width-generic differentiable
path (sgnn_amd/autograd.py), plus the explicit feature construction the
generic path feeds its modules.

  Encoder.forward(x, e)               graph_network.py:98-111
  InteractionNetwork.forward(x, ei, e) graph_network.py:150-222 -> (x', 2e)
  Processor.forward(x, ei, e)          graph_network.py:276-293
  Decoder.forward(x)                   graph_network.py:324-333
  G2M / M2M / M2G block forward        multi_scale_gnn.py:84-205 (same math)
  EncodeProcessDecode / MultiScaleGNN forward

Under autograd (a parameter or an input requires grad) every module runs the
differentiable path at any widths / depth.  In inference the fused kernels run
wherever they are built for the widths (InteractionNetwork / EncodeProcessDecode
/ MultiScaleGNN at hidden = latent in {64, 128}); everything else runs the
generic path's forward.

PyG semantics (flow source_to_target): x_i = x[edge_index[1]] (receiver),
x_j = x[edge_index[0]] (sender); messages m = edge_fn(cat[x_i, x_j, e]) in the
COO order given; aggr='add' onto receivers (summed in the stable receiver-CSR
order); x' = node_fn(cat[aggr, x]) + x; the edge latent returned is e + e
(update hands back its input edge features)."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import autograd, engine
from ._hip import check, lib, stream_ptr


def needs_grad(module: nn.Module, *tensors) -> bool:
    """True when this call must build an autograd graph."""
    if not torch.is_grad_enabled():
        return False
    return any(p.requires_grad for p in module.parameters()) or any(
        isinstance(t, torch.Tensor) and t.requires_grad for t in tensors)


def edge_features(g: "engine.CsrGraph", pos: torch.Tensor, offset: int, stride: int, dim: int, radius: float):
    """Edge features of a CSR graph (learned_simulator.py:299-312) via sgnn_edge_features."""
    out = torch.empty(g.edge_cap, dim + 1, dtype=torch.float32, device=pos.device)
    check(lib().sgnn_edge_features(pos.data_ptr() + 4 * offset, stride, dim, float(radius), g.rowptr.data_ptr(),
                                   g.send.data_ptr(), g.recv.data_ptr(), g.n, g.edge_cap, out.data_ptr(),
                                   stream_ptr(pos.device)), "sgnn_edge_features")
    return out[:g.num_edges]


def predict_step(sim, inp: "engine.StepInputs", use_emb: bool):
    """LearnedSimulator's decoder output (learned_simulator.py:413-491) on the
    generic path: the HIP radius graph, the feature kernels and the module-by-
    module EncodeProcessDecode -- differentiable (autograd) when grad is enabled,
    for widths / depths the fused step is not built for."""
    pos = inp.pos_seq
    n, T, d = pos.shape
    R = sim._connectivity_radius
    counts = (inp.ex_ptr[1:] - inp.ex_ptr[:-1]).tolist()
    g = engine.radius_graph_csr(pos[:, -1], R, sim._max_num_neighbors, True, counts)
    nf = autograd.node_features(pos, inp.types, sim._particle_type_embedding.weight, use_emb, inp.vel_mean,
                                inp.vel_std, R, 1.0, sim._nparticle_types)
    ef = edge_features(g, pos, (T - 1) * d, T * d, d, R)
    ei = torch.stack([g.send[:g.num_edges], g.recv[:g.num_edges]])
    return autograd.epd_forward(sim._encode_process_decode, nf, ei, ef)


def fast_shapes(epd: nn.Module) -> bool:
    """True when the fused MFMA kernels implement this EncodeProcessDecode:
    hidden = latent in {64, 128}, nmlp_layers 1 or 2, <= 4 edge features and
    the node-feature widths the encoder kernels tile (<= 96 / 64)."""
    H = epd.latent_dim
    return (H in (64, 128) and epd.mlp_hidden_dim == H and epd.nmlp_layers in (1, 2) and epd.nedge_in <= 4
            and epd.nnode_in <= (96 if H == 64 else 64))


def ms_fast_shapes(gnn: nn.Module) -> bool:
    """The same for MultiScaleGNN (nedge_out must equal latent_dim there)."""
    H = gnn.latent_dim
    return (H in (64, 128) and gnn.nedge_out == H and gnn.nmlp_layers in (1, 2) and gnn.nedge_in <= 4
            and gnn.nnode_in <= (96 if H == 64 else 64))


def block_fast_shapes(block: nn.Module) -> bool:
    """One InteractionNetwork / G2M / M2M / M2G block the fused edge / node kernels
    implement: node and edge latents and the MLP hidden width all 64 or 128,
    nmlp_layers 1 or 2."""
    lin = [m for m in block.edge_fn.modules() if isinstance(m, nn.Linear)]
    nlin = [m for m in block.node_fn.modules() if isinstance(m, nn.Linear)]
    H = lin[0].out_features
    return (H in (64, 128) and len(lin) in (2, 3) and len(nlin) == len(lin)
            and lin[0].in_features == 3 * H and lin[-1].out_features == H
            and all(m.out_features == H for m in lin + nlin) and nlin[0].in_features == 2 * H)


def message_passing(block: nn.Module, x: torch.Tensor, edge_index: torch.Tensor, edge_features: torch.Tensor):
    """One block's forward: the fused edge / node kernels in inference at the fast
    widths (engine.interaction_forward), else the differentiable path."""
    if not needs_grad(block, x, edge_features) and block_fast_shapes(block):
        return engine.interaction_forward(block, x, edge_index, edge_features)
    return autograd.message_passing(block, x, autograd.cached_edge_graph(edge_index, x.shape[0]), edge_features)


def processor_forward(proc: nn.Module, x, edge_index, edge_features):
    """Processor.forward (graph_network.py:276-293)."""
    if not needs_grad(proc, x, edge_features) and all(block_fast_shapes(b) for b in proc.gnn_stacks):
        g = engine.coo_to_csr(edge_index, x.shape[0], with_perm=True)
        for gnn in proc.gnn_stacks:
            x, edge_features = engine.interaction_forward(gnn, x, edge_index, edge_features, graph=g)
        return x, edge_features
    return autograd.processor_forward(proc, x, edge_index, edge_features)


def epd_forward(epd: nn.Module, x, edge_index, edge_features) -> torch.Tensor:
    """EncodeProcessDecode.forward (graph_network.py:388-406): the fused chain in
    inference at the fast widths, else module by module (differentiable)."""
    if not needs_grad(epd, x, edge_features) and fast_shapes(epd):
        return engine.epd_forward(epd, x, edge_index, edge_features)
    return autograd.epd_forward(epd, x, edge_index, edge_features)


def ms_gnn_forward(gnn: nn.Module, *args) -> torch.Tensor:
    """MultiScaleGNN.forward (multi_scale_gnn.py:277-326)."""
    if not needs_grad(gnn, *args) and ms_fast_shapes(gnn):
        from .multi_scale import ms_engine
        return ms_engine.gnn_forward(gnn, *args)
    return autograd.ms_gnn_forward(gnn, *args)
