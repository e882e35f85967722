"""Width-generic path on the generic.hip kernels (any latent / hidden / edge
widths, nmlp_layers 1 or 2): the reference's per-module forwards on explicit
tensors and whole models whose widths the MFMA kernels are not built for.

  Encoder.forward(x, e)               graph_network.py:98-111
  InteractionNetwork.forward(x, ei, e) graph_network.py:150-222 -> (x', 2e)
  Processor.forward(x, ei, e)          graph_network.py:276-293
  Decoder.forward(x)                   graph_network.py:324-333
  G2M / M2M / M2G block forward        multi_scale_gnn.py:84-205 (same math)
  EncodeProcessDecode / MultiScaleGNN forward when the fast kernels do not apply

PyG semantics (flow source_to_target): x_i = x[edge_index[1]] (receiver),
x_j = x[edge_index[0]] (sender); messages m = edge_fn(cat[x_i, x_j, e]) in the
COO order given; aggr='add' onto receivers (summed in the stable receiver-CSR
order of sgnn_coo_to_csr); x' = node_fn(cat[aggr, x]) + x; the edge latent
returned is e + e (update hands back its input edge features)."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import engine
from ._hip import SgnnRowsSrc, check, lib, require_gpu_tensor, stream_ptr


def _rows(t: torch.Tensor, name: str) -> torch.Tensor:
    require_gpu_tensor(t, name)
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(t.shape)}")
    return t.to(torch.float32).contiguous()


def rows_mlp(seq: nn.Module, has_ln: bool, sources: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor]]],
             n: int, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[r] = seq(cat_k sources[k][0][idx_k[r]]) (+ residual[r]) via sgnn_rows_mlp.
    `seq` is a reference-layout Sequential(build_mlp[, LayerNorm])."""
    m = engine.mlp_struct(seq, has_ln)
    dev = sources[0][0].device
    out = torch.empty(n, m.out_dim, dtype=torch.float32, device=dev)
    if n == 0:
        return out
    keep = []
    srcs = (SgnnRowsSrc * len(sources))()
    for k, (t, idx) in enumerate(sources):
        if idx is not None:
            idx = idx.to(torch.int32).contiguous()
            keep.append(idx)
        srcs[k] = SgnnRowsSrc(data=t.data_ptr(), index=idx.data_ptr() if idx is not None else 0,
                              ld=t.shape[1], dim=t.shape[1], scale=1.0)
    if residual is not None and tuple(residual.shape) != (n, m.out_dim):
        raise ValueError(f"residual {tuple(residual.shape)} does not match the output [{n}, {m.out_dim}]")
    check(lib().sgnn_rows_mlp(srcs, len(sources), n, ctypes.byref(m),
                              residual.data_ptr() if residual is not None else None, out.data_ptr(),
                              stream_ptr(dev)), "sgnn_rows_mlp")
    return out


def encoder_forward(enc: nn.Module, x: torch.Tensor, edge_features: torch.Tensor):
    """Encoder.forward (graph_network.py:98-111): (node_fn(x), edge_fn(e))."""
    x, e = _rows(x, "x"), _rows(edge_features, "edge_features")
    return (rows_mlp(enc.node_fn, True, [(x, None)], x.shape[0]),
            rows_mlp(enc.edge_fn, True, [(e, None)], e.shape[0]))


def decoder_forward(dec: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Decoder.forward (graph_network.py:324-333; no LayerNorm)."""
    x = _rows(x, "x")
    return rows_mlp(dec.node_fn, False, [(x, None)], x.shape[0])


def message_passing(block: nn.Module, x: torch.Tensor, edge_index: torch.Tensor, edge_features: torch.Tensor,
                    graph: Optional[engine.CsrGraph] = None):
    """One InteractionNetwork / G2M / M2M / M2G block forward: (x', e + e)."""
    x, e = _rows(x, "x"), _rows(edge_features, "edge_features")
    require_gpu_tensor(edge_index, "edge_index")
    n, E = x.shape[0], edge_index.shape[1]
    if e.shape[0] != E:
        raise ValueError(f"{e.shape[0]} edge feature rows for {E} edges")
    g = graph if graph is not None else engine.coo_to_csr(edge_index, n, with_perm=True)
    em = block.edge_fn
    width = em[1].normalized_shape[0]
    ei = edge_index.to(torch.int32)
    m = rows_mlp(em, True, [(x, ei[1]), (x, ei[0]), (e, None)], E) if E else \
        torch.zeros(0, width, dtype=torch.float32, device=x.device)
    agg = torch.empty(n, width, dtype=torch.float32, device=x.device)
    check(lib().sgnn_segment_sum(m.data_ptr() if E else agg.data_ptr(), g.rowptr.data_ptr(), g.perm.data_ptr(), n,
                                 width, agg.data_ptr(), stream_ptr(x.device)), "sgnn_segment_sum")
    x_new = rows_mlp(block.node_fn, True, [(agg, None), (x, None)], n, residual=x)
    return x_new, e + e


def processor_forward(proc: nn.Module, x, edge_index, edge_features):
    """Processor.forward (graph_network.py:276-293)."""
    g = engine.coo_to_csr(edge_index, x.shape[0], with_perm=True)
    for gnn in proc.gnn_stacks:
        x, edge_features = message_passing(gnn, x, edge_index, edge_features, graph=g)
    return x, edge_features


def epd_forward(epd: nn.Module, x, edge_index, edge_features) -> torch.Tensor:
    """EncodeProcessDecode.forward (graph_network.py:388-406), module by module."""
    x, e = encoder_forward(epd._encoder, x, edge_features)
    x, e = processor_forward(epd._processor, x, edge_index, e)
    return decoder_forward(epd._decoder, x)


def ms_gnn_forward(gnn: nn.Module, x, g2m_ei, g2m_e, m2m_ei, m2m_e, m2g_ei, m2g_e) -> torch.Tensor:
    """MultiScaleGNN.forward (multi_scale_gnn.py:277-326), block by block."""
    x = _rows(x, "x")
    n = x.shape[0]
    h = rows_mlp(gnn.grid_node_encoder, True, [(x, None)], n)
    enc = lambda seq, t: rows_mlp(seq, True, [(_rows(t, "edge_features"), None)], t.shape[0])
    eg, em, eo = enc(gnn.g2m_edge_encoder, g2m_e), enc(gnn.m2m_edge_encoder, m2m_e), enc(gnn.m2g_edge_encoder, m2g_e)
    h, eg = message_passing(gnn.g2m_block, h, g2m_ei, eg)
    gm = engine.coo_to_csr(m2m_ei, n, with_perm=True)
    for blk in gnn.m2m_blocks:
        h, em = message_passing(blk, h, m2m_ei, em, graph=gm)
    h, eo = message_passing(gnn.m2g_block, h, m2g_ei, eo)
    return rows_mlp(gnn.prediction_head, False, [(h, None)], n)


def node_features(pos_seq: torch.Tensor, types, emb_w, use_emb: bool, vel_mean, vel_std, wall_max: float,
                  wall_div: float) -> torch.Tensor:
    """_encoder_preprocessor's node features (learned_simulator.py:256-290) via sgnn_node_features."""
    n, T, d = pos_seq.shape
    emb_dim = emb_w.shape[1] if use_emb else 0
    out = torch.empty(n, (T - 1) * d + 1 + emb_dim, dtype=torch.float32, device=pos_seq.device)
    check(lib().sgnn_node_features(pos_seq.data_ptr(), n, T, d, types.data_ptr() if use_emb else None,
                                   emb_w.data_ptr() if use_emb else None, emb_dim, int(use_emb),
                                   vel_mean.data_ptr(), vel_std.data_ptr(), float(wall_max), float(wall_div),
                                   out.data_ptr(), stream_ptr(pos_seq.device)), "sgnn_node_features")
    return out


def edge_features(g: "engine.CsrGraph", pos: torch.Tensor, offset: int, stride: int, dim: int, radius: float):
    """Edge features of a CSR graph (learned_simulator.py:299-312) via sgnn_edge_features."""
    out = torch.empty(g.edge_cap, dim + 1, dtype=torch.float32, device=pos.device)
    check(lib().sgnn_edge_features(pos.data_ptr() + 4 * offset, stride, dim, float(radius), g.rowptr.data_ptr(),
                                   g.send.data_ptr(), g.recv.data_ptr(), g.n, g.edge_cap, out.data_ptr(),
                                   stream_ptr(pos.device)), "sgnn_edge_features")
    return out[:g.num_edges]


def predict_step(sim, inp: "engine.StepInputs", use_emb: bool):
    """LearnedSimulator.predict_positions' decoder output (learned_simulator.py:
    413-436) for widths the fused step is not built for: the HIP radius graph,
    the feature kernels and the module-by-module EncodeProcessDecode."""
    pos = inp.pos_seq
    n, T, d = pos.shape
    R = sim._connectivity_radius
    counts = (inp.ex_ptr[1:] - inp.ex_ptr[:-1]).tolist()
    g = engine.radius_graph_csr(pos[:, -1], R, sim._max_num_neighbors, True, counts)
    nf = node_features(pos, inp.types, sim._particle_type_embedding.weight, use_emb, inp.vel_mean, inp.vel_std,
                       R, 1.0)
    ef = edge_features(g, pos, (T - 1) * d, T * d, d, R)
    ei = torch.stack([g.send[:g.num_edges], g.recv[:g.num_edges]])
    return epd_forward(sim._encode_process_decode, nf, ei, ef)


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
