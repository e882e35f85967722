"""Launch sequence of one multi-scale step on the HIP kernels
(MultiScaleSimulator.predict_positions, multi_scale_simulator.py:288-326,
through MultiScaleGNN.forward, multi_scale_gnn.py:262-326).

    encode_nodes   x0 = grid_node_encoder(features) ; u,v for g2m_block.edge_fn
    encode_edges   e_g2m, e_m2m, e_m2g (three edge encoders, three CSR graphs)
    G2M            edge_layer(g2m, scale 1)  -> node_layer(g2m.node_fn; u,v of m2m_blocks[0])
    M2M k=0..L-1   edge_layer(m2m, scale 2^k) -> node_layer(...; u,v of the next block)
    M2G            edge_layer(m2g, scale 1)  -> node_layer_decode(m2g.node_fn, prediction_head)

All blocks run over the n grid nodes; only the CSR graph changes.  The same
kernels as the single-scale path (sgnn_amd/csrc/epd_fwd.hip) with nmlp_layers
= 2 (3 Linear layers) and H = 128 for the reference configuration.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from .. import engine
from .._hip import check, lib, stream_ptr

EDGE_TYPES = ("g2m", "m2m", "m2g")


class MSWorkspace:
    """HBM buffers for one (n, T, static graph) shape."""

    def __init__(self, n: int, T: int, dim: int, hidden: int, graphs: Dict[str, engine.CsrGraph],
                 device: torch.device):
        L = lib()
        f32 = dict(dtype=torch.float32, device=device)
        self.n, self.T, self.dim, self.H = n, T, dim, hidden
        self.x_a = torch.empty(n, hidden, **f32)
        self.x_b = torch.empty(n, hidden, **f32)
        self.u = torch.empty(n, hidden, **f32)
        self.v = torch.empty(n, hidden, **f32)
        self.agg = torch.empty(n, hidden, **f32)
        nt = max(g.ntiles for g in graphs.values())
        self.cin = torch.empty(nt, hidden, **f32)
        self.cout = torch.empty(nt, hidden, **f32)
        self.e0t = {k: torch.empty(int(L.sgnn_edge_latent_floats(g.edge_cap, hidden)), **f32)
                    for k, g in graphs.items()}


class ParamPack:
    """ctypes parameter structs of one MultiScaleGNN, rebuilt only when a
    parameter tensor is replaced (e.g. after .to())."""

    def __init__(self, gnn):
        ms = engine.mlp_struct
        self.key = tuple(p.data_ptr() for p in gnn.parameters())
        chain = gnn.chain()
        self.edge = [ms(b.edge_fn, True) for b in chain]
        self.node = [ms(b.node_fn, True) for b in chain]
        self.enc = ms(gnn.grid_node_encoder, True)
        self.head = ms(gnn.prediction_head, False)
        self.enc_edge = {"g2m": ms(gnn.g2m_edge_encoder, True), "m2m": ms(gnn.m2m_edge_encoder, True),
                         "m2g": ms(gnn.m2g_edge_encoder, True)}

    @staticmethod
    def get(gnn) -> "ParamPack":
        key = tuple(p.data_ptr() for p in gnn.parameters())
        pk = getattr(gnn, "_sgnn_pack", None)
        if pk is None or pk.key != key:
            pk = ParamPack(gnn)
            gnn._sgnn_pack = pk
        return pk


def forward_step(gnn, emb_weight: Optional[torch.Tensor], use_emb: bool, inp: engine.StepInputs,
                 graphs: Dict[str, engine.CsrGraph], grid_radius: float, mesh_radius: float,
                 ws: MSWorkspace, pred: torch.Tensor, next_pos: torch.Tensor,
                 window_out: Optional[torch.Tensor] = None) -> None:
    L = lib()
    s = stream_ptr(inp.pos_seq.device)
    pos = inp.pos_seq
    n, T, d, H = ws.n, ws.T, ws.dim, ws.H
    pk = ParamPack.get(gnn)
    chain = gnn.chain()
    kinds = ["g2m"] + ["m2m"] * (len(chain) - 2) + ["m2g"]
    scales = [1.0] + [float(2.0 ** k) for k in range(len(chain) - 2)] + [1.0]
    edge_s, node_s, enc, head, enc_s = pk.edge, pk.node, pk.enc, pk.head, pk.enc_edge
    emb_dim = emb_weight.shape[1] if (use_emb and emb_weight is not None) else 0
    # wall feature clamp(x + 2, 0, R_g) / R_g (multi_scale_simulator.py:193-196)
    check(L.sgnn_encode_nodes(pos.data_ptr(), n, T, d, engine._ptr(inp.types) if use_emb else 0,
                              engine._ptr(emb_weight) if use_emb else 0, emb_dim, int(use_emb),
                              inp.vel_mean.data_ptr(), inp.vel_std.data_ptr(), float(grid_radius),
                              float(grid_radius), ctypes.byref(enc), ctypes.byref(edge_s[0]),
                              ws.x_a.data_ptr(), ws.u.data_ptr(), ws.v.data_ptr(), None, s),
          "sgnn_encode_nodes")
    radii = {"g2m": grid_radius, "m2m": mesh_radius, "m2g": grid_radius}   # :221-241
    for k in EDGE_TYPES:
        g = graphs[k]
        check(L.sgnn_encode_edges(pos.data_ptr() + 4 * (T - 1) * d, T * d, d, float(radii[k]),
                                  g.rowptr.data_ptr(), g.send.data_ptr(), g.recv.data_ptr(), n,
                                  g.edge_cap, ctypes.byref(enc_s[k]), ws.e0t[k].data_ptr(), None, s),
              "sgnn_encode_edges")
    x_in, x_out = ws.x_a, ws.x_b
    for b in range(len(chain)):
        g = graphs[kinds[b]]
        check(L.sgnn_edge_layer(ws.u.data_ptr(), ws.v.data_ptr(), ws.e0t[kinds[b]].data_ptr(), scales[b],
                                g.rowptr.data_ptr(), g.send.data_ptr(), g.recv.data_ptr(), n, g.edge_cap,
                                ctypes.byref(edge_s[b]), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                ws.cout.data_ptr(), None, s), "sgnn_edge_layer")
        if b < len(chain) - 1:
            check(L.sgnn_node_layer(x_in.data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                    ws.cout.data_ptr(), g.rowptr.data_ptr(), n, ctypes.byref(node_s[b]),
                                    ctypes.byref(edge_s[b + 1]), x_out.data_ptr(), ws.u.data_ptr(),
                                    ws.v.data_ptr(), None, s), "sgnn_node_layer")
            x_in, x_out = x_out, x_in
        else:
            check(L.sgnn_node_layer_decode(x_in.data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                           ws.cout.data_ptr(), g.rowptr.data_ptr(), n,
                                           ctypes.byref(node_s[b]), ctypes.byref(head), pos.data_ptr(), T,
                                           d, inp.acc_mean.data_ptr(), inp.acc_std.data_ptr(), 0,
                                           pred.data_ptr(), next_pos.data_ptr(),
                                           engine._ptr(window_out), None, s), "sgnn_node_layer_decode")


def gnn_forward(gnn, x, g2m_edge_index, g2m_edge_features, m2m_edge_index, m2m_edge_features,
                m2g_edge_index, m2g_edge_features) -> torch.Tensor:
    """MultiScaleGNN.forward (multi_scale_gnn.py:262-326) on explicit features:
    grid node features [N, F], the three COO edge lists and their features ->
    prediction head output [N, d+1]."""
    x = engine._feature_rows(x, "x")
    n = x.shape[0]
    eis = {"g2m": g2m_edge_index, "m2m": m2m_edge_index, "m2g": m2g_edge_index}
    efs = {"g2m": g2m_edge_features, "m2m": m2m_edge_features, "m2g": m2g_edge_features}
    graphs = {k: engine.coo_to_csr(torch.as_tensor(eis[k]).to(x.device), n, with_perm=True) for k in EDGE_TYPES}
    efeats = {k: engine._feature_rows(efs[k], f"{k}_edge_features") for k in EDGE_TYPES}
    pk = ParamPack.get(gnn)
    nb = len(gnn.chain())
    kinds = ["g2m"] + ["m2m"] * (nb - 2) + ["m2g"]
    scales = [1.0] + [float(2.0 ** k) for k in range(nb - 2)] + [1.0]
    return engine.run_chain(pk.enc, pk.enc_edge, pk.edge, pk.node, pk.head, kinds, scales, x, graphs, efeats,
                            pk.head.out_dim)
