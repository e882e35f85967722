"""Multi-scale GNN parameter tree (sgnn/multi_scale/multi_scale_gnn.py).

Same module classes, construction order and therefore the same state_dict
keys and random initialisation as the reference (a reference checkpoint loads
unchanged; under one seed both draw identical weights).  The arithmetic of
`MultiScaleGNN.forward` runs as the fused HIP chain in `ms_engine`
(encoder -> G2M -> M2M x L -> M2G -> prediction head), driven by
`MultiScaleSimulator`; `MultiScaleGNN.forward` on explicit features runs the
same kernels, and each block's own forward (and any width the fused kernels
are not built for, e.g. nedge_out != latent_dim, and every forward under
autograd) runs on the differentiable width-generic path (`sgnn_amd.autograd`).

Semantics the kernels implement (what PyG executes for these blocks):
  message  m = LN(MLP_e([x_i, x_j, e]))   (multi_scale_gnn.py:96-101)
  aggregate a_i = sum_{edges into i} m    (aggr='add', :67)
  update   x' = LN(MLP_n([a, x])) + x     (:103-107, residual :94)
  edges    e' = e + e  — `update` hands back the block's INPUT edge features
           (:107), so a block's edge latent is 2x its input; M2M block k sees
           2^k times the encoded m2m latent.
Every block runs over all grid nodes; nodes without incoming edges of the
block's type aggregate zero but still pass through node_fn.
"""
from __future__ import annotations

from typing import List

import torch.nn as nn

from ..graph_network import build_mlp


def _mlp_ln(nin: int, hidden: int, nout: int, nmlp_layers: int) -> nn.Sequential:
    return nn.Sequential(*[build_mlp(nin, [hidden for _ in range(nmlp_layers)], nout), nn.LayerNorm(nout)])


class _Block(nn.Module):
    """G2MBlock / M2MBlock / M2GBlock (:63-181): node_fn built before edge_fn."""

    def __init__(self, nnode_in: int, nnode_out: int, nedge_in: int, nedge_out: int,
                 nmlp_layers: int, latent_dim: int):
        super().__init__()
        self.node_fn = _mlp_ln(nnode_in + nedge_out, latent_dim, nnode_out, nmlp_layers)
        self.edge_fn = _mlp_ln(nnode_in + nnode_in + nedge_in, latent_dim, nedge_out, nmlp_layers)

    def forward(self, x, edge_index, edge_features):
        """multi_scale_gnn.py:84-94 (and :132-142, :179-189) -> (x + node_fn([aggr, x]), e + e)."""
        from .. import generic
        return generic.message_passing(self, x, edge_index, edge_features)


class G2MBlock(_Block):
    """multi_scale_gnn.py:63-107 (grid -> mesh)."""


class M2MBlock(_Block):
    """multi_scale_gnn.py:110-152 (mesh <-> mesh, the processor)."""


class M2GBlock(_Block):
    """multi_scale_gnn.py:155-199 (mesh -> grid, the decoder block)."""


class MultiScaleGNN(nn.Module):
    """multi_scale_gnn.py:202-326"""

    def __init__(self, nnode_in_features: int, nnode_out_features: int, nedge_in_features: int,
                 nedge_out_features: int, latent_dim: int, nmessage_passing_steps: int,
                 nmlp_layers: int, num_scales: int, share_weights_across_scales: bool = False):
        super().__init__()
        self.num_scales = num_scales
        self.latent_dim = latent_dim
        self.nmessage_passing_steps = nmessage_passing_steps
        self.nnode_in = nnode_in_features
        self.nedge_in = nedge_in_features
        self.nedge_out = nedge_out_features
        self.nmlp_layers = nmlp_layers
        L, E = latent_dim, nedge_out_features
        self.grid_node_encoder = _mlp_ln(nnode_in_features, L, L, nmlp_layers)
        self.g2m_edge_encoder = _mlp_ln(nedge_in_features, L, E, nmlp_layers)
        self.m2m_edge_encoder = _mlp_ln(nedge_in_features, L, E, nmlp_layers)
        self.m2g_edge_encoder = _mlp_ln(nedge_in_features, L, E, nmlp_layers)
        self.g2m_block = G2MBlock(L, L, E, E, nmlp_layers, L)
        self.m2m_blocks = nn.ModuleList([M2MBlock(L, L, E, E, nmlp_layers, L)
                                         for _ in range(nmessage_passing_steps)])
        self.m2g_block = M2GBlock(L, L, E, E, nmlp_layers, L)
        self.prediction_head = build_mlp(L, [L for _ in range(nmlp_layers)], nnode_out_features)

    def chain(self) -> List[nn.Module]:
        """Blocks in execution order (:301-319)."""
        return [self.g2m_block, *self.m2m_blocks, self.m2g_block]

    def forward(self, x, g2m_edge_index, g2m_edge_features, m2m_edge_index, m2m_edge_features,
                m2g_edge_index, m2g_edge_features, graph_hierarchy=None):
        """multi_scale_gnn.py:262-326 on explicit features (HIP kernels: the fused
        chain in inference at the widths it is built for, else block by block on
        the differentiable path); graph_hierarchy is unused, as in the reference."""
        from .. import generic
        return generic.ms_gnn_forward(self, x, g2m_edge_index, g2m_edge_features, m2m_edge_index,
                                      m2m_edge_features, m2g_edge_index, m2g_edge_features)
