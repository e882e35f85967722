"""Parameter containers with the reference's module tree.

Mirrors sgnn/single_scale/graph_network.py (build_mlp :7-45, Encoder :48-111,
InteractionNetwork :114-222, Processor :225-293, Decoder :296-333,
EncodeProcessDecode :336-406) so that `state_dict()` keys, shapes and the
default-initialisation RNG order are identical to the reference's — reference
checkpoints load unchanged.  The arithmetic runs in libsgnn_hip.so: a
whole EncodeProcessDecode (and LearnedSimulator's steps) through the fused
MFMA kernels (`sgnn_amd.engine`); each module's own forward on explicit
tensors through the fused edge / node kernels in inference at the fast widths,
and otherwise -- any widths, any depth, and whenever autograd needs a graph --
through the differentiable width-generic path (`sgnn_amd.autograd`, dispatch in
`sgnn_amd.generic`).
"""
from __future__ import annotations

from typing import List

import torch.nn as nn


def build_mlp(input_size: int, hidden_layer_sizes: List[int], output_size: int = None,
              output_activation=nn.Identity, activation=nn.ReLU) -> nn.Sequential:
    """Same container and names as graph_network.py:7-45 ("NN-k", "Act-k")."""
    sizes = [input_size] + list(hidden_layer_sizes) + ([output_size] if output_size else [])
    n = len(sizes) - 1
    mlp = nn.Sequential()
    for i in range(n):
        mlp.add_module(f"NN-{i}", nn.Linear(sizes[i], sizes[i + 1]))
        mlp.add_module(f"Act-{i}", (output_activation if i == n - 1 else activation)())
    return mlp


def mlp_ln(nin: int, hidden: int, nout: int, nmlp_layers: int) -> nn.Sequential:
    return nn.Sequential(build_mlp(nin, [hidden] * nmlp_layers, nout), nn.LayerNorm(nout))


class Encoder(nn.Module):
    """graph_network.py:48-111"""

    def __init__(self, nnode_in_features, nnode_out_features, nedge_in_features, nedge_out_features,
                 nmlp_layers, mlp_hidden_dim):
        super().__init__()
        self.node_fn = mlp_ln(nnode_in_features, mlp_hidden_dim, nnode_out_features, nmlp_layers)
        self.edge_fn = mlp_ln(nedge_in_features, mlp_hidden_dim, nedge_out_features, nmlp_layers)

    def forward(self, x, edge_features):
        """graph_network.py:98-111 -> (node latent, edge latent)."""
        from . import autograd
        return autograd.encoder_forward(self, x, edge_features)


class InteractionNetwork(nn.Module):
    """graph_network.py:114-148 (node_fn built before edge_fn, as there)."""

    def __init__(self, nnode_in, nnode_out, nedge_in, nedge_out, nmlp_layers, mlp_hidden_dim):
        super().__init__()
        self.node_fn = mlp_ln(nnode_in + nedge_out, mlp_hidden_dim, nnode_out, nmlp_layers)
        self.edge_fn = mlp_ln(nnode_in + nnode_in + nedge_in, mlp_hidden_dim, nedge_out, nmlp_layers)

    def forward(self, x, edge_index, edge_features):
        """graph_network.py:150-176 -> (x + node_fn([aggr, x]), e + e)."""
        from . import generic
        return generic.message_passing(self, x, edge_index, edge_features)


class Processor(nn.Module):
    """graph_network.py:225-274"""

    def __init__(self, nnode_in, nnode_out, nedge_in, nedge_out, nmessage_passing_steps, nmlp_layers,
                 mlp_hidden_dim):
        super().__init__()
        self.gnn_stacks = nn.ModuleList([
            InteractionNetwork(nnode_in, nnode_out, nedge_in, nedge_out, nmlp_layers, mlp_hidden_dim)
            for _ in range(nmessage_passing_steps)])

    def forward(self, x, edge_index, edge_features):
        """graph_network.py:276-293"""
        from . import generic
        return generic.processor_forward(self, x, edge_index, edge_features)


class Decoder(nn.Module):
    """graph_network.py:296-322 (no LayerNorm)."""

    def __init__(self, nnode_in, nnode_out, nmlp_layers, mlp_hidden_dim):
        super().__init__()
        self.node_fn = build_mlp(nnode_in, [mlp_hidden_dim] * nmlp_layers, nnode_out)

    def forward(self, x):
        """graph_network.py:324-333"""
        from . import autograd
        return autograd.decoder_forward(self, x)


class EncodeProcessDecode(nn.Module):
    """graph_network.py:336-386.  Calling it runs the HIP path (engine.epd_forward)."""

    def __init__(self, nnode_in_features, nnode_out_features, nedge_in_features, latent_dim,
                 nmessage_passing_steps, nmlp_layers, mlp_hidden_dim):
        super().__init__()
        self._encoder = Encoder(nnode_in_features, latent_dim, nedge_in_features, latent_dim,
                                nmlp_layers, mlp_hidden_dim)
        self._processor = Processor(latent_dim, latent_dim, latent_dim, latent_dim,
                                    nmessage_passing_steps, nmlp_layers, mlp_hidden_dim)
        self._decoder = Decoder(latent_dim, nnode_out_features, nmlp_layers, mlp_hidden_dim)
        self.latent_dim = latent_dim
        self.mlp_hidden_dim = mlp_hidden_dim
        self.nlayers = nmessage_passing_steps
        self.nmlp_layers = nmlp_layers
        self.nnode_in = nnode_in_features
        self.nedge_in = nedge_in_features
        self.nnode_out = nnode_out_features

    def forward(self, x, edge_index, edge_features):
        """graph_network.py:388-406 on explicit features: the fused MFMA chain
        (engine.epd_forward) in inference at the widths it is built for, else
        module by module on the differentiable path."""
        from . import generic
        return generic.epd_forward(self, x, edge_index, edge_features)
