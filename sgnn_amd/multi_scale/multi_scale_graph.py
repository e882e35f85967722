"""Static multi-scale graph hierarchy (sgnn/multi_scale/multi_scale_graph.py).

Same classes, attributes and returned dict as the reference; the radius
searches run in libsgnn_hip (torch_cluster's max_num_neighbors rule: keep the
K smallest neighbour ids, strict `d^2 < r^2`), the sampling and filtering run
as torch ops on the positions' device.  Edge lists come back as int64 COO
`[senders; receivers]` in the reference's order (receiver-major, neighbour
ids ascending), so `MultiScaleSimulator.set_static_graph` accepts either this
or a dict built by the reference on the CPU.

Note (parity): the reference builds these graphs once per trajectory with
torch_cluster's CPU radius search (static_graph_data_loader.py:96-106).  Where
more than `max_neighbors` = 24 candidates lie inside the radius (3D lattices
at radius_multiplier 2 have 33), which 24 the CPU kd-tree keeps is
implementation-defined; we keep the 24 smallest ids (the CUDA rule).  In 2D
(13 candidates) the graphs are identical.
"""
from __future__ import annotations

from typing import Any, Dict, Tuple

import torch

from .. import engine


class MultiScaleConfig:
    """multi_scale_graph.py:14-37"""

    def __init__(self, num_scales: int = 3, window_size: int = 3, radius_multiplier: float = 2.0):
        if num_scales < 2:
            raise ValueError(f"num_scales must be >= 2 (need grid + at least 1 mesh level), got {num_scales}")
        self.num_scales = num_scales
        self.window_size = window_size
        self.grid_spacing = 0.5
        self.radius_multiplier = radius_multiplier
        self.max_neighbors = 24


def _radius_edges(positions: torch.Tensor, r: float, k: int) -> torch.Tensor:
    """radius_graph(positions, r, loop=True, max_num_neighbors=k) -> [2, E] int64."""
    return engine.radius_graph_csr(positions, r, k, True).edge_index()


class MultiScaleGraph:
    """multi_scale_graph.py:39-283"""

    def __init__(self, config: MultiScaleConfig):
        self.config = config
        self.grid_positions = None
        self.graph_hierarchy: Dict[int, Dict[str, Any]] = {}

    def create_all_edges(self, grid_positions: torch.Tensor) -> Dict[str, Any]:
        """:48-96 -> {'graph_hierarchy', 'grid2mesh_edges', 'mesh2mesh_edges', 'mesh2grid_edges'}"""
        if not self.graph_hierarchy:
            self.build_hierarchy(grid_positions)
        g2m, m2g = self._create_grid_mesh_connectivity(grid_positions)
        m2m = [e for e in (self._create_mesh2mesh_edges(s) for s in range(1, self.config.num_scales))
               if e.shape[1] > 0]
        if m2m:
            m2m_edges = torch.cat(m2m, dim=1)
        else:
            m2m_edges = torch.empty((2, 0), dtype=torch.long, device=grid_positions.device)
        return {"graph_hierarchy": self.graph_hierarchy, "grid2mesh_edges": g2m,
                "mesh2mesh_edges": m2m_edges, "mesh2grid_edges": m2g}

    def build_hierarchy(self, grid_positions: torch.Tensor) -> Dict[str, Any]:
        """:98-136"""
        self.grid_positions = grid_positions
        self.graph_hierarchy[0] = {
            "sampling_indices": torch.arange(len(grid_positions), dtype=torch.long,
                                             device=grid_positions.device),
            "spacing": self.config.grid_spacing,
            "num_particles": len(grid_positions)}
        cur, spacing = grid_positions, self.config.grid_spacing
        for scale in range(1, self.config.num_scales):
            cur, spacing, idx = self._sample_coarser_scale(cur, spacing, scale)
            self.graph_hierarchy[scale] = {"sampling_indices": idx, "spacing": spacing,
                                           "num_particles": len(cur)}
        return self.graph_hierarchy

    def _sample_coarser_scale(self, current_positions: torch.Tensor, current_spacing: float,
                              scale: int) -> Tuple[torch.Tensor, float, torch.Tensor]:
        """:138-191: keep every window_size-th distinct x AND y coordinate
        (z is not sampled, as in the reference)."""
        w = self.config.window_size
        x, y = current_positions[:, 0], current_positions[:, 1]
        sx = torch.unique(x)[::w]   # torch.unique returns sorted values
        sy = torch.unique(y)[::w]
        local = torch.where(torch.isin(x, sx) & torch.isin(y, sy))[0]
        parent = self.graph_hierarchy[scale - 1]["sampling_indices"].to(local.device)
        return current_positions[local], current_spacing * w, parent[local]

    def _create_grid_mesh_connectivity(self, grid_positions: torch.Tensor):
        """:193-241: one radius graph on the grid, split by mesh membership."""
        if 1 not in self.graph_hierarchy:
            raise ValueError("First mesh level 1 not found")
        mesh = self.graph_hierarchy[1]["sampling_indices"].to(grid_positions.device)
        r = self.config.radius_multiplier * self.config.grid_spacing
        ei = _radius_edges(grid_positions, r, self.config.max_neighbors)
        g2m = ei[:, torch.isin(ei[1], mesh)]
        m2g = ei[:, torch.isin(ei[0], mesh)]
        return g2m, m2g

    def _create_mesh2mesh_edges(self, scale: int) -> torch.Tensor:
        """:244-281: radius graph among one mesh level, mapped to grid ids."""
        if scale not in self.graph_hierarchy:
            raise ValueError(f"Scale {scale} not found")
        data = self.graph_hierarchy[scale]
        r = data["spacing"] * self.config.radius_multiplier
        idx = data["sampling_indices"].to(self.grid_positions.device)
        ei = _radius_edges(self.grid_positions[idx], r, self.config.max_neighbors)
        return torch.stack([idx[ei[0]], idx[ei[1]]])


def build_static_multi_scale_graph(initial_positions: torch.Tensor, num_scales: int = 3,
                                   window_size: int = 3, radius_multiplier: float = 2.0) -> Dict[str, Any]:
    """static_graph_data_loader.py:27-60 on the GPU (positions must be a CUDA tensor)."""
    cfg = MultiScaleConfig(num_scales=num_scales, window_size=window_size,
                           radius_multiplier=radius_multiplier)
    return MultiScaleGraph(cfg).create_all_edges(initial_positions)
