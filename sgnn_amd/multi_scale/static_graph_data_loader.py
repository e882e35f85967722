"""Multi-scale datasets and collate (sgnn/multi_scale/static_graph_data_loader.py),
with the static graphs built by the GPU builder (multi_scale_graph.py here) and
the batch > 1 fix behind a flag.

Reference behaviour, kept as the default: every trajectory's static graph is
built once from its first frame (:100-118, :178-196) and
`multi_scale_collate_fn` gives the WHOLE batch the graph of its first sample
(:228-229) -- with batch_size > 1 and samples from different trajectories the
other samples' particles are wired with sample 0's edges (and a batch with
more particles than sample 0 indexes past them).

`per_sample_graphs=True` instead merges the samples' graphs into one
block-diagonal graph over the concatenated batch (node ids of sample k offset
by the particle count before it; the hierarchy's sampling indices likewise;
spacings are config-derived and identical).  Every sample then sees exactly
its own graph, and the batch is the union of independent samples -- what the
single-scale path does with nparticles_per_example.
"""
from __future__ import annotations

import functools
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import data as D
from .multi_scale_graph import build_static_multi_scale_graph as _build_on_device


def build_static_multi_scale_graph(initial_positions: torch.Tensor, num_scales: int = 3, window_size: int = 3,
                                   radius_multiplier: float = 2.0, device=None) -> Dict[str, Any]:
    """:27-60.  Built by the HIP radius graph + device sampling; host positions
    are moved to `device` (default: the current CUDA device)."""
    dev = torch.device(device) if device is not None else (
        initial_positions.device if initial_positions.is_cuda else torch.device("cuda"))
    return _build_on_device(initial_positions.to(dev, torch.float32), num_scales, window_size, radius_multiplier)


def _to_host(obj):
    """Every tensor of a (nested) graph dict moved to host memory."""
    if isinstance(obj, torch.Tensor):
        return obj.cpu()
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    return obj


def _graphs_for(trajectories, num_scales, window_size, radius_multiplier, device, graph_builder):
    """One static graph per trajectory, built on the GPU and kept in HOST memory
    as the reference's are (:100-118): the DataLoader may then pin the batch
    (pin_memory=True, the reference's default) and fork workers; the simulator
    moves the edges to its device once per graph (`set_static_graph` / `_csr`)."""
    build = graph_builder or functools.partial(build_static_multi_scale_graph, device=device)
    return {i: _to_host(build(torch.tensor(pos[0], dtype=torch.float32), num_scales, window_size,
                              radius_multiplier))
            for i, (pos, _, _) in enumerate(trajectories)}


class MultiScaleTaylorImpactSamplesDataset(D.TaylorImpactSamplesDataset):
    """:63-141: samples + the static graph of their trajectory under 'graph'.
    graph_builder(positions, num_scales, window_size, radius_multiplier) may
    replace the GPU builder (e.g. a graph dict prepared elsewhere)."""

    def __init__(self, data_path: str, input_length_sequence: int = 3, load_stress_stats: bool = True,
                 num_scales: int = 3, window_size: int = 3, radius_multiplier: float = 2.0, device=None,
                 graph_builder: Optional[Callable] = None):
        super().__init__(data_path, input_length_sequence, load_stress_stats)
        self._num_scales, self._window_size = num_scales, window_size
        self._static_graphs = _graphs_for(self._data, num_scales, window_size, radius_multiplier, device,
                                          graph_builder)

    def __getitem__(self, idx: int) -> Dict:
        sample = super().__getitem__(idx)
        sample["graph"] = self._static_graphs[int(sample["meta"]["trajectory_idx"])]
        return sample


class MultiScaleTaylorImpactTrajectoriesDataset(D.TaylorImpactTrajectoriesDataset):
    """:144-215: whole trajectories + their static graph under 'graph'."""

    def __init__(self, data_path: str, load_stress_stats: bool = True, num_scales: int = 3, window_size: int = 3,
                 radius_multiplier: float = 2.0, device=None, graph_builder: Optional[Callable] = None):
        super().__init__(data_path, load_stress_stats)
        self._num_scales, self._window_size = num_scales, window_size
        self._static_graphs = _graphs_for(self._data, num_scales, window_size, radius_multiplier, device,
                                          graph_builder)

    def __getitem__(self, idx: int) -> Dict:
        traj = super().__getitem__(idx)
        traj["graph"] = self._static_graphs[idx]
        return traj


def merge_static_graphs(graphs: Sequence[Dict[str, Any]], counts: Sequence[int]) -> Dict[str, Any]:
    """Block-diagonal union of per-sample static graphs over the concatenated
    batch (sample k's node ids offset by sum(counts[:k]))."""
    if len(graphs) != len(counts):
        raise ValueError("one graph per sample")
    offsets = np.concatenate([[0], np.cumsum([int(c) for c in counts])[:-1]]).tolist()
    out: Dict[str, Any] = {}
    for key in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges"):
        out[key] = torch.cat([g[key] + off for g, off in zip(graphs, offsets)], dim=1)
    hier = {}
    for s, lvl0 in graphs[0]["graph_hierarchy"].items():
        spacing = lvl0["spacing"]
        for g in graphs[1:]:
            if not np.isclose(float(g["graph_hierarchy"][s]["spacing"]), float(spacing)):
                raise ValueError(f"scale {s}: samples with different mesh spacings cannot share one batch graph")
        hier[s] = {"sampling_indices": torch.cat([g["graph_hierarchy"][s]["sampling_indices"] + off
                                                  for g, off in zip(graphs, offsets)]),
                   "spacing": spacing,
                   "num_particles": int(sum(int(g["graph_hierarchy"][s]["num_particles"]) for g in graphs))}
    out["graph_hierarchy"] = hier
    return out


def multi_scale_collate_fn(batch: List[Dict], per_sample_graphs: bool = False) -> Dict:
    """:218-231.  Default: the batch carries sample 0's graph (the reference's
    behaviour).  per_sample_graphs=True: the merged block-diagonal graph."""
    out = D.collate_fn(batch)
    if "graph" in batch[0]:
        if per_sample_graphs:
            out["graph"] = merge_static_graphs([b["graph"] for b in batch],
                                               [int(b["input"]["n_particles_per_example"]) for b in batch])
        else:
            out["graph"] = batch[0]["graph"]
    return out


def get_multi_scale_data_loader_by_samples(path: str, input_length_sequence: int = 3, batch_size: int = 2,
                                           shuffle: bool = True, num_workers: int = 0, pin_memory: bool = True,
                                           load_stress_stats: bool = True, num_scales: int = 3,
                                           window_size: int = 3, radius_multiplier: float = 2.0,
                                           per_sample_graphs: bool = False, device=None,
                                           graph_builder: Optional[Callable] = None):
    """:234-279 (+ per_sample_graphs, device, graph_builder)."""
    ds = MultiScaleTaylorImpactSamplesDataset(path, input_length_sequence, load_stress_stats, num_scales,
                                              window_size, radius_multiplier, device, graph_builder)
    return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                                       pin_memory=pin_memory,
                                       collate_fn=functools.partial(multi_scale_collate_fn,
                                                                    per_sample_graphs=per_sample_graphs))


def get_multi_scale_data_loader_by_trajectories(path: str, num_workers: int = 0, pin_memory: bool = True,
                                                load_stress_stats: bool = True, num_scales: int = 3,
                                                window_size: int = 3, radius_multiplier: float = 2.0, device=None,
                                                graph_builder: Optional[Callable] = None):
    """:282-317"""
    ds = MultiScaleTaylorImpactTrajectoriesDataset(path, load_stress_stats, num_scales, window_size,
                                                   radius_multiplier, device, graph_builder)
    return torch.utils.data.DataLoader(ds, batch_size=None, shuffle=False, num_workers=num_workers,
                                       pin_memory=pin_memory)
