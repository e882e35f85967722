"""Multi-scale (grid + mesh hierarchy) simulator on the HIP kernels
(sgnn/multi_scale/__init__.py)."""
from .multi_scale_gnn import MultiScaleGNN
from .multi_scale_graph import MultiScaleConfig, MultiScaleGraph, build_static_multi_scale_graph
from .multi_scale_simulator import MultiScaleSimulator

__all__ = ["MultiScaleSimulator", "MultiScaleGraph", "MultiScaleConfig", "MultiScaleGNN",
           "build_static_multi_scale_graph"]
