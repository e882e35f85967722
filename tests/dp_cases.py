"""Shared cases of the multi-rank GPU training test (tests/test_gpu_dp.py):
whole-graph data parallelism of the HIP trainers with ragged, real-size
graphs, run identically by the single-process reference run and by every
rank (tests/gpu_dp_child.py).  Noise is drawn on the CPU from seeded
generators, so every process sees the same windows."""
from __future__ import annotations

import numpy as np
import torch

LR = 1e-3
STEPS = 2
# single scale: the real Taylor-bar sizes (120/160/200 x 40 lattices = 4,800 / 6,400 / 8,000 particles)
SS_GRAPHS = [(120, 40), (160, 40), (200, 40), (100, 40), (160, 40), (200, 40), (120, 40), (160, 40),
             (250, 100), (250, 100)]
SS_RANKS = [[0, 1], [2]]          # rank 0 holds two graphs (4,800 + 6,400), rank 1 one (8,000)
SS_RANKS4 = [[0], [1], [2], [3]]  # four ranks, one graph each (4,800 / 6,400 / 8,000 / 4,000)
# C3 at its own shape (BASELINE configs[2], train.py:257-273): a global batch of 8 real-size Taylor graphs,
# one whole graph per rank, 8 ranks -- 4,800 / 6,400 / 8,000 / 4,000 / 6,400 / 8,000 / 4,800 / 6,400
SS_RANKS8 = [[g] for g in range(8)]
# the C2 graph size split over two ranks: 250 x 100 = 25,000 particles each (C2 is 250 x 200 = 50,000)
SS_RANKS_C2 = [[8], [9]]
# multi scale (nmlp_layers 2, two scales): one graph per rank, unequal sizes
MS_GRAPHS = [(30, 14), (36, 12), (28, 15), (33, 12)]
MS_RANKS = [[0], [1]]
MS_RANKS4 = [[0], [1], [2], [3]]
T_SS, T_MS = 11, 6


def _stats(dim=2):
    from sgnn_amd import synthetic
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    return {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}


def _window(nx, ny, T, seed, x0=0.25):
    """(window [n,T,2], next position [n,2], next strain [n], noise [n,T,2]) on the CPU."""
    from oracle import sgnn_oracle as O
    from sgnn_amd import synthetic
    seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny, x0=x0), T + STEPS, seed=seed)
    out = []
    for s in range(STEPS):
        pos = torch.from_numpy(np.ascontiguousarray(seq[:, s:s + T]))
        nxt = torch.from_numpy(np.ascontiguousarray(seq[:, s + T]))
        strain = torch.from_numpy(np.random.default_rng(seed + s).normal(0, 1, seq.shape[0]).astype(np.float32))
        noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(seed * 7 + s))
        out.append((pos, nxt, strain, noise))
    return out


def _cat(items):
    return [torch.cat([it[k] for it in items], 0) for k in range(4)]


def _result(tr, losses, sim):
    return {"loss": torch.tensor(losses, dtype=torch.float64), "grad": tr.flat.grad.detach().cpu().clone(),
            "param": tr.flat.param.detach().cpu().clone(),
            "names": [(name, p.numel()) for name, p in sim.named_parameters()]}   # the flat layout


def run_single_scale(graph_ids, overlap=False, force=False):
    """STEPS Trainer steps on the concatenation of `graph_ids` (this process's
    share of the global batch); DP bookkeeping from the default process group.
    overlap: the per-layer gradient buckets go out asynchronously on the side
    stream during the backward (the RCCL path), here through gloo's own
    device-tensor all-reduce instead of the host staging."""
    from sgnn_amd.learned_simulator import LearnedSimulator
    from sgnn_amd.train import Trainer
    torch.manual_seed(7)
    sim = LearnedSimulator(2, 21, 3, 64, 5, 1, 64, 0.6, _stats(), 1, 9).cuda()
    tr = Trainer(sim, lr_init=LR)
    if overlap:
        tr.dp.host_staging = False
        tr.dp.force_overlap = force
        assert tr.dp.world == 1 or tr.dp.overlaps_buckets()
    wins = {g: _window(*SS_GRAPHS[g], T_SS, 100 + g) for g in graph_ids}
    losses = []
    for s in range(STEPS):
        parts = [wins[g][s] for g in graph_ids]
        pos, nxt, strain, noise = _cat(parts)
        counts = [p[0].shape[0] for p in parts]
        out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), counts, noise=noise.cuda())
        losses.append(float(out["loss"]))
    torch.cuda.synchronize()
    return _result(tr, losses, sim)


def run_multi_scale(graph_ids, overlap=False, force=False, global_ids=None):
    """STEPS MultiScaleTrainer steps on `graph_ids` (one static graph each,
    merged block-diagonally when a process holds several).  overlap: the
    per-block gradient buckets go out asynchronously from the side stream
    during the backward (as run_single_scale).  global_ids: the whole global
    batch (every rank's graphs in rank order): (n_global, particle_offset) are
    then passed host-side, as train() does, so the 1/N_global scaling sits
    inside the backward exactly as in the one-process run -- these small 2D
    multi-scale graphs are too ill-conditioned in fp32 for the deferred count
    path's different rounding (its scaling after the sum all-reduce) to stay
    inside the gradient bound; the single-scale cases exercise that path."""
    from sgnn_amd.multi_scale import MultiScaleSimulator
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    from sgnn_amd.multi_scale.multi_scale_graph import build_static_multi_scale_graph
    from sgnn_amd.multi_scale.static_graph_data_loader import merge_static_graphs
    torch.manual_seed(5)
    sim = MultiScaleSimulator(2, (T_MS - 1) * 2 + 1, 3, 64, 64, 3, 2, _stats(), 1, 9, 2, 2, 2.0).cuda()
    wins = [_window(nx, ny, T_MS, 300 + g, x0=-1.75) for g, (nx, ny) in enumerate(MS_GRAPHS)]
    graphs = [build_static_multi_scale_graph(wins[g][0][0][:, 0].cuda(), 2, 2, 2.0) for g in graph_ids]
    counts = [wins[g][0][0].shape[0] for g in graph_ids]
    sim.set_static_graph(graphs[0] if len(graphs) == 1 else merge_static_graphs(graphs, counts))
    tr = MultiScaleTrainer(sim, lr_init=LR)
    if overlap:
        tr.dp.host_staging = False
        tr.dp.force_overlap = force
        assert tr.dp.world == 1 or tr.dp.overlaps_buckets()
    kw = {}
    if global_ids is not None:
        sizes = {g: MS_GRAPHS[g][0] * MS_GRAPHS[g][1] for g in global_ids}
        first = global_ids.index(graph_ids[0])
        kw = dict(n_global=sum(sizes.values()), particle_offset=sum(sizes[g] for g in global_ids[:first]))
    losses = []
    for s in range(STEPS):
        pos, nxt, strain, noise = _cat([wins[g][s] for g in graph_ids])
        if kw:
            assert sum(MS_GRAPHS[g][0] * MS_GRAPHS[g][1] for g in graph_ids) == pos.shape[0]
        out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), noise=noise.cuda(), **kw)
        losses.append(float(out["loss"]))
    torch.cuda.synchronize()
    return _result(tr, losses, sim)


def run_single_scale_overlap(graph_ids):
    return run_single_scale(graph_ids, overlap=True)


def run_single_scale_rccl(graph_ids):
    """The overlapped bucket path on a one-rank RCCL (nccl) group: every layer's bucket goes out
    with dist.all_reduce(async_op=True) from the side stream during the backward, the launch stream
    waits on the handles before Adam -- the C3 / C5 collective path on real RCCL."""
    import torch.distributed as dist
    if dist.is_initialized():
        assert dist.get_backend() == "nccl"
    return run_single_scale(graph_ids, overlap=True, force=dist.is_initialized())


def run_multi_scale_overlap(graph_ids, global_ids=None):
    return run_multi_scale(graph_ids, overlap=True, global_ids=global_ids)


def run_multi_scale_rccl(graph_ids, global_ids=None):
    """The multi-scale trainer's per-block buckets on a one-rank RCCL (nccl) group (C5's collective
    path), as run_single_scale_rccl."""
    import torch.distributed as dist
    if dist.is_initialized():
        assert dist.get_backend() == "nccl"
    return run_multi_scale(graph_ids, overlap=True, force=dist.is_initialized(), global_ids=global_ids)


CASES = {"ss": (run_single_scale, SS_GRAPHS, SS_RANKS), "ms": (run_multi_scale, MS_GRAPHS, MS_RANKS),
         "ss_overlap": (run_single_scale_overlap, SS_GRAPHS, SS_RANKS),
         "ss_rccl1": (run_single_scale_rccl, SS_GRAPHS, [[0, 1, 2]]),
         "ms_overlap": (run_multi_scale_overlap, MS_GRAPHS, MS_RANKS),
         "ms_rccl1": (run_multi_scale_rccl, MS_GRAPHS, [[0, 1]]),
         # four ranks (the C3 / C5 sharding at world 4; gloo, the ranks share the one leased GPU)
         "ss4_overlap": (run_single_scale_overlap, SS_GRAPHS, SS_RANKS4),
         "ss8": (run_single_scale_overlap, SS_GRAPHS, SS_RANKS8),
         "ss_c2": (run_single_scale_overlap, SS_GRAPHS, SS_RANKS_C2),
         "ms4": (run_multi_scale, MS_GRAPHS, MS_RANKS4)}
RCCL_CASES = {"ss_rccl1", "ms_rccl1"}
MS_CASES = {"ms", "ms_overlap", "ms_rccl1", "ms4"}   # run(..., global_ids=...): host-side counts
