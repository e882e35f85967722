#!/usr/bin/env python3
"""Benchmark: particle-steps/s (+ M edge-messages/s) of the 2D Taylor-impact
learned simulator on MI355X (BASELINE.json `metric`).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode train|rollout]
                  [--workload c2|c1_r15|c1_r06]

--mode train (default; BASELINE configs[1] "~50k particles, 5 layers,
hidden=64, fp32, forward+backward"): one step = the reference training step
(train.py:231-280): random-walk noise, predict_accelerations forward, loss,
backward, [N>1: RCCL all-reduce of the flat gradient], Adam, LR decay.  Each
rank owns one whole graph (weak scaling, whole-graph DDP over xGMI).
--mode rollout: one step = one autoregressive predict_positions (radius
graph + features + encoder + L layers + decoder + Euler + window shift),
the steps replayed from a captured HIP graph; multi-GPU rollout is replicas
only (no collective).
Inputs are resident in HBM before the timed region.  Synthetic lattice data
and random-init weights (no dataset/checkpoint offline).

Extra keys: "roofline" (dominant kernel, timed live with HIP events on the
launch stream, traffic from the committed rocprofv3 PMC summary),
"cpu_baseline" (the oracle = plain-torch CPU restatement of the reference on
this box's host cores, rank 0 at N=1 only, bounded sample) and "rollout"
(C2 and C1 forward-rollout rates with their own CPU baselines).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sgnn_amd import engine, synthetic  # noqa: E402
from sgnn_amd.learned_simulator import LearnedSimulator  # noqa: E402

WORKLOADS = {
    # name: (lattice dims, radius, hidden, layers)
    "c2": ((250, 200), 0.6, 64, 5),        # BASELINE configs[1]: ~50k particles, 5 layers, H=64, fp32
    "c1_r15": ((50, 40), 15.0, 64, 5),     # configs[0] shape at the BASELINE radius (cap binds)
    "c1_r06": ((50, 40), 0.6, 64, 5),      # configs[0] shape at the reference default radius
    "c4": ((100, 50, 40), 0.75, 128, 10),  # configs[3]: 3D 200k particles, 10 layers, H=128
}
MS_WORKLOADS = {
    # name: (lattice dims, num_scales, window, radius_multiplier, hidden, layers, nmlp_layers)
    "c5": ((100, 100, 100), 2, 2, 2.0, 128, 10, 2),   # configs[4]: multi-scale 3D ~1M per GPU
    "c5_small": ((40, 40, 40), 2, 2, 2.0, 128, 10, 2),
    "ms2d": ((240, 200), 2, 2, 2.0, 128, 10, 2),      # multi_scale_config.yaml widths, 2D
}


def lattice(dims):
    return synthetic.lattice_2d(*dims) if len(dims) == 2 else synthetic.lattice_3d(*dims)
T_SEQ = 11                # config.yaml:20 input_sequence_length
MFMA_F32_PEAK = 157.3e12  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["train", "rollout", "ms-train", "ms-rollout"], default="train")
    ap.add_argument("--workload", choices=sorted(WORKLOADS) + sorted(MS_WORKLOADS), default=None)
    ap.add_argument("--cpu-steps", type=int, default=10, help="oracle steps for cpu_baseline (0: skip)")
    ap.add_argument("--no-rollout-extras", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args()


def init_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def make_sim(H, L, radius, dim, device, seed):
    torch.manual_seed(seed)
    stats = synthetic.normalization_stats(dim, noise_std=0.02)
    st = {k: {kk: torch.tensor(vv) for kk, vv in v.items()} for k, v in stats.items()}
    sim = LearnedSimulator(dim, (T_SEQ - 1) * dim + 1, dim + 1, H, L, 1, H, radius, st, 1, 9,
                           device=device)
    return sim.to(device)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def profiled_traffic(workload, mode, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/r*_summary.json: FETCH_SIZE x2 + WRITE_SIZE), newest matching tag."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json"))):
        d = json.load(open(path))
        if d.get("workload") != workload or d.get("mode", "rollout") != mode:
            continue
        for k, v in d["kernels"].items():
            if k.split("<")[0] == kernel and "hbm_bytes" in v:
                best = (v["hbm_bytes"], os.path.relpath(path, ROOT))
    return best


def sync_barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, device):
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


# ----------------------------------------------------------------------------- rollout
def quiet_decoder(sim):
    """Scale the random-init decoder's output layer by 1e-3 so that the
    autoregressive rollout of an untrained model stays physical (particles
    stay on the lattice, the graph keeps its Taylor-bar connectivity instead
    of collapsing towards the K-cap).  Work per step is unchanged."""
    with torch.no_grad():
        last = [m for m in sim.modules() if isinstance(m, torch.nn.Linear)][-1]
        last.weight.mul_(1e-3)
        last.bias.mul_(1e-3)
    return sim


def rollout_setup(workload, device, seed, rank):
    dims, radius, H, L = WORKLOADS[workload]
    dim = len(dims)
    sim = quiet_decoder(make_sim(H, L, radius, dim, device, seed))
    seq = synthetic.trajectory(lattice(dims), T_SEQ, seed=1000 + rank)
    n = seq.shape[0]
    window0 = torch.from_numpy(seq)
    types_ = torch.zeros(n, dtype=torch.long, device=device)
    inp, use_emb = sim._step_inputs(window0.to(device), [n], types_)
    ws = sim._workspace(n, T_SEQ, device)
    win = [inp.pos_seq, torch.empty_like(inp.pos_seq)]
    pred = torch.empty(n, dim + 1, device=device)
    nxt = torch.empty(n, dim, device=device)

    def run(k0, nsteps, timers=None):
        for k in range(k0, k0 + nsteps):
            inp.pos_seq = win[k % 2]
            engine.forward_step(sim._encode_process_decode, sim._particle_type_embedding.weight, use_emb,
                                radius, inp, ws, pred, nxt, window_out=win[(k + 1) % 2], timers=timers)
    return sim, window0, ws, run, n, radius, H, L


CPU_SAMPLE_DIMS = {"c4": (40, 25, 20)}   # bounded CPU sample (same spacing / radius / model)


def cpu_rollout_baseline(sim, window, radius, L, steps, workload=None):
    """Oracle (test infrastructure: CPU restatement of the reference) rollout."""
    from oracle import sgnn_oracle as O
    state = {k: v.detach().cpu() for k, v in sim.state_dict().items()}
    if workload in CPU_SAMPLE_DIMS:
        window = torch.from_numpy(synthetic.trajectory(lattice(CPU_SAMPLE_DIMS[workload]), T_SEQ, seed=7))
    osim = O.OracleSimulator(state, window.shape[2], L, radius, sim._normalization_stats)
    cur, n = window.cpu(), window.shape[0]
    types_ = torch.zeros(n, dtype=torch.long)
    with torch.no_grad():
        nxt, _ = osim.predict_positions(cur, [n], types_)
        cur = torch.cat([cur[:, 1:], nxt[:, None]], 1)
        t0 = time.perf_counter()
        for _ in range(steps):
            nxt, _ = osim.predict_positions(cur, [n], types_)
            cur = torch.cat([cur[:, 1:], nxt[:, None]], 1)
        dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "particle-steps/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": cpu_model(), "seconds": dt,
            "sample": f"{steps} autoregressive oracle rollout steps (torch CPU fp32 restatement of the "
                      f"reference ops + C cell-list radius search), {n} particles, after 1 warm-up step"}


def bench_rollout(workload, steps, warmup, world, rank, device, seed, cpu_steps):
    """Timed region: `steps` autoregressive steps replayed from a captured HIP
    graph (evaluate.rollout's device path: the same kernels per step, no
    per-kernel launch cost); warm-up = capture + one untimed full rollout."""
    sim, window0, ws, run, n, radius, H, L = rollout_setup(workload, device, seed, rank)
    with torch.no_grad():
        types_ = torch.zeros(n, dtype=torch.long, device=device)
        w0 = window0.to(device)
        runner = sim.rollout_runner(w0, [n], types_, steps)
        for _ in range(max(1, warmup // max(steps, 1))):
            runner.run(w0)
        sync_barrier(world)
        t0 = time.perf_counter()
        runner.run(w0)
        sync_barrier(world)
        dt = time.perf_counter() - t0
        timers = []
        run(0, steps, timers=timers)   # from the initial window (win[0])
        torch.cuda.synchronize()
    dt = max_over_ranks(dt, world, device)
    E = ws.num_edges()
    edge_avg_s = float(np.mean([a.elapsed_time(b) for a, b in timers])) * 1e-3
    flops = E * 4 * H * H
    out = {"workload": f"{workload}: {'x'.join(map(str, WORKLOADS[workload][0]))} lattice = {n} particles/GPU, "
                       f"r={radius}, L={L}, H={H}", "particles": n,
           "edges": E, "value": n * steps * world / dt, "unit": "particle-steps/s",
           "ms_per_step": dt / steps * 1e3,
           "M_edge_messages_per_s": E * L * steps * world / dt / 1e6,
           "edge_kernel_us": edge_avg_s * 1e6, "edge_kernel_mfma_frac": flops / edge_avg_s / MFMA_F32_PEAK}
    if cpu_steps > 0 and rank == 0 and world == 1:
        out["cpu_baseline"] = cpu_rollout_baseline(sim, window0, radius, L, cpu_steps, workload)
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    return out, timers, flops, edge_avg_s, E, n, radius, H, L


# ----------------------------------------------------------------------------- train
def cpu_train_baseline(state, seq, strain, radius, L, steps, stats):
    """Oracle training step (noise + forward + torch autograd + torch Adam) on the CPU."""
    from oracle import sgnn_oracle as O
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in state.items()}
    osim = O.OracleSimulator(params, 2, L, radius, stats)
    osim.p = params
    opt = torch.optim.Adam([p for k, p in params.items() if "embedding" not in k], lr=1e-3)
    pos, nxt = torch.from_numpy(seq[:, :T_SEQ]), torch.from_numpy(seq[:, T_SEQ])
    n = pos.shape[0]
    types_ = torch.zeros(n, dtype=torch.long)

    def step():
        noise = O.random_walk_noise(pos, 0.02)
        pa, ta, ps = osim.predict_accelerations(nxt, noise, pos, [n], types_)
        loss = O.training_loss(pa, ta, ps, strain)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "particle-steps/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": cpu_model(), "seconds": dt,
            "sample": f"{steps} oracle training steps (noise + forward + torch autograd backward + Adam, "
                      f"torch CPU fp32 restatement of the reference ops), {n} particles, after 1 warm-up"}


def bench_train(args, world, rank, device):
    from sgnn_amd.train import Trainer
    dims, radius, H, L = WORKLOADS[args.workload]
    nx, ny = dims
    sim = make_sim(H, L, radius, 2, device, args.seed)
    state0 = {k: v.detach().cpu().clone() for k, v in sim.state_dict().items()}
    seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny), T_SEQ + 1, seed=2000 + rank)
    n = seq.shape[0]
    pos = torch.from_numpy(seq[:, :T_SEQ]).to(device)
    nxt = torch.from_numpy(seq[:, T_SEQ]).to(device)
    strain_np = np.random.default_rng(rank).normal(0, 1, n).astype(np.float32)
    strain = torch.from_numpy(strain_np).to(device)
    tr = Trainer(sim, lr_init=1e-3)
    for _ in range(args.warmup):
        tr.train_step(pos, nxt, strain, [n])
    sync_barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = tr.train_step(pos, nxt, strain, [n])
    sync_barrier(world)
    dt = time.perf_counter() - t0
    timers = {}
    t2 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step(pos, nxt, strain, [n], timers=timers)
    torch.cuda.synchronize()
    dt_ev = time.perf_counter() - t2
    dt = max_over_ranks(dt, world, device)
    tw = tr.workspace(n, T_SEQ, device)
    E = tw.f.num_edges()
    loss = float(out["loss"])
    kstats = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e-3 for k, v in timers.items()}
    # dominant kernel by total time: the edge-layer backward: W2^T dy, dW2 += dy h^T
    # (H = 64: dE0 and dW1e of all layers are formed afterwards by
    # k_edge_latent_grad; H = 128 adds W1e^T dh and dW1e += dh e0^T in-layer)
    dom = "k_edge_bwd"
    flops_bwd = E * (4 if tw.latent_pass else 8) * H * H
    achieved = flops_bwd / kstats[dom]
    prof = profiled_traffic(args.workload, "train", dom)
    res = {
        "metric": "particle-steps/sec (2D Taylor-impact, training fwd+bwd+Adam)",
        "value": n * args.steps * world / dt,
        "unit": "particle-steps/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (0.5 mm Taylor-bar lattice + random-walk frames, random-walk training "
                "noise; random-init weights)",
        "config": {"workload": f"{args.workload}: 2D lattice {nx}x{ny} = {n} particles per GPU, r={radius}, "
                               f"L={L}, H={H}, T={T_SEQ}, K=20, training step (noise+fwd+bwd+Adam)",
                   "particles_per_gpu": n, "edges_per_gpu": E, "global_batch_graphs": world,
                   "layers": L, "hidden": H, "radius": radius,
                   "parallelism": f"dp{world} (whole-graph, RCCL all-reduce)" if world > 1 else "single GPU"},
        "M_edge_messages_per_s": E * L * args.steps * world / dt / 1e6,
        "final_loss": loss,
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": achieved / 1e12,
                     "peak": MFMA_F32_PEAK / 1e12, "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK,
                     "traffic": prof[0] if prof else None,
                     "traffic_unit": "HBM bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": prof[1] if prof else None,
                     "avg_launch_us": kstats[dom] * 1e6, "flops_per_launch": flops_bwd,
                     "share_of_step": float(np.sum([a.elapsed_time(b) for a, b in timers[dom]])) / (dt_ev * 1e3)},
        "kernel_avg_us": {k: v * 1e6 for k, v in kstats.items()},
    }
    if rank == 0 and world == 1 and args.cpu_steps > 0:
        res["cpu_baseline"] = cpu_train_baseline(state0, seq, torch.from_numpy(strain_np), radius, L,
                                                 args.cpu_steps, sim._normalization_stats)
        res["speedup_vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    return res


# ----------------------------------------------------------------------------- multi-scale
def ms_setup(workload, device, seed, rank, nframes):
    from sgnn_amd.multi_scale import MultiScaleSimulator, build_static_multi_scale_graph
    dims, ns, win, mult, H, L, nmlp = MS_WORKLOADS[workload]
    dim = len(dims)
    torch.manual_seed(seed)
    stats = synthetic.normalization_stats(dim, noise_std=0.02)
    st = {k: {kk: torch.tensor(vv) for kk, vv in v.items()} for k, v in stats.items()}
    sim = MultiScaleSimulator(dim, (T_SEQ - 1) * dim + 1, dim + 1, H, H, L, nmlp, st, 1, 9, ns, win, mult,
                              device=str(device)).to(device)
    base = lattice(dims)
    base[:, 0] -= 2.0   # bar starts at the wall (x = -2): the wall feature is active
    seq = synthetic.trajectory(base, nframes, seed=3000 + rank)
    graph = build_static_multi_scale_graph(torch.from_numpy(seq[:, 0]).to(device), ns, win, mult)
    sim.set_static_graph(graph)
    edges = {k: int(graph[k].shape[1]) for k in ("grid2mesh_edges", "mesh2mesh_edges", "mesh2grid_edges")}
    desc = (f"{workload}: multi-scale {'x'.join(map(str, dims))} lattice = {seq.shape[0]} particles/GPU, "
            f"num_scales={ns}, window={win}, radius_multiplier={mult}, L={L} M2M blocks, H={H}, "
            f"nmlp_layers={nmlp}, T={T_SEQ}; edges g2m/m2m/m2g = {edges['grid2mesh_edges']}/"
            f"{edges['mesh2mesh_edges']}/{edges['mesh2grid_edges']}")
    return sim, seq, edges, desc, (dims, ns, win, mult, H, L, nmlp)


def ms_block_edges(edges, L):
    return edges["grid2mesh_edges"] + L * edges["mesh2mesh_edges"] + edges["mesh2grid_edges"]


def cpu_ms_train_baseline(sim, cfg, steps):
    """Oracle multi-scale training step (forward + torch autograd + Adam) on a
    bounded CPU sample of the same model (smaller lattice)."""
    from oracle import multi_scale_oracle as MO
    from oracle import sgnn_oracle as O
    dims, ns, win, mult, H, L, nmlp = cfg
    sdims = (24, 24, 16) if len(dims) == 3 else (60, 40)
    base = lattice(sdims)
    base[:, 0] -= 2.0
    seq = synthetic.trajectory(base, T_SEQ + 1, seed=9)
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in sim.state_dict().items()}
    graph = MO.create_all_edges(torch.from_numpy(seq[:, 0]), ns, win, mult)
    osim = MO.MultiScaleOracle(params, len(dims), L, sim._normalization_stats, graph, ns, mult, 1, nmlp)
    opt = torch.optim.Adam([p for k, p in params.items() if "embedding" not in k], lr=1e-3)
    pos, nxt = torch.from_numpy(seq[:, :T_SEQ]), torch.from_numpy(seq[:, T_SEQ])
    n = pos.shape[0]
    strain = torch.zeros(n)

    def step():
        noise = O.random_walk_noise(pos, 0.02)
        pa, ta, ps = osim.predict_accelerations(nxt, noise, pos)
        loss = O.training_loss(pa, ta, ps, strain)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "particle-steps/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": cpu_model(), "seconds": dt,
            "sample": f"{steps} oracle multi-scale training steps (forward + torch autograd + Adam, torch "
                      f"CPU fp32 restatement of sgnn/multi_scale) on a {'x'.join(map(str, sdims))} lattice "
                      f"= {n} particles, same model, after 1 warm-up"}


def bench_ms_train(args, world, rank, device):
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    sim, seq, edges, desc, cfg = ms_setup(args.workload, device, args.seed, rank, T_SEQ + 1)
    n = seq.shape[0]
    H, L = cfg[4], cfg[5]
    pos = torch.from_numpy(seq[:, :T_SEQ]).to(device)
    nxt = torch.from_numpy(seq[:, T_SEQ]).to(device)
    strain = torch.from_numpy(np.random.default_rng(rank).normal(0, 1, n).astype(np.float32)).to(device)
    tr = MultiScaleTrainer(sim, lr_init=1e-3)
    for _ in range(args.warmup):
        tr.train_step(pos, nxt, strain)
    sync_barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = tr.train_step(pos, nxt, strain)
    sync_barrier(world)
    dt = time.perf_counter() - t0
    timers = {}
    for _ in range(min(args.steps, 3)):
        tr.train_step(pos, nxt, strain, timers=timers)
    torch.cuda.synchronize()
    dt = max_over_ranks(dt, world, device)
    kstats = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e-3 for k, v in timers.items()}
    nmlp = cfg[6]
    eb = ms_block_edges(edges, L)
    # edge backward per edge: last (+ middle) Linear W^T dy and dW, W1e^T dh and dW1e
    flops_bwd = eb / (L + 2) * (8 + (4 if nmlp == 2 else 0)) * H * H
    dom = "k_edge_bwd"
    achieved = flops_bwd / kstats[dom]
    res = {
        "metric": "particle-steps/sec (multi-scale training fwd+bwd+Adam)",
        "value": n * args.steps * world / dt, "unit": "particle-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (0.5 mm lattice + random-walk frames; random-init weights)",
        "config": {"workload": desc + ", training step (noise+fwd+bwd+Adam)", "particles_per_gpu": n,
                   "edge_evaluations_per_step": eb, "global_batch_graphs": world,
                   "parallelism": f"dp{world} (whole-graph, RCCL all-reduce)" if world > 1 else "single GPU"},
        "M_edge_messages_per_s": eb * args.steps * world / dt / 1e6,
        "final_loss": float(out["loss"]),
        "hbm_peak_gib": torch.cuda.max_memory_allocated(device) / 2 ** 30,
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": achieved / 1e12, "peak": MFMA_F32_PEAK / 1e12,
                     "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK, "traffic": None,
                     "avg_launch_us": kstats[dom] * 1e6, "flops_per_launch": flops_bwd},
        "kernel_avg_us": {k: v * 1e6 for k, v in kstats.items()},
    }
    if rank == 0 and world == 1 and args.cpu_steps > 0:
        res["cpu_baseline"] = cpu_ms_train_baseline(sim, cfg, max(1, args.cpu_steps // 3))
        res["speedup_vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    return res


def bench_ms_rollout(args, world, rank, device):
    sim, seq, edges, desc, cfg = ms_setup(args.workload, device, args.seed, rank, T_SEQ)
    n = seq.shape[0]
    L = cfg[5]
    cur = torch.from_numpy(seq).to(device).contiguous()
    nxt_win = torch.empty_like(cur)
    types_ = None

    def run(k):
        nonlocal cur, nxt_win
        for _ in range(k):
            sim._run(cur, types_, window_out=nxt_win)
            cur, nxt_win = nxt_win, cur

    with torch.no_grad():
        run(args.warmup)
        sync_barrier(world)
        t0 = time.perf_counter()
        run(args.steps)
        sync_barrier(world)
        dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, world, device)
    eb = ms_block_edges(edges, L)
    return {"metric": "particle-steps/sec (multi-scale rollout)", "value": n * args.steps * world / dt,
            "unit": "particle-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (0.5 mm lattice + random-walk frames; random-init weights)",
            "config": {"workload": desc + ", rollout", "particles": n,
                       "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
            "M_edge_messages_per_s": eb * args.steps * world / dt / 1e6}


def main():
    args = parse()
    world, rank, local = init_dist()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if args.workload is None:
        args.workload = "c5" if args.mode.startswith("ms") else "c2"
    if args.mode == "ms-train":
        res = bench_ms_train(args, world, rank, device)
    elif args.mode == "ms-rollout":
        res = bench_ms_rollout(args, world, rank, device)
    elif args.mode == "train":
        res = bench_train(args, world, rank, device)
        if not args.no_rollout_extras and world == 1:
            # the other BASELINE configs, each with its own bounded CPU baseline
            res["rollout"] = {}
            for wl, cs in (("c2", 2), ("c1_r15", 3), ("c4", 1)):
                r = bench_rollout(wl, 20 if wl != "c4" else 10, 3, world, rank, device, args.seed,
                                  cs if args.cpu_steps > 0 else 0)[0]
                res["rollout"][wl] = r
            import argparse as _ap
            ms_args = _ap.Namespace(**{**vars(args), "workload": "c5", "steps": 3, "warmup": 1})
            ms = bench_ms_train(ms_args, world, rank, device)
            res["multi_scale_c5_train"] = {k: ms[k] for k in ("value", "unit", "ms_per_step", "config",
                                                              "M_edge_messages_per_s", "hbm_peak_gib",
                                                              "roofline", "cpu_baseline", "speedup_vs_cpu")
                                           if k in ms}
    else:
        r, timers, flops, edge_avg_s, E, n, radius, H, L = bench_rollout(
            args.workload, args.steps, args.warmup, world, rank, device, args.seed, args.cpu_steps)
        prof = profiled_traffic(args.workload, "rollout", "k_edge_layer")
        res = {"metric": "particle-steps/sec (2D Taylor-impact rollout)", "value": r["value"],
               "unit": "particle-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": r["ms_per_step"], "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (0.5 mm Taylor-bar lattice + random-walk frames; random-init weights)",
               "config": {"workload": r["workload"] + ", rollout", "particles": n, "edges": E,
                          "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
               "M_edge_messages_per_s": r["M_edge_messages_per_s"],
               "roofline": {"bound": "mfma", "kernel": "k_edge_layer", "achieved": flops / edge_avg_s / 1e12,
                            "peak": MFMA_F32_PEAK / 1e12, "unit": "TFLOP/s",
                            "frac": flops / edge_avg_s / MFMA_F32_PEAK,
                            "traffic": prof[0] if prof else None,
                            "traffic_unit": "HBM bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                            "traffic_source": prof[1] if prof else None,
                            "avg_launch_us": edge_avg_s * 1e6, "flops_per_launch": flops}}
        if "cpu_baseline" in r:
            res["cpu_baseline"] = r["cpu_baseline"]
            res["speedup_vs_cpu"] = r["speedup_vs_cpu"]
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
