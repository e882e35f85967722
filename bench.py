#!/usr/bin/env python3
"""Benchmark: particle-steps/s (+ M edge-messages/s) of the 2D Taylor-impact
learned simulator on MI355X (BASELINE.json `metric`).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode rollout|train]
                  [--workload c2|c1_r15|c1_r06]

One "step" of --mode rollout is one autoregressive LearnedSimulator
.predict_positions (radius graph + features + encoder + L interaction layers
+ decoder + Euler + window shift) on inputs already resident in HBM.
Multi-GPU: rollout is "replicas only" (one independent trajectory per rank,
no collective on the data path); value = particles x steps summed over ranks
/ max-over-ranks wall time.  Synthetic lattice data, random-init weights.

Extra keys: "roofline" (dominant kernel = the fused edge layer, timed live
with HIP events on the launch stream) and "cpu_baseline" (the oracle — the
plain-torch CPU restatement of the reference path — on this box's host cores,
rank 0 at N=1 only, bounded sample).
"""
from __future__ import annotations

import argparse
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
    # name: (lattice nx, ny, radius, hidden, layers)
    "c2": (250, 200, 0.6, 64, 5),        # BASELINE configs[1]: ~50k particles, 5 layers, H=64, fp32
    "c1_r15": (50, 40, 15.0, 64, 5),     # configs[0] shape at the BASELINE radius (cap binds)
    "c1_r06": (50, 40, 0.6, 64, 5),      # configs[0] shape at the reference default radius
}
T_SEQ = 11          # config.yaml:20 input_sequence_length
MFMA_F32_PEAK = 157.3e12  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
HBM_PEAK = 8.0e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["rollout"], default="rollout")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--cpu-steps", type=int, default=8, help="oracle steps for cpu_baseline (0: skip)")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args()


def init_dist(args):
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
    return sim.to(device), st


def cpu_baseline(sim, window, radius, L, steps):
    """The oracle (test infrastructure, CPU restatement of the reference) on a
    bounded sample: `steps` autoregressive rollout steps of the same workload."""
    from oracle import sgnn_oracle as O
    state = {k: v.detach().cpu() for k, v in sim.state_dict().items()}
    osim = O.OracleSimulator(state, window.shape[2], L, radius, sim._normalization_stats)
    cur = window.cpu()
    n = cur.shape[0]
    types_ = torch.zeros(n, dtype=torch.long)
    with torch.no_grad():
        nxt, _ = osim.predict_positions(cur, [n], types_)  # warm-up
        cur = torch.cat([cur[:, 1:], nxt[:, None]], 1)
        t0 = time.perf_counter()
        for _ in range(steps):
            nxt, _ = osim.predict_positions(cur, [n], types_)
            cur = torch.cat([cur[:, 1:], nxt[:, None]], 1)
        dt = time.perf_counter() - t0
    cpu_model = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": n * steps / dt, "unit": "particle-steps/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": cpu_model,
            "sample": f"{steps} autoregressive oracle rollout steps (torch CPU fp32 restatement + C "
                      f"cell-list radius search) on the same {n}-particle workload, after 1 warm-up step",
            "seconds": dt}


def profiled_traffic(workload, kernel="k_edge_layer"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/*_summary.json, FETCH_SIZE x2 + WRITE_SIZE), newest matching tag."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json"))):
        d = json.load(open(path))
        if d.get("workload") != workload:
            continue
        for k, v in d["kernels"].items():
            if k.startswith(kernel) and "hbm_bytes" in v:
                best = (v["hbm_bytes"], os.path.relpath(path, ROOT))
    return best


def main():
    args = parse()
    world, rank, local = init_dist(args)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    nx, ny, radius, H, L = WORKLOADS[args.workload]
    dim = 2
    sim, stats = make_sim(H, L, radius, dim, device, args.seed)
    seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny), T_SEQ, seed=1000 + rank)
    n = seq.shape[0]
    window0 = torch.from_numpy(seq)
    types_ = torch.zeros(n, dtype=torch.long, device=device)
    inp, use_emb = sim._step_inputs(window0.to(device), [n], types_)
    ws = sim._workspace(n, T_SEQ, device)
    win = [inp.pos_seq, torch.empty_like(inp.pos_seq)]
    pred = torch.empty(n, dim + 1, device=device)
    next_pos = torch.empty(n, dim, device=device)
    epd = sim._encode_process_decode
    emb_w = sim._particle_type_embedding.weight

    def run(k0, nsteps, timers=None):
        for k in range(k0, k0 + nsteps):
            inp.pos_seq = win[k % 2]
            engine.forward_step(epd, emb_w, use_emb, radius, inp, ws, pred, next_pos,
                                window_out=win[(k + 1) % 2], timers=timers)

    with torch.no_grad():
        run(0, args.warmup)
        torch.cuda.synchronize()
        # pass 1: wall clock of exactly K steps (no instrumentation)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.warmup, args.steps)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        dt = time.perf_counter() - t0
        # pass 2: same K steps with HIP events around every edge-layer launch
        timers = []
        t2 = time.perf_counter()
        run(args.warmup + args.steps, args.steps, timers=timers)
        torch.cuda.synchronize()
        dt_events = time.perf_counter() - t2
    edge_ms = [a.elapsed_time(b) for a, b in timers]
    E = ws.num_edges()
    t = torch.tensor([dt], device=device)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    value = n * args.steps * world / dt
    # dominant kernel: fused edge layer; algorithmic work per launch = E edges x
    # (H x H of the e-block of W1 + H x H of W2) multiply-adds + LayerNorm.
    edge_avg_s = float(np.mean(edge_ms)) * 1e-3
    flops_edge = E * (2 * H * H * 2)
    achieved = flops_edge / edge_avg_s
    prof = profiled_traffic(args.workload)
    out = {
        "metric": "particle-steps/sec (2D Taylor-impact rollout)",
        "value": value,
        "unit": "particle-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (0.5 mm Taylor-bar lattice + random-walk frames; random-init weights)",
        "config": {"workload": f"{args.workload}: 2D lattice {nx}x{ny} = {n} particles/GPU, r={radius}, "
                               f"L={L}, H={H}, T={T_SEQ}, K=20, rollout", "particles": n, "edges": E,
                   "layers": L, "hidden": H, "radius": radius,
                   "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
        "edge_messages_per_s": E * L * args.steps * world / dt,
        "M_edge_messages_per_s": E * L * args.steps * world / dt / 1e6,
        "roofline": {"bound": "mfma", "kernel": "k_edge_layer", "achieved": achieved / 1e12,
                     "peak": MFMA_F32_PEAK / 1e12, "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK,
                     "traffic": prof[0] if prof else None,
                     "traffic_unit": "bytes/launch (rocprofv3 PMC)",
                     "traffic_source": prof[1] if prof else None, "avg_launch_us": edge_avg_s * 1e6,
                     "flops_per_launch": flops_edge,
                     "edge_share_of_step": float(np.sum(edge_ms)) / (dt_events * 1e3)},
    }
    if rank == 0 and world == 1 and args.cpu_steps > 0:
        out["cpu_baseline"] = cpu_baseline(sim, window0, radius, L, args.cpu_steps)
        out["speedup_vs_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
