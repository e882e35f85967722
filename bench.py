#!/usr/bin/env python3
"""Benchmark: particle-steps/s + M edge-messages/s of the 2D Taylor-impact
learned-simulator ROLLOUT on MI355X (BASELINE.json `metric`), with the
1/2/4/8-GPU training curve and the other BASELINE configs as extras.

  python bench.py [--gpus N] [--steps K] [--warmup W]
                  [--mode rollout|train|train-c3|ms-train|ms-rollout] [--workload ...]

Default (`--mode rollout --workload c1_r15`, BASELINE.md §3's 10x config):
one step = one autoregressive `predict_positions` (radius graph + features +
encoder + 5 InteractionNetworks + decoder + Euler + window shift) on a
2,000-particle 2D Taylor-bar lattice at r = 15 (cap K = 20 binds), the loop of
evaluate.py:117-145 issued as ONE `sgnn_rollout` C call.  Inputs are resident
in HBM before the timed region.  With N > 1 every rank rolls out its own
trajectory (rollout shards as replicas only) and `value`
counts all ranks' particle-steps over the max-over-ranks time.

Extras in the same JSON line (every N):
  "training"      C2 training step (noise + fwd + bwd + RCCL all-reduce + Adam),
                  50k particles per rank, whole-graph DDP: weak scaling.  This
                  is the north_star's 1/2/4/8-GPU training curve.
  "training_c3"   C3: global batch of 8 real-size graphs (4,800/6,400/8,000
                  particles) split over the N ranks: strong scaling.
  "rollout_extra" C2 (50k, r = 0.6), C1 at r = 0.6, the real Taylor-bar sizes
                  (4,800 / 6,400 / 8,000 particles, r = 0.6) and C4 (3D 200k,
                  L = 10, H = 128) rollouts (replicas at N > 1).
  "multi_scale_c5_train"  C5: multi-scale 3D 1M particles per rank, DDP.
CPU baselines (rank 0 at N = 1 only): the oracle (plain-torch CPU restatement
of the reference, test infrastructure) on this box's host cores; >= 20 timed
rollout steps after one warm-up; training legs bounded to ~10-30 s.

`--gpus N` without a torch.distributed environment re-launches this script
under `python -m torch.distributed.run --nproc-per-node N` as a CHILD process
(before anything touches the GPU) and exits with its status.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sgnn_amd import synthetic  # noqa: E402

WORKLOADS = {
    # name: (lattice dims, radius, hidden, layers)
    "c2": ((250, 200), 0.6, 64, 5),        # BASELINE configs[1]: ~50k particles, 5 layers, H=64, fp32
    "c1_r15": ((50, 40), 15.0, 64, 5),     # configs[0] shape at the BASELINE radius (cap binds)
    "c1_r06": ((50, 40), 0.6, 64, 5),      # configs[0] shape at the reference default radius
    "c4": ((100, 50, 40), 0.75, 128, 10),  # configs[3]: 3D 200k particles, 10 layers, H=128
    # the real Taylor-bar sizes: 60/80/100 mm x 20 mm bars at 0.5 mm, default radius
    "t4800": ((120, 40), 0.6, 64, 5),
    "t6400": ((160, 40), 0.6, 64, 5),
    "t8000": ((200, 40), 0.6, 64, 5),
}
MS_WORKLOADS = {
    # name: (lattice dims, num_scales, window, radius_multiplier, hidden, layers, nmlp_layers)
    "c5": ((100, 100, 100), 2, 2, 2.0, 128, 10, 2),   # configs[4]: multi-scale 3D ~1M per GPU
    "c5_small": ((40, 40, 40), 2, 2, 2.0, 128, 10, 2),
    "ms2d": ((240, 200), 2, 2, 2.0, 128, 10, 2),      # multi_scale_config.yaml widths, 2D
}
# C3 (BASELINE configs[2]): global batch of 8 whole graphs at the real Taylor
# bar sizes (120/160/200 x 40 lattices = 4,800/6,400/8,000 particles)
C3_GRAPHS = [(120, 40), (160, 40), (200, 40), (120, 40), (160, 40), (200, 40), (120, 40), (160, 40)]

T_SEQ = 11                # config.yaml:20 input_sequence_length
MFMA_F32_PEAK = 157.3e12  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
HBM_PEAK = 8.0e12         # MI355X HBM3E bytes/s (MI355X_MICROARCH.md)
DATA = "synthetic (0.5 mm Taylor-bar lattice + random-walk frames; random-init weights)"


def progress(msg):
    """One progress line on stderr per bench leg (a long default run keeps
    writing, and the log shows where time went)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def lattice(dims):
    return synthetic.lattice_2d(*dims) if len(dims) == 2 else synthetic.lattice_3d(*dims)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["rollout", "train", "train-c3", "ms-train", "ms-rollout"],
                    default="rollout")
    ap.add_argument("--workload", choices=sorted(WORKLOADS) + sorted(MS_WORKLOADS), default=None)
    ap.add_argument("--cpu-steps", type=int, default=20,
                    help="timed oracle rollout steps for cpu_baseline (0: skip); training legs use fewer")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="the headline cpu_baseline keeps stepping until this much CPU work (<= 20x --cpu-steps)")
    ap.add_argument("--no-extras", "--no-rollout-extras", dest="no_extras", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--selftest-launch", action="store_true",
                    help="launcher self-test: gloo on CPU, a stub step, no GPU (tests/test_bench_launch.py)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launch / dist
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_workers(args, argv) -> int:
    """`--gpus N` outside a torch.distributed environment: start N ranks with
    torch.distributed.run as a child process (this parent never initialises
    HIP, so nothing is exec'd over a GPU context) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N ranks with "
                         f"torch.distributed.run --nproc-per-node N, or pass only --gpus N")
    if world > 1:
        if args.selftest_launch:
            torch.distributed.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def sync_barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, device):
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, device):
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(t)
    return float(t.item())


def selftest_launch(world, rank):
    """Stub step for the launcher test: one gloo all-reduce, no GPU."""
    t = torch.ones(1)
    if world > 1:
        torch.distributed.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": "selftest", "n_gpus": world, "allreduce_sum": float(t.item()),
                          "ranks_env": os.environ.get("WORLD_SIZE")}))
    if world > 1:
        torch.distributed.destroy_process_group()


# ----------------------------------------------------------------------------- CPU baseline helpers
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_threads(n=None) -> dict:
    """Threads for a CPU baseline leg: `n`, or every core this process may run
    on (sched_getaffinity -- BASELINE.md §3's os.cpu_count() restricted to what
    the process may use) capped by OMP_NUM_THREADS when the environment sets it
    (on the GPU box that is the box's CPU share, while os.cpu_count() shows the
    whole host).  Reported with the raw counts."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if n is None:
        n = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    torch.set_num_threads(n)
    return {"cores": torch.get_num_threads(), "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": omp, "cpu_model": cpu_model(), "kind": "port"}


def thread_counts():
    """The CPU-leg thread counts: the box's share (OMP_NUM_THREADS) and every
    CPU of the affinity mask (BASELINE.md §3's os.cpu_count()), when they
    differ -- the affinity leg only while it is at most 4x the share: on the GPU
    box the mask shows the whole host (256 CPUs) but the job gets a 16-CPU
    share, and 256 OpenMP threads on 16 CPUs did not finish one step in 3
    minutes.  Returns (counts, note on any leg left out)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    share = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    if aff > 4 * share:
        return [share], (f"affinity leg ({aff} threads) not timed: {aff} OpenMP threads on this job's "
                         f"{share}-CPU share (OMP_NUM_THREADS) oversubscribe it")
    return sorted({share, aff}), None


def profiled(workload, mode, kernel):
    """Per-launch HBM bytes and duration of `kernel` from the newest committed
    rocprofv3 summary (profiles/r*_summary.json: FETCH_SIZE x2 + WRITE_SIZE).
    `kernel` is a name (all its template variants, weighted by launches) or a
    composite "a + 3 b<..>" (one launch of a plus three of b<..>, exact names:
    a timed region that issues several kernels)."""
    parts = []
    for term in kernel.split(" + "):
        mult, _, name = term.partition(" ") if term.split(" ")[0].isdigit() else ("1", "", term)
        parts.append((int(mult), name.strip()))
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json"))):
        d = json.load(open(path))
        if d.get("workload") != workload or d.get("mode", "rollout") != mode:
            continue
        tot_b = tot_us = 0.0
        ok = True
        for mult, name in parts:
            exact = "<" in name or len(parts) > 1
            ks = [v for k, v in d["kernels"].items()
                  if (k == name if exact else k.split("<")[0] == name) and "hbm_bytes" in v]
            if not ks:
                ok = False
                break
            calls = sum(v["calls"] for v in ks)
            tot_b += mult * sum(v["hbm_bytes"] * v["calls"] for v in ks) / calls
            tot_us += mult * sum(v["avg_us"] * v["calls"] for v in ks) / calls
        if ok:
            best = {"bytes": tot_b, "avg_us": tot_us, "source": os.path.relpath(path, ROOT)}
    return best


def roofline(kernel, flops, avg_s, workload, mode, alg_bytes=None, executed_flops=None, whole=True):
    """The dominant kernel against the dense fp32 MFMA peak.  `whole`: the launch
    does whole layers / the whole step (k_step16, k_layer16), so `frac` is
    SURVEY.md §8(d)'s ALGORITHMIC FLOPs per launch / the live average launch
    time, with `exe_frac` the FLOPs it actually multiplies (the
    u/v factorisation removes 2H^2 of every edge's first Linear).  A split kernel
    (k_edge_layer: the node kernel forms the u/v half of the first edge Linear;
    the backward kernels) is charged only what it executes: `frac` = executed
    FLOPs / time (§8(d) per edge inflated the edge kernel past the
    peak); the whole-step §8(d) rate sits beside it in the leg (`alg_step_tflops`).
    `traffic` = HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE) and
    `prof_us` the trace-mode duration, both from this round's profiles/ summary."""
    prof = profiled(workload, mode, kernel)
    exe = flops if executed_flops is None else executed_flops
    charged = flops if whole else exe
    frac = charged / avg_s / MFMA_F32_PEAK
    r = {"bound": "mfma", "kernel": kernel, "achieved": charged / avg_s / 1e12, "peak": MFMA_F32_PEAK / 1e12,
         "unit": "TFLOP/s", "frac": frac, "flops": "8d" if whole else "executed",
         "exe_frac": exe / avg_s / MFMA_F32_PEAK, "flops_per_launch": charged,
         "traffic": prof["bytes"] if prof else None, "live_us": avg_s * 1e6}
    if prof:
        r["prof_us"] = prof["avg_us"]
        r["src"] = os.path.basename(prof["source"])
        # achieved HBM bandwidth of the same launch (north_star: "achieved-HBM-fraction"): the profiled
        # bytes over the profiled (trace-mode) duration, against the ~8 TB/s HBM3E peak
        r["hbm_gbs"] = prof["bytes"] / (prof["avg_us"] * 1e-6) / 1e9
        r["hbm_frac"] = r["hbm_gbs"] * 1e9 / HBM_PEAK
    if alg_bytes is not None:
        r["alg_bytes"] = alg_bytes
    if frac > 1.0:
        # physically impossible: the leg is marked invalid and its fraction withheld; one
        # noisy leg does not discard the whole line, and bench_line_errors() lists it
        r["error"] = f"frac {frac:.3f} > 1: the FLOP count or the timing is wrong"
        r["invalid_frac"], r["frac"], r["achieved"] = frac, None, None
    return r


def bench_line_errors(line) -> list:
    """Every leg of a bench line whose roofline carries an error (tests assert this is empty)."""
    bad = []

    def walk(d, path):
        if isinstance(d, dict):
            if "error" in d:
                bad.append((path, d["error"]))
            for k, v in d.items():
                walk(v, f"{path}.{k}" if path else k)
    walk(line, "")
    return bad


def _r(x):
    """4 significant digits (the JSON line stays a few KB)."""
    if isinstance(x, float):
        return float(f"{x:.4g}")
    if isinstance(x, dict):
        return {k: _r(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_r(v) for v in x]
    return x


def leg(r):
    """An extra leg of the line, numbers only (the contract keys live at the top level)."""
    out = {k: r[k] for k in ("value", "ms_per_step", "M_edge_messages_per_s", "particles", "edges",
                             "hbm_peak_gib", "final_loss", "alg_step_tflops", "scaling") if k in r}
    if "roofline" in r:
        rf = r["roofline"]
        out["rf"] = {k: rf[k] for k in ("kernel", "frac", "flops", "exe_frac", "traffic", "alg_bytes", "live_us",
                                        "prof_us", "hbm_frac", "src", "error", "invalid_frac") if k in rf}
    if "cpu_baseline" in r:
        out["cpu"] = {k: r["cpu_baseline"][k] for k in ("value", "cores", "sample")}
        out["x_cpu"] = r["speedup_vs_cpu"]
    return out


# ----------------------------------------------------------------------------- models / data
def make_sim(H, L, radius, dim, device, seed):
    from sgnn_amd.learned_simulator import LearnedSimulator
    torch.manual_seed(seed)
    stats = synthetic.normalization_stats(dim, noise_std=0.02)
    st = {k: {kk: torch.tensor(vv) for kk, vv in v.items()} for k, v in stats.items()}
    sim = LearnedSimulator(dim, (T_SEQ - 1) * dim + 1, dim + 1, H, L, 1, H, radius, st, 1, 9,
                           device=device)
    return sim.to(device)


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


# ----------------------------------------------------------------------------- rollout
CPU_SAMPLE_DIMS = {}   # workload -> a bounded CPU sample (same spacing / radius / model); none since round 6
# workloads whose CPU leg runs the full configuration for this many timed steps (after one warm-up step):
# C4 (3D, 200k particles, L = 10, H = 128) takes ~30 s per oracle step on 16 threads, so one step at its
# own size replaces round 5's 20x20x20 per-particle extrapolation
CPU_FULL_STEPS = {"c4": 1}


def cpu_rollout_baseline(sim, window, radius, L, steps, workload, min_seconds=0.0):
    """Oracle (test infrastructure: CPU restatement of the reference) rollout:
    one warm-up step, then at least `steps` timed autoregressive steps, more
    until `min_seconds` of CPU work (at most 20x steps) -- graph build +
    features + EPD + integration all inside the timed region.  Run at every
    thread count of thread_counts(); `value` is the fastest leg (the baseline
    most favourable to the CPU), every leg is listed."""
    from oracle import sgnn_oracle as O
    state = {k: v.detach().cpu() for k, v in sim.state_dict().items()}
    sample = ""
    if workload in CPU_SAMPLE_DIMS:
        window = torch.from_numpy(synthetic.trajectory(lattice(CPU_SAMPLE_DIMS[workload]), T_SEQ, seed=7))
        sample = f" ({'x'.join(map(str, CPU_SAMPLE_DIMS[workload]))} sample: per-particle rate)"
    osim = O.OracleSimulator(state, window.shape[2], L, radius, sim._normalization_stats)
    n = window.shape[0]
    types_ = torch.zeros(n, dtype=torch.long)
    legs = []
    counts, skipped = thread_counts()
    for nthreads in counts:
        info = cpu_threads(nthreads)
        progress(f"  cpu rollout leg: {nthreads} threads")
        cur = window.cpu()
        with torch.no_grad():
            nxt, _ = osim.predict_positions(cur, [n], types_)
            cur = torch.cat([cur[:, 1:], nxt[:, None]], 1)
            t0 = time.perf_counter()
            done = 0
            while done < steps or (time.perf_counter() - t0 < min_seconds and done < 20 * steps):
                nxt, _ = osim.predict_positions(cur, [n], types_)
                cur = torch.cat([cur[:, 1:], nxt[:, None]], 1)
                done += 1
            dt = time.perf_counter() - t0
            edges = int(O.radius_graph(cur[:, -1], [n], radius)[0].shape[0])
        legs.append({"value": n * done / dt, "unit": "particle-steps/s", **info, "seconds": dt, "steps": done,
                     "M_edge_messages_per_s": edges * L * done / dt / 1e6})
    cpu_threads()
    best = max(legs, key=lambda r: r["value"])
    out = {k: best[k] for k in ("value", "unit", "cores", "kind")}
    out["sample"] = f"{best['steps']} oracle rollout steps, {n} particles{sample}, {best['cores']} threads"
    out["host"] = {"cpu_model": best["cpu_model"], "os_cpu_count": best["os_cpu_count"],
                   "affinity_cpus": best["affinity_cpus"], "legs": {str(r["cores"]): r["value"] for r in legs}}
    if skipped:
        out["host"]["note"] = skipped
    return out


def step_flops(n, E, H, L, dim, feat):
    """(algorithmic, executed) FLOPs of one predict_positions step.
    Algorithmic = SURVEY.md §8(d) (2 in out per Linear row, first edge Linear
    3H x H): n (2 F_n H + 2H^2 + L 6H^2 + 2H^2 + 2H(d+1)) + E (2 F_e H + 2H^2 + L 8H^2).
    Executed = what the kernels multiply after the u/v factorisation (first
    edge Linear H x H per edge, u = W1_i x and v = W1_j x once per node)."""
    fe = dim + 1
    alg = n * (2 * feat * H + 2 * H * H + L * 6 * H * H + 2 * H * H + 2 * H * (dim + 1)) + \
        E * (2 * fe * H + 2 * H * H + L * 8 * H * H)
    exe = n * (2 * feat * H + 2 * H * H + 4 * H * H + (L - 1) * 10 * H * H + 6 * H * H + 2 * H * H + 2 * H * (dim + 1)) + \
        E * (2 * fe * H + 2 * H * H + L * 4 * H * H)
    return alg, exe


def bench_rollout(workload, steps, warmup, world, rank, device, seed, cpu_steps, cpu_seconds=0.0, reps=1):
    """Timed region: `steps` autoregressive steps issued as ONE sgnn_rollout
    call (evaluate.rollout's device path: the C driver launches every kernel of
    every step; no host round trip).  Warm-up: full untimed rollouts.  The
    dominant kernel's launch time comes from a second, event-timed pass."""
    from sgnn_amd import engine
    progress(f"rollout {workload}")
    dims, radius, H, L = WORKLOADS[workload]
    dim = len(dims)
    feat = (T_SEQ - 1) * dim + 1
    sim = quiet_decoder(make_sim(H, L, radius, dim, device, seed))
    seq = synthetic.trajectory(lattice(dims), T_SEQ, seed=1000 + rank)
    n = seq.shape[0]
    window0 = torch.from_numpy(seq)
    types_ = torch.zeros(n, dtype=torch.long, device=device)
    with torch.no_grad():
        w0 = window0.to(device)
        runner = sim.rollout_runner(w0, [n], types_, steps)
        one_launch, nt, grid = engine.step_path(runner.epd, runner.sin, runner.ws)
        for _ in range(max(1, -(-warmup // max(steps, 1)))):
            runner.run(w0)
        # `reps` timed calls of `steps` steps each, the median taken (the extras: one host hiccup in a
        # single ~2 ms call once read as 10x the step time); the headline times one call (reps = 1)
        dts = []
        for _ in range(reps):
            sync_barrier(world)
            t0 = time.perf_counter()
            runner.run(w0)
            sync_barrier(world)
            dts.append(time.perf_counter() - t0)
        dt = float(np.median(dts))
        if one_launch:
            # the whole step is ONE k_step16 launch: one event pair on the launch stream around the
            # `steps` back-to-back launches of a rollout call (a spin kernel first, so the host has
            # queued them all before the GPU reaches them); per launch = elapsed / steps
            torch.cuda._sleep(2_000_000)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            runner.run(w0, check_step=False)
            ev1.record()
            runner.ws.check_step(device)   # raises SgnnError if a tile timed out (after ev1: not timed)
            torch.cuda.synchronize()
            kernel_s = ev0.elapsed_time(ev1) * 1e-3 / steps
            edges = [runner.ws.step_edges()]
        else:
            # event-timed pass (same kernels, launched from Python per step)
            inp, use_emb = sim._step_inputs(w0, [n], types_)
            ws = sim._workspace(n, T_SEQ, device)
            win = [inp.pos_seq.clone(), torch.empty_like(inp.pos_seq)]
            pred = torch.empty(n, dim + 1, device=device)
            nxt = torch.empty(n, dim, device=device)
            timers = []
            edges = []
            for k in range(steps):
                inp.pos_seq = win[k % 2]
                # a spin kernel ahead of the step lets the host queue all of the step's launches and events
                # before the GPU reaches them, so no host gap lands inside an event pair
                torch.cuda._sleep(2_000_000)
                engine.forward_step(sim._encode_process_decode, sim._particle_type_embedding.weight, use_emb,
                                    radius, inp, ws, pred, nxt, window_out=win[(k + 1) % 2], timers=timers)
                edges.append(ws.num_edges())
            torch.cuda.synchronize()
            kernel_s = float(np.mean([a.elapsed_time(b) for a, b in timers])) * 1e-3
    dt = max_over_ranks(dt, world, device)
    E = float(np.mean(edges))
    E_all = sum_over_ranks(E, world, device)
    alg_step, exe_step = step_flops(n, E, H, L, dim, feat)
    if one_launch:
        kernel = "k_step16"
        flops, exe = alg_step, exe_step
        # window read + written (n T d 4 each), each layer's u/v written and read once (16 H n), outputs
        alg_bytes = n * (2 * T_SEQ * dim * 4 + L * 16 * H + 4 * (2 * dim + 1))
    elif H == 64 and n <= engine.FUSED_MAX_N:
        kernel_s /= L      # one event pair per step around the L fused launches
        kernel = "k_layer16"
        # per launch, averaged over the L launches: edge MLP (two H x H Linears per edge after the u/v
        # factorisation) + node MLP + the next u/v, layer 0's Encoder.edge_fn and the last layer's decoder
        exe = (L * E * 4 * H * H + E * 2 * (H * H + (dim + 1) * H)
               + (L - 1) * n * 10 * H * H + n * (8 * H * H + 2 * H * (dim + 1))) / L
        # the same launches by §8(d)'s count: the processor's and the edge encoder's share of the step
        flops = (alg_step - n * (2 * feat * H + 2 * H * H)) / L
        alg_bytes = E * (4 * H + 8) + n * 24 * H
    else:
        kernel = "k_edge_layer"
        exe = E * 4 * H * H          # two H x H Linears per edge (u/v factorised out of the first)
        flops = E * 8 * H * H        # §8(d): 3H x H + H x H per edge
        # e0 row (4H) + sender/receiver ids (8) per edge, u/v rows per node (8H), agg row written (4H)
        alg_bytes = E * (4 * H + 8) + n * 12 * H
    out = {"workload": f"{workload}: {'x'.join(map(str, dims))} lattice = {n} particles/GPU, "
                       f"r={radius}, L={L}, H={H}, T={T_SEQ}, K=20", "particles": n, "edges": E,
           "value": n * steps * world / dt, "unit": "particle-steps/s",
           "ms_per_step": dt / steps * 1e3,
           "M_edge_messages_per_s": E_all * L * steps / dt / 1e6,
           "path": (f"k_step16 x{grid}x{nt}" if one_launch else "kernel sequence"),
           # the whole step by §8(d)'s count over the step time: an ALGORITHMIC rate (it can pass the
           # hardware peak where the u/v factorisation skips 2H^2 of every edge's first Linear), beside a
           # split kernel's executed `frac`
           "alg_step_tflops": alg_step / (dt / steps) / 1e12,
           "roofline": roofline(kernel, flops, kernel_s, workload, "rollout", alg_bytes, exe,
                                whole=kernel != "k_edge_layer")}
    out["roofline"]["share_of_step"] = kernel_s * (1 if one_launch else L) / (dt / steps)
    if cpu_steps > 0 and rank == 0 and world == 1:
        progress(f"rollout {workload}: cpu baseline")
        out["cpu_baseline"] = cpu_rollout_baseline(sim, window0, radius, L, CPU_FULL_STEPS.get(workload, cpu_steps),
                                                   workload, 0.0 if workload in CPU_FULL_STEPS else cpu_seconds)
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    return out


# ----------------------------------------------------------------------------- train
def cpu_train_baseline(state, graphs, radius, L, steps, stats):
    """Oracle training step (noise + forward + torch autograd + torch Adam) on the
    CPU over the same concatenated batch."""
    from oracle import sgnn_oracle as O
    info = cpu_threads()
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in state.items()}
    osim = O.OracleSimulator(params, 2, L, radius, stats)
    osim.p = params
    opt = torch.optim.Adam([p for k, p in params.items() if "embedding" not in k], lr=1e-3)
    pos = torch.from_numpy(np.concatenate([g[:, :T_SEQ] for g, _ in graphs]))
    nxt = torch.from_numpy(np.concatenate([g[:, T_SEQ] for g, _ in graphs]))
    strain = torch.from_numpy(np.concatenate([s for _, s in graphs]))
    counts = [g.shape[0] for g, _ in graphs]
    n = pos.shape[0]
    types_ = torch.zeros(n, dtype=torch.long)

    def step():
        noise = O.random_walk_noise(pos, 0.02)
        pa, ta, ps = osim.predict_accelerations(nxt, noise, pos, counts, types_)
        loss = O.training_loss(pa, ta, ps, strain)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "particle-steps/s", "cores": info["cores"], "kind": "port",
            "sample": f"{steps} oracle training steps (noise+fwd+autograd+Adam), {n} particles, "
                      f"{info['cores']} threads"}


def _train_graph(dims, seed):
    seq = synthetic.trajectory(synthetic.lattice_2d(*dims), T_SEQ + 1, seed=seed)
    strain = np.random.default_rng(seed).normal(0, 1, seq.shape[0]).astype(np.float32)
    return seq, strain


def bench_train(mode, steps, warmup, world, rank, device, seed, cpu_steps):
    """C2 (`train`: one 50k graph per rank, weak scaling) or C3 (`train-c3`: a
    global batch of 8 real-size graphs split over the ranks, strong scaling).
    One step = Trainer.train_step: fused noise, saved-activation forward, fused
    loss + backward, SUM all-reduce of the flat gradient over RCCL, Adam, LR."""
    from sgnn_amd.train import Trainer, split_batch
    progress(mode)
    if mode == "train":
        dims, radius, H, L = WORKLOADS["c2"]
        all_graphs = [dims] * world
        mine_idx = [rank]
        desc = (f"c2: 2D lattice {dims[0]}x{dims[1]} = {dims[0] * dims[1]} particles per GPU (one whole graph "
                f"per rank), r={radius}, L={L}, H={H}, T={T_SEQ}, K=20, training step (noise+fwd+bwd+Adam)")
        scaling = "weak"
    else:
        _, radius, H, L = WORKLOADS["c2"]
        all_graphs = C3_GRAPHS
        mine_idx = split_batch(list(range(len(all_graphs))), rank, world)
        desc = (f"c3: global batch of {len(all_graphs)} whole graphs "
                f"({'/'.join(str(a * b) for a, b in all_graphs)} particles, real Taylor-bar sizes) split "
                f"contiguously over the ranks, r={radius}, L={L}, H={H}, T={T_SEQ}, K=20, training step")
        scaling = "strong"
    sim = make_sim(H, L, radius, 2, device, seed)
    state0 = {k: v.detach().cpu().clone() for k, v in sim.state_dict().items()}
    graphs = [_train_graph(all_graphs[i], 2000 + i) for i in mine_idx]
    counts = [g.shape[0] for g, _ in graphs]
    all_counts = [a * b for a, b in all_graphs]
    n_global = sum(all_counts)
    offset = sum(all_counts[:mine_idx[0]])
    n = sum(counts)
    pos = torch.from_numpy(np.concatenate([g[:, :T_SEQ] for g, _ in graphs])).to(device)
    nxt = torch.from_numpy(np.concatenate([g[:, T_SEQ] for g, _ in graphs])).to(device)
    strain = torch.from_numpy(np.concatenate([s for _, s in graphs])).to(device)
    tr = Trainer(sim, lr_init=1e-3)
    kw = dict(n_global=n_global, particle_offset=offset)
    for _ in range(warmup):
        tr.train_step(pos, nxt, strain, counts, **kw)
    sync_barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = tr.train_step(pos, nxt, strain, counts, **kw)
    sync_barrier(world)
    dt = time.perf_counter() - t0
    timers = {}
    t2 = time.perf_counter()
    for _ in range(steps):
        tr.train_step(pos, nxt, strain, counts, timers=timers, **kw)
    torch.cuda.synchronize()
    dt_ev = time.perf_counter() - t2
    dt = max_over_ranks(dt, world, device)
    tw = tr.workspace(n, T_SEQ, device)
    E = tw.f.num_edges()
    E_all = sum_over_ranks(E, world, device)
    kstats = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e-3 for k, v in timers.items()}
    # dominant kernel: the edge-layer backward (H = 64, nmlp_layers 1: k_edge_bwd64, Wl^T dy and
    # dWl += dy h^T; dE0 / dW1e of all layers are formed afterwards by k_edge_latent_grad)
    dom = "k_edge_bwd"
    flops_bwd = E * (4 if tw.latent_pass else 8) * H * H
    kname = "k_edge_bwd64" if (H == 64 and tw.nlin == 2) else "k_edge_bwd"
    res = {
        "metric": "particle-steps/sec (2D Taylor-impact, training fwd+bwd+Adam)",
        "value": n_global * steps / dt, "unit": "particle-steps/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": dt / steps * 1e3, "scaling": scaling, "dtype": "f32", "data": DATA,
        "config": {"workload": desc, "particles_global": n_global, "particles_rank0": n, "edges_rank": E,
                   "global_batch_graphs": len(all_graphs), "layers": L, "hidden": H, "radius": radius,
                   "parallelism": f"dp{world} (whole-graph, RCCL all-reduce)" if world > 1 else "single GPU"},
        "M_edge_messages_per_s": E_all * L * steps / dt / 1e6,
        "final_loss": float(out["loss"]),
        # fwd + bwd ~ 3x the forward by §8(d)'s count, over the step time (algorithmic rate, TFLOP/s)
        "alg_step_tflops": 3 * step_flops(n_global, E_all, H, L, 2, (T_SEQ - 1) * 2 + 1)[0] / (dt / steps) / 1e12,
        "roofline": roofline(kname, flops_bwd, kstats[dom], "c2" if mode == "train" else "c3", "train",
                             whole=False),
        "kernel_avg_us": {k: v * 1e6 for k, v in kstats.items()},
    }
    res["roofline"]["share_of_step"] = float(np.sum([a.elapsed_time(b) for a, b in timers[dom]])) / (dt_ev * 1e3)
    if rank == 0 and world == 1 and cpu_steps > 0:
        progress(f"{mode}: cpu baseline")
        res["cpu_baseline"] = cpu_train_baseline(state0, graphs, radius, L, max(3, cpu_steps // 2),
                                                 sim._normalization_stats)
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
    info = cpu_threads()
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
    return {"value": n * steps / dt, "unit": "particle-steps/s", "cores": info["cores"], "kind": "port",
            "sample": f"{steps} oracle multi-scale training steps, {'x'.join(map(str, sdims))} sample = {n} "
                      f"particles (per-particle rate), {info['cores']} threads"}


def bench_ms_train(workload, steps, warmup, world, rank, device, seed, cpu_steps):
    from sgnn_amd.multi_scale.ms_training import MultiScaleTrainer
    progress(f"ms-train {workload}")
    sim, seq, edges, desc, cfg = ms_setup(workload, device, seed, rank, T_SEQ + 1)
    n = seq.shape[0]
    H, L, nmlp = cfg[4], cfg[5], cfg[6]
    pos = torch.from_numpy(seq[:, :T_SEQ]).to(device)
    nxt = torch.from_numpy(seq[:, T_SEQ]).to(device)
    strain = torch.from_numpy(np.random.default_rng(rank).normal(0, 1, n).astype(np.float32)).to(device)
    tr = MultiScaleTrainer(sim, lr_init=1e-3)
    kw = dict(n_global=n * world, particle_offset=n * rank)
    for _ in range(warmup):
        tr.train_step(pos, nxt, strain, **kw)
    sync_barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = tr.train_step(pos, nxt, strain, **kw)
    sync_barrier(world)
    dt = time.perf_counter() - t0
    timers = {}
    for _ in range(min(steps, 3)):
        tr.train_step(pos, nxt, strain, timers=timers, **kw)
    torch.cuda.synchronize()
    dt = max_over_ranks(dt, world, device)
    kstats = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e-3 for k, v in timers.items()}
    eb = ms_block_edges(edges, L)
    # edge backward per edge: last (+ middle) Linear W^T dy and dW, W1e^T dh and dW1e; at H = 128 with
    # nmlp_layers 2 the items kernel also re-forms h2 = relu(Wm h1 + bm) and Wl h2 (the forward's values,
    # not saved: DESIGN.md 8.4), 4 H^2 more that it executes
    flops_bwd = eb / (L + 2) * (8 + (4 if nmlp == 2 else 0) + (4 if (H == 128 and nmlp == 2) else 0)) * H * H
    dom = "k_edge_bwd"
    # H = 128: one sgnn_edge_layer_bwd call = the per-edge items kernel + one split-K weight-gradient
    # GEMM per Linear (3 at nmlp_layers 2)
    # (exact kernel names as rocprofv3 lists them: the profile summary's per-launch bytes and time
    # of the composite come from the same names)
    kname = "k_edge_bwd64" if (H == 64 and nmlp == 1) else \
        (f"k_edge_items<{H // 32}, {nmlp + 1}> + {nmlp + 1} k_wgrad_full<1>" if H == 128 else
         f"k_edge_items<{H // 32}, {nmlp + 1}> + {nmlp + 1} k_wgrad<{H // 32}, {H // 32}>")
    res = {
        "metric": "particle-steps/sec (multi-scale training fwd+bwd+Adam)",
        "value": n * steps * world / dt, "unit": "particle-steps/s", "n_gpus": world,
        "steps": steps, "warmup": warmup, "ms_per_step": dt / steps * 1e3, "scaling": "weak", "dtype": "f32",
        "data": DATA,
        "config": {"workload": desc + ", training step (noise+fwd+bwd+Adam)", "particles_per_gpu": n,
                   "edge_evaluations_per_step": eb, "global_batch_graphs": world,
                   "parallelism": f"dp{world} (whole-graph, RCCL all-reduce)" if world > 1 else "single GPU"},
        "M_edge_messages_per_s": eb * steps * world / dt / 1e6,
        "final_loss": float(out["loss"]),
        "hbm_peak_gib": torch.cuda.max_memory_allocated(device) / 2 ** 30,
        "roofline": roofline(kname, flops_bwd, kstats.get(dom, float("nan")), workload, "train", whole=False),
        "kernel_avg_us": {k: v * 1e6 for k, v in kstats.items()},
    }
    if rank == 0 and world == 1 and cpu_steps > 0:
        progress(f"ms-train {workload}: cpu baseline")
        res["cpu_baseline"] = cpu_ms_train_baseline(sim, cfg, max(3, cpu_steps // 2))
        res["speedup_vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    return res


def bench_ms_rollout(workload, steps, warmup, world, rank, device, seed):
    sim, seq, edges, desc, cfg = ms_setup(workload, device, seed, rank, T_SEQ)
    n = seq.shape[0]
    L = cfg[5]
    cur = torch.from_numpy(seq).to(device).contiguous()
    with torch.no_grad():
        runner = sim.rollout_runner(cur, None, steps)
        for _ in range(max(1, -(-warmup // max(steps, 1)))):
            runner.run(cur)
        sync_barrier(world)
        t0 = time.perf_counter()
        runner.run(cur)
        sync_barrier(world)
        dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, world, device)
    eb = ms_block_edges(edges, L)
    return {"metric": "particle-steps/sec (multi-scale rollout)", "value": n * steps * world / dt,
            "unit": "particle-steps/s", "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": dt / steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": DATA,
            "config": {"workload": desc + ", rollout", "particles": n,
                       "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
            "M_edge_messages_per_s": eb * steps * world / dt / 1e6}


# ----------------------------------------------------------------------------- main
def headline(r, args, world, metric, parallel):
    res = {"metric": metric, "value": r["value"], "unit": r["unit"], "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": r["ms_per_step"], "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": DATA,
           "config": {"workload": r["workload"] + ", autoregressive rollout (radius graph + features + EPD + "
                                                  "Euler + window shift per step), one sgnn_rollout call",
                      "particles_per_gpu": r["particles"], "edges_per_gpu": r["edges"],
                      "parallelism": parallel},
           "M_edge_messages_per_s": r["M_edge_messages_per_s"], "alg_step_tflops": r["alg_step_tflops"],
           "roofline": r["roofline"]}
    if "cpu_baseline" in r:
        res["cpu_baseline"] = r["cpu_baseline"]
        res["speedup_vs_cpu"] = r["speedup_vs_cpu"]
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_workers(args, argv)          # parent: no GPU call before this point
    world, rank, local = init_dist(args)
    if args.selftest_launch:
        return selftest_launch(world, rank)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if args.workload is None:
        args.workload = {"rollout": "c1_r15", "ms-train": "c5", "ms-rollout": "c5"}.get(args.mode, "c2")
    parallel = f"replicas x{world} (one trajectory per GPU, no collective)" if world > 1 else "single GPU"
    cs = args.cpu_steps
    if args.mode == "ms-train":
        res = bench_ms_train(args.workload, args.steps, args.warmup, world, rank, device, args.seed, cs)
    elif args.mode == "ms-rollout":
        res = bench_ms_rollout(args.workload, args.steps, args.warmup, world, rank, device, args.seed)
    elif args.mode in ("train", "train-c3"):
        res = bench_train(args.mode, args.steps, args.warmup, world, rank, device, args.seed, cs)
        res["higher_is_better"], res["vs_baseline"] = True, None
    else:
        r = bench_rollout(args.workload, args.steps, args.warmup, world, rank, device, args.seed, cs,
                          args.cpu_seconds)
        res = headline(r, args, world, "particle-steps/sec (2D Taylor-impact rollout)", parallel)
        if not args.no_extras:
            # extras: numbers only (leg()), so the whole line stays a few KB
            res["training"] = leg(bench_train("train", 10, 3, world, rank, device, args.seed, cs))
            res["training_c3"] = leg(bench_train("train-c3", 10, 3, world, rank, device, args.seed, 0))
            res["rollout_extra"] = {}
            for wl, st in (("c2", 20), ("c1_r06", 20), ("t4800", 20), ("t6400", 20), ("t8000", 20), ("c4", 10)):
                res["rollout_extra"][wl] = leg(bench_rollout(wl, st, 3, world, rank, device, args.seed, cs, reps=3))
            res["multi_scale_c5_train"] = leg(bench_ms_train("c5", 3, 1, world, rank, device, args.seed, cs))
    if rank == 0:
        errs = bench_line_errors(res)
        if errs:
            res["invalid_legs"] = [p for p, _ in errs]
            print(f"bench: legs with an invalid roofline: {errs}", file=sys.stderr, flush=True)
        print(json.dumps(_r(res), separators=(",", ":")))
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
