"""Host-sync check of the data-parallel training step.

  run:      python3 tools/dp_sync_trace.py run
            a one-rank RCCL group (backend "nccl") on the box's GPU, the C3 global batch (8 whole Taylor
            graphs, bench.C3_GRAPHS) through sgnn_amd.train.Trainer with the deferred-count path forced on
            (DataParallel.force_deferred: no n_global / particle_offset from the caller, so the count rides
            in the gradient all-reduce) and the overlapped per-layer buckets (force_overlap).  Each timed
            step is preceded by ONE sentinel kernel (torch.cuda._sleep); then the same steps with the
            round-5 layout (an all_gather of the local count + .tolist() before the step) are each
            preceded by TWO sentinels, as the analyser's control: it must find the sync there.
            Meant to run under  rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv.
  analyze:  python3 tools/dp_sync_trace.py analyze DIR
            joins the HIP API trace with the kernel trace (correlation ids), cuts the launching thread's
            API calls at the sentinels and lists, per step, the blocking calls (synchronize / synchronous
            copies) and whether any comes before the step's first forward kernel is launched.
"""
import csv
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

STEPS = 4
BLOCKING = ("Synchronize", "hipMemcpyWithStream", "hipMemcpy", "hipMemcpyDtoH", "hipMemcpy2D")


def run():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29731")
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    from sgnn_amd.train import Trainer
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    _, radius, H, L = bench.WORKLOADS["c2"]
    sim = bench.make_sim(H, L, radius, 2, dev, 0)
    graphs = [bench._train_graph(g, 2000 + i) for i, g in enumerate(bench.C3_GRAPHS)]
    counts = [g.shape[0] for g, _ in graphs]
    pos = torch.from_numpy(np.concatenate([g[:, :bench.T_SEQ] for g, _ in graphs])).to(dev)
    nxt = torch.from_numpy(np.concatenate([g[:, bench.T_SEQ] for g, _ in graphs])).to(dev)
    strain = torch.from_numpy(np.concatenate([s for _, s in graphs])).to(dev)
    tr = Trainer(sim, lr_init=1e-3)
    tr.dp.force_deferred = True
    tr.dp.force_overlap = True
    for _ in range(3):
        tr.train_step(pos, nxt, strain, counts)
    torch.cuda.synchronize()
    for _ in range(STEPS):                       # the shipping step: no count collective, no host sync
        torch.cuda._sleep(1000)
        out = tr.train_step(pos, nxt, strain, counts)
    torch.cuda.synchronize()
    tr.dp.force_deferred = False
    for _ in range(STEPS):                       # control: the round-5 layout() gather before the step
        torch.cuda._sleep(1000)
        torch.cuda._sleep(1000)
        t = torch.tensor([pos.shape[0]], dtype=torch.int64, device=dev)
        got = [torch.empty_like(t)]
        dist.all_gather(got, t)
        c = torch.cat(got).tolist()
        out = tr.train_step(pos, nxt, strain, counts, n_global=int(sum(c)), particle_offset=0)
    torch.cuda.synchronize()
    print("loss", float(out["loss"]), "particles", pos.shape[0], flush=True)
    dist.destroy_process_group()


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _short(k):
    m = re.search(r"(\w+)(<[^(]*>)?\(", k)
    return m.group(1) if m else k[:40]


def _after(calls, j):
    """The kernel launched last before call j (where in the step a blocking call sits)."""
    return "after " + _short(next((c[1] for c in reversed(calls[:j]) if c[1]), ""))


def analyze(d):
    api = _rows(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])
    kern = _rows(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])
    kname = {r["Correlation_Id"]: r["Kernel_Name"] for r in kern}
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    spins = [r for r in api if "spin" in kname.get(r["Correlation_Id"], "")]
    if not spins:
        sys.exit("no sentinel kernels in the trace")
    tid = spins[0]["Thread_Id"]
    calls = [r for r in api if r["Thread_Id"] == tid and int(r["Start_Timestamp"]) >= int(spins[0]["Start_Timestamp"])]
    steps, cur = [], None
    for r in calls:
        k = kname.get(r["Correlation_Id"], "")
        if "spin" in k:
            if cur is not None and not any(c[1] for c in cur["calls"]):
                cur["spins"] += 1
                continue
            cur = {"spins": 1, "calls": [], "t0": int(r["Start_Timestamp"])}
            steps.append(cur)
            continue
        cur["calls"].append((r["Function"], k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    lines = []
    for i, s in enumerate(steps):
        kind = "deferred (shipping)" if s["spins"] == 1 else "control: all_gather + tolist"
        first_fwd = next((j for j, c in enumerate(s["calls"]) if re.search(r"\bk_", c[1]) and "noise" not in c[1]),
                         None)
        block = [(j, c[0], (c[3] - c[2]) / 1e3) for j, c in enumerate(s["calls"])
                 if any(b in c[0] for b in BLOCKING) and "Async" not in c[0]]
        before = [b for b in block if first_fwd is not None and b[0] < first_fwd]
        t_first = (s["calls"][first_fwd][2] - s["t0"]) / 1e3 if first_fwd is not None else float("nan")
        nk = sum(1 for c in s["calls"] if c[1])
        lines.append(f"step {i} [{kind}]: {len(s['calls'])} HIP API calls, {nk} kernel launches; first forward "
                     f"kernel {_short(s['calls'][first_fwd][1]) if first_fwd is not None else '-'} launched "
                     f"{t_first:.1f} us after the sentinel; blocking calls before it: {len(before)} "
                     f"{[(b[1], round(b[2], 1)) for b in before]}; blocking calls in the step: {len(block)} "
                     f"{[(b[1], round(b[2], 1), _after(s['calls'], b[0])) for b in block][:6]}")
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        analyze(sys.argv[2])
