"""Per-call overhead of a device rollout (C1 r = 15, the headline): host wall time of one sgnn_rollout call
of K steps with the error-word check (the bench's timed region), without it (stream sync only), and
without the window copy, against the event-timed span of its K launches.

  python tools/exp_call_overhead.py [K] [calls]      # on the GPU box"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sgnn_amd import synthetic  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dims, radius, H, L = bench.WORKLOADS["c1_r15"]
dev = torch.device("cuda", 0)
sim = bench.quiet_decoder(bench.make_sim(H, L, radius, len(dims), dev, 0))
seq = synthetic.trajectory(bench.lattice(dims), bench.T_SEQ, seed=1000)
w0 = torch.from_numpy(seq).to(dev)
n = seq.shape[0]
runner = sim.rollout_runner(w0, [n], torch.zeros(n, dtype=torch.long, device=dev), K)
for _ in range(5):
    runner.run(w0)
torch.cuda.synchronize()


def wall(fn):
    ts = []
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
spans = []
for _ in range(calls):
    ev0.record()
    runner.run(w0, check_step=False)
    ev1.record()
    torch.cuda.synchronize()
    spans.append(ev0.elapsed_time(ev1) * 1e3)
res = {
    "checked call (bench timed region)": wall(lambda: runner.run(w0)),
    "no error-word check": wall(lambda: runner.run(w0, check_step=False)),
    "no check, no window copy": wall(lambda: runner.run(None, check_step=False)),
    "events around the call (GPU span incl. copy + memset)": float(np.median(spans)),
}
for k, v in res.items():
    print(f"{k:55s} {v:9.1f} us per call = {v / K:7.2f} us per step (K = {K})")
t0 = time.perf_counter()
for _ in range(200):
    runner.ws.check_step(dev)
print(f"sgnn_step_check alone (idle stream): {(time.perf_counter() - t0) / 200 * 1e6:.1f} us")
