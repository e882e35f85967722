"""Phase timing of the one-launch step (k_step16) from an experiment build
with per-wave s_memtime marks (-DSGNN_PROBE, sgnn_set_probe16).

  python tools/exp_probe_step16.py build          # here (CPU): builds _lib/libsgnn_hip_probe.so
  python tools/exp_probe_step16.py [workload]     # on the GPU box

Prints per-phase cycle percentiles over the waves: radius search, encoder,
and per layer the wait for the sender tiles, the edge phase, the node phase."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROBE_LIB = os.path.join(ROOT, "sgnn_amd", "_lib", "libsgnn_hip_probe.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    from sgnn_amd import build_lib
    print(build_lib.build(defines=("SGNN_PROBE",), lib=PROBE_LIB))
    sys.exit(0)
import numpy as np
import torch
from sgnn_amd import _hip
_hip.load_library(PROBE_LIB)
import bench
from sgnn_amd import engine, synthetic

wl = sys.argv[1] if len(sys.argv) > 1 else "c1_r15"
dims, radius, H, L = bench.WORKLOADS[wl]
dev = torch.device("cuda", 0)
sim = bench.quiet_decoder(bench.make_sim(H, L, radius, len(dims), dev, 0))
seq = synthetic.trajectory(bench.lattice(dims), bench.T_SEQ, seed=1000)
n = seq.shape[0]
w0 = torch.from_numpy(seq).to(dev)
types_ = torch.zeros(n, dtype=torch.long, device=dev)
runner = sim.rollout_runner(w0, [n], types_, 3)   # marks of the last step (contiguous pos_last)
one, nt, grid = engine.step_path(runner.epd, runner.sin, runner.ws)
assert one, "workload does not take the one-launch step"
for _ in range(20):
    runner.run(w0)
torch.cuda.synchronize()
buf = torch.zeros(grid * 4 * 64, dtype=torch.int64, device=dev)
lib = _hip.lib()
lib.sgnn_set_probe16.argtypes = [ctypes.c_void_p]
lib.sgnn_set_probe16(ctypes.c_void_p(buf.data_ptr()))
runner.run(w0)
torch.cuda.synchronize()
lib.sgnn_set_probe16(ctypes.c_void_p(0))
t = buf.view(grid * 4, 64).cpu().numpy().astype(np.float64)
nl = min(L, 5)
last = 3 + 8 * (nl - 1) + 7
print(f"{wl}: n={n} grid={grid} nt={nt} L={L}; wave life (to layer {nl - 1}'s end) p50/p90/max "
      f"{np.percentile(t[:, last] - t[:, 0], [50, 90, 100]).round()} cycles (s_memtime)")


def show(a, b, nm, sel=None):
    sel = (t[:, a] > 0) & (t[:, b] > 0) if sel is None else sel & (t[:, a] > 0) & (t[:, b] > 0)
    if not sel.any():
        print(f"  {nm:28s} (no wave reaches it)")
        return
    d = t[sel, b] - t[sel, a]
    print(f"  {nm:28s} p10 {np.percentile(d, 10):8.0f}  p50 {np.percentile(d, 50):8.0f}  p90 {np.percentile(d, 90):8.0f}"
          f"  max {d.max():8.0f}")


show(0, 56, "positions staged")
show(56, 1, "radius scan")
show(1, 58, "weights to LDS")
show(58, 59, "tile CSR")
show(59, 2, "node encoder")
for k in range(nl):
    s0 = 3 + 8 * k
    show(2 if k == 0 else s0 - 1, s0, f"L{k} layer boundary")
    show(s0, s0 + 1, f"L{k} node weights requested")
    show(s0 + 1, s0 + 2, f"L{k} pre-wait to publish")
    show(s0 + 2, s0 + 3, f"L{k} pre-wait rest")
    show(s0 + 3, s0 + 4, f"L{k} wait")
    show(s0 + 4, s0 + 5, f"L{k} edge phase")
    show(s0 + 5, s0 + 6, f"L{k} node phase")
    show(s0 + 6, s0 + 7, f"L{k} stage + barrier")
print("layer 1 detail:")
three = t[:, 51] > 0
show(3 + 8 + 4, 48, "gather issue")
show(48, 49, "half 0")
show(49, 50, "half 1")
show(50, 51, "half 2", three)
show(3 + 8 + 5, 52, "node: sums + barriers")
show(52, 53, "node: first Linear")
show(53, 3 + 8 + 6, "node: tail")
