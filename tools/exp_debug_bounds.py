"""Bounds-checked run of the rollout step on every launch path (VERDICT r02
item 9): a debug build (-DSGNN_DEBUG_BOUNDS: index checks on the edge lists,
padded neighbour lists, tile CSRs and gathers that print `SGNN-BOUNDS ...` and
clamp, no trap) runs eager rollouts and the HIP-graph capture/replay test of
tests/test_gpu_graph.py on the one-launch step, the fused per-layer kernels and
the general edge/node kernels.

  python tools/exp_debug_bounds.py build   # here (CPU): _lib/libsgnn_hip_dbg.so
  python tools/exp_debug_bounds.py         # on the GPU box; grep the output for SGNN-BOUNDS
  python tools/exp_debug_bounds.py train128   # the H = 128 gradient tests (the
                                              # k_wgrad_half operand loads, LDS images, slab tiles and
                                              # column sums are checked against their extents)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DBG_LIB = os.path.join(ROOT, "sgnn_amd", "_lib", "libsgnn_hip_dbg.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    from sgnn_amd import build_lib
    print(build_lib.build(defines=("SGNN_DEBUG_BOUNDS",), lib=DBG_LIB))
    sys.exit(0)
import torch
from sgnn_amd import _hip
_hip.load_library(DBG_LIB)
import bench
from tests import test_gpu_graph as tg

if len(sys.argv) > 1 and sys.argv[1] == "train128":
    from tests import test_gpu_configs as tc, test_gpu_multi_scale_training as tm, test_gpu_training as tt
    for args in [(2, 128, 1, 3), (3, 128, 2, 3)]:   # [2-128-1-3] is the shape that faulted in round 3
        tt.test_wide_and_deep_mlp_gradients_against_oracle(*args)
        print(f"H = 128 gradients vs oracle (dim, H, nmlp, L) = {args}: ok", flush=True)
    for fn in (tm.test_multi_scale_3d_h128_gradients_against_oracle,
               tc.test_c4_shapes_l10_h128_forward_and_gradients_against_float64_oracle,
               tc.test_c5_shapes_l10_h128_forward_and_gradients_against_float64_oracle):
        fn()
        print(f"{fn.__name__}: ok", flush=True)
    print("debug-bounds train128 run done")
    sys.exit(0)

dev = torch.device("cuda", 0)
for dims, radius, path in [((50, 40), 15.0, "one-launch"), ((50, 40), 0.6, "one-launch"),
                           ((80, 60), 0.6, "fused layers"), ((120, 100), 0.6, "edge/node"),
                           ((100, 50, 8), 0.75, "edge/node")]:
    if len(dims) == 2:
        tg.test_graph_replay_matches_eager(dims, radius, path)
        print(f"graph replay == eager: {dims} r={radius} ({path})", flush=True)
    sim = bench.quiet_decoder(bench.make_sim(64, 5, radius, len(dims), dev, 0))
    from sgnn_amd import synthetic
    seq = synthetic.trajectory(bench.lattice(dims), bench.T_SEQ, seed=7)
    n = seq.shape[0]
    runner = sim.rollout_runner(torch.from_numpy(seq).to(dev), [n], torch.zeros(n, dtype=torch.long, device=dev), 20)
    pos, _ = runner.run()
    torch.cuda.synchronize()
    print(f"rollout 20 steps: {dims} r={radius} finite={bool(torch.isfinite(pos).all())}", flush=True)
print("debug-bounds run done")
