"""Fused-layer experiment: time one sgnn_interaction_layer launch (HIP events,
100 launches) at a bench workload, optionally at forced receivers-per-tile counts.

  python tools/exp_layer16.py build              # here (CPU): _lib/libsgnn_hip_exp.so (-DSGNN_EXPERIMENT)
  python tools/exp_layer16.py <workload> [nt...] # on the GPU box (SGNN_NT, clamped to 8..16, is read only
                                                 # by that experiment build)"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EXP_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sgnn_amd", "_lib",
                       "libsgnn_hip_exp.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    from sgnn_amd import build_lib
    print(build_lib.build(defines=("SGNN_EXPERIMENT",), lib=EXP_LIB))
    sys.exit(0)
import numpy as np
import torch
from sgnn_amd import _hip
_hip.load_library(EXP_LIB)
import bench
from sgnn_amd import engine, synthetic
from sgnn_amd._hip import lib, check, stream_ptr

wl = sys.argv[1]
dims, radius, H, L = bench.WORKLOADS[wl]
dev = torch.device("cuda", 0)
sim = bench.quiet_decoder(bench.make_sim(H, L, radius, len(dims), dev, 0))
seq = synthetic.trajectory(bench.lattice(dims), bench.T_SEQ, seed=1000)
n = seq.shape[0]
w0 = torch.from_numpy(seq).to(dev)
types_ = torch.zeros(n, dtype=torch.long, device=dev)
inp, use_emb = sim._step_inputs(w0, [n], types_)
ws = sim._workspace(n, bench.T_SEQ, dev)
pred = torch.empty(n, len(dims) + 1, device=dev); nxt = torch.empty(n, len(dims), device=dev)
engine.forward_step(sim._encode_process_decode, sim._particle_type_embedding.weight, use_emb, radius, inp, ws, pred, nxt)
pk = engine.ParamPack.get(sim._encode_process_decode)
s = stream_ptr(dev)
def call():
    check(lib().sgnn_interaction_layer(ws.x_a.data_ptr(), ws.u.data_ptr(), ws.v.data_ptr(), ws.e0t.data_ptr(), 2.0,
                                       ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n,
                                       ctypes.byref(pk.edge[1]), ctypes.byref(pk.node[1]), ctypes.byref(pk.edge[2]),
                                       ws.x_b.data_ptr(), ws.u2.data_ptr(), ws.v2.data_ptr(), s), "layer")
for nt in (sys.argv[2:] or [""]):
    if nt:
        os.environ["SGNN_NT"] = nt
    for _ in range(20): call()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(100): call()
    b.record(); torch.cuda.synchronize()
    print(f"{wl} nt={nt or 'auto'}: {a.elapsed_time(b) / 100 * 1e3:.2f} us/launch")
