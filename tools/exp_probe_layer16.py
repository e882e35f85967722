"""Fused-layer phase timing (experiment builds with per-wave s_memtime marks in
k_layer16, `sgnn_set_probe16`): one middle-layer launch at a bench workload,
per-phase cycle percentiles over the waves."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from sgnn_amd import engine, synthetic
from sgnn_amd._hip import lib, check, stream_ptr

wl = sys.argv[1] if len(sys.argv) > 1 else "c1_r15"
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
for _ in range(20): call()
torch.cuda.synchronize()
buf = torch.zeros(4096 * 4 * 8, dtype=torch.int64, device=dev)
lib().sgnn_set_probe16(ctypes.c_void_p(buf.data_ptr()))
call()
torch.cuda.synchronize()
lib().sgnn_set_probe16(ctypes.c_void_p(0))
t = buf.view(-1, 8).cpu().numpy().astype(np.float64)
t = t[t[:, 0] > 0]
names = ["prologue(staging)", "loop top sync", "edge phase", "edge barrier", "agg sums+sync", "node phase"]
print(f"{wl}: {t.shape[0]} waves; total wave life p50/p90 {np.percentile(t[:, 6] - t[:, 0], [50, 90]).round()}")
for k, nm in enumerate(names):
    d = t[:, k + 1] - t[:, k]
    print(f"  {nm:20s} p10 {np.percentile(d, 10):8.0f}  p50 {np.percentile(d, 50):8.0f}  p90 {np.percentile(d, 90):8.0f}")
# wave start skew within the launch (same-XCD clocks only: use per-XCD groups by blockIdx % 8)
blk = np.arange(t.shape[0]) // 4
for x in range(2):
    sel = (blk % 8) == x
    st = t[sel, 0] - t[sel, 0].min(); en = t[sel, 6] - t[sel, 0].min()
    print(f"  xcd{x}: start spread p50/max {np.percentile(st, 50):.0f}/{st.max():.0f}, end p50/max {np.percentile(en, 50):.0f}/{en.max():.0f}")
