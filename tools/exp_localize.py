"""Localise a one-launch step parity failure: run one tests/test_gpu_step.py
oracle case on a library build (SGNN_LIB) several times and print where the
decoder output departs from the oracle (particles -> tile, node sub-tile, row;
which output channels), and whether repeated launches agree with each other.

  SGNN_LIB=... python tools/exp_localize.py DIM DIMS RADIUS N_EX NTYPES K [REPS]
  e.g. python tools/exp_localize.py 3 16,16,12 0.75 2 3 20 3"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import sgnn_oracle as O  # noqa: E402
from sgnn_amd import engine, synthetic  # noqa: E402
from sgnn_amd.learned_simulator import LearnedSimulator  # noqa: E402
from tests.test_gpu_step import _run  # noqa: E402

dim, dims, radius, n_ex, ntypes, K = (int(sys.argv[1]), tuple(int(v) for v in sys.argv[2].split(",")),
                                      float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]))
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 3
lat = synthetic.lattice_2d if dim == 2 else synthetic.lattice_3d
seqs = [synthetic.trajectory(lat(*dims), 11, seed=60 + k) for k in range(n_ex)]
for k, sq in enumerate(seqs):
    sq[..., 0] += 0.17 * k
seq = np.concatenate(seqs, 0)
counts = [s.shape[0] for s in seqs]
n = seq.shape[0]
st = synthetic.normalization_stats(dim, noise_std=0.02)
stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
torch.manual_seed(11)
emb = 16 if ntypes > 1 else 0
sim = LearnedSimulator(dim, 10 * dim + 1 + emb, dim + 1, 64, 5, 1, 64, radius, stats, ntypes, emb or 9)
sim._max_num_neighbors = K
state = {k: v.detach().clone() for k, v in sim.state_dict().items()}
types_ = torch.from_numpy(np.random.default_rng(2).integers(0, ntypes, n))
pos = torch.from_numpy(seq)
osim = O.OracleSimulator(state, dim, 5, radius, stats, ntypes)
osim.max_num_neighbors = K
ref_next, ref_strain = osim.predict_positions(pos, counts, types_)
sim = sim.cuda()
outs = []
FILL = os.environ.get("FILL", "none")   # NaN-fill part of the step workspace before every launch after the first
for r in range(reps):
    if r > 0 and FILL != "none":
        ws0 = sim._workspace(n, 11, torch.device("cuda", 0))
        assert ws0.uvl is not None
        nH = 5 * 2 * n * 64
        if FILL in ("all", "uv"):
            ws0.uvl[:nH].fill_(float("nan"))
        if FILL in ("all", "e0"):
            ws0.uvl[nH:].fill_(float("nan"))
        torch.cuda.synchronize()
    pred, nxt, ws, path = _run(sim, pos.cuda(), counts, types_.cuda(), True)
    outs.append(pred.cpu().numpy())
    nt = path[1]
    err = np.abs(pred[:, -1].cpu().numpy() - ref_strain.numpy())
    bad = np.nonzero(~(err <= 2e-4 + 1e-4 * np.abs(ref_strain.numpy())))[0]   # NaN counts as bad
    nonfin = int((~np.isfinite(pred.cpu().numpy())).any(axis=1).sum())
    print(f"rep {r}: path {path}, timeout {ws.step_timeout()}, edges {ws.step_edges()}, bad particles {bad.size} "
          f"max err {np.nanmax(err):.3e} nonfinite {nonfin}", flush=True)
    if bad.size and os.environ.get("DUMP_BAD") and not os.path.exists(os.environ["DUMP_BAD"] + "_e0.npy"):
        wsd = sim._workspace(n, 11, torch.device("cuda", 0))
        nHd = 5 * 2 * n * 64
        np.save(os.environ["DUMP_BAD"] + "_e0.npy", wsd.uvl[nHd:].cpu().numpy())
        np.save(os.environ["DUMP_BAD"] + "_uv.npy", wsd.uvl[:nHd].cpu().numpy())
        np.save(os.environ["DUMP_BAD"] + "_deg.npy", wsd.step_deg.cpu().numpy())
        np.save(os.environ["DUMP_BAD"] + "_pred.npy", pred.cpu().numpy())
    if bad.size:
        tiles = bad // nt
        rows = bad % nt
        print(f"  tiles {np.unique(tiles)[:40]} ({np.unique(tiles).size} tiles)")
        print(f"  rows in tile (0..{nt - 1}): {np.bincount(rows, minlength=nt)}")
        print(f"  first bad: {bad[:12]}")
DUMP = os.environ.get("DUMP")   # save the step workspace's e0 region / u,v region after the last launch
if DUMP:
    ws0 = sim._workspace(n, 11, torch.device("cuda", 0))
    nH = 5 * 2 * n * 64
    np.save(DUMP + "_e0.npy", ws0.uvl[nH:].cpu().numpy())
    np.save(DUMP + "_uv.npy", ws0.uvl[:nH].cpu().numpy())
    np.save(DUMP + "_deg.npy", ws0.step_deg.cpu().numpy())
for r in range(1, reps):
    print(f"rep {r} == rep 0 bitwise: {np.array_equal(outs[r], outs[0])}")
