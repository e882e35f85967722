"""Expected HBM/MALL traffic of one k_step16 launch, term by term (VERDICT r04 item 2:
attribute the measured FETCH_SIZE / WRITE_SIZE bytes before changing the kernel).

Terms, per launch (one predict_positions step):
  window      the position window read + written (2 n T d 4 B) -- algorithmic
  uv_write    every layer's node halves u_k, v_k written through (sc1) once: 2 n H 4 B per layer -- algorithmic
  uv_read     what the consumers fetch: every tile reads the u rows of its own receivers and the v rows of its
              UNIQUE senders.  An sc1 store drops the line from the writer's XCD L2, so the first reader on
              an XCD fetches it from MALL/HBM and later readers on that XCD hit L2.  Under the dispatch order
              (blocks b, b + 8, ... share an XCD) neighbouring tiles sit on different XCDs: each (row, XCD)
              pair is one fetch.  The algorithmic count is one read per row (uv_read_alg).
  weights     every layer's weights (edge W1e, W2 into LDS; node W1 [2H x H], W2, next u/v halves [2H x H] into
              VGPRs) read by every workgroup: one L2 miss per XCD per layer
  e0          two-sub-tile graphs (> 16 receivers per tile) keep the tile's edge latents in a per-tile HBM block:
              written once, read back every layer (L2-resident only while it fits)

  python tools/traffic_model.py [workload ...]      (CPU only: the oracle's radius graph)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import sgnn_oracle as O  # noqa: E402
from sgnn_amd import synthetic  # noqa: E402

XCDS = 8


def tiles_to_xcd(G, order):
    """XCD of each tile: dispatch order (tile = block, XCD = block mod 8) or XCD-contiguous tiles."""
    if order == "dispatch":
        return np.arange(G) % XCDS
    q, r = divmod(G, XCDS)
    x = np.empty(G, np.int64)
    t = 0
    for c in range(XCDS):
        k = q + (1 if c < r else 0)
        x[t:t + k] = c
        t += k
    return x


def model(wl, order="dispatch", K=20):
    dims, radius, H, L = bench.WORKLOADS[wl]
    seq = synthetic.trajectory(bench.lattice(dims), bench.T_SEQ, seed=1000)
    n, T, d = seq.shape
    ei = O.radius_graph(torch.from_numpy(seq[:, -1]), [n], radius, max_num_neighbors=K).numpy()
    E = ei.shape[1]
    nt = max(8, -(-n // 256))
    G = -(-n // nt)
    send, recv = ei[0], ei[1]
    xcd = tiles_to_xcd(G, order)
    pairs = set()          # (row, XCD) fetches of v rows
    for t in range(G):
        for s in np.unique(send[recv // nt == t]):
            pairs.add((int(s), int(xcd[t])))
    row = 4 * H
    terms = {
        "window": 2 * n * T * d * 4,
        "uv_write": 2 * n * row * L,
        "uv_read_alg": 2 * n * row * L,
        "uv_read": (len(pairs) + n) * row * L,     # v rows per (row, XCD) + own u rows
        "weights": XCDS * L * (2 * H * H + 2 * H * H + H * H + 2 * H * H) * 4,
        "e0": (E * (H + 4) * 4 * (1 + L)) if nt > 16 else 0,
    }
    alg = terms["window"] + terms["uv_write"] + terms["uv_read_alg"]
    exp = terms["window"] + terms["uv_write"] + terms["uv_read"] + terms["weights"] + terms["e0"]
    return n, E, nt, G, terms, alg, exp


if __name__ == "__main__":
    for wl in sys.argv[1:] or ["c1_r15", "c1_r06", "t4800", "t6400", "t8000"]:
        for order in ("dispatch", "xcd"):
            n, E, nt, G, t, alg, exp = model(wl, order)
            print(f"{wl:7s} {order:8s} n={n} E={E} nt={nt} G={G}: algorithmic {alg / 1e6:6.2f} MB, expected "
                  f"{exp / 1e6:6.2f} MB = " + ", ".join(f"{k} {v / 1e6:.2f}" for k, v in t.items() if k != "uv_read_alg"))
