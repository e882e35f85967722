"""Compare two step-workspace dumps of tools/exp_localize.py (DUMP=...): the
per-tile HBM e0 rows (within each tile's edge count) and the node halves."""
import sys
import numpy as np
A, B = sys.argv[1], sys.argv[2]
n, nt, cap, LDX, L = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), 68, 5
G = -(-n // nt)
ecap = nt * cap
b, m = np.load(A + "_e0.npy"), np.load(B + "_e0.npy")
db, dm = np.load(A + "_deg.npy"), np.load(B + "_deg.npy")
print("deg equal", np.array_equal(db, dm))
bb, mm = b[:G * ecap * LDX].reshape(G, ecap, LDX), m[:G * ecap * LDX].reshape(G, ecap, LDX)
Et = np.array([db[t * nt:(t + 1) * nt].sum() for t in range(G)])
bad, nanr, shown = 0, 0, 0
for t in range(G):
    E = Et[t]
    eb, em = bb[t, :E, :64], mm[t, :E, :64]
    diff = ~np.isclose(eb, em, atol=1e-6, rtol=0, equal_nan=True)
    rows = np.nonzero(diff.any(1))[0]
    bad += len(rows)
    nanr += int(np.isnan(em).any(1).sum())
    if len(rows) and shown < 6:
        shown += 1
        print(f"tile {t} Et {E}: {len(rows)} rows differ, first {rows[:16]}, cols {np.nonzero(diff[rows[0]])[0][:16]}, "
              f"B row {em[rows[0], :4]} A row {eb[rows[0], :4]}")
print(f"e0 rows differing {bad}, B rows with NaN {nanr}, Et {Et.min()}..{Et.max()}")
ub, um = np.load(A + "_uv.npy").reshape(2 * L, n, 64), np.load(B + "_uv.npy").reshape(2 * L, n, 64)
for k in range(2 * L - 2):
    d = np.abs(ub[k] - um[k])
    print(f"uv buffer {k}: max diff {np.nanmax(d):.3e}, rows > 1e-4: {(d.max(1) > 1e-4).sum()}, NaN rows {np.isnan(um[k]).any(1).sum()}")
for k in (4, 5, 6):
    d = np.abs(ub[k] - um[k]).max(1)
    rows = np.nonzero(d > 1e-4)[0]
    print(f"buffer {k}: differing rows mod nt {np.bincount(rows % nt, minlength=nt)}; tiles {np.unique(rows // nt).size}; "
          f"first rows {rows[:12]}")
