"""Hand-off check of the one-launch step (k_step16).

A check build (-DSGNN_HANDOFF_CHECK, step16.hip) tags every node-half row a
tile hands off with the phase it is published with and records, per gathered
half and lane, a hash of the u / v words the consumer actually used; after its
last layer every tile publishes a final phase, waits for the whole grid, re-
gathers every half of every layer and compares hashes (a row read before its
producer's stores landed differs from the settled value).  Consumers also
compare the tags of every row they gather with the phase they polled for.

Variant: base = the shipping kernel.  (Round 5 also built the reconstructed round-4 experiments xcd1 /
xcd2 / xhalf here; their defines were removed from step16.hip in round 6, their records are
profiles/r05_handoff_*.log and DESIGN.md section 8.1.)

  python tools/exp_handoff.py build VARIANT          # here (CPU): _lib/libsgnn_hip_hc_VARIANT.so
  python tools/exp_handoff.py run VARIANT [SKEW]     # on the GPU box: every step test case, one line each

Each line: case, parity (ok / FAIL + message), stale halves (hash), tag mismatches, workgroups that ran
the final check.  SKEW sets sgnn_step_ws.step_skew (tile-dependent sleeps before every publish)."""
import ctypes
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {"base": ()}


def lib_path(v):
    return os.path.join(ROOT, "sgnn_amd", "_lib", f"libsgnn_hip_hc_{v}.so")


if __name__ == "__main__" and sys.argv[1] == "build":
    from sgnn_amd import build_lib
    v = sys.argv[2]
    print(build_lib.build(defines=("SGNN_HANDOFF_CHECK",) + VARIANTS[v], lib=lib_path(v)))
    sys.exit(0)

variant = sys.argv[2]
skew = int(sys.argv[3]) if len(sys.argv) > 3 else 0
import torch  # noqa: E402
from sgnn_amd import _hip, engine  # noqa: E402
engine.set_test_step_skew(skew)
_hip.load_library(lib_path(variant))
from tests import test_gpu_parity as tp, test_gpu_step as ts  # noqa: E402

lib = _hip.lib()
lib.sgnn_set_handoff_check.argtypes = [ctypes.c_void_p]
lib.sgnn_set_handoff_check.restype = ctypes.c_int
# [16] counters + tags [L][n][4] + hashes [grid][L][128][64][2] for L <= 10, n <= 8192, grid <= 256
WORDS = 16 + 10 * 8192 * 4 + 256 * 10 * 128 * 64 * 2
buf = torch.zeros(WORDS, dtype=torch.int32, device="cuda")
assert lib.sgnn_set_handoff_check(ctypes.c_void_p(buf.data_ptr())) == 0


class _MP:
    """a minimal monkeypatch for the test that takes one"""
    def __init__(self):
        self.undo = []

    def setattr(self, obj, name, val):
        self.undo.append((obj, name, getattr(obj, name)))
        setattr(obj, name, val)

    def close(self):
        for obj, name, val in reversed(self.undo):
            setattr(obj, name, val)


cases = [(f"golden[{c}]", ts.test_one_launch_matches_golden_and_kernel_sequence, (c,)) for c in tp.FWD_H64]
params = [(2, (30, 20), 15.0, 3, 3, 20), (3, (12, 10, 8), 0.75, 1, 1, 20), (2, (64, 64), 0.6, 1, 1, 20),
          (2, (9, 7), 2.0, 2, 1, 33), (2, (120, 40), 0.6, 1, 1, 20), (2, (200, 40), 0.6, 1, 1, 20),
          (3, (16, 16, 12), 0.75, 2, 3, 20), (2, (90, 40), 15.0, 2, 1, 20)]
cases += [(f"oracle[{p[0]}d {p[1]} r={p[2]} ex={p[3]}]", ts.test_one_launch_against_oracle, p) for p in params]
cases += [("rollout20[c1 r=15]", ts.test_headline_rollout_20_steps_against_oracle, ()),
          ("rollout5[6400 two sub-tiles]", ts.test_two_subtile_rollout_against_oracle, ())]
cases += [(f"one_step[{d} r={r}]", ts.test_one_step_rollout_is_one_device_call, (d, r))
          for d, r in [((50, 40), 15.0), ((160, 40), 0.6)]]
print(f"variant {variant}, skew {skew}", flush=True)
bad = 0
for name, fn, args in cases:
    buf.zero_()
    torch.cuda.synchronize()
    mp = _MP()
    try:
        if fn is ts.test_one_step_rollout_is_one_device_call:
            fn(*args, mp)
        else:
            fn(*args)
        parity = "ok"
    except AssertionError as e:
        parity = "FAIL " + " ".join(str(e).split())[:300]
    except Exception as e:  # noqa: BLE001
        parity = "ERROR " + type(e).__name__ + ": " + " ".join(str(e).split())[:300]
        traceback.print_exc()
    finally:
        mp.close()
    torch.cuda.synchronize()
    c = buf[:4].cpu().tolist()
    bad += (parity != "ok") + (c[0] > 0) + (c[1] > 0)
    print(f"{name:40s} parity {parity:6s} stale-halves {c[0]:6d} tag-mismatches {c[1]:6d} final-checks {c[3]:6d}",
          flush=True)
lib.sgnn_set_handoff_check(ctypes.c_void_p(0))
print(f"variant {variant} skew {skew}: {'CLEAN' if bad == 0 else f'{bad} problems'}", flush=True)
