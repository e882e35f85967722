"""Same-box A/B of library builds on bench legs: every (library, workload) pair runs in a fresh
process (the library is chosen before anything loads the default one), alternating A, B, A, B.

  python tools/exp_ab.py build NAME DEFINE[=V] ...   # here (CPU): _lib/libsgnn_hip_NAME.so
  python tools/exp_ab.py run LIB_A,LIB_B WORKLOAD,... [reps]   # on the GPU box (LIB: default or NAME, optionally @VAR=VALUE;
                                                             # WORKLOAD: a rollout workload, train or train-c3)"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIBDIR = os.path.join(ROOT, "sgnn_amd", "_lib")


def lib_path(name):
    return os.path.join(LIBDIR, "libsgnn_hip.so" if name == "default" else f"libsgnn_hip_{name}.so")


if sys.argv[1] == "build":
    from sgnn_amd import build_lib
    print(build_lib.build(defines=tuple(sys.argv[3:]), lib=lib_path(sys.argv[2])))
elif sys.argv[1] == "one":   # child: one bench leg on one library
    import torch
    from sgnn_amd import _hip
    _hip.load_library(lib_path(sys.argv[2].split("@")[0]))
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if sys.argv[3] in ("train", "train-c3"):   # the C2 / C3 training step (kernel = the edge backward)
        r = bench.bench_train(sys.argv[3], 20, 5, 1, 0, dev, 0, 0)
    elif sys.argv[3] == "c5":                  # the C5 multi-scale training step
        r = bench.bench_ms_train("c5", 3, 1, 1, 0, dev, 0, 0)
    else:
        r = bench.bench_rollout(sys.argv[3], 20, 5, 1, 0, dev, 0, 0)
    print(json.dumps({"lib": sys.argv[2], "workload": sys.argv[3], "ms_per_step": r["ms_per_step"],
                      "kernel_us": r["roofline"]["live_us"]}))
else:
    libs, wls = sys.argv[2].split(","), sys.argv[3].split(",")
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    for wl in wls:
        for rep in range(reps):
            for lib in libs:
                env = dict(os.environ)   # LIB@VAR=VALUE: the child runs with VAR=VALUE set (Python-side switches)
                for kv in lib.split("@")[1:]:
                    env[kv.split("=")[0]] = kv.split("=", 1)[1]
                out = subprocess.run([sys.executable, os.path.abspath(__file__), "one", lib, wl], capture_output=True,
                                     text=True, timeout=300, cwd=ROOT, env=env)
                if out.returncode != 0:
                    print(out.stderr[-2000:])
                    sys.exit(out.returncode)
                print(out.stdout.strip().splitlines()[-1], flush=True)
