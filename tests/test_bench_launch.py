"""bench.py's multi-rank launch (CPU, no GPU): `python bench.py --gpus 2`
without a torch.distributed environment must start 2 ranks itself (as a child
torch.distributed.run, before any GPU call), each joining one process group,
and rank 0 must print one JSON line with n_gpus = 2.  The stub step
(--selftest-launch) all-reduces a one over gloo instead of touching a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=240)


def test_gpus_flag_launches_that_many_ranks():
    p = _run(["--gpus", "2", "--selftest-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout          # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["allreduce_sum"] == 2.0 and out["ranks_env"] == "2"


def test_gpus_flag_must_agree_with_world_size():
    p = _run(["--gpus", "4", "--selftest-launch"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in p.stderr


def test_every_roofline_kernel_resolves_in_this_rounds_profiles():
    """The dominant kernel each bench leg names must be found in a committed
    rocprofv3 summary of the same workload (its `traffic` and
    `profiled_avg_us` come from there): a renamed template (e.g. a new
    template argument) would otherwise leave the line's traffic null."""
    import bench
    cases = [("c1_r15", "rollout", "k_step16"), ("c1_r06", "rollout", "k_step16"),
             ("t4800", "rollout", "k_step16"), ("t6400", "rollout", "k_step16"), ("t8000", "rollout", "k_step16"),
             ("c2", "rollout", "k_edge_layer"), ("c4", "rollout", "k_edge_layer"),
             ("c2", "train", "k_edge_bwd64"), ("c3", "train", "k_edge_bwd64"),
             ("c5", "train", "k_edge_items<4, 3> + 3 k_wgrad_full<1>")]
    for wl, mode, kernel in cases:
        prof = bench.profiled(wl, mode, kernel)
        assert prof is not None, (wl, mode, kernel)
        assert prof["bytes"] > 0 and prof["avg_us"] > 0
        assert "r06_" in prof["source"] or "r05_" in prof["source"], prof["source"]   # this round or the last


def test_cpu_thread_counts_skip_an_oversubscribed_affinity_leg(monkeypatch):
    import bench
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    counts, note = bench.thread_counts()
    assert counts == [16] and "256" in note
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(8)))
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.thread_counts() == ([8], None)


def test_impossible_roofline_marks_the_leg_invalid():
    """A fraction above the hardware peak is recorded as an error, its frac withheld (null), and
    bench_line_errors() lists the leg, so no physically impossible number reaches the line unmarked;
    a valid leg carries the achieved-HBM fraction of its profiled launch."""
    sys.path.insert(0, ROOT)
    import bench
    ok = bench.roofline("k_step16", 7.18e9, 85e-6, "c1_r15", "rollout")
    assert ok["frac"] is not None and 0 < ok["frac"] < 1 and "error" not in ok
    assert 0 < ok["hbm_frac"] < 1 and ok["hbm_gbs"] > 0
    bad = bench.roofline("k_step16", 7.18e9, 1e-6, "c1_r15", "rollout")
    assert bad["frac"] is None and bad["invalid_frac"] > 1 and "error" in bad
    line = {"roofline": ok, "rollout_extra": {"x": bench.leg({"value": 1.0, "roofline": bad})}}
    assert [p for p, _ in bench.bench_line_errors(line)] == ["rollout_extra.x.rf"]
    assert bench.bench_line_errors({"roofline": ok}) == []
