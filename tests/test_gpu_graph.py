"""HIP-graph capture and replay of the predict_positions step (VERDICT r02
item 9: round 1 saw an illegal address replaying a captured Python-driven
rollout at the C1 r = 15 shape).  The step is captured as two ping-pong steps
(window A -> B -> A, the old runner's form) with torch.cuda.graph and replayed;
every replay must reproduce the eager steps bit for bit -- the same kernels on
the same inputs -- on each launch path the step has: the one-launch step
(k_step16, n <= 8,192), the per-layer fused kernels (its fallback, n <= 8,192) and the
general edge/node kernels with the cell-list radius graph (larger n).  A stale
host-side plan or an out-of-range read that eager execution happens to survive
shows up here as a mismatch or a fault."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sim(n_dims, radius, dev):
    import bench
    return bench.quiet_decoder(bench.make_sim(64, 5, radius, len(n_dims), dev, 0))


@pytest.mark.parametrize("dims,radius,path", [
    ((50, 40), 15.0, "one-launch"),      # C1 r = 15: the shape round 1 faulted at
    ((80, 60), 0.6, "one-launch"),       # 4,800 particles: two node sub-tiles per workgroup
    ((80, 60), 0.6, "fused layers"),     # the same with the one-launch step off (its fallback)
    ((120, 100), 0.6, "edge/node"),      # 12,000 particles
])
def test_graph_replay_matches_eager(dims, radius, path):
    import bench
    from sgnn_amd import engine, synthetic
    dev = torch.device("cuda", 0)
    sim = _sim(dims, radius, dev)
    seq = synthetic.trajectory(bench.lattice(dims), bench.T_SEQ, seed=5)
    n = seq.shape[0]
    w0 = torch.from_numpy(seq).to(dev)
    types_ = torch.zeros(n, dtype=torch.long, device=dev)
    inp, use_emb = sim._step_inputs(w0, [n], types_)
    ws = sim._workspace(n, bench.T_SEQ, dev)
    if path == "fused layers":
        ws = engine.StepWorkspace(n, bench.T_SEQ, len(dims), 64, sim._max_num_neighbors, True, dev, one_launch=False)
    pk = engine.ParamPack.get(sim._encode_process_decode)
    one = engine.step_path(pk.epd, engine.step_in(inp, ws, radius, sim._particle_type_embedding.weight, use_emb),
                           ws)[0]
    assert one == (path == "one-launch"), (path, one)
    emb = sim._particle_type_embedding.weight
    win = [inp.pos_seq.clone(), torch.empty_like(inp.pos_seq)]
    pred = torch.empty(n, len(dims) + 1, device=dev)
    nxt = torch.empty(n, len(dims), device=dev)
    out = torch.empty(2, n, len(dims), device=dev)

    def two_steps():
        for k in range(2):
            inp.pos_seq = win[k]
            engine.forward_step(sim._encode_process_decode, emb, use_emb, radius, inp, ws, pred, nxt,
                                window_out=win[1 - k])
            out[k].copy_(nxt)

    # eager reference: 6 steps from the initial window
    ref = []
    with torch.no_grad():
        for _ in range(3):
            two_steps()
            ref.append(out.clone())
        torch.cuda.synchronize()
        # capture (warm-up on a side stream first, as torch.cuda.graph asks), then replay from the start
        win[0].copy_(w0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            two_steps()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            two_steps()
        win[0].copy_(w0)
        got = []
        for _ in range(3):
            g.replay()
            got.append(out.clone())
        torch.cuda.synchronize()
    for r, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"{path}: replay {r} differs from eager by {float((a - b).abs().max()):.3e}"
    if one:
        assert not ws.step_timeout()
    assert np.isfinite(got[-1].cpu().numpy()).all()
