"""GPU: the fused random-walk noise kernel (noise_utils.py:4-39 +
learned_simulator.py:467).  The reference draws on torch's CPU generator, so
parity is distributional: iid N(0, (std/sqrt(T-1))^2) velocity increments,
integrated twice, zero first frame, noisy = pos + noise exactly; plus
reproducibility per seed."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_random_walk_noise_distribution_and_structure():
    from sgnn_amd.train import device_random_walk_noise
    n, T, d, std = 200_000, 11, 2, 0.02
    pos = torch.randn(n, T, d, device="cuda")
    noise, noisy = device_random_walk_noise(pos, std, seed=1234, offset=7)
    assert torch.equal(noisy, pos + noise)
    assert torch.all(noise[:, 0] == 0)
    nz = noise.double().cpu().numpy()
    vel = np.diff(nz, axis=1)                  # cumsum of increments
    inc = np.diff(np.concatenate([np.zeros((n, 1, d)), vel], axis=1), axis=1)   # increments
    sigma = std / np.sqrt(T - 1)
    m, s = inc.mean(), inc.std()
    assert abs(m) < 5 * sigma / np.sqrt(inc.size), m
    assert abs(s / sigma - 1) < 0.01, s / sigma
    # independence across time steps and coordinates
    flat = inc.reshape(n, -1)
    c = np.corrcoef(flat[:, :6].T)
    assert np.abs(c - np.eye(6)).max() < 0.02
    # tails of a normal: P(|z| > 3) = 0.27 %
    frac = (np.abs(inc) > 3 * sigma).mean()
    assert 0.0022 < frac < 0.0032, frac
    # per-seed reproducibility; different seeds / offsets differ
    a, _ = device_random_walk_noise(pos, std, seed=1234, offset=7)
    b, _ = device_random_walk_noise(pos, std, seed=1234, offset=8)
    e, _ = device_random_walk_noise(pos, std, seed=99, offset=7)
    assert torch.equal(a, noise) and not torch.equal(a, b) and not torch.equal(a, e)


def test_noise_offset_is_the_global_particle_index():
    """Data parallelism: a rank owning particles [a, b) of the concatenated
    batch passes offset=a and draws exactly that slice of the one-process
    noise (so ranks never share a stream and DP == one process)."""
    from sgnn_amd.train import device_random_walk_noise
    n, T, d = 10_000, 11, 2
    pos = torch.randn(n, T, d, device="cuda")
    full, _ = device_random_walk_noise(pos, 0.02, seed=77, offset=0)
    for a, b in ((0, 3000), (3000, 3001), (3001, 10_000)):
        part, _ = device_random_walk_noise(pos[a:b].contiguous(), 0.02, seed=77, offset=a)
        assert torch.equal(part, full[a:b])
    other, _ = device_random_walk_noise(pos[:3000].contiguous(), 0.02, seed=77, offset=3000)
    assert not torch.equal(other, full[:3000])


def test_trainer_default_noise_is_seeded_by_torch():
    from sgnn_amd import synthetic
    from sgnn_amd.learned_simulator import LearnedSimulator
    from sgnn_amd.train import Trainer
    seq = synthetic.trajectory(synthetic.lattice_2d(20, 10), 12, seed=3)
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    losses = []
    for _ in range(2):
        torch.manual_seed(5)
        sim = LearnedSimulator(2, 21, 3, 64, 2, 1, 64, 0.6, stats, 1, 9).cuda()
        tr = Trainer(sim)
        pos, nxt = torch.from_numpy(seq[:, :11]).cuda(), torch.from_numpy(seq[:, 11]).cuda()
        out = tr.train_step(pos, nxt, torch.zeros(seq.shape[0], device="cuda"), [seq.shape[0]])
        losses.append(float(out["loss"]))
    assert losses[0] == losses[1]
