import numpy as np, torch, sys
sys.path.insert(0, '.')
from oracle import sgnn_oracle as O
from sgnn_amd import synthetic
from sgnn_amd.learned_simulator import LearnedSimulator
from sgnn_amd.train import Trainer
for L in [int(x) for x in sys.argv[1:]]:
    dim, H, nmlp, T, R = 2, 64, 1, 6, 0.75
    base = synthetic.lattice_2d(30, 20)
    seq = synthetic.trajectory(base, T + 1, seed=5)
    n = seq.shape[0]
    st = synthetic.normalization_stats(dim, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    torch.manual_seed(11)
    sim = LearnedSimulator(dim, (T - 1) * dim + 1, dim + 1, H, L, nmlp, H, R, stats, 1, 9)
    state = {k: v.detach().clone().double().requires_grad_(True) for k, v in sim.state_dict().items()}
    pos, nxt = torch.from_numpy(seq[:, :T]), torch.from_numpy(seq[:, T])
    strain = torch.from_numpy(np.random.default_rng(2).normal(0, 1, n).astype(np.float32))
    noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(3))
    st64 = {k: {kk: vv.double() for kk, vv in v.items()} for k, v in stats.items()}
    osim = O.OracleSimulator(state, dim, L, R, st64, 1, nmlp_layers=nmlp)
    pa, ta, ps = osim.predict_accelerations(nxt.double(), noise.double(), pos.double(), [n], torch.zeros(n, dtype=torch.long))
    ref_loss = O.training_loss(pa, ta, ps, strain.double())
    ref_loss.backward()
    sim = sim.cuda()
    tr = Trainer(sim, lr_init=1e-3)
    out = tr.train_step(pos.cuda(), nxt.cuda(), strain.cuda(), [n], noise=noise.cuda())
    torch.cuda.synchronize()
    print("L", L, "loss", float(out["loss"]), ref_loss.item())
    rows = []
    for k, p in sim.named_parameters():
        if state[k].grad is not None:
            g, r = p.grad.cpu().double().numpy(), state[k].grad.numpy()
            rows.append((np.abs(g - r).max() / max(np.abs(r).max(), 1e-30), k))
    rows.sort(reverse=True)
    for e, k in rows[:5]:
        print(f"   {e:.3e} {k}")
