"""GPU: the training / rollout harness on a Taylor-format dataset (SURVEY §8(f)
rows 1-3): train() from device-resident samples with validation-gated
checkpoints, resume from those files (weights + fused-Adam state + step), and
predict() writing the reference's rollout pickles."""
import json
import os
import pickle

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dataset(root):
    from sgnn_amd import data as D, synthetic
    frames = 14
    def split(name, seeds, sizes):
        tr = {}
        for s, (nx, ny) in zip(seeds, sizes):
            seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny), frames, seed=s)   # [N, T, 2]
            pos = np.transpose(seq, (1, 0, 2)).copy()                                 # [T, N, 2]
            stress = np.random.default_rng(s).normal(size=(frames, pos.shape[1]))
            tr[f"{name}_{s}"] = (pos, np.zeros(pos.shape[1], np.int64), stress)
        D.save_trajectories(os.path.join(root, f"{name}.npz"), tr, reference_format=True)
        return [k + ".npz" for k in tr]
    md = {"sequence_length": frames, "dim": 2, "num_particle_types": 1,
          "vel_mean": [-1e-3, 2e-3], "vel_std": [2e-2, 3e-2], "acc_mean": [1e-4, -2e-4], "acc_std": [3e-3, 4e-3],
          "stress_mean": 0.0, "stress_std": 1.0}
    md["file_train"] = split("train", [1, 2], [(10, 8), (12, 8)])
    md["file_valid"] = split("valid", [3], [(10, 8)])
    md["file_test"] = split("test", [4, 5], [(10, 8), (11, 8)])
    with open(os.path.join(root, "metadata.json"), "w") as f:
        json.dump(md, f)
    return md


def _config(root):
    return {"mode": "train", "data_path": str(root), "model_path": str(root / "models"),
            "output_path": str(root / "rollouts"), "layers": 2, "hidden_dim": 64, "dim": 2,
            "particle_type_embedding_size": 9, "input_sequence_length": 6, "connection_radius": 0.6,
            "batch_size": 2, "noise_std": 0.02, "ntraining_steps": 4, "nsave_steps": 2,
            "loss_weight_position": 1.0, "loss_weight_strain": 1.0, "lr_init": 1e-3, "lr_decay": 0.1,
            "lr_decay_steps": 100, "run_name": "r", "model_file": None, "train_state_file": "train_state.pt",
            "inference_mode": "autoregressive"}


def test_train_checkpoint_resume_and_predict(tmp_path):
    from sgnn_amd import data as D, train as T
    md = _dataset(str(tmp_path))
    cfg = _config(tmp_path)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    sim = T._get_simulator(D.read_metadata(str(tmp_path)), 0.02, 0.02, dev, cfg).to(dev)
    res = T.train(sim, md, dev, cfg, log_every=1)
    assert res["step"] == 4
    losses = [l for _, l in res["history"]]
    assert len(losses) == 4 and all(np.isfinite(losses))
    run = tmp_path / "models" / "r"
    assert (run / "model-best-000002.pt").exists() and (run / "train_state-best-000002.pt").exists()
    assert res["trainer"].opt.step_count == 4

    # resume from the step-2 checkpoint and continue to step 5
    cfg2 = dict(cfg, model_file="model-best-000002.pt", train_state_file="train_state-best-000002.pt",
                ntraining_steps=5, nsave_steps=0)
    torch.manual_seed(1)
    sim2 = T._get_simulator(md, 0.02, 0.02, dev, cfg).to(dev)
    res2 = T.train(sim2, md, dev, cfg2, log_every=1)
    assert res2["history"][0][0] == 3 and res2["step"] == 5
    assert res2["trainer"].opt.step_count == 5
    assert (run / "model-final-000005.pt").exists()
    ts = torch.load(run / "train_state-final-000005.pt", weights_only=True)
    opt = torch.optim.Adam(sim2.parameters())
    opt.load_state_dict(ts["optimizer_state"])          # reference-loadable
    assert ts["global_train_state"]["step"] == 5

    # rollout mode: one pickle per test case with the reference's keys
    cfg3 = dict(cfg, mode="rollout", model_file="model-final-000005.pt")
    losses = T.predict(sim2, md, dev, cfg3)
    assert len(losses) == 2 and all(np.isfinite(losses))
    for name in md["file_test"]:
        with open(tmp_path / "rollouts" / "r" / name.replace(".npz", ".pkl"), "rb") as f:
            out = pickle.load(f)     # written by this test
        assert out["case_name"] == name.replace(".npz", "")
        assert out["predicted_rollout"].shape[0] == md["sequence_length"] - cfg["input_sequence_length"]
        assert out["rmse_position"].shape == (8,) and out["metadata"]["file_test"] == md["file_test"]
