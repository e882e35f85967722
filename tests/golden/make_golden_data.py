#!/usr/bin/env python3
"""Golden fixture for real-data ingestion, produced BY
THE REFERENCE'S OWN LOADER.

Run here (the build container), never on the GPU box.  It writes a small
synthetic split in the reference's on-disk format (a `trajectories` dict of
(positions[T,N,2], particle_types[N], stresses[T,N]) saved with np.savez, plus
metadata.json) into a temporary directory -- a file this script wrote, not
one shipped with the reference -- then runs the reference's
datasets/taylor_impact_2d/taylor_impact_data_loader.py on it:
TaylorImpactSamplesDataset (length, __getitem__ at chosen indices),
collate_fn, the DataLoader of get_data_loader_by_samples (no shuffle),
TaylorImpactTrajectoriesDataset, get_dataset_info and denormalize_stress.
Only the input arrays and the loader's outputs are stored
(tests/golden/loader_taylor.npz); no reference source is kept.

Usage:  python tests/golden/make_golden_data.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF_LOADER = "/root/reference/datasets/taylor_impact_2d/taylor_impact_data_loader.py"

SIZES = (20, 24, 16)       # particles per trajectory
FRAMES = (14, 12, 15)      # frames per trajectory
INPUT_LEN = 6              # input_length_sequence
SAMPLE_IDX = (0, 1, 7, 8, 9, 13, 14, 15, 21, 22)   # len = 8 + 6 + 9 = 23
STRESS_MEAN, STRESS_STD = 2.5, 4.0


def _load_reference_loader():
    spec = importlib.util.spec_from_file_location("reference_taylor_impact_loader", REF_LOADER)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def synthetic_split(seed=0):
    rng = np.random.default_rng(seed)
    out = {}
    for k, (n, t) in enumerate(zip(SIZES, FRAMES)):
        pos = rng.normal(size=(t, n, 2)).astype(np.float32)
        types_ = np.full(n, k % 2, dtype=np.int64)       # one type per trajectory (the loader reads types[0])
        stress = rng.normal(size=(t, n)).astype(np.float64)
        out[f"traj_{k}"] = (pos, types_, stress)
    return out


def main():
    L = _load_reference_loader()
    trajs = synthetic_split()
    res = {"input_len": np.int64(INPUT_LEN), "sample_idx": np.asarray(SAMPLE_IDX, np.int64),
           "stress_mean": np.float64(STRESS_MEAN), "stress_std": np.float64(STRESS_STD)}
    for k, (name, (p, t, s)) in enumerate(trajs.items()):
        res[f"in{k}_positions"], res[f"in{k}_types"], res[f"in{k}_stresses"] = p, t, s
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "train.npz")
        np.savez(path, trajectories=trajs)   # build_dataset.py:313's format
        with open(os.path.join(d, "metadata.json"), "w") as f:
            json.dump({"stress_mean": STRESS_MEAN, "stress_std": STRESS_STD, "sequence_length": 14}, f)
        ds = L.TaylorImpactSamplesDataset(path, input_length_sequence=INPUT_LEN)
        res["samples_len"] = np.int64(len(ds))
        items = [ds[i] for i in SAMPLE_IDX]
        for i, it in zip(SAMPLE_IDX, items):
            res[f"s{i}_positions"] = it["input"]["positions"]
            res[f"s{i}_particle_type"] = it["input"]["particle_type"]
            res[f"s{i}_n"] = np.int64(it["input"]["n_particles_per_example"])
            res[f"s{i}_next_position"] = it["output"]["next_position"]
            res[f"s{i}_next_strain"] = it["output"]["next_strain"]
            res[f"s{i}_traj"] = np.int64(it["meta"]["trajectory_idx"])
            res[f"s{i}_time"] = np.int64(it["meta"]["time_idx"])
        b = L.collate_fn([ds[i] for i in (1, 9, 21)])
        res["c_positions"] = b["input"]["positions"].numpy()
        res["c_particle_type"] = b["input"]["particle_type"].numpy()
        res["c_n"] = b["input"]["n_particles_per_example"].numpy()
        res["c_next_position"] = b["output"]["next_position"].numpy()
        res["c_next_strain"] = b["output"]["next_strain"].numpy()
        res["c_traj"] = b["meta"]["trajectory_idx"].numpy()
        res["c_time"] = b["meta"]["time_idx"].numpy()
        dl = L.get_data_loader_by_samples(path, input_length_sequence=INPUT_LEN, batch_size=4, shuffle=False,
                                          pin_memory=False)
        batches = list(dl)
        res["dl_nbatches"] = np.int64(len(batches))
        for k in (0, len(batches) - 1):
            res[f"dl{k}_positions"] = batches[k]["input"]["positions"].numpy()
            res[f"dl{k}_n"] = batches[k]["input"]["n_particles_per_example"].numpy()
            res[f"dl{k}_time"] = batches[k]["meta"]["time_idx"].numpy()
            res[f"dl{k}_next_strain"] = batches[k]["output"]["next_strain"].numpy()
        res["dl_last"] = np.int64(len(batches) - 1)
        tds = L.TaylorImpactTrajectoriesDataset(path)
        res["traj_len"] = np.int64(len(tds))
        for k in range(len(tds)):
            it = tds[k]
            res[f"t{k}_positions"] = it["positions"].numpy()
            res[f"t{k}_particle_type"] = it["particle_type"].numpy()
            res[f"t{k}_n"] = np.int64(it["n_particles_per_example"].item())
            res[f"t{k}_strains"] = it["strains"].numpy()
        info = L.get_dataset_info(path)
        res["info_json"] = np.asarray(json.dumps({k: (v if not isinstance(v, list) else [float(x) for x in v])
                                                  for k, v in info.items()}, sort_keys=True))
        res["denorm_in"] = np.linspace(-2.0, 2.0, 5)
        res["denorm_out"] = ds.denormalize_stress(res["denorm_in"])
    out = os.path.join(HERE, "loader_taylor.npz")
    np.savez_compressed(out, **res)
    print(f"loader_taylor: {len(SAMPLE_IDX)} samples, {int(res['dl_nbatches'])} loader batches -> "
          f"{os.path.getsize(out) / 1e3:.0f} KB")


if __name__ == "__main__":
    torch.manual_seed(0)
    main()
