"""Shared test helpers (golden fixture -> product / oracle simulators)."""
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def hparams(z):
    return {k[3:]: z[k].item() for k in z.files if k.startswith("hp_")}


def stats_of(z, device="cpu"):
    t = lambda a: torch.from_numpy(z[a]).to(device)
    return {"acceleration": {"mean": t("acc_mean"), "std": t("acc_std")},
            "velocity": {"mean": t("vel_mean"), "std": t("vel_std")}}


def state_of(z, prefix="w/"):
    return {k[len(prefix):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(prefix)}


def product_sim(z, device="cuda", prefix="w/"):
    from sgnn_amd.learned_simulator import LearnedSimulator
    hp = hparams(z)
    d, T, H = hp["dim"], hp["T"], hp["H"]
    nnode_in = (T - 1) * d + 1 + (hp["emb"] if hp["ntypes"] > 1 else 0)
    sim = LearnedSimulator(d, nnode_in, d + 1, H, hp["L"], 1, H, hp["R"], stats_of(z, device),
                           hp["ntypes"], hp["emb"], device=device)
    sim.load_state_dict(state_of(z, prefix))
    return sim.to(device)


def oracle_sim(z, prefix="w/"):
    from oracle import sgnn_oracle as O
    hp = hparams(z)
    return O.OracleSimulator(state_of(z, prefix), hp["dim"], hp["L"], hp["R"], stats_of(z), hp["ntypes"])
