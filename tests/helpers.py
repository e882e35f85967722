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


MS_CASES = ["ms2d_s3", "ms3d_h128"]


def ms_graph_of(z, device="cpu"):
    """Static graph dict (the reference's layout) from a multi-scale fixture."""
    hp = hparams(z)
    t = lambda a: torch.from_numpy(z[a]).to(device)
    gh = {s: {"sampling_indices": t(f"scale{s}_indices"), "spacing": float(z[f"scale{s}_spacing"]),
              "num_particles": int(z[f"scale{s}_indices"].shape[0])} for s in range(hp["num_scales"])}
    return {"graph_hierarchy": gh, "grid2mesh_edges": t("g2m"), "mesh2mesh_edges": t("m2m"),
            "mesh2grid_edges": t("m2g")}


def ms_product_sim(z, device="cuda"):
    from sgnn_amd.multi_scale import MultiScaleSimulator
    hp = hparams(z)
    d, T, H = hp["dim"], hp["T"], hp["H"]
    nnode_in = (T - 1) * d + 1 + (hp["emb"] if hp["ntypes"] > 1 else 0)
    sim = MultiScaleSimulator(d, nnode_in, d + 1, H, H, hp["L"], hp["nmlp"], stats_of(z, device),
                              hp["ntypes"], hp["emb"], hp["num_scales"], hp["window"], hp["mult"],
                              device=device)
    sim.load_state_dict(state_of(z))
    sim = sim.to(device)
    sim.set_static_graph(ms_graph_of(z, device))
    return sim


def ms_oracle_sim(z, graph=None):
    from oracle.multi_scale_oracle import MultiScaleOracle
    hp = hparams(z)
    return MultiScaleOracle(state_of(z), hp["dim"], hp["L"], stats_of(z), graph or ms_graph_of(z),
                            hp["num_scales"], hp["mult"], hp["ntypes"], hp["nmlp"])
