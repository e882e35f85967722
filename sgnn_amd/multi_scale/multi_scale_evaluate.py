"""Multi-scale rollout with the reference's signature and output dict
(sgnn/multi_scale/multi_scale_evaluate.py:139-252).  Each step is one fused
HIP launch chain; the position window shifts on the device (no torch.cat)."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch


@torch.no_grad()
def evaluate_multi_scale_rollout(simulator, positions: torch.Tensor, particle_type: torch.Tensor,
                                 n_particles_per_example, strains: torch.Tensor, nsteps: int, dim: int,
                                 device, input_sequence_length: int,
                                 inference_mode: str = "autoregressive") -> Dict[str, Any]:
    T = input_sequence_length
    cur = positions[:, :T].to(torch.float32).contiguous().clone()
    nxt_win = torch.empty_like(cur)
    pred_pos, pred_str, rmse_p, rmse_s = [], [], [], []
    for step in range(nsteps):
        target = positions[:, T + step]
        target_strain = strains[T + step, :]
        if inference_mode == "autoregressive":
            # predict + shift the window inside node_layer_decode (window_out)
            _, pred, nxt = simulator._run(cur, particle_type, window_out=nxt_win)
            cur, nxt_win = nxt_win, cur
        else:
            _, pred, nxt = simulator._run(cur, particle_type)
            cur = torch.cat([cur[:, 1:], target.unsqueeze(1).to(cur.dtype)], dim=1).contiguous()
        st = pred[:, -1]
        pe = torch.norm(nxt - target, dim=-1)
        se = torch.abs(st - target_strain)
        rmse_p.append(torch.sqrt(torch.mean(pe ** 2)).item())
        rmse_s.append(torch.sqrt(torch.mean(se ** 2)).item())
        pred_pos.append(nxt.cpu().numpy())
        pred_str.append(st.cpu().numpy())
    gt = positions[:, T:T + nsteps].cpu().numpy()
    return {
        "initial_positions": positions[:, :T].cpu().numpy().transpose(1, 0, 2),
        "initial_strains": strains[:T].cpu().numpy(),
        "predicted_rollout": np.array(pred_pos),
        "ground_truth_rollout": gt.transpose(1, 0, 2),
        "ground_truth_strain": strains[T:T + nsteps].cpu().numpy(),
        "predicted_strain": np.array(pred_str),
        "particle_types": particle_type.cpu().numpy(),
        "rmse_position": np.array(rmse_p),
        "rmse_strain": np.array(rmse_s),
        "run_time": 0.0,
        "inference_mode": inference_mode,
    }
