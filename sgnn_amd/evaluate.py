"""Rollout loop and metric with the reference's signature and output dict
(sgnn/single_scale/evaluate.py:23-175)."""
from __future__ import annotations

import time

import numpy as np
import torch

EROSIONAL_PARTICLE_ID = -1  # evaluate.py:17
RMSE_PRINT_INTERVAL = 3


def rollout_rmse(pred: np.ndarray, gt: np.ndarray, verbose: bool = False) -> np.ndarray:
    """evaluate.py:23-48: accumulated RMSE sqrt(cumsum(mean sq)/t)."""
    if pred.shape != gt.shape:
        raise ValueError(f"Shape mismatch: pred {pred.shape} vs gt {gt.shape}")
    t = gt.shape[0]
    sq = np.square(pred - gt).reshape(t, -1)
    loss = np.sqrt(np.cumsum(np.mean(sq, axis=1), axis=0) / np.arange(1, t + 1))
    if verbose:
        for s in range(0, t, RMSE_PRINT_INTERVAL):
            print("Testing rmse @ step %d loss: %.2e" % (s, loss[s]))
    return loss


@torch.no_grad()
def rollout(simulator, position: torch.Tensor, particle_types: torch.Tensor, n_particles_per_example,
            strains: torch.Tensor, nsteps: int, particle_dim: int, device, input_sequence_length: int = 3,
            inference_mode: str = "autoregressive") -> dict:
    """evaluate.py:51-175 (same validation, loop, erosional mask and dict)."""
    if position.dim() != 3:
        raise ValueError(f"Position tensor must be 3D, got {position.dim()}D")
    if strains.dim() != 2:
        raise ValueError(f"Strains tensor must be 2D, got {strains.dim()}D")
    if position.shape[0] != strains.shape[1]:
        raise ValueError(f"Number of particles mismatch: position {position.shape[0]} vs strains {strains.shape[1]}")
    if position.shape[1] < input_sequence_length:
        raise ValueError(f"Position sequence length {position.shape[1]} must be >= input_sequence_length "
                         f"{input_sequence_length}")
    if inference_mode not in ("autoregressive", "one_step"):
        raise ValueError(f"Unknown inference_mode: {inference_mode}. Must be 'autoregressive' or 'one_step'")
    initial_positions = position[:, :input_sequence_length]
    initial_strains = strains[:input_sequence_length, :]
    ground_truth_positions = position[:, input_sequence_length:]
    ground_truth_strains = strains[input_sequence_length:, :]
    nsteps = ground_truth_strains.shape[0]
    current = initial_positions
    pred_positions, pred_strains = [], []
    erosional = (particle_types == EROSIONAL_PARTICLE_ID).clone().detach().to(device)
    erosional = erosional.bool()[:, None].expand(-1, particle_dim)
    any_erosional = bool(erosional.any())
    start = time.time()
    fast = (not any_erosional and nsteps > 0 and hasattr(simulator, "rollout_runner") and position.is_cuda
            and getattr(simulator, "_fast_path", lambda: True)())
    if fast:
        # device-resident loop: one sgnn_rollout call (window shift fused into the
        # decoder kernel; same kernels and arithmetic as predict_positions); one_step
        # (:140-143) is one sgnn_rollout_one_step call: each next window ends with the
        # step's ground-truth frame
        runner = simulator.rollout_runner(initial_positions, [n_particles_per_example], particle_types, nsteps)
        gt = None if inference_mode == "autoregressive" else ground_truth_positions
        pred_positions, pred_strains = runner.run(ground_truth=gt)
        nsteps = 0
    for step in range(nsteps):
        nxt, ps = simulator.predict_positions(current, nparticles_per_example=[n_particles_per_example],
                                              particle_types=particle_types)
        gt_pos = ground_truth_positions[:, step]
        if any_erosional:
            nxt = torch.where(erosional, gt_pos, nxt)
            ps = torch.where(erosional[:, 0], ground_truth_strains[step, :], ps)
        pred_positions.append(nxt)
        pred_strains.append(ps)
        src = nxt if inference_mode == "autoregressive" else gt_pos
        current = torch.cat([current[:, 1:], src[:, None, :]], dim=1)
    if torch.cuda.is_available() and position.is_cuda:
        torch.cuda.synchronize(position.device)
    run_time = time.time() - start
    if not fast:
        pred_positions = torch.stack(pred_positions)
        pred_strains = torch.stack(pred_strains)
    ground_truth_positions = ground_truth_positions.permute(1, 0, 2)
    rmse_position = rollout_rmse(pred_positions.cpu().numpy(), ground_truth_positions.cpu().numpy())
    rmse_strain = rollout_rmse(pred_strains.cpu().numpy(), ground_truth_strains.cpu().numpy())
    return {
        "initial_positions": initial_positions.permute(1, 0, 2).cpu().numpy(),
        "initial_strains": initial_strains.cpu().numpy(),
        "predicted_rollout": pred_positions.cpu().numpy(),
        "ground_truth_rollout": ground_truth_positions.cpu().numpy(),
        "ground_truth_strain": ground_truth_strains.cpu().numpy(),
        "predicted_strain": pred_strains.cpu().numpy(),
        "particle_types": particle_types.cpu().numpy(),
        "rmse_position": rmse_position,
        "rmse_strain": rmse_strain,
        "run_time": run_time,
        "inference_mode": inference_mode,
    }
