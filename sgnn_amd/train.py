"""Trainer: the reference's training step (sgnn/single_scale/train.py:231-280)
on the HIP kernels, with whole-graph data parallelism over RCCL.

One step = random-walk noise (noise_utils.py:4-39) -> noisy window ->
saved-activation forward -> fused loss + backward -> (world > 1: one SUM
all-reduce of the flat gradient over RCCL/xGMI) -> fused Adam -> LR decay
`lr_init * lr_decay ** (step / lr_decay_steps) + 1e-6` applied after the step
(train.py:276-278).

Data parallelism: every rank owns whole graphs.  The
reference averages the loss over all particles of the concatenated batch
(train.py:268), so each rank scales its loss gradient by 1/N_global (the
particle count over all ranks) and the SUM all-reduce yields exactly the
single-process gradient; every rank then applies the identical Adam update.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import engine, training


def random_walk_noise(position_sequence: torch.Tensor, noise_std_last_step: float,
                      generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """noise_utils.py:4-39 on the tensor's device (the reference draws on the CPU
    default generator; pass a CPU tensor + generator for its exact stream)."""
    n, T, d = position_sequence.shape
    nv = T - 1
    vn = torch.randn((n, nv, d), generator=generator, dtype=torch.float32,
                     device=position_sequence.device) * (noise_std_last_step / nv ** 0.5)
    vn = torch.cumsum(vn, dim=1)
    return torch.cat([torch.zeros_like(vn[:, 0:1]), torch.cumsum(vn, dim=1)], dim=1)


class DataParallel:
    """Whole-graph DP bookkeeping shared by the GPU trainer and its CPU (gloo) tests."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1

    def global_count(self, n_local: int, device) -> int:
        """N_global = sum of particles over ranks (train.py:268 mean denominator)."""
        if self.world == 1:
            return int(n_local)
        t = torch.tensor([float(n_local)], dtype=torch.float64, device=device)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def allreduce_(self, *tensors: torch.Tensor) -> None:
        """SUM all-reduce (RCCL over xGMI on MI355X; gloo in CPU tests)."""
        if self.world == 1:
            return
        for t in tensors:
            dist.all_reduce(t, group=self.group)


class Trainer:
    """Drop-in training loop body for a sgnn_amd.LearnedSimulator."""

    def __init__(self, simulator, lr_init: float = 1e-3, lr_decay: float = 0.1,
                 lr_decay_steps: int = 30000, noise_std: float = 0.02,
                 loss_weight_position: float = 1.0, loss_weight_strain: float = 1.0,
                 group=None, nslab: int = training.DEFAULT_NSLAB):
        self.sim = simulator
        self.epd = simulator._encode_process_decode
        training.check_trainable(self.epd, simulator._nparticle_types)
        self.flat = training.FlatParams(simulator)
        self.opt = training.Adam(self.flat, lr_init)
        self.grads: Dict[str, torch.Tensor] = {k: p.grad for k, p in simulator.named_parameters()}
        self.lr_init, self.lr_decay, self.lr_decay_steps = lr_init, lr_decay, lr_decay_steps
        self.noise_std = noise_std
        self.w_pos, self.w_strain = loss_weight_position, loss_weight_strain
        self.dp = DataParallel(group)
        self.nslab = nslab
        self.step = 0
        self._tw: Dict[tuple, training.TrainWorkspace] = {}
        self._count_cache: Dict[int, int] = {}

    def workspace(self, n: int, T: int, device) -> training.TrainWorkspace:
        key = (n, T, str(device))
        tw = self._tw.get(key)
        if tw is None:
            if len(self._tw) > 4:
                self._tw.clear()
            tw = training.TrainWorkspace(self.epd, n, T, self.sim._particle_dimensions,
                                         self.sim._max_num_neighbors, True, device, self.nslab)
            self._tw[key] = tw
        return tw

    def train_step(self, position: torch.Tensor, next_position: torch.Tensor,
                   next_strain: torch.Tensor, nparticles_per_example, particle_types=None,
                   noise: Optional[torch.Tensor] = None, n_global: Optional[int] = None,
                   timers: Optional[dict] = None) -> dict:
        """One optimisation step on this rank's graphs; returns device-side loss
        terms (no host sync).  `noise` defaults to fresh random-walk noise."""
        pos = position.to(torch.float32).contiguous()
        if noise is None:
            noise = random_walk_noise(pos, self.noise_std)
        noise = noise.to(pos.device, torch.float32).contiguous()
        noisy = (pos + noise).contiguous()                          # learned_simulator.py:467
        inp, _ = self.sim._step_inputs(noisy, nparticles_per_example, particle_types)
        n, T, _ = noisy.shape
        tw = self.workspace(n, T, pos.device)
        if n_global is None:
            n_global = self._count_cache.get(n)
            if n_global is None:
                n_global = self.dp.global_count(n, pos.device)
                self._count_cache[n] = n_global
        radius = self.sim._connectivity_radius
        emb = self.sim._particle_type_embedding.weight if self.sim._nparticle_types > 1 else None
        training.train_forward(self.epd, radius, inp, tw, timers=timers, emb_weight=emb)
        training.train_backward(self.epd, radius, inp, tw, self.grads, timers=timers,
                                next_pos=next_position.to(torch.float32).contiguous(), noise=noise,
                                next_strain=next_strain.to(torch.float32).contiguous(),
                                w_pos=self.w_pos, w_strain=self.w_strain, inv_count=1.0 / n_global,
                                emb_weight=emb, emb_grad=self.grads.get("_particle_type_embedding.weight"))
        self.dp.allreduce_(self.flat.grad, tw.loss_out)
        self.opt.step()
        # train.py:276-278: LR for the NEXT step, computed from the pre-increment step
        self.opt.lr = self.lr_init * (self.lr_decay ** (self.step / self.lr_decay_steps)) + 1e-6
        self.step += 1
        lo = tw.loss_out
        return {"loss": lo[0] / n_global, "loss_position": (lo[1] + lo[2] + lo[3]) / n_global,
                "loss_strain": lo[4] / n_global, "loss_xyz": lo[1:4] / n_global,
                "n_global": n_global, "lr": self.opt.lr}
