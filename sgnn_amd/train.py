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
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import engine, training


def device_random_walk_noise(position_sequence: torch.Tensor, noise_std_last_step: float,
                             seed: Optional[int] = None, offset: int = 0):
    """(noise, noisy window) from one HIP pass (sgnn_random_walk_noise): the
    distribution of noise_utils.py:4-39 on a Philox stream; `seed` defaults to
    a draw from torch's CPU generator, so torch.manual_seed fixes it."""
    from ._hip import check, lib, require_gpu_tensor, stream_ptr
    pos = position_sequence
    require_gpu_tensor(pos, "position_sequence")
    if pos.dtype != torch.float32 or not pos.is_contiguous():
        pos = pos.to(torch.float32).contiguous()
    n, T, d = pos.shape
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    noise, noisy = torch.empty_like(pos), torch.empty_like(pos)
    check(lib().sgnn_random_walk_noise(pos.data_ptr(), n, T, d, float(noise_std_last_step),
                                       seed & (2 ** 64 - 1), offset & (2 ** 64 - 1), noise.data_ptr(),
                                       noisy.data_ptr(), stream_ptr(pos.device)), "sgnn_random_walk_noise")
    return noise, noisy


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
        on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        # gloo (CPU tests, or several ranks sharing one GPU) reduces host tensors: device buffers are
        # staged through host memory; nccl (= RCCL on ROCm) reduces them in place over xGMI
        self.host_staging = on and dist.get_backend(group) == "gloo"
        # test hook: the overlapped bucket path on a one-rank RCCL group (tests/test_gpu_dp.py: RCCL refuses
        # two ranks on one device, so the box's one GPU runs the collectives' stream logic at world size 1)
        self.force_overlap = False
        # test / trace hook: the deferred-count path (below) on a one-rank group (tools/dp_sync_trace.py)
        self.force_deferred = False
        self._count_src = {}

    def layout(self, n_local: int, device) -> Tuple[int, int]:
        """(N_global, offset): the particle count over all ranks (the mean
        denominator of train.py:268) and the index of this rank's first particle
        in the concatenated batch (ranks in order).  ONE all_gather, issued by
        every rank on every call, so ranks whose local counts differ or change
        from step to step can never pair it with a different collective."""
        if self.world == 1:
            return int(n_local), 0
        t = torch.tensor([int(n_local)], dtype=torch.int64, device="cpu" if self.host_staging else device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        counts = torch.cat(out).tolist()
        return int(sum(counts)), int(sum(counts[:self.rank]))

    def global_count(self, n_local: int, device) -> int:
        return self.layout(n_local, device)[0]

    # The counts of a step whose caller does not pass (n_global, particle_offset): no collective and no
    # host sync before the step's work is queued.  The backward then forms the gradient of this rank's
    # loss SUM (inv_count 1), the rank's particle count rides in the flat buffer's tail through the SAME
    # sum all-reduce(s) as the gradient (two float slots, hi * 2^20 + lo: exact for any count up to
    # 2^44 over up to 16 ranks), and the reduced gradient and loss sums are divided by the reduced count
    # on the device (the gradient is linear in the loss scale, so this is the reference's mean over the
    # concatenated batch, train.py:268, up to fp32 rounding of where the 1/N is applied).  The noise
    # stream offset is the rank's own 2^40-particle slice (disjoint across ranks; pass particle_offset,
    # e.g. from split_batch's host-side counts as train() does, for the single-process stream).
    COUNT_HI, COUNT_LO = 6, 7            # slots of FlatParams.loss (the loss sums use 0..4)
    RANK_NOISE_STRIDE = 1 << 40

    def plan(self, n_local: int, n_global: Optional[int], particle_offset: Optional[int]):
        """(inv_count for the backward kernels, particle offset, deferred) of one step."""
        if self.world == 1 and not self.force_deferred:
            return 1.0 / (n_global or n_local), particle_offset or 0, False
        off = self.rank * self.RANK_NOISE_STRIDE if particle_offset is None else particle_offset
        if n_global is None:
            return 1.0, off, True
        return 1.0 / n_global, off, False

    def put_count(self, loss_tail: torch.Tensor, n_local: int) -> None:
        """This rank's particle count into the all-reduced tail (queued after the backward's writes)."""
        # a device-to-device copy from a per-count cached tensor: assigning Python floats to device
        # elements is a synchronous host-to-device copy, which waited ~0.8 ms for the backward to drain
        # (tools/dp_sync_trace.py, profiles/r06_dp_sync_trace.txt)
        key = (n_local, loss_tail.device)
        src = self._count_src.get(key)
        if src is None:
            src = torch.tensor([float(n_local >> 20), float(n_local & ((1 << 20) - 1))],
                               dtype=loss_tail.dtype).to(loss_tail.device)
            self._count_src[key] = src
        loss_tail[self.COUNT_HI:self.COUNT_LO + 1].copy_(src, non_blocking=True)

    def take_count(self, grad: torch.Tensor, loss_tail: torch.Tensor) -> torch.Tensor:
        """After the all-reduce: N_global as a device scalar; the gradient scaled by 1/N_global in place."""
        cnt = loss_tail[self.COUNT_HI].double() * float(1 << 20) + loss_tail[self.COUNT_LO].double()
        grad.mul_((1.0 / cnt).float())
        return cnt.float()

    def overlaps_buckets(self) -> bool:
        """Per-layer gradient buckets all-reduced on the side stream while the
        layers below run their backward (device collectives only: gloo stages
        device buffers through host memory, so it keeps the one collective)."""
        return OVERLAP_BUCKETS and (self.world > 1 or self.force_overlap) and not self.host_staging

    def allreduce_async(self, t: torch.Tensor, stream: torch.cuda.Stream):
        """SUM all-reduce of `t` ordered after the work queued on `stream`; the
        returned handle's wait() orders the caller's current stream after it."""
        with torch.cuda.stream(stream):
            return dist.all_reduce(t, group=self.group, async_op=True)

    def allreduce_(self, *tensors: torch.Tensor) -> None:
        """SUM all-reduce (RCCL over xGMI on MI355X; gloo in CPU tests)."""
        if self.world == 1 and not (self.force_overlap or self.force_deferred):
            return
        for t in tensors:
            if self.host_staging and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, group=self.group)


def split_batch(idx: Sequence[int], rank: int, world: int) -> Optional[List[int]]:
    """This rank's whole graphs of one global batch: a contiguous, balanced
    slice (rank r gets idx[s_r:s_{r+1}]), so the ranks' local batches
    concatenated in rank order ARE the reference's concatenated batch
    (collate, taylor_impact_data_loader.py:243-284).  None when the batch has
    fewer graphs than ranks (an epoch's short last batch): every rank sees the
    same idx, so every rank skips it together and no collective is left
    unmatched."""
    idx = list(idx)
    if len(idx) < world:
        return None
    q, r = divmod(len(idx), world)
    start = rank * q + min(rank, r)
    return idx[start:start + q + (1 if rank < r else 0)]


OVERLAP_BUCKETS = True   # DataParallel.overlaps_buckets


def layer_ranges(epd, flat: training.FlatParams) -> Tuple[List[Tuple[int, int]], Tuple[int, int]]:
    """[start, end) of every interaction layer's parameters in the flat
    gradient buffer (module.parameters() order keeps each layer contiguous),
    and the span [lo, hi) they cover together: the buckets of the overlapped
    all-reduce are the layers, then [0, lo) (embedding, encoder) and [hi, end)
    (decoder, loss sums)."""
    out = []
    for layer in epd._processor.gnn_stacks:
        offs = sorted(flat.offsets[id(p)] for p in layer.parameters())
        s, e = offs[0][0], offs[-1][0] + offs[-1][1]
        if e - s != sum(n for _, n in offs):
            raise RuntimeError("interaction layer parameters are not contiguous in the flat buffer")
        out.append((s, e))
    lo, hi = min(r[0] for r in out), max(r[1] for r in out)
    if hi - lo != sum(e - s for s, e in out):
        raise RuntimeError("interaction layers are not contiguous in the flat buffer")
    return out, (lo, hi)


def block_buckets(blocks, flat: training.FlatParams) -> Tuple[List[Tuple[int, int]], List[Tuple[int, int]]]:
    """The overlapped all-reduce's buckets for a chain of message-passing blocks: [start, end) of each
    block's parameters in the flat gradient buffer (each contiguous), and the intervals of the buffer
    no block covers (encoders, head, loss sums) -- reduced together after the backward."""
    out = []
    for blk in blocks:
        offs = sorted(flat.offsets[id(p)] for p in blk.parameters())
        s, e = offs[0][0], offs[-1][0] + offs[-1][1]
        if e - s != sum(n for _, n in offs):
            raise RuntimeError("block parameters are not contiguous in the flat buffer")
        out.append((s, e))
    rest, at = [], 0
    for s, e in sorted(out):
        if s > at:
            rest.append((at, s))
        at = max(at, e)
    if at < flat.comm.numel():
        rest.append((at, flat.comm.numel()))
    return out, rest


class Trainer:
    """Drop-in training loop body for a sgnn_amd.LearnedSimulator."""

    def __init__(self, simulator, lr_init: float = 1e-3, lr_decay: float = 0.1,
                 lr_decay_steps: int = 30000, noise_std: float = 0.02,
                 loss_weight_position: float = 1.0, loss_weight_strain: float = 1.0,
                 group=None, nslab: Optional[int] = None):
        self.sim = simulator
        self.epd = simulator._encode_process_decode
        # the fused kernels where they are built for the widths, else the width-generic autograd path
        self.fused = training.fused_trainable(self.epd, simulator._nparticle_types)
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
        self._buckets = None   # layer_ranges(...) of the overlapped all-reduce, computed once

    def workspace(self, n: int, T: int, device) -> training.TrainWorkspace:
        cap = training.capacity(n)
        key = (cap, T, str(device))
        tw = self._tw.get(key)
        if tw is None:
            if len(self._tw) > 4:
                self._tw.clear()
            tw = training.TrainWorkspace(self.epd, cap, T, self.sim._particle_dimensions,
                                         self.sim._max_num_neighbors, True, device, self.nslab)
            tw.loss_out = self.flat.loss   # loss sums land in the gradient buffer's tail
            self._tw[key] = tw
        return tw.activate(n)

    def train_step(self, position: torch.Tensor, next_position: torch.Tensor,
                   next_strain: torch.Tensor, nparticles_per_example, particle_types=None,
                   noise: Optional[torch.Tensor] = None, n_global: Optional[int] = None,
                   particle_offset: Optional[int] = None, timers: Optional[dict] = None) -> dict:
        """One optimisation step on this rank's graphs; returns device-side loss
        terms.  `noise` defaults to fresh random-walk noise.

        Data parallel (world > 1): `n_global` is the particle count of the whole
        global batch and `particle_offset` the index of this rank's first
        particle in it.  A caller that knows the global batch (train() does)
        passes both; otherwise one all_gather per step computes them (every rank
        issues it every step: no rank-local caching that could desync the
        collectives).  The noise stream is counted by global particle index, so
        ranks draw disjoint slices of the one-process noise."""
        pos = position.to(torch.float32).contiguous()
        n = pos.shape[0]
        # no collective / host sync here: see DataParallel.plan (deferred: the count rides in the all-reduce)
        inv_count, particle_offset, deferred = self.dp.plan(n, n_global, particle_offset)
        if noise is None:       # fused: draw + cumsum twice + noisy window in one kernel
            # the seed is a draw from torch's CPU generator: the same on every
            # rank (it also drives the shared shuffle); the offset separates them
            noise, noisy = device_random_walk_noise(pos, self.noise_std, offset=particle_offset)
        else:
            noise = noise.to(pos.device, torch.float32).contiguous()
            noisy = (pos + noise).contiguous()                      # learned_simulator.py:467
        if not self.fused:
            return self._generic_step(pos, noise, next_position, next_strain, nparticles_per_example,
                                      particle_types, inv_count, deferred)
        inp, _ = self.sim._step_inputs(noisy, nparticles_per_example, particle_types)
        n, T, _ = noisy.shape
        tw = self.workspace(n, T, pos.device)
        radius = self.sim._connectivity_radius
        emb = self.sim._particle_type_embedding.weight if self.sim._nparticle_types > 1 else None
        training.train_forward(self.epd, radius, inp, tw, timers=timers, emb_weight=emb)
        works, layer_done = [], None
        if self.dp.overlaps_buckets():
            if self._buckets is None:
                self._buckets = layer_ranges(self.epd, self.flat)
            ranges, (lo, hi) = self._buckets

            def layer_done(k, stream):   # layer k's gradients are final once its slab reduction ran
                works.append(self.dp.allreduce_async(self.flat.comm[ranges[k][0]:ranges[k][1]], stream))
        training.train_backward(self.epd, radius, inp, tw, self.grads, timers=timers,
                                next_pos=next_position.to(torch.float32).contiguous(), noise=noise,
                                next_strain=next_strain.to(torch.float32).contiguous(),
                                w_pos=self.w_pos, w_strain=self.w_strain, inv_count=inv_count,
                                emb_weight=emb, emb_grad=self.grads.get("_particle_type_embedding.weight"),
                                layer_done=layer_done)
        if deferred:
            self.dp.put_count(self.flat.loss, n)
        if layer_done is None:
            self.dp.allreduce_(self.flat.comm)   # gradient + loss sums: one collective
        else:
            # the layers' buckets went out during the backward; embedding / encoder and decoder / loss
            # sums after the final slab reduction, then the launch stream waits for all of them
            self.dp.allreduce_(self.flat.comm[:lo], self.flat.comm[hi:])
            for w in works:
                w.wait()
        count = self.dp.take_count(self.flat.grad, self.flat.loss) if deferred else 1.0 / inv_count
        self.opt.step()
        return self._finish(count)

    def _finish(self, n_global) -> dict:
        """`n_global`: an int, or (deferred counts) the all-reduced count as a device scalar."""
        # train.py:276-278: LR for the NEXT step, computed from the pre-increment step
        self.opt.lr = self.lr_init * (self.lr_decay ** (self.step / self.lr_decay_steps)) + 1e-6
        self.step += 1
        if not torch.is_tensor(n_global):
            n_global = int(round(n_global))
        lo = self.flat.loss[:5] / n_global     # one kernel; the terms are views of it
        return {"loss": lo[0], "loss_position": lo[1:4].sum(), "loss_strain": lo[4],
                "loss_xyz": lo[1:4], "n_global": n_global, "lr": self.opt.lr}

    def _generic_step(self, pos, noise, next_position, next_strain, nparticles_per_example, particle_types,
                      inv_count: float, deferred: bool) -> dict:
        """The step at shapes the fused kernels are not built for (autograd_step)."""
        count = autograd_step(self, lambda: self.sim.predict_accelerations(
            next_position.to(pos.device, torch.float32), noise, pos, nparticles_per_example, particle_types),
            next_strain.to(pos.device, torch.float32), inv_count, pos.shape[0] if deferred else None)
        return self._finish(count)


def autograd_step(trainer, predict, next_strain: torch.Tensor, inv_count: float, deferred_n: Optional[int] = None):
    """One optimisation step on the differentiable width-generic path (HIP forward
    and backward, sgnn_amd.autograd): `predict()` = predict_accelerations, the
    reference's loss (train.py:257-268 / multi_scale_train.py:160-176) as this
    rank's sums times inv_count = 1/N_global, backward into the flat gradient views,
    the loss sums into the buffer's tail, one all-reduce of both, the fused Adam.
    deferred_n (DataParallel.plan): inv_count is 1 and this rank's count rides in the
    all-reduce; the gradient is scaled by the reduced count after it.  Returns N_global
    (an int, or the reduced count as a device scalar)."""
    flat = trainer.flat
    flat.comm.zero_()
    with torch.enable_grad():
        pa, ta, ps = predict()
        sq = (pa - ta) ** 2
        ls = (ps - next_strain) ** 2
        per = trainer.w_pos * sq.sum(-1) + trainer.w_strain * ls
        (per.sum() * inv_count).backward()   # AccumulateGrad adds into the flat gradient views
    with torch.no_grad():
        d = sq.shape[1]
        flat.loss[0] = per.sum()
        flat.loss[1:1 + d] = sq.sum(0)
        flat.loss[4] = ls.sum()
        if deferred_n is not None:
            trainer.dp.put_count(flat.loss, deferred_n)
    trainer.dp.allreduce_(flat.comm)
    count = trainer.dp.take_count(flat.grad, flat.loss) if deferred_n is not None else 1.0 / inv_count
    trainer.opt.step()
    return count


# ---------------------------------------------------------------------------
# Harness around the step (train.py:29-491): config, simulator factory, the
# training loop with validation-gated best-model checkpoints, resume, and
# rollout prediction with the reference's output files.
def load_config(config_path: str) -> dict:
    """train.py:29-45 (yaml.safe_load)."""
    import yaml
    from pathlib import Path
    p = Path(config_path)
    if not p.exists():
        raise FileNotFoundError(f"Config file not found: {config_path}")
    with open(p) as f:
        return yaml.safe_load(f)


def _get_simulator(metadata: dict, acc_noise_std: float, vel_noise_std: float, device, config: dict):
    """train.py:431-491: stats sigma = sqrt(sigma_meta^2 + noise^2); nnode_in =
    (T-1)*dim + 1 (+ embedding size when there is more than one particle type);
    nmlp_layers = 1."""
    from .learned_simulator import LearnedSimulator
    f = lambda k: torch.tensor(metadata[k], dtype=torch.float32)
    stats = {"acceleration": {"mean": f("acc_mean").to(device),
                              "std": torch.sqrt(f("acc_std") ** 2 + acc_noise_std ** 2).to(device)},
             "velocity": {"mean": f("vel_mean").to(device),
                          "std": torch.sqrt(f("vel_std") ** 2 + vel_noise_std ** 2).to(device)}}
    ntypes = metadata.get("num_particle_types", 1)
    dim = config["dim"]
    nnode_in = (config["input_sequence_length"] - 1) * dim + 1
    if ntypes > 1:
        nnode_in += config["particle_type_embedding_size"]
    return LearnedSimulator(particle_dimensions=dim, nnode_in=nnode_in, nedge_in=dim + 1,
                            latent_dim=config["hidden_dim"], nmessage_passing_steps=config["layers"],
                            nmlp_layers=1, mlp_hidden_dim=config["hidden_dim"],
                            connectivity_radius=config["connection_radius"], normalization_stats=stats,
                            nparticle_types=ntypes,
                            particle_type_embedding_size=config["particle_type_embedding_size"],
                            device=device)


def rollout_split(simulator, metadata: dict, device, config: dict, split: str):
    """Rollouts over every trajectory of `split` (train.py:84-135 / :318-349).
    Yields (index, example_output) with example_output['metadata'] set."""
    import os
    from . import data, evaluate
    loader = data.get_data_loader_by_trajectories(os.path.join(config["data_path"], f"{split}.npz"))
    nsteps = metadata["sequence_length"] - config["input_sequence_length"]
    for i, traj in enumerate(loader):
        out = evaluate.rollout(simulator, traj["positions"].to(device), traj["particle_type"].to(device),
                               traj["n_particles_per_example"].to(device), traj["strains"].to(device),
                               nsteps, config["dim"], device, config["input_sequence_length"],
                               config.get("inference_mode", "autoregressive"))
        out["metadata"] = metadata
        yield i, out


def rollout_losses(out: dict) -> dict:
    """train.py:110-114."""
    rp, rs = out["rmse_position"], out["rmse_strain"]
    return {"loss_total": float(rp[-1] + rs[-1]), "loss_position": float(rp[-1]),
            "loss_strain": float(rs[-1]), "loss_oneStep": float(rp[0] + rs[0])}


def predict(simulator, metadata: dict, device, config: dict) -> list:
    """train.py:53-166: load the model, roll out `test` (mode 'rollout') or
    `valid`, and in rollout mode write `<output_path>/<run_name>/<case>.pkl`
    (the rollout dict + 'metadata' + 'case_name', evaluate.py:161-173)."""
    import os
    import pickle
    from pathlib import Path
    model_path = Path(config["model_path"]) / config["run_name"] / config["model_file"]
    simulator.load(str(model_path))
    simulator.to(device)
    simulator.eval()
    split = "test" if config["mode"] == "rollout" else "valid"
    losses = []
    for i, out in rollout_split(simulator, metadata, device, config, split):
        losses.append(rollout_losses(out)["loss_total"])
        if config["mode"] == "rollout":
            case = metadata["file_test"][i].replace(".npz", "")
            out["case_name"] = case
            save_dir = Path(config["output_path"]) / config["run_name"]
            save_dir.mkdir(parents=True, exist_ok=True)
            with open(save_dir / f"{case}.pkl", "wb") as f:
                pickle.dump(out, f)
    return losses


def train(simulator, metadata: dict, device, config: dict, group=None, log_every: int = 10,
          generator: Optional[torch.Generator] = None) -> dict:
    """train.py:185-428 on the HIP step.

    Batches come from the split resident in device memory (data.DeviceSamples:
    the reference DataLoader's samples and order, sliced on the device).  With
    a process group of W ranks every global batch of `batch_size` windows is
    split into contiguous, balanced slices over the ranks (`split_batch`: whole
    graphs per rank, rank order = the concatenated batch's order, one all-reduce
    of gradient + loss sums per step) so the update equals the single-process
    one.
    Validation every `nsave_steps` keeps only improving checkpoints
    (model-best-<step>.pt + train_state-best-<step>.pt); without any
    validation the final state is saved as model-final-<step>.pt.  Resumes from
    config['model_file'] / config['train_state_file'] when model_file is set."""
    import os
    from pathlib import Path
    from . import checkpoint_utils, data
    rank = dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    simulator.to(device)
    trainer = Trainer(simulator, lr_init=config["lr_init"], lr_decay=config["lr_decay"],
                      lr_decay_steps=config["lr_decay_steps"], noise_std=config["noise_std"],
                      loss_weight_position=config.get("loss_weight_position", 1.0),
                      loss_weight_strain=config.get("loss_weight_strain", 1.0), group=group)
    if config.get("model_file"):
        model_dir = os.path.join(config["model_path"], config["run_name"]) + "/"
        checkpoint_utils.load_model(simulator, model_dir, config["model_file"], config["train_state_file"],
                                    device, trainer=trainer)
    samples = data.DeviceSamples(
        data.TaylorImpactSamplesDataset(os.path.join(config["data_path"], "train.npz"),
                                        config["input_sequence_length"]), device)
    save_dir = Path(config["model_path"]) / config["run_name"]
    lowest = float("inf")
    history = []
    nsteps = config["ntraining_steps"]
    while trainer.step < nsteps:
        for idx in samples.index_batches(config["batch_size"], shuffle=True, generator=generator):
            mine = split_batch(idx, rank, world)    # this rank's whole graphs of the global batch
            if mine is None:
                continue                            # short last batch: skipped by every rank alike
            batch = samples.batch(mine)
            inp, outp = batch["input"], batch["output"]
            out = trainer.train_step(inp["positions"], outp["next_position"], outp["next_strain"],
                                     inp["n_particles_per_example"].tolist(), inp["particle_type"],
                                     n_global=samples.count(idx),
                                     particle_offset=samples.count(idx[:idx.index(mine[0])]))
            step = trainer.step
            if step % log_every == 0:
                history.append((step, float(out["loss"])))
                if rank == 0:
                    print(f"Step {step}: Total Loss = {history[-1][1]:.6f}")
            if config.get("nsave_steps") and step % config["nsave_steps"] == 0:
                simulator.eval()
                losses = [rollout_losses(o)["loss_total"]
                          for _, o in rollout_split(simulator, metadata, device, config, "valid")]
                simulator.train()
                mean = float(sum(losses) / len(losses))
                if mean < lowest:
                    lowest = mean
                    if rank == 0:
                        save_dir.mkdir(parents=True, exist_ok=True)
                        simulator.save(str(save_dir / f"model-best-{step:06}.pt"))
                        checkpoint_utils.save_train_state(str(save_dir / f"train_state-best-{step:06}.pt"),
                                                          trainer.opt.state_dict(), step,
                                                          lowest_eval_loss=lowest)
            if step >= nsteps:
                break
    if lowest == float("inf") and rank == 0:
        save_dir.mkdir(parents=True, exist_ok=True)
        simulator.save(str(save_dir / f"model-final-{trainer.step:06}.pt"))
        checkpoint_utils.save_train_state(str(save_dir / f"train_state-final-{trainer.step:06}.pt"),
                                          trainer.opt.state_dict(), trainer.step)
    return {"step": trainer.step, "lowest_eval_loss": lowest, "history": history, "trainer": trainer}
