"""Multi-scale training step on the HIP kernels (multi_scale_train.py:140-186:
noise -> MultiScaleSimulator.predict_accelerations -> loss -> backward ->
Adam -> LR decay), whole-graph data parallel over RCCL like the
single-scale Trainer (sgnn_amd/train.py).

Backward order (reverse of ms_engine.forward_step):
  prediction head + loss        -> g = dL/dx_{B}
  block b = B-1 .. 0 (M2G, M2M L-1 .. 0, G2M):
     node_bwd(b) -> dagg, dx' ; edge_bwd(b) -> dU, dh rows, dE0[kind] ;
     uv_bwd(b) -> g = dL/dx_b
     slab reduction of block b on the side stream (+ its all-reduce bucket under DP)
  grid encoder backward, three edge-encoder backwards (one per edge type)
  slab reduction of the encoders / head -> flat gradient
The edge latent of M2M block k is 2^k e0_m2m, so dE0_m2m accumulates
2^k W1e^T dh over the M2M blocks; g2m / m2g latents feed one block each.
Sender-sorted transposes of the three static graphs are built once.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from .. import _hip, engine
from .._hip import check, lib, stream_ptr
from ..train import DataParallel, block_buckets, device_random_walk_noise
from ..training import (MAX_TYPES, MS_NSLAB, Adam, FlatParams, SlabArena, _saves, _Timer, emb_args,
                        embedding_backward, encode_nodes_backward, nslab_table, typed_embedding)
from . import ms_engine
from .ms_engine import EDGE_TYPES

KIND_SLOT = {"g2m": 0, "m2m": 1, "m2g": 2}


def fused_trainable(sim) -> bool:
    """The fused multi-scale training kernels implement this model (latent =
    nedge_out in {64, 128}, nmlp_layers 1 or 2, the encoder widths they tile,
    <= 256 particle types); every other shape trains on the differentiable
    width-generic path (sgnn_amd.autograd)."""
    from .. import generic
    return generic.ms_fast_shapes(sim._multi_scale_gnn) and sim._nparticle_types <= MAX_TYPES


class MSTrainWorkspace:
    """Saved activations, backward buffers and slabs for one (n, T, static graph)."""

    def __init__(self, gnn, n: int, T: int, dim: int, graphs: Dict[str, engine.CsrGraph],
                 device: torch.device, nslab: int = MS_NSLAB):
        L = lib()
        H = gnn.latent_dim
        self.H, self.n, self.T, self.dim = H, n, T, dim
        self.nlin = gnn.nmlp_layers + 1
        self.nb = len(gnn.chain())
        self.kinds = ["g2m"] + ["m2m"] * (self.nb - 2) + ["m2g"]
        self.scales = [1.0] + [float(2.0 ** k) for k in range(self.nb - 2)] + [1.0]
        self.graphs = graphs
        self.f = ms_engine.MSWorkspace(n, T, dim, H, graphs, device)
        f32 = dict(dtype=torch.float32, device=device)
        e = lambda *s: torch.empty(*s, **f32)
        two = self.nlin == 3
        tl = {k: int(L.sgnn_edge_latent_floats(g.edge_cap, H)) for k, g in graphs.items()}
        cap = {k: g.edge_cap for k, g in graphs.items()}
        self.enc_h, self.enc_yh, self.enc_rstd = e(n, H), e(n, H), e(n)
        self.enc_h2 = e(n, H) if two else None
        self.ee_yh = {k: e(tl[k]) for k in EDGE_TYPES}
        self.ee_rstd = {k: e(cap[k]) for k in EDGE_TYPES}
        self.ee_h2 = {k: (e(tl[k]) if two else None) for k in EDGE_TYPES}
        kb = self.kinds
        self.e_h = [e(tl[kb[b]]) for b in range(self.nb)]
        # hidden 128, nmlp 2: the edge backward forms h2 and yhat again from h (bit-identical to the
        # forward's), so the blocks keep one [E][H] activation instead of three
        rc = H == 128 and two
        self.e_h2 = [e(tl[kb[b]]) if two and not rc else None for b in range(self.nb)]
        self.e_yh = [None if rc else e(tl[kb[b]]) for b in range(self.nb)]
        self.e_rstd = [e(cap[kb[b]]) for b in range(self.nb)]
        self.n_agg = [e(n, H) for _ in range(self.nb)]
        self.n_h = [e(n, H) for _ in range(self.nb)]
        self.n_h2 = [e(n, H) if two else None for _ in range(self.nb)]
        self.n_yh = [e(n, H) for _ in range(self.nb)]
        self.n_rstd = [e(n) for _ in range(self.nb)]
        self.xs = [e(n, H) for _ in range(self.nb + 1)]
        self.hd = e(n, H)
        self.hd2 = e(n, H) if two else None
        self.pred = e(n, dim + 1)
        self.next_scratch = e(n, dim)
        self.g, self.dxp, self.dagg, self.du = e(n, H), e(n, H), e(n, H), e(n, H)
        self.dh_rows = e(max(cap.values()), H)
        self.de0t = {k: e(tl[k]) for k in EDGE_TYPES}
        # sender-sorted transposes of the static graphs (for dV), built once
        i32 = dict(dtype=torch.int32, device=device)
        self.tptr, self.tperm = {}, {}
        s = stream_ptr(device)
        for k, g in graphs.items():
            self.tptr[k] = torch.empty(n + 1, **i32)
            self.tperm[k] = torch.empty(g.edge_cap, **i32)
            tws = torch.empty(int(L.sgnn_transpose_workspace_bytes(n, g.edge_cap)) + 256,
                              dtype=torch.uint8, device=device)
            check(L.sgnn_transpose_csr(g.rowptr.data_ptr(), g.send.data_ptr(), n, g.edge_cap,
                                       (tws.data_ptr() + 255) & ~255, self.tptr[k].data_ptr(),
                                       self.tperm[k].data_ptr(), s), "sgnn_transpose_csr")
        self.nslab_of = nslab_table(nslab)
        keys = [(_hip.SLAB_DECODER, 0)] + [(_hip.SLAB_NODE, b) for b in range(self.nb)] + \
               [(_hip.SLAB_EDGE, b) for b in range(self.nb)] + [(_hip.SLAB_UV, b) for b in range(self.nb)] + \
               [(_hip.SLAB_ENC_NODE, 0)] + [(_hip.SLAB_ENC_EDGE, KIND_SLOT[k]) for k in EDGE_TYPES]
        self.feat = gnn.nnode_in
        self.slabs = SlabArena(H, self.nlin, self.feat, keys, self.nslab_of, device)
        self.loss_out = torch.zeros(8, **f32)
        self.emb_g = torch.zeros(32, H, **f32)
        sc = lambda kind, items: int(L.sgnn_bwd_scratch_floats(kind, H, items, self.nlin))
        self.scratch = e(max(1, sc(_hip.SLAB_EDGE, max(cap.values())), sc(_hip.SLAB_ENC_EDGE, max(cap.values())),
                             sc(_hip.SLAB_NODE, n), sc(_hip.SLAB_UV, n)))
        self._descs_key = None

    def slab(self, kind: int, k: int = 0) -> int:
        return self.slabs.ptr(kind, k)

    def descriptors(self, grads: Dict[str, torch.Tensor], use_emb: bool = False) -> None:
        key = tuple(g.data_ptr() for g in grads.values()) + (use_emb,)
        if key == self._descs_key:
            return
        pre = "_multi_scale_gnn."
        g = lambda name: grads[pre + name]
        lay = self.slabs.layout(self.H, self.nlin, self.feat, self.dim)
        lay.enc_node(g, "grid_node_encoder.", self.emb_g if use_emb else None)
        for k in EDGE_TYPES:
            lay.enc_edge(g, f"{k}_edge_encoder.", KIND_SLOT[k])
        lay.decoder(g, "prediction_head.", self.loss_out)
        dev = self.slabs.arena.device
        self._descs_dev, self._block_start, self._ndesc, self._nblocks = lay.upload(dev)
        # one table per block, reduced on the side stream as soon as that block's backward is done
        prefixes = ["g2m_block."] + [f"m2m_blocks.{k}." for k in range(self.nb - 2)] + ["m2g_block."]
        self._reduce_block = []
        for b, p in enumerate(prefixes):
            lb = self.slabs.layout(self.H, self.nlin, self.feat, self.dim)
            lb.interaction(g, p, b, self.scales[b], slot=b)
            self._reduce_block.append(lb.upload(dev))
        self._descs_key = key

    def side(self, device: torch.device):
        """The side stream of the per-block slab reductions (and their all-reduce buckets) + events."""
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=device)
            self._ev = {k: torch.cuda.Event() for k in ("g", "blocks")}
        return self._side, self._ev


def train_forward(gnn, inp: engine.StepInputs, tw: MSTrainWorkspace, grid_radius: float,
                  mesh_radius: float, timers: Optional[dict] = None,
                  emb_weight: Optional[torch.Tensor] = None) -> None:
    """ms_engine.forward_step with every activation the backward needs saved."""
    L = lib()
    pk = ms_engine.ParamPack.get(gnn)
    ws, graphs = tw.f, tw.graphs
    n, T, d = tw.n, tw.T, tw.dim
    s = stream_ptr(inp.pos_seq.device)
    pos = inp.pos_seq
    sv = _saves(h=tw.enc_h, yhat=tw.enc_yh, rstd=tw.enc_rstd, h2=tw.enc_h2)
    check(L.sgnn_encode_nodes(pos.data_ptr(), n, T, d, *emb_args(inp, emb_weight), inp.vel_mean.data_ptr(),
                              inp.vel_std.data_ptr(), float(grid_radius), float(grid_radius),
                              ctypes.byref(pk.enc), ctypes.byref(pk.edge[0]), tw.xs[0].data_ptr(),
                              ws.u.data_ptr(), ws.v.data_ptr(), ctypes.byref(sv), s), "sgnn_encode_nodes")
    radii = {"g2m": grid_radius, "m2m": mesh_radius, "m2g": grid_radius}
    for k in EDGE_TYPES:
        g = graphs[k]
        sv = _saves(yhat=tw.ee_yh[k], rstd=tw.ee_rstd[k], h2=tw.ee_h2[k])
        check(L.sgnn_encode_edges(pos.data_ptr() + 4 * (T - 1) * d, T * d, d, float(radii[k]),
                                  g.rowptr.data_ptr(), g.send.data_ptr(), g.recv.data_ptr(), n, g.edge_cap,
                                  ctypes.byref(pk.enc_edge[k]), ws.e0t[k].data_ptr(), ctypes.byref(sv), s),
              "sgnn_encode_edges")
    for b in range(tw.nb):
        kind = tw.kinds[b]
        g = graphs[kind]
        sv = _saves(h=tw.e_h[b], yhat=tw.e_yh[b], rstd=tw.e_rstd[b], h2=tw.e_h2[b])
        with _Timer(timers, "k_edge_layer(train)"):
            check(L.sgnn_edge_layer(ws.u.data_ptr(), ws.v.data_ptr(), ws.e0t[kind].data_ptr(), tw.scales[b],
                                    g.rowptr.data_ptr(), g.send.data_ptr(), g.recv.data_ptr(), n,
                                    g.edge_cap, ctypes.byref(pk.edge[b]), ws.agg.data_ptr(),
                                    ws.cin.data_ptr(), ws.cout.data_ptr(), ctypes.byref(sv), s),
                  "sgnn_edge_layer")
        if b < tw.nb - 1:
            sv = _saves(h=tw.n_h[b], yhat=tw.n_yh[b], rstd=tw.n_rstd[b], agg=tw.n_agg[b], h2=tw.n_h2[b])
            check(L.sgnn_node_layer(tw.xs[b].data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                    ws.cout.data_ptr(), g.rowptr.data_ptr(), n, ctypes.byref(pk.node[b]),
                                    ctypes.byref(pk.edge[b + 1]), tw.xs[b + 1].data_ptr(), ws.u.data_ptr(),
                                    ws.v.data_ptr(), ctypes.byref(sv), s), "sgnn_node_layer")
        else:
            sv = _saves(h=tw.n_h[b], yhat=tw.n_yh[b], rstd=tw.n_rstd[b], agg=tw.n_agg[b], hd=tw.hd,
                        h2=tw.n_h2[b], hd2=tw.hd2)
            check(L.sgnn_node_layer_decode(tw.xs[b].data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                           ws.cout.data_ptr(), g.rowptr.data_ptr(), n,
                                           ctypes.byref(pk.node[b]), ctypes.byref(pk.head), pos.data_ptr(),
                                           T, d, inp.acc_mean.data_ptr(), inp.acc_std.data_ptr(),
                                           tw.xs[b + 1].data_ptr(), tw.pred.data_ptr(),
                                           tw.next_scratch.data_ptr(), 0, ctypes.byref(sv), s),
                  "sgnn_node_layer_decode")


def train_backward(gnn, inp: engine.StepInputs, tw: MSTrainWorkspace, grads: Dict[str, torch.Tensor],
                   grid_radius: float, mesh_radius: float, dpred: Optional[torch.Tensor] = None,
                   next_pos: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                   next_strain: Optional[torch.Tensor] = None, w_pos: float = 1.0, w_strain: float = 1.0,
                   inv_count: float = 1.0, timers: Optional[dict] = None,
                   emb_weight: Optional[torch.Tensor] = None, emb_grad: Optional[torch.Tensor] = None,
                   block_done=None) -> None:
    """block_done(b, side_stream), when given, is called as soon as block b's slab reduction is queued
    on the side stream (its gradients are final there): the trainer's all-reduce bucket for it."""
    L = lib()
    pk = ms_engine.ParamPack.get(gnn)
    use_emb = emb_weight is not None and inp.types is not None
    tw.descriptors(grads, use_emb and not typed_embedding(emb_weight, use_emb))
    ws, graphs = tw.f, tw.graphs
    n, T, d = tw.n, tw.T, tw.dim
    s = stream_ptr(inp.pos_seq.device)
    p = engine._ptr
    ns = tw.nslab_of
    check(L.sgnn_decoder_loss_bwd(tw.pred.data_ptr(), inp.pos_seq.data_ptr(), p(next_pos), p(noise),
                                  p(next_strain), inp.acc_mean.data_ptr(), inp.acc_std.data_ptr(), n, T, d,
                                  float(w_pos), float(w_strain), float(inv_count), p(dpred),
                                  ctypes.byref(_saves(hd=tw.hd, hd2=tw.hd2)), tw.xs[tw.nb].data_ptr(),
                                  ctypes.byref(pk.head), tw.g.data_ptr(), tw.slab(_hip.SLAB_DECODER),
                                  ns[_hip.SLAB_DECODER], s), "sgnn_decoder_loss_bwd")
    side, ev = tw.side(inp.pos_seq.device)
    main = torch.cuda.current_stream(inp.pos_seq.device)
    seen = set()
    for b in range(tw.nb - 1, -1, -1):
        kind = tw.kinds[b]
        g = graphs[kind]
        nsv = _saves(h=tw.n_h[b], yhat=tw.n_yh[b], rstd=tw.n_rstd[b], agg=tw.n_agg[b], h2=tw.n_h2[b])
        check(L.sgnn_node_layer_bwd(tw.g.data_ptr(), n, ctypes.byref(nsv), tw.xs[b].data_ptr(),
                                    ctypes.byref(pk.node[b]), tw.dagg.data_ptr(), tw.dxp.data_ptr(),
                                    tw.slab(_hip.SLAB_NODE, b), ns[_hip.SLAB_NODE],
                                    tw.scratch.data_ptr(), s), "sgnn_node_layer_bwd")
        esv = _saves(h=tw.e_h[b], yhat=tw.e_yh[b], rstd=tw.e_rstd[b], h2=tw.e_h2[b])
        with _Timer(timers, "k_edge_bwd"):
            check(L.sgnn_edge_layer_bwd(tw.dagg.data_ptr(), g.rowptr.data_ptr(), g.send.data_ptr(),
                                        g.recv.data_ptr(), n, ctypes.byref(esv), ws.e0t[kind].data_ptr(),
                                        tw.scales[b], ctypes.byref(pk.edge[b]), tw.du.data_ptr(),
                                        ws.cin.data_ptr(), ws.cout.data_ptr(), tw.dh_rows.data_ptr(),
                                        tw.de0t[kind].data_ptr(), int(kind in seen),
                                        tw.slab(_hip.SLAB_EDGE, b), ns[_hip.SLAB_EDGE],
                                        tw.scratch.data_ptr(), g.edge_cap, s),
                  "sgnn_edge_layer_bwd")
        seen.add(kind)
        check(L.sgnn_uv_bwd(tw.dxp.data_ptr(), tw.du.data_ptr(), ws.cin.data_ptr(), ws.cout.data_ptr(),
                            g.rowptr.data_ptr(), tw.dh_rows.data_ptr(), tw.tptr[kind].data_ptr(),
                            tw.tperm[kind].data_ptr(), tw.xs[b].data_ptr(), n, ctypes.byref(pk.edge[b]),
                            tw.g.data_ptr(), tw.slab(_hip.SLAB_UV, b), ns[_hip.SLAB_UV],
                            tw.scratch.data_ptr(), s), "sgnn_uv_bwd")
        # block b's slabs (NODE, EDGE, UV) are complete: sum them into its gradients on the side
        # stream, beside the blocks below
        ev["g"].record(main)
        side.wait_event(ev["g"])
        dd, bs, nd, nbk = tw._reduce_block[b]
        check(L.sgnn_reduce_slabs(dd.data_ptr(), bs.data_ptr(), nd, nbk, side.cuda_stream), "sgnn_reduce_slabs")
        if block_done is not None:
            block_done(b, side)
    ev["blocks"].record(side)
    encode_nodes_backward(tw, tw.g, inp, n, T, d, emb_weight, grid_radius, grid_radius,
                          _saves(h=tw.enc_h, yhat=tw.enc_yh, rstd=tw.enc_rstd, h2=tw.enc_h2), pk.enc,
                          tw.slab(_hip.SLAB_ENC_NODE), ns[_hip.SLAB_ENC_NODE], s)
    radii = {"g2m": grid_radius, "m2m": mesh_radius, "m2g": grid_radius}
    for k in EDGE_TYPES:
        g = graphs[k]
        if g.num_edges == 0:
            continue
        check(L.sgnn_encode_edges_bwd(tw.de0t[k].data_ptr(), inp.pos_seq.data_ptr() + 4 * (T - 1) * d, T * d,
                                      d, float(radii[k]), g.rowptr.data_ptr(), g.send.data_ptr(),
                                      g.recv.data_ptr(), n,
                                      ctypes.byref(_saves(yhat=tw.ee_yh[k], rstd=tw.ee_rstd[k], h2=tw.ee_h2[k])),
                                      ctypes.byref(pk.enc_edge[k]), tw.slab(_hip.SLAB_ENC_EDGE, KIND_SLOT[k]),
                                      ns[_hip.SLAB_ENC_EDGE], tw.scratch.data_ptr(), g.edge_cap, s),
                  "sgnn_encode_edges_bwd")
    check(L.sgnn_reduce_slabs(tw._descs_dev.data_ptr(), tw._block_start.data_ptr(), tw._ndesc,
                              tw._nblocks, s), "sgnn_reduce_slabs")
    if use_emb:
        embedding_backward(tw, gnn.grid_node_encoder[0][0].weight, emb_weight, emb_grad, (T - 1) * d, s)
    main.wait_event(ev["blocks"])   # Adam (and the next step's slabs) after the blocks' reductions


class MultiScaleTrainer:
    """Drop-in body of the multi_scale_train.py:140-186 loop for a sgnn_amd
    MultiScaleSimulator (static graph set with set_static_graph)."""

    def __init__(self, simulator, lr_init: float = 1e-3, lr_decay: float = 0.1,
                 lr_decay_steps: int = 15000, noise_std: float = 0.02,
                 loss_weight_position: float = 1.0, loss_weight_strain: float = 1.0,
                 group=None, nslab: int = MS_NSLAB):
        self.fused = fused_trainable(simulator)
        self.sim = simulator
        self.gnn = simulator._multi_scale_gnn
        self.flat = FlatParams(simulator)
        self.opt = Adam(self.flat, lr_init)
        self.grads = {k: p.grad for k, p in simulator.named_parameters()}
        self.lr_init, self.lr_decay, self.lr_decay_steps = lr_init, lr_decay, lr_decay_steps
        self.noise_std = noise_std
        self.w_pos, self.w_strain = loss_weight_position, loss_weight_strain
        self.dp = DataParallel(group)
        self.nslab = nslab
        self.step = 0
        self._tw: Dict[tuple, MSTrainWorkspace] = {}
        self._buckets = None   # block_buckets(...) of the overlapped all-reduce, computed once

    def workspace(self, n: int, T: int, device) -> MSTrainWorkspace:
        graphs = self.sim._csr(n, device)
        key = (n, T, str(device), id(graphs))
        tw = self._tw.get(key)
        if tw is None:
            if len(self._tw) > 2:
                self._tw.clear()
            tw = MSTrainWorkspace(self.gnn, n, T, self.sim._kinematic_dimensions, graphs, device, self.nslab)
            tw.loss_out = self.flat.loss   # loss sums land in the gradient buffer's tail
            self._tw[key] = tw
        return tw

    def train_step(self, position: torch.Tensor, next_position: torch.Tensor, next_strain: torch.Tensor,
                   particle_types=None, noise: Optional[torch.Tensor] = None,
                   n_global: Optional[int] = None, particle_offset: Optional[int] = None,
                   timers: Optional[dict] = None) -> dict:
        """One step on this rank's graph.  DP bookkeeping as Trainer.train_step:
        (n_global, particle_offset) from the caller or from one all_gather every
        step; the default noise (fused Philox kernel) is counted by global
        particle index, so every rank draws its own slice."""
        pos = position.to(torch.float32).contiguous()
        n = pos.shape[0]
        # no collective / host sync here: train.DataParallel.plan (deferred: the count rides in the all-reduce)
        inv_count, particle_offset, deferred = self.dp.plan(n, n_global, particle_offset)
        if noise is None:
            noise, noisy = device_random_walk_noise(pos, self.noise_std, offset=particle_offset)
        else:
            noise = noise.to(pos.device, torch.float32).contiguous()
            noisy = (pos + noise).contiguous()
        if not self.fused:   # differentiable width-generic path (e.g. nedge_out != latent_dim)
            from ..train import autograd_step
            count = autograd_step(self, lambda: self.sim.predict_accelerations(
                next_position.to(pos.device, torch.float32), noise, pos, None, particle_types),
                next_strain.to(pos.device, torch.float32), inv_count, n if deferred else None)
            return self._finish(self.flat.loss, count)
        inp, _ = self.sim._step_inputs(noisy, particle_types)
        n, T, _ = noisy.shape
        tw = self.workspace(n, T, pos.device)
        rg, rm = self.sim._grid_radius(), self.sim._mesh_radius()
        emb = self.sim._particle_type_embedding.weight if self.sim._nparticle_types > 1 else None
        train_forward(self.gnn, inp, tw, rg, rm, timers=timers, emb_weight=emb)
        works, block_done = [], None
        if self.dp.overlaps_buckets():   # per-block buckets, all-reduced during the backward (train.Trainer)
            if self._buckets is None:
                self._buckets = block_buckets(self.gnn.chain(), self.flat)
            ranges, _ = self._buckets

            def block_done(b, stream):
                works.append(self.dp.allreduce_async(self.flat.comm[ranges[b][0]:ranges[b][1]], stream))
        train_backward(self.gnn, inp, tw, self.grads, rg, rm, next_pos=next_position.to(torch.float32).contiguous(),
                       noise=noise, next_strain=next_strain.to(torch.float32).contiguous(), w_pos=self.w_pos,
                       w_strain=self.w_strain, inv_count=inv_count, timers=timers, emb_weight=emb,
                       emb_grad=self.grads.get("_particle_type_embedding.weight"), block_done=block_done)
        if deferred:
            self.dp.put_count(self.flat.loss, n)
        if block_done is None:
            self.dp.allreduce_(self.flat.comm)   # gradient + loss sums: one collective
        else:   # encoders, head and loss sums after the final reduction; then wait for the blocks' buckets
            self.dp.allreduce_(*[self.flat.comm[a:b] for a, b in self._buckets[1]])
            for w in works:
                w.wait()
        count = self.dp.take_count(self.flat.grad, self.flat.loss) if deferred else 1.0 / inv_count
        self.opt.step()
        return self._finish(tw.loss_out, count)

    def _finish(self, lo: torch.Tensor, n_global) -> dict:
        """`n_global`: an int, or (deferred counts) the all-reduced count as a device scalar."""
        self.opt.lr = self.lr_init * (self.lr_decay ** (self.step / self.lr_decay_steps)) + 1e-6
        self.step += 1
        if not torch.is_tensor(n_global):
            n_global = int(round(n_global))
        return {"loss": lo[0] / n_global, "loss_position": (lo[1] + lo[2] + lo[3]) / n_global,
                "loss_strain": lo[4] / n_global, "loss_xyz": lo[1:4] / n_global,
                "n_global": n_global, "lr": self.opt.lr}
