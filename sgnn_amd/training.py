"""Training step on the HIP kernels: saved-activation forward, fused backward,
slab reduction into a flat gradient buffer, RCCL all-reduce, fused Adam.

Mirrors the reference training step (sgnn/single_scale/train.py:231-280):
noise -> LearnedSimulator.predict_accelerations (learned_simulator.py:440-491)
-> loss (train.py:257-268) -> backward -> Adam -> exponential LR decay.
Whole-graph data parallelism: each rank owns whole
graphs; the reference's mean over all particles of the concatenated batch is
reproduced by scaling every rank's loss gradient by 1/N_global, so the SUM
all-reduce of the flat gradient equals the single-process gradient.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _hip, engine
from ._hip import SgnnReduceDesc, SgnnSaves, check, lib, stream_ptr

DEFAULT_NSLAB = 512  # persistent edge-backward workgroups: two per CU (k_edge_bwd64 sizes its LDS for that)
WIDE_NSLAB = 256     # the other single-scale variants (H = 64 with nmlp_layers 2, H = 128): larger LDS,
                     # one workgroup per CU, so 512 would run in two rounds
MS_NSLAB = 256      # multi-scale (H = 128 items / weight-gradient kernels, one workgroup per CU)
NODE_NSLAB = 256     # node-level backward kernels (128 measured slower: fewer CUs busy)


class FlatParams:
    """Point every parameter of `module` into one flat fp32 buffer, and its
    `.grad` into one flat gradient buffer (+ the step's loss sums in its tail):
    one RCCL all-reduce, one Adam launch."""

    def __init__(self, module: nn.Module):
        params = list(module.parameters())
        dev = params[0].device
        total = sum(p.numel() for p in params)
        self.param = torch.empty(total, dtype=torch.float32, device=dev)
        # the flat gradient and an 8-float tail for the loss sums (the decoder's slab reduction writes
        # them there): one buffer, so a data-parallel step is ONE all-reduce
        self.comm = torch.zeros(total + 8, dtype=torch.float32, device=dev)
        self.grad = self.comm[:total]
        self.loss = self.comm[total:]
        self.offsets: Dict[int, Tuple[int, int]] = {}
        self.order = []   # (offset, numel, shape) in parameters() order
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.param[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.param[off:off + n].view_as(p)
                p.grad = self.grad[off:off + n].view_as(p)
                self.offsets[id(p)] = (off, n)
                self.order.append((off, n, tuple(p.shape)))
                off += n
        self.numel = total


W_PARTIALS = 4  # per-wave partial rows of every slab vector (kWaves in epd_bwd.hip)


def _lin(prefix: str, nl: int, has_ln: bool):
    """Parameter names of one reference MLP (graph_network.py:7-45 build_mlp,
    optionally wrapped Sequential(mlp, LayerNorm)): (first, middle, last, ln)."""
    mp = prefix + ("0." if has_ln else "")
    first = mp + "NN-0."
    mid = mp + "NN-1." if nl == 3 else None
    last = mp + f"NN-{nl - 1}."
    ln = prefix + "1." if has_ln else None
    return first, mid, last, ln


class GradLayout:
    """Slab -> parameter-gradient reduction table (include/sgnn.h slab layouts),
    uploaded once per (slab arena, gradient buffers)."""

    def __init__(self, H: int, nl: int, feat: int, dim: int, arena: torch.Tensor,
                 slab_off: Dict[tuple, int], slab_floats: Dict[int, int], nslab_of: Dict[int, int]):
        self.H, self.nl, self.feat, self.dim = H, nl, feat, dim
        self.arena, self.slab_off, self.slab_floats, self.nslab_of = arena, slab_off, slab_floats, nslab_of
        self.descs: List[SgnnReduceDesc] = []

    def add(self, kind, k, offset, dst, nrows, ncols, src_ld, dst_ld=None, nrep=1, rep_stride=0,
            scale=1.0, dst_off=0):
        d = SgnnReduceDesc()
        d.src = self.arena.data_ptr() + 4 * self.slab_off[(kind, k)]
        d.dst = dst.data_ptr() + 4 * dst_off
        d.slab_stride = self.slab_floats[kind]
        d.offset = offset
        d.rep_stride = rep_stride
        d.nslab, d.nrep, d.src_ld = self.nslab_of[kind], nrep, src_ld
        d.nrows, d.ncols = nrows, ncols
        d.dst_ld = dst_ld if dst_ld is not None else ncols
        d.accumulate = 0
        d.scale = scale
        self.descs.append(d)

    def vec(self, kind, k, off, dst, n=None, width=None):
        """A [W][width] per-wave partial vector -> dst[:n]."""
        H = self.H
        width = width or H
        self.add(kind, k, off, dst, 1, n or width, width, nrep=W_PARTIALS, rep_stride=width)

    def nmat(self, kind: int) -> int:
        H, nl = self.H, self.nl
        mid = H * H if nl == 3 else 0
        fpad = 32 * ((self.feat + 31) // 32)
        return {_hip.SLAB_EDGE: 2 * H * H + mid, _hip.SLAB_NODE: 3 * H * H + mid,
                _hip.SLAB_UV: 2 * H * H, _hip.SLAB_DECODER: 32 * H + H * H + mid,
                _hip.SLAB_ENC_NODE: H * H + H * fpad + mid,
                _hip.SLAB_ENC_EDGE: H * H + H * 32 + mid}[kind]

    # -- one reference MLP per call -------------------------------------------------
    def enc_node(self, g, prefix, emb_g: Optional[torch.Tensor] = None):
        """emb_g: [32][H] destination of the per-type dh sums (embeddings)."""
        H, nl, W = self.H, self.nl, W_PARTIALS
        K = _hip.SLAB_ENC_NODE
        fpad = 32 * ((self.feat + 31) // 32)
        first, mid, last, ln = _lin(prefix, nl, True)
        vb = self.nmat(K)
        self.add(K, 0, H * H, g(first + "weight"), H, self.feat, fpad)
        self.add(K, 0, 0, g(last + "weight"), H, H, H)
        if mid:
            self.add(K, 0, H * H + H * fpad, g(mid + "weight"), H, H, H)
        self._vecs5(K, 0, vb, g, first, last, ln, mid)
        if emb_g is not None:
            self.add(K, 0, vb + (5 if mid else 4) * W * H, emb_g, 32, H, H)

    def enc_edge(self, g, prefix, k=0):
        H, nl = self.H, self.nl
        K = _hip.SLAB_ENC_EDGE
        first, mid, last, ln = _lin(prefix, nl, True)
        vb = self.nmat(K)
        self.add(K, k, H * H, g(first + "weight"), H, self.dim + 1, 32)
        self.add(K, k, 0, g(last + "weight"), H, H, H)
        if mid:
            self.add(K, k, H * H + H * 32, g(mid + "weight"), H, H, H)
        self._vecs5(K, k, vb, g, first, last, ln, mid)

    def _vecs5(self, K, k, vb, g, first, last, ln, mid):
        H, W = self.H, W_PARTIALS
        self.vec(K, k, vb, g(first + "bias"))
        self.vec(K, k, vb + W * H, g(last + "bias"))
        self.vec(K, k, vb + 2 * W * H, g(ln + "weight"))
        self.vec(K, k, vb + 3 * W * H, g(ln + "bias"))
        if mid:
            self.vec(K, k, vb + 4 * W * H, g(mid + "bias"))

    def interaction(self, g, prefix, k, e_scale, slot=None):
        """edge_fn (EDGE + UV slabs of layer slot) and node_fn (NODE slab)."""
        H, nl, W = self.H, self.nl, W_PARTIALS
        slot = k if slot is None else slot
        first, mid, last, ln = _lin(prefix + "edge_fn.", nl, True)
        E, U, N = _hip.SLAB_EDGE, _hip.SLAB_UV, _hip.SLAB_NODE
        # edge MLP first Linear: [x_i | x_j] from UV, [e] from EDGE (x 2^k)
        self.add(U, slot, 0, g(first + "weight"), H, 2 * H, 2 * H, dst_ld=3 * H)
        self.add(E, slot, H * H, g(first + "weight"), H, H, H, dst_ld=3 * H, scale=float(e_scale),
                 dst_off=2 * H)
        self.vec(U, slot, 2 * H * H, g(first + "bias"))
        self.add(E, slot, 0, g(last + "weight"), H, H, H)
        vb = self.nmat(E)
        self.vec(E, slot, vb, g(last + "bias"))
        self.vec(E, slot, vb + W * H, g(ln + "weight"))
        self.vec(E, slot, vb + 2 * W * H, g(ln + "bias"))
        if mid:
            self.add(E, slot, 2 * H * H, g(mid + "weight"), H, H, H)
            self.vec(E, slot, vb + 3 * W * H, g(mid + "bias"))
        first, mid, last, ln = _lin(prefix + "node_fn.", nl, True)
        self.add(N, slot, H * H, g(first + "weight"), H, 2 * H, 2 * H)
        self.add(N, slot, 0, g(last + "weight"), H, H, H)
        if mid:
            self.add(N, slot, 3 * H * H, g(mid + "weight"), H, H, H)
        self._vecs5(N, slot, self.nmat(N), g, first, last, ln, mid)

    def decoder(self, g, prefix, loss_out):
        H, nl, W = self.H, self.nl, W_PARTIALS
        D = _hip.SLAB_DECODER
        first, mid, last, _ = _lin(prefix, nl, False)
        d1 = self.dim + 1
        vb = self.nmat(D)
        self.add(D, 0, 32 * H, g(first + "weight"), H, H, H)
        self.add(D, 0, 0, g(last + "weight"), d1, H, H)
        if mid:
            self.add(D, 0, 32 * H + H * H, g(mid + "weight"), H, H, H)
        self.vec(D, 0, vb, g(last + "bias"), n=d1, width=32)
        self.vec(D, 0, vb + W * 32, g(first + "bias"))
        self.vec(D, 0, vb + W * 32 + W * H, loss_out, n=5, width=8)
        if mid:
            self.vec(D, 0, vb + W * 32 + W * H + W * 8, g(mid + "bias"))

    def upload(self, device):
        descs = self.descs
        arr = (SgnnReduceDesc * len(descs))(*descs)
        raw = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))),
                               dtype=torch.uint8)
        starts, nb = [], 0
        for d in descs:
            starts.append(nb)
            nb += (d.nrows * d.ncols + 31) // 32
        return raw.to(device), torch.tensor(starts, dtype=torch.int32).to(device), len(descs), nb


class SlabArena:
    """One fp32 arena holding every backward kernel's per-workgroup partial slabs."""

    def __init__(self, H: int, nl: int, feat: int, keys: List[tuple], nslab_of: Dict[int, int],
                 device: torch.device):
        L = lib()
        self.slab_floats = {k: int(L.sgnn_bwd_slab_floats(k, H, feat, nl)) for k in range(6)}
        self.nslab_of = nslab_of
        self.slab_off: Dict[Tuple[int, int], int] = {}
        off = 0
        for key in keys:
            self.slab_off[key] = off
            off += nslab_of[key[0]] * self.slab_floats[key[0]]
        self.arena = torch.empty(max(off, 1), dtype=torch.float32, device=device)

    def ptr(self, kind: int, k: int = 0) -> int:
        return self.arena.data_ptr() + 4 * self.slab_off[(kind, k)]

    def layout(self, H, nl, feat, dim) -> GradLayout:
        return GradLayout(H, nl, feat, dim, self.arena, self.slab_off, self.slab_floats, self.nslab_of)


def default_nslab(H: int, nlin: int) -> int:
    """Persistent backward workgroups for this variant: two per CU only where the
    k_*_bwd64 kernels (H = 64, nmlp_layers 1) are dispatched."""
    return DEFAULT_NSLAB if (H == 64 and nlin == 2) else WIDE_NSLAB


def nslab_table(nslab: int) -> Dict[int, int]:
    node_ns = max(1, min(nslab, NODE_NSLAB))
    # the edge, uv and node backward (H = 64: 80 KB kernels, two workgroups per CU) take the full
    # count; the decoder / encoder-node backward with larger LDS run one workgroup per CU
    return {_hip.SLAB_EDGE: nslab, _hip.SLAB_ENC_EDGE: nslab, _hip.SLAB_NODE: nslab,
            _hip.SLAB_UV: nslab, _hip.SLAB_DECODER: node_ns, _hip.SLAB_ENC_NODE: node_ns}


def capacity(n: int) -> int:
    """Particle capacity of the workspace that serves a batch of n particles:
    n rounded up to 1/8-1/16 of its power of two (min 256), so batches of
    varying composition (concatenated graphs of different sizes) reuse a few
    workspaces instead of allocating one per distinct n."""
    if n <= 2048:
        return max(256, -(-n // 256) * 256)
    q = 1 << (n.bit_length() - 4)
    return -(-n // q) * q


class TrainWorkspace:
    """Forward saves + backward buffers + weight-gradient slabs for up to n
    particles (`activate(n)` selects the batch size within the capacity)."""

    def __init__(self, epd: nn.Module, n: int, T: int, dim: int, K: int, loop: bool,
                 device: torch.device, nslab: Optional[int] = None):
        L = lib()
        H, nl = epd.latent_dim, epd.nlayers
        self.nlin = epd.nmlp_layers + 1
        nslab = default_nslab(H, self.nlin) if nslab is None else nslab
        self.H, self.L, self.n, self.T, self.dim, self.nslab = H, nl, n, T, dim, nslab
        self.n_cap = n
        self.nslab_of = nslab_table(nslab)
        self.feat = epd.nnode_in
        self.f = engine.StepWorkspace(n, T, dim, H, K, loop, device)
        cap = self.f.edge_cap
        tl = int(L.sgnn_edge_latent_floats(cap, H))
        f32 = dict(dtype=torch.float32, device=device)
        e = lambda *s: torch.empty(*s, **f32)
        two = self.nlin == 3
        self.enc_h, self.enc_yh, self.enc_rstd = e(n, H), e(n, H), e(n)
        self.enc_h2 = e(n, H) if two else None
        self.ee_yh, self.ee_rstd = e(tl), e(cap)
        self.ee_h2 = e(tl) if two else None
        self.e_h = [e(tl) for _ in range(nl)]
        self.e_h2 = [e(tl) if two else None for _ in range(nl)]
        self.e_yh = [e(tl) for _ in range(nl)]
        self.e_rstd = [e(cap) for _ in range(nl)]
        self.n_agg = [e(n, H) for _ in range(nl)]
        self.n_h = [e(n, H) for _ in range(nl)]
        self.n_h2 = [e(n, H) if two else None for _ in range(nl)]
        self.n_yh = [e(n, H) for _ in range(nl)]
        self.n_rstd = [e(n) for _ in range(nl)]
        self.xs = [e(n, H) for _ in range(nl + 1)]
        self.hd = e(n, H)
        self.hd2 = e(n, H) if two else None
        self.pred = e(n, dim + 1)
        self.next_scratch = e(n, dim)
        self.g, self.dxp, self.dagg, self.du = e(n, H), e(n, H), e(n, H), e(n, H)
        # H = 64: one dh-rows buffer per layer, dE0 formed afterwards in one pass
        # (sgnn_edge_latent_grad); H = 128 accumulates dE0 inside the layers
        self.latent_pass = H == 64 and nl <= 9
        self.dh_layers = [e(cap, H) for _ in range(nl if self.latent_pass else 1)]
        self.dh_rows = self.dh_layers[0]
        self.de0t = e(tl)
        self._dh_ptrs = (ctypes.c_void_p * len(self.dh_layers))(*[t.data_ptr() for t in self.dh_layers])
        self._scales = (ctypes.c_float * nl)(*[float(2.0 ** k) for k in range(nl)])
        i32 = dict(dtype=torch.int32, device=device)
        self.tptr = torch.empty(n + 1, **i32)
        self.tperm = torch.empty(cap, **i32)
        self.tws = torch.empty(int(L.sgnn_transpose_workspace_bytes(n, cap)) + 256, dtype=torch.uint8,
                               device=device)
        keys = [(_hip.SLAB_DECODER, 0)] + [(_hip.SLAB_NODE, k) for k in range(nl)] + \
               [(_hip.SLAB_EDGE, k) for k in range(nl)] + [(_hip.SLAB_UV, k) for k in range(nl)] + \
               [(_hip.SLAB_ENC_NODE, 0), (_hip.SLAB_ENC_EDGE, 0)]
        self.slabs = SlabArena(H, self.nlin, self.feat, keys, self.nslab_of, device)
        self.arena = self.slabs.arena
        self.loss_out = torch.zeros(8, **f32)
        self.emb_g = torch.zeros(32, H, **f32)   # per-type dh sums (particle-type embeddings)
        sc = lambda kind, items: int(L.sgnn_bwd_scratch_floats(kind, H, items, self.nlin))
        self.scratch = e(max(1, sc(_hip.SLAB_EDGE, cap), sc(_hip.SLAB_ENC_EDGE, cap),
                             sc(_hip.SLAB_NODE, n), sc(_hip.SLAB_UV, n)))
        self._descs_key = None
        self._side = None

    def side(self, device: torch.device):
        """Second HIP stream for work off the critical path (the transpose CSR
        beside the forward layers, the encoder-node backward beside the edge-
        latent pass) and the events that order it against the launch stream."""
        if self._side is None:
            self._side = torch.cuda.Stream(device=device)
            self._ev = {k: torch.cuda.Event() for k in ("pos", "encn", "graph", "tcsr", "g", "enc")}
        return self._side, self._ev

    def activate(self, n: int) -> "TrainWorkspace":
        """Run the next step on n <= n_cap particles (every kernel reads the
        edge count from rowptr[n]; buffers are sized for the capacity)."""
        if not 0 < n <= self.n_cap:
            raise ValueError(f"batch of {n} particles does not fit a workspace of {self.n_cap}")
        self.n = self.f.n = n
        return self

    def slab(self, kind: int, k: int = 0) -> int:
        return self.slabs.ptr(kind, k)

    def tws_ptr(self) -> int:
        return (self.tws.data_ptr() + 255) & ~255

    def descriptors(self, epd: nn.Module, grads: Dict[str, torch.Tensor], use_emb: bool = False) -> None:
        """Build the slab -> parameter-gradient reduction table (device copy)."""
        key = tuple(g.data_ptr() for g in grads.values()) + (use_emb,)
        if key == self._descs_key:
            return
        pre = "_encode_process_decode."
        g = lambda name: grads[pre + name]
        dev = self.arena.device
        # one table per interaction layer (reduced on the side stream as soon
        # as that layer's backward is done) + one for the encoders / decoder
        self._reduce_layer = []
        for k in range(self.L):
            lay = self.slabs.layout(self.H, self.nlin, self.feat, self.dim)
            lay.interaction(g, f"_processor.gnn_stacks.{k}.", k, 2.0 ** k)
            self._reduce_layer.append(lay.upload(dev))
        lay = self.slabs.layout(self.H, self.nlin, self.feat, self.dim)
        lay.enc_node(g, "_encoder.node_fn.", self.emb_g if use_emb else None)
        lay.enc_edge(g, "_encoder.edge_fn.")
        lay.decoder(g, "_decoder.node_fn.", self.loss_out)
        self._descs_dev, self._block_start, self._ndesc, self._nblocks = lay.upload(dev)
        self._descs_key = key


def _saves(h=None, yhat=None, rstd=None, agg=None, hd=None, h2=None, hd2=None) -> SgnnSaves:
    p = engine._ptr
    return SgnnSaves(h=p(h), yhat=p(yhat), rstd=p(rstd), agg=p(agg), hd=p(hd), h2=p(h2), hd2=p(hd2))


def fused_trainable(epd: nn.Module, nparticle_types: int) -> bool:
    """The fused training kernels implement this model (hidden = latent in {64, 128},
    nmlp_layers 1 or 2, the encoder widths they tile, <= 256 particle types); every
    other shape trains on the differentiable width-generic path (sgnn_amd.autograd)."""
    from . import generic
    return generic.fast_shapes(epd) and nparticle_types <= MAX_TYPES


class _Timer:
    """Optional HIP-event timing of named launches on the current stream."""

    def __init__(self, timers: Optional[dict], name: str):
        self.timers, self.name = timers, name

    def __enter__(self):
        if self.timers is not None:
            self.ev0 = torch.cuda.Event(enable_timing=True)
            self.ev0.record()

    def __exit__(self, *exc):
        if self.timers is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self.timers.setdefault(self.name, []).append((self.ev0, ev1))


def emb_args(inp: engine.StepInputs, emb_weight: Optional[torch.Tensor]):
    """(types, emb_w, emb_dim, use_emb) for the encoder kernels."""
    if emb_weight is None or inp.types is None:
        return 0, 0, 0, 0
    return inp.types.data_ptr(), emb_weight.data_ptr(), int(emb_weight.shape[1]), 1


DW1E_IN_LAYER = False  # experiment switch (tools/exp_train_ablate.py): measured slower, see DESIGN §3
MAX_TYPES = 256   # particle types the training path differentiates (sgnn_encode_nodes_bwd_typed)


def typed_embedding(emb_weight: Optional[torch.Tensor], use_emb: bool) -> bool:
    """More than 32 particle types: the per-type sums G come from
    sgnn_encode_nodes_bwd_typed (dh rows + a deterministic type sum) instead of
    the encoder slab's one-hot G[32][H] block."""
    return use_emb and int(emb_weight.shape[0]) > 32


def encode_nodes_backward(tw, g: torch.Tensor, inp: engine.StepInputs, n: int, T: int, d: int,
                          emb_weight: Optional[torch.Tensor], wall_max: float, wall_div: float,
                          saves: SgnnSaves, enc: "ctypes.Structure", slab: int, nslab: int, stream: int) -> None:
    """Encoder node-MLP backward (+ the per-type sums for the embedding
    gradient): sgnn_encode_nodes_bwd, or its typed form past 32 types."""
    L = lib()
    ty, ew, ed, ue = emb_args(inp, emb_weight)
    if typed_embedding(emb_weight, bool(ue)):
        nt = int(emb_weight.shape[0])
        need = int(L.sgnn_type_sums_workspace_bytes(n, tw.H, nt))
        if getattr(tw, "type_ws", None) is None or tw.type_ws.numel() < need or tw.emb_gt.shape[0] != nt:
            tw.type_ws = torch.empty(need, dtype=torch.uint8, device=g.device)
            tw.emb_gt = torch.zeros(nt, tw.H, dtype=torch.float32, device=g.device)
        check(L.sgnn_encode_nodes_bwd_typed(g.data_ptr(), inp.pos_seq.data_ptr(), n, T, d, ty, ew, ed, nt,
                                            inp.vel_mean.data_ptr(), inp.vel_std.data_ptr(), float(wall_max),
                                            float(wall_div), ctypes.byref(saves), ctypes.byref(enc), slab, nslab,
                                            tw.emb_gt.data_ptr(), tw.type_ws.data_ptr(), stream),
              "sgnn_encode_nodes_bwd_typed")
        return
    check(L.sgnn_encode_nodes_bwd(g.data_ptr(), inp.pos_seq.data_ptr(), n, T, d, ty, ew, ed,
                                  int(emb_weight.shape[0]) if ue else 0, ue, inp.vel_mean.data_ptr(),
                                  inp.vel_std.data_ptr(), float(wall_max), float(wall_div), ctypes.byref(saves),
                                  ctypes.byref(enc), slab, nslab, stream), "sgnn_encode_nodes_bwd")


def embedding_backward(tw, enc_w1: torch.Tensor, emb_weight: torch.Tensor, demb: torch.Tensor,
                       nvel: int, stream: int) -> None:
    """dEmb = G . W1[:, emb columns] after the slab reduction filled tw.emb_g
    (or sgnn_encode_nodes_bwd_typed filled tw.emb_gt)."""
    G = tw.emb_gt if typed_embedding(emb_weight, True) else tw.emb_g
    check(lib().sgnn_embedding_grad(G.data_ptr(), int(emb_weight.shape[0]), tw.H, enc_w1.data_ptr(),
                                    int(enc_w1.shape[1]), nvel + 1, int(emb_weight.shape[1]),
                                    demb.data_ptr(), 0, stream), "sgnn_embedding_grad")


def train_forward(epd: nn.Module, radius: float, inp: engine.StepInputs, tw: TrainWorkspace,
                  timers: Optional[dict] = None, emb_weight: Optional[torch.Tensor] = None) -> None:
    """predict_accelerations' forward with every activation the backward needs saved."""
    L = lib()
    pk = engine.ParamPack.get(epd)
    ws = tw.f
    n, T, d = ws.n, ws.T, ws.dim
    s = stream_ptr(inp.pos_seq.device)
    pos = inp.pos_seq
    side, ev = tw.side(pos.device)
    main = torch.cuda.current_stream(pos.device)
    # the node encoder (and layer-0 u / v) needs only the positions: side
    # stream, beside the radius graph; the first edge layer waits for it
    ev["pos"].record(main)
    side.wait_event(ev["pos"])
    sv = _saves(h=tw.enc_h, yhat=tw.enc_yh, rstd=tw.enc_rstd, h2=tw.enc_h2)
    check(L.sgnn_encode_nodes(pos.data_ptr(), n, T, d, *emb_args(inp, emb_weight), inp.vel_mean.data_ptr(),
                              inp.vel_std.data_ptr(), float(radius), 1.0, ctypes.byref(pk.enc_node),
                              ctypes.byref(pk.edge[0]), tw.xs[0].data_ptr(), ws.u.data_ptr(),
                              ws.v.data_ptr(), ctypes.byref(sv), side.cuda_stream), "sgnn_encode_nodes")
    ev["encn"].record(side)
    engine.radius_graph(ws, pos, (T - 1) * d, T * d, inp.ex_ptr, inp.n_ex, radius)
    ev["graph"].record(main)
    # the edge encoder is queued on the launch stream before the side-stream
    # work below, so the GPU has it in hand while the host issues the rest
    sv = _saves(yhat=tw.ee_yh, rstd=tw.ee_rstd, h2=tw.ee_h2)
    check(L.sgnn_encode_edges(pos.data_ptr() + 4 * (T - 1) * d, T * d, d, float(radius),
                              ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n,
                              ws.edge_cap, ctypes.byref(pk.enc_edge), ws.e0t.data_ptr(),
                              ctypes.byref(sv), s), "sgnn_encode_edges")
    # x0, u, v of layer 0 come from the side stream.  The launch stream's wait is queued BEFORE the
    # transpose below goes to the side stream: queued after it, the first edge layer started only once the
    # transpose had finished (C2 trace, round 6: ~93 us idle on the launch stream)
    main.wait_event(ev["encn"])
    # sender-sorted transpose of the new graph (for dV) on the side stream,
    # overlapping the forward layers; train_backward waits for it
    side.wait_event(ev["graph"])
    check(L.sgnn_transpose_csr(ws.rowptr.data_ptr(), ws.send.data_ptr(), n, ws.edge_cap,
                               tw.tws_ptr(), tw.tptr.data_ptr(), tw.tperm.data_ptr(), side.cuda_stream),
          "sgnn_transpose_csr")
    ev["tcsr"].record(side)
    nl = len(pk.edge)
    for k in range(nl):
        sv = _saves(h=tw.e_h[k], yhat=tw.e_yh[k], rstd=tw.e_rstd[k], h2=tw.e_h2[k])
        with _Timer(timers, "k_edge_layer(train)"):
          check(L.sgnn_edge_layer(ws.u.data_ptr(), ws.v.data_ptr(), ws.e0t.data_ptr(), float(2.0 ** k),
                                ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n,
                                ws.edge_cap, ctypes.byref(pk.edge[k]), ws.agg.data_ptr(),
                                ws.cin.data_ptr(), ws.cout.data_ptr(), ctypes.byref(sv), s),
              "sgnn_edge_layer")
        if k < nl - 1:
            sv = _saves(h=tw.n_h[k], yhat=tw.n_yh[k], rstd=tw.n_rstd[k], agg=tw.n_agg[k], h2=tw.n_h2[k])
            check(L.sgnn_node_layer(tw.xs[k].data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                    ws.cout.data_ptr(), ws.rowptr.data_ptr(), n,
                                    ctypes.byref(pk.node[k]), ctypes.byref(pk.edge[k + 1]),
                                    tw.xs[k + 1].data_ptr(), ws.u.data_ptr(), ws.v.data_ptr(),
                                    ctypes.byref(sv), s), "sgnn_node_layer")
        else:
            sv = _saves(h=tw.n_h[k], yhat=tw.n_yh[k], rstd=tw.n_rstd[k], agg=tw.n_agg[k], hd=tw.hd,
                        h2=tw.n_h2[k], hd2=tw.hd2)
            check(L.sgnn_node_layer_decode(tw.xs[k].data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                           ws.cout.data_ptr(), ws.rowptr.data_ptr(), n,
                                           ctypes.byref(pk.node[k]), ctypes.byref(pk.dec),
                                           pos.data_ptr(), T, d, inp.acc_mean.data_ptr(),
                                           inp.acc_std.data_ptr(), tw.xs[k + 1].data_ptr(),
                                           tw.pred.data_ptr(), tw.next_scratch.data_ptr(), 0,
                                           ctypes.byref(sv), s), "sgnn_node_layer_decode")


def train_backward(epd: nn.Module, radius: float, inp: engine.StepInputs, tw: TrainWorkspace,
                   grads: Dict[str, torch.Tensor], dpred: Optional[torch.Tensor] = None,
                   next_pos: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                   next_strain: Optional[torch.Tensor] = None, w_pos: float = 1.0,
                   w_strain: float = 1.0, inv_count: float = 1.0, timers: Optional[dict] = None,
                   emb_weight: Optional[torch.Tensor] = None,
                   emb_grad: Optional[torch.Tensor] = None, layer_done=None) -> None:
    """Gradients of every parameter into `grads` (name -> tensor views);
    layer_done(k, side_stream), when given, is called as soon as layer k's
    slab reduction is queued on the side stream (its gradients are final
    there: the data-parallel trainer starts that layer's all-reduce);
    with emb_weight, the particle-type embedding gradient into emb_grad.
    With dpred: dL/dpred is given (autograd path); otherwise the loss of
    train.py:257-268 is differentiated in-kernel (its sums land in tw.loss_out)."""
    L = lib()
    pk = engine.ParamPack.get(epd)
    use_emb = emb_weight is not None and inp.types is not None
    tw.descriptors(epd, grads, use_emb and not typed_embedding(emb_weight, use_emb))
    ws = tw.f
    n, T, d = ws.n, ws.T, ws.dim
    s = stream_ptr(inp.pos_seq.device)
    ns = tw.nslab
    p = engine._ptr
    check(L.sgnn_decoder_loss_bwd(tw.pred.data_ptr(), inp.pos_seq.data_ptr(), p(next_pos), p(noise),
                                  p(next_strain), inp.acc_mean.data_ptr(), inp.acc_std.data_ptr(), n, T,
                                  d, float(w_pos), float(w_strain), float(inv_count), p(dpred),
                                  ctypes.byref(_saves(hd=tw.hd, hd2=tw.hd2)), tw.xs[tw.L].data_ptr(),
                                  ctypes.byref(pk.dec),
                                  tw.g.data_ptr(), tw.slab(_hip.SLAB_DECODER), tw.nslab_of[_hip.SLAB_DECODER], s),
          "sgnn_decoder_loss_bwd")
    side, ev = tw.side(inp.pos_seq.device)
    main = torch.cuda.current_stream(inp.pos_seq.device)
    main.wait_event(ev["tcsr"])          # tptr / tperm of this step's graph
    # H = 64, nmlp_layers 1: each layer's dW1e in its edge backward (k_edge_bwd64<true>) instead
    # of a k_edge_w1e_grad launch per layer on the side stream
    dw1e_in_layer = tw.latent_pass and tw.H == 64 and tw.nlin == 2 and DW1E_IN_LAYER
    for k in range(tw.L - 1, -1, -1):
        nsv = _saves(h=tw.n_h[k], yhat=tw.n_yh[k], rstd=tw.n_rstd[k], agg=tw.n_agg[k], h2=tw.n_h2[k])
        check(L.sgnn_node_layer_bwd(tw.g.data_ptr(), n, ctypes.byref(nsv), tw.xs[k].data_ptr(),
                                    ctypes.byref(pk.node[k]), tw.dagg.data_ptr(), tw.dxp.data_ptr(),
                                    tw.slab(_hip.SLAB_NODE, k), tw.nslab_of[_hip.SLAB_NODE],
                                    tw.scratch.data_ptr(), s),
              "sgnn_node_layer_bwd")
        with _Timer(timers, "k_edge_bwd"):
          esv = _saves(h=tw.e_h[k], yhat=tw.e_yh[k], rstd=tw.e_rstd[k], h2=tw.e_h2[k])
          dh_rows = tw.dh_layers[k] if tw.latent_pass else tw.dh_rows
          check(L.sgnn_edge_layer_bwd(tw.dagg.data_ptr(), ws.rowptr.data_ptr(), ws.send.data_ptr(),
                                    ws.recv.data_ptr(), n, ctypes.byref(esv), ws.e0t.data_ptr(), float(2.0 ** k),
                                    ctypes.byref(pk.edge[k]), tw.du.data_ptr(), ws.cin.data_ptr(),
                                    ws.cout.data_ptr(), dh_rows.data_ptr(),
                                    None if tw.latent_pass else tw.de0t.data_ptr(),
                                    (2 if dw1e_in_layer else int(k != tw.L - 1)), tw.slab(_hip.SLAB_EDGE, k),
                                    tw.nslab_of[_hip.SLAB_EDGE], tw.scratch.data_ptr(), ws.edge_cap, s),
              "sgnn_edge_layer_bwd")
        if tw.latent_pass and not dw1e_in_layer:
            # dW1e_k = sum_e dh_k e0^T needs only this layer's dh: side stream,
            # beside the node-level backward of the layers below
            ev["g"].record(main)
            side.wait_event(ev["g"])
            slab_k = (ctypes.c_void_p * 1)(tw.slab(_hip.SLAB_EDGE, k))
            check(L.sgnn_edge_latent_grad(ctypes.addressof(tw._dh_ptrs) + 8 * k,
                                          ctypes.addressof(pk.edge_arr) + ctypes.sizeof(_hip.SgnnMlp) * k,
                                          ctypes.addressof(tw._scales) + 4 * k, 1, ws.rowptr.data_ptr(), n,
                                          ws.edge_cap, ws.e0t.data_ptr(), None, slab_k,
                                          tw.nslab_of[_hip.SLAB_EDGE], side.cuda_stream),
                  "sgnn_edge_latent_grad")
        check(L.sgnn_uv_bwd(tw.dxp.data_ptr(), tw.du.data_ptr(), ws.cin.data_ptr(), ws.cout.data_ptr(),
                            ws.rowptr.data_ptr(), dh_rows.data_ptr(), tw.tptr.data_ptr(),
                            tw.tperm.data_ptr(), tw.xs[k].data_ptr(), n, ctypes.byref(pk.edge[k]),
                            tw.g.data_ptr(), tw.slab(_hip.SLAB_UV, k), tw.nslab_of[_hip.SLAB_UV],
                            tw.scratch.data_ptr(), s),
              "sgnn_uv_bwd")
        # layer k's slabs (NODE, EDGE + its dW1e on the side stream, UV) are
        # complete: sum them into the gradients on the side stream, beside the
        # layers below (HBM-bound, small LDS: it fits next to the main kernels)
        ev["g"].record(main)
        side.wait_event(ev["g"])
        dd, bs, nd, nb = tw._reduce_layer[k]
        check(L.sgnn_reduce_slabs(dd.data_ptr(), bs.data_ptr(), nd, nb, side.cuda_stream), "sgnn_reduce_slabs")
        if layer_done is not None:
            layer_done(k, side)
    # the encoder-node backward needs only g = dL/dx_0: side stream, beside
    # the edge-latent pass and the edge-encoder backward
    ev["g"].record(main)
    side.wait_event(ev["g"])
    encode_nodes_backward(tw, tw.g, inp, n, T, d, emb_weight, radius, 1.0,
                          _saves(h=tw.enc_h, yhat=tw.enc_yh, rstd=tw.enc_rstd, h2=tw.enc_h2), pk.enc_node,
                          tw.slab(_hip.SLAB_ENC_NODE), tw.nslab_of[_hip.SLAB_ENC_NODE], side.cuda_stream)
    ev["enc"].record(side)
    if tw.latent_pass:   # dE0 = sum_k 2^k W1e_k^T dh_k (the dW1e halves ran per layer)
        check(L.sgnn_edge_latent_grad(tw._dh_ptrs, ctypes.byref(pk.edge_arr), tw._scales, tw.L,
                                      ws.rowptr.data_ptr(), n, ws.edge_cap, ws.e0t.data_ptr(),
                                      tw.de0t.data_ptr(), None, tw.nslab_of[_hip.SLAB_EDGE], s),
              "sgnn_edge_latent_grad")
    check(L.sgnn_encode_edges_bwd(tw.de0t.data_ptr(), inp.pos_seq.data_ptr() + 4 * (T - 1) * d, T * d,
                                  d, float(radius), ws.rowptr.data_ptr(), ws.send.data_ptr(),
                                  ws.recv.data_ptr(), n,
                                  ctypes.byref(_saves(yhat=tw.ee_yh, rstd=tw.ee_rstd, h2=tw.ee_h2)),
                                  ctypes.byref(pk.enc_edge), tw.slab(_hip.SLAB_ENC_EDGE),
                                  tw.nslab_of[_hip.SLAB_ENC_EDGE], tw.scratch.data_ptr(), ws.edge_cap, s),
          "sgnn_encode_edges_bwd")
    main.wait_event(ev["enc"])
    check(L.sgnn_reduce_slabs(tw._descs_dev.data_ptr(), tw._block_start.data_ptr(), tw._ndesc,
                              tw._nblocks, s), "sgnn_reduce_slabs")
    if use_emb:
        embedding_backward(tw, epd._encoder.node_fn[0][0].weight, emb_weight, emb_grad, (T - 1) * d, s)


class Adam:
    """torch.optim.Adam(lr) semantics (train.py:199) on a FlatParams buffer, one
    fused kernel per step; `lr` may be changed between steps (train.py:276-278)."""

    def __init__(self, flat: FlatParams, lr: float, betas=(0.9, 0.999), eps: float = 1e-8):
        self.flat = flat
        self.lr, self.betas, self.eps = lr, betas, eps
        self.exp_avg = torch.zeros_like(flat.param)
        self.exp_avg_sq = torch.zeros_like(flat.param)
        self.step_count = 0

    def state_dict(self) -> dict:
        """torch.optim.Adam.state_dict() layout (per-parameter exp_avg /
        exp_avg_sq / step, parameters numbered in module.parameters() order), so
        the reference's train_state files and these are interchangeable."""
        f = self.flat
        group = dict(torch.optim.Adam([torch.zeros(1)], lr=self.lr, betas=self.betas,
                                      eps=self.eps).state_dict()["param_groups"][0])
        group["params"] = list(range(len(f.order)))
        state = {}
        if self.step_count > 0:
            for i, (off, n, shape) in enumerate(f.order):
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": self.exp_avg[off:off + n].view(shape).detach().clone(),
                            "exp_avg_sq": self.exp_avg_sq[off:off + n].view(shape).detach().clone()}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd: dict) -> None:
        f = self.flat
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(f.order):
            raise ValueError(f"optimizer state has {sum(len(g['params']) for g in groups)} parameters "
                             f"in {len(groups)} groups; this model has {len(f.order)} in one")
        g = groups[0]
        self.lr, self.betas, self.eps = float(g["lr"]), tuple(g["betas"]), float(g["eps"])
        steps = set()
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for slot, pid in enumerate(g["params"]):
                st = sd["state"].get(pid)
                if st is None:
                    continue
                off, n, shape = f.order[slot]
                if tuple(st["exp_avg"].shape) != tuple(shape):
                    raise ValueError(f"optimizer state {pid}: shape {tuple(st['exp_avg'].shape)} != {tuple(shape)}")
                self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"parameters at different Adam steps {sorted(steps)}: one fused update cannot resume them")
        self.step_count = steps.pop() if steps else 0

    def step(self) -> None:
        self.step_count += 1
        f = self.flat
        check(lib().sgnn_adam_step(f.param.data_ptr(), f.grad.data_ptr(), self.exp_avg.data_ptr(),
                                   self.exp_avg_sq.data_ptr(), f.numel, float(self.lr),
                                   float(self.betas[0]), float(self.betas[1]), float(self.eps),
                                   self.step_count, stream_ptr(f.param.device)), "sgnn_adam_step")
