"""One message-passing block under autograd on the fused training kernels.

InteractionNetwork.forward(x, edge_index, e) (graph_network.py:150-222) and the
G2M / M2M / M2G blocks (multi_scale_gnn.py:84-205, the same math) at the widths
the fused kernels are built for (node / edge latent = MLP hidden = 64 or 128,
nmlp_layers 1 or 2): the forward is the training forward of one layer
(sgnn_edge_layer + sgnn_node_layer with every activation the backward needs
saved), the backward the training step's per-layer chain for that layer

  sgnn_node_layer_bwd  -> dagg, dx'            (node MLP, LayerNorm, residual)
  sgnn_edge_layer_bwd  -> dU, dh rows (, dE0)  (edge MLP, LayerNorm, receiver sums)
  sgnn_edge_latent_grad (H = 64)               -> dE0, dW1e
  sgnn_uv_bwd          -> dx                   (x_i / x_j halves of the first edge Linear)
  sgnn_reduce_slabs    -> every parameter gradient (fixed summation order)

instead of the width-generic GEMM chain (autograd.py).  The block's explicit
edge latent e (COO rows) goes into the kernels' tiled layout through the COO ->
CSR permutation and its gradient comes back the same way; the returned latent
is e + e (update hands back its input edge features, :176 / :222), so
dL/de = dE0 + 2 dL/d(2e).  Deterministic like the training step (no float
atomics)."""
from __future__ import annotations

import ctypes
from typing import Dict, List

import torch
import torch.nn as nn

from . import _hip, engine, training
from ._hip import check, lib, stream_ptr


class FusedGraph:
    """The kernels' view of one edge_index: the stable receiver CSR with the COO
    permutation, and its sender-sorted transpose (for dV), built once per graph."""

    def __init__(self, edge_index: torch.Tensor, n: int):
        self.g = engine.coo_to_csr(edge_index, n, with_perm=True)
        L = lib()
        dev = edge_index.device
        cap = self.g.edge_cap
        self.tptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        self.tperm = torch.empty(cap, dtype=torch.int32, device=dev)
        ws = torch.empty(int(L.sgnn_transpose_workspace_bytes(n, cap)) + 256, dtype=torch.uint8, device=dev)
        check(L.sgnn_transpose_csr(self.g.rowptr.data_ptr(), self.g.send.data_ptr(), n, cap, (ws.data_ptr() + 255) & ~255,
                                   self.tptr.data_ptr(), self.tperm.data_ptr(), stream_ptr(dev)), "sgnn_transpose_csr")
        self._ws = ws   # kept until the queued transpose has run


def _dense(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.float32).contiguous()


def applies(block: nn.Module, x: torch.Tensor, e: torch.Tensor, num_edges: int) -> bool:
    """The fused kernels implement this block and these inputs."""
    from .generic import block_fast_shapes
    if num_edges == 0 or not block_fast_shapes(block):
        return False
    H = engine.mlp_struct(block.edge_fn, True).hidden
    return (x.is_cuda and e.is_cuda and x.dim() == 2 and e.dim() == 2 and x.shape[1] == H and e.shape[1] == H
            and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in block.parameters()))


def block_backward(ctx, dx_out, de_out):
    """The per-layer backward chain of the training step for this block (module
    docstring); returns (dx, de, parameter gradients in named_parameters order)."""
    L = lib()
    g, fg = ctx.fg.g, ctx.fg
    x, e0t = ctx.saved_tensors[:2]
    sv = ctx.sv
    H, nlin, n, E = ctx.H, ctx.nlin, g.n, g.num_edges
    cap = g.edge_cap
    dev = x.device
    s = stream_ptr(dev)
    f32 = dict(dtype=torch.float32, device=dev)
    edge_fn, node_fn = ctx.edge_fn, ctx.node_fn
    gx = _dense(dx_out) if dx_out is not None else torch.zeros(n, H, **f32)
    nslab_of = training.nslab_table(training.default_nslab(H, nlin))
    keys = [(_hip.SLAB_NODE, 0), (_hip.SLAB_EDGE, 0), (_hip.SLAB_UV, 0)]
    arena = training.SlabArena(H, nlin, 0, keys, nslab_of, dev)
    sc = lambda kind, items: int(L.sgnn_bwd_scratch_floats(kind, H, items, nlin))
    scratch = torch.empty(max(1, sc(_hip.SLAB_EDGE, cap), sc(_hip.SLAB_NODE, n), sc(_hip.SLAB_UV, n)), **f32)
    dagg, dxp, du, dx = (torch.empty(n, H, **f32) for _ in range(4))
    check(L.sgnn_node_layer_bwd(gx.data_ptr(), n, ctypes.byref(sv["node"]), x.data_ptr(), ctypes.byref(node_fn),
                                dagg.data_ptr(), dxp.data_ptr(), arena.ptr(_hip.SLAB_NODE),
                                nslab_of[_hip.SLAB_NODE], scratch.data_ptr(), s), "sgnn_node_layer_bwd")
    cin, cout = torch.empty(g.ntiles, H, **f32), torch.empty(g.ntiles, H, **f32)
    dh = torch.empty(cap, H, **f32)
    de0t = torch.empty(int(L.sgnn_edge_latent_floats(cap, H)), **f32)
    latent_pass = H == 64   # as the training step: dE0 / dW1e after the layer at H = 64, inside it at 128
    check(L.sgnn_edge_layer_bwd(dagg.data_ptr(), g.rowptr.data_ptr(), g.send.data_ptr(), g.recv.data_ptr(), n,
                                ctypes.byref(sv["edge"]), e0t.data_ptr(), 1.0, ctypes.byref(edge_fn), du.data_ptr(),
                                cin.data_ptr(), cout.data_ptr(), dh.data_ptr(), None if latent_pass else de0t.data_ptr(),
                                0, arena.ptr(_hip.SLAB_EDGE), nslab_of[_hip.SLAB_EDGE], scratch.data_ptr(), cap, s),
          "sgnn_edge_layer_bwd")
    if latent_pass:
        dh_ptrs = (ctypes.c_void_p * 1)(dh.data_ptr())
        fns = (_hip.SgnnMlp * 1)(edge_fn)
        scales = (ctypes.c_float * 1)(1.0)
        slabs = (ctypes.c_void_p * 1)(arena.ptr(_hip.SLAB_EDGE))
        check(L.sgnn_edge_latent_grad(dh_ptrs, fns, scales, 1, g.rowptr.data_ptr(), n, cap, e0t.data_ptr(),
                                      de0t.data_ptr(), slabs, nslab_of[_hip.SLAB_EDGE], s), "sgnn_edge_latent_grad")
    check(L.sgnn_uv_bwd(dxp.data_ptr(), du.data_ptr(), cin.data_ptr(), cout.data_ptr(), g.rowptr.data_ptr(),
                        dh.data_ptr(), fg.tptr.data_ptr(), fg.tperm.data_ptr(), x.data_ptr(), n, ctypes.byref(edge_fn),
                        dx.data_ptr(), arena.ptr(_hip.SLAB_UV), nslab_of[_hip.SLAB_UV], scratch.data_ptr(), s),
          "sgnn_uv_bwd")
    grads: Dict[str, torch.Tensor] = {nm: torch.empty(shape, **f32) for nm, shape in ctx.pshapes}
    lay = arena.layout(H, nlin, 0, 0)
    lay.interaction(lambda nm: grads[nm], "", 0, 1.0)
    dd, bs, nd, nb = lay.upload(dev)
    check(L.sgnn_reduce_slabs(dd.data_ptr(), bs.data_ptr(), nd, nb, s), "sgnn_reduce_slabs")
    de = torch.empty(E, H, **f32)
    acc = 0
    if de_out is not None:   # the returned latent is e + e
        from .autograd import gather_into
        gather_into(de, 0, _dense(de_out), None, 2.0)
        acc = 1
    check(L.sgnn_edge_tiles_to_rows(de0t.data_ptr(), H, g.perm.data_ptr(), g.rowptr.data_ptr(), n, E, 1.0,
                                    de.data_ptr(), H, acc, s), "sgnn_edge_tiles_to_rows")
    return dx, de, [grads[nm] for nm, _ in ctx.pshapes]


class _FusedBlock(torch.autograd.Function):
    """(x', 2e) = block(x, edge_index, e) with the training kernels' forward and backward."""

    @staticmethod
    def forward(ctx, block, fg: FusedGraph, x, e, *params):
        L = lib()
        g = fg.g
        n, cap = g.n, g.edge_cap
        dev = x.device
        s = stream_ptr(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        x, e = _dense(x), _dense(e)
        edge_fn, node_fn = engine.mlp_struct(block.edge_fn, True), engine.mlp_struct(block.node_fn, True)
        H, nlin = edge_fn.hidden, edge_fn.nlin
        from .autograd import gather_into, gemm
        lin = [m for m in block.edge_fn.modules() if isinstance(m, nn.Linear)]
        w1, b1 = lin[0].weight, lin[0].bias
        u = gemm(x, w1[:, :H], tb=True, bias=b1)          # W1_i x + b1 (receiver half)
        v = gemm(x, w1[:, H:2 * H], tb=True)              # W1_j x (sender half)
        tl = int(L.sgnn_edge_latent_floats(cap, H))
        e0t = torch.empty(tl, **f32)
        check(L.sgnn_edge_rows_to_tiles(e.data_ptr(), H, H, g.perm.data_ptr(), g.rowptr.data_ptr(), n, cap,
                                        e0t.data_ptr(), s), "sgnn_edge_rows_to_tiles")
        two = nlin == 3
        keep: List[torch.Tensor] = []
        new = lambda *shape: keep.append(torch.empty(*shape, **f32)) or keep[-1]
        esv = training._saves(h=new(tl), yhat=new(tl), rstd=new(cap), h2=new(tl) if two else None)
        agg, cin, cout = new(n, H), new(g.ntiles, H), new(g.ntiles, H)
        check(L.sgnn_edge_layer(u.data_ptr(), v.data_ptr(), e0t.data_ptr(), 1.0, g.rowptr.data_ptr(),
                                g.send.data_ptr(), g.recv.data_ptr(), n, cap, ctypes.byref(edge_fn), agg.data_ptr(),
                                cin.data_ptr(), cout.data_ptr(), ctypes.byref(esv), s), "sgnn_edge_layer")
        nsv = training._saves(h=new(n, H), yhat=new(n, H), rstd=new(n), agg=new(n, H), h2=new(n, H) if two else None)
        x_out = torch.empty(n, H, **f32)
        # (the kernel also forms a next block's u / v: given this block's edge_fn, into scratch)
        check(L.sgnn_node_layer(x.data_ptr(), agg.data_ptr(), cin.data_ptr(), cout.data_ptr(), g.rowptr.data_ptr(), n,
                                ctypes.byref(node_fn), ctypes.byref(edge_fn), x_out.data_ptr(), u.data_ptr(),
                                v.data_ptr(), ctypes.byref(nsv), s), "sgnn_node_layer")
        e2 = torch.empty_like(e)
        gather_into(e2, 0, e, None, 2.0)   # e + e
        ctx.fg, ctx.H, ctx.nlin = fg, H, nlin
        ctx.edge_fn, ctx.node_fn = edge_fn, node_fn
        ctx.sv = {"edge": esv, "node": nsv}
        ctx.keep = keep                      # the saves the structs point into
        ctx.pshapes = [(nm, tuple(p.shape)) for nm, p in block.named_parameters()]
        ctx.save_for_backward(x, e0t, *params)
        return x_out, e2

    @staticmethod
    def backward(ctx, dx_out, de_out):
        dx, de, grads = block_backward(ctx, dx_out, de_out)
        return (None, None, dx, de, *grads)


def message_passing(block: nn.Module, x: torch.Tensor, fg: FusedGraph, e: torch.Tensor):
    """One block, differentiable, on the fused training kernels (see applies())."""
    if e.shape[0] != fg.g.num_edges:
        raise ValueError(f"{e.shape[0]} edge feature rows for {fg.g.num_edges} edges")
    return _FusedBlock.apply(block, fg, x, e, *block.parameters())
