"""Differentiable width-generic modules on the autograd.hip kernels.

The reference's modules are differentiable at any widths and depths (build_mlp
graph_network.py:7-45 with any `nmlp_layers`; `latent_dim` and `mlp_hidden_dim`
independent, learned_simulator.py:12-25; multi-scale `nedge_out` independent of
`latent_dim`, multi_scale_gnn.py:225-272).  Here every such module is a
composition of three torch.autograd.Functions whose forward AND backward run
in libsgnn_hip.so (include/sgnn.h, "Width-generic differentiable building
blocks"):

  MLP        build_mlp (+ LayerNorm) (+ residual): sgnn_gemm with the bias / ReLU
             epilogue per Linear, sgnn_layernorm; backward sgnn_layernorm_bwd,
             sgnn_colsum (dbias, dgamma, dbeta), sgnn_gemm (dW = dY^T A,
             dA = dY W), sgnn_relu_bwd
  GatherCat  cat([src_0[idx_0], src_1[idx_1], ...]) -- the message input
             cat([x_i, x_j, e]) (graph_network.py:197), cat([aggr, x]) (:220),
             2e (:176, the edge-latent doubling), the type embedding
             (learned_simulator.py:287-290); backward: column blocks, or CSR
             segment sums over the index (deterministic, no atomics)
  SegmentSum aggr='add' onto the receivers (:136) in the stable receiver-CSR
             order; backward: a row gather

Everything is deterministic.  The fused MFMA kernels (engine / training) stay
the fast path for the widths they are built for; this is the path for every
other shape and for the per-module forwards under autograd.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import engine
from ._hip import check, lib, require_gpu_tensor, stream_ptr


# ----------------------------------------------------------------------------- kernel wrappers
def _c(t: torch.Tensor) -> torch.Tensor:
    """fp32, row-major with unit column stride (a leading dimension is fine)."""
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t
    return t.contiguous()


def _dense(t: torch.Tensor) -> torch.Tensor:
    """fp32 and fully contiguous: for the kernels that index rows as r * width
    (sgnn_layernorm's residual, sgnn_layernorm_bwd's dout; ADVICE r04 -- torch.cat's
    backward hands each input a row-strided narrow() view)."""
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t.contiguous()


def gemm(a: torch.Tensor, b: torch.Tensor, ta: bool = False, tb: bool = False,
         bias: Optional[torch.Tensor] = None, relu: bool = False, out: Optional[torch.Tensor] = None,
         accumulate: bool = False) -> torch.Tensor:
    """op(a) @ op(b) (+ out) (+ bias) (ReLU) through sgnn_gemm; a / b as stored."""
    a, b = _c(a), _c(b)
    M, K = (a.shape[1], a.shape[0]) if ta else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if tb else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm: inner dimensions {K} != {Kb}")
    dev = a.device
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=dev)
    if M == 0 or N == 0:
        return out
    L = lib()
    nws = int(L.sgnn_gemm_workspace_bytes(M, N, K))
    ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=dev) if nws else None
    if bias is not None:
        bias = bias.to(torch.float32).contiguous()
    check(L.sgnn_gemm(int(ta), int(tb), M, N, K, a.data_ptr() if a.numel() else None, max(a.stride(0), 1),
                      b.data_ptr() if b.numel() else None, max(b.stride(0), 1),
                      bias.data_ptr() if bias is not None else None, int(relu), out.data_ptr(), out.stride(0),
                      int(accumulate), ws.data_ptr() if ws is not None else None, nws, stream_ptr(dev)), "sgnn_gemm")
    return out


def colsum(x: torch.Tensor, mul: Optional[torch.Tensor] = None) -> torch.Tensor:
    x = _c(x)
    n, w = x.shape
    dev = x.device
    out = torch.empty(w, dtype=torch.float32, device=dev)
    L = lib()
    nws = int(L.sgnn_colsum_workspace_bytes(n, w))
    ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=dev)
    if mul is not None:
        mul = _c(mul)
    check(L.sgnn_colsum(x.data_ptr() if n else None, x.stride(0), mul.data_ptr() if mul is not None else None,
                        mul.stride(0) if mul is not None else 0, n, w, out.data_ptr(), 0, ws.data_ptr(), nws,
                        stream_ptr(dev)), "sgnn_colsum")
    return out


def gather_into(out: torch.Tensor, col: int, src: torch.Tensor, index: Optional[torch.Tensor],
                scale: float = 1.0) -> None:
    """out[:, col:col + w] = scale * src[index] (or src)."""
    src = _c(src)
    n, w = out.shape[0], src.shape[1]
    check(lib().sgnn_gather_rows(src.data_ptr(), src.stride(0), w, index.data_ptr() if index is not None else None,
                                 n, float(scale), out.data_ptr() + 4 * col, out.stride(0),
                                 stream_ptr(out.device)), "sgnn_gather_rows")


def segment_sum_into(out: torch.Tensor, src: torch.Tensor, col: int, width: int, rowptr: torch.Tensor,
                     perm: Optional[torch.Tensor], scale: float = 1.0, accumulate: bool = False) -> None:
    """out[i] (+)= scale * sum_p src[perm[p], col:col + width] over p in [rowptr[i], rowptr[i+1])."""
    check(lib().sgnn_segment_sum_cols(src.data_ptr() + 4 * col, src.stride(0), width, rowptr.data_ptr(),
                                      perm.data_ptr() if perm is not None else None, out.shape[0], float(scale),
                                      out.data_ptr(), out.stride(0), int(accumulate), stream_ptr(out.device)),
          "sgnn_segment_sum_cols")


# ----------------------------------------------------------------------------- graphs
@dataclass
class Grouping:
    """Rows grouped by an index value (CSR over the values, stable): the backward
    of a gather src[index] sums the output rows of each value in this order."""
    rowptr: torch.Tensor
    perm: torch.Tensor
    n: int


def grouping(index: torch.Tensor, n: int) -> Grouping:
    """CSR of `index` (values in [0, n)) through sgnn_coo_to_csr (stable)."""
    idx = index.to(torch.int64).reshape(-1)
    # only the receiver side matters: perm maps each CSR position to its row of `index`
    g = engine.coo_to_csr(torch.stack([idx, idx]), n, with_perm=True)
    return Grouping(g.rowptr, g.perm, n)


class EdgeGraph:
    """One edge_index [2, E] (row 0 senders, row 1 receivers, PyG source_to_target)
    with the groupings its gathers and sums need: receivers (aggregation, dx_i)
    and senders (dx_j)."""

    def __init__(self, edge_index: torch.Tensor, n: int):
        require_gpu_tensor(edge_index, "edge_index")
        if edge_index.dim() != 2 or edge_index.shape[0] != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
        ei = edge_index.to(torch.int64)
        self.n, self.E = n, int(ei.shape[1])
        self.send = ei[0].to(torch.int32).contiguous()
        self.recv = ei[1].to(torch.int32).contiguous()
        self.by_recv = grouping(ei[1], n)   # also range-checks the indices (one host sync)
        self.by_send = grouping(ei[0], n)
        self._ei, self._fused = ei, None

    def fused(self):
        """The fused kernels' CSR (+ COO permutation, sender transpose) of this graph, built once."""
        if self._fused is None:
            from .fused_block import FusedGraph
            self._fused = FusedGraph(self._ei, self.n)
        return self._fused


_GRAPH_CACHE: List[Tuple[torch.Tensor, int, int, "EdgeGraph"]] = []


def cached_edge_graph(edge_index: torch.Tensor, n: int) -> EdgeGraph:
    """The EdgeGraph of this edge_index tensor, built once while the tensor is unchanged: a block
    called again on the same graph (each layer of a Processor / MultiScaleGNN called module by module)
    reuses its groupings and fused CSR instead of rebuilding them (each build syncs the host).  Keyed
    by tensor identity + its in-place version counter; the last few graphs are kept."""
    for t, ver, nn_, g in _GRAPH_CACHE:
        if t is edge_index and ver == edge_index._version and nn_ == n:
            return g
    g = EdgeGraph(edge_index, n)
    _GRAPH_CACHE.insert(0, (edge_index, edge_index._version, n, g))
    del _GRAPH_CACHE[4:]
    return g


# ----------------------------------------------------------------------------- Functions
def _linears(seq: nn.Module) -> List[nn.Linear]:
    return [m for m in seq.modules() if isinstance(m, nn.Linear)]


class _MLP(torch.autograd.Function):
    """y = LN(build_mlp(x)) (+ residual) or build_mlp(x); params = [W0, b0, W1, b1, ..., (gamma, beta)]."""

    @staticmethod
    def forward(ctx, nlin: int, has_ln: bool, x, residual, *params):
        acts = [x]
        h = x
        for k in range(nlin):
            h = gemm(h, params[2 * k], tb=True, bias=params[2 * k + 1], relu=k < nlin - 1)
            acts.append(h)
        yhat = rstd = None
        if has_ln:
            gamma, beta = params[2 * nlin], params[2 * nlin + 1]
            n, w = h.shape
            out = torch.empty_like(h)
            yhat = torch.empty_like(h)
            rstd = torch.empty(n, dtype=torch.float32, device=h.device)
            res = _dense(residual) if residual is not None else None
            check(lib().sgnn_layernorm(h.data_ptr() if n else None, n, w, gamma.data_ptr(), beta.data_ptr(),
                                       res.data_ptr() if res is not None else None, out.data_ptr() if n else None,
                                       yhat.data_ptr() if n else None, rstd.data_ptr() if n else None,
                                       stream_ptr(h.device)), "sgnn_layernorm")
        else:
            if residual is not None:
                raise ValueError("a residual needs the LayerNorm form")
            out = h
        ctx.nlin, ctx.has_ln, ctx.has_res = nlin, has_ln, residual is not None
        ctx.save_for_backward(*acts, yhat, rstd, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        nlin, has_ln = ctx.nlin, ctx.has_ln
        saved = ctx.saved_tensors
        acts = saved[:nlin + 1]
        yhat, rstd = saved[nlin + 1], saved[nlin + 2]
        params = saved[nlin + 3:]
        dout = _dense(dout) if has_ln else _c(dout)
        n = dout.shape[0]
        grads: List[Optional[torch.Tensor]] = [None] * len(params)
        if has_ln:
            gamma = params[2 * nlin]
            grads[2 * nlin] = colsum(dout, yhat)
            grads[2 * nlin + 1] = colsum(dout)
            g = torch.empty_like(dout)
            check(lib().sgnn_layernorm_bwd(dout.data_ptr() if n else None, yhat.data_ptr() if n else None,
                                           rstd.data_ptr() if n else None, gamma.data_ptr(), n, dout.shape[1],
                                           g.data_ptr() if n else None, stream_ptr(dout.device)),
                  "sgnn_layernorm_bwd")
        else:
            g = dout
        need_x = ctx.needs_input_grad[2]
        for k in range(nlin - 1, -1, -1):
            a = acts[k]
            grads[2 * k] = gemm(g, a, ta=True)      # dW [out, in] = dY^T A
            grads[2 * k + 1] = colsum(g)             # db
            if k > 0 or need_x:
                g2 = gemm(g, params[2 * k])          # dA [rows, in] = dY W
                if k > 0:                            # through the ReLU of the previous Linear
                    check(lib().sgnn_relu_bwd(g2.data_ptr() if n else None, g2.stride(0),
                                              a.data_ptr() if n else None, a.stride(0), n, g2.shape[1],
                                              stream_ptr(g2.device)), "sgnn_relu_bwd")
                g = g2
        dx = g if need_x else None
        dres = dout if (ctx.has_res and ctx.needs_input_grad[3]) else None
        return (None, None, dx, dres, *grads)


def mlp(seq: nn.Module, has_ln: bool, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """A reference-layout Sequential(build_mlp[, LayerNorm]) on rows x (any widths / depth)."""
    if has_ln:
        lins, ln = _linears(seq[0]), seq[1]
        params = [t for l in lins for t in (l.weight, l.bias)] + [ln.weight, ln.bias]
    else:
        lins = _linears(seq)
        params = [t for l in lins for t in (l.weight, l.bias)]
    for p in params:
        require_gpu_tensor(p, "parameter")
    if x.shape[1] != lins[0].in_features:
        raise ValueError(f"MLP input width {x.shape[1]} != {lins[0].in_features}")
    return _MLP.apply(len(lins), has_ln, _c(x), residual, *params)


class _GatherCat(torch.autograd.Function):
    """out[r] = cat_k(scale_k * src_k[idx_k[r]]) over `nrows` rows; spec_k = (idx, scale, grouping)."""

    @staticmethod
    def forward(ctx, nrows: int, specs, *srcs):
        widths = [s.shape[1] for s in srcs]
        dev = srcs[0].device
        out = torch.empty(nrows, sum(widths), dtype=torch.float32, device=dev)
        col = 0
        for (idx, scale, _), s, w in zip(specs, srcs, widths):
            if nrows:
                gather_into(out, col, s, idx, scale)
            col += w
        ctx.specs, ctx.widths, ctx.rows = specs, widths, [s.shape[0] for s in srcs]
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = _c(dout)
        grads = []
        col = 0
        for k, ((idx, scale, grp), w, rows) in enumerate(zip(ctx.specs, ctx.widths, ctx.rows)):
            if not ctx.needs_input_grad[2 + k]:
                grads.append(None)
            elif idx is None:
                d = torch.empty(rows, w, dtype=torch.float32, device=dout.device)
                if rows:
                    check(lib().sgnn_gather_rows(dout.data_ptr() + 4 * col, dout.stride(0), w, None, rows,
                                                 float(scale), d.data_ptr(), w, stream_ptr(dout.device)),
                          "sgnn_gather_rows")
                grads.append(d)
            else:
                d = torch.empty(rows, w, dtype=torch.float32, device=dout.device)
                if rows:
                    segment_sum_into(d, dout, col, w, grp.rowptr, grp.perm, scale)
                grads.append(d)
            col += w
        return (None, None, *grads)


def gather_cat(nrows: int, parts: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor], float, Optional[Grouping]]]):
    """cat of (src, index, scale, grouping-of-index) column blocks over nrows rows."""
    specs = tuple((idx, float(scale), grp) for _, idx, scale, grp in parts)
    return _GatherCat.apply(nrows, specs, *[_c(s) for s, _, _, _ in parts])


class _SegmentSum(torch.autograd.Function):
    """agg[i] = sum of m over the edges into i, in the stable receiver-CSR order."""

    @staticmethod
    def forward(ctx, graph: EdgeGraph, m):
        agg = torch.empty(graph.n, m.shape[1], dtype=torch.float32, device=m.device)
        if graph.n:
            if graph.E:
                segment_sum_into(agg, m, 0, m.shape[1], graph.by_recv.rowptr, graph.by_recv.perm)
            else:
                agg.zero_()
        ctx.graph = graph
        return agg

    @staticmethod
    def backward(ctx, dagg):
        g = ctx.graph
        dagg = _c(dagg)
        dm = torch.empty(g.E, dagg.shape[1], dtype=torch.float32, device=dagg.device)
        if g.E:
            gather_into(dm, 0, dagg, g.recv)
        return None, dm


# ----------------------------------------------------------------------------- modules
def message_passing(block: nn.Module, x: torch.Tensor, graph: EdgeGraph, e: torch.Tensor):
    """InteractionNetwork.forward (graph_network.py:150-222) / G2M / M2M / M2G block
    (multi_scale_gnn.py:84-205): (x + LN(node_fn([aggr, x])), e + e) with
    aggr = sum over receivers of LN(edge_fn([x_i, x_j, e])).  At the widths the
    fused kernels are built for (latents = MLP hidden = 64 / 128, nmlp_layers 1 / 2)
    forward and backward run the training step's fused layer kernels
    (sgnn_amd/fused_block.py); the GEMM chain below serves every other shape."""
    from . import fused_block
    if fused_block.applies(block, x, e, graph.E):
        return fused_block.message_passing(block, x, graph.fused(), e)
    x, e = _c(x), _c(e)
    if e.shape[0] != graph.E:
        raise ValueError(f"{e.shape[0]} edge feature rows for {graph.E} edges")
    msg_in = gather_cat(graph.E, [(x, graph.recv, 1.0, graph.by_recv), (x, graph.send, 1.0, graph.by_send),
                                  (e, None, 1.0, None)])
    m = mlp(block.edge_fn, True, msg_in)
    agg = _SegmentSum.apply(graph, m)
    x_new = mlp(block.node_fn, True, gather_cat(graph.n, [(agg, None, 1.0, None), (x, None, 1.0, None)]),
                residual=x)
    return x_new, gather_cat(graph.E, [(e, None, 2.0, None)])


def encoder_forward(enc: nn.Module, x: torch.Tensor, edge_features: torch.Tensor):
    """Encoder.forward (graph_network.py:98-111)."""
    return mlp(enc.node_fn, True, _rows(x, "x")), mlp(enc.edge_fn, True, _rows(edge_features, "edge_features"))


def decoder_forward(dec: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Decoder.forward (graph_network.py:324-333; no LayerNorm)."""
    return mlp(dec.node_fn, False, _rows(x, "x"))


def processor_forward(proc: nn.Module, x, edge_index, edge_features, graph: Optional[EdgeGraph] = None):
    """Processor.forward (graph_network.py:276-293)."""
    x = _rows(x, "x")
    g = graph if graph is not None else cached_edge_graph(edge_index, x.shape[0])
    e = _rows(edge_features, "edge_features")
    for gnn in proc.gnn_stacks:
        x, e = message_passing(gnn, x, g, e)
    return x, e


def epd_forward(epd: nn.Module, x, edge_index, edge_features, graph: Optional[EdgeGraph] = None):
    """EncodeProcessDecode.forward (graph_network.py:388-406)."""
    x, e = encoder_forward(epd._encoder, x, edge_features)
    x, e = processor_forward(epd._processor, x, edge_index, e, graph)
    return decoder_forward(epd._decoder, x)


def ms_gnn_forward(gnn: nn.Module, x, g2m_ei, g2m_e, m2m_ei, m2m_e, m2g_ei, m2g_e,
                   graphs: Optional[dict] = None) -> torch.Tensor:
    """MultiScaleGNN.forward (multi_scale_gnn.py:277-326), block by block."""
    x = _rows(x, "x")
    n = x.shape[0]
    gs = graphs or {"g2m": cached_edge_graph(g2m_ei, n), "m2m": cached_edge_graph(m2m_ei, n),
                    "m2g": cached_edge_graph(m2g_ei, n)}
    h = mlp(gnn.grid_node_encoder, True, x)
    eg = mlp(gnn.g2m_edge_encoder, True, _rows(g2m_e, "g2m_edge_features"))
    em = mlp(gnn.m2m_edge_encoder, True, _rows(m2m_e, "m2m_edge_features"))
    eo = mlp(gnn.m2g_edge_encoder, True, _rows(m2g_e, "m2g_edge_features"))
    h, eg = message_passing(gnn.g2m_block, h, gs["g2m"], eg)
    for blk in gnn.m2m_blocks:
        h, em = message_passing(blk, h, gs["m2m"], em)
    h, eo = message_passing(gnn.m2g_block, h, gs["m2g"], eo)
    return mlp(gnn.prediction_head, False, h)


def _rows(t: torch.Tensor, name: str) -> torch.Tensor:
    require_gpu_tensor(t, name)
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(t.shape)}")
    return _c(t)


def node_features(pos_seq: torch.Tensor, types: Optional[torch.Tensor], emb_w: Optional[torch.Tensor],
                  use_emb: bool, vel_mean, vel_std, wall_max: float, wall_div: float,
                  ntypes: int = 1) -> torch.Tensor:
    """_encoder_preprocessor's node features (learned_simulator.py:256-290): the
    velocity / wall columns from sgnn_node_features, the type embedding as a
    differentiable gather of the embedding rows (its gradient: per-type sums in
    node order)."""
    n, T, d = pos_seq.shape
    base = torch.empty(n, (T - 1) * d + 1, dtype=torch.float32, device=pos_seq.device)
    check(lib().sgnn_node_features(pos_seq.data_ptr(), n, T, d, None, None, 0, 0, vel_mean.data_ptr(),
                                   vel_std.data_ptr(), float(wall_max), float(wall_div), base.data_ptr(),
                                   stream_ptr(pos_seq.device)), "sgnn_node_features")
    if not use_emb:
        return base
    t32 = types.to(torch.int32).contiguous()
    return gather_cat(n, [(base, None, 1.0, None), (emb_w, t32, 1.0, grouping(types, ntypes))])
