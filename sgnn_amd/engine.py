"""Host orchestration of the HIP kernels: parameter packing, HBM workspaces,
and the per-step launch sequence.  Everything here launches on the current
torch stream through the C-ABI (no host synchronisation inside a step; a
whole rollout is one sgnn_rollout call).

Data layout in HBM (per graph of n particles, hidden H, cap K):
  rowptr[n+1], send[n*K], recv[n*K]   int32 receiver-sorted CSR (E = rowptr[n])
  e0t   [ceil(nK/32)][TH][4][64][4]   fp32 encoder edge latent, 32-edge tiles in
                                      MFMA C-layout order (one 1 KiB load per
                                      wave instruction)
  x_a/x_b [n][H] ping-pong node latents; u, v [n][H] per-node halves of the
  next edge MLP's first Linear; agg [n][H]; cin/cout [nK/32][H] tile carries.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import _hip
from ._hip import SgnnMlp, check, lib, stream_ptr

MAX_NUM_NEIGHBORS = 20  # learned_simulator.py:117
FUSED_MAX_N = 8192      # fused per-layer kernel for graphs up to this size (sgnn_predict_positions)

# Test hook (include/sgnn.h sgnn_step_ws.step_skew): workspaces created after set_test_step_skew(k) make
# the one-launch step's tiles sleep before their phase publishes.  0 in every product run; no environment
# variable reaches it.
_TEST_STEP_SKEW = 0


def set_test_step_skew(k: int) -> None:
    """Uneven-load test hook for the one-launch step's hand-off (tests / tools only)."""
    global _TEST_STEP_SKEW
    _TEST_STEP_SKEW = int(k)


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _linears(seq: nn.Module) -> List[nn.Linear]:
    return [m for m in seq.modules() if isinstance(m, nn.Linear)]


def mlp_struct(seq: nn.Module, has_ln: bool) -> SgnnMlp:
    """struct sgnn_mlp from a reference-layout Sequential(mlp[, LayerNorm])."""
    if has_ln:
        mlp, ln = seq[0], seq[1]
    else:
        mlp, ln = seq, None
    lin = _linears(mlp)
    for p in [*(l.weight for l in lin), *(l.bias for l in lin)] + ([ln.weight, ln.bias] if ln else []):
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
            raise ValueError("sgnn_amd parameters must be contiguous fp32 GPU tensors "
                             "(call simulator.to('cuda'))")
    if len(lin) not in (2, 3):
        raise NotImplementedError("libsgnn_hip implements nmlp_layers = 1 or 2 MLPs")
    return SgnnMlp(w1=lin[0].weight.data_ptr(), b1=lin[0].bias.data_ptr(),
                   w2=lin[1].weight.data_ptr(), b2=lin[1].bias.data_ptr(),
                   ln_g=_ptr(ln.weight) if ln is not None else 0,
                   ln_b=_ptr(ln.bias) if ln is not None else 0,
                   in_dim=lin[0].in_features, hidden=lin[0].out_features,
                   out_dim=lin[-1].out_features, nlin=len(lin),
                   w3=lin[2].weight.data_ptr() if len(lin) == 3 else 0,
                   b3=lin[2].bias.data_ptr() if len(lin) == 3 else 0)


class ParamPack:
    """The ctypes parameter structs of one EncodeProcessDecode, rebuilt only
    when a parameter tensor is replaced (e.g. after .to())."""

    def __init__(self, epd: nn.Module):
        self.key = tuple(p.data_ptr() for p in epd.parameters())
        self.enc_node = mlp_struct(epd._encoder.node_fn, True)
        self.enc_edge = mlp_struct(epd._encoder.edge_fn, True)
        self.edge = [mlp_struct(g.edge_fn, True) for g in epd._processor.gnn_stacks]
        self.node = [mlp_struct(g.node_fn, True) for g in epd._processor.gnn_stacks]
        self.dec = mlp_struct(epd._decoder.node_fn, False)
        nl = len(self.edge)
        self.edge_arr = (SgnnMlp * nl)(*self.edge)
        self.node_arr = (SgnnMlp * nl)(*self.node)
        self.epd = _hip.SgnnEpd(nlayers=nl, enc_node=ctypes.addressof(self.enc_node),
                                enc_edge=ctypes.addressof(self.enc_edge), edge=ctypes.addressof(self.edge_arr),
                                node=ctypes.addressof(self.node_arr), dec=ctypes.addressof(self.dec))

    @staticmethod
    def get(epd: nn.Module) -> "ParamPack":
        key = tuple(p.data_ptr() for p in epd.parameters())
        pack = getattr(epd, "_sgnn_pack", None)
        if pack is None or pack.key != key:
            pack = ParamPack(epd)
            epd._sgnn_pack = pack
        return pack


class StepWorkspace:
    """HBM buffers for one (n, T, dim, H, K, loop) step shape."""

    def __init__(self, n: int, T: int, dim: int, hidden: int, K: int, loop: bool,
                 device: torch.device, one_launch: bool = True):
        L = lib()
        self.n, self.T, self.dim, self.H, self.K, self.loop = n, T, dim, hidden, K, loop
        cap = K + (0 if loop else 1)
        self.edge_cap = max(1, n * cap)
        ntiles = (self.edge_cap + 31) // 32
        i32 = dict(dtype=torch.int32, device=device)
        f32 = dict(dtype=torch.float32, device=device)
        self.radius_ws = torch.empty(int(L.sgnn_radius_workspace_bytes(n, K, int(loop))) + 256,
                                     dtype=torch.uint8, device=device)
        self.rowptr = torch.zeros(n + 1, **i32)
        self.send = torch.empty(self.edge_cap, **i32)
        self.recv = torch.empty(self.edge_cap, **i32)
        self.e0t = torch.empty(int(L.sgnn_edge_latent_floats(self.edge_cap, hidden)), **f32)
        self.x_a = torch.empty(n, hidden, **f32)
        self.x_b = torch.empty(n, hidden, **f32)
        self.u = torch.empty(n, hidden, **f32)
        self.v = torch.empty(n, hidden, **f32)
        # second node-half buffers: small graphs at hidden 64 run each layer as one fused
        # sgnn_interaction_layer launch (u/v ping-pong); the C driver applies the same limit
        fused = hidden == 64 and n <= FUSED_MAX_N
        self.u2 = torch.empty(n, hidden, **f32) if fused else None
        self.v2 = torch.empty(n, hidden, **f32) if fused else None
        self.agg = torch.empty(n, hidden, **f32)
        self.cin = torch.empty(ntiles, hidden, **f32)
        self.cout = torch.empty(ntiles, hidden, **f32)
        # one-launch step buffers: allocated by prepare_step the first time sgnn_step_path says a call
        # takes that path (every layer's node halves, the per-workgroup phase counters, the neighbour counts)
        self.uvl = self.step_flags = self.step_deg = None
        self.c = _hip.SgnnStepWs(struct_size=ctypes.sizeof(_hip.SgnnStepWs), radius_ws=self.radius_ws_ptr(), rowptr=self.rowptr.data_ptr(),
                                 send=self.send.data_ptr(), recv=self.recv.data_ptr(), edge_cap=self.edge_cap,
                                 e0t=self.e0t.data_ptr(), x_a=self.x_a.data_ptr(), x_b=self.x_b.data_ptr(),
                                 u=self.u.data_ptr(), v=self.v.data_ptr(), agg=self.agg.data_ptr(),
                                 cin=self.cin.data_ptr(), cout=self.cout.data_ptr(),
                                 u2=_ptr(self.u2), v2=_ptr(self.v2), uvl=0, step_flags=0, step_deg=0,
                                 step_poll_limit=0, step_skew=_TEST_STEP_SKEW)
        self.device = device
        # False: never allocate them (calls take the kernel sequence).  SGNN_ONE_LAUNCH=0: the same for every
        # workspace of the process (several processes sharing one device, include/sgnn.h "Co-residency")
        self.one_launch = one_launch and os.environ.get("SGNN_ONE_LAUNCH", "1") != "0"

    def prepare_step(self, epd_struct, sin) -> bool:
        """Allocate the one-launch step's buffers when sgnn_step_path says calls with these
        arguments take it (True then); the C driver still decides per call (its co-residency
        guard may run the kernel sequence instead)."""
        if self.step_flags is not None:
            return True
        if not self.one_launch:
            return False
        probe = _hip.SgnnStepWs.from_buffer_copy(self.c)
        probe.uvl = probe.step_flags = probe.step_deg = 1   # only tested for NULL by sgnn_step_path
        if not lib().sgnn_step_path(ctypes.byref(epd_struct), ctypes.byref(sin), ctypes.byref(probe), None, None):
            return False
        n, H, K = self.n, self.H, self.K
        f32 = dict(dtype=torch.float32, device=self.device)
        self.uvl = torch.empty(epd_struct.nlayers * 2 * n * H + (n + 32) * K * (H + 4), **f32)
        self.step_flags = torch.zeros(_hip.STEP_FLAG_WORDS, dtype=torch.int32, device=self.device)
        self.step_deg = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.c.uvl, self.c.step_flags, self.c.step_deg = (self.uvl.data_ptr(), self.step_flags.data_ptr(),
                                                          self.step_deg.data_ptr())
        return True

    def check_step(self, device) -> None:
        """Raise SgnnError if the last call's one-launch step timed out waiting for its sender tiles
        (sgnn_step_check: its outputs are invalid).  Synchronises the stream; skipped while a HIP
        graph is being captured (the replays' caller checks) and when the step buffers do not exist."""
        if self.step_flags is None or torch.cuda.is_current_stream_capturing():
            return
        check(lib().sgnn_step_check(ctypes.byref(self.c), stream_ptr(device)), "predict_positions")

    def radius_ws_ptr(self) -> int:
        p = self.radius_ws.data_ptr()
        return (p + 255) & ~255

    def num_edges(self) -> int:
        """E of the CSR the kernel sequence built (host sync) — API/diagnostics only."""
        return int(self.rowptr[self.n].item())

    def step_edges(self) -> int:
        """E of the last one-launch step (sum of its neighbour counts; host sync)."""
        return int(self.step_deg.sum().item())

    def step_timeout(self) -> bool:
        """True if a workgroup of the last one-launch step gave up waiting (its error word; tests)."""
        return self.step_flags is not None and int(self.step_flags[_hip.STEP_FLAG_ERR].item()) != 0


def step_path(epd_struct, sin, ws: StepWorkspace):
    """(one_launch, nodes per workgroup, workgroups) of sgnn_predict_positions for these arguments."""
    ws.prepare_step(epd_struct, sin)
    nt, grid = ctypes.c_int32(0), ctypes.c_int32(0)
    one = lib().sgnn_step_path(ctypes.byref(epd_struct), ctypes.byref(sin), ctypes.byref(ws.c),
                               ctypes.byref(nt), ctypes.byref(grid))
    return bool(one), nt.value, grid.value


def ex_ptr_tensor(counts: Sequence[int], device: torch.device) -> torch.Tensor:
    ptr = [0]
    for c in counts:
        ptr.append(ptr[-1] + int(c))
    return torch.tensor(ptr, dtype=torch.int64).to(device, non_blocking=False)


def counts_of(nparticles_per_example) -> List[int]:
    """learned_simulator.py:89-94 and evaluate.py:121 (`[tensor(N)]`)."""
    if isinstance(nparticles_per_example, torch.Tensor):
        return [int(v) for v in nparticles_per_example.detach().reshape(-1).cpu().tolist()]
    out = []
    for v in nparticles_per_example:
        if isinstance(v, torch.Tensor):
            out.extend(int(x) for x in v.detach().reshape(-1).cpu().tolist())
        else:
            out.append(int(v))
    return out


def radius_graph(ws: StepWorkspace, pos: torch.Tensor, pos_offset_floats: int, pos_stride: int,
                 ex_ptr: torch.Tensor, n_ex: int, radius: float) -> None:
    check(lib().sgnn_radius_graph(pos.data_ptr() + 4 * pos_offset_floats, pos_stride, ws.n, ws.dim,
                                  ex_ptr.data_ptr(), n_ex, float(radius), ws.K, int(ws.loop),
                                  ws.radius_ws_ptr(), ws.rowptr.data_ptr(), ws.send.data_ptr(),
                                  ws.recv.data_ptr(), ws.edge_cap, stream_ptr(pos.device)),
          "sgnn_radius_graph")


@dataclass
class CsrGraph:
    """A static receiver-sorted CSR graph over n nodes (int32, on the GPU)."""
    rowptr: torch.Tensor   # [n+1]
    send: torch.Tensor     # [max(E,1)]
    recv: torch.Tensor     # [max(E,1)]
    n: int
    num_edges: int

    @property
    def edge_cap(self) -> int:
        return max(1, self.num_edges)

    @property
    def ntiles(self) -> int:
        return (self.edge_cap + 31) // 32

    def edge_index(self) -> torch.Tensor:
        """[2, E] int64 = [senders; receivers] in CSR order."""
        e = self.num_edges
        return torch.stack([self.send[:e], self.recv[:e]]).to(torch.int64)


def coo_to_csr(edge_index: torch.Tensor, n: int, with_perm: bool = False) -> CsrGraph:
    """edge_index [2, E] (row 0 senders, row 1 receivers, PyG source_to_target)
    -> stable receiver-sorted CSR through sgnn_coo_to_csr.  Index range is
    checked here (one host sync: static graphs are built once)."""
    if edge_index.dim() != 2 or edge_index.shape[0] != 2:
        raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
    require = _hip.require_gpu_tensor
    require(edge_index, "edge_index")
    ei = edge_index.to(torch.int64).contiguous()
    E = int(ei.shape[1])
    dev = ei.device
    if E > 0:
        lo, hi = int(ei.min().item()), int(ei.max().item())
        if lo < 0 or hi >= n:
            raise ValueError(f"edge_index values must lie in [0, {n}), got [{lo}, {hi}]")
    L = lib()
    ws = torch.empty(int(L.sgnn_coo_workspace_bytes(n, E)) + 256, dtype=torch.uint8, device=dev)
    rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    send = torch.zeros(max(E, 1), dtype=torch.int32, device=dev)
    recv = torch.zeros(max(E, 1), dtype=torch.int32, device=dev)
    src, dst = ei[0].contiguous(), ei[1].contiguous()
    perm = torch.zeros(max(E, 1), dtype=torch.int32, device=dev) if with_perm else None
    check(L.sgnn_coo_to_csr(src.data_ptr() if E else None, dst.data_ptr() if E else None, E, n,
                            (ws.data_ptr() + 255) & ~255, rowptr.data_ptr(), send.data_ptr(),
                            recv.data_ptr(), _ptr(perm), stream_ptr(dev)), "sgnn_coo_to_csr")
    g = CsrGraph(rowptr, send, recv, n, E)
    g.perm = perm
    return g


def radius_graph_csr(pos: torch.Tensor, radius: float, K: int, loop: bool,
                     counts: Optional[Sequence[int]] = None) -> CsrGraph:
    """torch_cluster radius_graph(pos, r, batch, loop, max_num_neighbors=K) as a
    CSR graph sized to its edge count (one host sync: for static graphs)."""
    _hip.require_gpu_tensor(pos, "positions")
    p = pos.to(torch.float32).contiguous()
    n, d = p.shape
    dev = p.device
    counts = [n] if counts is None else list(counts)
    ex_ptr = ex_ptr_tensor(counts, dev)
    L = lib()
    cap = max(1, n * (K + (0 if loop else 1)))
    ws = torch.empty(int(L.sgnn_radius_workspace_bytes(n, K, int(loop))) + 256, dtype=torch.uint8,
                     device=dev)
    rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    send = torch.empty(cap, dtype=torch.int32, device=dev)
    recv = torch.empty(cap, dtype=torch.int32, device=dev)
    check(L.sgnn_radius_graph(p.data_ptr(), d, n, d, ex_ptr.data_ptr(), len(counts), float(radius),
                              K, int(loop), (ws.data_ptr() + 255) & ~255, rowptr.data_ptr(),
                              send.data_ptr(), recv.data_ptr(), cap, stream_ptr(dev)),
          "sgnn_radius_graph")
    E = int(rowptr[n].item())
    return CsrGraph(rowptr, send[:max(E, 1)].clone(), recv[:max(E, 1)].clone(), n, E)


@dataclass
class StepInputs:
    pos_seq: torch.Tensor           # [n, T, dim] fp32 contiguous, GPU
    ex_ptr: torch.Tensor            # [n_ex+1] int64, GPU
    n_ex: int
    types: Optional[torch.Tensor]   # [n] int64 GPU (only with embeddings)
    vel_mean: torch.Tensor
    vel_std: torch.Tensor
    acc_mean: torch.Tensor
    acc_std: torch.Tensor


def step_in(inp: StepInputs, ws: StepWorkspace, radius: float, emb_weight: Optional[torch.Tensor],
            use_emb: bool) -> "_hip.SgnnStepIn":
    """struct sgnn_step_in of one single-scale step (wall feature clamp(x+2, 0, R))."""
    emb_dim = emb_weight.shape[1] if (use_emb and emb_weight is not None) else 0
    return _hip.SgnnStepIn(n=ws.n, T=ws.T, dim=ws.dim, ex_ptr=inp.ex_ptr.data_ptr(), n_ex=inp.n_ex,
                           radius=float(radius), K=ws.K, types=_ptr(inp.types) if use_emb else 0,
                           emb_w=_ptr(emb_weight) if use_emb else 0, emb_dim=emb_dim, use_emb=int(use_emb),
                           vel_mean=inp.vel_mean.data_ptr(), vel_std=inp.vel_std.data_ptr(),
                           acc_mean=inp.acc_mean.data_ptr(), acc_std=inp.acc_std.data_ptr(),
                           wall_max=float(radius), wall_div=1.0)


def forward_step(epd: nn.Module, emb_weight: Optional[torch.Tensor], use_emb: bool, radius: float,
                 inp: StepInputs, ws: StepWorkspace, pred: torch.Tensor, next_pos: torch.Tensor,
                 window_out: Optional[torch.Tensor] = None, timers: Optional[list] = None) -> None:
    """One LearnedSimulator.predict_positions (learned_simulator.py:413-438):
    radius graph -> encoder -> L interaction layers -> decoder -> Euler.
    Issued as ONE sgnn_predict_positions call (the launch sequence runs in C);
    with `timers`, launched kernel by kernel so the edge layers can be timed
    (one event pair per edge layer; small graphs: one pair around all L fused
    layers)."""
    L = lib()
    pk = ParamPack.get(epd)
    if timers is None:
        sin = step_in(inp, ws, radius, emb_weight, use_emb)
        ws.prepare_step(pk.epd, sin)
        check(L.sgnn_predict_positions(ctypes.byref(pk.epd), ctypes.byref(sin), inp.pos_seq.data_ptr(),
                                       ctypes.byref(ws.c), pred.data_ptr(), next_pos.data_ptr(),
                                       _ptr(window_out), stream_ptr(inp.pos_seq.device)), "sgnn_predict_positions")
        ws.check_step(inp.pos_seq.device)
        return
    n, T, d = ws.n, ws.T, ws.dim
    s = stream_ptr(inp.pos_seq.device)
    pos = inp.pos_seq
    radius_graph(ws, pos, (T - 1) * d, T * d, inp.ex_ptr, inp.n_ex, radius)
    emb_dim = emb_weight.shape[1] if (use_emb and emb_weight is not None) else 0
    check(L.sgnn_encode_nodes(pos.data_ptr(), n, T, d, _ptr(inp.types) if use_emb else 0,
                              _ptr(emb_weight) if use_emb else 0, emb_dim, int(use_emb),
                              inp.vel_mean.data_ptr(), inp.vel_std.data_ptr(), float(radius), 1.0,
                              ctypes.byref(pk.enc_node), ctypes.byref(pk.edge[0]),
                              ws.x_a.data_ptr(), ws.u.data_ptr(), ws.v.data_ptr(), None, s),
          "sgnn_encode_nodes")
    nl = len(pk.edge)
    # same launch sequence as sgnn_predict_positions (rollout.hip)
    enc_in_layer0 = ws.u2 is not None and nl > 1 and pk.enc_edge.nlin == 2 and pk.node[0].nlin == 2
    if not enc_in_layer0:
        check(L.sgnn_encode_edges(pos.data_ptr() + 4 * (T - 1) * d, T * d, d, float(radius),
                                  ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n,
                                  ws.edge_cap, ctypes.byref(pk.enc_edge), ws.e0t.data_ptr(), None, s),
              "sgnn_encode_edges")
    x_in, x_out = ws.x_a, ws.x_b
    if ws.u2 is not None:   # small graphs at hidden 64: one fused launch per layer
        uv_in, uv_out = (ws.u, ws.v), (ws.u2, ws.v2)
        # one event pair around the L back-to-back fused launches (events between them would add
        # their own cost to every launch); the caller divides by L
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        for k in range(nl):
            if k == 0 and enc_in_layer0:
                check(L.sgnn_interaction_layer_encode(
                    pos.data_ptr() + 4 * (T - 1) * d, T * d, d, float(radius), ctypes.byref(pk.enc_edge),
                    ws.e0t.data_ptr(), x_in.data_ptr(), uv_in[0].data_ptr(), uv_in[1].data_ptr(),
                    ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n, ctypes.byref(pk.edge[0]),
                    ctypes.byref(pk.node[0]), ctypes.byref(pk.edge[1]), x_out.data_ptr(), uv_out[0].data_ptr(),
                    uv_out[1].data_ptr(), s), "sgnn_interaction_layer_encode")
                x_in, x_out = x_out, x_in
                uv_in, uv_out = uv_out, uv_in
            elif k < nl - 1:
                check(L.sgnn_interaction_layer(x_in.data_ptr(), uv_in[0].data_ptr(), uv_in[1].data_ptr(),
                                               ws.e0t.data_ptr(), float(2.0 ** k), ws.rowptr.data_ptr(),
                                               ws.send.data_ptr(), ws.recv.data_ptr(), n, ctypes.byref(pk.edge[k]),
                                               ctypes.byref(pk.node[k]), ctypes.byref(pk.edge[k + 1]),
                                               x_out.data_ptr(), uv_out[0].data_ptr(), uv_out[1].data_ptr(), s),
                      "sgnn_interaction_layer")
                x_in, x_out = x_out, x_in
                uv_in, uv_out = uv_out, uv_in
            else:
                check(L.sgnn_interaction_layer_decode(
                    x_in.data_ptr(), uv_in[0].data_ptr(), uv_in[1].data_ptr(), ws.e0t.data_ptr(), float(2.0 ** k),
                    ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n, ctypes.byref(pk.edge[k]),
                    ctypes.byref(pk.node[k]), ctypes.byref(pk.dec), pos.data_ptr(), T, d, inp.acc_mean.data_ptr(),
                    inp.acc_std.data_ptr(), pred.data_ptr(), next_pos.data_ptr(), _ptr(window_out), s),
                    "sgnn_interaction_layer_decode")
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        timers.append((ev0, ev1))
        return
    for k in range(nl):
        if timers is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        check(L.sgnn_edge_layer(ws.u.data_ptr(), ws.v.data_ptr(), ws.e0t.data_ptr(), float(2.0 ** k),
                                ws.rowptr.data_ptr(), ws.send.data_ptr(), ws.recv.data_ptr(), n,
                                ws.edge_cap, ctypes.byref(pk.edge[k]), ws.agg.data_ptr(),
                                ws.cin.data_ptr(), ws.cout.data_ptr(), None, s), "sgnn_edge_layer")
        if timers is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            timers.append((ev0, ev1))
        if k < nl - 1:
            check(L.sgnn_node_layer(x_in.data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                    ws.cout.data_ptr(), ws.rowptr.data_ptr(), n,
                                    ctypes.byref(pk.node[k]), ctypes.byref(pk.edge[k + 1]),
                                    x_out.data_ptr(), ws.u.data_ptr(), ws.v.data_ptr(), None, s),
                  "sgnn_node_layer")
            x_in, x_out = x_out, x_in
        else:
            check(L.sgnn_node_layer_decode(x_in.data_ptr(), ws.agg.data_ptr(), ws.cin.data_ptr(),
                                           ws.cout.data_ptr(), ws.rowptr.data_ptr(), n,
                                           ctypes.byref(pk.node[k]), ctypes.byref(pk.dec),
                                           pos.data_ptr(), T, d, inp.acc_mean.data_ptr(),
                                           inp.acc_std.data_ptr(), 0, pred.data_ptr(),
                                           next_pos.data_ptr(), _ptr(window_out), None, s),
                  "sgnn_node_layer_decode")


class ChainBuffers:
    """Node / edge buffers of one explicit-feature forward (n nodes, edge sets)."""

    def __init__(self, n: int, hidden: int, graphs: Dict[str, "CsrGraph"], device):
        L = lib()
        f32 = dict(dtype=torch.float32, device=device)
        self.x_a, self.x_b = torch.empty(n, hidden, **f32), torch.empty(n, hidden, **f32)
        self.u, self.v = torch.empty(n, hidden, **f32), torch.empty(n, hidden, **f32)
        self.agg = torch.empty(n, hidden, **f32)
        nt = max(g.ntiles for g in graphs.values())
        self.cin, self.cout = torch.empty(nt, hidden, **f32), torch.empty(nt, hidden, **f32)
        self.e0t = {k: torch.empty(int(L.sgnn_edge_latent_floats(g.edge_cap, hidden)), **f32)
                    for k, g in graphs.items()}


def _feature_rows(t: torch.Tensor, name: str) -> torch.Tensor:
    _hip.require_gpu_tensor(t, name)
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(t.shape)}")
    return t.to(torch.float32).contiguous()


def run_chain(enc_node, enc_edges: Dict[str, SgnnMlp], edges: List[SgnnMlp], nodes: List[SgnnMlp],
              decoder: SgnnMlp, kinds: List[str], scales: List[float], x: torch.Tensor,
              graphs: Dict[str, "CsrGraph"], efeats: Dict[str, torch.Tensor], out_dim: int) -> torch.Tensor:
    """Encoder -> blocks -> decoder on explicit features (no integrator): the
    operator boundary EncodeProcessDecode.forward / MultiScaleGNN.forward."""
    L = lib()
    n, feat = x.shape
    H = edges[0].hidden
    dev = x.device
    s = stream_ptr(dev)
    b = ChainBuffers(n, H, graphs, dev)
    check(L.sgnn_encode_node_features(x.data_ptr(), n, feat, ctypes.byref(enc_node), ctypes.byref(edges[0]),
                                      b.x_a.data_ptr(), b.u.data_ptr(), b.v.data_ptr(), s),
          "sgnn_encode_node_features")
    for k, g in graphs.items():
        if g.num_edges == 0:
            continue
        ef = efeats[k]
        if ef.shape[0] != g.num_edges:
            raise ValueError(f"edge features of {k}: {ef.shape[0]} rows for {g.num_edges} edges")
        check(L.sgnn_encode_edge_features(ef.data_ptr(), ef.shape[1], g.perm.data_ptr(), g.rowptr.data_ptr(), n,
                                          g.edge_cap, ctypes.byref(enc_edges[k]), b.e0t[k].data_ptr(), s),
              "sgnn_encode_edge_features")
    pred = torch.empty(n, out_dim, dtype=torch.float32, device=dev)
    x_in, x_out = b.x_a, b.x_b
    nb = len(edges)
    for i in range(nb):
        g = graphs[kinds[i]]
        check(L.sgnn_edge_layer(b.u.data_ptr(), b.v.data_ptr(), b.e0t[kinds[i]].data_ptr(), float(scales[i]),
                                g.rowptr.data_ptr(), g.send.data_ptr(), g.recv.data_ptr(), n, g.edge_cap,
                                ctypes.byref(edges[i]), b.agg.data_ptr(), b.cin.data_ptr(), b.cout.data_ptr(),
                                None, s), "sgnn_edge_layer")
        if i < nb - 1:
            check(L.sgnn_node_layer(x_in.data_ptr(), b.agg.data_ptr(), b.cin.data_ptr(), b.cout.data_ptr(),
                                    g.rowptr.data_ptr(), n, ctypes.byref(nodes[i]), ctypes.byref(edges[i + 1]),
                                    x_out.data_ptr(), b.u.data_ptr(), b.v.data_ptr(), None, s),
                  "sgnn_node_layer")
            x_in, x_out = x_out, x_in
        else:
            check(L.sgnn_node_layer_decode(x_in.data_ptr(), b.agg.data_ptr(), b.cin.data_ptr(), b.cout.data_ptr(),
                                           g.rowptr.data_ptr(), n, ctypes.byref(nodes[i]), ctypes.byref(decoder),
                                           None, 0, out_dim - 1, None, None, 0, pred.data_ptr(), None, None,
                                           None, s), "sgnn_node_layer_decode")
    return pred


def epd_forward(epd, x, edge_index, edge_features):
    """EncodeProcessDecode.forward(x, edge_index, edge_features)
    (graph_network.py:388-406) on the HIP kernels: explicit node features
    [N, F], edge_index [2, E] (senders; receivers), edge features [E, F_e] ->
    decoder output [N, d+1]."""
    x = _feature_rows(x, "x")
    ef = _feature_rows(edge_features, "edge_features")
    g = coo_to_csr(edge_index, x.shape[0], with_perm=True)
    pk = ParamPack.get(epd)
    nl = len(pk.edge)
    return run_chain(pk.enc_node, {"e": pk.enc_edge}, pk.edge, pk.node, pk.dec, ["e"] * nl,
                     [2.0 ** k for k in range(nl)], x, {"e": g}, {"e": ef}, pk.dec.out_dim)


def interaction_forward(block: nn.Module, x: torch.Tensor, edge_index: torch.Tensor, edge_features: torch.Tensor,
                        graph: Optional[CsrGraph] = None):
    """One InteractionNetwork / G2M / M2M / M2G block forward in inference
    (graph_network.py:150-222) on the fused kernels: u = W1_i x + b1 and v = W1_j x
    (the node halves of the first edge Linear, sgnn_gemm), the given edge latent
    rows in the tiled layout (sgnn_edge_rows_to_tiles), then sgnn_edge_layer
    (k_edge_layer: gather, edge MLP, LayerNorm, receiver sums) and sgnn_node_layer
    (k_node_layer: node MLP, LayerNorm, residual).  Returns (x', 2e)."""
    from . import autograd
    x = _feature_rows(x, "x")
    e = _feature_rows(edge_features, "edge_features")
    n = x.shape[0]
    g = graph if graph is not None else coo_to_csr(edge_index, n, with_perm=True)
    if e.shape[0] != g.num_edges:
        raise ValueError(f"{e.shape[0]} edge feature rows for {g.num_edges} edges")
    L = lib()
    dev = x.device
    s = stream_ptr(dev)
    edge_fn, node_fn = mlp_struct(block.edge_fn, True), mlp_struct(block.node_fn, True)
    H = edge_fn.hidden
    w1 = _linears(block.edge_fn[0])[0]
    u = autograd.gemm(x, w1.weight[:, :H], tb=True, bias=w1.bias)
    v = autograd.gemm(x, w1.weight[:, H:2 * H], tb=True)
    f32 = dict(dtype=torch.float32, device=dev)
    e0t = torch.empty(int(L.sgnn_edge_latent_floats(g.edge_cap, H)), **f32)
    check(L.sgnn_edge_rows_to_tiles(e.data_ptr() if g.num_edges else None, max(e.stride(0), H), H, g.perm.data_ptr(),
                                    g.rowptr.data_ptr(), n, g.edge_cap, e0t.data_ptr(), s), "sgnn_edge_rows_to_tiles")
    agg = torch.empty(n, H, **f32)
    cin, cout = torch.empty(g.ntiles, H, **f32), torch.empty(g.ntiles, H, **f32)
    check(L.sgnn_edge_layer(u.data_ptr(), v.data_ptr(), e0t.data_ptr(), 1.0, g.rowptr.data_ptr(), g.send.data_ptr(),
                            g.recv.data_ptr(), n, g.edge_cap, ctypes.byref(edge_fn), agg.data_ptr(), cin.data_ptr(),
                            cout.data_ptr(), None, s), "sgnn_edge_layer")
    x_out = torch.empty(n, H, **f32)
    # sgnn_node_layer also forms the next block's u / v: given this block's edge_fn, into scratch
    check(L.sgnn_node_layer(x.data_ptr(), agg.data_ptr(), cin.data_ptr(), cout.data_ptr(), g.rowptr.data_ptr(), n,
                            ctypes.byref(node_fn), ctypes.byref(edge_fn), x_out.data_ptr(), u.data_ptr(),
                            v.data_ptr(), None, s), "sgnn_node_layer")
    e2 = torch.empty_like(e)
    if g.num_edges:
        autograd.gather_into(e2, 0, e, None, 2.0)   # update returns the input edge features: e + e
    return x_out, e2


class DeviceRollout:
    """Autoregressive rollout issued as ONE sgnn_rollout call (evaluate.py:
    117-145): the C driver ping-pongs two window buffers (the shift is fused
    into the decoder kernel) and writes every step's prediction straight into
    its output slot — no host round trip, no Python per kernel."""

    def __init__(self, epd_struct, sin, ws: StepWorkspace, window: torch.Tensor, n: int, dim: int,
                 nsteps: int, keep=()):
        dev = window.device
        self.epd, self.sin, self.ws, self.keep = epd_struct, sin, ws, keep
        ws.prepare_step(epd_struct, sin)
        self.n, self.dim, self.nsteps = n, dim, nsteps
        self.win = [window.to(torch.float32).contiguous().clone(), torch.empty_like(window, dtype=torch.float32)]
        self.out_pos = torch.empty(max(nsteps, 1), n, dim, dtype=torch.float32, device=dev)
        self.out_pred = torch.empty(max(nsteps, 1), n, dim + 1, dtype=torch.float32, device=dev)

    def run(self, window: Optional[torch.Tensor] = None, check_step: bool = True,
            ground_truth: Optional[torch.Tensor] = None):
        """Returns (positions [nsteps, n, dim], strain [nsteps, n]) on the device.  With check_step
        (default) the call ends with sgnn_step_check (a stream sync) and raises SgnnError when a
        one-launch step timed out; a caller passing False must call ws.check_step itself.
        ground_truth [n, >= nsteps, dim] switches to the teacher-forced ("one_step") rollout
        (evaluate.py:140-143): each next window ends with the ground-truth frame of the step, not the
        prediction -- still ONE library call (sgnn_rollout_one_step)."""
        if window is not None:
            self.win[0].copy_(window)
        dev = self.win[0].device
        if ground_truth is None:
            check(lib().sgnn_rollout(ctypes.byref(self.epd), ctypes.byref(self.sin), self.win[0].data_ptr(),
                                     self.win[1].data_ptr(), ctypes.byref(self.ws.c), self.nsteps,
                                     self.out_pos.data_ptr(), self.out_pred.data_ptr(), stream_ptr(dev)),
                  "sgnn_rollout")
        else:
            _hip.require_gpu_tensor(ground_truth, "ground_truth")
            if (ground_truth.dim() != 3 or ground_truth.shape[0] != self.n or ground_truth.shape[2] != self.dim
                    or ground_truth.shape[1] < self.nsteps):
                raise ValueError(f"ground_truth must be [{self.n}, >= {self.nsteps}, {self.dim}], "
                                 f"got {tuple(ground_truth.shape)}")
            gt = ground_truth.to(torch.float32)
            if gt.stride(2) != 1:
                gt = gt.contiguous()
            self.keep_gt = gt
            check(lib().sgnn_rollout_one_step(ctypes.byref(self.epd), ctypes.byref(self.sin), self.win[0].data_ptr(),
                                              self.win[1].data_ptr(), ctypes.byref(self.ws.c), self.nsteps,
                                              gt.data_ptr(), gt.stride(0), gt.stride(1), self.out_pos.data_ptr(),
                                              self.out_pred.data_ptr(), stream_ptr(dev)), "sgnn_rollout_one_step")
        if check_step:
            self.ws.check_step(self.win[0].device)
        return self.out_pos[:self.nsteps], self.out_pred[:self.nsteps, :, -1]
