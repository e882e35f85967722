"""ctypes binding of libsgnn_hip.so (the C-ABI declared in include/sgnn.h).

The library is the product: if it is missing or no GPU is visible, every
entry point raises — there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(HERE, "_lib", "libsgnn_hip.so")
# SGNN_LIB: an experiment build of the same library (tools/exp_ab.py, tools/exp_localize.py) in place of the
# product one -- for same-box A/Bs of the test suite; load_library warns loudly whenever it is set
LIB_PATH = os.environ.get("SGNN_LIB") or PRODUCT_LIB

ABI_VERSION = 6                               # include/sgnn.h SGNN_ABI_VERSION: checked at load
STEP_FLAG_WORDS, STEP_FLAG_ERR = 4128, 4096   # include/sgnn.h SGNN_STEP_FLAG_WORDS / _ERR: checked at load
SGNN_OK, SGNN_ERR_INVALID, SGNN_ERR_UNSUPPORTED, SGNN_ERR_HIP, SGNN_ERR_STEP_TIMEOUT = 0, 1, 2, 3, 4

c_void_p, c_int64, c_int32, c_float = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float


class SgnnMlp(ctypes.Structure):
    """struct sgnn_mlp (include/sgnn.h)."""
    _fields_ = [("w1", c_void_p), ("b1", c_void_p), ("w2", c_void_p), ("b2", c_void_p),
                ("ln_g", c_void_p), ("ln_b", c_void_p),
                ("in_dim", c_int32), ("hidden", c_int32), ("out_dim", c_int32), ("nlin", c_int32),
                ("w3", c_void_p), ("b3", c_void_p)]


P_MLP = ctypes.POINTER(SgnnMlp)


class SgnnSaves(ctypes.Structure):
    """struct sgnn_saves (include/sgnn.h)."""
    _fields_ = [("h", c_void_p), ("yhat", c_void_p), ("rstd", c_void_p), ("agg", c_void_p),
                ("hd", c_void_p), ("h2", c_void_p), ("hd2", c_void_p)]


class SgnnEpd(ctypes.Structure):
    """struct sgnn_epd (include/sgnn.h)."""
    _fields_ = [("nlayers", c_int32), ("enc_node", c_void_p), ("enc_edge", c_void_p), ("edge", c_void_p),
                ("node", c_void_p), ("dec", c_void_p)]


class SgnnStepIn(ctypes.Structure):
    """struct sgnn_step_in (include/sgnn.h)."""
    _fields_ = [("n", c_int64), ("T", c_int32), ("dim", c_int32), ("ex_ptr", c_void_p), ("n_ex", c_int32),
                ("radius", c_float), ("K", c_int32), ("types", c_void_p), ("emb_w", c_void_p),
                ("emb_dim", c_int32), ("use_emb", c_int32), ("vel_mean", c_void_p), ("vel_std", c_void_p),
                ("acc_mean", c_void_p), ("acc_std", c_void_p), ("wall_max", c_float), ("wall_div", c_float)]


class SgnnStepWs(ctypes.Structure):
    """struct sgnn_step_ws (include/sgnn.h)."""
    _fields_ = [("struct_size", c_int64), ("radius_ws", c_void_p), ("rowptr", c_void_p), ("send", c_void_p), ("recv", c_void_p),
                ("edge_cap", c_int64), ("e0t", c_void_p), ("x_a", c_void_p), ("x_b", c_void_p),
                ("u", c_void_p), ("v", c_void_p), ("agg", c_void_p), ("cin", c_void_p), ("cout", c_void_p),
                ("u2", c_void_p), ("v2", c_void_p), ("uvl", c_void_p), ("step_flags", c_void_p),
                ("step_deg", c_void_p), ("step_poll_limit", c_int32), ("step_skew", c_int32)]


class SgnnReduceDesc(ctypes.Structure):
    """struct sgnn_reduce_desc (include/sgnn.h)."""
    _fields_ = [("src", c_void_p), ("dst", c_void_p), ("slab_stride", c_int64), ("offset", c_int64),
                ("rep_stride", c_int64), ("nslab", c_int32), ("nrep", c_int32), ("src_ld", c_int32),
                ("nrows", c_int32), ("ncols", c_int32), ("dst_ld", c_int32), ("accumulate", c_int32),
                ("scale", c_float)]


P_SAVES = ctypes.POINTER(SgnnSaves)
SLAB_EDGE, SLAB_NODE, SLAB_UV, SLAB_DECODER, SLAB_ENC_NODE, SLAB_ENC_EDGE = range(6)

# name -> (restype, argtypes); every symbol include/sgnn.h declares
SIGNATURES = {
    "sgnn_version": (ctypes.c_char_p, []),
    "sgnn_last_error": (ctypes.c_char_p, []),
    "sgnn_abi_version": (c_int32, []),
    "sgnn_step_flag_words": (c_int32, []),
    "sgnn_radius_workspace_bytes": (ctypes.c_size_t, [c_int64, c_int32, c_int32]),
    "sgnn_radius_graph": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int32,
                                         c_float, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_int64, c_void_p]),
    "sgnn_encode_nodes": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                                         c_int32, c_int32, c_void_p, c_void_p, c_float, c_float,
                                         P_MLP, P_MLP, c_void_p, c_void_p, c_void_p, P_SAVES,
                                         c_void_p]),
    "sgnn_edge_latent_floats": (c_int64, [c_int64, c_int32]),
    "sgnn_encode_edges": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_float, c_void_p, c_void_p,
                                         c_void_p, c_int64, c_int64, P_MLP, c_void_p, P_SAVES,
                                         c_void_p]),
    "sgnn_edge_layer": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                       c_void_p, c_int64, c_int64, P_MLP, c_void_p, c_void_p,
                                       c_void_p, P_SAVES, c_void_p]),
    "sgnn_node_layer": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                       P_MLP, P_MLP, c_void_p, c_void_p, c_void_p, P_SAVES,
                                       c_void_p]),
    "sgnn_node_layer_decode": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_int64, P_MLP, P_MLP, c_void_p, c_int32, c_int32,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, P_SAVES, c_void_p]),
    "sgnn_interaction_layer": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                                              c_void_p, c_void_p, c_int64, P_MLP, P_MLP, P_MLP, c_void_p,
                                              c_void_p, c_void_p, c_void_p]),
    "sgnn_interaction_layer_decode": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                                                     c_void_p, c_void_p, c_void_p, c_int64, P_MLP, P_MLP,
                                                     P_MLP, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "sgnn_interaction_layer_encode": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_float, P_MLP, c_void_p,
                                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                     c_int64, P_MLP, P_MLP, P_MLP, c_void_p, c_void_p, c_void_p,
                                                     c_void_p]),
    "sgnn_coo_workspace_bytes": (ctypes.c_size_t, [c_int64, c_int64]),
    "sgnn_coo_to_csr": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "sgnn_encode_node_features": (ctypes.c_int, [c_void_p, c_int64, c_int32, P_MLP, P_MLP, c_void_p,
                                                 c_void_p, c_void_p, c_void_p]),
    "sgnn_encode_edge_features": (ctypes.c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_int64,
                                                 P_MLP, c_void_p, c_void_p]),
    "sgnn_bwd_slab_floats": (c_int64, [c_int32, c_int32, c_int32, c_int32]),
    "sgnn_bwd_scratch_floats": (c_int64, [c_int32, c_int32, c_int64, c_int32]),
    "sgnn_reduce_slabs": (ctypes.c_int, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "sgnn_transpose_workspace_bytes": (ctypes.c_size_t, [c_int64, c_int64]),
    "sgnn_transpose_csr": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                          c_void_p, c_void_p]),
    "sgnn_decoder_loss_bwd": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_int64, c_int32, c_int32, c_float,
                                             c_float, c_float, c_void_p, P_SAVES, c_void_p, P_MLP,
                                             c_void_p, c_void_p, c_int32, c_void_p]),
    "sgnn_node_layer_bwd": (ctypes.c_int, [c_void_p, c_int64, P_SAVES, c_void_p, P_MLP, c_void_p,
                                           c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "sgnn_edge_layer_bwd": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                           P_SAVES, c_void_p, c_float, P_MLP,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_int32, c_void_p, c_int32, c_void_p, c_int64, c_void_p]),
    "sgnn_uv_bwd": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_int64, P_MLP, c_void_p,
                                   c_void_p, c_int32, c_void_p, c_void_p]),
    "sgnn_encode_nodes_bwd": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                             c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                             c_void_p, c_void_p, c_float, c_float, P_SAVES,
                                             P_MLP, c_void_p, c_int32, c_void_p]),
    "sgnn_encode_nodes_bwd_typed": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                                   c_void_p, c_void_p, c_int32, c_int32,
                                                   c_void_p, c_void_p, c_float, c_float, P_SAVES,
                                                   P_MLP, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "sgnn_type_sums_workspace_bytes": (ctypes.c_size_t, [c_int64, c_int32, c_int32]),
    "sgnn_edge_latent_grad": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64,
                                             c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "sgnn_embedding_grad": (ctypes.c_int, [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32,
                                           c_int32, c_void_p, c_int32, c_void_p]),
    "sgnn_encode_edges_bwd": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int32, c_float,
                                             c_void_p, c_void_p, c_void_p, c_int64, P_SAVES,
                                             P_MLP, c_void_p, c_int32, c_void_p, c_int64, c_void_p]),
    "sgnn_predict_positions": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p]),
    "sgnn_node_features": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                          c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p]),
    "sgnn_edge_features": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_float, c_void_p, c_void_p, c_void_p, c_int64,
                                          c_int64, c_void_p, c_void_p]),
    "sgnn_step_path": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sgnn_step_check": (ctypes.c_int, [c_void_p, c_void_p]),
    "sgnn_rollout": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                    c_void_p, c_void_p]),
    "sgnn_edge_tiles_to_rows": (ctypes.c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_int64, c_float,
                                               c_void_p, c_int64, c_int32, c_void_p]),
    "sgnn_rollout_one_step": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                             c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "sgnn_random_walk_noise": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_float, ctypes.c_uint64,
                                              ctypes.c_uint64, c_void_p, c_void_p, c_void_p]),
    "sgnn_adam_step": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float,
                                      c_float, c_float, c_float, c_int64, c_void_p]),
    "sgnn_gemm_workspace_bytes": (ctypes.c_size_t, [c_int64, c_int64, c_int64]),
    "sgnn_gemm": (ctypes.c_int, [c_int32, c_int32, c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                 c_void_p, c_int32, c_void_p, c_int64, c_int32, c_void_p, ctypes.c_size_t, c_void_p]),
    "sgnn_layernorm": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p]),
    "sgnn_layernorm_bwd": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p,
                                          c_void_p]),
    "sgnn_colsum_workspace_bytes": (ctypes.c_size_t, [c_int64, c_int32]),
    "sgnn_colsum": (ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int32,
                                   c_void_p, ctypes.c_size_t, c_void_p]),
    "sgnn_relu_bwd": (ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p]),
    "sgnn_gather_rows": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_float, c_void_p, c_int64,
                                        c_void_p]),
    "sgnn_segment_sum_cols": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int64, c_float,
                                             c_void_p, c_int64, c_int32, c_void_p]),
    "sgnn_edge_rows_to_tiles": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int64, c_int64,
                                               c_void_p, c_void_p]),
}

_LIB: Optional[ctypes.CDLL] = None


class SgnnError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """dlopen the library and bind every symbol (no GPU needed)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise SgnnError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                        "(the HIP library is required; there is no CPU fallback)")
    if os.path.abspath(path) != os.path.abspath(PRODUCT_LIB):
        import sys
        import warnings
        msg = f"sgnn_amd: loading a NON-PRODUCT library build {path} (SGNN_LIB / experiment tool)"
        print("WARNING: " + msg, file=sys.stderr, flush=True)
        warnings.warn(msg, stacklevel=2)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sgnn_abi_version() != ABI_VERSION or lib.sgnn_step_flag_words() != STEP_FLAG_WORDS:
        raise SgnnError(f"{path}: ABI {lib.sgnn_abi_version()} / {lib.sgnn_step_flag_words()} flag words, this "
                        f"binding expects {ABI_VERSION} / {STEP_FLAG_WORDS}: rebuild the library")
    _LIB = lib
    return lib


def lib() -> ctypes.CDLL:
    return _LIB if _LIB is not None else load_library()


def check(status: int, what: str) -> None:
    if status != SGNN_OK:
        msg = lib().sgnn_last_error().decode()
        kind = {SGNN_ERR_INVALID: ValueError, SGNN_ERR_UNSUPPORTED: NotImplementedError}.get(status, SgnnError)
        raise kind(f"{what}: {msg} (status {status})")


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu_tensor(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor (sgnn_amd runs on MI355X only; no CPU path)")
