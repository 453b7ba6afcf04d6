"""ctypes binding of liblgnn.so (the C ABI declared in include/lgnn.h).

The library is loaded from this package directory only (in-tree build, `make` or
``__graft_entry__.build()``). There is no fallback: if the library or a GPU is missing, every
product op raises. torch is imported first so that the HIP runtime torch ships
(libamdhip64.so.7) is the one the library binds to — one runtime per process.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# LGNN_LIB_PATH: an alternative build of the same library (A/B timing of kernel variants,
# tools/ab_lib.sh); the default is the in-tree build
LIB_PATH = os.environ.get("LGNN_LIB_PATH") or os.path.join(_HERE, "liblgnn.so")

LGNN_LOOPS_KEEP, LGNN_LOOPS_REMAINING, LGNN_LOOPS_READD = 0, 1, 2
LGNN_NORM_NONE, LGNN_NORM_GCN = 0, 1
LGNN_ACT_NONE, LGNN_ACT_ELU = 0, 1
LGNN_BN_GSTATS, LGNN_BN_GIN = 3, 4
LGNN_GRAD_DIRECT, LGNN_GRAD_POOL, LGNN_GRAD_TRANSPOSE = 0, 1, 2
LGNN_SLOT_FLAG0 = 7  # tile_open: count + six barrier words, then the partial-slot skip words
LGNN_SLOT_FLAGS = 256
LGNN_TILE_OPEN_EXTRA = LGNN_SLOT_FLAG0 + LGNN_SLOT_FLAGS  # words after the per-tile flags
LGNN_S3_ADJT_TILE_BYTES = 16384  # lgnn.h: fp32 Â per tile, split-3 forward -> fused backward
LGNN_OPT_GAT_PIPE, LGNN_OPT_GAT_BPC, LGNN_OPT_GRAPH_SORTED = 0, 1, 2  # lgnn_set_option

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float
F64 = ctypes.c_double
SZ = ctypes.c_size_t


class CeSrc(ctypes.Structure):
    """lgnn_ce_src (include/lgnn.h): the readout's CE factors the logits gradient is formed from,
    dlogits[i][c] = gloss * wt[i] / wsum * pm[i][c]."""
    _fields_ = [("pm", P), ("wt", P), ("wsum", P), ("gloss", P)]


LGNN_PLANE_JOB_MAX = 8


class PlaneJob(ctypes.Structure):
    """lgnn_plane_job (include/lgnn.h): the split-3 weight planes lgnn_graph_build_planes writes
    beside the build (lgnn_weight_planes' arguments)."""
    _fields_ = [("nl", I32), ("widths", I32 * (LGNN_PLANE_JOB_MAX + 1)),
                ("W", P * LGNN_PLANE_JOB_MAX), ("planes", P), ("planes_t", P)]


# name -> (restype, argtypes); mirrors include/lgnn.h exactly
SIGNATURES: dict[str, tuple] = {
    "lgnn_abi_version": (I32, []),
    "lgnn_status_string": (ctypes.c_char_p, [I32]),
    "lgnn_set_option": (I32, [I32, I32]),
    "lgnn_get_option": (I32, [I32]),
    "lgnn_graph_workspace_bytes": (SZ, [I64, I64]),
    "lgnn_graph_build_path": (I32, [P, I64, I64, P]),
    "lgnn_graph_build_lazy": (I32, [P, I64, I64, I32, I32, P, P, P, P, P, P, P, P, P, I64, P, P,
                                    P, SZ, P]),
    "lgnn_graph_build": (I32, [P, I64, I64, I32, I32, P, P, P, P, P, P, P, P, P, I64, P, P, P,
                               SZ, P]),
    "lgnn_graph_build_planes": (I32, [P, I64, I64, I32, I32, P, P, P, P, P, P, P, P, P, I64, P,
                                      P, P, SZ, I32, P, P]),
    "lgnn_batch_ptr": (I32, [P, I64, I64, P, P]),
    "lgnn_node_linear_fwd": (I32, [P, I64, I32, P, P, P, F32, P, P, I32, I32, P, P, P]),
    "lgnn_bwd_num_partials": (I32, [I64, I32, I32, I32]),
    "lgnn_node_linear_bwd": (I32, [I32, P, P, P, I32, P, P, P, F32, P, I32, P, I64, I32,
                                   P, P, P, F32, P, I32, P, P, P, I32, P]),
    "lgnn_reduce_partials": (I32, [P, I32, I64, P, P]),
    "lgnn_node_linear_bwd_tiles": (I32, [I32, P, P, P, I32, P, P, P, F32, P, I32, P, I64, I32,
                                         P, P, P, F32, P, I32, P, P, P, I32, P, I32, I32, P]),
    "lgnn_gcn_stack_bwd_partials": (I32, [I64]),
    "lgnn_adam_step": (I32, [I32, P, P, P, P, P, P, P, F32, F32, F32, F32, F32, I32, I32, I32,
                             P]),
    "lgnn_gcn_stack_bwd": (I32, [P, P, P, I32, P, P, P, P, I64, I32, P, P, P, P, P, I32, P, P]),
    "lgnn_spmm": (I32, [P, P, P, F32, P, I64, I32, P, P]),
    "lgnn_reduce_partials_multi": (I32, [I32, P, P, P, P, P]),
    "lgnn_reduce_jobs": (I32, [I32, P, P, P, P, P, P, P]),
    "lgnn_reduce_jobs_ce": (I32, [I32, P, P, P, P, P, P, P, ctypes.POINTER(CeSrc), I32, P]),
    "lgnn_ce_fwd": (I32, [P, P, P, I64, I32, P, P, P, P, P]),
    "lgnn_ce_fwd_factors": (I32, [P, P, P, I64, I32, P, P, P, P, P, P, P]),
    "lgnn_ce_bwd": (I32, [P, P, P, I64, I32, P, P, P, P, P]),
    "lgnn_pool_head_fwd": (I32, [P, P, I64, I32, I32, P, P, I32, P, P, P]),
    "lgnn_pool_head_bwd": (I32, [P, P, I64, I32, P, I32, P, P, P, P]),
    "lgnn_pool_bwd": (I32, [P, P, P, I64, I32, I32, P, P]),
    "lgnn_bn_workspace_bytes": (SZ, [I64, I32]),
    "lgnn_bn_stats": (I32, [P, I64, I32, P, P, SZ, P]),
    "lgnn_bn_finalize": (I32, [P, F64, P, P, F32, F32, I32, I32, P, P, P, P, P, P, P, P]),
    "lgnn_bn_act": (I32, [P, I64, I32, P, P, P, P, P]),
    "lgnn_bn_bwd_stats": (I32, [P, P, P, I64, I32, P, P, P, P, P, P, SZ, P]),
    "lgnn_gat_att": (I32, [P, I64, I32, I32, P, P, P, P, P]),
    "lgnn_bf16_kpad": (I32, [I32]),
    "lgnn_bf16_gemm_att": (I32, [P, I32, I64, I32, P, I32, P, P, P, P, I32, I32, P, P, P]),
    "lgnn_bf16_weight_prep": (I32, [P, I32, I32, P, P, P]),
    "lgnn_bf16_weight_prep_multi": (I32, [I32, P, P, P, P, P, P]),
    "lgnn_bf16_gemm": (I32, [P, I32, I64, I32, P, P, I32, P, P, P, P]),
    "lgnn_bf16_wgrad_partials": (I32, [I64, I32]),
    "lgnn_bf16_wgrad": (I32, [P, I32, P, I32, I64, I32, P, I32, P]),
    "lgnn_gat_fwd": (I32, [P, P, P, P, P, I64, I32, I32, F32, P, P, I32, P, P, P, P]),
    "lgnn_gat_bwd_edge": (I32, [P, P, P, P, P, P, P, P, P, I32, I64, I32, I32, F32, P, P, P, P]),
    "lgnn_gat_bwd_edge_pool": (I32, [P, P, P, P, P, P, P, P, I32, I64, I32, I32, F32, P, P, I32,
                                      P, P, I32, P, P, P, P]),
    "lgnn_regression_fwd": (I32, [P, P, I32, I64, F32, F32, I32, P, P, P]),
    "lgnn_regression_bwd": (I32, [P, P, I32, I64, F32, F32, I32, P, P, P, P]),
    "lgnn_gat_bwd_num_partials": (I32, [I64]),
    "lgnn_gat_bwd_node": (I32, [P, P, P, P, P, P, P, P, P, P, P, I64, I32, I32, P, P, I32, P,
                                P]),
    "lgnn_gcn_stack_fwd": (I32, [P, I64, I32, I32, P, P, P, I32, P, P, P, P, P, P]),
    "lgnn_gcn_stack_fwd_s3": (I32, [P, I64, I32, I32, P, P, P, I32, P, P, P, P, P, P, P]),
    "lgnn_weight_planes_bytes": (SZ, [I32]),
    "lgnn_weight_planes": (I32, [I32, P, P, P, P, P]),
    "lgnn_gcn_stack_bwd_s3_partials": (I32, [I64]),
    "lgnn_gcn_stack_bwd_s3": (I32, [P, P, P, I32, I64, P, P, P, P, I64, I32, P, P, P, P, P, I32,
                                    P, P, P]),
    "lgnn_knn_workspace_bytes": (SZ, [I64]),
    "lgnn_knn_graph": (I32, [P, I64, I32, P, P, I64, I32, I32, P, I64, P, SZ, P]),
    "lgnn_radius_workspace_bytes": (SZ, [I64]),
    "lgnn_radius_count": (I32, [P, I64, I32, P, P, I64, F64, I32, I32, P, SZ, P]),
    "lgnn_radius_graph": (I32, [P, I64, I32, P, P, I64, F64, I32, I32, P, I64, P, SZ, P]),
    "lgnn_gaussian_distance": (I32, [P, I32, I64, I32, P, I64, F64, P, I32, P, P]),
    "lgnn_tile_count": (I32, [I64]),
    "lgnn_tile_open": (I32, [P, P, I64, P, P]),
    "lgnn_node_linear_fwd_tiles": (I32, [P, I64, I32, P, P, P, F32, P, P, I32, I32, P, P, P, I32,
                                         P]),
    "lgnn_bn_bwd_apply": (I32, [P, P, P, I64, I32, P, P, P, P, P, F64, I32, P, P, P, P]),
    "lgnn_bn_partials_reduce": (I32, [P, I32, I32, P, P, P, P]),
    "lgnn_bn_partials_finalize": (I32, [P, I32, I32, P, F64, P, P, F32, F32, P, P, P, P, P, P, P,
                                        P]),
    "lgnn_bn_fused_partials": (I32, [I64]),
    "lgnn_node_linear_fwd_bn": (I32, [P, I64, I32, P, P, P, F32, P, P, I32, I32, P, P, P, P, P, P,
                                      P, P]),
    "lgnn_node_linear_bwd_bn": (I32, [I32, P, P, I32, P, I64, I32, P, I32, P, P, P, I32, P, P, P,
                                      P, P, P, P, P, F64, I32, P]),
    "lgnn_node_linear_bwd_bn_gather": (I32, [P, P, P, P, F32, P, I32, P, I64, I32, P, I32, P, P,
                                              P, I32, P, P, P, P, P, P, P, P]),
    "lgnn_node_linear_bwd_bn_pool": (I32, [I32, P, P, I32, P, I64, I32, P, I32, P, P, P, I32, P,
                                           P, P, P, P, P, P, P, F64, I32, P, P, I32, P, P, I32,
                                           P]),
    "lgnn_gcn_stack_bwd_s3f": (I32, [P, P, P, I32, I64, P, P, P, P, I64, I32, P, P, P, P, P,
                                     I32, P, P, P]),
    "lgnn_gcn_stack_fwd_s3_all": (I32, [P, I64, I32, I32, P, P, P, I32, P, P, P, P, P, P, P, P, P]),
    "lgnn_gcn_stack_bwd_s3f_all": (I32, [P, P, P, I32, I64, P, P, P, P, P, P, P, I64, I32, P, P, P,
                                         P, P, P, P, I32, P, P, P, P, I32, P, P]),
    "lgnn_gcn_stack_bwd_s3f_ce": (I32, [P, P, I32, I64, P, P, P, P, P, P, P, I64, I32, P, P, P, P,
                                        P, P, P, I32, P, P, ctypes.POINTER(CeSrc), P, I32, P, P]),
    "lgnn_fused_grid_capacity": (I32, [I32]),
    "lgnn_dropout_masks": (I32, [I32, P, P, P, P, P, I32, P]),
    "lgnn_s3_weight_planes_numel": (SZ, [I32, I32, I32]),
    "lgnn_s3_weight_planes": (I32, [P, I32, I32, I32, I32, P, P]),
    "lgnn_s3_weight_planes_multi": (I32, [I32, P, P, P, P, I32, P, P]),
    "lgnn_s3_gemm_att": (I32, [P, I64, I32, P, I32, I32, P, P, P, I32, I32, P, P, P]),
    "lgnn_s3_gemm_act": (I32, [P, I64, I32, P, I32, P, I32, P, P]),
    "lgnn_s3_gemm": (I32, [P, I64, I32, P, I32, I32, P, P, P, P]),
    "lgnn_s3_wgrad_partials": (I32, [I64, I32, I32]),
    "lgnn_s3_wgrad": (I32, [P, I32, P, I64, I32, I32, P, I32, P, P]),
    "lgnn_mask_mul": (I32, [P, P, P, I64, P]),
    "lgnn_act_bwd": (I32, [P, P, P, I64, I32, P]),
    "lgnn_sort_pool_workspace_bytes": (SZ, []),
    "lgnn_sort_pool_fwd": (I32, [P, I64, I32, P, I64, I32, P, P, P, P, SZ, P]),
    "lgnn_sort_pool_bwd": (I32, [P, P, P, P, P, I64, I32, I32, P, P]),
    "lgnn_cc_pool_workspace_bytes": (SZ, [I64, I32, I32]),
    "lgnn_cc_pool": (I32, [P, I32, I64, P, I32, I32, P, P, P, P, SZ, P]),
}

ABI_VERSION = 39

_lib = None


class LgnnError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load and type the library (no GPU needed to load)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LgnnError(f"{LIB_PATH} is missing: build it with `make` or __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.lgnn_abi_version() != ABI_VERSION:
        raise LgnnError("liblgnn.so ABI version mismatch; rebuild")
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().lgnn_status_string(status)
        raise LgnnError(f"{what} failed: {status} ({msg.decode() if msg else '?'})")


@contextlib.contextmanager
def path_option(option: int, value: int):
    """Set one of the library's process-wide path options (lgnn_set_option: the alternative kernel
    a test checks the default against) for the duration of a with-block."""
    lib = load()
    old = lib.lgnn_set_option(option, int(value))
    if old < 0:
        raise LgnnError(f"lgnn_set_option({option}, {value}) failed: {old}")
    try:
        yield
    finally:
        lib.lgnn_set_option(option, old)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(*tensors: torch.Tensor) -> None:
    """The product path is HIP-only: refuse CPU tensors instead of silently falling back."""
    for t in tensors:
        # meta tensors only while torch.compile / torch.export traces (shape propagation
        # through the fake kernels of library.py; nothing is launched)
        if t is not None and not t.is_cuda and not (t.is_meta and torch.compiler.is_compiling()):
            raise LgnnError("lesion_gnn_amd ops run on the GPU only (HIP kernels); got a CPU "
                            "tensor. There is no CPU fallback by design.")


# Measurement hook (bench.py's per-entry HIP-event timing): when set, every call() runs as
# _TRACER(name, args, launch) so the tracer can bracket the launch with events on its stream.
_TRACER = None


def set_tracer(tracer) -> None:
    global _TRACER
    _TRACER = tracer


def call(name: str, *args) -> None:
    fn = getattr(load(), name)
    if _TRACER is None:
        check(fn(*args), name)
    else:
        check(_TRACER(name, args, lambda: fn(*args)), name)
