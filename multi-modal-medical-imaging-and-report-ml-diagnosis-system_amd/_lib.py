"""ctypes binding of libmmdx_hip.so (the C ABI declared in include/mmdx.h).

The product path has exactly one implementation: these HIP kernels.  If the library is
missing or fails to load, every op raises — there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# MMDX_LIB_PATH: an alternative build of the same library (A/B measurements of two builds
# in one GPU session); the product path loads the in-tree lib/libmmdx_hip.so
LIB_PATH = os.environ.get("MMDX_LIB_PATH") or os.path.join(_HERE, "lib", "libmmdx_hip.so")

F32, BF16, F16 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_GELU, ACT_GELU_BWD = 0, 1, 2, 3

vp, i32, i64, f32, sz, u64 = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_size_t, C.c_uint64


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("N", "H", "W", "C", "K", "R", "S", "stride_h", "stride_w", "pad_h", "pad_w",
                 "P", "Q")]


class AdamWTensor(C.Structure):
    _fields_ = [("p", vp), ("g", vp), ("m", vp), ("v", vp), ("n", C.c_long), ("off", C.c_long),
                ("lr", C.c_float), ("wd", C.c_float)]


CD = C.POINTER(ConvDesc)


class PackItem(C.Structure):
    """mmdx_pack_item (include/mmdx.h): one weight of a multi-tensor pack launch."""
    _fields_ = [("w", vp), ("krsc", vp), ("crsk", vp), ("K", C.c_int), ("C", C.c_int),
                ("c_master", C.c_int), ("RS", C.c_int), ("first_block", C.c_long)]


class PlanOp(C.Structure):
    """mmdx_plan_op (include/mmdx.h): one recorded operation of a launch plan."""
    _fields_ = [("op", C.c_int), ("dtype", C.c_int), ("stream", C.c_int), ("i", C.c_int * 8),
                ("l", C.c_long * 4),
                ("f", C.c_float * 4), ("p", C.c_void_p * 12), ("ext", C.c_int * 12),
                ("d", ConvDesc)]


(OP_EVENT, OP_NCHW2NHWC, OP_CONV_PACK, OP_CONV_FWD, OP_BN_FWD, OP_MAXPOOL_FWD,
 OP_AVGPOOL_FWD, OP_CAST, OP_AVGPOOL_BWD, OP_MAXPOOL_BWD, OP_BN_BWD, OP_CONV_WGRAD,
 OP_CONV_DGRAD, OP_SIGNAL, OP_WAIT, OP_CONV_DGRAD_BNSTAT, OP_STEM_PAIR_INPUT,
 OP_STEM_PAIR_PACK, OP_STEM_PAIR_GRAD, OP_CONV_PACK_MULTI, OP_CONV_FWD_BNEVAL,
 OP_MAXPOOL_BN_FWD, OP_BN_BWD_POOL, OP_CONV_DGRAD_ACCMASK, OP_BN_BWD_MASKED_DY,
 OP_GEMM, OP_ATTN_FWD, OP_ATTN_BWD, OP_LN_FWD, OP_LN_BWD, OP_GELU_BWD, OP_BIAS_GRAD, OP_ADD,
 OP_DROPOUT_FWD, OP_DROPOUT_BWD, OP_AXPBY, OP_ATTN_FWD_LSE, OP_ATTN_BWD_LSE, OP_LN_FWD_DROP,
 OP_LN_BWD_DROP, OP_GEMM_BIAS_GRAD, OP_RETIRED_42, OP_BN_APPLY) = range(1, 44)

# name -> (restype, argtypes).  Kept in header order; tests check this table against
# include/mmdx.h so the binding cannot drift from the ABI.
SIGNATURES = {
    "mmdx_version": (i32, []),
    "mmdx_last_error": (C.c_char_p, []),
    "mmdx_reload_config": (i32, []),
    "mmdx_stream_create": (i32, [i32, i32, C.POINTER(vp)]),
    "mmdx_stream_destroy": (i32, [vp]),
    "mmdx_gemm_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_gemm": (i32, [i32, i32, i32, i32, vp, i64, i32, vp, i64, i32, vp, i64, i32, vp, vp,
                        i32, f32, f32, vp, vp, sz, vp]),
    "mmdx_conv_pack_weight": (i32, [i32, CD, i32, vp, vp, vp, vp]),
    "mmdx_conv_pack_blocks": (i64, [i32, i32, i32]),
    "mmdx_conv_pack_multi": (i32, [i32, vp, i32, i64, vp]),
    "mmdx_conv_fwd_stat_blocks": (i32, [CD]),
    "mmdx_conv_fwd_stat_rows": (i32, [CD]),
    "mmdx_conv_fwd": (i32, [i32, CD, vp, vp, vp, vp, vp]),
    "mmdx_conv_fwd_rows": (i32, [i32, CD, vp, vp, vp, vp, i32, vp]),
    "mmdx_conv_fwd_bn_eval": (i32, [i32, CD, vp, vp, vp, vp, vp, vp, vp, f32, vp, i32, vp]),
    "mmdx_conv_dgrad": (i32, [i32, CD, vp, vp, vp, f32, vp]),
    "mmdx_conv_dgrad_stat_blocks": (i32, [i32, CD]),
    "mmdx_conv_dgrad_bnstat": (i32, [i32, CD, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, i32, vp,
                                     vp]),
    "mmdx_conv_dgrad_accmask": (i32, [i32, CD, vp, vp, vp, vp, vp, vp]),
    "mmdx_conv_wgrad_workspace_size": (sz, [i32, CD]),
    "mmdx_conv_wgrad": (i32, [i32, CD, i32, vp, vp, vp, f32, vp, sz, vp]),
    "mmdx_stem_pair_desc": (i32, [i32, i32, i32, i32, i32, i32, i32, i32, i32, CD]),
    "mmdx_stem_pair_input": (i32, [vp, i32, i32, i32, i32, i32, vp, vp]),
    "mmdx_stem_pair_pack_weight": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "mmdx_stem_pair_grad": (i32, [vp, i32, i32, i32, i32, vp, f32, vp]),
    "mmdx_bn_workspace_size": (sz, [i64, i32]),
    "mmdx_bn_fwd": (i32, [i32, i32, vp, i64, i32, vp, i32, i64, vp, vp, vp, vp, f32, f32, vp, vp,
                          vp, i32, vp, vp, sz, vp]),
    "mmdx_bn_fwd_ex": (i32, [i32, i32, vp, i64, i32, vp, i32, i64, vp, vp, vp, vp, f32, f32, vp,
                             vp, vp, i32, vp, vp, vp, sz, vp]),
    "mmdx_bn_finalize": (i32, [vp, i32, i64, i64, i32, vp, vp, vp, vp, f32, f32, vp, vp, vp, vp,
                               vp]),
    "mmdx_bn_apply": (i32, [i32, vp, vp, i64, i32, vp, vp, i32, vp, vp, vp]),
    "mmdx_bn_bwd": (i32, [i32, i32, vp, vp, vp, i64, i32, vp, vp, vp, vp, i32, vp, i32, vp, vp,
                          vp, vp, f32, vp, sz, vp]),
    "mmdx_bn_bwd_masked_dy": (i32, [i32, i32, vp, vp, vp, i64, i32, vp, vp, vp, vp, vp, vp, vp,
                                    f32, vp, sz, vp]),
    "mmdx_bn_bwd_ex": (i32, [i32, i32, vp, vp, vp, i64, i32, vp, vp, vp, vp, i32, vp, i32, vp,
                             vp, vp, vp, f32, vp, vp, sz, vp]),
    "mmdx_bn_bwd_pool": (i32, [i32, i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32,
                               i32, vp, vp, vp, vp, i32, vp, vp, vp, f32, vp, sz, vp]),
    "mmdx_img_desc_size": (sz, []),
    "mmdx_image_preprocess": (i32, [vp, vp, i32, vp, i32, i32, i32, vp, vp, vp]),
    "mmdx_plan_run": (i32, [C.POINTER(PlanOp), i32, vp, vp, vp, i32]),
    "mmdx_plan_op_size": (sz, []),
    "mmdx_maxpool_fwd": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, i32, i32,
                               vp]),
    "mmdx_maxpool_bn_fwd": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp,
                                  i32, vp, vp, i32, i32, vp]),
    "mmdx_maxpool_bwd": (i32, [i32, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp,
                               vp]),
    "mmdx_avgpool_fwd": (i32, [i32, vp, i32, i32, i32, vp, vp]),
    "mmdx_avgpool_bwd": (i32, [i32, vp, i32, i32, i32, vp, vp]),
    "mmdx_nchw_to_nhwc": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp]),
    "mmdx_cast": (i32, [i32, i32, vp, i64, vp, vp]),
    "mmdx_axpby": (i32, [i64, f32, vp, f32, vp, vp, vp]),
    "mmdx_layernorm_fwd": (i32, [i32, vp, vp, i64, i32, vp, vp, f32, vp, vp, vp, vp, vp]),
    "mmdx_layernorm_bwd": (i32, [i32, vp, vp, i64, i32, vp, vp, vp, vp, vp, vp, f32, vp, sz,
                                 vp]),
    "mmdx_layernorm_workspace_size": (sz, [i64, i32]),
    "mmdx_layernorm_bwd_residual": (i32, [i32, vp, vp, i64, i32, vp, vp, vp, vp, vp, vp, vp,
                                          f32, vp, sz, vp]),
    "mmdx_gemm_res": (i32, [i32, i32, i32, i32, vp, i64, i32, vp, i64, i32, vp, i64, i32, vp, vp,
                            i32, f32, f32, vp, vp, vp, sz, vp]),
    "mmdx_gemm_bias_grad_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_gemm_bias_grad": (i32, [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, i32, vp, vp, sz,
                                  vp]),
    "mmdx_layernorm_fwd_dropout": (i32, [i32, vp, vp, i64, i32, vp, vp, f32, f32, u64, vp, vp,
                                         vp, vp, vp, vp, vp]),
    "mmdx_layernorm_bwd_dropout": (i32, [i32, vp, vp, i64, i32, vp, vp, vp, f32, vp, vp, vp, vp,
                                         vp, f32, vp, sz, vp]),
    "mmdx_gelu_bwd": (i32, [i32, vp, vp, i64, vp, vp]),
    "mmdx_bias_grad": (i32, [i32, vp, i64, i32, vp, f32, vp, sz, vp]),
    "mmdx_bias_grad_workspace_size": (sz, [i64, i32]),
    "mmdx_dropout_fwd": (i32, [i32, vp, i64, f32, u64, u64, vp, vp, vp, vp]),
    "mmdx_dropout_bwd": (i32, [i32, vp, vp, i64, f32, vp, vp]),
    "mmdx_bce_logits_fwd": (i32, [vp, vp, i32, i32, vp, vp]),
    "mmdx_bce_logits_bwd": (i32, [vp, vp, i32, i32, vp, vp, vp]),
    "mmdx_embed_ln_fwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, f32, vp, vp, vp,
                                vp, vp]),
    "mmdx_embed_bwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp, vp, vp, i32, vp]),
    "mmdx_masked_mean_fwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp]),
    "mmdx_masked_mean_bwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp]),
    "mmdx_embed_mean_fwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp, vp]),
    "mmdx_embed_mean_bwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp, vp]),
    "mmdx_embed_gather": (i32, [i32, vp, i64, i32, vp, vp, vp]),
    "mmdx_embed_scatter": (i32, [i32, vp, i64, i32, vp, vp, vp]),
    "mmdx_attention_fwd": (i32, [i32, vp, vp, i32, i32, i32, f32, f32, u64, vp, vp, vp, vp]),
    "mmdx_attention_fwd_ex": (i32, [i32, vp, vp, vp, i32, i32, i32, i32, f32, f32, u64, vp, vp,
                                    vp, vp]),
    "mmdx_attention_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_attention_bwd": (i32, [i32, vp, vp, vp, vp, i32, i32, i32, f32, f32, vp, vp, sz, vp]),
    "mmdx_attention_fwd_lse": (i32, [i32, vp, vp, i32, i32, i32, f32, f32, u64, vp, vp, vp, vp,
                                     vp]),
    "mmdx_attention_lse_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_attention_bwd_lse": (i32, [i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, vp,
                                     vp, sz, vp]),
    "mmdx_lstm_fwd": (i32, [i32, vp, vp, i32, i32, i32, vp, vp, vp, vp, sz, vp, i64, i32, vp]),
    "mmdx_lstm_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_lstm_fwd_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_lstm_bwd": (i32, [i32, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, sz, vp, i64, i32,
                            vp]),
    "mmdx_patchify": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp]),
    "mmdx_vit_tokens_fwd": (i32, [i32, vp, vp, vp, i32, i32, i32, vp, vp]),
    "mmdx_vit_tokens_bwd": (i32, [i32, vp, i32, i32, i32, vp, vp]),
    "mmdx_rows_copy": (i32, [i32, vp, i64, vp, i64, i64, i32, vp]),
    "mmdx_add": (i32, [i32, i64, vp, vp, vp, vp]),
    "mmdx_rmsnorm_fwd": (i32, [i32, vp, i64, i32, vp, f32, vp, vp, vp]),
    "mmdx_rmsnorm_workspace_size": (sz, [i64, i32]),
    "mmdx_rmsnorm_bwd": (i32, [i32, vp, vp, i64, i32, vp, vp, vp, f32, vp, f32, vp, sz, vp]),
    "mmdx_t5_position_bias": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "mmdx_t5_position_bias_bwd": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, vp, f32, vp]),
    "mmdx_xattn_fwd": (i32, [i32, vp, i64, vp, i32, i32, i32, i32, f32, f32, u64, vp, vp, vp,
                             vp]),
    "mmdx_xattn_workspace_size": (sz, [i32, i32, i32, i32]),
    "mmdx_xattn_bwd": (i32, [i32, vp, i64, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, i64,
                             vp, vp, sz, vp]),
    "mmdx_cross_entropy_workspace_size": (sz, [i64]),
    "mmdx_cross_entropy_fwd": (i32, [vp, vp, i64, i64, vp, vp, vp, sz, vp]),
    "mmdx_cross_entropy_bwd": (i32, [i32, vp, vp, i64, i64, vp, vp, vp, vp, vp]),
    "mmdx_log_softmax": (i32, [vp, i64, i64, vp, vp]),
    "mmdx_relu_bwd": (i32, [i32, vp, vp, i64, vp, vp]),
    "mmdx_t5_decode_attn": (i32, [i32, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]),
    "mmdx_beam_topk": (i32, [vp, i32, i32, i64, vp, vp, i32, i32, i32, vp, vp, vp]),
    "mmdx_adamw_multi": (i32, [i32, vp, f32, f32, f32, vp, vp, vp]),
    "mmdx_grad_norm_workspace_size": (sz, [i32]),
    "mmdx_grad_norm": (i32, [i32, vp, f32, vp, vp, vp, sz, vp]),
    "mmdx_scale_grads": (i32, [i32, vp, vp, vp]),
    "mmdx_adamw_patch_grads": (i32, [i32, vp, vp, i32, vp, vp]),
    "mmdx_grad_norm_amp": (i32, [i32, vp, f32, vp, i32, vp, vp, vp, vp, sz, vp]),
    "mmdx_adamw_multi_amp": (i32, [i32, vp, f32, f32, f32, vp, vp, vp, vp]),
    "mmdx_amp_update_scale": (i32, [vp, vp, vp, f32, f32, i32, vp]),
    "mmdx_mul_dev_scalar": (i32, [vp, i64, vp, vp, vp]),
}

_lib = None
_lock = threading.Lock()


class MmdxLibraryError(RuntimeError):
    pass


def lib():
    """Load libmmdx_hip.so once; raise loudly if it is absent (no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise MmdxLibraryError(
                f"libmmdx_hip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        h = C.CDLL(LIB_PATH)
        missing = []
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(h, name)
            except AttributeError:
                missing.append(name)
                continue
            fn.restype = res
            fn.argtypes = args
        h.mmdx_missing_symbols = missing
        _lib = h
    return _lib


def reload_config():
    """Re-read the MMDX_* launch-heuristic knobs (the library reads them once per process):
    for tests / A-B runs that change one with os.environ between launches."""
    call("mmdx_reload_config")


def check(rc: int, name: str):
    if rc != 0:
        msg = lib().mmdx_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (rc={rc}): {msg}")


def call(name: str, *args):
    """Invoke a C-ABI entry point and raise RuntimeError on a non-zero return code."""
    fn = getattr(lib(), name)
    rc = fn(*args)
    if fn.restype is i32 and name not in ("mmdx_version",):
        check(rc, name)
    return rc


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float16:
        return F16   # the C5 path (GEMM, attention, norms, ViT / BERT kernels)
    raise TypeError(f"mmdx kernels compute in float32, bfloat16 or float16, got {dt}")


_RNG_COUNTERS: dict = {}


def rng_counter(device) -> torch.Tensor:
    """Per-device uint64 dropout counter (int64 storage) advanced on the GPU by every dropout
    launch, so RNG state lives on the device and graph replays draw fresh masks."""
    key = (device.type, device.index)
    t = _RNG_COUNTERS.get(key)
    if t is None:
        t = _RNG_COUNTERS[key] = torch.zeros(1, dtype=torch.int64, device=device)
    return t


def dropout_seed(base: int) -> int:
    """Host seed of a dropout launch: the call site's constant mixed with torch's initial
    seed and, under torch.distributed, the process rank — so data-parallel replicas draw
    independent masks (as one process's nn.Dropout over the global batch would), while a
    given (seed, rank) stays reproducible and graph-replayable (the per-launch counter
    lives on the device, rng_counter)."""
    rank = 0
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            rank = dist.get_rank()
    except Exception:  # pragma: no cover
        rank = 0
    x = (base ^ (torch.initial_seed() * 0x9E3779B97F4A7C15) ^ (rank * 0xBF58476D1CE4E5B9))
    return x & 0xFFFFFFFFFFFFFFFF


def workspace(nbytes: int, device) -> torch.Tensor | None:
    if nbytes <= 0:
        return None
    return torch.empty(int(nbytes), dtype=torch.uint8, device=device)


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "mmdx ops run only on the GPU (HIP); got a CPU tensor. Move the model and "
                "inputs to 'cuda' — there is no CPU fallback.")
        if not t.is_contiguous():
            raise RuntimeError("mmdx ops need contiguous tensors")
