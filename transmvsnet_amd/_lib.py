"""ctypes binding of the C-ABI in include/transmvs.h (libtransmvs_hip.so, built in-tree).

There is no fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TMVS_LIB_PATH") or os.path.join(_HERE, "libtransmvs_hip.so")  # override: A/B experiments

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
S = ctypes.c_size_t
D = ctypes.c_double

# name -> (restype, argtypes); every symbol include/transmvs.h declares
SIGNATURES = {
    "tmvs_abi_version": (I, []),
    "tmvs_status_string": (ctypes.c_char_p, [I]),
    "tmvs_bn_fold": (I, [P, P, P, P, I, F, P, P]),
    "tmvs_stage_hypotheses": (I, [P, I, P, I, I, I, I, F, I, I, I, P, P]),
    "tmvs_warp_corr": (I, [P, P, P, P, P, I, I, I, P, I, I, I, I, I, I, I, P, P, P, P]),
    "tmvs_aggregate_finalize": (I, [P, P, I, I, I, I, P]),
    "tmvs_homo_warping": (I, [P, P, P, I, I, I, I, I, I, P, P]),
    "tmvs_costregnet_workspace": (S, [I, I, I, I, I]),
    "tmvs_costregnet": (I, [P, I, I, I, I, P, P, S, P, P]),
    "tmvs_costregnet_wta": (I, [P, P, I, I, I, I, P, P, S, F, F, P, P, P, P, P]),
    "tmvs_conv3d_bn_relu": (I, [P, I, I, I, I, I, P, P, P, I, I, P, P]),
    "tmvs_deconv3d_bn_relu_add": (I, [P, I, I, I, I, I, P, P, P, I, P, P, P]),
    "tmvs_softmax_wta": (I, [P, P, I, I, I, I, F, F, P, P, P, P, P]),
    "tmvs_fmt_embed": (I, [P, L, P, I, I, I, I, I, I, P, P]),
    "tmvs_fmt_kv_workspace": (S, [I, I]),
    "tmvs_fmt_kv": (I, [P, I, I, P, P, S, P, P]),
    "tmvs_fmt_apply": (I, [P, I, I, P, L, P, P]),
    "tmvs_fmt_pathway": (I, [P, P, L, P, P, I, I, I, I, I, P, P]),
    "tmvs_fmt_forward_workspace": (S, [I, I]),
    "tmvs_fmt_forward": (I, [P, L, P, I, I, I, I, I, P, P, S, P, P]),
    "tmvs_fmt_forward_split_workspace": (S, [I, I]),
    "tmvs_fmt_forward_split": (I, [P, L, P, I, I, I, I, I, P, P, S, P, P, P]),
    "tmvs_fmt_kv_grouped_workspace": (S, [I, I, I]),
    "tmvs_fmt_kv_grouped": (I, [P, I, I, I, P, P, S, P, P]),
    "tmvs_depth_stage_workspace": (S, [I, I, I, I]),
    "tmvs_depth_stage": (I, [P, I, P, I, I, P, I, I, I, F, I, I, I, P, P, P, I, I, P, P, S, F, F, P, P, P, P, P, P]),
    "tmvs_deform_conv2d_packed_floats": (S, [I]),
    "tmvs_deform_conv2d_pack": (I, [P, I, I, P]),
    "tmvs_deform_conv2d": (I, [P, P, P, P, P, P, I, I, I, I, I, I, P, P, P]),
    "tmvs_dcn_fused": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, P, P, P]),
    "tmvs_conv3x3_nhwc": (I, [P, P, P, P, P, I, I, I, I, I, I, P, P, P]),
    "tmvs_conv3x3_nhwc_acc": (I, [P, P, I, I, I, I, I, P, P]),
    "tmvs_fpn_merge": (I, [P, P, I, P, P, I, I, I, P, P]),
    "tmvs_conv2d_packed_floats": (S, [I, I, I]),
    "tmvs_conv2d_pack": (I, [P, I, I, I, P]),
    "tmvs_conv2d_bn_relu": (I, [P, I, I, I, I, P, I, I, I, P, P, I, P, P]),
    "tmvs_fusibile": (I, [P, P, I, I, I, I, I, F, P, P, P]),
    "tmvs_entropy_loss_workspace": (S, [I, I, I]),
    "tmvs_entropy_loss": (I, [P, P, I, P, P, I, I, I, I, F, P, S, P, P, P, P, P]),
    "tmvs_depth_metrics_workspace": (S, [I]),
    "tmvs_depth_metrics": (I, [P, P, P, I, F, P, S, P, P]),
    "tmvs_warp_corr_backward_workspace": (S, [I, I, I, I, I]),
    "tmvs_warp_corr_backward": (I, [P, P, P, P, P, I, I, I, I, I, I, P, S, P, P, P]),
    "tmvs_pixelwise_train_workspace": (S, []),
    "tmvs_pixelwise_train_forward": (I, [P, I, I, I, I, P, P, S, P, P, P, P]),
    "tmvs_aggregate_train": (I, [P, P, I, I, I, I, I, P, P, P]),
    "tmvs_aggregate_train_backward": (I, [P, P, P, P, P, I, I, I, I, I, P, P, P]),
    "tmvs_pixelwise_train_backward": (I, [P, I, I, I, I, P, P, P, P, P, P, S, P, P, P]),
    "tmvs_upsample2_add_nhwc": (I, [P, P, I, I, I, I, P, P]),
    "tmvs_upsample2_backward_nhwc": (I, [P, I, I, I, I, P, P]),
    "tmvs_token_linear": (I, [P, L, I, I, P, P, I, P, I, P, P]),
    "tmvs_token_linear_res": (I, [P, L, I, I, P, P, I, P, P, P, P]),
    "tmvs_token_wgrad_workspace": (S, [L, I, I]),
    "tmvs_token_wgrad": (I, [P, I, P, I, L, P, S, P, P, I, P]),
    "tmvs_layer_norm_fwd": (I, [P, L, P, P, P, P]),
    "tmvs_layer_norm_bwd_workspace": (S, [L]),
    "tmvs_layer_norm_bwd": (I, [P, P, L, P, P, S, P, P, I, P]),
    "tmvs_linattn_fwd": (I, [P, L, L, P, L, P, P]),
    "tmvs_linattn_bwd_workspace": (S, [L, L]),
    "tmvs_linattn_bwd_q": (I, [P, P, L, L, P, L, P, S, P, P, P]),
    "tmvs_linattn_bwd_kv": (I, [P, P, L, L, P, P, P, P]),
    "tmvs_adam_step": (I, [P, P, P, P, L, D, D, D, D, D, I, P]),
    "tmvs_adam_step_dev": (I, [P, P, P, P, L, D, P, D, D, D, D, P, P, P]),
    "tmvs_conv3d_generic": (I, [P, I, I, I, I, I, P, I, I, I, I, I, I, P, P]),
    "tmvs_conv3d_mfma": (I, [P, I, I, I, I, I, P, I, I, I, P, P, P]),
    "tmvs_conv3d_wgrad_workspace": (S, [I, I, I, I, I, I]),
    "tmvs_conv3d_wgrad": (I, [P, I, I, I, I, I, P, I, I, I, I, I, P, S, P, P]),
    "tmvs_bn_train_workspace": (S, [L, I]),
    "tmvs_bn_stats": (I, [P, L, I, P, S, P, P, P]),
    "tmvs_bn_relu_train": (I, [P, L, I, P, P, P, P, F, P, P, P]),
    "tmvs_bn_relu_backward": (I, [P, P, L, I, P, P, P, P, F, P, S, P, P, P, P]),
    "tmvs_bn_train_workspace_grouped": (S, [I, L, I]),
    "tmvs_bn_stats_grouped": (I, [P, I, L, I, P, S, P, P, P]),
    "tmvs_bn_relu_train_grouped": (I, [P, I, L, I, P, P, P, P, F, P, P, P]),
    "tmvs_bn_relu_backward_grouped": (I, [P, P, I, L, I, P, P, P, P, F, P, S, P, P, P, P]),
    "tmvs_conv2d_generic": (I, [P, I, I, I, I, P, P, I, I, I, I, I, I, I, P, P]),
    "tmvs_conv2d_wgrad_workspace": (S, [I, I, I, I, I, I]),
    "tmvs_conv2d_wgrad": (I, [P, I, I, I, I, P, I, I, I, I, I, I, P, S, P, P]),
    "tmvs_colsum_workspace": (S, [L, I]),
    "tmvs_colsum": (I, [P, L, I, P, S, P, P]),
    "tmvs_dcn_forward_train": (I, [P, P, P, P, P, I, I, I, I, I, P, P, P, P]),
    "tmvs_dcn_backward_workspace": (S, [I, I, I, I]),
    "tmvs_dcn_backward": (I, [P, P, P, P, I, I, I, I, I, P, S, P, P, P, P]),
    "tmvs_dcn_backward_set": (I, [P, P, P, P, I, I, I, I, I, P, S, P, P, P, P, P]),
    "tmvs_nearest_up2_backward_nhwc": (I, [P, I, I, I, I, I, P, P]),
    "tmvs_softmax_backward": (I, [P, P, I, I, I, I, P, P]),
}

ABI_VERSION = 9
PW_NPARAMS = 201
ENC_NPARAMS = 8544
KV_NFLOATS = 160
WARP_PARTIAL = 1
WARP_ROT_PLAIN = 2
WARP_BWD_PLANES = 4
CONV_TRANSPOSED = 1
CONV_ACCUMULATE = 2


class CostRegWeights(ctypes.Structure):
    """TmvsCostRegWeights (include/transmvs.h)."""
    _fields_ = [("w", P * 11), ("alpha", P * 10), ("shift", P * 10), ("base_ch", I)]


_lib = None


def load():
    """Load and type the library; raises RuntimeError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"transmvsnet_amd HIP extension not built ({LIB_PATH} missing): "
                           "run `python -m transmvsnet_amd.build`")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.tmvs_abi_version() != ABI_VERSION:
        raise RuntimeError("libtransmvs_hip.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def check(status: int, what: str):
    if status != 0:
        msg = load().tmvs_status_string(status).decode()
        raise RuntimeError(f"{what} failed: {msg} ({status})")
