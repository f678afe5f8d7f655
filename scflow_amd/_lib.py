"""ctypes binding of libscflow_hip.so (the C ABI declared in include/scflow_hip.h).

The library is loaded AFTER torch, so its ``libamdhip64.so.7`` dependency resolves to the HIP
runtime torch already loaded (same SONAME): one HIP runtime per process, and the ``hipStream_t``
handles torch hands out are valid here.  There is no fallback: if the library is missing the
product path raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library is loaded)

LIB_PATH = os.environ.get("SCFLOW_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                       "lib", "libscflow_hip.so")

c_int, c_float, c_ll, c_vp = ctypes.c_int, ctypes.c_float, ctypes.c_longlong, ctypes.c_void_p

SCFLOW_ACT = {None: 0, "ReLU": 1, "Sigmoid": 2, "Tanh": 3}
EPI_PLAIN, EPI_GRU_ZR, EPI_GRU_Q = 0, 1, 2
CONV_WINO = 2  # scflow_conv_args.bk: Winograd F(2x2,3x3) packing/kernel (SCFLOW_CONV_WINO)
CONV_1X1W = 3  # scflow_conv_args.bk: wide 1x1 packing/kernel (SCFLOW_CONV_1X1W)
CONV_WINO4 = 4  # scflow_conv_args.bk: Winograd F(4x4,3x3) packing/kernel (SCFLOW_CONV_WINO4)
LAYOUT_NCHW, LAYOUT_NHWC = 0, 1
ABI_VERSION = 3  # SCFLOW_ABI_VERSION of include/scflow_hip.h this binding mirrors


class ConvArgs(ctypes.Structure):
    """Mirror of ``scflow_conv_args`` (include/scflow_hip.h)."""
    _fields_ = [
        ("src0", c_vp), ("c0", c_int), ("s0", c_int),
        ("src1", c_vp), ("c1", c_int), ("s1", c_int),
        ("weight", c_vp), ("bias", c_vp),
        ("out", c_vp), ("so", c_int),
        ("n", c_int), ("h", c_int), ("w", c_int),
        ("cout", c_int), ("kh", c_int), ("kw", c_int), ("ph", c_int), ("pw", c_int), ("stride", c_int),
        ("act", c_int), ("epilogue", c_int),
        ("gate", c_vp), ("sg", c_int),
        ("rh", c_vp), ("srh", c_int),
        ("hid", c_vp), ("sh", c_int),
        ("bias_map", c_vp), ("sbm", c_int),
        ("bk", c_int),
        ("in_scale", c_vp), ("in_shift", c_vp),
        ("out_scale", c_vp), ("out_shift", c_vp),
        ("res", c_vp), ("sres", c_int),
        ("ws", c_vp), ("ws_bytes", ctypes.c_longlong),
    ]


class EncConvArgs(ctypes.Structure):
    """Mirror of ``scflow_enc_conv_args`` (include/scflow_hip.h)."""
    _fields_ = [
        ("src", c_vp), ("cin", c_int), ("s_in", c_int),
        ("src1", c_vp), ("cin1", c_int), ("s_in1", c_int),
        ("ksplit", c_int),
        ("in_scale", c_vp), ("in_shift", c_vp),
        ("weight", c_vp), ("bias", c_vp),
        ("out_scale", c_vp), ("out_shift", c_vp),
        ("res", c_vp), ("s_res", c_int),
        ("out", c_vp), ("s_out", c_int),
        ("n", c_int), ("h", c_int), ("w", c_int), ("cout", c_int), ("kh", c_int), ("kw", c_int),
        ("stride", c_int), ("pad", c_int),
        ("act", c_int), ("act2", c_int), ("act_split", c_int),
    ]


class WgradArgs(ctypes.Structure):
    """Mirror of ``scflow_wgrad_args`` (include/scflow_hip.h)."""
    _fields_ = [
        ("dy", c_vp), ("sdy", c_int),
        ("src0", c_vp), ("cin0", c_int), ("s0", c_int),
        ("src1", c_vp), ("cin1", c_int), ("s1", c_int),
        ("dw", c_vp), ("db", c_vp),
        ("workspace", c_vp), ("workspace_floats", c_ll),
        ("n", c_int), ("h", c_int), ("w", c_int), ("cout", c_int), ("kh", c_int), ("kw", c_int),
        ("stride", c_int), ("ph", c_int), ("pw", c_int),
        ("accumulate", c_int),
    ]


class RenderArgs(ctypes.Structure):
    """Mirror of ``scflow_render_args`` (include/scflow_hip.h)."""
    _fields_ = [
        ("verts", c_vp), ("normals", c_vp), ("colors", c_vp), ("faces", c_vp),
        ("vert_img", c_vp), ("face_img", c_vp),
        ("R", c_vp), ("t", c_vp), ("K", c_vp),
        ("n_img", c_int), ("size", c_int), ("total_verts", c_int), ("total_faces", c_int),
        ("light_mode", c_int),
        ("light_location", c_vp), ("ambient", c_vp), ("diffuse", c_vp), ("specular", c_vp),
        ("shininess", c_float),
        ("background", c_vp),
        ("images", c_vp), ("zbuf", c_vp), ("pix_to_face", c_vp), ("bary", c_vp),
        ("workspace", c_vp), ("workspace_bytes", c_ll), ("light_out", c_vp),
    ]


SCFLOW_LIGHT_FIXED, SCFLOW_LIGHT_PER_IMAGE, SCFLOW_LIGHT_BATCH_ZNEAR = 0, 1, 2

# name -> (restype, argtypes); every function the header declares
SIGNATURES = {
    "scflow_version": (c_int, []),
    "scflow_strerror": (ctypes.c_char_p, [c_int]),
    "scflow_corr_pyramid_size": (c_ll, [c_int, c_int, c_int, c_int]),
    "scflow_corr_pyramid": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_corr_lookup": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                   c_int, c_vp]),
    "scflow_corr_lookup_ex": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_int, c_int, c_vp]),
    "scflow_corr_pyramid_tiled": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_corr_lookup_conv1x1": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                           c_int, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_corr_lookup_conv1x1_lds_bytes": (c_ll, []),
    "scflow_corr_lookup_tiled": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int,
                                         c_int, c_int, c_int, c_vp]),
    "scflow_in_apply": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_colsum": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp]),
    "scflow_colsum_workspace": (c_int, [c_int, c_int]),
    "scflow_in_apply_residual": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "scflow_in_backward_residual": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_int, c_int, c_int, c_int, c_vp]),
    "scflow_in_backward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                                   c_int, c_int, c_vp]),
    "scflow_bn_forward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp, c_ll, c_int, c_int, c_float, c_float, c_int, c_vp]),
    "scflow_bn_backward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_vp, c_ll, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_debug_lookup_stamps": (c_int, [c_vp]),
    "scflow_debug_conv_stamps": (c_int, [c_vp]),
    "scflow_debug_reload_switches": (c_int, []),
    "scflow_abi_version": (c_int, []),
    "scflow_conv_args_size": (c_ll, []),
    "scflow_conv_packed_size": (c_ll, [c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "scflow_conv_packed_size_bk": (c_ll, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "scflow_conv_pack_weights": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                         c_int, c_vp]),
    "scflow_conv_pick_bk": (c_int, [ctypes.POINTER(ConvArgs)]),
    "scflow_conv_workspace_bytes": (ctypes.c_longlong, [ctypes.POINTER(ConvArgs)]),
    "scflow_conv2d": (c_int, [ctypes.POINTER(ConvArgs), c_vp]),
    "scflow_conv2d_pair": (c_int, [ctypes.POINTER(ConvArgs), ctypes.POINTER(ConvArgs), c_vp]),
    "scflow_xhead_pred_workspace_bytes": (c_ll, [c_int, c_int, c_int, c_int, c_int]),
    "scflow_xhead_pred": (c_int, [ctypes.POINTER(ConvArgs), c_int, c_vp, c_vp, c_ll, c_vp, c_vp, c_int,
                                  c_int, c_vp, c_int, c_vp, c_int, c_vp]),
    "scflow_pose_update": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_float, c_int, c_vp]),
    "scflow_lift_points": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "scflow_pose_flow": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_vp]),
    "scflow_pose_update_flow": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                        c_int, c_int, c_float, c_int, c_float, c_vp]),
    "scflow_flow_downsample": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int,
                                       c_int, c_float, c_vp]),
    "scflow_flow_upsample": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                     c_float, c_vp]),
    "scflow_pose_step": (c_int, [c_vp] * 9 + [c_int, c_int, c_int, c_float, c_int, c_float] +
                         [c_vp] * 6 + [c_int, c_vp, c_int, c_int, c_int, c_float, c_float, c_vp]),
    "scflow_pose_step_part": (c_int, [c_vp] * 9 + [c_int, c_int, c_int, c_float, c_int, c_float] +
                              [c_vp] * 6 + [c_int, c_vp, c_int, c_int, c_int, c_float, c_float, c_int,
                                            c_vp]),
    "scflow_pose_step_heads": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                       c_int, c_vp, c_vp] + [c_vp] * 7 +
                               [c_int, c_int, c_int, c_float, c_int, c_float] + [c_vp] * 6 +
                               [c_int, c_vp, c_int, c_int, c_int, c_float, c_float, c_int, c_vp]),
    "scflow_sync_event_create": (c_int, [ctypes.POINTER(c_vp)]),
    "scflow_sync_event_destroy": (c_int, [c_vp]),
    "scflow_sync_event_record": (c_int, [c_vp, c_vp]),
    "scflow_stream_wait_event": (c_int, [c_vp, c_vp]),
    "scflow_timing_event_create": (c_int, [ctypes.POINTER(c_vp)]),
    "scflow_event_elapsed_ms": (c_int, [c_vp, c_vp, ctypes.POINTER(c_float)]),
    "scflow_transpose": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_ll, c_int, c_ll, c_int, c_vp]),
    "scflow_ph_conv_packed_size": (c_ll, [c_int, c_int, c_int, c_int]),
    "scflow_ph_conv_pack": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_ph_conv": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_ph_conv_split": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_int, c_vp]),
    "scflow_ph_fc_split": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                                   c_vp, c_int, c_vp, c_vp]),
    "scflow_ph_heads_sum": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp,
                                    c_vp, c_int, c_vp, c_vp, c_vp]),
    "scflow_ph_fc_sum": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int,
                                 c_vp]),
    "scflow_ph_gn_stats": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_float, c_vp, c_vp,
                                   c_vp]),
    "scflow_ph_gn_reduce": (c_int, [c_vp, c_int, c_ll, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp,
                                    c_float, c_vp, c_vp, c_vp]),
    "scflow_ph_fc_permute": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "scflow_ph_fc": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                             c_vp, c_vp]),
    "scflow_ph_heads": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp,
                                c_vp, c_vp]),
    "scflow_enc_conv_packed_size": (c_ll, [c_int, c_int, c_int, c_int]),
    "scflow_enc_conv_pack": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_enc_conv": (c_int, [ctypes.POINTER(EncConvArgs), c_vp]),
    "scflow_enc_stem_packed_size": (c_ll, [c_int, c_int, c_int, c_int]),
    "scflow_enc_stem_pack": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_enc_stem": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                c_int, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_enc_stats": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "scflow_enc_norm_finalize": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_float, c_vp, c_vp, c_vp]),
    "scflow_enc_apply": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "scflow_render_workspace": (c_ll, [c_int, c_int, c_int]),
    "scflow_render": (c_int, [ctypes.POINTER(RenderArgs), c_vp]),
    "scflow_conv_wgrad_workspace": (c_int, [ctypes.POINTER(WgradArgs), ctypes.POINTER(c_ll)]),
    "scflow_conv_wgrad": (c_int, [ctypes.POINTER(WgradArgs), c_vp]),
    "scflow_conv_wgrad_batched": (c_int, [ctypes.POINTER(WgradArgs), c_int, c_vp, c_vp, c_vp, c_vp]),
    "scflow_im2col": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_vp]),
    "scflow_im2col_ex": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_int, c_int, c_vp]),
    "scflow_pose_update6_train": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          c_int, c_float, c_int, c_int, c_int, c_vp]),
    "scflow_pm_loss": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_int, c_int, c_float, c_vp]),
    "scflow_pm_loss_backward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_int, c_int, c_float, c_vp]),
    "scflow_up_l1_loss": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_float,
                                  c_vp, c_float, c_float, c_vp, c_vp, c_vp, c_vp]),
    "scflow_knn1": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "scflow_group_norm_forward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                          c_float, c_int, c_vp]),
    "scflow_group_norm_backward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "scflow_gru_gate_forward": (c_int, [c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_vp]),
    "scflow_gru_gate_backward_q": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_ll, c_int, c_vp]),
    "scflow_gru_gate_backward_r": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                           c_ll, c_int, c_vp]),
    "scflow_col2im": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_vp]),
    "scflow_corr_lookup_backward": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int,
                                            c_int, c_int, c_vp]),
    "scflow_gemm_f32_splits": (c_int, [c_int, c_int, c_int, c_int]),
    "scflow_gemm_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int] + [c_ll] * 9 +
                        [c_float, c_float, c_int, c_int, c_vp, c_vp]),
    "scflow_timestamp": (c_int, [c_vp, c_int, c_vp]),
    "scflow_wallclock_khz": (c_ll, []),
}

_lib = None

# Weight-derived caches (packed / flipped / affine forms) are keyed by (data_ptr, _version) of
# the weights AND by this generation: an update that does not move the version counters — a
# replayed hipGraph of the optimizer step (TrainStep(graph=True)) writes the parameters without
# autograd seeing it — bumps the generation so every cache re-derives its forms.
_WEIGHTS_GEN = 0


def weights_generation() -> int:
    return _WEIGHTS_GEN


def bump_weights_generation() -> None:
    global _WEIGHTS_GEN
    _WEIGHTS_GEN += 1


class ScflowError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load (once) and return the library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise ScflowError(
                f"HIP library not found at {path}: build it with `python -m scflow_amd.build` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver, size = lib.scflow_abi_version(), lib.scflow_conv_args_size()
        if ver != ABI_VERSION or size != ctypes.sizeof(ConvArgs):
            raise ScflowError(f"{path}: ABI version {ver} / sizeof(scflow_conv_args) {size}, this "
                              f"binding expects {ABI_VERSION} / {ctypes.sizeof(ConvArgs)}: rebuild "
                              "the library (python -m scflow_amd.build)")
        _lib = lib
    return _lib


def reload_switches() -> None:
    """Make the library re-read its cached launch-time switches (SCFLOW_WINO4_DEPTH,
    SCFLOW_GNR_CB, SCFLOW_SMALLCIN_SPLIT, SCFLOW_SMALLCIN_WGS) after os.environ changed."""
    check(load().scflow_debug_reload_switches(), "scflow_debug_reload_switches")


def check(code: int, what: str) -> None:
    if code != 0:
        msg = load().scflow_strerror(code)
        raise ScflowError(f"{what} failed with code {code}: {msg.decode() if msg else '?'}")
