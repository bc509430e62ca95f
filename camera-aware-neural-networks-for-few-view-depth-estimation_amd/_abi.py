"""ctypes binding of include/cad/cad.h (libcad_hip.so, built in-tree for gfx950).

This is the ONLY way the Python host reaches device code: there is no CPU fallback.  If the shared
library is missing the import fails loudly (run `make -C <package dir>` or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# CAD_LIB selects an A/B variant build (make VARIANT=... -> libcad_hip_<variant>.so) for tuning runs
LIB_PATH = os.path.join(PKG_DIR, os.environ.get("CAD_LIB", "libcad_hip.so"))
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "cad", "cad.h")

P = C.c_void_p
F = C.c_float
I = C.c_int
I64 = C.c_int64
FP = C.POINTER(C.c_float)
I64P = C.POINTER(C.c_int64)


class UnetDesc(C.Structure):
    _fields_ = [("in_channels", I), ("init_features", I), ("max_depth", F), ("max_batch", I),
                ("height", I), ("width", I)]


class ResUnetDesc(C.Structure):
    _fields_ = [("in_channels", I), ("max_batch", I), ("height", I), ("width", I), ("max_depth", F)]


class GeoNetDesc(C.Structure):
    _fields_ = [("variant", I), ("in_channels", I), ("init_features", I), ("camera_dim", I), ("max_depth", F),
                ("use_pcl", I), ("use_attention", I), ("max_batch", I), ("height", I), ("width", I)]


class AdamOpts(C.Structure):
    _fields_ = [("lr", F), ("beta1", F), ("beta2", F), ("eps", F), ("weight_decay", F)]


class CommStats(C.Structure):
    """cad_comm_stats (cad.h): exchange accounting of the overlapped backward all-reduce."""
    _fields_ = [("calls", I64), ("timed_calls", I64), ("buckets", I64), ("bytes", I64), ("exposed_ms", C.c_double),
                ("span_ms", C.c_double)]


class ArchiveEntry(C.Structure):
    """cad_archive_entry (cad.h): one tensor / empty submodule of a torch::save archive."""
    _fields_ = [("name", C.c_char_p), ("kind", I), ("dtype", I), ("ndim", I), ("shape", C.c_int64 * 8),
                ("data", C.c_void_p)]


# name: (restype, argtypes)
SIGNATURES = {
    "cad_abi_version": (I, []),
    "cad_last_error": (C.c_char_p, []),
    "cad_device_count": (I, [C.POINTER(I)]),
    "cad_set_device": (I, [I]),
    "cad_stream_synchronize": (I, [P]),
    "cad_malloc": (I, [I, I64, C.POINTER(P)]),
    "cad_free": (None, [P]),
    "cad_memcpy": (I, [P, P, I64, I, P]),
    "cad_adam_state": (I, [P, C.POINTER(P), C.POINTER(P)]),
    "cad_adam_set_step_count": (I, [P, I64]),
    "cad_set_gemm_engine": (I, [I]),
    "cad_set_alias_check": (I, [I]),
    "cad_alias_views_overlap": (I, [P, I64, I64, I64, I64, I, P, I64, I64, I64, I64, I]),
    "cad_get_gemm_engine": (I, []),
    "cad_unet_create": (I, [C.POINTER(UnetDesc), I, C.POINTER(P)]),
    "cad_resunet_create": (I, [C.POINTER(ResUnetDesc), I, C.POINTER(P)]),
    "cad_resunet_destroy": (None, [P]),
    "cad_resunet_count_parameters": (I64, [P]),
    "cad_resunet_num_tensors": (I, [P, I]),
    "cad_resunet_tensor_info": (I, [P, I, I, C.POINTER(C.c_char_p), C.POINTER(I), I64P]),
    "cad_resunet_set_tensor": (I, [P, I, I, FP, I64]),
    "cad_resunet_get_tensor": (I, [P, I, I, FP, I64]),
    "cad_resunet_get_grad": (I, [P, I, FP, I64]),
    "cad_resunet_train": (I, [P, I]),
    "cad_resunet_set_fp8": (I, [P, I]),
    "cad_resunet_fp8_units": (I, [P]),
    "cad_resunet_flat": (I, [P, C.POINTER(P), C.POINTER(P), I64P]),
    "cad_resunet_forward": (I, [P, P, P, I, P]),
    "cad_resunet_backward": (I, [P, P, P]),
    "cad_resunet_num_stages": (I, [P]),
    "cad_resunet_debug_buffer": (I64, [P, C.c_char_p, FP, I64]),
    "cad_resunet_grad_layout": (I, [C.POINTER(I), I64P, I64P, I64P]),
    "cad_resunet_stage_grad_range": (I, [P, I, I64P, I64P]),
    "cad_resunet_backward_stage": (I, [P, I, P, P]),
    "cad_resunet_backward_allreduce": (I, [P, P, P, I64, P]),
    "cad_resunet_clip_grad_norm": (I, [P, F, F, P]),
    "cad_resunet_last_grad_norm": (I, [P, FP, P]),
    "cad_resunet_adam_step": (I, [P, F, F, F, F, F, P]),
    "cad_geonet_create": (I, [C.POINTER(GeoNetDesc), I, C.POINTER(P)]),
    "cad_geonet_destroy": (None, [P]),
    "cad_geonet_count_parameters": (I64, [P]),
    "cad_geonet_num_tensors": (I, [P, I]),
    "cad_geonet_tensor_info": (I, [P, I, I, C.POINTER(C.c_char_p), C.POINTER(I), I64P]),
    "cad_geonet_set_tensor": (I, [P, I, I, FP, I64]),
    "cad_geonet_get_tensor": (I, [P, I, I, FP, I64]),
    "cad_geonet_get_grad": (I, [P, I, FP, I64]),
    "cad_geonet_train": (I, [P, I]),
    "cad_geonet_flat": (I, [P, C.POINTER(P), C.POINTER(P), I64P]),
    "cad_geonet_forward": (I, [P, P, P, P, P, I, P]),
    "cad_geonet_backward": (I, [P, P, P]),
    "cad_geonet_num_stages": (I, [P]),
    "cad_geonet_grad_layout": (I, [C.POINTER(GeoNetDesc), C.POINTER(I), I64P, I64P, I64P]),
    "cad_geonet_stage_grad_range": (I, [P, I, I64P, I64P]),
    "cad_geonet_backward_stage": (I, [P, I, P, P]),
    "cad_geonet_backward_allreduce": (I, [P, P, P, I64, P]),
    "cad_geonet_clip_grad_norm": (I, [P, F, F, P]),
    "cad_geonet_last_grad_norm": (I, [P, FP, P]),
    "cad_geonet_adam_step": (I, [P, F, F, F, F, F, P]),
    "cad_geonet_num_batches_tracked": (I64, [P, I]),
    "cad_geonet_debug_buffer": (I64, [P, C.c_char_p, FP, I64]),
    "cad_op_cbam": (I, [P, P, P, I, I, I, I, P, P, P, P]),
    "cad_op_pcl": (I, [P, P, P, P, I, I, I, I, P, P, P, P, P]),
    "cad_unet_create_model": (I, [C.POINTER(UnetDesc), I, I, C.POINTER(P)]),
    "cad_unet_model": (I, [P]),
    "cad_unet_forward_cam": (I, [P, P, P, P, I, P]),
    "cad_camera_from_K": (I, [P, I, P, P]),
    "cad_unet_destroy": (None, [P]),
    "cad_unet_count_parameters": (I64, [P]),
    "cad_unet_num_params": (I, [P]),
    "cad_unet_num_buffers": (I, [P]),
    "cad_unet_tensor_info": (I, [P, I, I, C.POINTER(C.c_char_p), C.POINTER(I), I64P]),
    "cad_unet_set_tensor": (I, [P, I, I, FP, I64]),
    "cad_unet_get_tensor": (I, [P, I, I, FP, I64]),
    "cad_unet_get_grad": (I, [P, I, FP, I64]),
    "cad_unet_train": (I, [P, I]),
    "cad_unet_flat": (I, [P, C.POINTER(P), C.POINTER(P), I64P]),
    "cad_unet_use_external_slabs": (I, [P, P, P]),
    "cad_unet_forward": (I, [P, P, P, I, P]),
    "cad_unet_backward": (I, [P, P, P]),
    "cad_unet_num_stages": (I, [P]),
    "cad_unet_backward_stage": (I, [P, I, P, P]),
    "cad_unet_stage_grad_range": (I, [P, I, I64P, I64P]),
    "cad_clip_grad_norm": (I, [P, F, F, P]),
    "cad_unet_last_grad_norm": (I, [P, FP, P]),
    "cad_adam_create": (I, [P, C.POINTER(AdamOpts), C.POINTER(P)]),
    "cad_adam_destroy": (None, [P]),
    "cad_adam_step": (I, [P, P]),
    "cad_adam_set_lr": (I, [P, F]),
    "cad_adam_step_count": (I64, [P]),
    "cad_loss_create": (I, [F, F, F, F, I, I, I, I, C.POINTER(P)]),
    "cad_loss_destroy": (None, [P]),
    "cad_loss_forward_backward": (I, [P, P, P, P, P, I, P, P, P]),
    "cad_loss_get_components": (I, [P, FP, P]),
    "cad_depth_metrics": (I, [P, P, I, I, I, FP, P]),
    "cad_ray_directions": (I, [P, I, I, I, P, P]),
    "cad_unet_debug_buffer": (I64, [P, C.c_char_p, FP, I64]),
    "cad_profile_enable": (I, [I]),
    "cad_profile_reset": (I, []),
    "cad_profile_only": (I, [C.c_char_p]),
    "cad_profile_report": (I, [C.c_char_p, I]),
    "cad_op_conv3x3_fwd": (I, [P, I64, I, I, P, I, P, I64, I, I, I, I, P]),
    "cad_op_conv3x3_dgrad": (I, [P, I, P, I, P, I64, I, I, I, P]),
    "cad_op_conv3x3_wgrad": (I, [P, I, P, I64, I, I, P, I, I, I, P]),
    "cad_op_conv3x3_wgrad_bf16": (I, [P, I64, I, P, I64, I, I, P, I, I, I, P]),
    "cad_op_conv3x3_fwd_bf16": (I, [P, I64, I, I, P, I, P, I64, I, I, I, I, I, I, P]),
    "cad_op_conv3x3_dgrad_bf16": (I, [P, I64, I, P, I, P, I64, I, I, I, I, P]),
    "cad_op_mx8_quantize": (I, [P, I, I64, I, I, I64, P, P, I64, I, P]),
    "cad_op_dense_x8": (I, [P, P, I64, I, P, P, I64, I, P, I64, P]),
    "cad_op_conv3x3_x8": (I, [P, P, I64, I, P, P, I64, I, P, I, I, I, P]),
    "cad_op_convT_fwd": (I, [P, I, P, P, I, P, I64, I, I, I, I, P]),
    "cad_op_convT_fwd_bf16": (I, [P, I64, I, I, P, P, I, P, I64, I, I, I, I, P]),
    "cad_op_convT_dgrad": (I, [P, I64, I, I, P, I, P, I, I, I, P]),
    "cad_op_convT_wgrad": (I, [P, I, P, I64, I, I, P, I, I, I, P]),
    "cad_op_maxpool_fwd": (I, [P, I64, I, I, I, I, P, P, P]),
    "cad_batcher_create": (I, [I, I, I, I, C.POINTER(P)]),
    "cad_batcher_destroy": (None, [P]),
    "cad_batcher_assemble": (I, [P, C.c_void_p, I, P, P, P, P]),
    "cad_aug_sampler_create": (I, [C.c_void_p, C.c_uint32, C.POINTER(P)]),
    "cad_aug_sampler_destroy": (None, [P]),
    "cad_aug_sampler_draw": (I, [P, I, I, C.c_void_p]),
    "cad_loss_forward_backward_masked": (I, [P, P, P, P, P, P, I, P, P, P]),
    "cad_comm_get_unique_id": (I, [C.c_void_p]),
    "cad_comm_create": (I, [C.c_void_p, I, I, I, C.POINTER(P)]),
    "cad_comm_destroy": (None, [P]),
    "cad_comm_rank": (I, [P]),
    "cad_comm_size": (I, [P]),
    "cad_comm_set_timing": (I, [P, I]),
    "cad_comm_stats_read": (I, [P, P]),
    "cad_comm_allreduce": (I, [P, P, I64, I, P]),
    "cad_comm_broadcast": (I, [P, P, I64, I, P]),
    "cad_comm_broadcast_params": (I, [P, P, I, P]),
    "cad_grad_allreduce": (I, [P, P, P]),
    "cad_unet_backward_allreduce": (I, [P, P, P, I64, P]),
    "cad_plan_grad_buckets": (I, [I64P, I64P, I, I64, I64P, I64P, C.POINTER(I)]),
    "cad_model_grad_layout": (I, [I, I, I, C.POINTER(I), I64P, I64P, I64P]),
    "cad_unet_save_torch": (I, [P, C.c_char_p]),
    "cad_unet_load_torch": (I, [P, C.c_char_p]),
    "cad_unet_num_batches_tracked": (I64, [P]),
    "cad_archive_write": (I, [C.c_char_p, C.POINTER(ArchiveEntry), I]),
    "cad_archive_open": (I, [C.c_char_p, C.POINTER(P)]),
    "cad_archive_close": (None, [P]),
    "cad_archive_count": (I, [P]),
    "cad_archive_find": (I, [P, C.c_char_p]),
    "cad_archive_info": (I, [P, I, C.POINTER(C.c_char_p), C.POINTER(I), C.POINTER(I), I64P]),
    "cad_archive_read": (I, [P, I, P, I64]),
    "cad_dataset_open": (I, [C.c_char_p, C.POINTER(C.c_char_p), I, C.POINTER(P)]),
    "cad_dataset_synthetic": (I, [I64, I, I, C.c_uint32, C.POINTER(P)]),
    "cad_jpeg_decode": (I, [P, I64, P, I64, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "cad_dataset_destroy": (None, [P]),
    "cad_dataset_size": (I64, [P]),
    "cad_dataset_image_dir": (C.c_char_p, [P, I64]),
    "cad_dataset_read": (I, [P, I64, P, I64, P, I64, P]),
    "cad_loader_create": (I, [P, I, I, I, P, C.c_uint32, I, I, I, C.POINTER(P)]),
    "cad_loader_destroy": (None, [P]),
    "cad_loader_start_epoch": (I, [P, I64P, I64]),
    "cad_loader_next": (I, [P, P, P, P, P]),
}


class Sample(C.Structure):
    """cad_sample (cad.h): one decoded sample and its augmentation parameters."""
    _fields_ = [("rgb", P), ("depth", P), ("h0", I), ("w0", I), ("bgr", I), ("depth_scale", F),
                ("K", F * 9), ("aug", I), ("crop", I), ("crop_scale", F), ("crop_x", I), ("crop_y", I),
                ("flip", I), ("jitter", I), ("brightness", F), ("contrast", F), ("dh0", I), ("dw0", I)]


class DecodedInfo(C.Structure):
    """cad_decoded_info (cad.h)."""
    _fields_ = [("h0", I), ("w0", I), ("dh0", I), ("dw0", I), ("depth_scale", F), ("K", F * 9)]


class AugConfig(C.Structure):
    """cad_aug_config = AugmentationConfig (sunrgbd_loader.h:30-42), defaults as there."""
    _fields_ = [("enable_random_crop", I), ("crop_scale_min", F), ("crop_scale_max", F),
                ("enable_horizontal_flip", I), ("horizontal_flip_prob", F), ("enable_color_jitter", I),
                ("brightness_delta", F), ("contrast_delta", F)]

    def __init__(self, **kw):
        d = dict(enable_random_crop=1, crop_scale_min=0.7, crop_scale_max=1.0, enable_horizontal_flip=1,
                 horizontal_flip_prob=0.5, enable_color_jitter=1, brightness_delta=0.2, contrast_delta=0.2)
        d.update(kw)
        super().__init__(**d)


class CadError(RuntimeError):
    pass


def header_functions(path: str = HEADER):
    """Every function name declared in include/cad/cad.h."""
    with open(path) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cad_[A-Za-z0-9_]+)\s*\(", text)))


_lib = None


def load():
    """Load libcad_hip.so (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libcad_hip.so not built at {LIB_PATH}: run `make -C {PKG_DIR}` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if "CAD_LIB" in os.environ:   # an older A/B variant build (tools/ab_step.py): no such entry point
                continue
            raise AttributeError(f"{LIB_PATH} does not export {name} (stale build? run make)")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str = ""):
    if status != 0:
        msg = load().cad_last_error().decode(errors="replace")
        raise CadError(f"{what} failed (status {status}): {msg}")
