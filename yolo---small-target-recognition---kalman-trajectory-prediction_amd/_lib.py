"""ctypes binding of libyk.so (include/yk.h).

torch is imported before the library is loaded so that libyk.so's libamdhip64.so.7
resolves to torch's bundled HIP runtime: one runtime, one device context, and torch
tensors' data_ptr() can be handed to yk calls directly.  There is no fallback: if the
library is missing or fails to load, every product entry point raises YKError.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np
import torch  # noqa: F401  (load order: torch's HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YK_LIB", os.path.join(_HERE, "libyk.so"))

YK_OK, YK_ERR_ARG, YK_ERR_HIP, YK_ERR_CAPACITY, YK_ERR_STATE = 0, 1, 2, 3, 4
YK_F32, YK_F64 = 0, 1
OP_PREDICT, OP_UPDATE, OP_MARK_LOST, OP_INFO, OP_LONG_TERM, OP_LOST_PRED = range(6)
TRAJ_OUT, VEL_HIST, TRAJ_HIST = 30, 50, 150


class YKError(RuntimeError):
    """A libyk.so call failed (message from yk_last_error(); .status = the yk_status code, or
    None when the error is raised on the Python side)."""

    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status


# ---------------------------------------------------------------- ABI structs
class TrackerCfg(C.Structure):
    _fields_ = [("max_lost_frames", C.c_int32), ("min_hits", C.c_int32), ("iou_threshold", C.c_double),
                ("max_tracks", C.c_int32), ("max_dets", C.c_int32), ("policy", C.c_int32)]


POLICY_ENHANCED, POLICY_MOTION_RESET = 0, 1


class BtCfg(C.Structure):
    """yk_bt_cfg (ByteTrack / BoT-SORT)."""
    _fields_ = [("kind", C.c_int32), ("track_high_thresh", C.c_float), ("track_low_thresh", C.c_float),
                ("new_track_thresh", C.c_float), ("match_thresh", C.c_float), ("track_buffer", C.c_int32),
                ("frame_rate", C.c_int32), ("fuse_score", C.c_int32), ("max_tracks", C.c_int32),
                ("max_dets", C.c_int32), ("assignment", C.c_int32), ("reserved", C.c_int32),
                ("match_thresh_f64", C.c_double)]


BT_BYTETRACK, BT_BOTSORT = 0, 1
BT_LAP, BT_SCIPY = 0, 1  # yk_bt_assignment

STATS_DTYPE = np.dtype([(k, np.int64) for k in (
    "frame_count", "next_track_id", "total_tracks_created", "total_tracks_terminated",
    "current_active_tracks", "long_term_predictions", "successful_recoveries", "overflow",
    "individual_resets", "tracking_recoveries", "global_motion_events", "global_resets")])

GMD_OPTICAL_FLOW, GMD_FEATURE_MATCHING, GMD_HYBRID, GMD_SPARSE_OPTFLOW = 0, 1, 2, 3
GMD_METHODS = {"optical_flow": GMD_OPTICAL_FLOW, "feature_matching": GMD_FEATURE_MATCHING, "hybrid": GMD_HYBRID}
# yk_track_event (include/yk.h): one record per work item of a step
TRACK_EVENT_DTYPE = np.dtype([("kind", np.int32), ("track_num", np.int32), ("list_pos", np.int32), ("det", np.int32),
                              ("lost_frames", np.int32), ("deleted_tsu", np.int32), ("iou", np.float64),
                              ("x", np.float64), ("y", np.float64), ("vx", np.float64), ("vy", np.float64),
                              ("confidence", np.float64)])
EV_NONE, EV_RECOVERED, EV_LOST, EV_CREATED = 0, 1, 2, 3

MOTION_DTYPE = np.dtype([("valid", np.int32), ("is_motion", np.int32), ("should_reset", np.int32),
                         ("magnitude_kind", np.int32), ("magnitude", np.float32), ("vector", np.float32, (2,)),
                         ("consistency", np.float32), ("n_corners", np.int32), ("n_tracked", np.int32),
                         ("n_inliers", np.int32), ("first_frame", np.int32)], align=True)
GMD_STATS_DTYPE = np.dtype([("total_detections", np.int64), ("motion_events", np.int64), ("reset_triggers", np.int64),
                            ("avg_motion_magnitude", np.float32), ("pad", np.int32)], align=True)

RESET_DETAIL_DTYPE = np.dtype([("frame", np.int32), ("reasons", np.int32), ("value", np.float64, (3,)),
                               ("confidence", np.float64), ("motion_consistency", np.float64)], align=True)

TRACK_OUT_DTYPE = np.dtype([
    ("track_num", np.int32), ("status", np.int32), ("age", np.int32), ("hits", np.int32),
    ("hit_streak", np.int32), ("time_since_update", np.int32), ("traj_len", np.int32),
    ("is_stable_motion", np.int32), ("bbox", np.float64, (4,)), ("confidence", np.float64),
    ("velocity", np.float64, (2,)), ("motion_confidence", np.float64), ("speed", np.float64),
    ("direction", np.float64), ("traj", np.float64, (TRAJ_OUT, 2)),
    ("reset_count", np.int32), ("frames_since_reset", np.int32), ("reason_count", np.int32, (3,)),
    ("n_details", np.int32), ("motion_consistency", np.float64), ("reset_confidence_sum", np.float64),
    ("motion_consistency_sum", np.float64), ("details", RESET_DETAIL_DTYPE, (5,)),
    ("traj_count", np.int32), ("reserved", np.int32)], align=True)

TRACK_STATE_DTYPE = np.dtype([
    ("track_num", np.int32), ("age", np.int32), ("hits", np.int32), ("hit_streak", np.int32),
    ("time_since_update", np.int32), ("is_lost", np.int32), ("lost_frames", np.int32),
    ("vel_len", np.int32), ("traj_len", np.int32), ("max_lost_frames", np.int32),
    ("x", np.float64, (8,)), ("P", np.float64, (8, 8)), ("velocity_avg", np.float64, (2,)),
    ("velocity_std", np.float64, (2,)), ("direction", np.float64), ("speed", np.float64),
    ("stability_score", np.float64), ("prediction_confidence", np.float64),
    ("vel_hist", np.float64, (VEL_HIST, 2)), ("traj_hist", np.float64, (TRAJ_HIST, 2)),
    ("reset_count", np.int32), ("last_reset_frame", np.int32), ("motion_consistency", np.float64)], align=True)

_vp = C.c_void_p
_i32 = C.c_int32
class Tensor(C.Structure):
    """yk_tensor: one named fp32 state-dict tensor (host memory)."""
    _fields_ = [("name", C.c_char_p), ("ndim", C.c_int32), ("shape", C.c_int64 * 4), ("data", C.c_void_p)]


class Weights(C.Structure):
    _fields_ = [("n", C.c_int32), ("tensors", C.POINTER(Tensor))]


def weights_struct(sd: dict):
    """(yk_weights, keep-alive list) for a state dict of torch tensors / numpy arrays: every
    floating tensor as contiguous fp32 (what the checkpoint loader's .float() gives)."""
    import numpy as np

    keep, items = [], []
    for k, v in sd.items():
        a = v.detach().cpu().float().numpy() if hasattr(v, "detach") else np.asarray(v)
        if a.dtype.kind != "f" or a.ndim > 4:
            continue
        a = np.ascontiguousarray(a, dtype=np.float32)
        name = k.encode()
        keep += [a, name]
        t = Tensor()
        t.name = name
        t.ndim = a.ndim
        for d in range(a.ndim):
            t.shape[d] = a.shape[d]
        t.data = a.ctypes.data
        items.append(t)
    arr = (Tensor * len(items))(*items)
    keep.append(arr)
    w = Weights(len(items), arr)
    return w, keep


_SIGS = {
    "yk_abi_version": ([], C.c_int),
    "yk_last_error": ([], C.c_char_p),
    "yk_struct_size": ([C.c_int], C.c_int64),
    "yk_ctx_create": ([C.c_int, C.POINTER(_vp)], C.c_int),
    "yk_ctx_destroy": ([_vp], C.c_int),
    "yk_tracker_create": ([_vp, C.c_int, C.POINTER(TrackerCfg), C.POINTER(_vp)], C.c_int),
    "yk_tracker_destroy": ([_vp], C.c_int),
    "yk_tracker_reset": ([_vp, _vp], C.c_int),
    "yk_tracker_step": ([_vp, _vp, C.c_int, C.c_int, _vp, _vp], C.c_int),
    "yk_tracker_outputs": ([_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp)], C.c_int),
    "yk_tracker_download": ([_vp, _vp, _vp, _vp, _vp], C.c_int),
    "yk_tracker_download_async": ([_vp, _vp, _vp, _vp, C.c_int, _vp], C.c_int),
    "yk_upload_pinned_async": ([_vp, _vp, C.c_size_t, _vp], C.c_int),
    "yk_tracker_snapshot": ([_vp, C.c_int, _vp, C.POINTER(_i32), _vp], C.c_int),
    "yk_track_op": ([_vp, C.c_int, C.c_int, C.c_int, C.c_int, _vp, C.c_int, _vp, _vp, _vp], C.c_int),
    "yk_track_create": ([_vp, C.c_int, _vp, C.c_int, _i32, _i32, _vp], C.c_int),
    "yk_model_create": ([_vp, _vp, _vp, C.c_int64, C.POINTER(_vp)], C.c_int),
    "yk_model_destroy": ([_vp], C.c_int),
    "yk_detect": ([_vp, _vp, C.c_int, C.c_float, C.c_float, C.c_int, _vp, _vp, _vp], C.c_int),
    "yk_detect_graph": ([_vp, _vp, C.c_int, C.c_float, C.c_float, C.c_int, _vp, _vp, _vp], C.c_int),
    "yk_model_outputs": ([_vp, C.POINTER(_vp), C.POINTER(_vp)], C.c_int),
    "yk_model_candidates": ([_vp, C.POINTER(_vp), C.POINTER(_vp)], C.c_int),
    "yk_model_buffer": ([_vp, C.c_int, C.POINTER(_vp)], C.c_int),
    "yk_memcpy_d2h": ([_vp, _vp, C.c_int64], C.c_int),
    "yk_model_profile": ([_vp, _vp, C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, _vp, _vp], C.c_int),
    "yk_model_op_kernel": ([_vp, C.c_int, C.c_char_p, C.c_int], C.c_int),
    "yk_tracker_phase_ticks": ([_vp, C.c_int, _vp, _vp], C.c_int),
    "yk_tracker_set_events": ([_vp, C.c_int], C.c_int),
    "yk_tracker_events": ([_vp, C.c_int, _vp, _vp, _vp], C.c_int),
    "yk_model_set_lanes": ([_vp, C.c_int], C.c_int),
    "yk_model_set_schedule": ([_vp, C.c_int, C.c_int], C.c_int),
    "yk_model_set_plan": ([_vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int], C.c_int),
    "yk_model_autotune": ([_vp, _vp, C.c_int, C.c_float, C.c_int, _vp], C.c_int),
    "yk_model_get_schedule": ([_vp, _vp, _vp], C.c_int),
    "yk_model_graph_count": ([_vp, C.POINTER(_i32), C.POINTER(_i32)], C.c_int),
    "yk_store_check_count": ([_vp], C.c_int),
    "yk_model_get_plan": ([_vp, _vp, _vp], C.c_int),
    "yk_model_load": ([_vp, C.c_char_p, C.POINTER(_vp)], C.c_int),
    "yk_program_build": ([C.POINTER(Weights), C.c_char, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                          C.POINTER(_vp)], C.c_int),
    "yk_program_get": ([_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(C.c_int64)], C.c_int),
    "yk_program_destroy": ([_vp], C.c_int),
    "yk_model_load_weights": ([_vp, C.POINTER(Weights), C.c_char, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                               C.POINTER(_vp)], C.c_int),
    "yk_bt_create": ([_vp, C.c_int, C.POINTER(BtCfg), C.POINTER(_vp)], C.c_int),
    "yk_bt_destroy": ([_vp], C.c_int),
    "yk_bt_reset": ([_vp, _vp], C.c_int),
    "yk_bt_step": ([_vp, _vp, _vp, _vp], C.c_int),
    "yk_bt_step_warp": ([_vp, _vp, _vp, _vp, _vp], C.c_int),
    "yk_bt_outputs": ([_vp, C.POINTER(_vp), C.POINTER(_vp)], C.c_int),
    "yk_bt_download": ([_vp, _vp, _vp, _vp], C.c_int),
    "yk_gmd_create": ([_vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)], C.c_int),
    "yk_gmd_destroy": ([_vp], C.c_int),
    "yk_gmd_reset": ([_vp, _vp], C.c_int),
    "yk_gmd_reset_stats": ([_vp, _vp], C.c_int),
    "yk_gmd_set_thresholds": ([_vp, C.c_double, C.c_double], C.c_int),
    "yk_gmd_detect": ([_vp, _vp, _vp, _vp], C.c_int),
    "yk_gmd_detect_window": ([_vp, C.POINTER(_vp), C.c_int, _vp, _vp], C.c_int),
    "yk_gmd_outputs": ([_vp, C.POINTER(_vp)], C.c_int),
    "yk_gmd_debug_buffers": ([_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_i32)],
                             C.c_int),
    "yk_gmd_debug_pyramids": ([_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp),
                               C.POINTER(C.c_int64)], C.c_int),
    "yk_gmd_download": ([_vp, _vp, _vp, _vp], C.c_int),
    "yk_gmd_points": ([_vp, C.c_int, _vp, _vp, _vp, C.POINTER(_i32), _vp], C.c_int),
    "yk_gmc_apply": ([_vp, _vp, _vp, _vp], C.c_int),
    "yk_gmc_outputs": ([_vp, C.POINTER(_vp)], C.c_int),
    "yk_gmc_info": ([_vp, _vp, _vp], C.c_int),
    "yk_tracker_step_motion": ([_vp, _vp, C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "yk_nms": ([_vp, _vp, C.c_int, C.c_int, _vp, C.c_int, C.c_float, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "yk_nms_candidates": ([_vp, C.c_int, C.c_float, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "yk_model_nms_stats": ([_vp, _vp, C.c_int, _vp], C.c_int),
    "yk_model_check": ([_vp, _vp], C.c_int),
}

_lock = threading.Lock()
_lib = None


ABI_VERSION = 3  # include/yk.h YK_ABI_VERSION


def exported_symbols() -> list[str]:
    return sorted(_SIGS)


def lib() -> C.CDLL:
    """Load libyk.so once (raises YKError if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise YKError(f"libyk.so not found at {LIB_PATH}: build it with `python __graft_entry__.py build` "
                          "(or csrc/build.py); the HIP path has no CPU fallback")
        try:
            L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        except OSError as e:
            raise YKError(f"failed to load {LIB_PATH}: {e}") from e
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.yk_abi_version() != ABI_VERSION:
            raise YKError(f"libyk.so ABI version {L.yk_abi_version()}, this package expects {ABI_VERSION}")
        sizes = {0: C.sizeof(TrackerCfg), 1: STATS_DTYPE.itemsize, 2: TRACK_OUT_DTYPE.itemsize,
                 3: TRACK_STATE_DTYPE.itemsize, 7: C.sizeof(BtCfg), 8: MOTION_DTYPE.itemsize,
                 9: GMD_STATS_DTYPE.itemsize, 10: C.sizeof(Tensor), 11: TRACK_EVENT_DTYPE.itemsize}
        for k, v in sizes.items():
            if L.yk_struct_size(k) != v:
                raise YKError(f"ABI struct {k} size mismatch: C {L.yk_struct_size(k)} vs python {v}")
        _lib = L
        return L


def check(rc: int, what: str = "") -> None:
    if rc != YK_OK:
        msg = lib().yk_last_error().decode(errors="replace")
        raise YKError(f"{what or 'yk call'} failed (status {rc}): {msg}", rc)


def ptr(a) -> C.c_void_p:
    """Raw pointer of a numpy array or torch tensor (None -> NULL)."""
    if a is None:
        return C.c_void_p(0)
    if isinstance(a, torch.Tensor):
        return C.c_void_p(a.data_ptr())
    return C.c_void_p(a.ctypes.data)


_ctx: dict[int, C.c_void_p] = {}


def context(device: int = 0) -> C.c_void_p:
    """Process-wide yk_ctx for a device (one context per GPU, like select_device)."""
    if device in _ctx:
        return _ctx[device]
    if not torch.cuda.is_available():
        raise YKError("no HIP device visible: the yk hot path runs only on an AMD GPU (no CPU fallback)")
    torch.cuda.init()
    h = C.c_void_p()
    check(lib().yk_ctx_create(device, C.byref(h)), "yk_ctx_create")
    _ctx[device] = h
    return h


def current_stream(device: int = 0) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
