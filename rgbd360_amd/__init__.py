"""rgbd360_amd — MI355X-native (gfx950) registration hot path of rgbd360.

Python mirror of the reference's C++ class surface for the hot path, written over the C-ABI of
``rgbd360_amd/lib/librgbd360_hip.so`` (declared in ``include/rgbd360_hip.h``):

    Calib360          include/Calib360.h:44-132
    Frame360          include/Frame360.h:93-1150   (loadFrame / undistort / stitchSphericalImage /
                      buildSphereCloud / getPlanes)
    RegisterRGBD360   include/RegisterRGBD360.h:47-340 (RegisterPbMap / getPose / getInfoMat /
                      getMatchedPlanes / getAreaMatched / areaSource / areaTarget, Register alias)
    RegisterPhotoICP  include/RegisterPhotoICP.h:85-4784 (setSourceFrame / setTargetFrame /
                      alignFrames360 / getOptimalPose / getHessian / getGradient)

The HIP library is the only compute path: there is no CPU fallback.  Importing works without a
GPU (so the CPU test-suite can check that the library loads and exports its ABI); creating a
``Context`` on a machine without a GPU raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes as C
import os
import numpy as np

C = C  # re-exported for callers that drive the C-ABI directly (bench.py)

__all__ = [
    "lib", "Context", "Calib360", "Frame360", "RegisterPhotoICP", "RegisterRGBD360", "IcpParams", "IcpStats",
    "PHOTO_CONSISTENCY", "DEPTH_CONSISTENCY", "PHOTO_DEPTH", "synth_path_pose", "exp_se3",
    "LIB_PATH", "ABI_SYMBOLS", "Batch", "PairJob", "PairResult", "JOB_PBMAP_ONLY", "JOB_GATED", "JOB_ALWAYS",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("R360_LIB") or os.path.join(_HERE, "lib", "librgbd360_hip.so")
REPO_ROOT = os.path.dirname(_HERE)

PHOTO_CONSISTENCY, DEPTH_CONSISTENCY, PHOTO_DEPTH = 0, 1, 2
BUILD_UNDISTORT, BUILD_SPHERE, BUILD_PYRAMID, BUILD_CLOUD, BUILD_PLANES = 1, 2, 4, 8, 16
BUILD_SENSOR_PYRAMID = 32
PCD_ASCII, PCD_BINARY, PCD_BINARY_COMPRESSED = 0, 1, 2


class IcpParams(C.Structure):
    """r360_icp_params — RegisterPhotoICP settings (see include/rgbd360_hip.h)."""
    _fields_ = [
        ("n_pyr", C.c_int), ("max_iters", C.c_int), ("min_depth", C.c_float), ("max_depth", C.c_float),
        ("std_dev_photo", C.c_float), ("std_dev_depth", C.c_float), ("thres_sal_int", C.c_float),
        ("thres_sal_depth", C.c_float), ("tol_residual", C.c_double), ("tol_update", C.c_double),
        ("lambda_", C.c_double), ("fixed_iters_level0", C.c_int),
    ]

    @classmethod
    def default(cls) -> "IcpParams":
        p = cls()
        lib().r360_icp_default_params(C.byref(p))
        return p


class MatchParams(C.Structure):
    """r360_match_params — SubgraphMatcher thresholds, the keys of config_files/configLocaliser_*.ini that
    RegisterRGBD360(configFile) loads (RegisterRGBD360.h:97-100); angles in degrees."""
    _fields_ = [("min_planes_recognition", C.c_int), ("dist_d", C.c_float), ("angle", C.c_float),
                ("color_threshold", C.c_float), ("intensity_threshold", C.c_float),
                ("elongation_threshold", C.c_float), ("area_threshold", C.c_float), ("dist_threshold", C.c_float),
                ("angle_threshold", C.c_float), ("height_threshold", C.c_float), ("cos_angle_parallel", C.c_float),
                ("planar_normal_angle", C.c_float), ("max_nodes", C.c_long)]

    @classmethod
    def default(cls) -> "MatchParams":
        """configLocaliser_sphericalOdometry.ini (the odometry apps' file)."""
        m = cls()
        lib().r360_match_params_default(C.byref(m))
        return m

    @classmethod
    def load_ini(cls, path: str, base: "MatchParams | None" = None) -> "MatchParams":
        m = cls.default() if base is None else base
        _check(lib().r360_match_params_load_ini(path.encode(), C.byref(m)), "match_params_load_ini")
        return m


class IcpStats(C.Structure):
    _fields_ = [
        ("iters", C.c_int * 8), ("evals", C.c_int * 8), ("illposed", C.c_int), ("sso", C.c_float),
        ("error", C.c_double), ("passes", C.c_int), ("persistent", C.c_int),
        ("av_photo_residual", C.c_double), ("av_depth_residual", C.c_double), ("av_residual", C.c_float),
        ("residuals_set", C.c_int),
    ]


class PairJob(C.Structure):
    """r360_pair_job — one pair of a batched registration call (include/rgbd360_hip.h, §8f-4)."""
    _fields_ = [("ref", C.c_void_p), ("trg", C.c_void_p), ("dense", C.c_int), ("ref_is_source", C.c_int),
                ("guess", C.c_float * 16)]


class PairResult(C.Structure):
    """r360_pair_result — RegisterPbMap outputs and the dense refinement of one batched pair."""
    _fields_ = [("good", C.c_int), ("n_match", C.c_int), ("area_matched", C.c_float), ("area_src", C.c_float),
                ("area_trg", C.c_float), ("sso_pbmap", C.c_float), ("pbmap_pose", C.c_float * 16),
                ("pbmap_info", C.c_float * 36), ("dense_rc", C.c_int), ("pose", C.c_float * 16),
                ("hessian", C.c_float * 36), ("stats", IcpStats)]

    def as_dict(self) -> dict:
        return {"good": self.good, "n_match": self.n_match, "area_matched": self.area_matched,
                "area_src": self.area_src, "area_trg": self.area_trg, "sso_pbmap": self.sso_pbmap,
                "pbmap_pose": _from16(np.array(self.pbmap_pose, np.float32)),
                "pbmap_info": np.array(self.pbmap_info, np.float32).reshape(6, 6).T.copy(),
                "dense_rc": self.dense_rc, "pose": _from16(np.array(self.pose, np.float32)),
                "hessian": np.array(self.hessian, np.float32).reshape(6, 6).T.copy(),
                "sso": self.stats.sso, "error": self.stats.error}


JOB_PBMAP_ONLY, JOB_GATED, JOB_ALWAYS = 0, 1, 2


class DenseStats(C.Structure):
    """r360_dense_stats — RegisterDensePhotoICP per-level diagnostics."""
    _fields_ = [("error", C.c_double * 8), ("ran", C.c_int * 8), ("n_visible", C.c_int * 8), ("n_error", C.c_int * 8),
                ("illposed_level", C.c_int), ("levels", C.c_int), ("info_set", C.c_int), ("pad", C.c_int),
                ("gradient", C.c_float * 6)]


class Plane(C.Structure):
    """r360_plane — the mrpt::pbmap::Plane fields used on the path (rig frame)."""
    _fields_ = [("normal", C.c_float * 3), ("center", C.c_float * 3), ("d", C.c_float), ("area", C.c_float),
                ("elongation", C.c_float), ("curvature", C.c_float), ("ppal", C.c_float * 3), ("nrgb", C.c_float * 3),
                ("intensity", C.c_float), ("id", C.c_int), ("sensor", C.c_int), ("n_inliers", C.c_int),
                ("n_hull", C.c_int)]


class Region(C.Structure):
    _fields_ = [("label", C.c_int), ("count", C.c_int), ("start_idx", C.c_int), ("n_contour", C.c_int),
                ("n_fit", C.c_int), ("centroid", C.c_float * 3), ("cov", C.c_float * 9), ("model", C.c_float * 4),
                ("curvature", C.c_float)]


DEFAULT_6DoF, PLANAR_3DoF, ODOMETRY_6DoF, PLANAR_ODOMETRY_3DoF = 0, 1, 2, 3


# (name, restype, argtypes) of every exported entry point of include/rgbd360_hip.h
_P = C.c_void_p
_FP = C.POINTER(C.c_float)
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int)
_SIGS = [
    ("r360_ctx_create", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("r360_ctx_destroy", None, [_P]),
    ("r360_ctx_sync", C.c_int, [_P]),
    ("r360_ctx_stream", _P, [_P]),
    ("r360_last_error", C.c_char_p, []),
    ("r360_version", C.c_char_p, []),
    ("r360_calib_create", C.c_int, [_P, C.c_int, C.c_int, C.POINTER(_P)]),
    ("r360_calib_destroy", None, [_P]),
    ("r360_calib_set_extrinsics", C.c_int, [_P, _FP]),
    ("r360_calib_get_extrinsics", C.c_int, [_P, _FP, _FP, _FP]),
    ("r360_calib_load_extrinsics", C.c_int, [_P, C.c_char_p]),
    ("r360_calib_load_intrinsics", C.c_int, [_P, C.c_char_p]),
    ("r360_frame_create", C.c_int, [_P, _P, C.POINTER(_P)]),
    ("r360_frame_destroy", None, [_P]),
    ("r360_frame_upload", C.c_int, [_P, _P, _P]),
    ("r360_frame_upload_device", C.c_int, [_P, _P, _P]),
    ("r360_frame_upload_async", C.c_int, [_P, _P, _P]),
    ("r360_frame_set_sphere", C.c_int, [_P, _P, _P, C.c_int, C.c_int]),
    ("r360_calib_create_sphere", C.c_int, [_P, C.c_int, C.c_int, C.POINTER(_P)]),
    ("r360_host_register", C.c_int, [_P, C.c_size_t]),
    ("r360_host_unregister", C.c_int, [_P]),
    ("r360_frame_load_bin", C.c_int, [_P, C.c_char_p]),
    ("r360_frame_save_bin", C.c_int, [_P, C.c_char_p]),
    ("r360_frame_set_timestamp", C.c_int, [_P, C.c_uint64]),
    ("r360_frame_get_timestamp", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("r360_frame_get_sphere_cloud", C.c_int, [_P, _FP, _P, C.c_size_t, _IP, _IP]),
    ("r360_pcd_write", C.c_int, [C.c_char_p, _FP, _P, C.c_int, C.c_int, C.c_int]),
    ("r360_pcd_read", C.c_int, [C.c_char_p, _FP, _P, C.c_size_t, C.POINTER(C.c_size_t), _IP, _IP]),
    ("r360_frame_save_cloud", C.c_int, [_P, C.c_char_p, C.c_int]),
    ("r360_frame_load_cloud", C.c_int, [_P, C.c_char_p]),
    ("r360_frame_save_planes", C.c_int, [_P, C.c_char_p]),
    ("r360_frame_load_pbmap", C.c_int, [_P, C.c_char_p]),
    ("r360_frame_save", C.c_int, [_P, C.c_char_p, C.c_uint]),
    ("r360_frame_load_pbmap_cloud", C.c_int, [_P, C.c_char_p, C.c_uint]),
    ("r360_frame_set_plane_label", C.c_int, [_P, C.c_int, C.c_char_p]),
    ("r360_frame_get_plane_label", C.c_int, [_P, C.c_int, C.c_char_p, C.c_int]),
    ("r360_frame_build", C.c_int, [_P, C.c_uint]),
    ("r360_frame_build_async", C.c_int, [_P, C.c_uint]),
    ("r360_frames_build", C.c_int, [_P, C.c_int, C.c_uint]),
    ("r360_frame_dims", C.c_int, [_P, _IP, _IP, _IP, _IP]),
    ("r360_frame_set_levels", C.c_int, [_P, C.c_int]),
    ("r360_frame_set_compaction", C.c_int, [_P, C.c_int]),
    ("r360_frame_built", C.c_int, [_P, C.POINTER(C.c_uint)]),
    ("r360_frame_get_sphere", C.c_int, [_P, _P, _P]),
    ("r360_frame_get_depth_m", C.c_int, [_P, _P]),
    ("r360_frame_get_level", C.c_int, [_P, C.c_int, _IP, _IP, _P, _P, _P, _P, _P, _P]),
    ("r360_frame_get_points", C.c_int, [_P, C.c_int, _FP, C.c_int, _IP]),
    ("r360_frame_get_sensor_level", C.c_int, [_P, C.c_int, C.c_int, _IP, _IP, _P, _P, _P, _P, _P, _P]),
    ("r360_icp_default_params", None, [C.POINTER(IcpParams)]),
    ("r360_align360", C.c_int, [_P, _P, _P, _FP, C.c_int, C.c_int, C.POINTER(IcpParams), _FP, _FP, _FP,
                                C.POINTER(IcpStats)]),
    ("r360_align360_async", C.c_int, [_P, _P, _P, _FP, C.c_int, C.c_int, C.POINTER(IcpParams)]),
    ("r360_align360_result", C.c_int, [_P, _FP, _FP, _FP, C.POINTER(IcpStats)]),
    ("r360_align360_batch_async", C.c_int, [_P, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), _FP, C.c_int,
                                            C.POINTER(IcpParams)]),
    ("r360_align360_batch_result", C.c_int, [_P, _FP, _FP, _FP, C.POINTER(IcpStats)]),
    ("r360_refine_eval", C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, _P]),
    ("r360_dense_queue_create", C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("r360_dense_queue_destroy", None, [_P]),
    ("r360_dense_queue_ctx", C.c_void_p, [_P]),
    ("r360_dense_queue_stats", C.c_int, [_P, C.POINTER(C.c_long), C.POINTER(C.c_long), _IP]),
    ("r360_dense_queue_submit", C.c_int, [_P, _P, _P, _FP, C.c_int, C.POINTER(IcpParams), C.POINTER(C.c_long)]),
    ("r360_dense_queue_collect", C.c_int, [_P, C.c_long, _FP, _FP, _FP, C.POINTER(IcpStats)]),
    ("r360_register_submit", C.c_int, [_P, _P, _P, _P, _FP, C.POINTER(IcpParams), C.c_size_t, C.c_int,
                                       C.POINTER(C.c_long)]),
    ("r360_register_collect", C.c_int, [_P, C.c_long, _FP, _FP, C.POINTER(IcpStats)]),
    ("r360_sequence_default_params", None, [_P]),
    ("r360_sequence_create", C.c_int, [C.c_int, _P, C.c_char_p, C.POINTER(_P)]),
    ("r360_sequence_destroy", None, [_P]),
    ("r360_sequence_run", C.c_int, [_P, C.c_int, C.c_int, _P, _P, C.c_int, C.c_int, _P, C.c_int, _P]),
    ("r360_sequence_info", C.c_int, [_P, _IP, C.POINTER(_P)]),
    ("r360_sequence_pipeline", C.c_int, [_P, C.c_int, C.POINTER(_P), C.POINTER(_P), _P, C.c_int, _IP,
                                         C.POINTER(C.c_long)]),
    ("r360_sequence_host_times", C.c_int, [_P, _P, C.c_int]),
    ("r360_sequence_plane_stats", C.c_int, [_P, C.POINTER(C.c_long), C.POINTER(C.c_long), _IP, C.POINTER(_P)]),
    ("r360_icp_eval", C.c_int, [_P, _P, _P, C.c_int, _FP, C.c_int, C.POINTER(IcpParams), _DP, _DP, _DP, _IP,
                                _IP]),
    ("r360_icp_eval_occ", C.c_int, [_P, _P, _P, C.c_int, _FP, C.c_int, C.c_int, C.POINTER(IcpParams), _DP, _DP,
                                    _DP, _IP, _IP]),
    ("r360_exp_se3", None, [_DP, C.c_int, _FP]),
    ("r360_align_pinhole", C.c_int, [_P, _P, _P, C.c_int, _FP, C.c_int, _FP, C.POINTER(IcpParams), _FP, _FP, _FP,
                                     C.POINTER(IcpStats)]),
    ("r360_align_pinhole_async", C.c_int, [_P, _P, _P, C.c_int, _IP, _FP, C.c_int, _FP, C.POINTER(IcpParams)]),
    ("r360_align_pinhole_result", C.c_int, [_P, _FP, _FP, _FP, C.POINTER(IcpStats)]),
    ("r360_pinhole_eval", C.c_int, [_P, _P, _P, C.c_int, C.c_int, _FP, C.c_int, _FP, C.POINTER(IcpParams), _DP, _DP,
                                    _DP, _DP, _IP]),
    ("r360_register_dense", C.c_int, [_P, _P, _P, _FP, C.c_int, C.c_int, C.POINTER(IcpParams), _FP, _FP,
                                      C.POINTER(DenseStats)]),
    ("r360_dense_robot_eval", C.c_int, [_P, _P, _P, C.c_int, _FP, C.c_int, C.POINTER(IcpParams), _DP, _DP, _DP,
                                        _IP]),
    ("r360_frame_get_planes", C.c_int, [_P, C.POINTER(Plane), C.c_int, _IP]),
    ("r360_frame_get_plane_hull", C.c_int, [_P, C.c_int, _FP, C.c_int, _IP]),
    ("r360_match_params_default", None, [C.POINTER(MatchParams)]),
    ("r360_match_params_load_ini", C.c_int, [C.c_char_p, C.POINTER(MatchParams)]),
    ("r360_ctx_set_match_params", C.c_int, [_P, C.POINTER(MatchParams)]),
    ("r360_ctx_get_match_params", C.c_int, [_P, C.POINTER(MatchParams)]),
    ("r360_ctx_match_stats", C.c_int, [_P, C.POINTER(C.c_long), C.POINTER(C.c_long), C.POINTER(C.c_long)]),
    ("r360_match_tree_search", C.c_int, [C.c_int, C.c_int, _P, _P, C.c_int, _P, C.c_long, _P, C.POINTER(C.c_long)]),
    ("r360_batch_set_match_params", C.c_int, [_P, C.POINTER(MatchParams)]),
    ("r360_register_pbmap", C.c_int, [_P, _P, _P, C.c_size_t, C.c_int, _FP, _FP, _IP, C.c_int, _IP, _FP, _FP, _FP]),
    ("r360_register", C.c_int, [_P, _P, _P, _FP, C.POINTER(IcpParams), C.c_size_t, C.c_int, _FP, _FP,
                                C.POINTER(IcpStats)]),
    ("r360_register_async", C.c_int, [_P, _P, _P, _FP, C.POINTER(IcpParams), C.c_size_t, C.c_int]),
    ("r360_register_result", C.c_int, [_P, _FP, _FP, C.POINTER(IcpStats)]),
    ("r360_pbmap_match_tables", C.c_int, [_P, _P, _P, C.c_size_t, C.c_int, _IP, _IP, _IP, _IP, _P, _P, C.c_int]),
    ("r360_batch_create", C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("r360_batch_destroy", None, [_P]),
    ("r360_batch_lanes", C.c_int, [_P]),
    ("r360_batch_register", C.c_int, [_P, C.POINTER(PairJob), C.c_int, C.c_size_t, C.c_int, C.c_int, C.c_float,
                                      C.POINTER(IcpParams), C.POINTER(PairResult)]),
    ("r360_track_frame", C.c_int, [_P, C.POINTER(C.c_void_p), C.c_int, _P, C.c_int, C.c_int, C.c_size_t, C.c_int,
                                   _IP, C.POINTER(PairResult), C.POINTER(PairResult)]),
    ("r360_frame_get_cloud", C.c_int, [_P, _FP, _P, _FP, _FP]),
    ("r360_frame_get_labels", C.c_int, [_P, _IP, _IP]),
    ("r360_frame_get_regions", C.c_int, [_P, C.c_int, C.POINTER(Region), C.c_int, _IP]),
    ("r360_comm_unique_id", C.c_int, [_P]),
    ("r360_comm_init", C.c_int, [C.c_int, C.c_int, C.c_int, _P, C.POINTER(_P)]),
    ("r360_comm_destroy", None, [_P]),
    ("r360_comm_allgather", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("r360_comm_allreduce_max", C.c_int, [_P, _DP, C.c_int]),
    ("r360_dev_alloc", C.c_int, [C.c_int, C.c_size_t, C.POINTER(_P)]),
    ("r360_dev_free", C.c_int, [_P]),
    ("r360_dev_copy", C.c_int, [_P, _P, C.c_size_t, C.c_int]),
    ("r360_synth_frame", C.c_int, [_P, C.c_uint32, _FP, _P, _P]),
    ("r360_synth_frame_rt", C.c_int, [C.c_int, C.c_int, _FP, C.c_uint32, _FP, _P, _P]),
    ("r360_synth_path_pose", C.c_int, [C.c_uint32, C.c_int, _FP]),
    ("r360_libm_eval", C.c_int, [_FP, _FP, _FP, C.c_int, _FP, _FP, C.c_int]),
    ("r360_rn_check", C.c_int, [C.c_uint, C.c_uint, C.POINTER(C.c_ulonglong)]),
    ("r360_rank6", C.c_int, [_FP, C.c_int, _IP]),
    ("r360_data_dir", C.c_char_p, []),
    ("r360_solve6", C.c_int, [_DP, _DP, C.c_int, _DP]),
    ("r360_proj_check_pose", C.c_int, [_FP, _FP, _FP, C.c_int, _FP, C.c_int, C.c_int, C.POINTER(C.c_ulonglong),
                                       C.POINTER(C.c_ulonglong)]),
    ("r360_proj_check", C.c_int, [_FP, _FP, _FP, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_ulonglong),
                                  C.POINTER(C.c_ulonglong)]),
    ("r360_ctx_debug_stamps", C.c_int, [_P, C.POINTER(C.c_ulonglong)]),
    ("r360_ctx_kernel_time", C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_long)]),
    ("r360_ctx_kernel_time_reset", C.c_int, [_P]),
    ("r360_ctx_host_times", C.c_int, [_P, C.POINTER(C.c_double), C.c_int]),
    ("r360_ctx_kernel_stats", C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_long),
                                        C.POINTER(C.c_long)]),
    ("r360_ctx_timing", C.c_int, [_P, C.c_int]),
    ("r360_ctx_persistent_levels", C.c_int, [_P, C.c_int]),
    ("r360_ctx_latency_mode", C.c_int, [_P, C.c_int]),
    ("r360_ctx_timing_read", C.c_int, [_P, C.c_char_p, _DP, C.POINTER(C.c_long)]),
    ("r360_ctx_timing_reset", C.c_int, [_P]),
]
ABI_SYMBOLS = [s[0] for s in _SIGS]

_lib = None


def lib() -> C.CDLL:
    """Load librgbd360_hip.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, res, args in _SIGS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise RuntimeError(f"{what} failed ({rc}): {lib().r360_last_error().decode()}")
    return rc


def pcd_write(path: str, xyz: np.ndarray, rgba: np.ndarray | None, width: int, height: int, mode: int = PCD_ASCII):
    """pcl::io::savePCDFile of a PointXYZRGBA cloud (host-only codec)."""
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    assert xyz.shape[0] == width * height
    if rgba is not None:
        rgba = np.ascontiguousarray(rgba, np.uint32).reshape(-1)
        assert rgba.shape[0] == xyz.shape[0]
    _check(lib().r360_pcd_write(path.encode(), _fptr(xyz), None if rgba is None else _vptr(rgba), width, height, mode),
           "pcd_write")


def pcd_read(path: str):
    """PCDReader::read into (xyz [n,3] f32, rgba [n] u32, width, height)."""
    n, w, h = C.c_size_t(), C.c_int(), C.c_int()
    _check(lib().r360_pcd_read(path.encode(), None, None, 0, C.byref(n), C.byref(w), C.byref(h)), "pcd_read")
    xyz = np.zeros((n.value, 3), np.float32)
    rgba = np.zeros(n.value, np.uint32)
    _check(lib().r360_pcd_read(path.encode(), _fptr(xyz), _vptr(rgba), n.value, C.byref(n), C.byref(w), C.byref(h)),
           "pcd_read")
    return xyz, rgba, w.value, h.value


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(_FP)


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(_DP)


def _vptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def _mat16(m) -> np.ndarray:
    """4x4 numpy (row-major semantic) -> column-major float[16] (Eigen::Matrix4f::data())."""
    return np.ascontiguousarray(np.asarray(m, dtype=np.float32).T).reshape(16).copy()


def _from16(a: np.ndarray) -> np.ndarray:
    return a.reshape(4, 4).T.copy()


class Context:
    """One HIP device + stream (r360_ctx).  Not thread-safe; use one per host thread."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(lib().r360_ctx_create(device, C.byref(h)), "r360_ctx_create")
        self.h = h
        self.device = device

    @classmethod
    def _view(cls, h, device: int) -> "Context":
        """A non-owning view of a context the library owns (a sequence runner's pipeline, a dense queue)."""
        c = cls.__new__(cls)
        c.h, c.device = h, device
        c.close = lambda: None
        return c

    def sync(self):
        _check(lib().r360_ctx_sync(self.h), "r360_ctx_sync")

    def persistent_levels(self, enable=True):
        """Lone alignFrames360 as one persistent launch per pyramid level (bit-identical; off by default)."""
        _check(lib().r360_ctx_persistent_levels(self.h, int(enable)), "persistent_levels")

    def latency_mode(self, enable=True):
        """On (the default): PbMap waits assemble the frame themselves, split uploads, graph-replayed lone plane
        stages; off for a context among many pipelines.  Results are identical either way."""
        _check(lib().r360_ctx_latency_mode(self.h, int(enable)), "latency_mode")

    def timing(self, enable):
        """0/False off, 1/True HIP events around every launch, 2 around the level-0 ICP passes only."""
        _check(lib().r360_ctx_timing(self.h, int(enable)), "timing")

    def timing_read(self, kernel: str):
        ms, n = C.c_double(), C.c_long()
        _check(lib().r360_ctx_timing_read(self.h, kernel.encode(), C.byref(ms), C.byref(n)), "timing_read")
        return ms.value, n.value

    def timing_reset(self):
        _check(lib().r360_ctx_timing_reset(self.h), "timing_reset")

    def kernel_time(self, level: int):
        """(summed in-kernel execution span in us, pass count) of the ICP passes at `level`."""
        us, n = C.c_double(), C.c_long()
        _check(lib().r360_ctx_kernel_time(self.h, level, C.byref(us), C.byref(n)), "kernel_time")
        return us.value, n.value

    def kernel_stats(self, level: int):
        """(summed in-kernel span in us, launches, job passes) of the ICP passes at `level`."""
        us, n, j = C.c_double(), C.c_long(), C.c_long()
        _check(lib().r360_ctx_kernel_stats(self.h, level, C.byref(us), C.byref(n), C.byref(j)), "kernel_stats")
        return us.value, n.value, j.value

    def host_times(self, reset: bool = False):
        """Host seconds of this ctx's RegisterPbMap calls: (waiting for the frames' PbMaps, match tables, tree search +
        ConsistencyTest, calls, PbMap assembly of its frames, frames)."""
        out = (C.c_double * 6)()
        _check(lib().r360_ctx_host_times(self.h, out, 1 if reset else 0), "host_times")
        return tuple(out)

    def kernel_time_reset(self):
        _check(lib().r360_ctx_kernel_time_reset(self.h), "kernel_time_reset")

    def match_stats(self):
        """(interpretation-tree searches, searches stopped by the node budget, most nodes of one search) on this ctx."""
        a, b, c = C.c_long(), C.c_long(), C.c_long()
        _check(lib().r360_ctx_match_stats(self.h, C.byref(a), C.byref(b), C.byref(c)), "match_stats")
        return a.value, b.value, c.value

    def close(self):
        if self.h:
            lib().r360_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Calib360:
    """Calib360 (include/Calib360.h:44-132): Rt_[8], Rt_inv[8], cameraMatrix, CLAMS models."""

    def __init__(self, ctx: Context, rows: int = 240, cols: int = 320, _sphere: tuple | None = None):
        h = C.c_void_p()
        if _sphere is None:
            _check(lib().r360_calib_create(ctx.h, rows, cols, C.byref(h)), "r360_calib_create")
        else:
            _check(lib().r360_calib_create_sphere(ctx.h, _sphere[0], _sphere[1], C.byref(h)), "r360_calib_create_sphere")
            rows = cols = 0
        self.h, self.ctx, self.rows, self.cols = h, ctx, rows, cols

    @classmethod
    def _view(cls, h, ctx: Context, rows: int, cols: int) -> "Calib360":
        """A non-owning view of a calibration the library owns."""
        c = cls.__new__(cls)
        c.h, c.ctx, c.rows, c.cols = h, ctx, rows, cols
        c.close = lambda: None
        return c

    @classmethod
    def for_sphere(cls, ctx: Context, sph_rows: int, sph_cols: int) -> "Calib360":
        """A calibration without sensors for spheres given as images (setSourceFrame / setTargetFrame(cv::Mat&,
        cv::Mat&), RegisterPhotoICP.h:480-516)."""
        return cls(ctx, _sphere=(sph_rows, sph_cols))

    def loadExtrinsicCalibration(self, path: str):
        _check(lib().r360_calib_load_extrinsics(self.h, path.encode()), "loadExtrinsicCalibration")

    def loadIntrinsicCalibration(self, path: str):
        _check(lib().r360_calib_load_intrinsics(self.h, path.encode()), "loadIntrinsicCalibration")

    def setRt(self, rt8: np.ndarray):
        """rt8: (8,4,4) rig extrinsics (row-major numpy)."""
        a = np.concatenate([_mat16(m) for m in rt8]).astype(np.float32)
        _check(lib().r360_calib_set_extrinsics(self.h, _fptr(a)), "setRt")

    def extrinsics(self):
        rt = np.zeros(128, np.float32)
        rti = np.zeros(128, np.float32)
        K = np.zeros(9, np.float32)
        _check(lib().r360_calib_get_extrinsics(self.h, _fptr(rt), _fptr(rti), _fptr(K)), "get_extrinsics")
        return rt, rti, K  # column-major blocks, as the C-ABI stores them

    def synth_frame(self, seed: int, rig_pose: np.ndarray):
        """Render a synthetic 8-camera frame of the procedural room (seed) at rig_pose (4x4)."""
        bgr = np.zeros((8, self.rows, self.cols, 3), np.uint8)
        dep = np.zeros((8, self.rows, self.cols), np.uint16)
        p = _mat16(rig_pose)
        _check(lib().r360_synth_frame(self.h, seed, _fptr(p), _vptr(bgr), _vptr(dep)), "synth_frame")
        return bgr, dep

    def close(self):
        if self.h:
            lib().r360_calib_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Frame360:
    """Frame360 (include/Frame360.h:93-1150) with device-resident images and sphere pyramid."""

    def __init__(self, calib: Calib360):
        h = C.c_void_p()
        _check(lib().r360_frame_create(calib.ctx.h, calib.h, C.byref(h)), "r360_frame_create")
        self.h, self.calib = h, calib
        r, c, sr, sc = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        lib().r360_frame_dims(h, C.byref(r), C.byref(c), C.byref(sr), C.byref(sc))
        self.rows, self.cols, self.sph_rows, self.sph_cols = r.value, c.value, sr.value, sc.value

    @classmethod
    def _view(cls, h, calib: Calib360) -> "Frame360":
        """A non-owning view of a frame the library owns (a sequence runner's ring buffer)."""
        f = cls.__new__(cls)
        f.h, f.calib = h, calib
        r, c, sr, sc = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        lib().r360_frame_dims(h, C.byref(r), C.byref(c), C.byref(sr), C.byref(sc))
        f.rows, f.cols, f.sph_rows, f.sph_cols = r.value, c.value, sr.value, sc.value
        f.close = lambda: None
        return f

    def setNumPyr(self, n: int):
        """r360_frame_set_levels: the frame's pyramid stops at n levels (RegisterPhotoICP::setNumPyr)."""
        _check(lib().r360_frame_set_levels(self.h, int(n)), "r360_frame_set_levels")

    def setCompaction(self, all_levels: bool):
        """r360_frame_set_compaction: compact every level's source points at the next build (default), or only the
        levels a batched pass cannot stream as an image."""
        _check(lib().r360_frame_set_compaction(self.h, int(bool(all_levels))), "r360_frame_set_compaction")

    def loadFrame(self, path: str):
        _check(lib().r360_frame_load_bin(self.h, path.encode()), "loadFrame")

    def serialize(self, fileName: str):
        """Frame360::serialize (Frame360.h:332-345): the raw images + timestamp as a .bin archive."""
        _check(lib().r360_frame_save_bin(self.h, fileName.encode()), "serialize")

    def setTimeStamp(self, timestamp: int):
        _check(lib().r360_frame_set_timestamp(self.h, int(timestamp)), "setTimeStamp")

    @property
    def timeStamp(self) -> int:
        t = C.c_uint64()
        _check(lib().r360_frame_get_timestamp(self.h, C.byref(t)), "timeStamp")
        return t.value

    def sphereCloud(self):
        """Frame360::sphereCloud: (xyz [n,3] f32, rgba [n] u32, width, height)."""
        w, h = C.c_int(), C.c_int()
        _check(lib().r360_frame_get_sphere_cloud(self.h, None, None, 0, C.byref(w), C.byref(h)), "sphereCloud")
        n = w.value * h.value
        xyz = np.zeros((n, 3), np.float32)
        rgba = np.zeros(n, np.uint32)
        _check(lib().r360_frame_get_sphere_cloud(self.h, _fptr(xyz), _vptr(rgba), n, C.byref(w), C.byref(h)),
               "sphereCloud")
        return xyz, rgba, w.value, h.value

    def loadCloud(self, pointCloudPath: str):
        _check(lib().r360_frame_load_cloud(self.h, pointCloudPath.encode()), "loadCloud")

    def loadPbMap(self, pbmapPath: str):
        _check(lib().r360_frame_load_pbmap(self.h, pbmapPath.encode()), "loadPbMap")

    def load_PbMap_Cloud(self, path: str, index_or_pbmap):
        """load_PbMap_Cloud(cloudPath, pbmapPath) or load_PbMap_Cloud(dir, index) (Frame360.h:212-228)."""
        if isinstance(index_or_pbmap, str):
            self.loadCloud(path)
            self.loadPbMap(index_or_pbmap)
        else:
            _check(lib().r360_frame_load_pbmap_cloud(self.h, path.encode(), int(index_or_pbmap)), "load_PbMap_Cloud")

    def savePlanes(self, pathPbMap: str):
        _check(lib().r360_frame_save_planes(self.h, pathPbMap.encode()), "savePlanes")

    def saveCloud(self, path: str, mode: int = PCD_ASCII):
        _check(lib().r360_frame_save_cloud(self.h, path.encode(), mode), "saveCloud")

    def save(self, path: str, frame: int):
        """Frame360::save (Frame360.h:320-330): path/sphereCloud_<frame>.pcd + path/spherePlanes_<frame>.pbmap."""
        _check(lib().r360_frame_save(self.h, path.encode(), int(frame)), "save")

    def setPlaneLabel(self, i: int, label: str):
        _check(lib().r360_frame_set_plane_label(self.h, i, label.encode()), "setPlaneLabel")

    def planeLabel(self, i: int) -> str:
        n = lib().r360_frame_get_plane_label(self.h, i, None, 0)
        _check(min(n, 0), "planeLabel")
        buf = C.create_string_buffer(n + 1)
        lib().r360_frame_get_plane_label(self.h, i, buf, n + 1)
        return buf.value.decode()

    def upload(self, bgr8: np.ndarray, depth8: np.ndarray):
        bgr8 = np.ascontiguousarray(bgr8, np.uint8)
        depth8 = np.ascontiguousarray(depth8, np.uint16)
        assert bgr8.shape == (8, self.rows, self.cols, 3) and depth8.shape == (8, self.rows, self.cols)
        _check(lib().r360_frame_upload(self.h, _vptr(bgr8), _vptr(depth8)), "upload")

    def set_sphere(self, bgr: np.ndarray, range_mm: np.ndarray):
        """The sphere as images (BGR u8 [H, W, 3], range u16 mm [H, W]; sphereRGB / sphereDepth) replaces the
        frame's; its ICP pyramid is rebuilt (setSourceFrame / setTargetFrame(cv::Mat&, cv::Mat&))."""
        bgr = np.ascontiguousarray(bgr, np.uint8)
        range_mm = np.ascontiguousarray(range_mm, np.uint16)
        H, W = range_mm.shape
        assert bgr.shape == (H, W, 3)
        _check(lib().r360_frame_set_sphere(self.h, _vptr(bgr), _vptr(range_mm), H, W), "set_sphere")

    def upload_async(self, bgr8: np.ndarray, depth8: np.ndarray):
        """Enqueue the upload on the frame's stream; the arrays must stay alive (and should be page-locked,
        see HostPinned) until the stream has consumed them."""
        assert bgr8.dtype == np.uint8 and depth8.dtype == np.uint16
        assert bgr8.flags.c_contiguous and depth8.flags.c_contiguous
        assert bgr8.shape == (8, self.rows, self.cols, 3) and depth8.shape == (8, self.rows, self.cols)
        _check(lib().r360_frame_upload_async(self.h, _vptr(bgr8), _vptr(depth8)), "upload_async")

    def upload_device(self, d_bgr: int, d_depth: int):
        _check(lib().r360_frame_upload_device(self.h, C.c_void_p(d_bgr), C.c_void_p(d_depth)), "upload_device")

    def build(self, flags: int = BUILD_UNDISTORT | BUILD_SPHERE | BUILD_PYRAMID, sync: bool = True):
        fn = lib().r360_frame_build if sync else lib().r360_frame_build_async
        _check(fn(self.h, flags), "r360_frame_build")

    def undistort(self):
        self.build(BUILD_UNDISTORT)

    def stitchSphericalImage(self):
        self.build(BUILD_SPHERE | BUILD_PYRAMID)

    def buildSphereCloud(self):
        self.build(BUILD_UNDISTORT | BUILD_CLOUD)

    def getPlanes(self):
        """Frame360::getPlanes (Frame360.h:615-640): builds the PbMap; returns the plane list."""
        self.build(BUILD_UNDISTORT | BUILD_PLANES)
        return self.planes()

    def planes(self) -> list[dict]:
        n = C.c_int()
        _check(lib().r360_frame_get_planes(self.h, None, 0, C.byref(n)), "get_planes")
        arr = (Plane * max(n.value, 1))()
        _check(lib().r360_frame_get_planes(self.h, arr, n.value, C.byref(n)), "get_planes")
        out = []
        for i, p in enumerate(arr[:n.value]):
            hull = np.zeros((max(p.n_hull, 1), 3), np.float32)
            m = C.c_int()
            _check(lib().r360_frame_get_plane_hull(self.h, i, _fptr(hull), p.n_hull, C.byref(m)), "get_plane_hull")
            out.append(dict(normal=np.array(p.normal[:]), center=np.array(p.center[:]), d=p.d, area=p.area,
                            elongation=p.elongation, curvature=p.curvature, ppal=np.array(p.ppal[:]),
                            nrgb=np.array(p.nrgb[:]), intensity=p.intensity, id=p.id, sensor=p.sensor,
                            n_inliers=p.n_inliers, hull=hull[:p.n_hull].copy()))
        return out

    def cloud(self):
        """Per-sensor organized clouds after downsample + bilateral filter, normals and distance map."""
        h, w = self.rows // 2, self.cols // 2
        xyz = np.zeros((8, h, w, 4), np.float32)
        rgb = np.zeros((8, h, w, 4), np.uint8)
        nrm = np.zeros((8, h, w, 4), np.float32)
        dist = np.zeros((8, h, w), np.float32)
        _check(lib().r360_frame_get_cloud(self.h, _fptr(xyz), _vptr(rgb), _fptr(nrm), _fptr(dist)), "get_cloud")
        return xyz, rgb, nrm, dist

    def labels(self):
        h, w = self.rows // 2, self.cols // 2
        lab = np.zeros((8, h, w), np.int32)
        labf = np.zeros((8, h, w), np.int32)
        _check(lib().r360_frame_get_labels(self.h, lab.ctypes.data_as(_IP), labf.ctypes.data_as(_IP)), "get_labels")
        return lab, labf

    def regions(self, sensor: int) -> list[dict]:
        n = C.c_int()
        arr = (Region * 64)()
        _check(lib().r360_frame_get_regions(self.h, sensor, arr, 64, C.byref(n)), "get_regions")
        return [dict(label=r.label, count=r.count, start_idx=r.start_idx, n_contour=r.n_contour, n_fit=r.n_fit,
                     centroid=np.array(r.centroid[:]), cov=np.array(r.cov[:]).reshape(3, 3),
                     model=np.array(r.model[:]), curvature=r.curvature) for r in arr[:n.value]]

    def sphere(self):
        bgr = np.zeros((self.sph_rows, self.sph_cols, 3), np.uint8)
        dep = np.zeros((self.sph_rows, self.sph_cols), np.uint16)
        _check(lib().r360_frame_get_sphere(self.h, _vptr(bgr), _vptr(dep)), "get_sphere")
        return bgr, dep

    def depth_m(self):
        d = np.zeros((8, self.rows, self.cols), np.float32)
        _check(lib().r360_frame_get_depth_m(self.h, _vptr(d)), "get_depth_m")
        return d

    def level(self, level: int):
        r, c = C.c_int(), C.c_int()
        _check(lib().r360_frame_get_level(self.h, level, C.byref(r), C.byref(c), None, None, None, None, None,
                                          None), "get_level")
        arrs = [np.zeros((r.value, c.value), np.float32) for _ in range(6)]
        _check(lib().r360_frame_get_level(self.h, level, C.byref(r), C.byref(c), *[_vptr(a) for a in arrs]),
               "get_level")
        return dict(zip(["gray", "depth", "gx", "gy", "dgx", "dgy"], arrs))

    def points(self, level: int) -> np.ndarray:
        """The level's compacted ICP source points: (n, 4) {x, y, z, gray} (valid depth, raster order)."""
        n = C.c_int()
        _check(lib().r360_frame_get_points(self.h, level, None, 0, C.byref(n)), "get_points")
        out = np.zeros((max(n.value, 1), 4), np.float32)
        _check(lib().r360_frame_get_points(self.h, level, _fptr(out), n.value, C.byref(n)), "get_points")
        return out[:n.value]

    def sensor_level(self, sensor: int, level: int):
        """Sensor k's pinhole pyramid level (BUILD_SENSOR_PYRAMID)."""
        r, c = C.c_int(), C.c_int()
        _check(lib().r360_frame_get_sensor_level(self.h, sensor, level, C.byref(r), C.byref(c), None, None, None,
                                                 None, None, None), "get_sensor_level")
        arrs = [np.zeros((r.value, c.value), np.float32) for _ in range(6)]
        _check(lib().r360_frame_get_sensor_level(self.h, sensor, level, C.byref(r), C.byref(c),
                                                 *[_vptr(a) for a in arrs]), "get_sensor_level")
        return dict(zip(["gray", "depth", "gx", "gy", "dgx", "dgy"], arrs))

    def close(self):
        if self.h:
            lib().r360_frame_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RegisterRGBD360:
    """RegisterRGBD360 (include/RegisterRGBD360.h:47-340): PbMap registration of two Frame360."""

    def __init__(self, ctx: "Context", config_file: str | None = None):
        # RegisterRGBD360(configFile): matcher.configLocaliser.load_params(configFile) (:97-100); without a
        # file, the configLocaliser_sphericalOdometry.ini values
        self.ctx = ctx
        self.config_file = config_file
        self.match = MatchParams.load_ini(config_file) if config_file else MatchParams.default()
        self.rigidTransf = np.eye(4, dtype=np.float32)
        self.informationM = np.zeros((6, 6), np.float32)
        self.bestMatch: dict[int, int] = {}
        self.areaMatched = self.areaSource = self.areaTarget = 0.0
        self.ref = self.trg = None
        self.max_match_planes = 0

    def setReference(self, ref: "Frame360", max_match_planes: int = 0):
        self.ref, self.max_match_planes = ref, max_match_planes

    def setTarget(self, trg: "Frame360", max_match_planes: int = 0):
        self.trg, self.max_match_planes = trg, max_match_planes

    def RegisterPbMap(self, frame1=None, frame2=None, max_match_planes: int = 0, registMode: int = DEFAULT_6DoF) -> bool:
        if frame1 is not None:
            self.setReference(frame1, max_match_planes)
        if frame2 is not None:
            self.setTarget(frame2, max_match_planes)
        pose = _mat16(self.rigidTransf)
        info = np.ascontiguousarray(self.informationM.T).reshape(36).copy()
        pairs = np.zeros(512, np.int32)
        n = C.c_int()
        am, as_, at = C.c_float(), C.c_float(self.areaSource), C.c_float(self.areaTarget)
        _check(lib().r360_ctx_set_match_params(self.ctx.h, C.byref(self.match)), "set_match_params")
        rc = _check(lib().r360_register_pbmap(self.ctx.h, self.ref.h, self.trg.h, self.max_match_planes, registMode,
                                              _fptr(pose), _fptr(info), pairs.ctypes.data_as(_IP), 256, C.byref(n),
                                              C.byref(am), C.byref(as_), C.byref(at)), "RegisterPbMap")
        self.bestMatch = {int(pairs[2 * k]): int(pairs[2 * k + 1]) for k in range(min(n.value, 256))}
        self.areaMatched = am.value
        if rc == 1:
            self.rigidTransf = _from16(pose)
            self.informationM = info.reshape(6, 6).T.copy()
            self.areaSource, self.areaTarget = as_.value, at.value
        return rc == 1

    def RegisterDensePhotoICP(self, frame1, frame2, pose_estim=None, method: int = PHOTO_CONSISTENCY,
                              registMode: int = DEFAULT_6DoF, params: "IcpParams | None" = None) -> bool:
        """RegisterDensePhotoICP (RegisterRGBD360.h:344-520): frame2's 8 sensor images aligned to frame1's in
        the rig frame.  Frames need BUILD_SENSOR_PYRAMID.  params None = RegisterPhotoICP()'s defaults."""
        init = _mat16(np.eye(4) if pose_estim is None else pose_estim)
        po = np.zeros(16, np.float32)
        info = np.ascontiguousarray(self.informationM.T).reshape(36).copy()
        self.dense_stats = DenseStats()
        rc = _check(lib().r360_register_dense(self.ctx.h, frame1.h, frame2.h, _fptr(init), method, registMode,
                                              None if params is None else C.byref(params), _fptr(po), _fptr(info),
                                              C.byref(self.dense_stats)), "RegisterDensePhotoICP")
        self.rigidTransf = _from16(po)
        if rc == 1:
            self.informationM = info.reshape(6, 6).T.copy()
        return rc == 1

    def eval_dense_robot(self, frame1, frame2, level: int, pose, method: int = PHOTO_CONSISTENCY,
                         params: "IcpParams | None" = None):
        """Per-sensor calcPhotoICPError_robot / calcHessianGradient_robot at `pose` on one level ->
        dict(err_photo[8], err_depth[8], H[8,6,6], g[8,6], n_error[8], n_depth[8], n_vis[8])."""
        err, H, g = np.zeros(16), np.zeros(8 * 36), np.zeros(8 * 6)
        cnt = np.zeros(24, np.int32)
        _check(lib().r360_dense_robot_eval(self.ctx.h, frame1.h, frame2.h, level, _fptr(_mat16(pose)), method,
                                           None if params is None else C.byref(params), err.ctypes.data_as(_DP),
                                           H.ctypes.data_as(_DP), g.ctypes.data_as(_DP), cnt.ctypes.data_as(_IP)),
               "eval_dense_robot")
        c = cnt.reshape(8, 3)
        return dict(err_photo=err[0::2].copy(), err_depth=err[1::2].copy(), H=H.reshape(8, 6, 6), g=g.reshape(8, 6),
                    n_error=c[:, 0].copy(), n_depth=c[:, 1].copy(), n_vis=c[:, 2].copy())

    def getPose(self): return self.rigidTransf
    def getInfoMat(self): return self.informationM
    def getCovMat(self):
        """covarianceM = informationM.inverse() (:208-215)."""
        return np.linalg.inv(self.informationM.astype(np.float64)).astype(np.float32)

    def calcEntropy(self) -> float:
        """0.5 (DOF (1 + log 2 pi) + log det(covariance)) (:230-238), DOF = 6, PI = 3.14159265359."""
        det = np.float32(np.linalg.det(self.getCovMat().astype(np.float64)))
        return float(np.float32(0.5 * (6 * (1 + np.log(2 * 3.14159265359)) + np.log(det))))

    def trackingScore(self):
        """(quality, score) of trackingScore(float& score) (:526-540): score = areaMatched / areaSource;
        0 GOOD (>= 0.7), 1 WEAK (>= 0.3), 2 BAD."""
        score = float(np.float32(np.float32(self.getAreaMatched()) / np.float32(self.areaSource))) \
            if self.areaSource else float("nan")
        return (0 if score >= 0.7 else 1 if score >= 0.3 else 2), score

    def getMatchedPlanes(self): return dict(self.bestMatch)
    def getAreaMatched(self): return self.areaMatched

    def match_tables(self, mode: int = PLANAR_3DoF, cap: int = 128):
        """k_match_tables output for the current reference/target subgraphs (inspection)."""
        ns, nt = C.c_int(), C.c_int()
        sid, tid = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
        un = np.zeros(cap * cap, np.uint8)
        words = (cap * cap + 63) // 64
        bi = np.zeros(cap * cap * words, np.uint64)
        _check(lib().r360_ctx_set_match_params(self.ctx.h, C.byref(self.match)), "set_match_params")
        w = _check(lib().r360_pbmap_match_tables(self.ctx.h, self.ref.h, self.trg.h, self.max_match_planes, mode,
                                                 C.byref(ns), C.byref(nt), sid.ctypes.data_as(_IP),
                                                 tid.ctypes.data_as(_IP), _vptr(un), _vptr(bi), cap), "match_tables")
        n, m = ns.value, nt.value
        return dict(sid=sid[:n].copy(), tid=tid[:m].copy(), unary=un[:n * m].reshape(n, m).copy(),
                    binary=bi[:n * m * w].reshape(n * m, w).copy(), words=w)


def frames_build(frames, flags: int = None):
    """r360_frames_build: Frame360::getPlanes (Frame360.h:615-640) of several frames with their plane stages batched
    (up to 8 frames of one size per launch, on frames[0]'s context stream).  Same results as building each alone."""
    if flags is None:
        flags = BUILD_UNDISTORT | BUILD_CLOUD | BUILD_PLANES | BUILD_SPHERE | BUILD_PYRAMID
    arr = (C.c_void_p * len(frames))(*[f.h for f in frames])
    _check(lib().r360_frames_build(arr, len(frames), flags), "r360_frames_build")


def register(ctx: "Context", ref: "Frame360", trg: "Frame360", guess=None, params: "IcpParams | None" = None,
             max_match_planes: int = 25, mode: int = PLANAR_3DoF):
    """Register() alias: PbMap -> rotOffset conjugation -> alignFrames360 (OdometryKeyFrame360.cpp:248-254).
    Returns (pose, info, stats, pbmap_ok)."""
    g = _mat16(np.eye(4) if guess is None else guess)
    pose, info = np.zeros(16, np.float32), np.zeros(36, np.float32)
    st = IcpStats()
    p = params if params is not None else IcpParams.default()
    rc = _check(lib().r360_register(ctx.h, ref.h, trg.h, _fptr(g), C.byref(p), max_match_planes, mode, _fptr(pose),
                                    _fptr(info), C.byref(st)), "register")
    return _from16(pose), info.reshape(6, 6).T.copy(), st, rc == 0


class Batch:
    """Batched pair registrations (r360_batch, §8f-4): `lanes` worker contexts on one GPU run the jobs of a
    call concurrently.  Each job is the single-pair code path, so results equal the sequential calls.

    * ``register_pairs`` — generic jobs (RegisterPbMap, optionally gated / always refined by alignFrames360).
    * ``track`` — SphereGraphSLAM's tracking step (SLAM/SphereGraphSLAM.cpp:169-231).
    * ``loop_closures`` — LoopClosure360's candidate checks (include/LoopClosure360.h:280-366).
    """

    def __init__(self, device: int = 0, lanes: int = 8):
        h = C.c_void_p()
        _check(lib().r360_batch_create(device, lanes, C.byref(h)), "r360_batch_create")
        self.h = h
        self.lanes = lib().r360_batch_lanes(h)

    def register_pairs(self, jobs, max_match_planes: int = 25, mode: int = PLANAR_3DoF, min_matches: int = 0,
                       min_area: float = 0.0, params: "IcpParams | None" = None) -> list[dict]:
        """jobs: iterable of dicts {ref, trg, dense=JOB_PBMAP_ONLY, ref_is_source=False, guess=None}."""
        jobs = list(jobs)
        arr = (PairJob * max(1, len(jobs)))()
        for a, j in zip(arr, jobs):
            a.ref, a.trg = j["ref"].h.value, j["trg"].h.value
            a.dense = int(j.get("dense", JOB_PBMAP_ONLY))
            a.ref_is_source = int(bool(j.get("ref_is_source", False)))
            g = j.get("guess")
            a.guess[:] = [float(v) for v in _mat16(np.eye(4) if g is None else g)]
        out = (PairResult * max(1, len(jobs)))()
        p = params if params is not None else IcpParams.default()
        _check(lib().r360_batch_register(self.h, arr, len(jobs), max_match_planes, mode, min_matches, min_area,
                                         C.byref(p), out), "r360_batch_register")
        return [out[i].as_dict() for i in range(len(jobs))]

    def track(self, keyframes, frame, num_check: int = 5, no_assoc_threshold: int = 40, max_match_planes: int = 25,
              mode: int = PLANAR_ODOMETRY_3DoF):
        """Register `frame` against the newest keyframes (list, oldest first) -> (index into keyframes or -1,
        winner's result dict or None, every candidate's result in the reference's order)."""
        kfs = list(keyframes)
        ptrs = (C.c_void_p * max(1, len(kfs)))(*[k.h.value for k in kfs])
        m = min(len(kfs), num_check, no_assoc_threshold)
        res, cand = PairResult(), (PairResult * max(1, m))()
        chosen = C.c_int()
        _check(lib().r360_track_frame(self.h, ptrs, len(kfs), frame.h, num_check, no_assoc_threshold,
                                      max_match_planes, mode, C.byref(chosen), C.byref(res), cand), "r360_track_frame")
        return chosen.value, (res.as_dict() if chosen.value >= 0 else None), [cand[i].as_dict() for i in range(m)]

    def loop_closures(self, pairs, min_matches: int = 5, min_area: float = 15.0, ref_is_source: bool = True,
                      params: "IcpParams | None" = None, max_match_planes: int = 25) -> list[dict]:
        """pairs: [(keyframe, new_keyframe)].  RegisterPbMap PLANAR_3DoF, the matches/area gate
        (LoopClosure360.h:114-115, 298) and the alignFrames360 refinement of the pairs that pass."""
        jobs = [{"ref": a, "trg": b, "dense": JOB_GATED, "ref_is_source": ref_is_source} for a, b in pairs]
        return self.register_pairs(jobs, max_match_planes, PLANAR_3DoF, min_matches, min_area, params)

    def close(self):
        if self.h:
            lib().r360_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


MAX_BATCH_ALIGN = 16


def align360_batch(ctx: "Context", pairs, inits=None, method: int = PHOTO_CONSISTENCY, params: "IcpParams" = None):
    """Batched alignFrames360 (r360_align360_batch_*): pairs = [(target Frame360, source Frame360), ...] (at most
    MAX_BATCH_ALIGN), inits = per-pair 4x4 guesses (identity if None).  Every pair's result equals
    RegisterPhotoICP.alignFrames360 on that pair alone.  Returns (poses [n,4,4], H [n,6,6], g [n,6], stats list,
    illposed count)."""
    n = len(pairs)
    p = params or IcpParams.default()
    trg = (C.c_void_p * n)(*[t.h for t, _ in pairs])
    src = (C.c_void_p * n)(*[s.h for _, s in pairs])
    init = np.concatenate([_mat16(np.eye(4) if inits is None or inits[j] is None else inits[j]) for j in range(n)])
    init = np.ascontiguousarray(init, np.float32)
    _check(lib().r360_align360_batch_async(ctx.h, n, trg, src, _fptr(init), method, C.byref(p)),
           "r360_align360_batch_async")
    po, Ho, go = np.zeros(16 * n, np.float32), np.zeros(36 * n, np.float32), np.zeros(6 * n, np.float32)
    st = (IcpStats * n)()
    ill = _check(lib().r360_align360_batch_result(ctx.h, _fptr(po), _fptr(Ho), _fptr(go), st),
                 "r360_align360_batch_result")
    poses = np.stack([_from16(po[16 * j:16 * j + 16]) for j in range(n)])
    H = np.stack([Ho[36 * j:36 * j + 36].reshape(6, 6).T.copy() for j in range(n)])
    return poses, H, go.reshape(n, 6).copy(), list(st), ill


class DenseQueue:
    """The alignFrames360 stage of many concurrent registrations batched on one stream (r360_dense_queue):
    submit from any thread, collect by ticket; a job's result equals the single-pair alignment."""

    def __init__(self, device: int = 0, max_batch: int = MAX_BATCH_ALIGN):
        h = C.c_void_p()
        _check(lib().r360_dense_queue_create(device, max_batch, C.byref(h)), "r360_dense_queue_create")
        self.h, self.device = h, device
        ctx = Context.__new__(Context)      # non-owning view of the queue's own context (timing reads)
        ctx.h, ctx.device = C.c_void_p(lib().r360_dense_queue_ctx(h)), device
        ctx.close = lambda: None
        self.ctx = ctx

    @classmethod
    def _view(cls, h, device: int) -> "DenseQueue":
        """A non-owning view of a dense queue the library owns (a sequence runner's)."""
        q = cls.__new__(cls)
        q.h, q.device = h, device
        q.ctx = Context._view(C.c_void_p(lib().r360_dense_queue_ctx(h)), device)
        q.close = lambda: None
        return q

    def submit(self, trg: "Frame360", src: "Frame360", init=None, method: int = PHOTO_DEPTH,
               params: "IcpParams" = None) -> int:
        t = C.c_long()
        i16 = _mat16(np.eye(4) if init is None else init)
        _check(lib().r360_dense_queue_submit(self.h, trg.h, src.h, _fptr(i16), method,
                                             C.byref(params or IcpParams.default()), C.byref(t)), "dense submit")
        return t.value

    def collect(self, ticket: int):
        po, Ho, go = np.zeros(16, np.float32), np.zeros(36, np.float32), np.zeros(6, np.float32)
        st = IcpStats()
        rc = _check(lib().r360_dense_queue_collect(self.h, ticket, _fptr(po), _fptr(Ho), _fptr(go), C.byref(st)),
                    "dense collect")
        return _from16(po), Ho.reshape(6, 6).T.copy(), go, st, rc

    def stats(self):
        b, j, m = C.c_long(), C.c_long(), C.c_int()
        _check(lib().r360_dense_queue_stats(self.h, C.byref(b), C.byref(j), C.byref(m)), "dense stats")
        return {"batches": b.value, "jobs": j.value, "max_batch": m.value}

    def close(self):
        if self.h:
            lib().r360_dense_queue_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RegisterPhotoICP:
    """RegisterPhotoICP spherical path (include/RegisterPhotoICP.h), frames stay in HBM."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.params = IcpParams.default()
        self.src = self.trg = None
        self.relPose = np.eye(4, dtype=np.float32)
        self.hessian = np.zeros((6, 6), np.float32)
        self.gradient = np.zeros(6, np.float32)
        self.stats = IcpStats()
        # public members (:180-192); the reference leaves the residuals uninitialised until an error function
        # that assigns them runs (NaN here)
        self.avResidual = self.avPhotoResidual = self.avDepthResidual = float("nan")
        self.SSO = 0.0
        self._own = {}         # sphere-only frames for spheres given as images, per (role, size)

    def _residuals(self):
        if self.stats.residuals_set & 1:
            self.avPhotoResidual = self.stats.av_photo_residual
            self.avDepthResidual = self.stats.av_depth_residual
        if self.stats.residuals_set & 2:
            self.avResidual = self.stats.av_residual
        self.SSO = self.stats.sso

    def setVisualization(self, b: bool):
        """visualizeIterations (OpenCV windows): no display here."""
        self.visualize = bool(b)

    # setters (:224-269)
    def setNumPyr(self, n: int): self.params.n_pyr = n
    def setMinDepth(self, d: float): self.params.min_depth = d
    def setMaxDepth(self, d: float): self.params.max_depth = d
    def setGrayVariance(self, s: float): self.params.std_dev_photo = s
    def setDepthVariance(self, s: float): self.params.std_dev_depth = s

    def useSaliency(self, b: bool):
        if b:
            raise NotImplementedError("saliency subsampling is commented out in the reference's sphere path")

    def _sphere_frame(self, role: str, bgr, range_mm) -> Frame360:
        H, W = np.asarray(range_mm).shape
        key = (role, H, W)
        if key not in self._own:
            cal = Calib360.for_sphere(self.ctx, H, W)
            self._own[key] = (cal, Frame360(cal))
        f = self._own[key][1]
        f.set_sphere(bgr, range_mm)
        return f

    def setSourceFrame(self, f, imgDepth=None):
        """setSourceFrame(Frame360) — the frame's sphere and pyramid in HBM — or setSourceFrame(imgRGB,
        imgDepth) with the sphere as images (BGR u8 [H, W, 3], range u16 mm [H, W]; :496-516)."""
        self.src = f if imgDepth is None else self._sphere_frame("src", f, imgDepth)

    def setTargetFrame(self, f, imgDepth=None):
        """setTargetFrame(Frame360) or setTargetFrame(imgRGB, imgDepth) (:480-494)."""
        self.trg = f if imgDepth is None else self._sphere_frame("trg", f, imgDepth)

    def alignFrames360(self, pose_guess=None, method: int = PHOTO_CONSISTENCY, occlusion: int = 0) -> int:
        init = _mat16(np.eye(4) if pose_guess is None else pose_guess)
        po, Ho, go = np.zeros(16, np.float32), np.zeros(36, np.float32), np.zeros(6, np.float32)
        rc = _check(lib().r360_align360(self.ctx.h, self.trg.h, self.src.h, _fptr(init), method, occlusion,
                                        C.byref(self.params), _fptr(po), _fptr(Ho), _fptr(go),
                                        C.byref(self.stats)), "alignFrames360")
        self._residuals()
        self.relPose = _from16(po)
        self.hessian = Ho.reshape(6, 6).T.copy()
        self.gradient = go.copy()
        return rc

    def getOptimalPose(self): return self.relPose
    def getHessian(self): return self.hessian
    def getGradient(self): return self.gradient

    # ---- pinhole per-sensor path (§8(f) rank 3): alignFrames (:4254-4512) on sensor images
    def setCameraMatrix(self, K):
        """cameraMatrix (3x3); None = the calibration's (f = 525*cols/640, c = (cols/2-0.5, rows/2-0.5))."""
        self.K = None if K is None else np.array([K[0][0], K[1][1], K[0][2], K[1][2]], np.float32)

    def setSourceSensor(self, f: Frame360, sensor: int):
        """setSourceFrame(frameRGBD_[sensor].getRGBImage(), getDepthImage()) (:496-516)."""
        self.src, self.src_sensor = f, sensor

    def setTargetSensor(self, f: Frame360, sensor: int):
        """setTargetFrame(frameRGBD_[sensor].getRGBImage(), getDepthImage()) (:480-494)."""
        self.trg, self.trg_sensor = f, sensor

    def _K(self):
        k = getattr(self, "K", None)
        return None if k is None else _fptr(k)

    def alignFrames(self, pose_guess=None, method: int = PHOTO_CONSISTENCY, occlusion: int = 0) -> int:
        if occlusion:
            raise NotImplementedError("pinhole alignFrames: occlusion variants 1/2 are not built")
        if self.src_sensor != self.trg_sensor:
            raise ValueError("source and target sensors differ")
        init = _mat16(np.eye(4) if pose_guess is None else pose_guess)
        po, Ho, go = np.zeros(16, np.float32), np.zeros(36, np.float32), np.zeros(6, np.float32)
        rc = _check(lib().r360_align_pinhole(self.ctx.h, self.trg.h, self.src.h, self.src_sensor, _fptr(init), method,
                                             self._K(), C.byref(self.params), _fptr(po), _fptr(Ho), _fptr(go),
                                             C.byref(self.stats)), "alignFrames")
        self._residuals()
        self.relPose = _from16(po)
        self.hessian = Ho.reshape(6, 6).T.copy()
        self.gradient = go.copy()
        return rc

    def alignSensors(self, trg: Frame360, src: Frame360, sensors, pose_guesses, method: int = PHOTO_DEPTH):
        """alignFrames on several sensors of one pair at once (one batched pass sequence).
        Returns (poses [n,4,4], hessians [n,6,6], stats list, n_illposed)."""
        sensors = np.ascontiguousarray(sensors, np.int32)
        n = len(sensors)
        init = np.concatenate([_mat16(P) for P in pose_guesses]).astype(np.float32)
        _check(lib().r360_align_pinhole_async(self.ctx.h, trg.h, src.h, n, sensors.ctypes.data_as(_IP), _fptr(init),
                                              method, self._K(), C.byref(self.params)), "alignSensors")
        po, Ho, go = np.zeros(16 * n, np.float32), np.zeros(36 * n, np.float32), np.zeros(6 * n, np.float32)
        st = (IcpStats * n)()
        ill = _check(lib().r360_align_pinhole_result(self.ctx.h, _fptr(po), _fptr(Ho), _fptr(go), st),
                     "alignSensors")
        poses = np.stack([_from16(po[16 * j:16 * j + 16]) for j in range(n)])
        Hs = np.stack([Ho[36 * j:36 * j + 36].reshape(6, 6).T for j in range(n)])
        return poses, Hs, list(st), ill

    def eval_pinhole(self, level: int, pose, method: int = PHOTO_DEPTH):
        """One errorPhotoICP + calcHessGrad pass -> dict(H, g, error, res_photo, res_depth, n_photo, n_depth, n_vis)."""
        H, g = np.zeros(36), np.zeros(6)
        err, res = C.c_double(), np.zeros(2)
        cnt = np.zeros(3, np.int32)
        _check(lib().r360_pinhole_eval(self.ctx.h, self.trg.h, self.src.h, self.src_sensor, level, _fptr(_mat16(pose)),
                                       method, self._K(), C.byref(self.params), H.ctypes.data_as(_DP),
                                       g.ctypes.data_as(_DP), C.byref(err), res.ctypes.data_as(_DP),
                                       cnt.ctypes.data_as(_IP)), "eval_pinhole")
        return dict(H=H.reshape(6, 6), g=g, error=err.value, res_photo=res[0], res_depth=res[1], n_photo=int(cnt[0]),
                    n_depth=int(cnt[1]), n_vis=int(cnt[2]))

    def eval(self, level: int, pose, method: int = PHOTO_DEPTH):
        """One fused errorPhotoICP_sphere + calcHessGrad_sphere pass at a fixed pose."""
        p = _mat16(pose)
        H, g = np.zeros(36), np.zeros(6)
        e2, nv, nvis = C.c_double(), C.c_int(), C.c_int()
        _check(lib().r360_icp_eval(self.ctx.h, self.trg.h, self.src.h, level, _fptr(p), method,
                                   C.byref(self.params), H.ctypes.data_as(_DP), g.ctypes.data_as(_DP),
                                   C.byref(e2), C.byref(nv), C.byref(nvis)), "icp_eval")
        return H.reshape(6, 6), g, e2.value, nv.value, nvis.value

    def eval_occ(self, level: int, pose, method: int = PHOTO_DEPTH, occlusion: int = 1):
        """One occlusion-aware pass at a fixed pose: H, g of calcHessGrad_sphereOcc{occlusion}, the value
        of errorPhotoICP_sphereOcc{occlusion}, its point count and numVisiblePixels."""
        p = _mat16(pose)
        H, g = np.zeros(36), np.zeros(6)
        e, nv, nvis = C.c_double(), C.c_int(), C.c_int()
        _check(lib().r360_icp_eval_occ(self.ctx.h, self.trg.h, self.src.h, level, _fptr(p), method, occlusion,
                                       C.byref(self.params), H.ctypes.data_as(_DP), g.ctypes.data_as(_DP),
                                       C.byref(e), C.byref(nv), C.byref(nvis)), "icp_eval_occ")
        return H.reshape(6, 6), g, e.value, nv.value, nvis.value


def match_tree_search(unary: np.ndarray, binary: np.ndarray, area, max_nodes: int = 4000000):
    """The interpretation-tree search alone (host only): unary [ns, nt] bool, binary [ns * nt, words] uint64 (bit k * nt
    + l of row i * nt + j: references i, k matched to targets j, l are consistent), area [ns].  Returns (best [ns]
    target or -1, nodes, truncated)."""
    unary = np.ascontiguousarray(unary, np.uint8)
    ns, nt = unary.shape
    words = (ns * nt + 63) // 64
    binary = np.ascontiguousarray(binary, np.uint64).reshape(ns * nt, words) if ns * nt else np.zeros((0, 0), np.uint64)
    area = np.ascontiguousarray(area, np.float64)
    best = np.zeros(max(ns, 1), np.int32)
    nodes = C.c_long()
    rc = _check(lib().r360_match_tree_search(ns, nt, _vptr(unary), _vptr(binary), words, _vptr(area), max_nodes,
                                             _vptr(best), C.byref(nodes)), "match_tree_search")
    return best[:ns], nodes.value, bool(rc)


def refine_eval(state: np.ndarray, mask: np.ndarray, rb: int = 0, return_fallbacks: bool = False):
    """refine()'s two sweeps on the device (parity hook): state int8 (8, h, w), mask uint64 (8, h, w); rb = -1 the
    wavefront sweeps (the default path; LDS-pipelined 64-row bands for h <= 512), -2 the barrier-per-diagonal
    wavefront, 0 the single-wave sweeps, rb > 0 banded.  With return_fallbacks, also the
    number of sensors whose wavefront second sweep needed wrap-push corrections (re-runs or the fallback)."""
    state = np.ascontiguousarray(state, np.int8)
    mask = np.ascontiguousarray(mask, np.uint64)
    _, h, w = state.shape
    out = np.zeros_like(state)
    nfb = _check(lib().r360_refine_eval(state.ctypes.data, mask.ctypes.data, w, h, rb, out.ctypes.data),
                 "r360_refine_eval")
    return (out, nfb) if return_fallbacks else out


def libm_eval(x, y, z, on_device: bool = False):
    """Evaluate the projection's asinf / atan2f port (libm_f32.h) on the host or the GPU."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    a, t = np.zeros_like(x), np.zeros_like(x)
    _check(lib().r360_libm_eval(_fptr(x), _fptr(y), _fptr(z), x.size, _fptr(a), _fptr(t), int(on_device)),
           "libm_eval")
    return a, t


class Comm:
    """RCCL communicator of one rank (r360_comm): the sequence driver's record all_gather over xGMI.
    Rank 0 calls unique_id() and hands the bytes to the other ranks (e.g. over a gloo process group)."""

    @staticmethod
    def unique_id() -> bytes:
        b = (C.c_uint8 * 128)()
        _check(lib().r360_comm_unique_id(b), "comm_unique_id")
        return bytes(b)

    def __init__(self, device: int, nranks: int, rank: int, uid: bytes):
        assert len(uid) == 128
        self.nranks = nranks
        self.h = C.c_void_p()
        b = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().r360_comm_init(device, nranks, rank, b, C.byref(self.h)), "comm_init")

    def allgather(self, a: np.ndarray) -> np.ndarray:
        """(nranks,) + a.shape: every rank's array, in rank order."""
        a = np.ascontiguousarray(a)
        out = np.zeros((self.nranks,) + a.shape, a.dtype)
        _check(lib().r360_comm_allgather(self.h, _vptr(a), _vptr(out), a.nbytes), "comm_allgather")
        return out

    def allreduce_max(self, v: float) -> float:
        x = np.array([v], np.float64)
        _check(lib().r360_comm_allreduce_max(self.h, x.ctypes.data_as(_DP), 1), "comm_allreduce_max")
        return float(x[0])

    def close(self):
        if self.h:
            lib().r360_comm_destroy(self.h)
            self.h = None


class DeviceArray:
    """A host array's copy resident in HBM (r360_dev_alloc); ptr(i) = device address of element i along
    the first axis."""

    def __init__(self, device: int, a: np.ndarray):
        a = np.ascontiguousarray(a)
        self.nbytes, self.row = a.nbytes, a[0].nbytes if a.ndim else a.nbytes
        self.p = C.c_void_p()
        _check(lib().r360_dev_alloc(device, self.nbytes, C.byref(self.p)), "dev_alloc")
        _check(lib().r360_dev_copy(self.p, _vptr(a), self.nbytes, 0), "dev_copy")

    def ptr(self, i: int = 0) -> int:
        return self.p.value + i * self.row

    def close(self):
        if self.p:
            lib().r360_dev_free(self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostPinned:
    """Page-locks numpy arrays for asynchronous uploads (hipHostRegister); released by close()."""

    def __init__(self, *arrays):
        self.arrays = []
        for a in arrays:
            assert a.flags.c_contiguous
            _check(lib().r360_host_register(_vptr(a), a.nbytes), "host_register")
            self.arrays.append(a)

    def close(self):
        for a in self.arrays:
            lib().r360_host_unregister(_vptr(a))
        self.arrays = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_frame_rt(rows: int, cols: int, rt8: np.ndarray, seed: int, rig_pose: np.ndarray):
    """Host-only synthetic frame (no GPU): rt8 = (8, 4, 4) extrinsics."""
    bgr = np.zeros((8, rows, cols, 3), np.uint8)
    dep = np.zeros((8, rows, cols), np.uint16)
    rt = np.ascontiguousarray(np.stack([_mat16(m) for m in rt8]), np.float32)
    p = _mat16(rig_pose)
    _check(lib().r360_synth_frame_rt(rows, cols, _fptr(rt), seed, _fptr(p), _vptr(bgr), _vptr(dep)), "synth_frame_rt")
    return bgr, dep


def synth_path_pose(seed: int, frame: int) -> np.ndarray:
    a = np.zeros(16, np.float32)
    lib().r360_synth_path_pose(seed, frame, _fptr(a))
    return _from16(a)


def exp_se3(mu, pseudo: bool = True) -> np.ndarray:
    m = np.asarray(mu, np.float64)
    T = np.zeros(16, np.float32)
    lib().r360_exp_se3(m.ctypes.data_as(_DP), int(pseudo), _fptr(T))
    return _from16(T)


DATA_DIR = os.path.join(REPO_ROOT, "data")
EXTRINSICS_DIR = os.path.join(DATA_DIR, "calib", "Extrinsics")   # Rt_0{1..8}.txt (reference rig)
INTRINSICS_DIR = os.path.join(DATA_DIR, "calib", "Intrinsics")   # CLAMS tables (compact form)
SAMPLES_DIR = os.path.join(DATA_DIR, "samples")                  # sphere_images_{1,10}.bin
