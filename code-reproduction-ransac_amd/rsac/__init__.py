"""rsac -- MI355X-native RANSAC engine (PnP camera pose + homography).

Drop-in for the RANSAC hot path of Mendel0408/Code-Reproduction-RANSAC, whose
scripts call cv2.solvePnPRansac (main_v1.py:497) and cv2.findHomography
(main_v1.py:312).  The compute runs in hand-written HIP kernels for gfx950
(librsac.so, built from ../csrc) reached through a ctypes C ABI
(include/rsac.h).  See DESIGN.md.
"""
from ._lib import Context, RsacError, context, lib  # noqa: F401
from . import dem  # noqa: F401
from .api import (LocationResult, OrientationResult, RansacInfo, Scan, compute_reprojection_error,  # noqa: F401
                  epnp_minimal, epnp_pose, estimate_camera_orientation, evaluate_range, fundamental_ransac, homography_fit,
                  homography_ransac, homography_ransac_batched, hypotheses, intrinsics_grid, local_opt,
                  location_search, pnp_ransac, pnp_ransac_batched, pnp_ransac_first_round, pnp_ransac_batched_rows, pnp_ransac_batched_flat, pose_mask, refine_pose,
                  refine_pose_device, reprojection_errors, rodrigues, score_poses, update_num_iters, winner)

__all__ = ["pnp_ransac", "pnp_ransac_batched", "pnp_ransac_batched_flat", "homography_ransac", "homography_ransac_batched", "score_poses",
           "evaluate_range", "hypotheses", "pose_mask", "refine_pose", "homography_fit", "rodrigues", "update_num_iters",
           "location_search", "LocationResult", "local_opt", "dem", "epnp_minimal", "epnp_pose", "fundamental_ransac", "winner", "Scan", "Context", "context", "RsacError", "RansacInfo", "lib",
           "estimate_camera_orientation", "OrientationResult", "intrinsics_grid", "reprojection_errors",
           "compute_reprojection_error", "refine_pose_device", "pnp_ransac_first_round",
           "pnp_ransac_batched_rows"]
