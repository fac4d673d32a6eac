"""GICPAlignment -- the reference class surface over the MI355X engine.

Mirrors /root/reference/include/GICPAlignment.h:32-224 and src/GICPAlignment.cpp:23-198
member for member (same names, argument meaning, defaults and quirks), with
pcl::GeneralizedIterativeClosestPoint replaced by GICPEngine (libmgicp.so):

* ctor(target, source, use_covariances) -- TARGET FIRST (GICPAlignment.h:47);
  defaults tf_epsilon 4e-3, max_iter 100, max_corresp_distance 0.04, ransac 1.0 (.cpp:29-32)
* run() = configParameters -> [applyCovariances] -> fineAlignment -> applyTFtoCloud(source)
* iterate() re-aligns the ORIGINAL source (PCL reuses its trees/covariances) and composes
  fine_tf_ = T * fine_tf_ (.cpp:111-121)
* applyTFtoCloud(cloud) writes the member aligned_cloud_, not `cloud` (.cpp:144-147)
* setMaxCorrespondenceDistance / setRANSACOutlierTh take ints: doubles truncate (GICPAlignment.h:138,145)
* use_covariances=True only filters NaN-normal points out of both clouds IN PLACE; the
  approximate covariances PCL computes are discarded by setInputSource/Target (.cpp:56-90)
"""
from __future__ import annotations

import logging
import time

import numpy as np

from .cloud import POINT_XYZRGB, PointCloudRGB
from .engine import GICPEngine

log = logging.getLogger("leica_point_cloud_processing_amd.GICPAlignment")


def is_valid_transform(T) -> bool:
    """Utils::isValidTransform (src/Utils.cpp:71-82): no NaN entry."""
    return not bool(np.isnan(np.asarray(T, dtype=np.float32)).any())


def matmul4f(a, b) -> np.ndarray:
    """Eigen Matrix4f * Matrix4f (column packets): ((a0 b0j + a1 b1j) + a2 b2j) + a3 b3j, float32."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    out = np.empty((4, 4), dtype=np.float32)
    for j in range(4):
        acc = a[:, 0] * b[0, j]
        acc = acc + a[:, 1] * b[1, j]
        acc = acc + a[:, 2] * b[2, j]
        out[:, j] = acc + a[:, 3] * b[3, j]
    return out


def _c_int(x) -> int:
    """C++ implicit double -> int conversion (truncation toward zero)."""
    return int(x)


class GICPAlignment:
    def __init__(self, target_cloud: PointCloudRGB, source_cloud: PointCloudRGB, use_covariances: bool,
                 device: int = -1):
        self.aligned_cloud_ = PointCloudRGB()
        self.backup_cloud_ = PointCloudRGB()
        self.target_cloud_ = target_cloud
        self.source_cloud_ = source_cloud
        self.covariances_ = bool(use_covariances)
        self.tf_epsilon_ = 4e-3
        self.max_iter_ = 100
        self.max_corresp_distance_ = 4e-2
        self.ransac_outlier_th_ = 1.0
        self.transform_exists_ = False
        self.fine_tf_ = np.eye(4, dtype=np.float32)
        self._device = device
        self._gicp = None  # the GPU context is created on first use

    # ------------------------------------------------------------------ engine ----------
    @property
    def gicp_(self) -> GICPEngine:
        if self._gicp is None:
            self._gicp = GICPEngine(device=self._device)
            self._apply_config()
        return self._gicp

    # ------------------------------------------------------------------ public ----------
    def run(self) -> None:
        self.configParameters()
        if self.covariances_:
            self.applyCovariances()
        self.fineAlignment()
        self.applyTFtoCloud(self.source_cloud_)

    def iterate(self) -> None:
        self.iterateFineAlignment(self.aligned_cloud_)

    def undo(self) -> None:
        self.aligned_cloud_.copy_from(self.backup_cloud_)

    def getFineTransform(self) -> np.ndarray:
        if not self.transform_exists_:
            log.error("No transform yet. Please run algorithm")
        return self.fine_tf_.copy()

    def getAlignedCloud(self, aligned_cloud: PointCloudRGB) -> None:
        aligned_cloud.copy_from(self.aligned_cloud_)

    def getAlignedCloudROSMsg(self) -> dict:
        """Utils::cloudToROSMsg -> sensor_msgs/PointCloud2 fields (pcl::toROSMsg layout)."""
        pts = self.aligned_cloud_.points
        return {
            "height": 1, "width": len(pts), "is_bigendian": False, "point_step": POINT_XYZRGB.itemsize,
            "row_step": POINT_XYZRGB.itemsize * len(pts), "is_dense": True,
            "fields": [("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1), ("rgb", 16, 7, 1)],
            "data": pts.tobytes(),
        }

    def applyTFtoCloud(self, cloud: PointCloudRGB) -> None:
        # pcl::transformPointCloud(*cloud, *aligned_cloud_, fine_tf_) -- writes the member
        self.gicp_.transform_cloud(self.fine_tf_, cloud, self.aligned_cloud_)

    def setSourceCloud(self, source_cloud: PointCloudRGB) -> None:
        self.source_cloud_ = source_cloud

    def setTargetCloud(self, target_cloud: PointCloudRGB) -> None:
        self.target_cloud_ = target_cloud

    def setMaxIterations(self, iterations: int) -> None:
        self.max_iter_ = _c_int(iterations)
        self.configParameters()

    def setTfEpsilon(self, tf_epsilon: float) -> None:
        self.tf_epsilon_ = float(tf_epsilon)
        self.configParameters()

    def setMaxCorrespondenceDistance(self, max_corresp_distance: int) -> None:
        self.max_corresp_distance_ = float(_c_int(max_corresp_distance))
        self.configParameters()

    def setRANSACOutlierTh(self, ransac_threshold: int) -> None:
        self.ransac_outlier_th_ = float(_c_int(ransac_threshold))
        self.configParameters()

    # ------------------------------------------------------------------ private ---------
    def configParameters(self) -> None:
        # parameters live in the members; they reach the GPU context now if it exists, or when
        # it is created on first use (so constructing / configuring needs no device)
        if self._gicp is not None:
            self._apply_config()

    def _apply_config(self) -> None:
        g = self._gicp
        g.setMaximumIterations(self.max_iter_)
        g.setMaxCorrespondenceDistance(self.max_corresp_distance_)
        g.setTransformationEpsilon(self.tf_epsilon_)
        g.setRANSACOutlierRejectionThreshold(self.ransac_outlier_th_)

    def getCovariances(self, cloud: PointCloudRGB) -> None:
        """Resolution of both clouds -> normal radius -> drop NaN-normal points from `cloud`
        in place (src/GICPAlignment.cpp:56-71).  The approximate covariances themselves are
        not computed: setInputSource/Target discard them before align."""
        g = self.gicp_
        target_res = g.cloud_resolution(self.target_cloud_)
        source_res = g.cloud_resolution(self.source_cloud_)
        normal_radius = (target_res + source_res) * 2.0
        log.info("Computing normals with radius: %f", normal_radius)
        keep = g.radius_filter(cloud, normal_radius, 3)
        cloud.extract(np.nonzero(keep)[0])

    def applyCovariances(self) -> None:
        log.info("Extract covariances from clouds")
        self.getCovariances(self.source_cloud_)
        self.getCovariances(self.target_cloud_)

    def fineAlignment(self) -> None:
        g = self.gicp_
        log.info("Perform GICP with %d iterations", g.getMaximumIterations())
        g.setInputSource(self.source_cloud_)
        g.setInputTarget(self.target_cloud_)
        begin = time.perf_counter()
        aligned_cloud = PointCloudRGB()
        log.info("This step may take a while ...")
        g.align(aligned_cloud)
        log.info("GICP time: %f s", time.perf_counter() - begin)
        if g.hasConverged():
            log.info("Converged in %f FitnessScore", g.getFitnessScore())
            self.fine_tf_ = g.getFinalTransformation()
            self.transform_exists_ = is_valid_transform(self.fine_tf_)
        else:
            log.error("GICP no converge")

    def iterateFineAlignment(self, cloud: PointCloudRGB) -> None:
        self.backUp(cloud)
        log.info("Computing iteration...")
        g = self.gicp_
        g.align(cloud)
        if g.hasConverged():
            temp_tf = g.getFinalTransformation()
            self.fine_tf_ = matmul4f(temp_tf, self.fine_tf_)
            log.info("%s", self.fine_tf_)
            log.info("Converged in %f FitnessScore", g.getFitnessScore())
        else:
            log.error("GICP no converge")

    def backUp(self, cloud: PointCloudRGB) -> None:
        self.backup_cloud_.copy_from(cloud)
