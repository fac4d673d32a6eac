"""Filter -- the reference's FOD-side filters that sit either side of the GICP path.

Mirrors the two Filter entry points SURVEY.md 8f names as the next rows of the hot path:
  * Filter::downsampleCloud (/root/reference/src/Filter.cpp:91-105): resolution log, VoxelGrid
    with a cubic leaf, resolution log -- the step feeding GICP in the state machine;
  * Filter::removeFromCloud (/root/reference/src/Filter.cpp:176-189): SegmentDifferences with a
    kd-tree search, called by FODDetectionState right after the GICP transform is applied
    (/root/reference/src/LeicaStateMachine.cpp:180-187).
Both run on the GPU through libmgicp.so (mgicp_voxel_grid, mgicp_segment_differences,
mgicp_cloud_resolution); there is no CPU path.  The crop-box / RANSAC-floor / outlier filters of
Filter are not on the GICP path and are out of scope.
"""
from __future__ import annotations

import logging

import numpy as np

from .cloud import PointCloudRGB
from .engine import GICPEngine

log = logging.getLogger(__name__)
_ENGINE: list = []


def _engine() -> GICPEngine:
    """One helper context per process (mgicp_create resolves every kernel once)."""
    if not _ENGINE:
        _ENGINE.append(GICPEngine())
    return _ENGINE[0]


class Filter:
    def __init__(self, leaf_size: float, noise_threshold: float = 0.0, floor_threshold: float = 0.0):
        self.leaf_size_ = float(leaf_size)
        self.noise_threshold_ = float(noise_threshold)
        self.floor_threshold_ = float(floor_threshold)

    def setLeafSize(self, leaf_size: float) -> None:
        self.leaf_size_ = float(leaf_size)

    def downsampleCloud(self, cloud: PointCloudRGB, cloud_downsampled: PointCloudRGB) -> None:
        """VoxelGrid<PointXYZRGB> with leaf (l, l, l) (Filter.cpp:91-105).  The leaf goes through
        Eigen::Vector4f, i.e. it is rounded to float before 1/leaf is taken."""
        e = _engine()
        log.info("Downsample cloud with leaf_size : %f", self.leaf_size_)
        log.info("Pointcloud resolution before downsampling: %f", e.cloud_resolution(cloud))
        leaf = float(np.float32(self.leaf_size_))
        out = e.voxel_grid(cloud, (leaf, leaf, leaf))
        cloud_downsampled.points = out.points
        log.info("Pointcloud resolution after downsampling: %f", e.cloud_resolution(cloud_downsampled))

    @staticmethod
    def removeFromCloud(input_cloud: PointCloudRGB, substract_cloud: PointCloudRGB, threshold: float,
                        cloud_filtered: PointCloudRGB, transform=None) -> None:
        """SegmentDifferences (Filter.cpp:176-189): the records of input_cloud whose nearest
        neighbour in substract_cloud has squared distance > threshold (PCL compares the value
        given to setDistanceThreshold with the squared distance).  `transform` optionally fuses
        the preceding pcl::transformPointCloud of LeicaStateMachine.cpp:182 (the input records
        are then output transformed, as the FSM's in-place transform would leave them)."""
        log.info("Difference from segment with threshold: %f", threshold)
        keep, _ = _engine().segment_differences(input_cloud, substract_cloud, threshold, T=transform)
        if transform is not None:
            moved = PointCloudRGB()
            _engine().transform_cloud(transform, input_cloud, moved)
            cloud_filtered.points = moved.points[keep].copy()
        else:
            cloud_filtered.points = input_cloud.points[keep].copy()
