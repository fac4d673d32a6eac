"""pcl::PointCloud<pcl::PointXYZRGB> stand-in with the exact 32-byte record layout.

The reference passes `PointCloudRGB::Ptr` (boost::shared_ptr) everywhere on the GICP path
(/root/reference/include/GICPAlignment.h:35,47,89,103,110,117).  A Python object reference
gives the same sharing semantics; `points` is a numpy structured array whose records match
pcl::PointXYZRGB in memory: x, y, z at bytes 0/4/8, data[3] at 12, rgb at 16, 12 bytes pad.
That lets the C-ABI read xyz in place with a 32-byte stride.
"""
from __future__ import annotations

import numpy as np

POINT_XYZRGB = np.dtype(
    {
        "names": ["x", "y", "z", "w", "rgb", "_pad"],
        "formats": ["<f4", "<f4", "<f4", "<f4", "<u4", ("<u4", 3)],
        "offsets": [0, 4, 8, 12, 16, 20],
        "itemsize": 32,
    }
)
assert POINT_XYZRGB.itemsize == 32


class PointCloudRGB:
    """Minimal PointCloud<PointXYZRGB>: `points` (structured array), width/height, copy helpers."""

    def __init__(self, n: int = 0):
        self.points = np.zeros(n, dtype=POINT_XYZRGB)
        self.points["w"] = 1.0

    # -- construction -----------------------------------------------------------------
    @classmethod
    def from_xyz(cls, xyz, rgb: int = 0) -> "PointCloudRGB":
        xyz = np.asarray(xyz, dtype=np.float32).reshape(-1, 3)
        c = cls(len(xyz))
        c.points["x"] = xyz[:, 0]
        c.points["y"] = xyz[:, 1]
        c.points["z"] = xyz[:, 2]
        c.points["rgb"] = rgb
        return c

    def xyz(self) -> np.ndarray:
        """(n, 3) float32 copy of the coordinates."""
        return np.stack([self.points["x"], self.points["y"], self.points["z"]], axis=1).astype(np.float32)

    # -- pcl-like API ------------------------------------------------------------------
    def size(self) -> int:
        return int(self.points.shape[0])

    __len__ = size

    @property
    def width(self) -> int:
        return self.size()

    @property
    def height(self) -> int:
        return 1

    def copy_from(self, other: "PointCloudRGB") -> None:
        """pcl::copyPointCloud(other, *this)."""
        self.points = other.points.copy()

    def extract(self, indices) -> None:
        """In place ExtractIndices (keep `indices`), as Filter::extractIndices(cloud, cloud, idx)."""
        self.points = self.points[np.asarray(indices, dtype=np.int64)].copy()

    def ctypes_xyz(self):
        """(pointer, n, stride) for the C-ABI; the array must be C-contiguous."""
        if not self.points.flags["C_CONTIGUOUS"]:
            self.points = np.ascontiguousarray(self.points)
        return self.points.ctypes.data, self.size(), POINT_XYZRGB.itemsize
