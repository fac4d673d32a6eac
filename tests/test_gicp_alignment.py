"""GICPAlignment mirror: the reference's own test_gicp_alignment.cpp, plus the class-surface
quirks the drop-in must preserve.  GPU tests run through libmgicp.so
and compare with the oracle; CPU tests cover the host-side semantics."""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from conftest import frob


def _rgb(xyz):
    from leica_point_cloud_processing_amd.cloud import PointCloudRGB

    return PointCloudRGB.from_xyz(xyz)


# ------------------------------------------------------------------------------ CPU ------
def test_constructor_defaults(cube_clouds):
    """testApplyTF / testRun: ASSERT_EQ(getFineTransform(), Identity) right after the ctor."""
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment

    src, tgt, _ = cube_clouds
    a = GICPAlignment(_rgb(tgt), _rgb(src), False)
    assert np.array_equal(a.getFineTransform(), np.eye(4, dtype=np.float32))
    assert a.transform_exists_ is False
    assert (a.tf_epsilon_, a.max_iter_, a.max_corresp_distance_, a.ransac_outlier_th_) == (4e-3, 100, 4e-2, 1.0)


def test_int_setters_truncate():
    """setMaxCorrespondenceDistance(int) / setRANSACOutlierTh(int): 5e-2 -> 0 (GICPAlignment.h:138,145)."""
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment

    a = GICPAlignment(_rgb(np.zeros((1, 3))), _rgb(np.zeros((1, 3))), False)
    a.setMaxCorrespondenceDistance(5)
    a.setRANSACOutlierTh(5e-2)
    a.setTfEpsilon(5e-4)
    a.setMaxIterations(100)
    assert a.max_corresp_distance_ == 5.0
    assert a.ransac_outlier_th_ == 0.0
    a.setMaxCorrespondenceDistance(0.04)
    assert a.max_corresp_distance_ == 0.0
    assert a.tf_epsilon_ == 5e-4 and a.max_iter_ == 100


def test_undo_restores_backup():
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment

    a = GICPAlignment(_rgb(np.zeros((1, 3))), _rgb(np.zeros((1, 3))), False)
    first = _rgb(np.arange(12, dtype=np.float32).reshape(4, 3))
    a.aligned_cloud_.copy_from(first)
    a.backUp(a.aligned_cloud_)
    a.aligned_cloud_.points["x"] += 1
    a.undo()
    np.testing.assert_array_equal(a.aligned_cloud_.xyz(), first.xyz())


def test_cloud_layout_is_pcl_xyzrgb():
    from leica_point_cloud_processing_amd.cloud import POINT_XYZRGB

    assert POINT_XYZRGB.itemsize == 32
    assert [POINT_XYZRGB.fields[f][1] for f in ("x", "y", "z", "rgb")] == [0, 4, 8, 16]


# ------------------------------------------------------------------------------ GPU ------
@pytest.mark.gpu
def test_testApplyTF(cube_clouds):
    """test_gicp_alignment.cpp:50-75 at defaults; applyTFtoCloud writes aligned_cloud_, the
    argument stays untouched (the reference's x check therefore compares the raw source)."""
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment
    from leica_point_cloud_processing_amd.synth import transform_points

    src, tgt, Trot = cube_clouds
    sourceRGB, targetRGB = _rgb(src), _rgb(tgt)
    a = GICPAlignment(targetRGB, sourceRGB, False)
    a.run()
    before = sourceRGB.xyz()
    a.applyTFtoCloud(sourceRGB)
    np.testing.assert_array_equal(sourceRGB.xyz(), before)
    np.testing.assert_array_equal(a.aligned_cloud_.xyz(), transform_points(a.fine_tf_, src))
    assert a.transform_exists_
    assert np.abs(a.getFineTransform() - Trot).max() < 1e-4


@pytest.mark.gpu
def test_testRun(cube_clouds):
    """test_gicp_alignment.cpp:77-104 with its exact setter calls, checked against the oracle."""
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment
    from oracle import ref

    src, tgt, Trot = cube_clouds
    a = GICPAlignment(_rgb(tgt), _rgb(src), False)
    a.setMaxIterations(100)
    a.setMaxCorrespondenceDistance(5)
    a.setRANSACOutlierTh(5e-2)
    a.setTfEpsilon(5e-4)
    a.run()
    aligned = _rgb(np.zeros((0, 3)))
    a.getAlignedCloud(aligned)
    assert a.transform_exists_
    assert aligned.size() == len(src)
    o = ref.RefGICP(max_corr_dist=5.0, transformation_epsilon=5e-4)
    o.set_source(src)
    o.set_target(tgt)
    T_ref, _ = o.align()
    assert frob(a.getFineTransform(), T_ref) <= 1e-4
    msg = a.getAlignedCloudROSMsg()
    assert msg["width"] == len(src) and msg["point_step"] == 32


@pytest.mark.gpu
def test_testRunWithCov(cube_clouds):
    """test_gicp_alignment.cpp:106-131: run() with covariances, then iterate(): fine_tf_ becomes
    T*T (PCL re-registers the original source) and aligned_cloud_ = T * source."""
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment, matmul4f
    from leica_point_cloud_processing_amd.synth import transform_points

    src, tgt, _ = cube_clouds
    sourceRGB, targetRGB = _rgb(src), _rgb(tgt)
    a = GICPAlignment(targetRGB, sourceRGB, True)
    a.run()
    assert a.transform_exists_
    T = a.getFineTransform()
    a.iterate()
    assert a.transform_exists_
    np.testing.assert_array_equal(a.getFineTransform(), matmul4f(T, T))
    np.testing.assert_array_equal(a.aligned_cloud_.xyz(), transform_points(T, sourceRGB.xyz()))
    a.undo()  # back to the pre-iterate aligned cloud (T * source as well)
    np.testing.assert_array_equal(a.aligned_cloud_.xyz(), transform_points(T, sourceRGB.xyz()))


def _resolution_np(xyz):
    d, _ = cKDTree(xyz.astype(np.float64)).query(xyz.astype(np.float64), k=2)
    # re-evaluate the 2nd neighbour distance in float32 like FLANN, sqrt in float32
    _, idx = cKDTree(xyz.astype(np.float64)).query(xyz.astype(np.float64), k=2)
    diff = xyz - xyz[idx[:, 1]]
    d2 = diff[:, 0] * diff[:, 0]
    d2 = d2 + diff[:, 1] * diff[:, 1]
    d2 = d2 + diff[:, 2] * diff[:, 2]
    return float(np.sqrt(d2).astype(np.float64).mean())


@pytest.mark.gpu
def test_covariance_path_filter(part_small):
    """computeCloudResolution + the NaN-normal radius filter against brute force on the CPU."""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = part_small
    e = GICPEngine()
    res = e.cloud_resolution(scan)
    assert abs(res - _resolution_np(scan)) <= 1e-9 * res
    # sparse cloud so that some points have < 3 neighbours within the radius
    rng = np.random.default_rng(11)
    pts = rng.random((4000, 3)).astype(np.float32)
    radius = 0.05
    keep = e.radius_filter(pts, radius, 3)
    tree = cKDTree(pts.astype(np.float64))
    cand = tree.query_ball_point(pts.astype(np.float64), radius * 1.001)
    r2 = np.float32(radius * radius)
    exp = np.zeros(len(pts), bool)
    for i, c in enumerate(cand):
        d = pts[i] - pts[np.asarray(c)]
        d2 = d[:, 0] * d[:, 0]
        d2 = d2 + d[:, 1] * d[:, 1]
        d2 = d2 + d[:, 2] * d[:, 2]
        exp[i] = int((d2 < r2).sum()) >= 3
    np.testing.assert_array_equal(keep, exp)
    assert 0 < exp.sum() < len(pts)


@pytest.mark.gpu
def test_covariance_path_nonfinite_records(part_small):
    """non-finite records on the use_covariances path.  Utils::computeCloudResolution
    skips them as queries and its KdTree never holds them (src/Utils.cpp:152-160);
    NormalEstimation gives them NaN normals, so getCovariances drops them (GICPAlignment.cpp:62-67).
    The GICP that follows then runs on finite clouds (PCL: same as the oracle on the kept points)."""
    from leica_point_cloud_processing_amd.engine import GICPEngine
    from leica_point_cloud_processing_amd.gicp_alignment import GICPAlignment
    from oracle import ref

    scan, cad, _ = part_small
    bad = scan.copy()
    rng = np.random.default_rng(3)
    idx = rng.choice(len(bad), 50, replace=False)
    bad[idx[:20], 0] = np.nan
    bad[idx[20:35], 1] = np.inf
    bad[idx[35:], 2] = -np.nan
    finite = np.isfinite(bad).all(axis=1)
    e = GICPEngine()
    res = e.cloud_resolution(bad)
    assert abs(res - _resolution_np(bad[finite])) <= 1e-9 * res
    radius = 2.0 * (res + e.cloud_resolution(cad)) * 0.25  # small: some finite points lose the test
    keep = e.radius_filter(bad, radius, 3)
    assert not keep[~finite].any()
    keep_f = e.radius_filter(bad[finite], radius, 3)
    np.testing.assert_array_equal(keep[finite], keep_f)
    assert e.cloud_resolution(np.full((5, 3), np.nan, np.float32)) == 0.0
    # the class path: both clouds filtered in place, then GICP on the finite remainder
    a = GICPAlignment(_rgb(cad), _rgb(bad), True)
    a.run()
    assert a.transform_exists_
    kept_src = a.source_cloud_.xyz()
    assert np.isfinite(kept_src).all() and len(kept_src) <= finite.sum()
    o = ref.RefGICP()
    o.set_source(kept_src)
    o.set_target(a.target_cloud_.xyz())
    T_ref, _ = o.align()
    assert frob(a.getFineTransform(), T_ref) <= 1e-4


@pytest.mark.gpu
def test_seeded_debug_after_new_target_is_refused(part_small):
    """a seeded sweep must never seed from the previous target's sorted positions."""
    from leica_point_cloud_processing_amd import _lib
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = part_small
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    e.debug_correspondences(np.eye(4, dtype=np.float32), len(scan))
    e.set_target_xyz(cad[:1000])
    with pytest.raises(_lib.MgicpError) as ei:
        e.debug_correspondences_seeded(np.eye(4, dtype=np.float32), len(scan))
    assert ei.value.code == _lib.MGICP_E_INVALID
    with pytest.raises(_lib.MgicpError):
        e.debug_moments(np.eye(4, dtype=np.float32))
    m, tj, _ = e.debug_correspondences(np.eye(4, dtype=np.float32), len(scan))  # unseeded: fine
    assert tj.max() < 1000
    e.close()
