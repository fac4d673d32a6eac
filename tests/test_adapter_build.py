"""The drop-in adapter passes a real compiler and runs (VERDICT r01 "Compile the drop-in").

adapter/GICPAlignment.cpp (replaces /root/reference/src/GICPAlignment.cpp) and
adapter/Filter_mi355x.cpp (the Filter::downsampleCloud / removeFromCloud bodies) are compiled with
g++ -std=c++14 -Wall -Wextra -Werror against layout-exact stand-ins of pcl::PointXYZRGB,
pcl::PointCloud, Eigen::Matrix4f, ros::Time / ROS_*, sensor_msgs::PointCloud2 and the reference's
Utils / Filter headers (tests/adapter_standins), and linked to libmgicp.so together with a replay of
test/test_gicp_alignment.cpp:50-131 (`make adapter-replay`).
  * CPU: the build itself, and the no-device path (construct, run -> transform_exists_ false);
  * GPU: the replay of testApplyTF / testRun / testRunWithCov through the adapter CLASS, its
    transforms compared with the oracle, plus the Filter members.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, frob

REPLAY = os.path.join(ROOT, "adapter", "build", "replay_test_gicp_alignment")


def _parse(out: str):
    tfs, checks = {}, {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 20 and parts[1] == "T":
            tfs[parts[0]] = (np.array([float(v) for v in parts[2:18]], np.float32).reshape(4, 4).T, parts[19] == "1")
        elif len(parts) == 2 and parts[1] in ("ok", "FAIL"):
            checks[parts[0]] = parts[1] == "ok"
    return tfs, checks


def test_adapter_compiles_against_standins():
    r = subprocess.run(["make", "-s", "-C", ROOT, "adapter-replay"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(REPLAY)
    nm = subprocess.run(["nm", "-C", REPLAY], capture_output=True, text=True).stdout
    for sym in ("GICPAlignment::run()", "GICPAlignment::iterate()", "GICPAlignment::applyTFtoCloud",
                "Filter::downsampleCloud", "Filter::removeFromCloud"):
        assert sym in nm, sym


def test_adapter_without_device_fails_soft():
    """No HIP device (this container): the class still constructs and run() ends with
    transform_exists_ == false and an error log -- the adapter's mirror of PCL's caught solver
    exception; nothing throws across the ROS callback."""
    if os.path.exists("/dev/kfd"):  # the ROCm kernel driver: a GPU may be visible
        pytest.skip("a GPU is present: the no-device path cannot be exercised here")
    subprocess.run(["make", "-s", "-C", ROOT, "adapter-replay"], check=True)
    r = subprocess.run([REPLAY, "--no-device"], capture_output=True, text=True, timeout=120)
    _, checks = _parse(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert checks == {"nodev_ctor_identity": True, "nodev_no_transform": True}


@pytest.mark.gpu
def test_adapter_replays_reference_gicp_tests(cube_clouds, tmp_path):
    from oracle import ref

    src, tgt, Trot = cube_clouds
    ps, pt = tmp_path / "source.bin", tmp_path / "target.bin"
    np.ascontiguousarray(src, np.float32).tofile(ps)
    np.ascontiguousarray(tgt, np.float32).tofile(pt)
    r = subprocess.run([REPLAY, str(ps), str(pt)], capture_output=True, text=True, timeout=300)
    tfs, checks = _parse(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert checks and all(checks.values()), checks
    # testApplyTF: defaults (0.04 m, 4e-3); testRun: setMaxCorrespondenceDistance(5), setTfEpsilon(5e-4)
    for case, kw in (("testApplyTF", {}), ("testRun", dict(max_corr_dist=5.0, transformation_epsilon=5e-4))):
        T, exists = tfs[case]
        o = ref.RefGICP(**kw)
        o.set_source(src)
        o.set_target(tgt)
        T_ref, info = o.align()
        assert exists and info["converged"] == 1
        assert frob(T, T_ref) <= 1e-4, (case, frob(T, T_ref))
        assert np.abs(T - Trot).max() < 1e-4  # the fixture's implied answer Rz(0.175)
    # testRunWithCov: the cube keeps every point through the NaN-normal filter; iterate composes T*T
    T_run, _ = tfs["testRunWithCov_run"]
    T_it, _ = tfs["testRunWithCov_iterate"]
    assert "testRunWithCov_sizes 5000 5000" in r.stdout
    assert frob(T_run, tfs["testApplyTF"][0]) == 0.0
    from leica_point_cloud_processing_amd.gicp_alignment import matmul4f

    np.testing.assert_array_equal(T_it, matmul4f(T_run, T_run))
    # error paths: logged, transform_exists_ / fine_tf_ untouched
    for name in ("errors_empty_source", "errors_too_few_points", "errors_empty_target"):
        assert checks[name + "_logged"] and checks[name + "_untouched"], name
    # solver failure: PCL still writes output = final * source, so iterate()
    # overwrites aligned_cloud_ while fine_tf_ stays
    for name in ("solver_run_logged", "solver_run_untouched", "solver_iterate_logged", "solver_iterate_untouched",
                 "solver_iterate_output_written"):
        assert checks[name], name
