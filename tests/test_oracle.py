"""CPU tests of the oracle (oracle/gicp_ref.c) -- the checker every GPU parity test relies on.

Pinning (DESIGN.md "Oracle"): PCL 1.8.1 is absent, so the reference itself cannot run.  The
oracle is pinned by (1) the reference unit test's own scenario, regenerated bit-exactly from
test/cube.ply with glibc rand() (test_gicp_alignment.cpp:32-47 -> T = Rz(0.175)); (2) the
independent NumPy/SciPy restatement's frozen outputs in tests/golden/*.npz
(oracle/golden_numpy.py).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN, frob

CASES = ["k1_cube_testconfig", "k2_cube_defaults", "k3_part_6k"]


def _golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)


def _ref_for(g):
    from oracle import ref

    dmax, tf_eps, rot_eps, max_iter, k = g["params"]
    o = ref.RefGICP(max_corr_dist=float(dmax), transformation_epsilon=float(tf_eps),
                    rotation_epsilon=float(rot_eps), max_iterations=int(max_iter), k=int(k))
    o.set_source(g["source"])
    o.set_target(g["target"])
    return o


def test_glibc_rand_reproduction():
    """synth.GlibcRand is glibc's rand() (TYPE_3, srand(1) default) bit for bit."""
    from leica_point_cloud_processing_amd import synth

    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    g = synth.GlibcRand(1)
    assert [libc.rand() for _ in range(20000)] == [g.rand() for _ in range(20000)]
    libc.srand(12345)
    g = synth.GlibcRand(12345)
    assert [libc.rand() for _ in range(5000)] == [g.rand() for _ in range(5000)]


def test_cube_fixture_regenerates(cube_clouds):
    """The committed fixture input equals the reference test's CADToPointCloud + rotateCloud."""
    src, tgt, T = cube_clouds
    g = _golden("k1_cube_testconfig")
    np.testing.assert_array_equal(g["source"], src)
    np.testing.assert_array_equal(g["target"], tgt)
    assert src.shape == (5000, 3)
    # every sample lies on the cube's surface
    assert np.allclose(np.abs(src).max(axis=1), 1.0, atol=1e-6)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_golden(name):
    g = _golden(name)
    o = _ref_for(g)
    T, info = o.align(want_trace=True)
    assert info["converged"] == 1
    assert info["iterations"] == int(g["iterations"])
    assert frob(T, g["final_T"]) <= 1e-6
    for a, b in zip(info["trace"], g["trace"]):
        assert frob(a, b) <= 1e-6


@pytest.mark.parametrize("name", CASES)
def test_oracle_covariances_and_correspondences(name):
    from oracle import ref

    g = _golden(name)
    cs = ref.covariances(g["source"])
    ct = ref.covariances(g["target"])
    scale = np.abs(g["cov_source_head"]).max()
    assert np.abs(cs[:256] - g["cov_source_head"]).max() <= 1e-9 * scale
    assert np.abs(ct[:256] - g["cov_target_head"]).max() <= 1e-9 * scale
    o = _ref_for(g)
    m, tj, _, _ = o.correspondences(np.eye(4, dtype=np.float32))
    np.testing.assert_array_equal(tj, g["corr_identity"])
    assert m == int((g["corr_identity"] >= 0).sum())


def test_known_answer_rz(cube_clouds):
    """test_gicp_alignment.cpp: target = Rz(0.175) * source -> GICP recovers Rz(0.175)."""
    from oracle import ref

    src, tgt, Trot = cube_clouds
    for kw in (dict(max_corr_dist=5.0, transformation_epsilon=5e-4), {}):
        o = ref.RefGICP(**kw)
        o.set_source(src)
        o.set_target(tgt)
        T, info = o.align()
        assert info["converged"] == 1
        assert np.abs(T - Trot).max() < 1e-4
        assert not np.isnan(T).any()  # Utils::isValidTransform


def test_known_answer_cube_ply_vs_obj():
    """BASELINE.json configs[0]: cube.ply sampled vs cube.obj sampled and rotated by Rz(0.175) (two
    independent samplings, synth.cube_ply_vs_obj): the oracle converges and recovers the rotation to
    the sampling noise (5e-4 max-abs); both mesh readers see the same 2 x 2 x 2 cube."""
    import os

    from conftest import GOLDEN
    from leica_point_cloud_processing_amd import synth
    from oracle import ref

    v1, t1 = synth.read_ply(os.path.join(GOLDEN, "cube.ply"))
    v2, t2 = synth.read_obj(os.path.join(GOLDEN, "cube.obj"))
    assert len(t1) == len(t2) == 12
    assert np.array_equal(v1.min(0), v2.min(0)) and np.array_equal(v1.max(0), v2.max(0))
    src, tgt, Trot = synth.cube_ply_vs_obj(os.path.join(GOLDEN, "cube.ply"), os.path.join(GOLDEN, "cube.obj"))
    assert not np.array_equal(src, synth.transform_points(np.linalg.inv(Trot).astype(np.float32), tgt))
    for kw in (dict(max_corr_dist=5.0, transformation_epsilon=5e-4), {}):
        o = ref.RefGICP(**kw)
        o.set_source(src)
        o.set_target(tgt)
        T, info = o.align()
        assert info["converged"] == 1
        assert np.abs(T - Trot).max() < 5e-4


def test_knn_exact_against_bruteforce():
    from oracle import ref

    rng = np.random.default_rng(3)
    pts = rng.random((3000, 3)).astype(np.float32)
    pts[1500:1600] = pts[:100]  # exact duplicates -> ties broken by index
    q = pts[::7]
    idx, d2 = ref.knn(pts, q, 20)
    d = q[:, None, :] - pts[None, :, :]
    D = d[..., 0] * d[..., 0]
    D = D + d[..., 1] * d[..., 1]
    D = D + d[..., 2] * d[..., 2]
    order = np.lexsort((np.broadcast_to(np.arange(len(pts)), D.shape), D), axis=1)[:, :20]
    np.testing.assert_array_equal(idx, order)
    np.testing.assert_array_equal(d2, np.take_along_axis(D, order, 1))


def test_gradient_matches_finite_differences(part_small):
    """computeRDerivative / df against central differences of f."""
    from oracle import ref

    scan, cad, _ = part_small
    o = ref.RefGICP()
    o.set_source(scan)
    o.set_target(cad)
    o.correspondences(np.eye(4, dtype=np.float32))
    x = np.array([0.004, -0.003, 0.002, 0.002, -0.001, 0.0015])
    f0, g = o.fdf(x)
    for i in range(6):
        h = 1e-4
        e = np.zeros(6)
        e[i] = h
        fp, _ = o.fdf(x + e)
        fm, _ = o.fdf(x - e)
        fd = (fp - fm) / (2 * h)
        assert abs(fd - g[i]) <= 2e-3 * max(1.0, abs(g[i])), (i, fd, g[i])


def test_moment_form_matches_functor(part_small):
    """The moment form of the objective (oracle objective=1) is PCL's functor up to
    the fp32 rounding of A*s: identical at the expansion point, ~1e-6 relative elsewhere."""
    from oracle import ref

    scan, cad, _ = part_small
    o = ref.RefGICP()
    o.set_source(scan)
    o.set_target(cad)
    T0 = np.eye(4, dtype=np.float32)
    o.correspondences(T0)
    o.moments(T0)
    rng = np.random.default_rng(3)
    for scale in (0.0, 1e-5, 1e-3, 1e-2):
        x = rng.normal(size=6) * scale
        o.set_params(objective=0)
        f0, g0 = o.fdf(x)
        o.set_params(objective=1)
        f1, g1 = o.fdf(x)
        tol = 1e-12 if scale == 0.0 else 1e-4
        assert abs(f1 - f0) <= tol * abs(f0), (scale, f0, f1)
        assert np.abs(g1 - g0).max() <= max(tol, 1e-4) * max(1.0, np.abs(g0).max()), (scale, g0, g1)


def test_apply_state_matches_numpy_restatement():
    from oracle import golden_numpy, ref

    rng = np.random.default_rng(5)
    for _ in range(20):
        x = rng.normal(0, 0.3, 6)
        np.testing.assert_array_equal(ref.apply_state(x), golden_numpy.apply_state(x))


def test_threaded_oracle_agrees(part_small):
    """The OpenMP variant (the thread-share CPU baseline) reproduces the single-thread result."""
    from oracle import ref

    scan, cad, _ = part_small
    out = []
    for th in (1, 4):
        o = ref.RefGICP(threads=th)
        o.set_source(scan)
        o.set_target(cad)
        T, info = o.align()
        out.append((T, info["iterations"]))
    assert out[0][1] == out[1][1]
    assert frob(out[0][0], out[1][0]) <= 1e-6


def test_oracle_errors():
    from oracle import ref

    o = ref.RefGICP()
    pts = np.random.default_rng(0).random((10, 3)).astype(np.float32)
    o.set_source(pts)
    o.set_target(pts)
    _, info = o.align()
    assert info["rc"] == -2  # fewer points than k_correspondences
    bad = pts.copy()
    bad[0, 0] = np.nan
    assert o.set_source(bad) == -4
