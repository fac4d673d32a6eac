"""MGICP_SOLVER_GN (opt-in fast mode): engine vs the oracle's GN restatement, and the
fixed-point protocol of SURVEY.md 8c (iii).

The GN mode is not a PCL 1.8.1 algorithm (PCL 1.8.1 only has BFGS), so its checker is the
oracle's restatement (oracle/gicp_ref.c estimate_gn, ref_params.solver = 1) on the same
correspondences, plus properties: the GN optimum is a stationary point of PCL's own objective
(OptimizationFunctorWithIndices) on the final correspondence set, and it lands near the
synthetic ground truth.  Bars:
  * moments (one device pass, fp64 sums in a different order): 1e-10 relative to the
    moment's magnitude scale;
  * final transform vs oracle GN: 1e-5 Frobenius (same iteration count);
  * deviation from PCL's BFGS at default settings is reported, not asserted.
"""
import numpy as np
import pytest

from conftest import frob


def _oracle(src, tgt, **kw):
    from oracle import ref

    o = ref.RefGICP(**kw)
    o.set_source(src)
    o.set_target(tgt)
    return o


# ---------------------------------------------------------------------------------------
# CPU: the oracle's GN restatement
# ---------------------------------------------------------------------------------------
def test_oracle_gn_converges_near_truth(part_small):
    src, tgt, Ttrue = part_small
    T, info = _oracle(src, tgt, solver=1).align()
    assert info["rc"] == 0 and info["converged"] == 1
    # the synthetic scan was moved by inv(Ttrue): GN recovers it to the noise floor of 20k points
    assert np.abs(T.astype(np.float64) @ Ttrue - np.eye(4)).max() < 0.01


def test_oracle_gn_stationary_for_pcl_objective(part_small):
    """On a fixed correspondence set the GN optimum zeroes PCL's own gradient (functor f/df,
    objective = 0) up to the fp32 rounding noise of A*s (DESIGN.md 'moment form')."""
    from oracle import ref

    src, tgt, _ = part_small
    o = _oracle(src, tgt, solver=1, max_iterations=1, fixed_iterations=True)
    T1, info = o.align()
    assert info["iterations"] == 1
    # the correspondence set of that iteration was taken at T = I
    o.correspondences(np.eye(4, dtype=np.float32))
    x1 = np.array([T1[0, 3], T1[1, 3], T1[2, 3],
                   np.arctan2(T1[2, 1], T1[2, 2]), np.arcsin(-T1[2, 0]), np.arctan2(T1[1, 0], T1[0, 0])])
    o.set_params(objective=0)
    _, g0 = o.fdf(np.zeros(6))
    f1, g1 = o.fdf(x1)
    f0, _ = o.fdf(np.zeros(6))
    assert f1 < f0
    assert np.linalg.norm(g1) < 1e-3 * np.linalg.norm(g0)


# ---------------------------------------------------------------------------------------
# GPU: the engine's GN mode
# ---------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def engine_mod():
    from leica_point_cloud_processing_amd.engine import GICPEngine

    return GICPEngine


@pytest.mark.gpu
def test_gn_moments_match_oracle(engine_mod, part_small):
    from leica_point_cloud_processing_amd import _lib

    src, tgt, Ttrue = part_small
    o = _oracle(src, tgt)
    e = engine_mod(solver=_lib.MGICP_SOLVER_GN)
    e.set_source_xyz(src)
    e.set_target_xyz(tgt)
    for T in (np.eye(4, dtype=np.float32), np.linalg.inv(Ttrue).astype(np.float32)):
        m_ref, tgt_ref, _, _ = o.correspondences(T)
        m_gpu, tgt_gpu, _ = e.debug_correspondences(T, len(src))
        assert m_gpu == m_ref and np.array_equal(tgt_gpu, tgt_ref)
        mo_ref = o.moments(T)
        mo_gpu = e.debug_moments(T)
        assert mo_gpu[73] == mo_ref[73] == m_ref
        assert np.all(mo_gpu[74:] == 0)
        # per-block scale: entries of one block share units (S0, B, Q)
        for lo, hi in ((0, 1), (1, 13), (13, 73)):
            scale = np.abs(mo_ref[lo:hi]).max()
            np.testing.assert_allclose(mo_gpu[lo:hi], mo_ref[lo:hi], rtol=0, atol=1e-10 * scale)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["part", "cube"])
def test_gn_align_matches_oracle_gn(engine_mod, part_small, cube_clouds, which):
    from leica_point_cloud_processing_amd import _lib

    if which == "part":
        src, tgt, Ttrue = part_small
        kw, ekw = {}, {}
    else:
        src, tgt, Trot = cube_clouds
        kw = dict(max_corr_dist=5.0, transformation_epsilon=5e-4)
        ekw = dict(max_corr_dist=5.0, tf_eps=5e-4)
    T_ref, info = _oracle(src, tgt, solver=1, **kw).align(want_trace=True)
    e = engine_mod(solver=_lib.MGICP_SOLVER_GN, **ekw)
    e.set_source_xyz(src)
    e.set_target_xyz(tgt)
    T_gpu = e.align()
    assert e.hasConverged() and info["converged"] == 1
    assert e.last_result["iterations"] == info["iterations"]
    assert e.last_result["n_evals"] == info["iterations"]  # one device pass per outer iteration
    for a, b in zip(e.debug_trace(), info["trace"]):
        assert frob(a, b) <= 1e-5
    assert frob(T_gpu, T_ref) <= 1e-5
    if which == "cube":
        assert np.abs(T_gpu - Trot).max() < 1e-4  # the reference test's known answer Rz(0.175)
    else:
        assert np.abs(T_gpu.astype(np.float64) @ Ttrue - np.eye(4)).max() < 0.01


@pytest.mark.gpu
def test_gn_fixed_point_protocol(engine_mod, part_small):
    """tf_eps = rot_eps = 1e-9, max_iter = 200.  Engine GN and oracle GN reach
    the same fixed point; the engine with a guess lands there too."""
    from leica_point_cloud_processing_amd import _lib

    src, tgt, Ttrue = part_small
    kw = dict(transformation_epsilon=1e-9, rotation_epsilon=1e-9, max_iterations=60)
    T_ref, _ = _oracle(src, tgt, solver=1, **kw).align()
    e = engine_mod(solver=_lib.MGICP_SOLVER_GN, tf_eps=1e-9, rot_eps=1e-9, max_iter=60)
    e.set_source_xyz(src)
    e.set_target_xyz(tgt)
    T_gpu = e.align()
    assert frob(T_gpu, T_ref) <= 1e-5
    # starting from a guess near the answer (output = guess * input, final = T * guess)
    guess = (np.linalg.inv(Ttrue) @ _rz(2e-3)).astype(np.float32)
    T_g = e.align(guess=guess)
    assert frob(T_g, T_gpu) <= 1e-4


@pytest.mark.gpu
def test_gn_deterministic_and_iterate(engine_mod, part_small):
    from leica_point_cloud_processing_amd import _lib

    src, tgt, _ = part_small
    e = engine_mod(solver=_lib.MGICP_SOLVER_GN)
    e.set_source_xyz(src)
    e.set_target_xyz(tgt)
    T1 = e.align()
    T2 = e.align()
    assert np.array_equal(T1, T2)


@pytest.mark.gpu
def test_gn_too_few_correspondences(engine_mod, cube_clouds):
    """Fewer than 4 correspondences: PCL's solver throws -> converged stays false."""
    from leica_point_cloud_processing_amd import _lib

    src, tgt, _ = cube_clouds
    e = engine_mod(solver=_lib.MGICP_SOLVER_GN, max_corr_dist=1e-9)
    e.set_source_xyz(src + np.float32(10.0))
    e.set_target_xyz(tgt)
    e.align()
    assert not e.hasConverged()


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    R = np.eye(4)
    R[:2, :2] = [[c, -s], [s, c]]
    return R
