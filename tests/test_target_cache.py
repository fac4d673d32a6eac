"""r05 target cache: GICPState builds a fresh GICPAlignment for every scan and aligns it against the
same CAD cloud (/root/reference/src/LeicaStateMachine.cpp:141-150), so a destroyed engine leaves its
target's grid, covariances and 1-NN cell lists in a process-wide cache and the next engine whose
set_target uploads the same points (compared on the device, bit for bit) adopts them.  Everything an
adopting engine computes must equal a rebuild bit for bit: T, iterations, passes, correspondences,
Mahalanobis matrices, covariances -- and a target that differs in one bit, a new k or a new gate must
not reuse what no longer applies."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ON = {"target_cache": 1}
OFF = {"target_cache": 0}


def _clouds():
    from leica_point_cloud_processing_amd import synth

    return synth.scan_vs_cad(30_000, 30_000, clutter=0.04, debris=600)  # gate rejections included


def _cycle(opts, scan, cad, aligns=2, **params):
    """GICPState's cycle: a fresh engine, set_source then set_target (GICPAlignment.cpp:89-90), align
    (+ iterate()); returns per-align (T, iterations, passes, n_corr), the cache stats after set_target,
    the vlist stats after set_target and the engine (open)"""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    e = GICPEngine(options=opts, **params)
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    cs, vs = e.cache_stats(), e.vlist_stats()
    out = []
    for _ in range(aligns):
        T = e.align()
        r = e.last_result
        out.append((T, r["iterations"], r["n_evals"], r["n_corr"]))
    return out, cs, vs, e


def _same(a, b):
    for (Ta, *ra), (Tb, *rb) in zip(a, b):
        np.testing.assert_array_equal(Ta, Tb)
        assert ra == rb


def test_adopted_target_aligns_like_a_rebuild():
    """cycle 1 builds (and its 5 aligns build the cell lists), cycle 2 adopts grid + covariances +
    lists at set_target and runs its first align on the lists; cycles 1, 2 and a cache-off engine
    give the same aligns, and a correspondence sweep of the adopted engine equals the rebuilt one's"""
    scan, cad, Ttrue = _clouds()
    ref, _, _, r = _cycle(OFF, scan, cad, aligns=5)
    T_sweep = np.linalg.inv(Ttrue).astype(np.float32)
    m_ref, tj_ref, M_ref = r.debug_correspondences(T_sweep, len(scan))
    C_ref = r.debug_covariances("target", len(cad))
    r.close()
    a, cs_a, _, ea = _cycle(ON, scan, cad, aligns=5)
    assert cs_a["adopted"] == 0  # nothing cached yet
    ea.close()  # leaves its target (lists built by aligns 3-5)
    b, cs_b, vs_b, eb = _cycle(ON, scan, cad, aligns=5)
    assert cs_b["adopted"] == 1 and cs_b["cached"] == 0, cs_b
    assert vs_b["lists"] > 0, vs_b  # the lists came with the target
    _same(a, ref)
    _same(b, ref)
    m, tj, M = eb.debug_correspondences(T_sweep, len(scan))
    assert m == m_ref
    np.testing.assert_array_equal(tj, tj_ref)
    np.testing.assert_array_equal(M, M_ref)
    np.testing.assert_array_equal(eb.debug_covariances("target", len(cad)), C_ref)
    eb.close()


def test_changed_points_k_and_gate_are_not_reused():
    """a target differing in one coordinate bit is not adopted; a new k recomputes the covariances
    (grid reused); a new gate rebuilds the lists -- each exactly like a cache-off engine"""
    scan, cad, _ = _clouds()
    e, _, _, x = _cycle(ON, scan, cad, aligns=3)
    x.close()
    cad2 = cad.copy()
    cad2[7, 1] = np.nextafter(cad2[7, 1], np.float32(1e9))  # one ulp
    got, cs, _, y = _cycle(ON, scan, cad2)
    assert cs["adopted"] == 0, cs
    ref, _, _, z = _cycle(OFF, scan, cad2)
    _same(got, ref)
    y.close()  # leaves cad2
    z.close()
    for params in ({"k": 10}, {"max_corr_dist": 0.02}):
        got, cs, _, y = _cycle(ON, scan, cad2, **params)
        assert cs["adopted"] == 1, (params, cs)
        ref, _, _, z = _cycle(OFF, scan, cad2, **params)
        _same(got, ref)
        z.close()
        y.close()  # leaves cad2 again (with this k / gate)


def test_cache_release_and_multirank_contexts_skip_it():
    """mgicp_release_cache empties it; an engine with a shared row segment (N > 1 form) neither
    adopts nor leaves its target"""
    import os

    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = _clouds()
    _, _, _, x = _cycle(ON, scan, cad, aligns=1)
    x.close()
    e = GICPEngine(options=ON)
    assert e.cache_stats()["cached"] == 1
    GICPEngine.release_cache()
    assert e.cache_stats()["cached"] == 0
    e.close()
    s = GICPEngine(options=ON)
    s.comm_init(1, 0, None)
    s.attach_shm(f"/mgicp_tc_{os.getpid()}", len(scan))
    s.set_source_xyz(scan)
    s.set_target_xyz(cad)
    s.align()
    s.close()
    f = GICPEngine(options=ON)
    assert f.cache_stats()["cached"] == 0
    f.close()


def test_source_set_first_with_a_cache_equals_cache_off():
    """GICPState sets the source first (GICPAlignment.cpp:89-90): its grid and covariances start at
    set_source (r06: a grid depends on its own cloud alone), then the target is adopted from the cache or
    rebuilt; a second set_source before any target starts over.  Every form aligns exactly like a
    cache-off engine."""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = _clouds()
    _, _, _, x = _cycle(ON, scan, cad, aligns=1)
    x.close()  # the cache holds cad
    small = np.ascontiguousarray(cad[: len(cad) * 3 // 4])  # another target: other point count, other cell size
    got, cs, _, y = _cycle(ON, scan, small)
    assert cs["adopted"] == 0 and cs["source_spec"] == "none", cs
    ref, _, _, z = _cycle(OFF, scan, small)
    _same(got, ref)
    y.close()  # the cache now holds `small`
    z.close()
    # two set_source calls before the target (the second one a different scan), then the cached target
    e = GICPEngine(options=ON)
    e.set_source_xyz(np.ascontiguousarray(scan[::2]))
    e.set_source_xyz(scan)
    e.set_target_xyz(small)
    cs = e.cache_stats()
    assert cs["adopted"] == 1 and cs["source_spec"] == "none", cs
    got = []
    for _ in range(2):
        T = e.align()
        r = e.last_result
        got.append((T, r["iterations"], r["n_evals"], r["n_corr"]))
    e.close()
    _same(got, ref)
