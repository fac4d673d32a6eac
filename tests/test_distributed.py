"""N > 1 path: source point-range shards, target replicated, one all-reduce of
the 16 objective sums per BFGS pass.

CPU (world_size 2):
  * the decomposition itself -- per-shard partial sums of the oracle's objective all-reduced
    over torch.distributed gloo equal the single-process sums;
  * the TCP control plane bench.py uses (id broadcast, barrier, max-over-ranks timer).
GPU (one device): two "detached" shard contexts (mgicp_comm_init(ctx, 2, r, NULL)) whose
partial sums must add up to the unsharded context's -- the engine's shard bookkeeping
(covariance ranges, correspondence ranges, pass ranges) without RCCL.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.parallel import shard_range
    from oracle import ref

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scan, cad, _ = synth.scan_vs_cad(6000, 6000)
    o = ref.RefGICP()
    o.set_source(scan)
    o.set_target(cad)
    m, _, _, _ = o.correspondences(np.eye(4, dtype=np.float32))
    x = np.array([0.003, -0.002, 0.001, 0.001, -0.0005, 0.002])
    c0, c1 = shard_range(m, world, rank)
    part = torch.tensor(o.fdf_sums(x, c0, c1), dtype=torch.float64)
    dist.all_reduce(part, op=dist.ReduceOp.SUM)
    full = o.fdf_sums(x, 0, m)
    f_ref, g_ref = o.fdf(x)
    s = part.numpy()
    f = s[0] / s[13]
    # Gauss-Newton mode: one all-reduce of the 74 moments per outer iteration
    T0 = np.eye(4, dtype=np.float32)
    mom = torch.tensor(o.moments_range(T0, c0, c1), dtype=torch.float64)
    dist.all_reduce(mom, op=dist.ReduceOp.SUM)
    mfull = o.moments(T0)
    rel_mom = max(float(np.abs(mom.numpy()[a:b] - mfull[a:b]).max() / np.abs(mfull[a:b]).max())
                  for a, b in ((0, 1), (1, 13), (13, 74)))
    q.put((rank, float(np.abs(s - full).max() / np.abs(full).max()), abs(f - f_ref) / abs(f_ref), int(s[13]), m,
           rel_mom))
    dist.destroy_process_group()


def test_sharded_objective_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rel_sums, rel_f, cnt, m, rel_mom in res:
        assert cnt == m
        assert rel_sums <= 1e-12
        assert rel_f <= 1e-12
        assert rel_mom <= 1e-12


def _rdv_worker(rank, world, port, q):
    from leica_point_cloud_processing_amd.parallel import Rendezvous

    r = Rendezvous(rank, world, addr="127.0.0.1", port=port, timeout=60)
    uid = r.broadcast(bytes(range(128)) if rank == 0 else None)
    r.barrier()
    mx = r.allreduce_max(float(rank) + 0.5)
    r.barrier()
    r.close()
    q.put((rank, uid == bytes(range(128)), mx))


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_control_plane(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rdv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert all(mx == world - 0.5 for _, _, mx in res)


def _bogus_then_real(port, q):
    """A pickle payload and an out-of-range rank arrive before the real rank 1: rank 0 must drop
    them (nothing is unpickled) and finish the rendezvous."""
    import pickle
    import struct
    import time as _t

    from leica_point_cloud_processing_amd import parallel

    def connect():
        for _ in range(200):
            try:
                return socket.create_connection(("127.0.0.1", port), timeout=5.0)
            except OSError:
                _t.sleep(0.05)
        raise RuntimeError("no server")

    class Boom:
        def __reduce__(self):
            return (os._exit, (3,))

    s1 = connect()
    s1.sendall(struct.pack("<Q", 64) + pickle.dumps(Boom()).ljust(64, b"\0"))
    s2 = connect()
    s2.sendall(parallel._hello(7))  # rank outside 1..world-1
    real = parallel.Rendezvous(1, 2, addr="127.0.0.1", port=port, timeout=60)
    uid = real.broadcast(None)
    real.barrier()
    q.put(uid)
    real.close()
    for s in (s1, s2):
        s.close()


def test_rendezvous_rejects_bogus_peers():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    peer = ctx.Process(target=_bogus_then_real, args=(port, q))
    peer.start()
    from leica_point_cloud_processing_amd.parallel import Rendezvous

    r = Rendezvous(0, 2, addr="127.0.0.1", port=port, timeout=60)
    r.broadcast(bytes(range(128)))
    r.barrier()
    assert q.get(timeout=60) == bytes(range(128))
    peer.join(timeout=30)
    assert peer.exitcode == 0
    r.close()
    from leica_point_cloud_processing_amd.parallel import _check_hello, _encode, _hello

    with pytest.raises(TypeError):
        _encode({"not": "allowed"})
    assert _check_hello(_hello(1), 3, {}) == 1
    assert _check_hello(_hello(1), 3, {1: None}) is None  # duplicate rank
    assert _check_hello(_hello(0), 3, {}) is None and _check_hello(_hello(3), 3, {}) is None


def test_shard_ranges_partition():
    from leica_point_cloud_processing_amd.parallel import shard_range

    for n in (0, 1, 7, 5_000_000, 20_000_001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


@pytest.mark.gpu
def test_detached_shards_sum_to_full(part_small):
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, Ttrue = part_small
    T = np.linalg.inv(Ttrue).astype(np.float32)
    full = GICPEngine()
    full.set_source_xyz(scan)
    full.set_target_xyz(cad)
    m_full, tj_full, _ = full.debug_correspondences(T, len(scan))
    x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
    s_full = full.debug_fdf_sums(x)
    mom_full = full.debug_moments(T)
    mom_total = np.zeros(80)
    total = np.zeros(16)
    tj = np.full(len(scan), -1, np.int32)
    m_sum = 0
    world = 3
    for r in range(world):
        e = GICPEngine()
        e.comm_init(world, r, None)
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        m_r, tj_r, _ = e.debug_correspondences(T, len(scan))
        m_sum += m_r
        own = tj_r >= 0
        tj[own] = tj_r[own]
        total += e.debug_fdf_sums(x)
        mom_total += e.debug_moments(T)
        with pytest.raises(Exception):
            e.align()  # detached shards cannot run the collective path
        e.close()
    assert m_sum == m_full
    np.testing.assert_array_equal(tj, tj_full)
    assert total[13] == s_full[13] == m_full
    assert np.abs(total - s_full).max() <= 1e-11 * np.abs(s_full).max()
    # Gauss-Newton mode: the shards' moments add up to the unsharded moment pass
    assert mom_total[73] == mom_full[73] == m_full
    for a, b in ((0, 1), (1, 13), (13, 73)):
        assert np.abs(mom_total[a:b] - mom_full[a:b]).max() <= 1e-11 * np.abs(mom_full[a:b]).max()


@pytest.mark.gpu
@pytest.mark.parametrize("solver", [0, 1])
def test_single_rank_comm_matches_plain(part_small, solver):
    """The collective code path (RCCL all-reduce per BFGS pass / per GN iteration, publish kernel,
    all-reduced fitness) on a real one-rank communicator gives the plain context's results bit
    for bit -- the only RCCL run a one-GPU box allows."""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = part_small
    plain = GICPEngine(solver=solver)
    plain.set_source_xyz(scan)
    plain.set_target_xyz(cad)
    T_plain = plain.align()
    f_plain = plain.getFitnessScore()
    coll = GICPEngine(solver=solver)
    coll.comm_init(1, 0, GICPEngine.unique_id())
    coll.set_source_xyz(scan)
    coll.set_target_xyz(cad)
    T_coll = coll.align()
    assert coll.last_result["iterations"] == plain.last_result["iterations"]
    assert coll.last_result["n_evals"] == plain.last_result["n_evals"]
    np.testing.assert_array_equal(T_coll, T_plain)
    assert coll.getFitnessScore() == f_plain
    np.testing.assert_array_equal(coll.align(), T_plain)  # iterate(): cached grids, same result
    coll.close()
    plain.close()
