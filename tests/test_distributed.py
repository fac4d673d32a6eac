"""N > 1 path: super-aligned source point-range shards, target covariances split
and all-gathered, one all-gather of the super partials per BFGS pass and a fixed-order total --
every N gives the single-GPU sums bit for bit.

CPU (gloo, world_size 2 and 3):
  * the decomposition itself -- the fixed tree over the oracle's objective, shards all-gathered
    over torch.distributed gloo, is bit-identical to the single-process tree;
  * the TCP control plane bench.py uses (id broadcast, barrier, max-over-ranks timer).
GPU (one device): N = 2, 3, 4 "detached" shard contexts (mgicp_comm_init(ctx, N, r, NULL)) whose
super partials (objective, GN moments, fitness) equal the unsharded context's bit for bit, and the
multi-GPU finish over them reproduces the unsharded totals bit for bit.
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


def _tree_sums(o, x, cpos, n, lo, hi):
    """Chunk partials of chunks [lo, hi) (oracle sums over each chunk's correspondences), then
    super partials (sequential in chunk order) -- the engine's fixed tree, emulated on the oracle."""
    from leica_point_cloud_processing_amd.parallel import CHUNK_PTS, SUPER_CHUNKS

    chunks = {j: np.asarray(o.fdf_sums(x, int(cpos[j * CHUNK_PTS]), int(cpos[min((j + 1) * CHUNK_PTS, n)])))
              for j in range(lo, hi)}
    sups = []
    for s0 in range(lo, hi, SUPER_CHUNKS):
        acc = chunks[s0].copy()
        for j in range(s0 + 1, min(s0 + SUPER_CHUNKS, hi)):
            acc = acc + chunks[j]
        sups.append(acc)
    return sups


def _fixed_total(sups):
    """The engine's own total order over supers (mirror wave_total, not a sequential sum)."""
    from leica_point_cloud_processing_amd.parallel import fixed_total

    return fixed_total(sups)


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.parallel import CHUNK_PTS, SUPER_PTS, combine_supers, shard_range
    from oracle import ref

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scan, cad, _ = synth.scan_vs_cad(140000, 60000)
    o = ref.RefGICP()
    o.set_source(scan)
    o.set_target(cad)
    m, tj, _, _ = o.correspondences(np.eye(4, dtype=np.float32))
    n = len(scan)
    cpos = np.concatenate([[0], np.cumsum(tj >= 0)])
    x = np.array([0.003, -0.002, 0.001, 0.001, -0.0005, 0.002])
    nsup = -(-n // SUPER_PTS)
    p0, p1 = shard_range(n, world, rank)
    mine = _tree_sums(o, x, cpos, n, p0 // CHUNK_PTS, -(-p1 // CHUNK_PTS)) if p1 > p0 else []
    maxsup = -(-nsup // world)
    rows = np.full((maxsup, 14), np.nan)  # padding is never read (the oracle reports 14 sums)
    if mine:
        rows[: len(mine)] = np.stack(mine)
    parts = [torch.zeros(maxsup, 14, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(parts, torch.from_numpy(rows))
    total = _fixed_total(combine_supers([p.numpy() for p in parts], nsup, world))
    single = _fixed_total(_tree_sums(o, x, cpos, n, 0, -(-n // CHUNK_PTS)))
    full = np.asarray(o.fdf_sums(x, 0, m))
    q.put((rank, bool(np.array_equal(total, single)), float(np.abs(total - full).max() / np.abs(full).max()),
           int(total[13]), m, (p0, p1)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_objective_gloo_bitwise_across_world(world):
    """N ranks (gloo, CPU) each reduce their super-aligned shard with the fixed tree, all-gather the
    supers and sum them in the fixed order: bit-identical to the single-process tree for N = 2, 3
    (and within 1e-12 of the oracle's straight sum)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = [r[5] for r in res]
    assert ranges[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    for rank, same, rel, cnt, m, _ in res:
        assert same, rank
        assert cnt == m
        assert rel <= 1e-12


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
    from leica_point_cloud_processing_amd.parallel import SUPER_PTS, shard_range

    for n in (0, 1, 7, 5_000_000, 20_000_001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert all(a % SUPER_PTS == 0 for a, _ in rs if a < n)  # super-aligned starts
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= SUPER_PTS


@pytest.fixture(scope="module")
def five_supers():
    from leica_point_cloud_processing_amd import synth

    scan, cad, Ttrue = synth.scan_vs_cad(150000, 80000)  # 5 supers of 32768 source points
    return scan, cad, Ttrue


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 4])
def test_detached_shards_bitwise_equal_single(five_supers, world):
    """N detached shards (mgicp_comm_init(ctx, N, r, NULL): the engine's shard bookkeeping without
    RCCL) on one device: their correspondences and super partials -- objective pass, GN moments,
    fitness -- are the unsharded context's bit for bit, and the multi-GPU finish over the padded
    rows (padding = NaN, never read) gives the unsharded totals bit for bit."""
    from leica_point_cloud_processing_amd.engine import GICPEngine
    from leica_point_cloud_processing_amd.parallel import SUPER_PTS, super_first

    scan, cad, Ttrue = five_supers
    T = np.linalg.inv(Ttrue).astype(np.float32)
    x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
    full = GICPEngine()
    full.set_source_xyz(scan)
    full.set_target_xyz(cad)
    m_full, tj_full, M_full = full.debug_correspondences(T, len(scan))
    ref = {"fdf": full.debug_supers("fdf", x), "moments": full.debug_supers("moments", T),
           "fitness": full.debug_supers("fitness", (T, 0.0))}
    tot = {"fdf": full.debug_fdf_sums(x), "moments": full.debug_moments(T)}
    nsup = -(-len(scan) // SUPER_PTS)
    assert all(len(v) == nsup for v in ref.values())
    maxsup = -(-nsup // world)
    rows = {k: np.full((world, maxsup, v.shape[1]), np.nan) for k, v in ref.items()}
    tj = np.full(len(scan), -1, np.int32)
    M = np.zeros_like(M_full)
    m_sum = 0
    for r in range(world):
        e = GICPEngine()
        e.comm_init(world, r, None)
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        m_r, tj_r, M_r = e.debug_correspondences(T, len(scan))
        m_sum += m_r
        own = tj_r >= 0
        tj[own] = tj_r[own]
        M[own] = M_r[own]
        for k in rows:
            arg = x if k == "fdf" else (T if k == "moments" else (T, 0.0))
            sup = e.debug_supers(k, arg)
            a, b = super_first(r, nsup, world), super_first(r + 1, nsup, world)
            assert len(sup) == b - a
            np.testing.assert_array_equal(sup, ref[k][a:b], err_msg=f"{k} rank {r}")
            rows[k][r, : b - a] = sup
        with pytest.raises(Exception):
            e.align()  # detached shards cannot run the collective path
        e.close()
    assert m_sum == m_full
    np.testing.assert_array_equal(tj, tj_full)
    np.testing.assert_array_equal(M, M_full)
    np.testing.assert_array_equal(full.debug_finish_supers(rows["fdf"], nsup, maxsup, world), tot["fdf"])
    np.testing.assert_array_equal(full.debug_finish_supers(rows["moments"], nsup, maxsup, world), tot["moments"])
    fit = full.debug_finish_supers(rows["fitness"], nsup, maxsup, world)
    assert fit[0] / fit[13] == full.fitness(T)
    full.close()


@pytest.mark.gpu
def test_pass_sums_independent_of_direction_and_finish(part_small, monkeypatch):
    """The fixed tree makes an objective pass's sums independent of the sweep direction (passes
    alternate it) and of where the total is taken (in-launch vs the separate finish kernel)."""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, Ttrue = part_small
    T = np.linalg.inv(Ttrue).astype(np.float32)
    x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
    res = {}
    for fused in ("1", "0"):
        e = GICPEngine(options={"fused_finish": int(fused)})
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        e.debug_correspondences(T, len(scan))
        a, b = e.debug_fdf_sums(x), e.debug_fdf_sums(x)  # consecutive passes: opposite directions
        np.testing.assert_array_equal(a, b)
        res[fused] = a
        e.close()
    np.testing.assert_array_equal(res["0"], res["1"])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [20_000, 2_500_000])
def test_resident_server_matches_launched_passes(part_small, monkeypatch, n):
    """The resident pass server (one launch per BFGS run, chunks kept in registers /
    LDS across passes) gives the launched passes' sums bit for bit -- at 20k points (every chunk in
    registers) and 2.5M points (register, LDS and streamed chunks) -- and aligns identically."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, Ttrue = part_small if n == 20_000 else synth.scan_vs_cad(n, n)
    T = np.linalg.inv(Ttrue).astype(np.float32)
    x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    e.debug_correspondences(T, len(scan))
    ms0, s0 = e.debug_pass_bench(x, 7, 0)
    ms1, s1 = e.debug_pass_bench(x, 7, 1)
    s2 = e.debug_fdf_sums(x)  # through the live-server path of the aligns
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(s0, s2)
    assert ms0 > 0 and ms1 > 0
    T_on = e.align()
    it_on = e.last_result["iterations"]
    e.close()
    f = GICPEngine(options={"resident": 0})
    f.set_source_xyz(scan)
    f.set_target_xyz(cad)
    T_off = f.align()
    assert f.last_result["iterations"] == it_on
    np.testing.assert_array_equal(T_on, T_off)
    f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bar,rows", [(1, 1), (0, 1), (1, 0)])
def test_server_forms_align_identically(monkeypatch, bar, rows):
    """Every form of the resident server -- commands through the BAR or the
    pinned copy, super partials as host rows or the device total -- aligns 300k points to the same
    T and iteration count as the launched passes, bit for bit."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = synth.scan_vs_cad(300_000, 300_000)
    res = {}
    for form in ("launched", "server"):
        e = GICPEngine(options={"resident": 0 if form == "launched" else 1, "bar_cmd": bar, "host_rows": rows})
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        T = e.align()
        res[form] = (T, e.last_result["iterations"], e.last_result["n_evals"])
        st = e.pass_stats()
        e.close()
        if form == "server":  # the server form really ran: every pass, BAR as asked
            assert st["server_launches"] == res[form][1] and st["server_passes"] == res[form][2], st
            assert st["launched_passes"] == 0 and st["takeovers"] == 0, st
            assert st["row_allocs"] == rows, st
            if bar:  # large-BAR devices (MI355X): commands through the BAR
                assert st["bar_commands"] == 1, st
            else:
                assert st["bar_commands"] == 0, st
        else:
            assert st["server_launches"] == 0 and st["launched_passes"] == res[form][2], st
    np.testing.assert_array_equal(res["server"][0], res["launched"][0])
    assert res["server"][1:] == res["launched"][1:]


@pytest.mark.gpu
def test_server_context_reuse_across_cloud_sizes(part_small):
    """One context aligning a 20k pair, then a 300k pair (the host rows grow), then the 20k pair
    again gives each fresh context's T bit for bit."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    small = part_small[:2]
    big = synth.scan_vs_cad(300_000, 300_000)[:2]

    def fresh(pair):
        f = GICPEngine()
        f.set_source_xyz(pair[0])
        f.set_target_xyz(pair[1])
        T = f.align()
        f.close()
        return T

    ref = {"small": fresh(small), "big": fresh(big)}
    e = GICPEngine()
    allocs = []
    for name, pair in (("small", small), ("big", big), ("small", small)):
        e.set_source_xyz(pair[0])
        e.set_target_xyz(pair[1])
        np.testing.assert_array_equal(e.align(), ref[name])
        allocs.append(e.pass_stats()["row_allocs"])
    st = e.pass_stats()
    e.close()
    # 20k points: one super (the 64-super minimum buffer); 300k: 10 supers fit it too -> one allocation
    assert allocs == [1, 1, 1], allocs
    assert st["server_passes"] > 0 and st["takeovers"] == 0, st


@pytest.mark.gpu
def test_server_context_rows_grow_past_minimum():
    """The host rows grow when a cloud needs more supers than the buffer holds (64-super minimum):
    a 2.2M-point source (68 supers) after a 20k one reallocates once, and both align bit for bit
    like fresh contexts."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    small = synth.scan_vs_cad(20_000, 20_000)[:2]
    big = synth.scan_vs_cad(2_200_000, 300_000)[:2]
    ref = {}
    for name, pair in (("small", small), ("big", big)):
        f = GICPEngine()
        f.set_source_xyz(pair[0])
        f.set_target_xyz(pair[1])
        ref[name] = f.align()
        f.close()
    e = GICPEngine()
    allocs = []
    for name, pair in (("small", small), ("big", big), ("small", small)):
        e.set_source_xyz(pair[0])
        e.set_target_xyz(pair[1])
        np.testing.assert_array_equal(e.align(), ref[name])
        allocs.append(e.pass_stats()["row_allocs"])
    e.close()
    assert allocs == [1, 2, 2], allocs


@pytest.mark.gpu
@pytest.mark.parametrize("stall", [0, 3])
def test_server_takeover_after_missed_deadline(monkeypatch, stall):
    """a server pass that cannot complete (here: its last block withholds pass
    `stall` of the first BFGS run, MGICP_SRV_STALL_PASS) is cancelled after the row deadline and
    re-run as a launched pass writing the same rows; the rest of the align runs launched passes.
    T, iterations and passes are bitwise those of an undisturbed align, and every later align of the
    context takes over once again (the knob stalls every server)."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = synth.scan_vs_cad(300_000, 300_000)
    ref = GICPEngine()
    ref.set_source_xyz(scan)
    ref.set_target_xyz(cad)
    T_ref = ref.align()
    it_ref, ev_ref = ref.last_result["iterations"], ref.last_result["n_evals"]
    ref.close()
    monkeypatch.setenv("MGICP_SRV_STALL_PASS", str(stall))
    monkeypatch.setenv("MGICP_ROW_DEADLINE_MS", "50")
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    for k in range(2):
        T = e.align()
        np.testing.assert_array_equal(T, T_ref)
        assert (e.last_result["iterations"], e.last_result["n_evals"]) == (it_ref, ev_ref)
        st = e.pass_stats()
        assert st["takeovers"] == k + 1, st
        assert st["server_launches"] == k + 1, st  # degraded after the take-over: no more servers
        assert st["launched_passes"] == (k + 1) * ev_ref - st["server_passes"] + st["takeovers"], st
    assert e.getFitnessScore() >= 0
    e.close()


@pytest.mark.gpu
def test_concurrent_contexts_share_one_device(part_small):
    """two host threads align on one device at the same time.  One context at a time
    runs the resident server (a process-wide per-device slot); the other runs launched passes (or
    takes a pass over if it missed the slot's release) -- both results are bitwise those of a lone
    context, repeatedly."""
    import threading

    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    pairs = [part_small[:2], synth.scan_vs_cad(300_000, 300_000)[:2]]
    refs = []
    for pr in pairs:
        f = GICPEngine()
        f.set_source_xyz(pr[0])
        f.set_target_xyz(pr[1])
        refs.append(f.align())
        f.close()
    engines = []
    for pr in pairs:
        e = GICPEngine()
        e.set_source_xyz(pr[0])
        e.set_target_xyz(pr[1])
        engines.append(e)
    out = [[], []]
    errs = []

    def run(i):
        try:
            for _ in range(6):
                out[i].append(engines[i].align())
        except Exception as exc:  # noqa: BLE001
            errs.append(repr(exc))

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    for i in range(2):
        assert len(out[i]) == 6
        for T in out[i]:
            np.testing.assert_array_equal(T, refs[i])
    st = [e.pass_stats() for e in engines]
    assert sum(s["server_launches"] for s in st) > 0, st
    for e in engines:
        e.close()


@pytest.mark.gpu
def test_shm_attach_detach_reattach_bitwise(part_small):
    """the row stamps restart at every attach / detach of the shared segment, so
    every buffer holding stamps of earlier passes (the server's stamped chunk partials, the private
    host rows) is cleared with them.  One context: a debug pass at another state and correspondence
    set (stamp 1), attach, align, detach, align, attach a new segment, align -- each T, iteration and
    pass count bitwise a fresh context's, every pass on the server, no take-over."""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, Ttrue = part_small
    f = GICPEngine()
    f.set_source_xyz(scan)
    f.set_target_xyz(cad)
    T_ref = f.align()
    res_ref = (f.last_result["iterations"], f.last_result["n_evals"])
    f.close()
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    T_off = np.linalg.inv(Ttrue).astype(np.float32)
    e.debug_correspondences(T_off, len(scan))
    e.debug_fdf_sums(np.array([0.002, -0.001, 0.001, 0.0005, -0.0004, 0.0003]))  # pass stamp 1, other sums
    names = [f"/mgicp_reattach_{os.getpid()}_{k}" for k in range(2)]
    try:
        for step in ("attach", "detach", "attach2"):
            if step == "detach":
                e.detach_shm()
            else:
                e.attach_shm(names[0 if step == "attach" else 1], len(scan))
            st0 = e.pass_stats()
            T = e.align()
            st1 = e.pass_stats()
            np.testing.assert_array_equal(T, T_ref, err_msg=step)
            assert (e.last_result["iterations"], e.last_result["n_evals"]) == res_ref, step
            assert st1["server_passes"] - st0["server_passes"] == res_ref[1], (step, st0, st1)
            assert st1["takeovers"] == 0 and st1["launched_passes"] == st0["launched_passes"], (step, st1)
            assert st1["transport"] == (0 if step == "detach" else 2), (step, st1)
    finally:
        e.close()
    for nm in names:
        assert not os.path.exists("/dev/shm" + nm)


@pytest.mark.gpu
def test_oversize_source_after_attach_frees_server_slot(part_small):
    """a source larger than the shared segment (a recoverable user error) fails
    the align before the device's server slot is taken -- another context then still gets a server."""
    from leica_point_cloud_processing_amd import _lib
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    big = synth.scan_vs_cad(100_000, 100_000)[:2]
    name = f"/mgicp_oversize_{os.getpid()}"
    e = GICPEngine()
    try:
        e.attach_shm(name, 40_000)  # 2 supers
        e.set_source_xyz(big[0])   # 4 supers
        e.set_target_xyz(big[1])
        with pytest.raises(_lib.MgicpError):
            e.align()
        assert e.pass_stats()["server_launches"] == 0
        g = GICPEngine()
        g.set_source_xyz(part_small[0])
        g.set_target_xyz(part_small[1])
        g.align()
        st = g.pass_stats()
        g.close()
        assert st["server_denied"] == 0 and st["server_passes"] == g.last_result["n_evals"] > 0, st
    finally:
        e.close()


@pytest.mark.gpu
def test_server_in_align_time_counts_every_pass():
    """mgicp_debug_server_time (bench.py's headline roofline): after aligns on
    the resident server, the summed launch durations cover every pass of every BFGS run."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = synth.scan_vs_cad(300_000, 300_000)
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    e.align()
    e.server_time(reset=True)
    its = evs = 0
    for _ in range(3):
        e.align()
        its += e.last_result["iterations"]
        evs += e.last_result["n_evals"]
    t = e.server_time()
    loop_ms = e.last_result["ms_loop"]
    e.close()
    assert t["launches"] == its and t["passes"] == evs, t
    assert 0 < t["ms_per_pass"] < loop_ms, t


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_target_cov_slices_assemble_to_unsharded(part_small, world):
    """the all-gather's data path without RCCL -- the N target-covariance slices
    that ranks 0..N-1 compute before their in-place ncclAllGather (target_cov: points [r cnt,
    (r + 1) cnt) of arrays of N cnt entries), assembled in rank order, are the single-rank target
    covariances bit for bit."""
    from leica_point_cloud_processing_amd.engine import GICPEngine

    scan, cad, _ = part_small
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    full = e.debug_target_cov_slice(1, 0, len(cad))
    assert full.shape == (len(cad), 6)
    parts = [e.debug_target_cov_slice(world, r, len(cad)) for r in range(world)]
    cnt = -(-len(cad) // world)
    assert [len(p) for p in parts] == [max(0, min(len(cad), (r + 1) * cnt) - r * cnt) for r in range(world)]
    asm = np.concatenate(parts)
    assert np.array_equal(asm.view(np.int64), full.view(np.int64))
    # and the cached covariances the aligns use are recomputed afterwards (the slice left them stale)
    T1 = e.align()
    f = GICPEngine()
    f.set_source_xyz(scan)
    f.set_target_xyz(cad)
    np.testing.assert_array_equal(T1, f.align())
    e.close()
    f.close()


def _quit_rank(name, world, rank, n, env, q):
    """one rank of the rank-failure test: rank 1 stops publishing at a pass (MGICP_DEBUG_QUIT_PASS)"""
    import time as _t

    try:
        env = dict(env)
        opts = {"srv_cus": int(env.pop("srv_cus"))} if "srv_cus" in env else {}
        xgmi = env.pop("xgmi", "0") == "1"
        os.environ.update(env)
        from leica_point_cloud_processing_amd import _lib, synth
        from leica_point_cloud_processing_amd.engine import GICPEngine

        scan, cad, _ = synth.scan_vs_cad(n, n)
        e = GICPEngine(device=0, options=opts)
        e.comm_init(world, rank, None)
        e.attach_shm(name, n)
        if xgmi:
            e.attach_xgmi()
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        t0 = _t.perf_counter()
        err = None
        try:
            e.align()
        except _lib.MgicpError as exc:
            err = (exc.code, str(exc))
        dt = _t.perf_counter() - t0
        st = e.pass_stats()
        t1 = _t.perf_counter()
        e.close()  # must not wait on a stuck server
        q.put((rank, err, dt, st, _t.perf_counter() - t1))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, repr(exc), None, None, None))


@pytest.mark.gpu
@pytest.mark.parametrize("xgmi", [0, 1])
def test_shm_rank_quits_mid_align_others_fail_fast(xgmi):
    """a rank that stops publishing its super rows mid-align (MGICP_DEBUG_QUIT_PASS
    on rank 1: its host gives up at pass 5, cancels its server and closes).  The surviving rank
    returns MGICP_E_COMM within the remote deadline (3 s here) -- no hang -- and its context closes at
    once (its server was cancelled, not left waiting for commands).  xgmi = 1 (r05): the rows travel
    through the ranks' IPC-mapped exchange buffers; the survivor's totaler never completes the pass
    and is cancelled with its server."""
    from leica_point_cloud_processing_amd import _lib

    n = 200_000
    name = f"/mgicp_quit_{os.getpid()}_{xgmi}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = []
    for r in range(2):
        env = {"srv_cus": "80", "MGICP_REMOTE_DEADLINE_S": "3", "xgmi": str(xgmi)}
        if r == 1:
            env["MGICP_DEBUG_QUIT_PASS"] = "5"
        procs.append(ctx.Process(target=_quit_rank, args=(name, 2, r, n, env, q)))
    for p in procs:
        p.start()
    got = sorted((q.get(timeout=240) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, err0, dt0, st0, close0), (r1, err1, dt1, st1, close1) = got
    assert not isinstance(err0, str) and err0 is not None, got
    assert err0[0] == _lib.MGICP_E_COMM, err0
    assert err1 is not None and err1[0] == _lib.MGICP_E_COMM, err1
    assert dt0 < 3.0 + 30.0, dt0  # the remote deadline, not the 120 s default or a hang
    assert close0 < 5.0 and close1 < 5.0, (close0, close1)
    assert st0["server_passes"] >= 4, st0
    assert not os.path.exists("/dev/shm" + name)


def _shm_rank(name, world, rank, n, solver, env, q):
    """One rank of an RCCL-free multi-process run on ONE device: detached shard + shared rows."""
    try:
        env = dict(env)
        opts = {"srv_cus": int(env.pop("srv_cus"))} if "srv_cus" in env else {}
        xgmi = env.pop("xgmi", "0") == "1"
        os.environ.update(env)
        from leica_point_cloud_processing_amd import synth
        from leica_point_cloud_processing_amd.engine import GICPEngine

        scan, cad, _ = synth.scan_vs_cad(n, n)
        e = GICPEngine(device=0, solver=solver, options=opts)
        e.comm_init(world, rank, None)
        e.attach_shm(name, n)
        if xgmi:
            e.attach_xgmi()
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        T = e.align()
        res = (e.last_result["iterations"], e.last_result["n_evals"])
        T2 = e.align()  # iterate(): cached grids, same result
        fit = e.getFitnessScore()
        st = e.pass_stats()
        e.close()
        q.put((rank, T, T2, res, fit, st))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, repr(exc), None, None, None, None))


@pytest.mark.gpu
@pytest.mark.parametrize("world,solver,stall,xgmi", [(1, 0, -1, 0), (2, 0, -1, 0), (2, 0, 1, 0), (3, 1, -1, 0),
                                                     (1, 0, -1, 1), (2, 0, -1, 1), (3, 0, -1, 1), (2, 1, -1, 1)])
def test_shared_rows_multiprocess_bitwise_single(world, solver, stall, xgmi):
    """the resident server for N > 1 without a collective.  `world` processes on
    the ONE device of this box (servers capped at 80 CUs each so they fit side by side; RCCL refuses
    two ranks on one GPU, so the ranks are RCCL-free detached shards joined by the shared segment):
    each rank's server writes its supers' rows into the segment, every host takes the fixed-order
    total.  T (first align and iterate()), iterations, passes and fitness are bitwise those of one
    context; with stall >= 0 rank 1 takes one pass over per align.  solver 1: the GN mode's
    moments (and the fitness) gather through the segment.  xgmi = 1 (r05): the
    per-pass rows travel through every rank's IPC-mapped device exchange buffer (the path xGMI carries
    between GPUs; here the ranks share one GPU) and each rank's totaler wave takes the total on the
    device -- bitwise the same."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    n = 400_000
    scan, cad, _ = synth.scan_vs_cad(n, n)
    ref = GICPEngine(solver=solver)
    ref.set_source_xyz(scan)
    ref.set_target_xyz(cad)
    T_ref = ref.align()
    res_ref = (ref.last_result["iterations"], ref.last_result["n_evals"])
    fit_ref = ref.getFitnessScore()
    ref.close()
    name = f"/mgicp_gpu_{os.getpid()}_{world}_{solver}_{stall}_{xgmi}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = []
    for r in range(world):
        env = {"srv_cus": "80", "MGICP_ROW_DEADLINE_MS": "100", "xgmi": str(xgmi)}
        if xgmi:
            env["MGICP_REMOTE_DEADLINE_S"] = "20"  # a missing row fails the test, not a 120 s wait
        if stall >= 0 and r == 1:
            env["MGICP_SRV_STALL_PASS"] = str(stall)
        procs.append(ctx.Process(target=_shm_rank, args=(name, world, r, n, solver, env, q)))
    for p in procs:
        p.start()
    got = sorted((q.get(timeout=240) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, T, T2, res, fit, st in got:
        assert not isinstance(T, str), T
        np.testing.assert_array_equal(T, T_ref)
        np.testing.assert_array_equal(T2, T_ref)
        assert res == res_ref
        assert fit == fit_ref
        assert st["transport"] == (4 if xgmi else 2), st
        if solver == 0:
            assert st["server_passes"] > 0, st
            assert st["takeovers"] == (2 if (stall >= 0 and rank == 1) else 0), st
    assert not os.path.exists("/dev/shm" + name)


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


class _FakeEngine:
    """Records the transport calls setup_transport makes (CPU test of its decisions)."""

    fail_comm_on = ()

    def __init__(self, rank):
        self.rank = rank
        self.calls = []

    @staticmethod
    def unique_id():
        return bytes(range(128))

    def comm_init(self, world, rank, uid):
        self.calls.append(("comm_init", uid is not None))
        if uid is not None and rank in self.fail_comm_on:
            raise RuntimeError("ncclCommInitRank: unhandled system error (simulated)")

    def attach_shm(self, name, n):
        self.calls.append(("attach_shm", name.startswith("/mgicp_")))

    def detach_shm(self):
        self.calls.append(("detach_shm",))

    def attach_xgmi(self, on=True):
        self.calls.append(("attach_xgmi", on))


def _transport_worker(rank, world, port, fail_on, transport, q):
    from leica_point_cloud_processing_amd.parallel import Rendezvous, setup_transport

    pg = Rendezvous(rank, world, addr="127.0.0.1", port=port, timeout=60)
    _FakeEngine.fail_comm_on = fail_on
    eng = _FakeEngine(rank)
    try:
        tr = setup_transport(eng, pg, world, rank, transport, 1000)
        q.put((rank, tr["transport"], tr["rccl"], eng.calls))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, repr(exc), None, eng.calls))
    pg.close()


@pytest.mark.parametrize("fail_on,transport", [((), "xgmi"), ((1,), "xgmi"), ((0, 1), "rccl"), ((1,), "shm")])
def test_setup_transport_degrades_when_rccl_fails(fail_on, transport):
    """if ncclCommInitRank fails on ANY rank, EVERY rank becomes an RCCL-free shard
    (comm_init(N, r, NULL)) and the rows go through the segment (an 'rccl' request too) / xGMI; all ranks
    agree on the same transport."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, world, port, fail_on, transport, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=60) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    names = {t for _, t, _, _ in res}
    assert len(names) == 1, res
    for rank, tname, rccl, calls in res:
        assert rccl == (not fail_on), res
        if fail_on:
            assert ("comm_init", False) in calls, calls  # the RCCL-free shard
            assert ("attach_shm", True) in calls, calls
            assert "no RCCL" in tname
        want_x = transport == "xgmi"
        assert (("attach_xgmi", True) in calls) == want_x, calls
        assert tname.startswith("xGMI" if want_x else "shm rows"), tname


def _fallback_rank(world, rank, port, n, transport, q):
    try:
        from leica_point_cloud_processing_amd import synth
        from leica_point_cloud_processing_amd.engine import GICPEngine
        from leica_point_cloud_processing_amd.parallel import Rendezvous, setup_transport

        os.environ["MGICP_REMOTE_DEADLINE_S"] = "20"
        pg = Rendezvous(rank, world, addr="127.0.0.1", port=port, timeout=120)
        scan, cad, _ = synth.scan_vs_cad(n, n)
        e = GICPEngine(device=0, options={"srv_cus": 80})
        tr = setup_transport(e, pg, world, rank, transport, n, force_rccl_fail=True)
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        T = e.align()
        res = (e.last_result["iterations"], e.last_result["n_evals"], e.last_result["n_corr"])
        st = e.pass_stats()
        e.close()
        pg.close()
        q.put((rank, T, res, st, tr["transport"]))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, repr(exc), None, None, None))


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["shm", "xgmi"])
def test_rccl_free_fallback_bitwise_single(transport):
    """a 2-process run whose RCCL init 'failed' (setup_transport(force_rccl_fail)) runs
    as RCCL-free shards -- the target's covariances computed whole on each rank, rows through the segment
    or the xGMI exchange -- and gives T, iterations, passes and n_corr bitwise equal to one context."""
    from leica_point_cloud_processing_amd import synth
    from leica_point_cloud_processing_amd.engine import GICPEngine

    n, world = 300_000, 2
    scan, cad, _ = synth.scan_vs_cad(n, n)
    ref = GICPEngine()
    ref.set_source_xyz(scan)
    ref.set_target_xyz(cad)
    T_ref = ref.align()
    res_ref = (ref.last_result["iterations"], ref.last_result["n_evals"], ref.last_result["n_corr"])
    ref.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_rank, args=(world, r, port, n, transport, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted((q.get(timeout=240) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, T, res, st, tname in got:
        assert not isinstance(T, str), T
        np.testing.assert_array_equal(T, T_ref)
        assert res == res_ref
        assert st["transport"] == (4 if transport == "xgmi" else 2), st
        assert "no RCCL" in tname, tname
