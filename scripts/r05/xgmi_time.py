"""r05: per-pass time of the N > 1 transports on ONE GPU (N processes, servers on 80 CUs each): the
shared host segment (rows through host memory, every host totals) vs the xGMI row exchange (rows into
IPC-mapped device buffers, a totaler wave per rank).  Small clouds, so a pass is mostly its round trip.
usage: python3 scripts/r05/xgmi_time.py [n_points] [aligns]"""
import json, os, sys, time
import multiprocessing as mp

sys.path.insert(0, os.getcwd())


def rank_main(name, world, rank, n, aligns, xgmi, q):
    try:
        from leica_point_cloud_processing_amd import synth
        from leica_point_cloud_processing_amd.engine import GICPEngine

        scan, cad, _ = synth.scan_vs_cad(n, n)
        e = GICPEngine(device=0, options={"srv_cus": 80})
        if world > 1 or xgmi >= 0:
            e.comm_init(world, rank, None)
            e.attach_shm(name, n)
            if xgmi == 1:
                e.attach_xgmi()
        e.set_source_xyz(scan)
        e.set_target_xyz(cad)
        e.align()
        e.align()
        e.server_time(reset=True)
        t0 = time.perf_counter()
        passes = 0
        for _ in range(aligns):
            e.align()
            passes += e.last_result["n_evals"]
        dt = time.perf_counter() - t0
        st = e.server_time(reset=True)
        e.close()
        q.put((rank, 1e3 * dt / passes, st["ms_per_pass"], passes))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, repr(exc), None, None))


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    aligns = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ctx = mp.get_context("spawn")
    for world, xgmi in ((1, -1), (1, 0), (1, 1), (2, 0), (2, 1), (3, 0), (3, 1)):
        q = ctx.Queue()
        name = f"/mgicp_xt_{os.getpid()}_{world}_{xgmi}"
        ps = [ctx.Process(target=rank_main, args=(name, world, r, n, aligns, xgmi, q)) for r in range(world)]
        for p in ps:
            p.start()
        got = sorted((q.get(timeout=300) for _ in ps), key=lambda t: t[0])
        for p in ps:
            p.join(timeout=60)
        label = {-1: "plain (host rows)", 0: "shared segment", 1: "xGMI exchange"}[xgmi]
        print(json.dumps({"world": world, "transport": label, "n": n,
                          "ms_per_pass_wall": [round(g[1], 4) if not isinstance(g[1], str) else g[1] for g in got],
                          "ms_per_pass_server": [round(g[2], 4) if g[2] else None for g in got],
                          "passes": got[0][3]}), flush=True)
