"""Multi-GPU plumbing: one process per GPU, point-range shards of the source cloud.

Data path: libmgicp.so all-gathers the ranks' super partials of every BFGS pass over RCCL (xGMI)
and sums them in a fixed order, so N GPUs reproduce the single-GPU sums bit for bit; the
communicator is created from a 128-byte unique id (mgicp_get_unique_id / mgicp_comm_init).

Control path (this module): a tiny TCP rendezvous for the id broadcast, barriers and the
max-over-ranks timer.  It deliberately does not use torch.distributed: importing torch loads
torch's own bundled HIP/HSA runtime (torch/lib/libamdhip64.so, ROCm 7.0) next to the ROCm 7.2
runtime libmgicp.so links, and two HIP runtimes in one process corrupt the heap at teardown
(observed on MI355X: "double free or corruption"; _lib.load() now refuses that combination).
Processes are still launched by `python -m torch.distributed.run`, which only sets RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT.

Wire format: nothing is unpickled.  Every message is a typed frame (1-byte tag, 4-byte length,
payload): raw bytes, one little-endian float64, or "none".  A connecting peer first sends a
fixed hello (magic, rank as int32, and the SHA-256 of MGICP_CTRL_SECRET when that variable is
set); rank 0 accepts only ranks 1..world-1, each once, and drops any other connection.
"""
from __future__ import annotations

import hashlib
import os
import socket
import struct
import time

_MAGIC = b"MGICPRV1"
_T_NONE, _T_BYTES, _T_F64 = 0, 1, 2
_MAX_FRAME = 1 << 20  # control messages are tiny (the unique id is 128 bytes)


# The fixed reduction tree (csrc/mgicp_internal.hpp): chunks of CHUNK_PTS grid-sorted source
# positions, supers of SUPER_CHUNKS chunks; shards start on super boundaries.
CHUNK_PTS = 1024
SUPER_CHUNKS = 32
SUPER_PTS = CHUNK_PTS * SUPER_CHUNKS


def super_first(rank: int, nsup: int, world: int) -> int:
    """First super of `rank` (mirrors mgicp::super_first)."""
    return nsup * rank // world


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Source points [p0, p1) (grid-sorted order) owned by `rank` -- mirrors the engine's
    mgicp_ctx::shard_p0/shard_p1: rank r owns supers [nsup * r / N, nsup * (r + 1) / N), so
    shards are contiguous, start on super boundaries and differ by at most one super."""
    nsup = -(-n // SUPER_PTS)
    return (min(n, super_first(rank, nsup, world) * SUPER_PTS),
            min(n, super_first(rank + 1, nsup, world) * SUPER_PTS))


def fixed_total(rows):
    """Host mirror of the device's total over supers (wave_total in mgicp_kernels.hip, and the
    host-row total of shm_rows.hpp): lane l sums supers l, l + 64, ... sequentially from 0.0, then
    the 64-lane shuffle tree lanes[i] += lanes[i + off] for off = 32 ... 1; lane 0 is the total.
    rows: sequence of equal-length float64 vectors in global super order."""
    import numpy as np

    rows = [np.asarray(r, np.float64) for r in rows]
    lanes = [np.zeros_like(rows[0]) for _ in range(64)]
    for sg, r in enumerate(rows):
        lanes[sg % 64] = lanes[sg % 64] + r
    off = 32
    while off:
        for i in range(off):
            lanes[i] = lanes[i] + lanes[i + off]
        off >>= 1
    return lanes[0]


def combine_supers(rows, nsup: int, world: int):
    """Host mirror of the multi-GPU finish's indexing: the supers of every rank (rows[r] = rank r's
    supers, padded to a common length) in global order."""
    out = []
    for r in range(world):
        cnt = super_first(r + 1, nsup, world) - super_first(r, nsup, world)
        out.extend(rows[r][:cnt])
    assert len(out) == nsup
    return out


def _secret_digest() -> bytes:
    s = os.environ.get("MGICP_CTRL_SECRET", "")
    return hashlib.sha256(s.encode()).digest() if s else bytes(32)


def _encode(obj) -> bytes:
    if obj is None:
        tag, payload = _T_NONE, b""
    elif isinstance(obj, (bytes, bytearray)):
        tag, payload = _T_BYTES, bytes(obj)
    elif isinstance(obj, (int, float)):
        tag, payload = _T_F64, struct.pack("<d", float(obj))
    else:
        raise TypeError(f"rendezvous carries bytes, float or None, not {type(obj).__name__}")
    if len(payload) > _MAX_FRAME:
        raise ValueError("rendezvous frame too large")
    return struct.pack("<BI", tag, len(payload)) + payload


def _send(sock: socket.socket, obj) -> None:
    sock.sendall(_encode(obj))


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket):
    tag, n = struct.unpack("<BI", _recv_exact(sock, 5))
    if n > _MAX_FRAME:
        raise ConnectionError("rendezvous frame too large")
    payload = _recv_exact(sock, n)
    if tag == _T_NONE and n == 0:
        return None
    if tag == _T_BYTES:
        return payload
    if tag == _T_F64 and n == 8:
        return struct.unpack("<d", payload)[0]
    raise ConnectionError(f"malformed rendezvous frame (tag {tag}, {n} bytes)")


def _hello(rank: int) -> bytes:
    return _MAGIC + struct.pack("<i", rank) + _secret_digest()


_HELLO_LEN = len(_MAGIC) + 4 + 32


def _check_hello(data: bytes, world: int, seen: dict) -> int | None:
    """The peer's rank when its hello is well-formed, authorised and new; else None."""
    if len(data) != _HELLO_LEN or data[:len(_MAGIC)] != _MAGIC:
        return None
    (r,) = struct.unpack("<i", data[len(_MAGIC):len(_MAGIC) + 4])
    if data[len(_MAGIC) + 4:] != _secret_digest():
        return None
    if not (1 <= r < world) or r in seen:
        return None
    return r


class Rendezvous:
    """Star-topology control plane: rank 0 serves, ranks 1..world-1 connect."""

    def __init__(self, rank: int, world: int, addr: str | None = None, port: int | None = None,
                 timeout: float = 300.0):
        self.rank, self.world = rank, world
        self.peers: list[socket.socket] = []
        self.sock: socket.socket | None = None
        if world == 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            # MASTER_PORT itself belongs to the launcher's c10d store
            port = int(os.environ.get("MGICP_CTRL_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 17))
        deadline = time.time() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            peers: dict[int, socket.socket] = {}
            try:
                while len(peers) < world - 1:
                    left = deadline - time.time()
                    if left <= 0:
                        raise TimeoutError(f"rendezvous: {len(peers)} of {world - 1} peers joined")
                    srv.settimeout(left)
                    conn, _ = srv.accept()
                    conn.settimeout(min(10.0, max(0.1, left)))
                    try:
                        r = _check_hello(_recv_exact(conn, _HELLO_LEN), world, peers)
                    except (OSError, ConnectionError):
                        r = None
                    if r is None:  # bogus, unauthorised or duplicate peer: drop it, keep waiting
                        conn.close()
                        continue
                    conn.settimeout(timeout)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    peers[r] = conn
            finally:
                srv.close()
            self.peers = [peers[r] for r in range(1, world)]
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(_hello(rank))
            self.sock = s

    def broadcast(self, obj=None):
        """Rank 0's `obj` (bytes, float or None) to every rank."""
        if self.world == 1:
            return obj
        if self.rank == 0:
            for p in self.peers:
                _send(p, obj)
            return obj
        return _recv(self.sock)

    def gather(self, obj):
        """List of every rank's `obj` on rank 0 (None elsewhere)."""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            return [obj] + [_recv(p) for p in self.peers]
        _send(self.sock, obj)
        return None

    def allreduce_max(self, x: float) -> float:
        vals = self.gather(float(x))
        return self.broadcast(max(vals) if self.rank == 0 else None)

    def barrier(self) -> None:
        self.gather(None)
        self.broadcast(None)

    def close(self) -> None:
        for p in self.peers:
            p.close()
        if self.sock is not None:
            self.sock.close()
        self.peers, self.sock = [], None


def setup_transport(eng, pg, world: int, rank: int, transport: str, n_source: int, probe=None,
                    force_rccl_fail: bool = False) -> dict:
    """Join `world` ranks (one engine per process) and pick the per-pass exchange; every rank calls this
    with the same arguments, every decision is agreed through `pg` (Rendezvous.broadcast /
    allreduce_max), so all ranks end on the same transport.

    r06: a first multi-GPU run degrades instead of dying.  RCCL carries only the
    one-time split of the target covariances (and the GN mode's per-iteration gathers when no segment
    exists); if the unique id or ncclCommInitRank fails on any rank, every rank becomes an RCCL-free
    shard (mgicp_comm_init(ctx, N, r, NULL)): the target's covariances are then computed whole on every
    rank (per-point values, the same bits as the split + all-gather) and the per-pass rows go through the
    node-wide shared segment (or over xGMI).  force_rccl_fail: take that path without trying RCCL (test).

    probe: optional (source, target) clouds for one align through the xGMI exchange; a failure there
    falls back to the host segment.  Returns {"transport": str, "rccl": bool, "notes": [...]}.
    """
    notes = []
    cerr = None
    if force_rccl_fail:
        cerr = "forced (force_rccl_fail)"
    else:
        uid = b""
        if rank == 0:
            try:
                uid = type(eng).unique_id()
            except Exception as exc:  # noqa: BLE001 -- rank 0's id failed: nobody tries RCCL
                cerr = f"unique id: {exc}"
        uid = pg.broadcast(uid if rank == 0 else None)
        if not uid:
            cerr = cerr or "unique id unavailable on rank 0"
        else:
            try:
                eng.comm_init(world, rank, uid)
            except Exception as exc:  # noqa: BLE001 -- reported
                cerr = f"ncclCommInitRank: {exc}"
    rccl = pg.allreduce_max(1.0 if cerr else 0.0) == 0
    if not rccl:
        notes.append(f"RCCL unavailable ({cerr or 'on another rank'}): RCCL-free shards, target covariances "
                     "computed whole on every rank")
        eng.comm_init(world, rank, None)
        if transport == "rccl":
            transport = "shm"
    if transport == "rccl":
        return {"transport": "rccl", "rccl": True, "notes": notes}
    import secrets

    name = pg.broadcast(f"/mgicp_{os.getpid()}_{secrets.token_hex(6)}".encode() if rank == 0 else None)
    err = None
    try:
        eng.attach_shm(name.decode(), n_source)
    except Exception as exc:  # noqa: BLE001 -- reported
        err = str(exc)
    if pg.allreduce_max(1.0 if err else 0.0) > 0:
        if not err:
            eng.detach_shm()
        if not rccl:
            raise RuntimeError(f"no exchange for {world} ranks: RCCL ({cerr}) and the shared segment "
                               f"({err or 'on another rank'}) both failed")
        return {"transport": f"rccl (shared segment unavailable: {err or 'on another rank'})", "rccl": True,
                "notes": notes}
    tail = "rccl (target covariances)" if rccl else "no RCCL (target covariances computed on every rank)"
    out = {"transport": f"shm rows + {tail}", "rccl": rccl, "notes": notes}
    if transport != "xgmi":
        return out
    xerr = None
    try:
        eng.attach_xgmi()
    except Exception as exc:  # noqa: BLE001 -- reported
        xerr = str(exc)
    if pg.allreduce_max(1.0 if xerr else 0.0) > 0:
        if not xerr:
            eng.attach_xgmi(False)
        out["transport"] = f"shm rows (xGMI exchange unavailable: {xerr or 'on another rank'}) + {tail}"
        return out
    out["transport"] = f"xGMI row exchange + device totals; shm rendezvous/gathers; {tail}"
    if probe is not None:
        # one align on a sample through the exchange: if rows written into peer GPUs' memory never show up
        # there, every rank falls back to the host segment (the same sums) instead of failing the run
        perr = None
        try:
            eng.set_source_xyz(probe[0])
            eng.set_target_xyz(probe[1])
            eng.align()
        except Exception as exc:  # noqa: BLE001 -- reported
            perr = str(exc)
        if pg.allreduce_max(1.0 if perr else 0.0) > 0:
            eng.attach_xgmi(False)
            out["transport"] = f"shm rows (xGMI probe align failed: {perr or 'on another rank'}) + {tail}"
    return out
