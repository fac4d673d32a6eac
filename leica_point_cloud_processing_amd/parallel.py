"""Multi-GPU plumbing: one process per GPU, point-range shards of the source cloud.

Data path: libmgicp.so all-reduces the 16 objective sums of every BFGS pass over RCCL (xGMI);
the communicator is created from a 128-byte unique id (mgicp_get_unique_id / mgicp_comm_init).

Control path (this module): a tiny TCP rendezvous for the id broadcast, barriers and the
max-over-ranks timer.  It deliberately does not use torch.distributed: importing torch loads
torch's own bundled HIP/HSA runtime (torch/lib/libamdhip64.so, ROCm 7.0) next to the ROCm 7.2
runtime libmgicp.so links, and two HIP runtimes in one process corrupt the heap at teardown
(observed on MI355X: "double free or corruption").  Processes are still launched by
`python -m torch.distributed.run`, which only sets RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT.
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import time


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Source points [p0, p1) (grid-sorted order) owned by `rank` -- mirrors the engine's
    mgicp_ctx::shard_p0/shard_p1 (contiguous, sizes differ by at most one)."""
    return n * rank // world, n * (rank + 1) // world


def _send(sock: socket.socket, obj) -> None:
    data = pickle.dumps(obj)
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return pickle.loads(_recv_exact(sock, n))


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
            srv.settimeout(timeout)
            peers = {}
            while len(peers) < world - 1:
                conn, _ = srv.accept()
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                peers[_recv(conn)] = conn
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
            _send(s, rank)
            self.sock = s

    def broadcast(self, obj=None):
        """Rank 0's `obj` to every rank."""
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
        vals = self.gather(x)
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
