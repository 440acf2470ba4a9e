"""Host-side process group for multi-GPU runs: a TCP star hosted by rank 0.

One process per GPU (launched by `torch.distributed.run`, which sets RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT).  The self-play path has no
data collective (games shard by id), so the ranks only need a start/stop
barrier, scalar reductions (sum of work, max of time) and, for the
data-parallel learner, the broadcast of the 128-byte RCCL unique id.  Doing
that over plain sockets keeps torch — and the HIP runtime it bundles under the
same SONAME as /opt/rocm's — out of the GPU processes, so every rank runs
libspai on the ROCm runtime it was built for.

Port: SPAI_GROUP_PORT, else MASTER_PORT + 17 (MASTER_PORT itself is taken by
the launcher's rendezvous store).
"""
import json
import os
import socket
import struct
import time

import numpy as np


def _send(sock, obj):
    data = json.dumps(obj).encode()
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("host group peer closed the connection")
        buf += chunk
    return bytes(buf)


def _send_bytes(sock, data):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_bytes(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


def _recv(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return json.loads(_recv_exact(sock, n))


class HostGroup:
    def __init__(self, rank=None, world=None, addr=None, port=None, timeout=600.0):
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
        self.peers = {}      # rank 0: rank -> socket
        self.sock = None     # other ranks: connection to rank 0
        if self.world == 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("SPAI_GROUP_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 17))
        deadline = time.time() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(max(1.0, deadline - time.time()))
            while len(self.peers) < self.world - 1:
                conn, _ = srv.accept()
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                self.peers[int(_recv(conn))] = conn
            srv.close()
        else:
            while True:
                try:
                    self.sock = socket.create_connection((addr, port), timeout=10.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.2)
            self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.sock.settimeout(None)
            _send(self.sock, self.rank)

    def allgather(self, obj):
        """list of every rank's obj (rank order) on every rank"""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [_recv(self.peers[r]) for r in range(1, self.world)]
            for r in range(1, self.world):
                _send(self.peers[r], out)
            return out
        _send(self.sock, obj)
        return _recv(self.sock)

    def allreduce(self, values, op="sum"):
        parts = self.allgather([float(v) for v in values])
        red = max if op == "max" else sum
        return [red(p[i] for p in parts) for i in range(len(values))]

    def barrier(self):
        self.allgather(0)

    def allreduce_f32(self, buf):
        """element-wise sum of a float32 array over the ranks, in place, summed in
        rank order at rank 0 (so every rank gets bit-identical values) — the host
        collective of spai.Learner.set_host_comm"""
        if self.world == 1:
            return buf
        if self.rank == 0:
            tot = np.array(buf, np.float32, copy=True)
            for r in range(1, self.world):
                tot += np.frombuffer(_recv_bytes(self.peers[r]), np.float32)
            data = tot.tobytes()
            for r in range(1, self.world):
                _send_bytes(self.peers[r], data)
            buf[:] = tot
        else:
            _send_bytes(self.sock, np.ascontiguousarray(buf, np.float32).tobytes())
            buf[:] = np.frombuffer(_recv_bytes(self.sock), np.float32)
        return buf

    def broadcast_bytes(self, data=None):
        """rank 0's bytes on every rank"""
        return bytes.fromhex(self.allgather(data.hex() if self.rank == 0 else "")[0])

    def close(self):
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None
