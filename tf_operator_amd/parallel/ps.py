"""Parameter-server data parallelism (reference payload
dist_mnist.py:149-219: replica_device_setter puts variables on /job:ps,
workers push gradients and pull parameters every step, optionally through
SyncReplicasOptimizer which aggregates N gradients before one update).

Kept for TFJob API parity (PS replicas), NOT the MI355X performance path
(that is RCCL all-reduce, :mod:`tf_operator_amd.parallel.ddp`).  The wire
protocol is a length-prefixed binary TCP stream:

    PULL                       -> version:int64, params:fp32[n]
    PUSH version grads:fp32[n] -> version:int64, params:fp32[n]
    STOP

* async (P1): every PUSH is applied immediately (Adam on the server);
* sync  (P2): the server waits for `replicas_to_aggregate` pushes of the same
  version, applies their mean once, then answers all of them.

Multiple PS replicas shard the flat parameter vector contiguously.
"""
from __future__ import annotations

import socket
import socketserver
import struct
import threading

import numpy as np

_HDR = struct.Struct("<cqq")  # op, version, nbytes


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k
    return bytes(buf)


def _send(sock, op, version, payload=b""):
    sock.sendall(_HDR.pack(op, version, len(payload)) + payload)


def _recv(sock):
    op, version, n = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return op, version, _recv_exact(sock, n) if n else b""


class _Adam:
    def __init__(self, n, lr, b1=0.9, b2=0.999, eps=1e-8):
        self.m = np.zeros(n, np.float32)
        self.v = np.zeros(n, np.float32)
        self.t = 0
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps

    def step(self, p, g):
        self.t += 1
        self.m = self.b1 * self.m + (1 - self.b1) * g
        self.v = self.b2 * self.v + (1 - self.b2) * g * g
        mh = self.m / (1 - self.b1 ** self.t)
        vh = self.v / (1 - self.b2 ** self.t)
        p -= self.lr * mh / (np.sqrt(vh) + self.eps)


class ParameterServer:
    """Owns one contiguous shard of the flat fp32 parameter vector."""

    def __init__(self, init_params: np.ndarray, lr=0.01, sync_replicas=0, host="0.0.0.0", port=0):
        self.params = np.array(init_params, dtype=np.float32, copy=True)
        self.opt = _Adam(self.params.size, lr)
        self.version = 0
        self.sync = int(sync_replicas)
        self.lock = threading.Condition()
        self.pending = []
        self.stopped = threading.Event()
        ps = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                sock = self.request
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                try:
                    while True:
                        op, version, payload = _recv(sock)
                        if op == b"L":
                            v, p = ps.pull()
                        elif op == b"P":
                            v, p = ps.push(version, np.frombuffer(payload, np.float32))
                        elif op == b"S":
                            ps.stopped.set()
                            return
                        else:
                            return
                        _send(sock, b"R", v, p.tobytes())
                except (ConnectionError, OSError):
                    return

        class Server(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self.server = Server((host, port), Handler)
        self.port = self.server.server_address[1]

    def pull(self):
        with self.lock:
            return self.version, self.params.copy()

    def push(self, version, grad):
        with self.lock:
            if self.sync <= 1:
                self.opt.step(self.params, grad)
                self.version += 1
                return self.version, self.params.copy()
            self.pending.append(grad.copy())
            target = self.version + 1
            if len(self.pending) >= self.sync:
                g = np.mean(self.pending[: self.sync], axis=0)
                self.pending = self.pending[self.sync:]
                self.opt.step(self.params, g)
                self.version += 1
                self.lock.notify_all()
            else:
                while self.version < target and not self.stopped.is_set():
                    self.lock.wait(timeout=1.0)
            return self.version, self.params.copy()

    def serve_forever(self):
        t = threading.Thread(target=self.server.serve_forever, daemon=True)
        t.start()
        self.stopped.wait()
        self.server.shutdown()

    def start(self):
        threading.Thread(target=self.server.serve_forever, daemon=True).start()
        return self

    def close(self):
        self.stopped.set()
        self.server.shutdown()
        self.server.server_close()


class PSClient:
    """Worker side: the flat vector is split contiguously over the PS shards."""

    def __init__(self, endpoints, sizes):
        self.socks = []
        for host, port in endpoints:
            s = socket.create_connection((host, port), timeout=60)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            self.socks.append(s)
        self.sizes = list(sizes)
        self.version = 0

    def _gather(self, replies):
        vs, ps = zip(*replies)
        self.version = max(vs)
        return np.concatenate([np.frombuffer(p, np.float32) for p in ps])

    def pull(self) -> np.ndarray:
        out = []
        for s in self.socks:
            _send(s, b"L", 0)
            _, v, p = _recv(s)
            out.append((v, p))
        return self._gather(out)

    def push(self, grad: np.ndarray) -> np.ndarray:
        off = 0
        for s, n in zip(self.socks, self.sizes):
            _send(s, b"P", self.version, np.ascontiguousarray(grad[off:off + n], np.float32).tobytes())
            off += n
        out = []
        for s in self.socks:
            _, v, p = _recv(s)
            out.append((v, p))
        return self._gather(out)

    def stop_servers(self):
        for s in self.socks:
            try:
                _send(s, b"S", 0)
            except OSError:
                pass

    def close(self):
        for s in self.socks:
            s.close()


def shard_sizes(n, num_ps):
    base, rem = divmod(n, num_ps)
    return [base + (1 if i < rem else 0) for i in range(num_ps)]
