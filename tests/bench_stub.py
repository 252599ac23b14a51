"""Launcher for the CPU test of bench.py's multi-rank orchestration (tests/test_shard.py): runs
``bench.main()`` with the device Solver and the RCCL communicator replaced by CPU stubs, so the
slicing, the barriers around the timed region, the max-over-ranks clock, the other-scaling leg,
the gather and the rank-0-only JSON line all execute across real processes without a GPU.

* ``StubSolver`` keeps bench.py's call surface (upload, scp_iterate, timing, getters) and sleeps a
  fixed time per SCP iteration, so the timed region is measurable;
* ``SocketComm`` restates the RcclComm surface over a TCP star at MASTER_PORT + 2: the id
  rendezvous of cmpc.shard.exchange_id (MASTER_PORT + 1), an elementwise max-reduction
  (allreduce_max / barrier) and the rank-ordered gather of every slice to rank 0.

Usage (one process per rank, via cmpc.shard.spawn_local): python tests/bench_stub.py OUT_DIR
<bench.py arguments>; rank r's stdout goes to OUT_DIR/rank<r>.txt and its gathered result, on
rank 0, to OUT_DIR/gather.npz.
"""
import io
import os
import socket
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]

import numpy as np  # noqa: E402

STEP_S = 0.002   # stub SCP iteration time


class StubSolver:
    def __init__(self, robot, N, max_batch, precision='fp64', device=0):
        self.robot, self.N, self.max_batch, self.B = robot, int(N), int(max_batch), 0
        self.nc = 4 if robot == 'solo12' else 2
        self.device = device
        self.iters = 0
        self._timing = None

    def upload(self, pb, set_params=True):
        assert pb.B <= self.max_batch and pb.N == self.N
        self.B = pb.B
        self.first = pb   # to check the slice on rank r is the global batch's [lo, hi)
        self.iters = 0

    def set_params(self, params):
        pass

    def scp_iterate(self, fixed_iters=True):
        time.sleep(STEP_S)
        self.iters += 1
        if self._timing is not None:
            self._timing['iterations'] += 1
            for k, f in (('linearize_ms', 0.1), ('assemble_ms', 0.05), ('qp_ms', 0.8), ('accept_ms', 0.05)):
                self._timing[k] += f * STEP_S * 1e3

    def synchronize(self):
        pass

    def timing_begin(self):
        self._timing = dict(linearize_ms=0.0, assemble_ms=0.0, qp_ms=0.0, accept_ms=0.0, iterations=0)

    def timing_end(self):
        t, self._timing = self._timing, None
        t['total_ms'] = sum(t[k] for k in ('linearize_ms', 'assemble_ms', 'qp_ms', 'accept_ms'))
        return t

    def qp_iterations_total(self):
        return 5 * self.B

    def qp_solution(self, with_y=True):
        return np.zeros((self.B, 1)), None, np.ones(self.B, np.int32), np.full(self.B, 5, np.int32)

    def qp_kernel(self):
        return 'stub'

    def qp_info(self):
        return np.full(self.B, 0.5), np.zeros(self.B, np.int32)

    def qp_exit(self):
        return np.zeros(self.B, np.int32), np.zeros(self.B, np.int32)

    def solve_scp(self, fixed_iters=False):
        self.scp_iterate()
        return 1

    def solution(self, pinned=False, with_ks=True):
        B, N = self.B, self.N
        X = np.broadcast_to(self.first.Xbar[:, :, :], (B, N + 1, 9)).copy()
        return dict(X=X, U=np.zeros((B, N, 12)), K=np.zeros((B, N, 12, 9)), Sigma=np.zeros((B, N + 1, 9, 9)),
                    n_accepted=np.ones(B, np.int32), iterations=np.ones(B, np.int32),
                    status=np.ones(B, np.int32), weight=np.zeros(B), radius=np.zeros(B))

    def prefetch_ks(self):
        pass

    def close(self):
        pass


def _send(sock, arr):
    """one numpy array (npy format, no pickling)"""
    buf = io.BytesIO()
    np.save(buf, np.asarray(arr), allow_pickle=False)
    b = buf.getvalue()
    sock.sendall(len(b).to_bytes(8, 'little') + b)


def _recv(sock):
    from cmpc.shard import _recv_exact
    n = int.from_bytes(_recv_exact(sock, 8), 'little')
    return np.load(io.BytesIO(_recv_exact(sock, n)), allow_pickle=False)


class SocketComm:
    """RcclComm's surface over a TCP star (rank 0 the hub)."""

    def __init__(self, solver, rank, world, addr='127.0.0.1', port=29500):
        from cmpc.shard import ID_BYTES, exchange_id
        self.s, self.rank, self.world = solver, rank, world
        self.uid = exchange_id(rank, world, lambda: bytes(ID_BYTES), addr, port, timeout=60.0)
        if rank == 0:
            srv = socket.socket()
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port + 2))
            srv.listen(world)
            srv.settimeout(60.0)
            self.peers = {}
            for _ in range(world - 1):
                c, _ = srv.accept()
                self.peers[int(_recv(c))] = c
            srv.close()
        else:
            deadline = time.monotonic() + 60.0
            while True:
                try:
                    self.hub = socket.create_connection((addr, port + 2), timeout=60.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            _send(self.hub, rank)
        self.n_allreduce = 0
        self.n_gather = 0

    def bcast_params(self, params=None, capacity=8):
        if self.rank == 0:
            for c in self.peers.values():
                _send(c, len(params))
        else:
            assert params is None and int(_recv(self.hub)) >= 1

    def allreduce_max(self, values):
        v = np.asarray(values, float).copy()
        self.n_allreduce += 1
        if self.rank == 0:
            for r in sorted(self.peers):
                v = np.maximum(v, _recv(self.peers[r]))
            for c in self.peers.values():
                _send(c, v)
            return v
        _send(self.hub, v)
        return _recv(self.hub)

    def barrier(self):
        self.allreduce_max([0.0])

    def gather_solution(self, root=0):
        sol = self.s.solution()
        mine = (sol['X'], sol['status'])
        self.n_gather += 1
        if self.rank != 0:
            _send(self.hub, mine[0])
            _send(self.hub, mine[1])
            return None
        parts = [mine] + [(_recv(self.peers[r]), _recv(self.peers[r])) for r in sorted(self.peers)]
        out = dict(X=np.concatenate([p[0] for p in parts]), status=np.concatenate([p[1] for p in parts]))
        self.gathered = out
        return out

    def close(self):
        for c in getattr(self, 'peers', {}).values():
            c.close()
        if hasattr(self, 'hub'):
            self.hub.close()


def main():
    out_dir = sys.argv[1]
    rank = int(os.environ.get('RANK', 0))
    sys.argv = [os.path.join(ROOT, 'bench.py')] + sys.argv[2:]
    import cmpc._lib
    import cmpc.shard
    cmpc._lib.Solver = StubSolver
    made = []

    class Comm(SocketComm):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            made.append(self)
    cmpc.shard.RcclComm = Comm
    import bench
    f = open(os.path.join(out_dir, 'rank%d.txt' % rank), 'w')
    sys.stdout = f
    try:
        bench.main()
    finally:
        sys.stdout = sys.__stdout__
        f.close()
    if rank == 0 and made and hasattr(made[0], 'gathered'):
        np.savez(os.path.join(out_dir, 'gather.npz'), **made[0].gathered)
    with open(os.path.join(out_dir, 'calls%d.txt' % rank), 'w') as g:
        g.write('%d %d' % (made[0].n_allreduce, made[0].n_gather) if made else '0 0')


if __name__ == '__main__':
    main()
