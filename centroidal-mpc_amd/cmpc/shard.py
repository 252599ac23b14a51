"""Multi-GPU batch split: one process per GPU, contiguous problem slices, RCCL over xGMI around the
loop and nothing inside it.  No PyTorch.

Problems are independent, so rank r of G solves problems [lo_r, hi_r) of the global batch on its
own device.  The only communication is RCCL through libcmpc's C ABI (include/cmpc.h,
``cmpc_comm_*``):

* ``RcclComm.bcast_params``: the shared parameter classes from rank 0;
* ``RcclComm.allreduce_max``: the barrier of a timed region and its max-over-ranks clock;
* ``RcclComm.gather_solution``: every rank's accepted X, U and statuses to rank 0, rank-major
  (= the global problem order of contiguous slices).

The RCCL unique id is handed from rank 0 to the others over a TCP socket at (MASTER_ADDR,
MASTER_PORT + 1) (``exchange_id``; torchrun keeps its own store on MASTER_PORT).  ``spawn_local``
starts the per-GPU processes itself when no launcher did (``bench.py --gpus N``); the parent
process never touches the GPU.
"""
import ctypes
import os
import socket
import subprocess
import sys
import time

import numpy as np

ID_BYTES = 128


def shard_bounds(B, rank, world):
    """[lo, hi) of rank's contiguous slice: floor(B / world) or ceil(B / world) problems per rank
    (the first B % world ranks one more), so no rank is empty while B >= world (an empty rank could
    not join the gather collective, csrc/comm.cpp).  B = 1024 over 1/2/4/8 ranks: equal slices."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('invalid rank %d of %d' % (rank, world))
    if B < world:
        raise ValueError('batch %d < %d ranks: a rank would hold no problem' % (B, world))
    return rank * B // world, (rank + 1) * B // world


def world_from_env():
    """(rank, world, local_rank, master_addr, master_port) of this process (launcher variables)."""
    return (int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)),
            int(os.environ.get('LOCAL_RANK', os.environ.get('RANK', 0))),
            os.environ.get('MASTER_ADDR', '127.0.0.1'), int(os.environ.get('MASTER_PORT', 29500)))


def _recv_exact(sock, n):
    buf = b''
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError('rendezvous peer closed the connection')
        buf += chunk
    return buf


def exchange_id(rank, world, make_id, addr='127.0.0.1', port=29500, timeout=120.0):
    """Rank 0 calls ``make_id()`` (ID_BYTES bytes) and serves it to the world - 1 other ranks over
    TCP at (addr, port + 1); they connect (retrying until ``timeout``) and read it.  Returns the id
    on every rank."""
    if world == 1:
        return make_id()
    if rank == 0:
        uid = make_id()
        if len(uid) != ID_BYTES:
            raise ValueError('unique id must be %d bytes' % ID_BYTES)
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((addr, port + 1))
        srv.listen(world)
        srv.settimeout(timeout)
        try:
            for _ in range(world - 1):
                conn, _ = srv.accept()
                with conn:
                    conn.sendall(uid)
                    _recv_exact(conn, 1)   # the peer's acknowledgement
        finally:
            srv.close()
        return uid
    deadline = time.monotonic() + timeout
    while True:
        try:
            with socket.create_connection((addr, port + 1), timeout=5.0) as c:
                uid = _recv_exact(c, ID_BYTES)
                c.sendall(b'k')
                return uid
        except (ConnectionRefusedError, ConnectionResetError, socket.timeout, OSError):
            if time.monotonic() > deadline:
                raise TimeoutError('rank %d: no RCCL id from rank 0 at %s:%d' % (rank, addr, port + 1))
            time.sleep(0.05)


def free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_local(nproc, argv, port=None, env=None, timeout=None):
    """Run ``python argv...`` as nproc processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT set (one per GPU).  Returns 0 when every process exits with 0, else the first
    nonzero exit code (the other processes are then terminated).  The caller must not have
    touched the GPU (it only starts children)."""
    port = port or free_port()
    procs = []
    for r in range(nproc):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


class RcclComm:
    """RCCL communicator bound to one ``Solver`` handle (libcmpc ``cmpc_comm_*``)."""

    def __init__(self, solver, rank, world, addr='127.0.0.1', port=29500):
        self.s = solver
        self.lib = solver.lib
        self.rank, self.world = rank, world

        def make_id():
            buf = (ctypes.c_uint8 * ID_BYTES)()
            rc = self.lib.cmpc_comm_get_unique_id(buf)
            if rc != 0:
                raise RuntimeError('cmpc_comm_get_unique_id failed (rc=%d)' % rc)
            return bytes(buf)

        uid = exchange_id(rank, world, make_id, addr, port)
        arr = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        solver._chk(self.lib.cmpc_comm_init(solver.h, world, rank, arr), 'cmpc_comm_init')

    def bcast_params(self, params=None, capacity=8):
        """Rank 0 passes its ModelParams list; every rank installs rank 0's classes."""
        from cmpc._lib import Params, params_struct
        n = len(params) if params is not None else capacity
        arr = (Params * n)(*([params_struct(p, self.s.nc) for p in params] if params is not None else []))
        self.s._chk(self.lib.cmpc_comm_bcast_params(self.s.h, 0, n, arr), 'cmpc_comm_bcast_params')

    def allreduce_max(self, values):
        v = np.ascontiguousarray(values, float).copy()
        self.s._chk(self.lib.cmpc_comm_allreduce_max(self.s.h, v.ctypes.data_as(ctypes.c_void_p), v.size),
                    'cmpc_comm_allreduce_max')
        return v

    def barrier(self):
        self.s.synchronize()
        self.allreduce_max([0.0])

    def gather_solution(self, root=0):
        """Every rank's accepted X (B_r, N+1, 9), U (B_r, N, 12) and statuses on root, concatenated
        in rank order (= the global order of contiguous slices, of any sizes); None elsewhere."""
        B, N, G = self.s.B, self.s.N, self.world
        is_root = self.rank == root
        sizes = np.zeros(G)
        sizes[self.rank] = B
        tot = int(self.allreduce_max(sizes).sum()) if is_root else 0   # slices may differ in size
        if not is_root:
            self.allreduce_max(sizes)
        X = np.zeros((tot, N + 1, 9)); U = np.zeros((tot, N, 12))
        st = np.zeros(tot, np.int32); it = np.zeros(tot, np.int32); qs = np.zeros(tot, np.int32)
        ptr = (lambda a: a.ctypes.data_as(ctypes.c_void_p)) if is_root else (lambda a: None)
        self.s._chk(self.lib.cmpc_comm_gather_solution(self.s.h, root, ptr(X), ptr(U), ptr(st), ptr(it), ptr(qs)),
                    'cmpc_comm_gather_solution')
        if not is_root:
            return None
        return dict(X=X, U=U, status=st, iterations=it, qp_status=qs)

    def close(self):
        if self.s.h is not None:
            self.lib.cmpc_comm_destroy(self.s.h)
