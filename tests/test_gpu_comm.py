"""GPU: the RCCL batch-split entry points (cmpc_comm_*) on one rank: the parameter broadcast
installs rank 0's classes, the max-reduction is the identity, and the gather returns the same
accepted solutions and statuses as the handle's own getters.  (Several ranks need several GPUs;
the driver's 8-GPU bench runs them, and tests/test_shard.py covers the multi-process plumbing.)"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.shard import RcclComm, free_port
from cmpc.synth import make_batch

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_roundtrip():
    pb = make_batch('trot', 30, 6)
    s = Solver(pb.robot, 30, 6, 'fp64')
    comm = RcclComm(s, 0, 1, '127.0.0.1', free_port())
    comm.bcast_params(pb.params)
    s.upload(pb, set_params=False)
    s.solve_scp(fixed_iters=False)
    v = comm.allreduce_max([1.5, -2.0, 3.0])
    assert list(v) == [1.5, -2.0, 3.0]
    g = comm.gather_solution(0)
    sol = s.solution()
    log = s.iteration_log()
    assert np.array_equal(g['X'], sol['X']) and np.array_equal(g['U'], sol['U'])
    assert np.array_equal(g['status'], sol['status']) and np.array_equal(g['iterations'], sol['iterations'])
    assert np.array_equal(g['qp_status'], log['qp_status'])
    comm.close()
    s.close()


def test_rccl_params_broadcast_matches_direct_upload():
    pb = make_batch('bound', 20, 3)
    outs = []
    for via_comm in (False, True):
        s = Solver(pb.robot, 20, 3, 'fp64')
        if via_comm:
            comm = RcclComm(s, 0, 1, '127.0.0.1', free_port())
            comm.bcast_params(pb.params)
            s.upload(pb, set_params=False)
        else:
            s.upload(pb)
        s.scp_iterate(fixed_iters=True)
        outs.append(s.qp_solution(with_y=False)[0])
        if via_comm:
            comm.close()
        s.close()
    assert np.array_equal(outs[0], outs[1])
