"""CPU: the TALOS QP on which the GPU IPM stalls, dumped from the GPU by
``scripts/dump_qp.py talos 200 512 2 argmax`` into ``tests/golden/talos_stall_qp.npz``.

The oracle's sparse IPM solves it; the GPU's capped answer (status -2 after 60 iterations) is
primal feasible to 1e-10 and within 1e-4 of the oracle's states, so the stall is a convergence
failure near the optimum, not a wrong QP.  The GPU side is pinned by the strict-xfail
``test_talos_shrunk_trust_region_qp_solves``."""
import os

import numpy as np
from scipy import sparse

from oracle.kkt import kkt_residuals
from oracle.sparse_ipm import solve_qp

FIX = os.path.join(os.path.dirname(__file__), 'golden', 'talos_stall_qp.npz')


def test_oracle_solves_the_stalling_talos_qp():
    d = np.load(FIX)
    P = sparse.csc_matrix((d['P_data'], d['P_indices'], d['P_indptr']), shape=tuple(d['P_shape']))
    A = sparse.csc_matrix((d['A_data'], d['A_indices'], d['A_indptr']), shape=tuple(d['A_shape']))
    ref = solve_qp(P, d['q'], A, d['l'], d['u'])
    assert ref.info.status == 'solved'
    assert int(d['status']) == -2 and int(d['ipm_iters']) == 60
    k = kkt_residuals(P, d['q'], A, d['l'], d['u'], d['z'], d['y'])
    assert k['prim'] <= 1e-10
    nx = 9 * 201
    err = np.abs(d['z'][:nx] - ref.x[:nx]).max() / np.abs(ref.x[:nx]).max()
    assert err <= 1e-4, err
