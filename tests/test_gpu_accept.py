"""GPU: the trust-region norm of the accept step (reference src/scp_solver.py:153,
np.linalg.norm(X_sol - X_prev, 2), the spectral norm, quirk Q6) against numpy's SVD on the
device's own QP solution, for every problem of a batch: the device computes the largest
eigenvalue of the 9 x 9 Gram matrix by multisection (scp.hip lambda_max_psd), bound 1e-12
relative."""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('robot,N,B', [('trot', 30, 64), ('bound', 20, 32), ('talos', 20, 16)])
def test_trust_region_norm_is_numpy_spectral_norm(robot, N, B):
    pb = make_batch(robot, N, B)
    s = Solver(pb.robot, N, B, 'fp64')
    s.upload(pb)
    s.scp_iterate(fixed_iters=True)
    z, _, st, _ = s.qp_solution(with_y=False)
    tr = s.iteration_log()['tr_norm']
    s.close()
    K1 = N + 1
    for b in range(B):
        X = z[b][:9 * K1].reshape(K1, 9)
        ref = np.linalg.norm((X - pb.Xbar[b]).T, 2)
        assert abs(tr[b] - ref) <= 1e-12 * max(ref, 1e-300), (b, tr[b], ref)
