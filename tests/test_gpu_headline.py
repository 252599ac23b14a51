"""GPU: the kernel that produces the headline number, checked against the oracle at the headline size.

BASELINE.json's metric runs Solo12 trot, N=100, 1024 problems per GPU.  There the library splits the QP
into two launches (cmpc_api.cpp qp_split): the head, k_qp_ipm<.., 64, 1>, one problem per wave (all 1024
at once, one per SIMD), from which the problems still running after the yield iteration k_qp_split
picked from the previous launch's Newton counts leave; and the tail, k_qp_ipm<.., 256, 2>, which
resumes those on four waves each (one per CU).  Solution polishing (the counterpart of the reference's
OSQP polish=True, qp_ipm.hip phase_polish_prep) is on.  The bench times steps after warm-up launches;
these tests reproduce that: two fixed-K SCP iterations, then a third QP launch on the same batch with
the same settings, whose QPs are compared with the oracle's independent sparse interior-point solver
(oracle/sparse_ipm.py) on:
  * the 8 problems with the most Newton steps, all of them finished by the tail launch (qp_tail > 0);
  * 8 seeded random problems.
Per problem: KKT residuals of the reference-form QP (the CSC the reference hands OSQP,
src/scp_solver.py:59-68) -- primal <= 1e-8, dual <= 1e-6 x the cost scale, multiplier signs exact --
and |X_gpu - X_oracle|_inf <= 1e-5 |X|_inf, the parity bar of tests/test_gpu_parity.py (the oracle
polishes its interior-point solution on the identified active set, oracle/sparse_ipm.py _polish).
The trot QPs are nearly flat along some contact-force directions (curvature 1 against objectives of
~5e6): two feasible points whose objectives agree to 1e-14 can differ by 2e-5 in a force.  Where the
two solutions differ by more than 1e-5, the GPU's must be feasible to 1e-8 and its objective no
higher than the oracle's by more than 1e-12 of it (problem 170 of the metric batch: the GPU's point is
the lower one).
The same on the 2-GPU shard of the metric (512 problems: a two-wave head k_qp_ipm<2> + the tail) and the
4-GPU shard (256 problems: k_qp_ipm<4>, four chains).
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle.kkt import kkt_residuals
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp

pytestmark = pytest.mark.gpu

N = 100


def _sorted_launch(B, seed_offset):
    pb = make_batch('trot', N, B, seed_offset=seed_offset)
    s = Solver(pb.robot, N, B, 'fp64')
    s.upload(pb)
    kernel = s.qp_kernel()
    s.scp_iterate(fixed_iters=True)
    s.scp_iterate(fixed_iters=True)
    # the third launch phase by phase, so the exported QP is exactly the one solved (scp_iterate's
    # accept step would move the trust region after it)
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution(with_y=True)
    return s, kernel, z, y, st, it


def _check(s, z, y, b):
    P, q, A, l, u = s.export_qp(b)
    k = kkt_residuals(P, q, A, l, u, z[b], y[b])
    scale = max(1.0, np.abs(P @ z[b]).max(), np.abs(q).max())
    assert k['prim'] <= 1e-8, (b, k['prim'])
    assert k['dual'] <= 1e-6 * scale, (b, k['dual'], scale)
    assert k['sign'] == 0.0, b
    ref = sparse_ipm_qp(P, q, A, l, u)
    assert ref.info.status == 'solved'
    nxu = 9 * (N + 1) + 12 * N
    err = np.abs(z[b][:nxu] - ref.x[:nxu]).max() / np.abs(ref.x[:nxu]).max()
    if err > 1e-5:   # flat directions: the GPU's point must be feasible and at least as good
        zb = z[b]
        f_gpu = 0.5 * zb @ (P @ zb) + q @ zb
        f_ref = 0.5 * ref.x @ (P @ ref.x) + q @ ref.x
        Az = A @ zb
        viol = max(float(np.maximum(Az - u, l - Az).max()), 0.0)
        assert viol <= 1e-8 and f_gpu <= f_ref + 1e-12 * abs(f_ref), (b, err, viol, f_gpu - f_ref)


def _sample(it, n_slow=8, n_rand=8, seed=0):
    slow = [int(b) for b in np.argsort(-it, kind='stable')[:n_slow]]
    rng = np.random.default_rng(seed)
    rest = np.setdiff1d(np.arange(len(it)), slow)
    return slow, [int(b) for b in rng.choice(rest, n_rand, replace=False)]


def test_metric_config_kernel_matches_oracle():
    B = 1024
    s, kernel, z, y, st, it = _sorted_launch(B, seed_offset=0)
    merit, _ = s.qp_info()
    tail, pol = s.qp_exit()
    try:
        assert kernel == 'k_qp_ipm<1>+tail<4>', kernel
        assert np.all(st == 1), np.unique(st, return_counts=True)
        assert np.all(merit <= 1.0)
        assert (pol > 0).sum() > 0, 'no problem was polished'
        slow, rand = _sample(it)
        # the slowest problems are the ones the tail launch finishes on four waves
        assert all(tail[b] > 0 for b in slow), [(b, int(it[b]), int(tail[b])) for b in slow]
        assert 0 < (tail > 0).sum() <= 256, (tail > 0).sum()
        for b in slow + rand:
            _check(s, z, y, b)
    finally:
        s.close()


@pytest.mark.parametrize('B,kernel', [(512, 'k_qp_ipm<2>+tail<4>'), (256, 'k_qp_ipm<4>')])
def test_metric_shards_match_oracle(B, kernel):
    """The 2- and 4-GPU slices of the metric's 1024 problems (cmpc/shard.py: contiguous slices)."""
    s, k, z, y, st, it = _sorted_launch(B, seed_offset=0)
    try:
        assert k == kernel, k
        assert np.all(st == 1), np.unique(st, return_counts=True)
        slow, rand = _sample(it, n_slow=4, n_rand=4, seed=1)
        for b in slow + rand:
            _check(s, z, y, b)
    finally:
        s.close()


def test_metric_config_first_launch_of_a_fresh_batch():
    """A never-solved batch (the reference's use: every solve_scp call is a new problem,
    src/scp_solver.py:118-179): its first grouped launch has no Newton counts to sort by.  All
    problems solved, and a handle that solved another batch before gives bit-identical results (no
    ordering key leaks from the previous upload)."""
    B = 1024
    pa = make_batch('trot', N, B, seed_offset=0)
    pb = make_batch('trot', N, B, seed_offset=5000)
    s = Solver(pa.robot, N, B, 'fp64')
    s.upload(pa)
    s.scp_iterate(fixed_iters=True)
    s.scp_iterate(fixed_iters=True)
    s.upload(pb)
    s.scp_iterate(fixed_iters=True)
    z1, _, st1, it1 = s.qp_solution(with_y=False)
    s.close()
    s2 = Solver(pb.robot, N, B, 'fp64')
    s2.upload(pb)
    s2.scp_iterate(fixed_iters=True)
    z2, _, st2, it2 = s2.qp_solution(with_y=False)
    s2.close()
    assert np.all(st1 == 1)
    np.testing.assert_array_equal(it1, it2)
    np.testing.assert_array_equal(z1, z2)
