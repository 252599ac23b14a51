"""GPU: split QP launches (cmpc_api.cpp qp_split; qp_ipm.hip k_qp_ipm MODE 1 / 2) solve the same
problems to the same answers as one launch of one wave per problem.

Batches of one wave per problem that fill the device (more problems than CUs) last as long as their
slowest problems.  The head launch runs every problem on one wave; a problem still running after the
stopping test of the yield iteration K (k_qp_split: the smallest K with at most one problem per CU
above it in the previous launch's Newton counts; on a batch's first launch the robot's prior, 6 on
Solo12) leaves its state
in the workspace, and the tail launch resumes it on four waves (two below N = 40), where the Schur
recurrence runs as four chains (a different elimination order) or two ends.  So: statuses and SCP
decisions agree, Newton counts within one, solutions to 1e-7 relative (TALOS: counts within 2,
solutions within the oracle parity bar 1e-5), with one- and two-wave heads, on the fixed-K path and the early-exit path (solve_scp,
only active problems); and two runs are bit-identical (the yield point depends on Newton counts only).
"""
import os

import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch

pytestmark = pytest.mark.gpu


class _split:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.old = os.environ.get('CMPC_QP_SPLIT')
        os.environ['CMPC_QP_SPLIT'] = '1' if self.on else '0'

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop('CMPC_QP_SPLIT', None)
        else:
            os.environ['CMPC_QP_SPLIT'] = self.old


def _run(pb, on, steps=3, waves=1):
    with _split(on):
        s = Solver(pb.robot, pb.N, pb.B, 'fp64')
        # (the same polishing tolerance either way: its default depends on whether the launch splits)
        s.set_qp_settings(waves_per_problem=waves, polish_eps=0.0 if str(pb.robot).lower() == 'talos' else 1e-7)
        s.upload(pb)
        kernel = s.qp_kernel()
        out = []
        for _ in range(steps):
            s.scp_iterate(fixed_iters=True)
            z, _, st, it = s.qp_solution(with_y=False)
            out.append((z.copy(), st.copy(), it.copy(), s.iteration_log()['decision'].copy(), s.qp_exit()[0].copy()))
        s.close()
    return kernel, out


CASES = [('trot', 100, 320, 1), ('trot', 30, 300, 1), ('pace', 60, 300, 1), ('bound', 60, 300, 1), ('talos', 40, 300, 1),
         ('trot', 100, 320, 2), ('talos', 80, 300, 2)]   # (two-wave heads: BASELINE C4's shape)


@pytest.mark.parametrize('cfg,N,B,waves', CASES)
def test_split_launches_match_one_launch(cfg, N, B, waves):
    pb = make_batch(cfg, N, B, seed_offset=71)
    k1, one = _run(pb, False, waves=waves)
    k2, spl = _run(pb, True, waves=waves)
    assert k1 == 'k_qp_ipm<%d>' % waves, k1
    assert k2 == 'k_qp_ipm<%d>+tail<%d>' % (waves, 4 if N >= 40 else 2), k2
    talos = cfg == 'talos'
    tails = 0
    for (z1, s1, i1, d1, t1), (z2, s2, i2, d2, t2) in zip(one, spl):
        assert np.all(s1 == 1) and np.all(s2 == 1), (s1, s2)
        assert np.abs(i1 - i2).max() <= (2 if talos else 1), (i1, i2)
        np.testing.assert_array_equal(d1, d2)
        err = np.abs(z1 - z2).max(axis=1) / np.abs(z1).max(axis=1)
        assert err.max() <= (1e-5 if talos else 1e-7), err.max()
        assert np.all(t1 == 0)
        tails += int((t2 > 0).sum())
    # a tail exists once the counts differ (bound: every problem takes the same number of steps)
    spread = any(o[2].max() > o[2].min() for o in one[:-1])
    assert (tails > 0) == spread, (tails, [np.unique(o[2]) for o in one])


def test_split_launches_are_reproducible():
    pb = make_batch('trot', 100, 320, seed_offset=73)
    _, a = _run(pb, True)
    _, b = _run(pb, True)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(u, v)


@pytest.mark.parametrize('cfg,N,B', [('trot', 50, 300), ('talos', 40, 300)])
def test_split_early_exit_path(cfg, N, B):
    """solve_scp: later QP launches hold inactive problems (k_qp_split counts them as zero steps);
    accepted outputs and SCP records agree with one launch."""
    pb = make_batch(cfg, N, B, seed_offset=79)
    res = {}
    for on in (False, True):
        with _split(on):
            s = Solver(pb.robot, N, B, 'fp64')
            s.set_qp_settings(waves_per_problem=1, polish_eps=0.0 if str(pb.robot).lower() == 'talos' else 1e-7)
            s.upload(pb)
            s.solve_scp(fixed_iters=False)
            res[on] = (s.solution(with_ks=False), s.iteration_history())
            s.close()
    (a, ha), (b, hb) = res[False], res[True]
    for k in ('n_accepted', 'iterations', 'status'):
        np.testing.assert_array_equal(a[k], b[k])
    tol = 1e-5 if cfg == 'talos' else 1e-7
    for k in ('X', 'U'):
        err = np.abs(a[k] - b[k]).max() / np.abs(a[k]).max()
        assert err <= tol, (k, err)
    np.testing.assert_array_equal(ha[1], hb[1])
    np.testing.assert_array_equal(ha[0]['decision'], hb[0]['decision'])


def test_split_on_a_fresh_batch_uses_the_prior():
    """A never-solved batch has no Newton counts: its first launch yields at the robot's prior
    (cmpc_api.cpp qp_split_prior, 6 on Solo12), so exactly the problems that need more than 6
    Newton-loop iterations finish in the tail; with the prior off (CMPC_QP_SPLIT_FRESH=0) the first
    launch is unsplit.  Both agree with one launch to 1e-7."""
    pb = make_batch('trot', 100, 320, seed_offset=83)
    _, one = _run(pb, False, steps=1)
    _, pri = _run(pb, True, steps=1)
    old = os.environ.get('CMPC_QP_SPLIT_FRESH')
    os.environ['CMPC_QP_SPLIT_FRESH'] = '0'
    try:
        _, off = _run(pb, True, steps=1)
    finally:
        if old is None:
            os.environ.pop('CMPC_QP_SPLIT_FRESH', None)
        else:
            os.environ['CMPC_QP_SPLIT_FRESH'] = old
    (z1, s1, i1, _, _), (z2, s2, i2, _, t2), (z3, s3, i3, _, t3) = one[0], pri[0], off[0]
    assert np.all(t3 == 0)
    np.testing.assert_array_equal(z1, z3)
    assert np.all(s2 == 1) and np.abs(i1 - i2).max() <= 1
    np.testing.assert_array_equal(t2 > 0, i2 > 6)
    assert (t2 > 0).sum() > 0
    err = np.abs(z1 - z2).max(axis=1) / np.abs(z1).max(axis=1)
    assert err.max() <= 1e-7, err.max()
