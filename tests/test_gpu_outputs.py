"""GPU: the host-output paths of cmpc_get_solution give identical arrays (the reference's
semantics end with the accepted X, U, K, Sigma on the host).

* the batched getter (device-side transposes / widening, one batch of async copies) into fresh
  pageable arrays, into page-locked arrays (cmpc_host_register), and with K / Sigma streamed
  during the solve (cmpc_prefetch_ks): bit-identical, fp64 and fp32;
* K and Sigma equal the linearization getter's (reference mode, quirk Q1) and NULL skips arrays;
* the prefetch is disarmed by a new upload: a second solve of other problems returns their own
  K / Sigma, not the first solve's.
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('cfg,prec', [('trot', 'fp64'), ('bound', 'fp32')])
def test_solution_paths_identical(cfg, prec):
    N, B = 40, 96
    pb = make_batch(cfg, N, B, seed_offset=17)
    with Solver(pb.robot, N, B, prec) as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=False)
        a = s.solution()
        lin = s.linearization()
        b = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in s.solution(pinned=True).items()}
        s.upload(pb)
        s.prefetch_ks()
        s.solve_scp(fixed_iters=False)
        c = s.solution(pinned=True)
        d = s.solution(with_ks=False)
    assert np.all(a['n_accepted'] >= 1)
    for k in ('X', 'U', 'K', 'Sigma', 'n_accepted', 'iterations', 'status'):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a[k], c[k], err_msg=k)
    np.testing.assert_array_equal(a['K'], lin['K'])
    np.testing.assert_array_equal(a['Sigma'], lin['Sigma'])
    np.testing.assert_array_equal(d['X'], a['X'])
    assert d['K'] is None and d['Sigma'] is None


def test_prefetch_is_per_upload():
    N, B = 30, 32
    p1 = make_batch('trot', N, B, seed_offset=1)
    p2 = make_batch('trot', N, B, seed_offset=500)
    with Solver(p1.robot, N, B, 'fp64') as s:
        s.upload(p1)
        s.prefetch_ks()
        s.solve_scp(fixed_iters=False)
        k1 = s.solution(pinned=True)['K'].copy()
        s.upload(p2)              # disarms: the next solve's K must be p2's
        s.solve_scp(fixed_iters=False)
        k2 = s.solution(pinned=True)['K'].copy()
        ref2 = s.solution()['K']
    np.testing.assert_array_equal(k2, ref2)
    assert not np.array_equal(k1, k2)
