"""CPU: the oracle's GuSTO-mode restatement.  With gusto=False it is the
reference loop (quirk Q1: one accepted iteration at most, convergence identically 0); with
gusto=True accepted solutions become linearization points and the loop runs until the
convergence measure (src/scp_solver.py:51-56) drops below the threshold."""
import numpy as np

from cmpc.synth import make_batch
from oracle import scp as OS
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp


def test_oracle_gusto_iterates_to_convergence():
    pb = make_batch('trot', 12, 1)
    p = pb.oracle_problem(0)
    sp = dict(p['scp_params'])
    log_ref, log_g = [], []
    ref = OS.solve_scp(p, sp, qp=sparse_ipm_qp, log=log_ref)
    g = OS.solve_scp(p, sp, qp=sparse_ipm_qp, log=log_g, gusto=True)
    assert len(ref['state']) <= 1 and all('conv' not in r for r in log_ref)
    # the first iteration is the same problem in both modes
    assert log_ref[0]['decision'] == log_g[0]['decision']
    np.testing.assert_array_equal(ref['state'][0], g['state'][0])
    convs = [r['conv'] for r in log_g if 'conv' in r]
    assert len(g['state']) == len(convs) >= 2
    if len(log_g) < sp['max_iterations']:
        assert convs[-1] < sp['convergence_threshold'] and log_g[-1]['decision'] == 'accept'
    # successive accepted solutions: linearizing at the previous one moves them less and less
    assert convs[-1] < convs[0]
