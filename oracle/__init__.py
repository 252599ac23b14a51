"""CPU oracle for the batched SCP centroidal-MPC hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``centroidal-mpc_amd/``) imports
this package; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it, and only as the checker / the timed CPU baseline.

The oracle is a clean-room numpy/scipy restatement of the reference's SCP path
(ahmadgazar/centroidal-MPC, read-only at /root/reference):

* ``model``          centroidal dynamics, closed-form Jacobians, LQR, covariance scan,
                     rollout and model-accuracy ratio
                     (src/centroidal_model.py:189-291, src/scp_solver.py:71-87)
* ``transcription``  QP cost and constraint matrices in the reference's exact row order
                     (src/cost.py, src/constraints.py, src/scp_solver.py:10-48)
* ``osqp_admm``      restatement of OSQP's published ADMM algorithm with Ruiz scaling,
                     adaptive rho and solution polishing (the third-party solver the
                     reference calls at src/scp_solver.py:59-68; osqp-python, version
                     unpinned by the reference's setup.py)
* ``kkt``            solver-independent KKT residual checker
* ``scp``            the SCP trust-region state machine (src/scp_solver.py:118-179)

Parity pinning: the model/transcription/state-machine restatement is pinned against
golden vectors generated from the reference's own code (tests/golden/make_golden.py).
The QP solver itself is pinned only by the KKT checker, since OSQP is not installed
here ("Oracle").
"""
