"""ctypes binding of libcmpc.so (the C ABI in include/cmpc.h).

The shared library is built in-tree (``make -C centroidal-mpc_amd/csrc``, or
``__graft_entry__.build()``).  There is no CPU fallback: every entry point runs on the GPU and
a missing library or GPU raises ``CmpcError``.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_VARIANT = os.environ.get('CMPC_LIB_VARIANT')   # 'diag': the cycle-stamp build (libcmpc_diag.so)
LIB_PATH = os.path.join(_HERE, 'libcmpc_%s.so' % _VARIANT if _VARIANT else 'libcmpc.so')

ROBOTS = {'solo12': 0, 'TALOS': 1}
PREC = {'fp64': 0, 'float64': 0, 'f64': 0, 'fp32': 1, 'float32': 1, 'f32': 1}
QP_STATUS = {1: 'solved', 2: 'solved inaccurate', -2: 'maximum iterations reached', -3: 'primal infeasible',
             -4: 'dual infeasible', -10: 'non-finite'}
SCP_STATUS = {0: 'running', 1: 'converged', 2: 'max_iter', -1: 'qp_failed'}
DECISION = {0: 'none', 1: 'accept', 2: 'reject_rho', 3: 'reject_tr', -1: 'qp_failed'}


class CmpcError(RuntimeError):
    pass


class Params(ctypes.Structure):
    _fields_ = [('mass', ctypes.c_double), ('gravity', ctypes.c_double), ('dt', ctypes.c_double),
                ('mu', ctypes.c_double), ('beta_u', ctypes.c_double), ('foot_range', ctypes.c_double * 4),
                ('Wx', ctypes.c_double * 9), ('Wu', ctypes.c_double * 12), ('Q', ctypes.c_double * 81),
                ('R', ctypes.c_double * 144), ('cov_w', ctypes.c_double * 144), ('cov_eta', ctypes.c_double * 81),
                ('stochastic', ctypes.c_int32), ('tracking', ctypes.c_int32),
                ('tr_radius0', ctypes.c_double), ('omega0', ctypes.c_double), ('omega_max', ctypes.c_double),
                ('rho0', ctypes.c_double), ('rho1', ctypes.c_double), ('beta_succ', ctypes.c_double),
                ('beta_fail', ctypes.c_double), ('gamma_fail', ctypes.c_double),
                ('convergence_threshold', ctypes.c_double), ('max_iterations', ctypes.c_int32)]


class QPSettings(ctypes.Structure):
    _fields_ = [('max_iter', ctypes.c_int32), ('eps_abs', ctypes.c_double), ('eps_rel', ctypes.c_double),
                ('step_fraction', ctypes.c_double), ('init_floor_s', ctypes.c_double),
                ('init_floor_l', ctypes.c_double), ('waves_per_problem', ctypes.c_int32),
                ('polish_eps', ctypes.c_double)]


class Gait(ctypes.Structure):
    _fields_ = [('type', ctypes.c_int32), ('nb_steps', ctypes.c_int32), ('step_knots', ctypes.c_int32),
                ('support_knots', ctypes.c_int32), ('step_length', ctypes.c_double)]


GAIT_TYPES = {'TROT': 0, 'PACE': 1, 'BOUND': 2}


class Timing(ctypes.Structure):
    _fields_ = [('linearize_ms', ctypes.c_float), ('assemble_ms', ctypes.c_float), ('qp_ms', ctypes.c_float),
                ('accept_ms', ctypes.c_float), ('total_ms', ctypes.c_float)]


class IterRecord(ctypes.Structure):
    """include/cmpc.h cmpc_iter_record"""
    _fields_ = [('weight', ctypes.c_double), ('radius', ctypes.c_double), ('tr_norm', ctypes.c_double),
                ('rho', ctypes.c_double), ('iteration', ctypes.c_int32), ('qp_status', ctypes.c_int32),
                ('qp_iters', ctypes.c_int32), ('decision', ctypes.c_int32)]


ITER_RECORD_DTYPE = np.dtype([('weight', 'f8'), ('radius', 'f8'), ('tr_norm', 'f8'), ('rho', 'f8'),
                              ('iteration', 'i4'), ('qp_status', 'i4'), ('qp_iters', 'i4'), ('decision', 'i4')])
DECISIONS = {1: 'accept', 2: 'reject_rho', 3: 'reject_tr', -1: 'qp_failed'}

EXPORTS = ['cmpc_create', 'cmpc_destroy', 'cmpc_last_error', 'cmpc_version', 'cmpc_default_qp_settings',
           'cmpc_set_qp_settings', 'cmpc_set_params', 'cmpc_upload', 'cmpc_set_trust_region', 'cmpc_rollout',
           'cmpc_linearize', 'cmpc_assemble',
           'cmpc_qp_solve', 'cmpc_accept', 'cmpc_scp_iterate', 'cmpc_solve_scp', 'cmpc_synchronize',
           'cmpc_get_linearization', 'cmpc_qp_sizes', 'cmpc_export_qp', 'cmpc_get_qp_solution',
           'cmpc_get_solution', 'cmpc_get_iteration_log', 'cmpc_get_timing', 'cmpc_timing_begin',
           'cmpc_timing_end', 'cmpc_get_qp_iterations_total', 'cmpc_debug_stamps', 'cmpc_get_qp_kernel', 'cmpc_set_scp_mode',
           'cmpc_get_linearization_point', 'cmpc_interpolate', 'cmpc_generate_contact_plans',
           'cmpc_upload_states', 'cmpc_get_contact_plans', 'cmpc_get_warm_start', 'cmpc_get_qp_info', 'cmpc_get_qp_exit',
           'cmpc_comm_get_unique_id', 'cmpc_comm_init', 'cmpc_comm_destroy', 'cmpc_comm_bcast_params',
           'cmpc_comm_allreduce_max', 'cmpc_comm_gather_solution', 'cmpc_load_qp', 'cmpc_get_iteration_history',
           'cmpc_get_accepted', 'cmpc_host_register', 'cmpc_host_unregister',
           'cmpc_prefetch_ks']
SCP_MODE = {'reference': 0, 'gusto': 1}

_lib = None


def load():
    """Load libcmpc.so (raises CmpcError when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CmpcError('libcmpc.so not found at %s: build it with `make -C centroidal-mpc_amd/csrc` '
                        '(or __graft_entry__.build()); there is no CPU fallback' % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    h = ctypes.c_void_p
    i32 = ctypes.c_int
    sig = {
        'cmpc_create': (i32, [P(h), i32, i32, i32, i32, i32]),
        'cmpc_destroy': (i32, [h]),
        'cmpc_last_error': (ctypes.c_char_p, [h]),
        'cmpc_version': (i32, []),
        'cmpc_default_qp_settings': (i32, [i32, P(QPSettings)]),
        'cmpc_set_qp_settings': (i32, [h, P(QPSettings)]),
        'cmpc_set_params': (i32, [h, i32, P(Params)]),
        'cmpc_upload': (i32, [h, i32, vp, vp, vp, vp, vp, vp]),
        'cmpc_set_trust_region': (i32, [h, vp, vp]),
        'cmpc_rollout': (i32, [h, vp, vp, vp]),
        'cmpc_linearize': (i32, [h]),
        'cmpc_assemble': (i32, [h]),
        'cmpc_qp_solve': (i32, [h]),
        'cmpc_accept': (i32, [h, i32]),
        'cmpc_scp_iterate': (i32, [h, i32]),
        'cmpc_solve_scp': (i32, [h, i32, P(ctypes.c_int)]),
        'cmpc_synchronize': (i32, [h]),
        'cmpc_get_linearization': (i32, [h, vp, vp, vp, vp, vp, vp]),
        'cmpc_qp_sizes': (i32, [h, vp, vp, vp, vp]),
        'cmpc_export_qp': (i32, [h, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        'cmpc_get_qp_solution': (i32, [h, vp, vp, vp, vp]),
        'cmpc_get_solution': (i32, [h, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        'cmpc_get_iteration_log': (i32, [h, vp, vp, vp, vp, vp]),
        'cmpc_get_timing': (i32, [h, P(Timing)]),
        'cmpc_timing_begin': (i32, [h]),
        'cmpc_timing_end': (i32, [h, P(Timing), P(ctypes.c_int)]),
        'cmpc_get_qp_iterations_total': (i32, [h, P(ctypes.c_int64)]),
        'cmpc_debug_stamps': (i32, [h, vp]),
        'cmpc_get_qp_kernel': (i32, [h, ctypes.c_char_p, i32]),
        'cmpc_set_scp_mode': (i32, [h, i32]),
        'cmpc_get_linearization_point': (i32, [h, vp, vp, vp]),
        'cmpc_interpolate': (i32, [h, i32, vp, vp]),
        'cmpc_generate_contact_plans': (i32, [h, i32, vp, vp]),
        'cmpc_upload_states': (i32, [h, i32, vp, vp, vp]),
        'cmpc_get_contact_plans': (i32, [h, vp, vp, vp]),
        'cmpc_get_warm_start': (i32, [h, vp, vp]),
        'cmpc_get_qp_info': (i32, [h, vp, vp]),
        'cmpc_get_qp_exit': (i32, [h, vp, vp]),
        'cmpc_comm_get_unique_id': (i32, [vp]),
        'cmpc_comm_init': (i32, [h, i32, i32, vp]),
        'cmpc_comm_destroy': (i32, [h]),
        'cmpc_comm_bcast_params': (i32, [h, i32, i32, P(Params)]),
        'cmpc_comm_allreduce_max': (i32, [h, vp, i32]),
        'cmpc_comm_gather_solution': (i32, [h, i32, vp, vp, vp, vp, vp]),
        'cmpc_load_qp': (i32, [h, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        'cmpc_get_iteration_history': (i32, [h, i32, vp, vp]),
        'cmpc_get_accepted': (i32, [h, i32, vp, vp, vp, vp]),
        'cmpc_host_register': (i32, [h, vp, ctypes.c_size_t]),
        'cmpc_host_unregister': (i32, [h, vp]),
        'cmpc_prefetch_ks': (i32, [h, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None and _VARIANT:   # an older diagnostic build (same-box A/B): entries it lacks stay unset
            continue
        if fn is None:
            raise CmpcError('%s lacks %s: rebuild it' % (LIB_PATH, name))
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def params_struct(p, nc):
    """ModelParams -> Params (C struct)."""
    s = Params()
    s.mass, s.gravity, s.dt, s.mu, s.beta_u = p.mass, p.gravity, p.dt, p.mu, p.beta_u
    s.foot_range[:] = list(p.foot_range)
    s.Wx[:] = list(np.asarray(p.Wx, float))
    s.Wu[:] = list(np.asarray(p.Wu, float))
    s.Q[:] = list(np.asarray(p.Q, float).ravel())
    R = np.zeros((12, 12)); R[:p.R.shape[0], :p.R.shape[1]] = p.R
    s.R[:] = list(R.ravel())
    W = np.zeros((12, 12)); nw = 3 * nc; W[:nw, :nw] = np.asarray(p.cov_w, float)[:nw, :nw]
    s.cov_w[:] = list(W.ravel())
    s.cov_eta[:] = list(np.asarray(p.cov_eta, float).ravel())
    s.stochastic = int(bool(p.stochastic))
    s.tracking = int(bool(p.tracking))
    sp = p.scp_params
    s.tr_radius0 = float(sp.get('trust_region_radius0', 100.0))
    s.omega0 = float(sp.get('omega0', 100.0))
    s.omega_max = float(sp.get('omega_max', 1e10))
    s.rho0 = float(sp.get('rho0', 0.4))
    s.rho1 = float(sp.get('rho1', 1.5))
    s.beta_succ = float(sp.get('beta_succ', 2.0))
    s.beta_fail = float(sp.get('beta_fail', 0.5))
    s.gamma_fail = float(sp.get('gamma_fail', 5.0))
    s.convergence_threshold = float(sp.get('convergence_threshold', 1e-3))
    s.max_iterations = int(sp.get('max_iterations', 10))
    return s


class Solver:
    """One device handle: B problems of one robot / horizon, resident in HBM."""

    def __init__(self, robot, N, max_batch, precision='fp64', device=0):
        self.lib = load()
        self.robot = robot
        self.N = int(N)
        self.nc = 4 if robot == 'solo12' else 2
        self.nu = 12
        self.prec = PREC[precision]
        self.max_batch = int(max_batch)
        self.B = 0
        self._params = []
        self._epoch = 0   # counts C-ABI calls: a cached export is valid only while no call followed it
        h = ctypes.c_void_p()
        rc = self.lib.cmpc_create(ctypes.byref(h), int(device), ROBOTS[robot], self.N, self.max_batch, self.prec)
        if rc == -5:
            raise CmpcError('cmpc_create: TALOS handles need fp64 (its QPs do not converge in fp32)')
        if rc != 0 or not h.value:
            raise CmpcError('cmpc_create failed (rc=%d): no usable GPU / HIP runtime?' % rc)
        self.h = h

    def _chk(self, rc, what):
        self._epoch += 1
        if rc != 0:
            msg = self.lib.cmpc_last_error(self.h)
            raise CmpcError('%s failed (rc=%d): %s' % (what, rc, msg.decode() if msg else ''))

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            for a in (getattr(self, '_pinned', None) or {}).values():
                self.lib.cmpc_host_unregister(self.h, a.ctypes.data_as(ctypes.c_void_p))
            self._pinned = None
            self.lib.cmpc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- setup
    def set_qp_settings(self, max_iter=None, eps_abs=None, eps_rel=None, step_fraction=None, init_floor_s=None,
                        init_floor_l=None, waves_per_problem=None, polish_eps=None):
        s = QPSettings()
        self.lib.cmpc_default_qp_settings(self.prec, ctypes.byref(s))
        if max_iter is not None: s.max_iter = int(max_iter)
        if eps_abs is not None: s.eps_abs = float(eps_abs)
        if eps_rel is not None: s.eps_rel = float(eps_rel)
        if step_fraction is not None: s.step_fraction = float(step_fraction)
        if init_floor_s is not None: s.init_floor_s = float(init_floor_s)
        if init_floor_l is not None: s.init_floor_l = float(init_floor_l)
        if waves_per_problem is not None: s.waves_per_problem = int(waves_per_problem)
        if polish_eps is not None: s.polish_eps = float(polish_eps)
        self._chk(self.lib.cmpc_set_qp_settings(self.h, ctypes.byref(s)), 'cmpc_set_qp_settings')

    def set_params(self, params):
        self._params = list(params)
        arr = (Params * len(params))(*[params_struct(p, self.nc) for p in params])
        self._chk(self.lib.cmpc_set_params(self.h, len(params), arr), 'cmpc_set_params')

    def upload(self, pb, set_params=True):
        """ProblemBatch -> device (resets the SCP state of every problem).  ``set_params=False``
        keeps the installed parameter classes (e.g. broadcast from rank 0 by RCCL)."""
        if pb.robot != self.robot or pb.N != self.N:
            raise CmpcError('batch robot/N (%s, %d) does not match the handle (%s, %d)'
                            % (pb.robot, pb.N, self.robot, self.N))
        if set_params:
            self.set_params(pb.params)
        self._keep = [np.ascontiguousarray(pb.class_id, np.int32), np.ascontiguousarray(pb.logic, np.int8),
                      np.ascontiguousarray(pb.pos, float), np.ascontiguousarray(pb.rot, float),
                      np.ascontiguousarray(pb.Xbar, float), np.ascontiguousarray(pb.Ubar, float)]
        self._chk(self.lib.cmpc_upload(self.h, pb.B, *[_ptr(a) for a in self._keep]), 'cmpc_upload')
        self.B = pb.B

    def generate_contact_plans(self, gaits, foot0):
        """Contact plans of len(gaits) problems built on the device (cmpc_generate_contact_plans).
        gaits: conf-style dicts (type, nbSteps, stepKnots, supportKnots, stepLength); foot0 (B, nc, 3)
        in the contact order FR, FL, HR, HL (solo12) / FR, FL (TALOS)."""
        B = len(gaits)
        g = (Gait * B)()
        for i, gd in enumerate(gaits):
            g[i].type = GAIT_TYPES[gd['type']]
            g[i].nb_steps, g[i].step_knots = int(gd['nbSteps']), int(gd['stepKnots'])
            g[i].support_knots, g[i].step_length = int(gd['supportKnots']), float(gd['stepLength'])
        f0 = np.ascontiguousarray(foot0, float)
        if f0.shape != (B, self.nc, 3):
            raise ValueError('foot0 must be (%d, %d, 3)' % (B, self.nc))
        self._chk(self.lib.cmpc_generate_contact_plans(self.h, B, g, _ptr(f0)), 'cmpc_generate_contact_plans')
        self.B = B

    def upload_states(self, params, class_id, Xbar, Ubar=None):
        """Warm starts for the device-planned problems; Ubar None -> the reference's warm-start
        controls built on the device."""
        self.set_params(params)
        self._keep = [np.ascontiguousarray(class_id, np.int32), np.ascontiguousarray(Xbar, float),
                      None if Ubar is None else np.ascontiguousarray(Ubar, float)]
        self._chk(self.lib.cmpc_upload_states(self.h, self.B, *[_ptr(a) for a in self._keep]), 'cmpc_upload_states')

    def contact_plans(self):
        B, N, nc = self.B, self.N, self.nc
        lg = np.zeros((B, N, nc), np.int8); pos = np.zeros((B, N, nc, 3)); rot = np.zeros((B, N, nc, 3, 3))
        self._chk(self.lib.cmpc_get_contact_plans(self.h, _ptr(lg), _ptr(pos), _ptr(rot)), 'cmpc_get_contact_plans')
        return lg, pos, rot

    def warm_start(self):
        X = np.zeros((self.B, self.N + 1, 9)); U = np.zeros((self.B, self.N, self.nu))
        self._chk(self.lib.cmpc_get_warm_start(self.h, _ptr(X), _ptr(U)), 'cmpc_get_warm_start')
        return X, U

    # ---- phases
    def set_trust_region(self, weight=None, radius=None):
        """Per-problem trust-region weight / radius (scalars broadcast to the batch)."""
        def arr(v):
            return None if v is None else np.ascontiguousarray(np.broadcast_to(np.asarray(v, float), (self.B,)))
        w, r = arr(weight), arr(radius)
        self._chk(self.lib.cmpc_set_trust_region(self.h, _ptr(w), _ptr(r)), 'cmpc_set_trust_region')

    def rollout(self, X, U):
        """Nonlinear rollout along X (B, N+1, 9), U (B, N, nu) -> (B, N+1, 9) on the device."""
        X = np.ascontiguousarray(X, dtype=float)
        U = np.ascontiguousarray(U, dtype=float)
        if X.shape != (self.B, self.N + 1, 9) or U.shape != (self.B, self.N, self.nu):
            raise ValueError('rollout expects X %s and U %s' % ((self.B, self.N + 1, 9), (self.B, self.N, self.nu)))
        out = np.zeros_like(X)
        self._chk(self.lib.cmpc_rollout(self.h, _ptr(X), _ptr(U), _ptr(out)), 'cmpc_rollout')
        return out

    def linearize(self): self._chk(self.lib.cmpc_linearize(self.h), 'cmpc_linearize')
    def assemble(self): self._chk(self.lib.cmpc_assemble(self.h), 'cmpc_assemble')
    def qp_solve(self): self._chk(self.lib.cmpc_qp_solve(self.h), 'cmpc_qp_solve')
    def accept(self, fixed_iters=False): self._chk(self.lib.cmpc_accept(self.h, int(fixed_iters)), 'cmpc_accept')

    def scp_iterate(self, fixed_iters=True):
        self._chk(self.lib.cmpc_scp_iterate(self.h, int(fixed_iters)), 'cmpc_scp_iterate')

    def solve_scp(self, fixed_iters=False):
        n = ctypes.c_int(0)
        self._chk(self.lib.cmpc_solve_scp(self.h, int(fixed_iters), ctypes.byref(n)), 'cmpc_solve_scp')
        return n.value

    def synchronize(self):
        self._chk(self.lib.cmpc_synchronize(self.h), 'cmpc_synchronize')

    def set_scp_mode(self, mode):
        """'reference' (default: quirk Q1, the linearization point stays at the warm start) or
        'gusto' (accepted solutions become the next linearization point; include/cmpc.h)."""
        self._chk(self.lib.cmpc_set_scp_mode(self.h, SCP_MODE[mode]), 'cmpc_set_scp_mode')

    def linearization_point(self):
        X = np.zeros((self.B, self.N + 1, 9)); U = np.zeros((self.B, self.N, 12)); conv = np.zeros(self.B)
        self._chk(self.lib.cmpc_get_linearization_point(self.h, _ptr(X), _ptr(U), _ptr(conv)),
                  'cmpc_get_linearization_point')
        return X, U, conv

    def interpolate(self, n_inner=10):
        """Device interpolate_SCP_solution of every problem's accepted solution:
        X (B, 9, N*n_inner), U (B, 12, (N-1)*n_inner)."""
        X = np.zeros((self.B, 9, self.N * n_inner)); U = np.zeros((self.B, 12, (self.N - 1) * n_inner))
        self._chk(self.lib.cmpc_interpolate(self.h, int(n_inner), _ptr(X), _ptr(U)), 'cmpc_interpolate')
        return X, U

    # ---- getters
    def linearization(self):
        B, N, nc = self.B, self.N, self.nc
        out = dict(f=np.zeros((B, N, 9)), A=np.zeros((B, N, 9, 9)), Bu=np.zeros((B, N, 9, 12)),
                   C=np.zeros((B, N, 9, 3 * nc)), K=np.zeros((B, N, 12, 9)), Sigma=np.zeros((B, N + 1, 9, 9)))
        self._chk(self.lib.cmpc_get_linearization(self.h, *[_ptr(out[k]) for k in ('f', 'A', 'Bu', 'C', 'K', 'Sigma')]),
                  'cmpc_get_linearization')
        return out

    def qp_sizes(self):
        v = [np.zeros(1, np.int32) for _ in range(4)]
        self._chk(self.lib.cmpc_qp_sizes(self.h, *[_ptr(a) for a in v]), 'cmpc_qp_sizes')
        return tuple(int(a[0]) for a in v)

    def load_qp(self, b, P, q, A, l, u):
        """Problem b's QP from the reference's CSC layout (scipy sparse P, A; q, l, u) into the
        device's structured form (cmpc_load_qp); raises CmpcError naming the offending row when the
        QP lacks the stage structure."""
        from scipy import sparse
        P = sparse.csc_matrix(P); A = sparse.csc_matrix(A)
        n, m = A.shape[1], A.shape[0]
        if P.shape != (n, n):
            raise CmpcError('P is %s, A has %d columns' % (P.shape, n))
        big = 1e30
        arrs = [np.ascontiguousarray(P.data, float), np.ascontiguousarray(P.indices, np.int32),
                np.ascontiguousarray(P.indptr, np.int32), np.ascontiguousarray(q, float).ravel(),
                np.ascontiguousarray(A.data, float), np.ascontiguousarray(A.indices, np.int32),
                np.ascontiguousarray(A.indptr, np.int32),
                np.ascontiguousarray(np.clip(np.asarray(l, float).ravel(), -big, big)),
                np.ascontiguousarray(np.clip(np.asarray(u, float).ravel(), -big, big))]
        if arrs[3].size != n or arrs[7].size != m or arrs[8].size != m:
            raise CmpcError('q, l, u sizes do not match P, A')
        self._chk(self.lib.cmpc_load_qp(self.h, int(b), n, m, *[_ptr(a) for a in arrs]), 'cmpc_load_qp')

    def export_qp(self, b):
        """(P, q, A, l, u) of problem b as scipy CSC, in the reference's row order."""
        from scipy import sparse
        n, m, nnzP, nnzA = self.qp_sizes()
        Px = np.zeros(nnzP); Pi = np.zeros(nnzP, np.int32); Pp = np.zeros(n + 1, np.int32)
        q = np.zeros(n)
        Ax = np.zeros(nnzA); Ai = np.zeros(nnzA, np.int32); Ap = np.zeros(n + 1, np.int32)
        l = np.zeros(m); u = np.zeros(m)
        self._chk(self.lib.cmpc_export_qp(self.h, int(b), *[_ptr(a) for a in (Px, Pi, Pp, q, Ax, Ai, Ap, l, u)]),
                  'cmpc_export_qp')
        P = sparse.csc_matrix((Px[:Pp[-1]], Pi[:Pp[-1]], Pp), shape=(n, n))
        A = sparse.csc_matrix((Ax[:Ap[-1]], Ai[:Ap[-1]], Ap), shape=(m, n))
        return P, q, A, l, u

    def qp_solution(self, with_y=True):
        n, m, _, _ = self.qp_sizes()
        z = np.zeros((self.B, n)); y = np.zeros((self.B, m)) if with_y else None
        st = np.zeros(self.B, np.int32); it = np.zeros(self.B, np.int32)
        self._chk(self.lib.cmpc_get_qp_solution(self.h, _ptr(z), _ptr(y), _ptr(st), _ptr(it)), 'cmpc_get_qp_solution')
        return z, y, st, it

    def qp_info(self):
        """Per-problem exit data of the last QP solve: final merit (<= 1 when solved) and the number of
        iterative-refinement steps taken."""
        merit = np.zeros(self.B); nref = np.zeros(self.B, np.int32)
        self._chk(self.lib.cmpc_get_qp_info(self.h, _ptr(merit), _ptr(nref)), 'cmpc_get_qp_info')
        return merit, nref

    def qp_exit(self):
        """Per problem: (tail, polish) of the last QP -- the Newton steps that ran on the whole grouped
        workgroup after the hand-over (0: solved on its own wave only), and the solution polishing
        (1 accepted, -1 rejected, 0 not tried)."""
        tail = np.zeros(self.B, np.int32); pol = np.zeros(self.B, np.int32)
        if _VARIANT and not hasattr(self.lib, 'cmpc_get_qp_exit'):   # an older diagnostic build
            return tail, pol
        self._chk(self.lib.cmpc_get_qp_exit(self.h, _ptr(tail), _ptr(pol)), 'cmpc_get_qp_exit')
        return tail, pol

    def qp_tail(self):
        return self.qp_exit()[0]

    def solution(self, pinned=False, with_ks=True):
        """Accepted X, U (and with_ks K, Sigma) plus the per-problem SCP state.  pinned=True writes
        into output arrays kept by this Solver and page-locked once (cmpc_host_register), so the
        copies run by DMA at full link rate and no fresh pages are faulted in per call; the arrays
        are then overwritten by the next pinned call (copy what must be kept)."""
        B, N = self.B, self.N
        shapes = dict(X=(B, N + 1, 9), U=(B, N, 12), K=(B, N, 12, 9), Sigma=(B, N + 1, 9, 9))
        if pinned:
            bufs = self._pinned_outputs()
            out = {k: bufs[k][:int(np.prod(v))].reshape(v) for k, v in shapes.items()}
        else:
            out = {k: np.zeros(v) for k, v in shapes.items()}
        if not with_ks:
            out['K'] = out['Sigma'] = None
        out.update(n_accepted=np.zeros(B, np.int32), iterations=np.zeros(B, np.int32), status=np.zeros(B, np.int32),
                   weight=np.zeros(B), radius=np.zeros(B))
        keys = ('X', 'U', 'K', 'Sigma', 'n_accepted', 'iterations', 'status', 'weight', 'radius')
        self._chk(self.lib.cmpc_get_solution(self.h, *[_ptr(out[k]) for k in keys]), 'cmpc_get_solution')
        return out

    def prefetch_ks(self):
        """Reference mode: stream the next solve's accepted K and Sigma into this Solver's pinned
        output arrays while it runs (cmpc_prefetch_ks); solution(pinned=True) then only waits."""
        bufs = self._pinned_outputs()
        self._chk(self.lib.cmpc_prefetch_ks(self.h, _ptr(bufs['K']), _ptr(bufs['Sigma'])), 'cmpc_prefetch_ks')

    def _pinned_outputs(self):
        """Flat fp64 output arrays for max_batch problems, page-locked once per Solver."""
        if getattr(self, '_pinned', None) is None:
            Bm, N = self.max_batch, self.N
            sizes = dict(X=Bm * (N + 1) * 9, U=Bm * N * 12, K=Bm * N * 12 * 9, Sigma=Bm * (N + 1) * 81)
            self._pinned = {}
            for k, n in sizes.items():
                a = np.empty(n)
                a.fill(0.0)   # fault the pages in once
                self._chk(self.lib.cmpc_host_register(self.h, a.ctypes.data_as(ctypes.c_void_p), a.nbytes),
                          'cmpc_host_register')
                self._pinned[k] = a
        return self._pinned

    def iteration_log(self):
        B = self.B
        out = dict(tr_norm=np.zeros(B), rho=np.zeros(B), qp_status=np.zeros(B, np.int32),
                   qp_iters=np.zeros(B, np.int32), decision=np.zeros(B, np.int32))
        keys = ('tr_norm', 'rho', 'qp_status', 'qp_iters', 'decision')
        self._chk(self.lib.cmpc_get_iteration_log(self.h, *[_ptr(out[k]) for k in keys]), 'cmpc_get_iteration_log')
        return out

    def iteration_history(self, cap=None):
        """Every SCP iteration of every problem since the upload (cmpc_get_iteration_history):
        (records (B, cap) of ITER_RECORD_DTYPE, n_records (B)); cap defaults to the largest
        max_iterations of the uploaded parameter classes."""
        if cap is None:
            cap = max(int(p.scp_params.get('max_iterations', 10)) for p in self._params) if self._params else 10
        rec = np.zeros((self.B, int(cap)), ITER_RECORD_DTYPE)
        n = np.zeros(self.B, np.int32)
        assert ITER_RECORD_DTYPE.itemsize == ctypes.sizeof(IterRecord)
        self._chk(self.lib.cmpc_get_iteration_history(self.h, int(cap), _ptr(rec), _ptr(n)),
                  'cmpc_get_iteration_history')
        return rec, n

    def accepted(self, j, with_ks=True):
        """Accepted iterate j of every problem (cmpc_get_accepted): X (B,N+1,9), U (B,N,12) and, with
        with_ks, K (B,N,12,9), Sigma (B,N+1,9,9); zeros for problems with fewer accepts."""
        B, N = self.B, self.N
        X = np.zeros((B, N + 1, 9)); U = np.zeros((B, N, 12))
        K = np.zeros((B, N, 12, 9)) if with_ks else None
        S = np.zeros((B, N + 1, 9, 9)) if with_ks else None
        self._chk(self.lib.cmpc_get_accepted(self.h, int(j), _ptr(X), _ptr(U), _ptr(K), _ptr(S)), 'cmpc_get_accepted')
        return dict(X=X, U=U, K=K, Sigma=S)

    def timing(self):
        t = Timing()
        self._chk(self.lib.cmpc_get_timing(self.h, ctypes.byref(t)), 'cmpc_get_timing')
        return dict(linearize_ms=t.linearize_ms, assemble_ms=t.assemble_ms, qp_ms=t.qp_ms,
                    accept_ms=t.accept_ms, total_ms=t.total_ms)

    def timing_begin(self):
        self._chk(self.lib.cmpc_timing_begin(self.h), 'cmpc_timing_begin')

    def timing_end(self):
        t = Timing(); n = ctypes.c_int(0)
        self._chk(self.lib.cmpc_timing_end(self.h, ctypes.byref(t), ctypes.byref(n)), 'cmpc_timing_end')
        return dict(linearize_ms=t.linearize_ms, assemble_ms=t.assemble_ms, qp_ms=t.qp_ms,
                    accept_ms=t.accept_ms, total_ms=t.total_ms, iterations=n.value)

    def qp_iterations_total(self):
        v = ctypes.c_int64(0)
        self._chk(self.lib.cmpc_get_qp_iterations_total(self.h, ctypes.byref(v)), 'cmpc_get_qp_iterations_total')
        return int(v.value)

    def qp_kernel(self):
        """Name of the QP kernel the library launches for the uploaded batch (cmpc_get_qp_kernel)."""
        buf = ctypes.create_string_buffer(64)
        self._chk(self.lib.cmpc_get_qp_kernel(self.h, buf, 64), 'cmpc_get_qp_kernel')
        return buf.value.decode()

    def debug_stamps(self):
        out = np.zeros((self.B, 16), np.uint64)
        self._chk(self.lib.cmpc_debug_stamps(self.h, _ptr(out)), 'cmpc_debug_stamps')
        return out
