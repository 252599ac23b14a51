"""Generate golden vectors by running the REFERENCE's own code (test infrastructure).

Run in the build container only (needs /root/reference; skipped when absent):
    python tests/golden/make_golden.py

The reference imports jax, pinocchio, casadi and osqp, none of which is installed (no network);
they are replaced by minimal numpy stand-ins that provide only the mechanics the reference
uses -- jit = identity, lax.fori_loop = Python loop, dynamic_update_slice, ``.at[].set/add``,
JAX's clamped out-of-range gather, and jacfwd/jacrev by unit forward differences (exact here:
the centroidal dynamics are linear in each argument separately).  All arithmetic that produces
the fixtures is the reference's own (src/centroidal_model.py, src/cost.py, src/constraints.py,
src/scp_solver.py, src/contact_plan.py).

Precision: the real reference runs its JAX parts in float32 (JAX's default; no x64 flag anywhere in
the reference).  The fixtures named ``*_f32`` keep that: under them every stand-in array op
returns float32, as jax.numpy does, and jacfwd returns the exact derivative rounded to float32
(the differences are taken in float64; the dynamics are affine in each argument, so the difference
is the derivative).  The other fixtures run the same code in float64.

QP: the osqp stand-in is the oracle's OSQP restatement (ADMM + polish) for the N=20 Solo12
fixtures, and the oracle's sparse interior-point solver for TALOS (ADMM needs > 20000 iterations
on its subproblems) and the N >= 50 fixtures.  Either way the solve_scp fixture pins the state
machine around the QP, not the QP solver (OSQP itself is not installed: parity with it is unpinned).

Only arrays are written (tests/golden/*.npz); no reference source is copied.
"""
import functools
import os
import sys
import tempfile
import types

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


# ----------------------------------------------------------------------------- stand-ins
class JArr(np.ndarray):
    """ndarray with JAX's functional updates and clamped integer gathers."""

    def __array_finalize__(self, obj):
        pass

    @property
    def at(self):
        return _At(self)

    def __getitem__(self, idx):
        idx = self._clamp(idx)
        return super().__getitem__(idx)

    def __iter__(self):   # iteration must stop at the end (clamping applies to explicit gathers only)
        for i in range(self.shape[0]):
            yield super().__getitem__(i)

    def _clamp(self, idx):
        tup = idx if isinstance(idx, tuple) else (idx,)
        out, ax = [], 0
        for c in tup:
            if c is Ellipsis or c is None:
                out.append(c)
                ax += 0 if c is None else 1
                continue
            if isinstance(c, (int, np.integer)) and not isinstance(c, bool) and ax < self.ndim:
                n = self.shape[ax]
                c = int(min(max(c, -n), n - 1))
            out.append(c)
            ax += 1
        return tuple(out) if isinstance(idx, tuple) else out[0]


class _At:
    def __init__(self, a):
        self.a = a

    def __getitem__(self, idx):
        a = self.a

        class _U:
            def set(_, v):
                b = np.array(a, copy=True).view(JArr)
                np.ndarray.__setitem__(b, idx, v)
                return b

            def add(_, v):
                b = np.array(a, copy=True).view(JArr)
                np.ndarray.__setitem__(b, idx, np.ndarray.__getitem__(b, idx) + v)
                return b
        return _U()


FP32 = [False]   # set while an *_f32 fixture is generated


def _fdt():
    return np.float32 if FP32[0] else np.float64


def _w(x):
    if np.isscalar(x):
        return x
    a = np.asarray(x)
    return np.asarray(a, dtype=_fdt() if a.dtype.kind in 'fc' else None).view(JArr)


def _jacfwd(f, argnums=0):
    def jf(*args):
        # differences in float64 even for the float32 fixtures: the result is the exact
        # derivative (affine dynamics), rounded once to the working precision as forward-mode
        # AD in float32 would be
        was = FP32[0]
        FP32[0] = False
        try:
            args = [np.asarray(a, float).view(JArr) if isinstance(a, np.ndarray) and a.dtype.kind == 'f' else a
                    for a in args]
            x0 = np.asarray(args[argnums], float)
            f0 = np.asarray(f(*args), float)
            J = np.zeros(f0.shape + x0.shape)
            for i in np.ndindex(*x0.shape):
                xp = x0.copy(); xp[i] += 1.0
                a2 = list(args); a2[argnums] = xp.view(JArr)
                J[(Ellipsis,) + i] = np.asarray(f(*a2), float) - f0
        finally:
            FP32[0] = was
        return _w(J)
    return jf


QP = [None]   # the osqp stand-in's solver for the fixture being generated


def install_standins():
    jax = types.ModuleType('jax')
    jnp = types.ModuleType('jax.numpy')
    for name in ('zeros', 'ones', 'eye', 'hstack', 'vstack', 'cross', 'arange', 'where', 'einsum', 'sum',
                 'concatenate', 'sqrt', 'diag', 'stack', 'reshape'):
        fn = getattr(np, name)
        setattr(jnp, name, (lambda fn_: lambda *a, **k: _w(fn_(*a, **k)))(fn))
    jnp.array = lambda x, *a, **k: _w(np.array(x, *a, **k))
    jnp.float32 = np.float32
    jnp.array_split = lambda x, n, *a: [_w(v) for v in np.array_split(np.asarray(x), n, *a)]
    jnp.linalg = types.SimpleNamespace(solve=lambda A, b: _w(np.linalg.solve(A, b)))

    def _to_j(a):
        if isinstance(a, np.ndarray) and a.dtype.kind == 'f' and a.dtype != _fdt():
            return np.asarray(a, _fdt()).view(JArr)   # a device array holds JAX's default float
        if isinstance(a, np.ndarray) and not isinstance(a, JArr):
            return a.view(JArr)
        if isinstance(a, dict):
            return {k: _to_j(v) for k, v in a.items()}
        return a

    def jit(f=None, **kw):
        # a jitted function sees device arrays (clamped gathers) -- convert at the boundary
        if f is None:
            return lambda g: jit(g)

        @functools.wraps(f)
        def wrapped(*a, **k):
            return f(*[_to_j(v) for v in a], **{kk: _to_j(v) for kk, v in k.items()})
        return wrapped
    jax.jit = jit
    lax = types.ModuleType('jax.lax')

    def fori_loop(lo, hi, body, init):
        v = init
        for i in range(lo, hi):
            v = body(i, v)
        return v

    def dus(a, upd, start):
        b = np.array(a, copy=True)
        upd = np.asarray(upd)
        sl = tuple(slice(int(s), int(s) + n) for s, n in zip(start, upd.shape))
        b[sl] = upd
        return b.view(JArr)

    def dus_dim(a, upd, start, axis):
        st = [0] * np.ndim(a); st[axis] = int(start)
        return dus(a, upd, st)
    lax.fori_loop = fori_loop
    lax.dynamic_update_slice = dus
    lax.dynamic_update_slice_in_dim = dus_dim
    jax.lax = lax
    jax.numpy = jnp
    jax.jacfwd = _jacfwd
    jax.jacrev = _jacfwd
    tu = types.ModuleType('jax.tree_util')
    tu.register_pytree_node_class = lambda c: c
    jax.tree_util = tu
    sys.modules.update({'jax': jax, 'jax.numpy': jnp, 'jax.lax': lax, 'jax.tree_util': tu})
    cas = types.ModuleType('casadi'); cas.__all__ = []
    sys.modules['casadi'] = cas
    pin = types.ModuleType('pinocchio')

    class SE3:
        def __init__(self, R, t):
            self.rotation = np.asarray(R, float); self.translation = np.asarray(t, float)

    class AngleAxis:
        def __init__(self, angle, axis):
            self.angle = angle; self.axis = np.asarray(axis, float)

        def matrix(self):
            a = self.axis
            K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
            return np.eye(3) + np.sin(self.angle) * K + (1 - np.cos(self.angle)) * K @ K
    pin.SE3 = SE3
    pin.AngleAxis = AngleAxis
    pin.forwardKinematics = lambda *a: None
    pin.updateFramePlacements = lambda *a: None
    sys.modules['pinocchio'] = pin
    osqp = types.ModuleType('osqp')

    class OSQP:
        def setup(self, P, q, A, l, u, **kw):
            self.args = (P, q, A, l, u)

        def solve(self):
            return QP[0](*self.args)
    osqp.OSQP = OSQP
    sys.modules['osqp'] = osqp


# ----------------------------------------------------------------------------- fixtures
class FakeRobot:
    def __init__(self, name, feet):
        self.name = name
        self.oMf = {k: types.SimpleNamespace(translation=np.array(v, float)) for k, v in feet.items()}

    def getFrameId(self, n):
        return n


PRODUCT = {}   # filled by main() before the reference's src/ is put on sys.path


def make_conf(kind, N):
    c = PRODUCT['confs'][kind]
    conf = types.SimpleNamespace(**{k: getattr(c, k) for k in dir(c) if not k.startswith('__')})
    feet = PRODUCT['solo_feet'] if kind != 'talos' else PRODUCT['talos_feet']
    rob = FakeRobot('solo' if kind != 'talos' else 'talos', feet)
    return conf, rob


def generate(kind, N, stochastic, tag, out, qp, fp32=False):
    QP[0] = qp
    FP32[0] = fp32
    try:
        _generate(kind, N, stochastic, tag, out, fp32)
    finally:
        FP32[0] = False


def _generate(kind, N, stochastic, tag, out, fp32):
    from src.contact_plan import create_contact_sequence as ref_seq   # reference module
    conf, rob = make_conf(kind, N)
    gait = dict(conf.gait)
    while True:
        _, seq = ref_seq(conf.dt, gait, conf.ee_frame_names, rob, rob, None)
        if int(round(seq[-1][0].t_end / conf.dt, 2)) >= N:
            break
        gait['nbSteps'] += 1
        _, rob = make_conf(kind, N)
    conf.contact_sequence = seq
    conf.N = N
    # synthetic warm start on the reference's own contact arrays
    from src.contact_plan import create_contact_trajectory as ref_traj
    ctraj = ref_traj(conf)
    names = list(ctraj.keys())
    logic = np.array([[1 if ctraj[c][k].ACTIVE else 0 for c in names] for k in range(N)], np.int8)
    pos = np.array([[ctraj[c][k].pose.translation if ctraj[c][k].ACTIVE else np.zeros(3) for c in names]
                    for k in range(N)])
    warm_start = PRODUCT['warm_start']
    rng = np.random.default_rng(4242)
    com_z = 0.24 if kind != 'talos' else 0.87
    X = warm_start(conf, logic, pos, rng, conf.robot_mass, com_z, conf.gravity_constant, conf.robot_name)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            np.savez('wholeBody_to_centroidal_traj.npz', X=X)
            from src.centroidal_model import Centroidal_model
            import src.scp_solver as scp
            model = Centroidal_model(conf, STOCHASTIC_OCP=stochastic)
            traj = model._init_trajectories
            tdat = model.compute_trajectory_data(traj)
            cost = scp.sum_up_all_costs(model)
            tr1 = {'weight': 100.0, 'radius': float(conf.scp_params['trust_region_radius0'])}
            tr2 = {'weight': 2500.0, 'radius': 0.3}
            c1 = scp.stack_up_all_constraints(model, traj, tdat, tr1)
            c2 = scp.stack_up_all_constraints(model, traj, tdat, tr2)
            rng2 = np.random.default_rng(7)
            Xs = np.asarray(traj['state']) + 1e-2 * rng2.normal(size=np.shape(traj['state']))
            Us = np.asarray(traj['control']) + 1e-1 * rng2.normal(size=np.shape(traj['control']))
            roll = model.integrate_dynamics_trajectory(dict(state=Xs.view(JArr), control=Us.view(JArr)))
            rho = scp.compute_model_accuracy(model, dict(state=Xs, control=Us), traj, tdat)
            interp = scp.interpolate_SCP_solution(dict(state=[Xs], control=[Us]))
            sol = scp.solve_scp(model, conf.scp_params)
        finally:
            os.chdir(cwd)
    d = dict(kind=kind, N=N, stochastic=int(stochastic), fp32=int(fp32), Xnpz=X,
             logic=np.asarray(model._contact_data['contacts_logic']),
             pos=np.asarray(model._contact_data['contacts_position']),
             rot=np.asarray(model._contact_data['contacts_orient']),
             Xbar=np.asarray(traj['state']), Ubar=np.asarray(traj['control']),
             dynamics=np.asarray(tdat['dynamics']), f_x=np.asarray(tdat['gradients']['f_x']),
             f_u=np.asarray(tdat['gradients']['f_u']), f_w=np.asarray(tdat['gradients']['f_w']),
             K=np.asarray(tdat['LQR_gains']), Covs=np.asarray(tdat['Covs']),
             cov_grad_maxabs=max(np.abs(tdat['Covs_gradients']['Cov_dx']).max(),
                                 np.abs(tdat['Covs_gradients']['Cov_du']).max()),
             P_data=cost.Q.data, P_indices=cost.Q.indices, P_indptr=cost.Q.indptr, q=np.asarray(cost.p),
             tr1=np.array([tr1['weight'], tr1['radius']]), tr2=np.array([tr2['weight'], tr2['radius']]),
             rollout_X=Xs, rollout_U=Us, rollout=np.asarray(roll), rho=float(rho),
             interp_X=interp['X'], interp_U=interp['U'], n=model._total_nb_optimizers)
    for tg, c in (('c1', c1), ('c2', c2)):
        A = c.mat.tocsc()
        d[tg + '_A_data'] = A.data; d[tg + '_A_indices'] = A.indices; d[tg + '_A_indptr'] = A.indptr
        d[tg + '_A_shape'] = np.array(A.shape); d[tg + '_l'] = np.asarray(c.lb); d[tg + '_u'] = np.asarray(c.ub)
    if sol is False:
        d['scp_ok'] = 0
    else:
        d['scp_ok'] = 1
        d['scp_n_accepted'] = len(sol['state'])
        d['scp_X'] = np.asarray(sol['state'][-1]); d['scp_U'] = np.asarray(sol['control'][-1])
    np.savez_compressed(os.path.join(out, 'golden_%s.npz' % tag), **d)
    print('wrote', tag, 'scp_ok', d['scp_ok'])


def FIXTURES(admm, ipm):
    """(kind, N, stochastic, tag, QP stand-in, float32).  N=50 is BASELINE C1's horizon, N=100
    the metric config's and C2 / C3's; bound_n100_f32 is C3 at the reference's own precision."""
    return (('trot', 20, False, 'trot', admm, False), ('trot', 20, True, 'trot_stoch', admm, False),
            ('bound', 20, False, 'bound', admm, False), ('pace', 20, False, 'pace', admm, False),
            ('talos', 20, False, 'talos', ipm, False),
            ('trot', 50, False, 'trot_n50', ipm, False), ('trot', 100, False, 'trot_n100', ipm, False),
            ('bound', 100, False, 'bound_n100', ipm, False),
            ('trot', 20, False, 'trot_f32', ipm, True), ('bound', 100, False, 'bound_n100_f32', ipm, True))


def main():
    if not os.path.isdir(REF):
        print('reference not present; nothing to do')
        return
    # 1. product helpers first (they import the product's src/ and config/ packages)
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
    from cmpc import synth
    from config import _robots
    from oracle.osqp_admm import solve_qp as oracle_qp
    from oracle.sparse_ipm import solve_qp as sparse_ipm_qp
    PRODUCT.update(confs={k: synth.load_conf(k) for k in ('trot', 'bound', 'pace', 'talos')},
                   warm_start=synth.warm_start, solo_feet=_robots.SOLO12_FEET, talos_feet=_robots.TALOS_FEET)
    # 2. swap in the reference's src/ package under the stand-ins
    for m in [m for m in sys.modules if m in ('src', 'config') or m.startswith(('src.', 'config.'))]:
        del sys.modules[m]
    install_standins()
    sys.path.insert(0, REF)
    import src  # noqa: F401
    assert os.path.realpath(os.path.dirname(src.__file__)).startswith(os.path.realpath(REF)), src.__file__
    admm = lambda P, q, A, l, u: oracle_qp(P, q, A, l, u, max_iter=20000)
    ipm = lambda P, q, A, l, u: sparse_ipm_qp(P, q, A, l, u)
    want = sys.argv[1:]
    for kind, N, stoch, tag, qp, f32 in FIXTURES(admm, ipm):
        if not want or tag in want:
            generate(kind, N, stoch, tag, HERE, qp, f32)


if __name__ == '__main__':
    main()
