"""npz hand-off with the whole-body DDP stages, batched.

The reference chains DDP -> SCP -> DDP through three npz files (demos/trot_demo.ipynb:40,61;
demos/bound_demo.ipynb:40,60-61; src/whole_body_control.py:41-44):

* ``wholeBody_to_centroidal_traj.npz``: key 'X', (N+1, 9) centroidal states of the DDP
  solution (rows = knots), the SCP warm start (src/centroidal_model.py:174: X.T);
* ``centroidal_to_wholeBody_traj.npz``: keys 'X' (9, N+1) and 'U' (nu, N), the last accepted
  SCP solution (scp_sol['state'][-1], scp_sol['control'][-1]) that the whole-body tracking
  problem loads when TRACK_CENTROIDAL (src/whole_body_control.py:41-44);
* ``scp_sol_interpol_*.npz``: keys 'X', 'U' of interpolate_SCP_solution.

These helpers read / write the same files for one problem or a whole batch (one file per
problem, ``<stem>_<b>.npz``), so the unchanged notebooks and the whole-body stages consume the
device solutions directly.  Host-side I/O only; the arrays cross the C ABI as in cmpc_upload.
"""
import os

import numpy as np

WARM_START = 'wholeBody_to_centroidal_traj.npz'
TO_WHOLE_BODY = 'centroidal_to_wholeBody_traj.npz'


def _batch_paths(path, B):
    stem, ext = os.path.splitext(path)
    return [path] if B == 1 else ['%s_%d%s' % (stem, b, ext or '.npz') for b in range(B)]


def load_warm_start(paths, N):
    """Xbar (B, N+1, 9) from DDP warm-start files (key 'X', (N+1, 9) each).  A longer DDP
    trajectory is truncated to N+1 knots (the reference's behaviour when conf.N is below the
    plan length); a shorter one is an error."""
    if isinstance(paths, str):
        paths = [paths]
    out = np.zeros((len(paths), N + 1, 9))
    for b, p in enumerate(paths):
        X = np.asarray(np.load(p)['X'], float)
        if X.ndim != 2 or X.shape[1] != 9 or X.shape[0] < N + 1:
            raise ValueError('%s: expected X of shape (>= %d, 9), got %s' % (p, N + 1, X.shape))
        out[b] = X[:N + 1]
    return out


def save_warm_start(path, Xbar):
    """Write DDP-style warm-start files from Xbar (B, N+1, 9) or (N+1, 9)."""
    Xbar = np.asarray(Xbar, float)
    Xbar = Xbar[None] if Xbar.ndim == 2 else Xbar
    paths = _batch_paths(path, len(Xbar))
    for p, X in zip(paths, Xbar):
        np.savez(p, X=X)
    return paths


def save_to_whole_body(path, results):
    """Write centroidal_to_wholeBody_traj.npz file(s) from solve_scp / solve_scp_batch results
    (X = state[-1] (9, N+1), U = control[-1] (nu, N)); problems whose solve returned False or
    accepted nothing get no file (None in the returned list)."""
    if isinstance(results, dict) or results is False:
        results = [results]
    paths = _batch_paths(path, len(results))
    out = []
    for p, r in zip(paths, results):
        if r is False or not r['state']:
            out.append(None)
            continue
        np.savez(p, X=np.asarray(r['state'][-1], float), U=np.asarray(r['control'][-1], float))
        out.append(p)
    return out


def save_interpolated(path, interpolated):
    """Write scp_sol_interpol_*.npz file(s): dict(X, U) or a list of them (e.g. the
    'interpolated' entries of solve_scp_batch(..., n_inner=10))."""
    if isinstance(interpolated, dict):
        interpolated = [interpolated]
    paths = _batch_paths(path, len(interpolated))
    for p, d in zip(paths, interpolated):
        np.savez(p, X=np.asarray(d['X'], float), U=np.asarray(d['U'], float))
    return paths


def load_tracking(path):
    """(X (9, N+1), U (nu, N)) as the whole-body stage reads centroidal_to_wholeBody_traj.npz
    (src/whole_body_control.py:41-44)."""
    f = np.load(path)
    return np.asarray(f['X']), np.asarray(f['U'])
