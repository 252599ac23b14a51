"""Device-side assembly shared by the drop-in cost / constraints / scp_solver modules.

The QP is assembled on the GPU (cmpc_linearize + cmpc_assemble) in the solver's structured
form; ``cmpc_export_qp`` writes it out as CSC in the reference's exact variable and row order
(z = [x | u | t | s], rows init | dyn | final | [cop] | friction | trust region | slack), which
is how the reference's matrix-building functions are answered here.
"""
import numpy as np


def export(model, traj_tuple=None, trust_region=None):
    """(solver, P, q, A, l, u) for ``model`` linearized at ``traj_tuple`` (default: the model's
    warm start) with ``trust_region`` = {'weight', 'radius'} (default omega0 / radius0)."""
    s = model._device_solver(traj_tuple)
    if trust_region is not None:
        s.set_trust_region(weight=float(np.asarray(trust_region['weight'])),
                           radius=float(np.asarray(trust_region['radius'])))
    s.linearize()
    s.assemble()
    P, q, A, l, u = s.export_qp(0)
    return s, P, q, A, l, u


def row_blocks(model):
    """Row ranges of each constraint family in the reference's stacking order
    (src/scp_solver.py:28-48)."""
    N, nx = model._N, model._n_x
    nc = len(model._contact_trajectory)
    out, r = {}, 0
    order = [('initial', nx), ('dynamics', nx * N), ('final', nx)]
    if model._robot == 'TALOS':
        order.append(('cop', 2 * nc * N))
    order += [('friction', 5 * nc * N), ('trust_region', 8 * (N + 1)), ('slack', N + 1)]
    for name, n in order:
        out[name] = (r, r + n)
        r += n
    return out


def rows(A, l, u, r0, r1):
    return A.tocsr()[r0:r1].tocsc(), l[r0:r1].copy(), u[r0:r1].copy()
