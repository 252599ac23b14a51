"""Batch sharding across GPUs: one process per GPU, contiguous problem slices, no collective in
the data path.

Problems are independent, so rank r of G solves problems [lo_r, hi_r) of the batch on its own
device (weak scaling when every rank holds a fixed number of problems).  The only
communication is around the loop: ``gather_results`` collects the per-rank result arrays on
rank 0 (``torch.distributed.gather_object`` over whatever process group is initialized; gloo
in the tests, RCCL for device tensors would need the same call pattern), and barriers bracket
timed regions in bench.py.
"""
import os

import numpy as np


def shard_bounds(B, rank, world):
    """[lo, hi) of rank's contiguous slice: ceil(B / world) problems per rank, the last ranks
    possibly short or empty."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('invalid rank %d of %d' % (rank, world))
    per = -(-B // world)
    lo = min(B, rank * per)
    return lo, min(B, lo + per)


def gpu_solve(pb, device=0, precision='fp64', fixed_iters=False):
    """Solve a ProblemBatch on one device; per-problem result arrays (leading dim = pb.B)."""
    from cmpc._lib import Solver
    with Solver(pb.robot, pb.N, max(pb.B, 1), precision, device) as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=fixed_iters)
        return s.solution()


def solve_shard(pb, rank, world, solve_fn=None, **kw):
    """This rank's slice of ``pb`` solved by ``solve_fn(pb_slice)`` (default: ``gpu_solve`` on
    device = LOCAL_RANK).  Returns (lo, hi, result dict)."""
    lo, hi = shard_bounds(pb.B, rank, world)
    if solve_fn is None:
        device = int(os.environ.get('LOCAL_RANK', rank))
        solve_fn = lambda p: gpu_solve(p, device=device, **kw)
    res = solve_fn(pb.subset(lo, hi)) if hi > lo else {}
    return lo, hi, res


def gather_results(lo, hi, res, B, dist=None):
    """Concatenate every rank's (lo, hi, res) on rank 0 in problem order; other ranks get None.
    Without an initialized process group this is the identity on the single shard."""
    if dist is None or not dist.is_initialized():
        return res
    parts = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object((lo, hi, {k: np.asarray(v) for k, v in res.items()}), parts, dst=0)
    if dist.get_rank() != 0:
        return None
    parts = sorted((p for p in parts if p[1] > p[0]), key=lambda p: p[0])
    if not parts or parts[0][0] != 0 or parts[-1][1] != B or any(a[1] != b[0] for a, b in zip(parts, parts[1:])):
        raise RuntimeError('shards do not tile the batch')
    return {k: np.concatenate([p[2][k] for p in parts]) for k in parts[0][2]}
