"""Multi-process sharding (world_size 2, gloo, CPU): slices tile the batch and the gathered
result equals the single-process result.  The per-shard solver is a deterministic stand-in
(the device solve itself is covered by the GPU tests)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from cmpc.shard import gather_results, shard_bounds, solve_shard
from cmpc.synth import make_batch


def fake_solve(pb):
    """Per-problem values that depend only on that problem's inputs."""
    X = pb.Xbar.copy()
    X[:, :, 0] += pb.logic.sum(axis=(1, 2))[:, None]
    return dict(X=X, n_accepted=pb.logic[:, 0, 0].astype(np.int32), status=np.ones(pb.B, np.int32))


def test_shard_bounds_tile_the_batch():
    for B in (1, 2, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert all(hi - lo <= -(-B // world) for lo, hi in spans)
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, out_path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    pb = make_batch('trot', 20, B, seed_offset=5)
    lo, hi, res = solve_shard(pb, rank, world, solve_fn=fake_solve)
    full = gather_results(lo, hi, res, B, dist)
    if rank == 0:
        np.savez(out_path, **full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('B', [5, 6])
def test_gloo_world2_gather_matches_single_process(tmp_path, B):
    out = str(tmp_path / 'full.npz')
    mp.start_processes(_worker, args=(2, _free_port(), B, out), nprocs=2, join=True, start_method='spawn')
    got = dict(np.load(out))
    ref = fake_solve(make_batch('trot', 20, B, seed_offset=5))
    assert set(got) == set(ref)
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k
