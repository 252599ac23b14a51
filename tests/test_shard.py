"""Multi-process plumbing of the batch split (CPU, no GPU): slices tile the batch, the RCCL id
rendezvous hands rank 0's bytes to every rank over TCP, ``spawn_local`` starts one process per
rank with the launcher variables and propagates failures, and the rank-major gather order equals
the global problem order.  The RCCL collectives themselves run in tests/test_gpu_comm.py."""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

from cmpc.shard import ID_BYTES, exchange_id, free_port, shard_bounds, spawn_local
from cmpc.synth import make_batch


def test_shard_bounds_tile_the_batch():
    """Contiguous slices of floor / ceil(B / world): none empty while B >= world (an empty rank could
    not take part in the gather), equal at the metric's 1024 over 1/2/4/8 ranks."""
    for B in (1, 2, 7, 9, 1024, 1025):
        for world in (1, 2, 3, 4, 8):
            if B < world:
                with pytest.raises(ValueError):
                    shard_bounds(B, 0, world)
                continue
            spans = [shard_bounds(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
    assert [shard_bounds(1024, r, 8) for r in range(8)] == [(128 * r, 128 * (r + 1)) for r in range(8)]
    assert [shard_bounds(9, r, 4)[1] - shard_bounds(9, r, 4)[0] for r in range(4)] == [2, 2, 2, 3]
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _rdzv_worker(rank, world, port, q):
    uid = exchange_id(rank, world, lambda: bytes(range(ID_BYTES)) if rank == 0 else None, '127.0.0.1', port,
                      timeout=30.0)
    q.put((rank, uid))


@pytest.mark.parametrize('world', [2, 3])
def test_rccl_id_rendezvous(world):
    port = free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rdzv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    assert sorted(got) == list(range(world))
    assert all(v == bytes(range(ID_BYTES)) for v in got.values())


def test_spawn_local_sets_launcher_env(tmp_path):
    script = tmp_path / 'child.py'
    script.write_text('import os, sys\n'
                      'open(os.path.join(sys.argv[1], "r%s" % os.environ["RANK"]), "w").write(\n'
                      '    " ".join(os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")))\n')
    rc = spawn_local(2, [str(script), str(tmp_path)], timeout=120)
    assert rc == 0
    assert (tmp_path / 'r0').read_text() == '0 0 2 127.0.0.1'
    assert (tmp_path / 'r1').read_text() == '1 1 2 127.0.0.1'


def test_spawn_local_propagates_a_failure(tmp_path):
    script = tmp_path / 'child.py'
    script.write_text('import os, sys, time\n'
                      'if os.environ["RANK"] == "1": sys.exit(3)\n'
                      'time.sleep(60)\n')
    rc = spawn_local(2, [str(script)], timeout=120)
    assert rc == 3


def test_rank_major_gather_is_the_global_order():
    """Contiguous slices generated per rank with seed offset lo reproduce the global batch, so the
    rank-major concatenation of per-rank results (what cmpc_comm_gather_solution returns) is the
    global problem order."""
    B, world = 12, 4
    full = make_batch('trot', 20, B, seed_offset=0)
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(B, r, world)
        parts.append(make_batch('trot', 20, hi - lo, seed_offset=lo))
    for k in ('Xbar', 'Ubar', 'logic', 'pos'):
        assert np.array_equal(np.concatenate([getattr(p, k) for p in parts]), getattr(full, k)), k


def test_bench_gpus_flag_spawns_one_process_per_gpu(tmp_path):
    """``bench.py --gpus 2`` without a launcher starts two ranks (here they stop at the missing GPU /
    library, which must surface as a nonzero exit code, never as a one-GPU number)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    env['HIP_VISIBLE_DEVICES'] = ''
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '1', '--warmup', '0',
                        '--batch', '2', '--N', '10', '--no-cpu-baseline'], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout


def test_bench_multirank_orchestration_on_cpu(tmp_path):
    """bench.py's multi-rank path end to end in two processes (tests/bench_stub.py: CPU stubs for the
    device Solver and a socket-based RcclComm): each rank uploads its contiguous slice of the
    global batch, the timed region sits between two barriers and takes the max over ranks, the
    weak-scaling leg runs, the accepted solutions are gathered to rank 0 in global order, and only
    rank 0 prints the one JSON line."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env['HIP_VISIBLE_DEVICES'] = ''
    B, N = 1024, 10
    rc = spawn_local(2, [os.path.join(root, 'tests', 'bench_stub.py'), str(tmp_path), '--gpus', '2', '--steps', '3',
                         '--warmup', '1', '--batch', str(B), '--N', str(N), '--no-cpu-baseline'], env=env, timeout=600)
    assert rc == 0
    lines0 = [l for l in (tmp_path / 'rank0.txt').read_text().splitlines() if l.strip()]
    lines1 = [l for l in (tmp_path / 'rank1.txt').read_text().splitlines() if l.strip()]
    assert len(lines0) == 1 and lines1 == []
    out = json.loads(lines0[0])
    assert out['n_gpus'] == 2 and out['scaling'] == 'strong' and out['steps'] == 3
    assert out['config']['global_batch'] == B and out['config']['batch_per_gpu'] == B // 2
    assert out['value'] == pytest.approx(B * 3 / (out['ms_per_step'] * 3 / 1e3))
    assert out['weak_scaling']['global_batch'] == 2 * B and out['weak_scaling']['per_gpu'] == B
    assert out['gather_ms'] >= 0 and out['early_exit']['scp_iterations'] == B
    # the gather holds both slices in the global problem order
    g = np.load(tmp_path / 'gather.npz')
    full = make_batch('trot', N, B, seed_offset=0)
    assert g['X'].shape == (B, N + 1, 9)
    np.testing.assert_array_equal(g['X'][:, 0, :], full.Xbar[:, 0, :])
    # barriers: 1 (timed, start) + 1 (clock) per timed leg x 2 legs, the gather's barrier, and the
    # early-exit barrier + clock: the same count on both ranks
    c0 = (tmp_path / 'calls0.txt').read_text().split()
    c1 = (tmp_path / 'calls1.txt').read_text().split()
    assert c0 == c1 and int(c0[1]) == 1 and int(c0[0]) >= 6
