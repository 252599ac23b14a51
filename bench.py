#!/usr/bin/env python3
"""Benchmark: SCP iterations/sec, Solo12-trot N=100, batch 1024 per GPU (BASELINE.json metric).

One "step" = one full SCP iteration (linearize -> structured assembly -> batched interior-point
QP -> trust-region accept/reject) for every problem resident on the GPU, in the benchmark's
fixed-K mode (every problem iterates each step).  Inputs are uploaded
to HBM before the timed region; nothing is copied in or out inside it.

Multi-GPU (launched by torch.distributed.run): one process per GPU, each rank owns its own
shard of 1024 problems (weak scaling, no collective in the data path); a gloo barrier brackets
the timed region and the max time over ranks is reported.

Extra fields ("Measurement"):
  roofline      QP kernel: algorithmic bytes per launch (SURVEY.md 8d per-IPM-iteration figure
                x IPM iterations actually run) / its mean duration from HIP events recorded
                on the library's stream over the timed region.
  cpu_baseline  the oracle (numpy/scipy restatement of the reference path, OSQP algorithm at
                the reference's eps 1e-7 with polish) on a bounded sample, rank 0 at N = 1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]

import numpy as np  # noqa: E402

METRIC = 'SCP iterations/sec, Solo12-trot N=100 batch=1024 @ 1/2/4/8 GPU'
WORKLOAD_NAMES = {'trot': 'conf_solo12_trot', 'bound': 'conf_solo12_bound', 'pace': 'conf_solo12_pace',
                  'talos': 'conf_talos', 'mixed': 'Solo12 pace+trot mixed contact plans'}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def algorithmic_qp_bytes(N, ipm_iters_total, w):
    """per IPM iteration one factorization pass N*w*(Lf + 2*103 + n_k + m_k)
    (Lf = 451, n_k = 22, m_k = 38) plus two Newton solves of ~N*w*1000 each."""
    per_iter = N * w * (451 + 2 * 103 + 22 + 38) + 2 * N * w * 1000
    return per_iter * ipm_iters_total


def cpu_baseline(N, seconds_target=12.0):
    """Time the oracle SCP iteration on host cores (bounded sample)."""
    import multiprocessing as mp
    cores = max(1, min(16, os.cpu_count() or 1))   # the GPU box's CPU share is 16
    n_prob = 96 * cores                              # ~10-20 s of oracle work on the box
    from cmpc.synth import make_batch
    pb = make_batch('trot', N, n_prob, seed_offset=777)
    probs = [pb.oracle_problem(b) for b in range(n_prob)]
    t0 = time.perf_counter()
    with mp.get_context('fork').Pool(cores, initializer=_cpu_init) as pool:
        pool.map(_cpu_one_iteration, probs, chunksize=1)
    dt = time.perf_counter() - t0
    return dict(value=n_prob / dt, unit='SCP iterations/s', cores=cores, kind='port',
                sample='%d synthetic Solo12-trot N=%d problems, one SCP iteration each (oracle: numpy '
                       'linearization + reference-order CSC assembly + OSQP-algorithm ADMM eps 1e-7 with '
                       'polish), %d worker processes, %.1f s wall' % (n_prob, N, cores, dt))


def _cpu_init():
    for v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ[v] = '1'


def _cpu_one_iteration(prob):
    from oracle import scp as S
    sp = dict(prob['scp_params']); sp['max_iterations'] = 1
    S.solve_scp(prob, sp, fixed_iters=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--batch', type=int, default=1024, help='problems per GPU')
    ap.add_argument('--N', type=int, default=100)
    ap.add_argument('--config', default='trot')
    ap.add_argument('--precision', default='fp64')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    args = ap.parse_args()

    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local_rank = int(os.environ.get('LOCAL_RANK', 0))

    # the library is loaded before torch so the process has exactly one HIP runtime
    from cmpc._lib import Solver
    from cmpc.synth import make_batch

    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo: barrier and timing reduction only (no data path)
        dist.init_process_group('gloo', rank=rank, world_size=world)

    if args.config == 'mixed':     # BASELINE C5: pace and trot contact plans alternating in one batch
        pb = make_batch('trot', args.N, args.batch, seed_offset=rank * args.batch, mixed=('pace', 'trot'))
    else:
        pb = make_batch(args.config, args.N, args.batch, seed_offset=rank * args.batch)
    solver = Solver(pb.robot, args.N, args.batch, args.precision, device=local_rank)
    solver.upload(pb)
    for _ in range(args.warmup):
        solver.scp_iterate(fixed_iters=True)
    solver.synchronize()

    def barrier():
        solver.synchronize()
        if dist is not None:
            dist.barrier()

    barrier()
    solver.timing_begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solver.scp_iterate(fixed_iters=True)
    solver.synchronize()
    t1 = time.perf_counter()
    tim = solver.timing_end()
    barrier()
    elapsed = t1 - t0
    ipm_total = solver.qp_iterations_total()        # IPM iterations of the last step, all problems
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    units = args.batch * world * args.steps
    value = units / elapsed
    w = 8 if args.precision in ('fp64', 'f64', 'float64') else 4
    qp_mean_s = tim['qp_ms'] / 1e3 / max(tim['iterations'], 1)
    achieved = algorithmic_qp_bytes(args.N, ipm_total, w) / qp_mean_s / 1e9
    traffic = None
    pmc = os.path.join(ROOT, 'profiles', 'qp_pmc_traffic.json')
    metric_config = (args.config, args.N, args.batch, w) == ('trot', 100, 1024, 8)
    if metric_config and os.path.exists(pmc):   # the PMC summary was measured on the metric config only
        try:
            traffic = json.load(open(pmc)).get('hbm_bytes_per_launch')
        except Exception:
            traffic = None
    out = {
        'metric': METRIC,
        'value': value,
        'unit': 'SCP iterations/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64' if w == 8 else 'f32',
        'data': 'synthetic (seeded contact plans + dynamically consistent warm starts, cmpc/synth.py)',
        'config': {'workload': '%s SCP iterations (fixed-K), N=%d, %d problems per GPU'
                               % (WORKLOAD_NAMES.get(args.config, args.config), args.N, args.batch),
                   'config': args.config, 'N': args.N, 'batch_per_gpu': args.batch,
                   'global_batch': args.batch * world, 'parallelism': 'batch-sharded x%d' % world},
        'phase_ms_per_step': {k: tim[k] / max(tim['iterations'], 1)
                              for k in ('linearize_ms', 'assemble_ms', 'qp_ms', 'accept_ms')},
        'qp_ipm_iterations_mean': ipm_total / args.batch,
        'roofline': {'kernel': 'k_qp_ipm', 'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out['cpu_baseline'] = cpu_baseline(args.N)
        except Exception as e:  # the baseline must never hide the GPU number
            out['cpu_baseline'] = {'error': repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    solver.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
