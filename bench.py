#!/usr/bin/env python
"""Throughput of the RAG + edge-feature hot path on MI355X.

Metric (BASELINE.json): Gvoxels/s for RAG + boundary edge features, and the
fraction of the HBM roofline.  One *step* = one pass of the hot path over a
resident synthetic volume: face scan (labels uint64 + float32 boundary map in
HBM) -> per-tile edge records -> radix sort -> per-edge reduction -> sorted
(E,2) edge table, node list and (E,10) float64 feature table in HBM.

Default (``--config 2``): BASELINE.json configs[2], the north_star volume --
2048^3 Voronoi supervoxels (cell 16, ~1.6e7 edges) + float32 boundary map,
103 GB resident on one MI355X at N=1.  N>1 (torch.distributed.run, one rank per
GPU): strong scaling of the same fixed volume, rank r owns the z-slab
[2048 r/N, 2048 (r+1)/N) (+1 halo plane below, ``ctg_mgpu_slab``), builds its
partial edge table and the ranks combine them over RCCL
(cluster_tools_amd/dist.py).

The other BASELINE configs are extra lines (``--config``), not the driver's
bench line:
  0    configs[0]: the drop-in per-block path end to end -- GraphWorkflow +
       EdgeFeaturesWorkflow job bodies (harness/workflow.py) on a
       125 x 1250 x 1250 volume in gzip N5 with 64 x 256 x 256 blocks, N5 in ->
       N5 out; value = end-to-end Gvoxels/s with every job its own process
       (the reference's LocalTask model), plus the same with job threads and
       the compute-only rate of the per-block calls on device-resident inputs
  1    configs[1]: 512^3 (cell 10, ~1e6 edges) per GPU; N>1: weak scaling,
       each rank owns a 512^3 z-slab of a (512N)x512x512 volume
  3    configs[3]: 1024^3, 3-channel nearest-neighbour affinities (N=1)
  3lr  configs[3]: 1024^3, 12-channel long-range affinities (N=1)
  4    configs[4]: 1024^3 high fragmentation (cell 5, ~5e7 edges), strong
       scaling like config 2
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak, GB/s (MI355X_MICROARCH.md)
EDGE_BYTES = 96                # 16 B (u,v) + 10 x float64 features


# BASELINE.json configs -> (cube edge, cell size, offsets or None, scaling, label)
WORKLOADS = {
    '0': (1250, 10, None, 'weak', 'BASELINE configs[0]: 125x%dx%d... per-block N5 workflow'),
    '1': (512, 10, None, 'weak', 'BASELINE configs[1]: %d^3 per GPU, cell %d, boundary map'),
    '2': (2048, 16, None, 'strong', 'BASELINE configs[2]: %d^3 boundary map, cell %d, z-slab sharded'),
    '3': (1024, 10, 'nn', 'strong', 'BASELINE configs[3]: %d^3, cell %d, 3-channel nearest-neighbour affinities'),
    '3lr': (1024, 10, 'lr', 'strong', 'BASELINE configs[3]: %d^3, cell %d, 12-channel long-range affinities '
                                      '(whole-volume rule: a sample counts when its pair is an edge of the global '
                                      'RAG; the per-block drop-in applies the block sub-graph rule, DESIGN 3.3)'),
    '4': (1024, 5, None, 'strong', 'BASELINE configs[4]: %d^3 high fragmentation, cell %d, boundary map'),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--config', default='2', choices=sorted(WORKLOADS))
    p.add_argument('--size', type=int, default=None, help='cube edge (voxels; per GPU for weak scaling)')
    p.add_argument('--cell', type=int, default=None)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--cpu-baseline-planes', type=int, default=None,
                   help='z-planes of the volume timed with the C oracle (0 = skip; default: 512 of '
                        'configs[1], 128 of configs[2] = 537 M voxels)')
    p.add_argument('--cpu-threads', type=int, default=min(16, os.cpu_count() or 1),
                   help='worker processes of the CPU baseline (the GPU box allots 16 cores per GPU)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    # rehearsal of the N>1 path on a one-GPU box: every rank on one device,
    # exchange over gloo (the driver's multi-GPU runs use the defaults: RCCL,
    # device = LOCAL_RANK)
    p.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'])
    p.add_argument('--write-output', default=None, metavar='DIR',
                   help='multi-GPU path: after the timed steps, gather the last step\'s shards on rank 0 and write '
                        'graph / features N5 under DIR (dist.write_global, SURVEY 8(e) Output); reported as '
                        '"output" beside the line, outside the timed region')
    p.add_argument('--dist-path', action='store_true',
                   help='run the multi-GPU step (cluster_tools_amd/dist.py: splitters, all_to_all exchange, merge) '
                        'even at WORLD_SIZE 1 -- an RCCL rehearsal on a one-GPU box (launch under torch.distributed.run)')
    p.add_argument('--device', type=int, default=None)
    return p.parse_args()


def pmc_traffic_per_launch(config='1'):
    """HBM bytes per face-scan launch of BASELINE config ``config`` at its
    default size, from the newest committed rocprofv3 PMC summary
    (profiles/*/pmc_summary.json for config 1, pmc_summary_c<config>.json for
    the others; written by tools/pmc_summary.py), the summary's path, and the
    scan's average duration in that summary's kernel trace (ns) -- or Nones."""
    import glob
    name = 'pmc_summary.json' if config == '1' else 'pmc_summary_c%s.json' % config
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', '*', name)))
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
            v = d.get('scan_hbm_bytes_per_launch')
            if v:
                return float(v), os.path.relpath(f, ROOT), d.get('scan_avg_ns')
        except Exception:
            continue
    return None, None, None


def cpu_baseline(labels_t, bnd_t, planes, workers):
    """C oracle (scalar port) on the first ``planes`` z-planes, cut into one
    z-chunk per worker process (each chunk with its halo plane below, faces
    owned by their upper voxel): the reference's target='local' layout of one
    single-threaded nifty job per block on every host core
    (cluster_tasks.py:521,544-547).  Workers are spawned child processes (not
    threads: the C call scales across processes here, not across threads).
    value = voxels / the slowest worker's C-call time (all run at once);
    loading the chunks and merging their tables are not timed."""
    import multiprocessing as mp
    import tempfile
    from concurrent.futures import ProcessPoolExecutor
    from oracle import c_oracle
    lab = labels_t[:planes].cpu().numpy().view(np.uint64)
    bnd = bnd_t[:planes].cpu().numpy()
    workers = max(1, min(workers, planes))
    import shutil
    need = lab.nbytes + bnd.nbytes + (1 << 30)
    tmp = '/dev/shm' if os.path.isdir('/dev/shm') and shutil.disk_usage('/dev/shm').free > need \
        else tempfile.gettempdir()
    d = tempfile.mkdtemp(prefix='ctg_cpu_', dir=tmp)
    lp, dp = os.path.join(d, 'labels.npy'), os.path.join(d, 'data.npy')
    try:
        np.save(lp, lab)
        np.save(dp, bnd)
        z = [planes * i // workers for i in range(workers + 1)]
        jobs = [(lp, dp, z[i], z[i + 1], 1 if z[i] > 0 else 0) for i in range(workers)]
        best = None
        with ProcessPoolExecutor(workers, mp_context=mp.get_context('spawn')) as ex:
            for _ in range(2):
                res = list(ex.map(c_oracle.chunk_job, jobs))
                t = max(r[1] for r in res)
                best = t if best is None else min(best, t)
    finally:
        for f in (lp, dp):
            if os.path.exists(f):
                os.remove(f)
        os.rmdir(d)
    n_edges = sum(r[0] for r in res)
    return lab.size / best / 1e9, dict(
        sample='%dx%dx%d z-slab of the same volume (%d voxels) in %d z-chunks on %d worker processes, '
               '%d chunk edges' % (lab.shape + (lab.size, workers, workers, n_edges)),
        seconds=best, threads=workers)


def _config0_write_inputs(path, shape, block, cell, seed):
    """configs[0] input: the synthetic volume generated on the GPU and written
    as gzip N5 (level 1) -- in a child process, so the bench process itself
    has not touched the device when the process-mode jobs start (the GPU box
    allows 16 processes on the card)."""
    import torch   # before libctg: the library then shares torch's HIP runtime (one runtime per process)
    from cluster_tools_amd import _lib, n5, rag
    torch.cuda.set_device(0)
    _lib.init_device(0)
    lt, bt = rag.synth_volume(shape, cell=cell, seed=seed)
    lab = lt.cpu().numpy().view(np.uint64)
    bnd = bt.cpu().numpy()
    comp = {'type': 'gzip', 'level': 1, 'useZlib': False}
    with n5.File(path) as f:
        for key, arr in (('seg', lab), ('bnd', bnd)):
            ds = f.create_dataset(key, shape=shape, chunks=block, dtype=arr.dtype, compression=comp)
            ds.n_threads = 16
            ds[:] = arr
    return sum(os.path.getsize(os.path.join(r, fn)) for r, _, fs in os.walk(path) for fn in fs)


def cpu_baseline_config0(inp, tmpdir, shape, block, workers):
    """configs[0] CPU baseline: the per-block job bodies (gzip N5 ROI reads,
    RAG + 10 features of every block on the scalar C restatement, varlength
    gzip chunk writes of nodes / edges / sub_features) over the same N5 input,
    one single-threaded job per worker process (blocks dealt k::workers, as
    LocalTask deals them); value = voxels / the slowest job (all at once).  The
    merge tasks (one job each) are not included."""
    import multiprocessing as mp
    import shutil
    from concurrent.futures import ProcessPoolExecutor
    from oracle import c_oracle
    from cluster_tools_amd import n5
    from cluster_tools_amd.blocking import blocking
    nb = blocking([0, 0, 0], list(shape), list(block)).numberOfBlocks
    workers = max(1, min(workers, nb))
    best = None
    for rep in range(2):
        out = os.path.join(tmpdir, 'cpu%d.n5' % rep)
        with n5.File(out) as fo:
            for k in ('s0/sub_graphs/nodes', 's0/sub_graphs/edges'):
                fo.require_dataset(k, shape=list(shape), chunks=list(block), compression='gzip', dtype='uint64')
            fo.require_dataset('s0/sub_features', shape=list(shape), chunks=list(block), compression='gzip',
                               dtype='float64')
        jobs = [(inp, out, list(block), list(range(nb))[k::workers]) for k in range(workers)]
        with ProcessPoolExecutor(workers, mp_context=mp.get_context('spawn')) as ex:
            res = list(ex.map(c_oracle.block_job, jobs))
        shutil.rmtree(out, ignore_errors=True)
        t = max(r[1] for r in res)
        best = t if best is None else min(best, t)
    V = int(np.prod(shape))
    return {'value': round(V / best / 1e9, 6), 'unit': 'Gvoxels/s', 'cores': workers, 'kind': 'port',
            'sample': 'the whole configs[0] volume (%dx%dx%d, %d blocks of %s): per-block job bodies (gzip N5 ROI '
                      'reads, RAG + features on oracle/ctg_oracle.c, varlength gzip writes of nodes / edges / '
                      'sub_features) on %d single-threaded worker processes, %.2f s slowest job (best of 2); '
                      'merge tasks not included' % (tuple(shape) + (nb, 'x'.join(map(str, block)), workers, best))}


# Job processes per task in process mode.  'gpu': one job per task -- each job
# is a GPU process, and creating / tearing down a device context costs ~60 ms
# that the driver serialises across processes (15 graph jobs exit in ~0.9 s),
# while one job runs all 50 blocks in ~0.1 s of device time; 'cpu_layout': the
# job counts of the CPU reference's layout (one job per core: 15 graph jobs,
# the GPU box allows 16 processes on the card), reported beside it.
CONFIG0_PROC_LAYOUTS = {'gpu': dict(graph=1, features=1, merge=1),
                        'cpu_layout': dict(graph=15, features=1, merge=4)}


def bench_config0(args):
    """BASELINE configs[0]: the per-block drop-in path, N5 in -> N5 out.

    Two job models over the same N5 input: ``processes`` (the reference's --
    LocalTask runs every job as its own process, cluster_tasks.py:528-550;
    this is ``value``) and ``threads`` (every job on a thread of this process,
    sharing the device state and the decoded-chunk cache), then the
    device-only time of the same per-block calls."""
    import multiprocessing as mp
    import shutil
    import tempfile
    from concurrent.futures import ProcessPoolExecutor
    # torch's HIP runtime is loaded (not started) before libctg, so the thread-mode
    # and compute-only parts below run libctg and torch on one runtime
    import torch
    from harness import workflow
    shape, block = (125, 1250, 1250), (64, 256, 256)
    V = int(np.prod(shape))
    cell = args.cell or 10
    tmp_root = '/dev/shm' if os.path.isdir('/dev/shm') and shutil.disk_usage('/dev/shm').free > 12e9 else None
    d = tempfile.mkdtemp(prefix='ctg_cfg0_', dir=tmp_root)
    try:
        inp = os.path.join(d, 'in.n5')
        with ProcessPoolExecutor(1, mp_context=mp.get_context('spawn')) as ex:
            in_bytes = ex.submit(_config0_write_inputs, inp, shape, block, cell, args.seed).result()

        def step(k, mode, jobs):
            # every step starts from cold decode caches (thread mode: the bench
            # process's cache would otherwise still hold the input of the last step)
            from cluster_tools_amd import _lib
            _lib.load().ctg_io_cache_clear()
            out = os.path.join(d, 'out%d.n5' % k)
            t = workflow.graph_workflow(inp, 'seg', out, 'graph', block, max_jobs=jobs['graph'], mode=mode)
            workflow.edge_features_workflow(inp, 'bnd', inp, 'seg', out, 'graph', out, 'features', block,
                                            max_jobs=jobs['features'], max_jobs_merge=jobs['merge'], timer=t,
                                            mode=mode)
            from cluster_tools_amd import n5
            with n5.File(out, 'r') as f:
                n_edges = int(f['graph'].attrs['numberOfEdges'])
            for key in ('s0/sub_features', 's0/sub_features_stats', 'features', 's0/sub_graphs'):
                p = os.path.join(out, key)
                out_bytes[key] = sum(os.path.getsize(os.path.join(r, fn)) for r, _, fs in os.walk(p) for fn in fs)
            shutil.rmtree(out)
            return t.stages, n_edges

        out_bytes = {}   # on-disk bytes of the outputs (last step)
        # a step is a whole workflow run (seconds): at most 1 warm-up + 3 steps
        args.warmup, args.steps = min(args.warmup, 1), max(1, min(args.steps, 3))

        def measure(mode, jobs, base):
            for k in range(args.warmup):
                step(base + k, mode, jobs)
            times, stages, feat_prof = [], {}, {}
            from cluster_tools_amd import ndist
            for k in range(args.steps):
                t0 = time.perf_counter()
                st, n_edges = step(base + 100 + k, mode, jobs)
                times.append(time.perf_counter() - t0)
                for key, v in st.items():
                    stages[key] = stages.get(key, 0.0) + v / args.steps
                if mode == 'threads':   # the (single) block-feature job's split, in this process
                    for key, v in ndist.last_profile.items():
                        feat_prof[key] = feat_prof.get(key, 0.0) + v / args.steps
            return float(np.mean(times)) * 1e3, stages, feat_prof, n_edges

        # process mode first: this process has not opened the device yet
        def split():
            out = {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()
                       if kk != 'body_profile_of_slowest'} for k, v in workflow.process_stats.items()}
            out['_block_features_job_profile'] = {
                k: round(v, 4) for k, v in workflow.process_stats.get('_block_features_job', {}).get(
                    'body_profile_of_slowest', {}).items()}
            return out
        ms_p, stages_p, _, n_edges = measure('processes', CONFIG0_PROC_LAYOUTS['gpu'], 0)
        proc_split = split()
        ms_c, stages_c, _, _ = measure('processes', CONFIG0_PROC_LAYOUTS['cpu_layout'], 500)
        proc_split_c = split()
        ms_t, stages_t, feat_prof, _ = measure('threads', dict(graph=16, features=1, merge=4), 1000)

        cpu = None if args.no_cpu_baseline else cpu_baseline_config0(inp, d, shape, block, args.cpu_threads)
        from cluster_tools_amd import _lib, n5, rag
        from cluster_tools_amd.blocking import blocking
        torch.cuda.set_device(0 if args.device is None else args.device)
        _lib.init_device(0 if args.device is None else args.device)
        with n5.File(inp, 'r') as f:
            lt = torch.from_numpy(f['seg'][:].view(np.int64)).cuda()
            bt = torch.from_numpy(f['bnd'][:]).cuda()
        # compute only: the same per-block calls on device-resident inputs
        blk = blocking([0, 0, 0], list(shape), list(block))
        descs, lo = [], 0
        arrays = []
        for b in range(blk.numberOfBlocks):
            bb = blk.getBlock(b)
            rb = [max(x - 1, 0) for x in bb.begin]
            sl = tuple(slice(x, y) for x, y in zip(rb, bb.end))
            shp = [y - x for x, y in zip(rb, bb.end)]
            descs.append(dict(label_offset=lo, data_offset=lo, shape=shp,
                              own=([x - r for x, r in zip(bb.begin, rb)], [y - r for y, r in zip(bb.end, rb)]),
                              graph=([0, 0, 0], shp)))
            arrays.append(sl)
            lo += int(np.prod(shp))
        la = torch.cat([lt[sl].reshape(-1) for sl in arrays])
        da = torch.cat([bt[sl].reshape(-1) for sl in arrays])
        del lt, bt
        rag.set_profiling(True)
        for _ in range(2):
            rag.rag_blocks_arena(la, descs)
            rag.rag_blocks_arena(la, descs, da, keep_stats=True)
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        n_rep = 5
        scan_ms, dev_ms = [], []
        for _ in range(n_rep):
            rag.rag_blocks_arena(la, descs)
            g = rag.last_timings()['total']
            rag.rag_blocks_arena(la, descs, da, keep_stats=True, nodes=False)
            tm = rag.last_timings()
            scan_ms.append(tm['scan'])
            dev_ms.append(g + tm['total'])
        torch.cuda.synchronize()
        wall_s = (time.perf_counter() - c0) / n_rep
        compute_s = float(np.mean(dev_ms)) * 1e-3
        rag.set_profiling(False)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    scan_avg = float(np.mean(scan_ms))
    alg = lo * 12                                   # the feature scan reads every block array (+ halo) once
    traffic, traffic_src, _ = pmc_traffic_per_launch('0') if not args.cell else (None, None, None)
    line = {
        'metric': 'Gvoxels/s RAG+edge features (per-block drop-in path, gzip N5 in -> N5 out, uint64 labels, '
                  'float32 boundary map)',
        'value': round(V / (ms_p * 1e-3) / 1e9, 4), 'unit': 'Gvoxels/s', 'n_gpus': 1, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(ms_p, 2), 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'dtype': 'u64 labels / f32 samples / f64 stats',
        'data': 'synthetic (jittered-grid Voronoi supervoxels + boundary map) written to gzip N5 (level 1)',
        'config': {'workload': 'BASELINE configs[0]: 125x1250x1250, 64x256x256 blocks (50), GraphWorkflow + '
                               'EdgeFeaturesWorkflow job bodies (harness/workflow.py), every job its own spawned '
                               'process as LocalTask runs them, one job per task (max_jobs 1: a GPU job runs all '
                               'blocks of its task)',
                   'volume': list(shape), 'block_shape': list(block), 'edges': n_edges,
                   'input_n5_bytes': in_bytes, 'output_bytes': out_bytes,
                   'stats_compression': os.environ.get('CTG_STATS_COMPRESSION', 'raw')},
        'stage_s': {k: round(v, 4) for k, v in stages_p.items()},
        'process_split_last_step': proc_split,
        'process_mode_cpu_layout': {'value': round(V / (ms_c * 1e-3) / 1e9, 4), 'unit': 'Gvoxels/s',
                                    'ms_per_step': round(ms_c, 2), 'jobs': CONFIG0_PROC_LAYOUTS['cpu_layout'],
                                    'stage_s': {k: round(v, 4) for k, v in stages_c.items()},
                                    'process_split_last_step': proc_split_c,
                                    'what': 'process mode with the job counts of the CPU layout (one graph job '
                                            'per core): every job process creates and tears down a device '
                                            'context'},
        'thread_mode': {'value': round(V / (ms_t * 1e-3) / 1e9, 4), 'unit': 'Gvoxels/s', 'ms_per_step': round(ms_t, 2),
                        'stage_s': {k: round(v, 4) for k, v in stages_t.items()},
                        'block_features_split_s': {k: round(v, 4) for k, v in feat_prof.items()},
                        'what': 'the same workflow with every job on a thread of the bench process (16 graph jobs; '
                                'jobs share the device state and the decoded-chunk cache)'},
        'compute_only': {'value': round(V / compute_s / 1e9, 4), 'unit': 'Gvoxels/s',
                         'ms': round(compute_s * 1e3, 3),
                         'with_d2h_ms': round(wall_s * 1e3, 3),
                         'what': 'device time (HIP events) of the ctg_rag_blocks graph call + feature call over '
                                 'the 50 block arrays (device-resident, halo planes included); with_d2h = wall '
                                 'time including the copies of the per-block results to host memory'},
        'roofline': {'bound': 'hbm', 'kernel': 'k_face_scan (batched blocks, features)',
                     'kernel_ms': round(scan_avg, 4), 'algorithmic_bytes': alg,
                     'achieved': round(alg / (scan_avg * 1e-3) / 1e9, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(alg / (scan_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'traffic_source': traffic_src},
        'cpu_baseline': cpu,
    }
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.config == '0':
        return bench_config0(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.gpus != world and world > 1:
        print('warning: --gpus %d but WORLD_SIZE %d' % (args.gpus, world), file=sys.stderr)
    use_dist = world > 1 or args.dist_path
    dev = local if args.device is None else args.device
    torch.cuda.set_device(dev)
    if use_dist:
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        else:
            dist.init_process_group('gloo')

    from cluster_tools_amd import rag
    from cluster_tools_amd import _lib

    _lib.init_device(dev)
    S0, cell0, aff, scaling, label = WORKLOADS[args.config]
    S = args.size or S0
    cell = args.cell or cell0
    if aff and world > 1:
        raise SystemExit('affinity workloads are single-GPU lines (--gpus 1)')
    if scaling == 'weak':
        gshape = (S * world, S, S)             # S owned planes per rank
    else:
        if S % world:
            raise SystemExit('--size must be divisible by the number of ranks')
        gshape = (S, S, S)
    # rank r owns z in [r*Zr, (r+1)*Zr) and reads the plane(s) below as halo:
    # the slab plan of the C ABI (ctg_mgpu_slab)
    from cluster_tools_amd.dist import slab_plan
    z_read, z_own, z_end = slab_plan(gshape[0], world, rank)
    Zr, halo = z_end - z_own, z_own - z_read
    lab, bnd = rag.synth_volume((Zr + halo, S, S), cell=cell, seed=args.seed, z_offset=z_read,
                                global_shape=gshape)
    own = (halo, 0, 0)
    offsets = None
    data = bnd
    n_ch = 1
    if aff:
        from cluster_tools_amd import synthetic
        offsets = synthetic.NN_OFFSETS if aff == 'nn' else synthetic.LR_OFFSETS
        data = rag.synth_affinities(bnd, offsets)
        n_ch = len(offsets)
        del bnd
        bnd = None
    torch.cuda.synchronize()

    if use_dist:
        from cluster_tools_amd import dist as cdist
        step_fn = lambda: cdist.rag_features_distributed(lab, data, offsets=offsets, own_begin=own)  # noqa: E731
    else:
        step_fn = lambda: rag.rag_features_handle(lab, data, offsets=offsets, own_begin=own)  # noqa: E731

    res = None
    for _ in range(args.warmup):
        if res is not None:
            res.free()
        res = step_fn()
    torch.cuda.synchronize()
    rag.set_profiling(True)
    scan_ms = []
    narrow_ms = 0.0
    if use_dist:
        del cdist.host_reads[:]   # device -> host reads of the exchange, counted over the timed steps
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if res is not None:
            res.free()
        res = step_fn()
        tm = rag.last_timings()
        # long-range affinity calls narrow the labels to u32 before the scan:
        # that pass is part of the roofline kernel time (the scan reads the copy)
        scan_ms.append(tm['scan'] + tm.get('narrow', 0.0))
        narrow_ms = tm.get('narrow', 0.0)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    t1 = time.perf_counter()
    rag.set_profiling(False)
    elapsed = t1 - t0
    if use_dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda' if args.backend == 'nccl' else 'cpu')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    n_edges_local = res.n_edges
    n_rec, n_direct = res.info()
    timings = rag.last_timings()

    V = Zr * S * S                            # owned voxels per rank
    total_vox = V * world
    ms_step = elapsed / args.steps * 1e3
    value = total_vox / (elapsed / args.steps) / 1e9
    n_edges = n_edges_local
    if use_dist:
        te = torch.tensor([n_edges_local], dtype=torch.int64, device='cuda' if args.backend == 'nccl' else 'cpu')
        dist.all_reduce(te)
        n_edges = int(te.item())

    # roofline of the dominant kernel (face scan): algorithmic bytes per launch
    # = voxels it scans x (8 B label + 4 B per channel), halo plane excluded
    scan_avg_ms = float(np.mean(scan_ms))
    vox_bytes = 8 + 4 * n_ch
    scan_bytes = V * vox_bytes
    achieved = scan_bytes / (scan_avg_ms * 1e-3) / 1e9
    traffic, traffic_src, trace_ns = (pmc_traffic_per_launch(args.config)
                                      if not args.size and not args.cell and (scaling == 'weak' or world == 1)
                                      else (None, None, None))
    step_bytes = total_vox * vox_bytes + n_edges * EDGE_BYTES

    output = None
    if use_dist and args.write_output:   # SURVEY 8(e) Output, outside the timed region
        ot = {}
        dist.barrier()
        w = cdist.write_global(res, os.path.join(args.write_output, 'graph.n5'), 'graph',
                               os.path.join(args.write_output, 'features.n5'), 'features', shape=list(gshape),
                               root=0, timings=ot)
        if rank == 0:
            output = {'gather_s': round(ot.get('gather_s', 0.0), 4), 'n5_write_s': round(ot.get('write_s', 0.0), 4),
                      'edges': w[0], 'nodes': w[1], 'path': args.write_output,
                      'what': 'dist.gather_to_host of the last step\'s shards on rank 0, then graph/{nodes,edges} '
                              '+ features N5 datasets as MergeSubGraphs / MergeEdgeFeatures write them'}

    line = None
    if rank == 0:
        cpu = None
        planes = args.cpu_baseline_planes
        if planes is None:
            planes = {'1': 512, '2': 128}.get(args.config, 0)
        if not args.no_cpu_baseline and planes > 0 and world == 1 and args.config in ('1', '2'):
            v, info = cpu_baseline(lab, bnd, min(planes, S), args.cpu_threads)
            cpu = {'value': round(v, 6), 'unit': 'Gvoxels/s', 'cores': info['threads'], 'kind': 'port',
                   'sample': info['sample'] + ', %.2f s slowest worker (best of 2), oracle/ctg_oracle.c scalar C restatement '
                                              '(nifty reference not present on this host)' % info['seconds']}
        line = {
            'metric': 'Gvoxels/s RAG+edge features (%s, uint64 labels, float32)'
                      % ('boundary map' if not aff else '%d-channel affinity map' % n_ch),
            'value': round(value, 4),
            'unit': 'Gvoxels/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms_step, 4),
            'higher_is_better': True,
            'scaling': scaling,
            'vs_baseline': None,
            'dtype': 'u64 labels / f32 samples / f64 stats',
            'data': 'synthetic (jittered-grid Voronoi supervoxels + boundary map, generated in HBM)',
            'config': {'workload': label % (S, cell),
                       'volume': list(gshape), 'edges': n_edges, 'parallelism': 'z-slab x%d' % world,
                       'step': 'dist.rag_features_distributed (%s)' % args.backend if use_dist else 'rag_features'},
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBS, 4),
                         'traffic': traffic,
                         'kernel': 'k_narrow_labels + k_face_scan' if narrow_ms > 0 else 'k_face_scan',
                         'kernel_ms': round(scan_avg_ms, 4), 'algorithmic_bytes': scan_bytes,
                         'traffic_source': traffic_src,
                         # headline 'frac' = this run's HIP events on the scan's stream;
                         # the committed trace (traffic_source's kernel trace) beside it
                         'kernel_ms_trace': round(trace_ns / 1e6, 4) if trace_ns else None,
                         'frac_trace': (round(scan_bytes / (trace_ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
                                        if trace_ns else None),
                         'timing': 'frac: HIP events of this run (scan stream); frac_trace: rocprofv3 kernel trace '
                                   'of the same workload in traffic_source'},
            'step_roofline_frac': round(step_bytes / (ms_step * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4),
            'phase_ms': {k: round(v, 4) for k, v in timings.items()},
            'records': n_rec, 'direct_faces': n_direct,
            'exchange_host_reads_per_step': ({k: cdist.host_reads.count(k) / args.steps for k in sorted(set(
                cdist.host_reads))} if use_dist else None),
            'cpu_baseline': cpu,
        }
        if output is not None:
            line['output'] = output
        print(json.dumps(line), flush=True)
    res.free()
    if use_dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
