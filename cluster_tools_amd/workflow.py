"""The hot path's two workflows run in-process, without luigi.

``GraphWorkflow`` (graph/graph_workflow.py:22-66) and ``EdgeFeaturesWorkflow``
(features/features_workflow.py:31-57) with ``n_scales=1`` and
``target='local'``: every task's run_impl is restated for the datasets and
attributes it creates, and its jobs -- ``block_list[k::n_jobs]``
(cluster_tasks.py:301-335) -- run the reference's job bodies (the ndist call
sequence) on job threads instead of job processes.  Job threads share the
library (its calls are serialised per device) and overlap their N5 decode.

    InitialSubGraphs   initial_sub_graphs.py:49-90, job :134-157
    MergeSubGraphs     merge_sub_graphs.py:52-96, job :155-195 (complete graph)
    MapEdgeIds         map_edge_ids.py:36-70, job :101-120
    BlockEdgeFeatures  block_edge_features.py:48-87, job :275-327 (_accumulate)
    MergeEdgeFeatures  merge_edge_features.py:35-84, job :110-149

This is what bench.py's ``--config 0`` times (BASELINE configs[0]) and what
the end-to-end GPU test runs; the luigi task classes themselves stay the
reference's.
"""
from __future__ import annotations

import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import ndist
from .blocking import blocks_in_volume


def _jobs(block_list, n_jobs):
    n_jobs = max(1, min(len(block_list), n_jobs))
    return [block_list[k::n_jobs] for k in range(n_jobs)]


def _run_jobs(fn, jobs):
    if len(jobs) == 1:
        fn(jobs[0])
        return
    with ThreadPoolExecutor(len(jobs)) as ex:
        for f in [ex.submit(fn, j) for j in jobs]:
            f.result()


class Timer:
    def __init__(self):
        self.stages = {}

    def stage(self, name):
        timer = self

        class _Ctx:
            def __enter__(self):
                self.t = time.perf_counter()

            def __exit__(self, *a):
                timer.stages[name] = timer.stages.get(name, 0.0) + time.perf_counter() - self.t
        return _Ctx()


def graph_workflow(input_path, input_key, graph_path, output_key, block_shape, max_jobs=16, threads_per_job=16,
                   ignore_label=False, timer=None):
    """GraphWorkflow(n_scales=1): per-block sub-graphs, the merged graph at
    ``output_key``, per-block edge ids."""
    timer = timer or Timer()
    with ndist._open(input_path, 'r') as f:
        shape = list(f[input_key].shape)
    block_list = blocks_in_volume(shape, block_shape)
    with timer.stage('initial_sub_graphs'):
        with ndist._open(graph_path) as f:                      # initial_sub_graphs.py:64-75
            g = f.require_group('s0/sub_graphs')
            g.attrs['shape'] = shape
            g.attrs['ignore_label'] = bool(ignore_label)
            for k in ('nodes', 'edges'):
                g.require_dataset(k, shape=shape, chunks=list(block_shape), compression='gzip', dtype='uint64')

        from .blocking import blocking
        blk = blocking([0, 0, 0], shape, list(block_shape))

        def job(blocks):                                          # initial_sub_graphs.py:134-157
            for b in blocks:
                block = blk.getBlock(b)
                ndist.computeMergeableRegionGraph(input_path, input_key, block.begin, block.end, graph_path,
                                                  's0/sub_graphs', ignore_label, increaseRoi=True,
                                                  serializeToVarlen=True)
        _run_jobs(job, _jobs(block_list, max_jobs))
    with timer.stage('merge_sub_graphs'):
        with ndist._open(graph_path) as f:                      # merge_sub_graphs.py:61-68
            g = f.require_group(output_key)
            g.attrs['ignore_label'] = bool(ignore_label)
            g.attrs['shape'] = shape
        ndist.mergeSubgraphs(graph_path, subgraphKey='s0/sub_graphs', blockIds=block_list, outKey=output_key,
                             numberOfThreads=threads_per_job, serializeToVarlen=False)
        with ndist._open(graph_path) as f:                      # merge_sub_graphs.py:136-137
            f[output_key].attrs['shape'] = shape
    with timer.stage('map_edge_ids'):
        with ndist._open(graph_path) as f:                      # map_edge_ids.py:44-53
            f.require_dataset('s0/sub_graphs/edge_ids', shape=shape, chunks=list(block_shape),
                              compression='gzip', dtype='uint64')
        ndist.mapEdgeIds(graph_path, output_key, subgraphKey='s0/sub_graphs', blockIds=block_list,
                         numberOfThreads=threads_per_job)
    return timer


def edge_features_workflow(input_path, input_key, labels_path, labels_key, graph_path, graph_key, output_path,
                           output_key, block_shape, max_jobs=1, max_jobs_merge=1, threads_per_job=16, offsets=None,
                           timer=None):
    """EdgeFeaturesWorkflow: per-block features into s0/sub_features, merged
    (E, 10) table at ``output_key``."""
    timer = timer or Timer()
    with ndist._open(graph_path, 'r') as f:
        shape = list(f['s0/sub_graphs'].attrs['shape'])
        n_edges = int(f[graph_key].attrs['numberOfEdges'])
    with ndist._open(input_path, 'r') as f:
        ds = f[input_key]
        dtype, ndim = ds.dtype, ds.ndim
    block_list = blocks_in_volume(shape, block_shape)
    with timer.stage('block_edge_features'):
        with ndist._open(output_path) as f:                     # block_edge_features.py:61-64
            ds = f.require_dataset('s0/sub_features', shape=shape, chunks=list(block_shape), compression='gzip',
                                   dtype='float64')
            ds.attrs['n_features'] = 10                           # :321-325

        def job(blocks):                                          # block_edge_features.py:113-148
            if ndim == 3:
                fn = ndist.extractBlockFeaturesFromBoundaryMaps_uint8 if dtype == np.uint8 else \
                    ndist.extractBlockFeaturesFromBoundaryMaps_float32
                fn(graph_path, 's0/sub_graphs', input_path, input_key, labels_path, labels_key, blocks,
                   output_path, 's0/sub_features', increaseRoi=True)
            else:
                fn = ndist.extractBlockFeaturesFromAffinityMaps_uint8 if dtype == np.uint8 else \
                    ndist.extractBlockFeaturesFromAffinityMaps_float32
                fn(graph_path, 's0/sub_graphs', input_path, input_key, labels_path, labels_key, blocks,
                   output_path, 's0/sub_features', offsets)
        _run_jobs(job, _jobs(block_list, max_jobs))
    with timer.stage('merge_edge_features'):
        chunk = min(262144, n_edges)
        with ndist._open(output_path) as f:                     # merge_edge_features.py:62-65
            f.require_dataset(output_key, shape=(n_edges, 10), chunks=(max(1, chunk), 1), compression='gzip',
                              dtype='float64')
        # edge chunks of chunk_size dealt to the merge jobs as consecutive runs
        # (merge_edge_features.py:74-79, cluster_tasks.py:305-329); one
        # mergeFeatureBlocks call per job over its run (:127-147)
        n_chunks = (n_edges + chunk - 1) // max(1, chunk)
        n_jobs = max(1, min(n_chunks, max_jobs_merge))
        per_job = [n_chunks // n_jobs + (1 if j < n_chunks % n_jobs else 0) for j in range(n_jobs)]
        runs, c0 = [], 0
        for n in per_job:
            runs.append((c0 * chunk, min(n_edges, (c0 + n) * chunk)))
            c0 += n

        def mjob(run):
            ndist.mergeFeatureBlocks(graph_path, 's0/sub_graphs', output_path, 's0/sub_features', output_path,
                                     output_key, blockIds=block_list, edgeIdBegin=run[0], edgeIdEnd=run[1],
                                     numberOfThreads=threads_per_job)
        if n_edges:
            _run_jobs(mjob, runs)
    return timer
