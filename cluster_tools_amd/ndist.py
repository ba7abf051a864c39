"""Drop-in mirror of the ``nifty.distributed`` functions on the hot path.

The reference's job bodies do ``import nifty.distributed as ndist`` and call
the functions below with container paths, keys and block ids; each call does
its own N5 I/O and returns None.  This module keeps the names,
argument order/keywords and on-disk effects, and runs the array work through
libctg.so (``cluster_tools_amd.rag``) on the GPU.  Swapping the import is the
whole integration:

    computeMergeableRegionGraph    graph/initial_sub_graphs.py:124-129
    mergeSubgraphs                 graph/merge_sub_graphs.py:130-135, 147-150
    mapEdgeIds                     graph/map_edge_ids.py:116-119
    extractBlockFeaturesFromBoundaryMaps_{float32,uint8}
                                   features/block_edge_features.py:127-134
    extractBlockFeaturesFromAffinityMaps_{float32,uint8}
                                   features/block_edge_features.py:138-145
    mergeFeatureBlocks             features/merge_edge_features.py:141-147
    serializeMergedGraph           multicut/reduce_problem.py:247-258
    Graph                          test/graph/test_graph.py:32,68,111;
                                   multicut/solve_subproblems.py:250

Errors surface as RuntimeError (``_lib.CtgError``), as pybind11 raises for
nifty's C++ exceptions, so a failing job never prints ``processed job N`` and
the reference's retry logic (cluster_tasks.py:114-159) applies unchanged.
"""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import n5
from . import rag
from .blocking import blocking

N_FEATURES = 10
# companion varlen dataset of sub_features (uint32): per edge the shifted sums
# (S1, S2) about a pivot p as 4 words, then the 48 words of the wide statistics
# record (42 histogram slots, count|ADJ, ordered min, ordered max, pivot p as
# float32 bits, 2 zero words) = 208 B (include/ctg.h, ctg_merge_stats)
STATS_SUFFIX = '_stats'
STATS_WORDS = 4 + rag.WIDE_WORDS
ORD_POS_INF = 0xFF800000   # order-preserving u32 code of +inf (ctg_internal.h f2ord)
ORD_NEG_INF = 0x007FFFFF   # ... of -inf


def _open(path, mode='a'):
    return n5.file_reader(path, mode)


def _split_container_path(path):
    """'/data/problem.n5/s0/graph' -> ('/data/problem.n5', 's0/graph'): the
    single-path form of ndist.Graph (ilastik/carving.py:28,
    edges_from_skeletons.py:146) names a group inside a container."""
    p = os.path.abspath(path)
    parts = p.split(os.sep)
    for i in range(len(parts), 0, -1):
        root = os.sep.join(parts[:i]) or os.sep
        if n5.is_container_root(root):
            return root, '/'.join(parts[i:])
    raise ValueError('%s is not inside an N5 / zarr container' % path)


def _map(fn, items, n_threads):
    items = list(items)
    if n_threads and n_threads > 1 and len(items) > 1:
        with ThreadPoolExecutor(int(n_threads)) as ex:
            return list(ex.map(fn, items))
    return [fn(i) for i in items]


def _roi(ds, begin, end):
    return ds[tuple(slice(int(b), int(e)) for b, e in zip(begin, end))]


def _subgraph_blocking(g):
    shape = [int(s) for s in g.attrs.get('shape', g['nodes'].shape)]
    return blocking([0, 0, 0], shape, list(g['nodes'].chunks)), shape


# ---------------------------------------------------------------------------
# graph
# ---------------------------------------------------------------------------

# seconds spent per phase by the last ndist call (read / compute / write);
# bench.py reports the end-to-end split from it
last_profile = {}
_prof_lock = threading.Lock()


def _prof(key, t0):
    with _prof_lock:
        last_profile[key] = last_profile.get(key, 0.0) + time.perf_counter() - t0
    return time.perf_counter()


IO_THREADS = int(os.environ.get('CTG_IO_THREADS', str(min(16, os.cpu_count() or 1))))


def _read_into(ds, box, out, n_threads=None):
    """ROI ``box`` [(b, e), ...] of ``ds`` into the C-contiguous array ``out``
    (native threaded decode straight into the staging buffer when possible)."""
    if ds.dtype.newbyteorder('=') == out.dtype and ds.read_box_native(box, n_threads=n_threads, out=out) is not None:
        return
    out[...] = ds[tuple(slice(b, e) for b, e in box)]


def computeMergeableRegionGraph(labelsPath, labelsKey, roiBegin, roiEnd, graphPath,  # noqa: N802,N803
                                subgraphKey, ignoreLabel, increaseRoi=True, serializeToVarlen=True):  # noqa: N803
    """Per-block sub-graph: sorted unique labels of the inner block (varlen
    ``nodes`` chunk) and the sorted unique (u<v) RAG edges of
    labels[max(begin-1,0):end] (varlen ``edges`` chunk, flattened; no chunk if
    empty), semantics of test_graph.py:42-84.  One ctg_rag_blocks call."""
    if not serializeToVarlen:
        raise NotImplementedError('computeMergeableRegionGraph only serializes to varlen chunks '
                                  '(the only mode the reference uses, initial_sub_graphs.py:129)')
    last_profile.clear()
    t = time.perf_counter()
    roiBegin = [int(b) for b in roiBegin]
    roiEnd = [int(e) for e in roiEnd]
    begin = [max(b - 1, 0) for b in roiBegin] if increaseRoi else list(roiBegin)
    shape = [e - b for b, e in zip(begin, roiEnd)]
    # decoded straight into a page-locked arena from the process pool: a job
    # calls this once per block, and a fresh pageable ROI would be faulted in
    # and staged by the runtime's pageable copy on every call
    nvox = int(np.prod(shape))
    arena = rag.host_arena(nvox * 8)
    try:
        labels = arena.view(np.uint64, nvox).reshape(shape)
        with _open(labelsPath, 'r') as f:
            _read_into(f[labelsKey], list(zip(begin, roiEnd)), labels)
        t = _prof('read', t)
        own = ([b - o for b, o in zip(roiBegin, begin)], [e - o for e, o in zip(roiEnd, begin)])
        res = rag.rag_blocks_arena(labels.reshape(-1), [dict(label_offset=0, shape=shape, own=own,
                                                             graph=([0, 0, 0], shape))],
                                   ignore_label=bool(ignoreLabel))[0]
    finally:
        rag.release_arena(arena)
    t = _prof('compute', t)
    with _open(graphPath) as f:
        g = f[subgraphKey]
        ds_nodes = g['nodes']
        pos = [b // c for b, c in zip(roiBegin, ds_nodes.chunks)]
        ds_nodes.write_chunk(pos, res['nodes'], True)
        if res['edges'].shape[0]:
            g['edges'].write_chunk(pos, res['edges'].ravel(), True)
    _prof('write', t)


def mergeSubgraphs(graphPath, subgraphKey, blockIds, outKey, numberOfThreads=1,  # noqa: N802,N803
                   serializeToVarlen=False):  # noqa: N803
    """Union of block sub-graphs.  serializeToVarlen=False writes the merged
    graph ``outKey/{nodes,edges}`` with attrs numberOfNodes / numberOfEdges
    (merge_sub_graphs.py:127-137); True writes one varlen chunk of the next
    scale's sub-graph dataset (merge_sub_graphs.py:140-152)."""
    with _open(graphPath) as f:
        g = f[subgraphKey]
        blk, shape = _subgraph_blocking(g)
        block_ids = [int(b) for b in blockIds]
        positions = [blk.blockGridPosition(b) for b in block_ids]
        node_list = [n for n in g['nodes'].read_chunks(positions, numberOfThreads) if n is not None and len(n)]
        edge_list = [e.reshape(-1, 2) for e in g['edges'].read_chunks(positions, numberOfThreads)
                     if e is not None and len(e)]
        nodes = np.concatenate(node_list).astype(np.uint64) if node_list else np.zeros(0, np.uint64)
        if nodes.size:
            nodes = rag.unique_labels(nodes.reshape(1, 1, -1))
        if edge_list:
            edges, _ = rag.unique_pairs(np.concatenate(edge_list, axis=0))
        else:
            edges = np.zeros((0, 2), np.uint64)
        if serializeToVarlen:
            # merge_sub_graphs.py:140-152: the old-scale blocks tile one block
            # of the coarser grid; its lower corner is the elementwise minimum
            # of their begins, whatever order the ids come in
            if not block_ids:
                return
            out = f[outKey]
            out_chunks = out['nodes'].chunks
            begins = np.array([blk.getBlock(b).begin for b in block_ids], dtype=np.int64)
            pos = [int(b) // c for b, c in zip(begins.min(axis=0), out_chunks)]
            out['nodes'].write_chunk(pos, nodes, True)
            if edges.shape[0]:
                out['edges'].write_chunk(pos, edges.ravel(), True)
            return
        out = f.require_group(outKey)
        n_nodes, n_edges = int(nodes.shape[0]), int(edges.shape[0])
        ds_n = out.require_dataset('nodes', shape=(n_nodes,), chunks=(max(1, min(n_nodes, 262144)),),
                                   dtype='uint64', compression='gzip')
        ds_e = out.require_dataset('edges', shape=(n_edges, 2), chunks=(max(1, min(n_edges, 262144)), 2),
                                   dtype='uint64', compression='gzip')
        ds_n.n_threads = ds_e.n_threads = max(1, int(numberOfThreads))
        if n_nodes:
            ds_n[:] = nodes
        if n_edges:
            ds_e[:] = edges
        out.attrs['numberOfNodes'] = n_nodes
        out.attrs['numberOfEdges'] = n_edges


def serializeMergedGraph(graphPath, graphBlockPrefix, shape, blockShape, newBlockShape, newBlockIds,  # noqa: N802,N803
                         nodeLabeling, edgeLabeling, outPath, graphOutPrefix, numberOfThreads=1,  # noqa: N803
                         serializeEdges=True):  # noqa: N803
    """Sub-graphs of the next (coarser) scale of the blockwise multicut
    (multicut/reduce_problem.py:247-258, lifted_multicut/reduce_lifted_problem.py:256).

    For every new block: the old-scale blocks inside it (``blockShape`` grid
    under ``graphBlockPrefix``) are united, their nodes mapped through
    ``nodeLabeling`` (dense, old node id -> new node id, reduce_problem.py:165-193)
    and written as the sorted unique varlen ``nodes`` chunk of
    ``graphOutPrefix`` at the new block's grid position -- the chunk
    solve_subproblems.py:135-136 reads at the next scale.  With
    ``serializeEdges`` the old block edges are mapped the same way, edges that
    collapse to one node are dropped, and the sorted unique ``edges`` chunk
    (flattened (u, v)) is written, plus ``edge_ids`` = ``edgeLabeling`` of the
    old global ids when the old scale has ``edge_ids`` chunks.  The reference
    only calls this with serializeEdges=False; the edge branch follows the
    same rule and is parity unpinned (nifty is not available).
    """
    node_lab = np.asarray(nodeLabeling, dtype=np.uint64)
    edge_lab = None if edgeLabeling is None else np.asarray(edgeLabeling, dtype=np.uint64)
    shape = [int(s) for s in shape]
    old_blk = blocking([0, 0, 0], shape, [int(b) for b in blockShape])
    new_blk = blocking([0, 0, 0], shape, [int(b) for b in newBlockShape])
    with _open(graphPath) as fi, _open(outPath) as fo:
        gi = fi[graphBlockPrefix]
        go = fo.require_group(graphOutPrefix)
        go.attrs['shape'] = shape
        keys = ('nodes', 'edges', 'edge_ids') if serializeEdges else ('nodes',)
        for k in keys:
            go.require_dataset(k, shape=shape, chunks=[int(b) for b in newBlockShape], dtype='uint64',
                               compression='gzip')
        has_ids = serializeEdges and edge_lab is not None and 'edge_ids' in gi

        def read(bid):   # N5 reads in the thread pool; library calls stay on this thread
            nb = new_blk.getBlock(int(bid))
            old_ids = old_blk.getBlockIdsOverlappingBoundingBox(nb.begin, nb.end)
            nodes, pairs, ids = [], [], []
            for ob in old_ids:
                opos = old_blk.blockGridPosition(int(ob))
                n = gi['nodes'].read_chunk(opos)
                if n is not None and len(n):
                    nodes.append(node_lab[n.astype(np.int64)])
                if serializeEdges:
                    e = gi['edges'].read_chunk(opos)
                    if e is not None and len(e):
                        pairs.append(node_lab[e.reshape(-1, 2).astype(np.int64)])
                        if has_ids:
                            ids.append(edge_lab[gi['edge_ids'].read_chunk(opos).astype(np.int64)])
            return new_blk.blockGridPosition(int(bid)), nodes, pairs, ids

        for pos, nodes, pairs, ids in _map(read, newBlockIds, numberOfThreads):
            if not nodes:
                continue
            go['nodes'].write_chunk(pos, rag.unique_labels(np.concatenate(nodes).reshape(1, 1, -1)), True)
            if not pairs:
                continue
            uv = np.concatenate(pairs)
            keep = uv[:, 0] != uv[:, 1]
            uv = np.sort(uv[keep], axis=1)
            if uv.shape[0] == 0:
                continue
            edges, _ = rag.unique_pairs(uv)
            go['edges'].write_chunk(pos, edges.ravel(), True)
            if has_ids:
                out_ids = np.zeros(edges.shape[0], dtype=np.uint64)
                out_ids[rag.map_edge_ids(edges, uv)] = np.concatenate(ids)[keep]
                go['edge_ids'].write_chunk(pos, out_ids, True)


def mapEdgeIds(graphPath, graphKey, subgraphKey, blockIds, numberOfThreads=1):  # noqa: N802,N803
    """Per block: global edge id of every local edge (varlen uint64
    ``edge_ids`` chunk), = full_graph.findEdges(uv) (test_graph.py:89-93)."""
    with _open(graphPath) as f:
        global_edges = f[graphKey]['edges'][:]
        g = f[subgraphKey]
        blk, _ = _subgraph_blocking(g)
        block_ids = [int(b) for b in blockIds]
        chunks = g['edges'].read_chunks([blk.blockGridPosition(b) for b in block_ids], numberOfThreads)
        have = [(b, c.reshape(-1, 2)) for b, c in zip(block_ids, chunks) if c is not None and c.size]
        if not have:
            return
        query = np.concatenate([c for _, c in have], axis=0)
        ids = rag.map_edge_ids(global_edges, query)
        if (ids < 0).any():
            raise RuntimeError('mapEdgeIds: %d sub-graph edges are missing from the merged graph'
                               % int((ids < 0).sum()))
        ds = g['edge_ids']
        off = 0
        positions, datas = [], []
        for b, c in have:
            positions.append(blk.blockGridPosition(b))
            datas.append(ids[off:off + c.shape[0]].astype(np.uint64))
            off += c.shape[0]
        ds.write_chunks(positions, datas, varlen=True, n_threads=numberOfThreads)


class Graph:
    """ndist.Graph: a graph over arbitrary uint64 node ids.

    Constructor forms used by the reference and its consumers:
      Graph(edges)                          test_graph.py:68, block_edge_features.py:187
      Graph(path, key[, numberOfThreads=n]) test_graph.py:32,111, solve_subproblems.py:250
      Graph(path_with_key)                  ilastik/carving.py:28
      Graph(path_with_key, n_threads)       edges_from_skeletons.py:146
    numberOfNodes is the count of distinct nodes: a block sub-graph may have
    fewer nodes than gridRag's max+1 (test_graph.py:78-80), and the scale-0
    consumer sizes its node arrays by len(nodes) (reduce_problem.py:322-326).
    For the dense 0..max labels of the reference's test data this equals
    seg.max()+1 (test_graph.py:113).
    """

    def __init__(self, *args, numberOfThreads=1):  # noqa: N803
        nodes = None
        if len(args) == 1 and not isinstance(args[0], (str, os.PathLike)):
            edges = np.asarray(args[0], dtype=np.uint64).reshape(-1, 2)
        elif 1 <= len(args) <= 3 and isinstance(args[0], (str, os.PathLike)):
            if len(args) >= 2 and isinstance(args[1], str):
                path, key = str(args[0]), args[1]
                rest = args[2:]
            else:
                path, key = _split_container_path(str(args[0]))
                rest = args[1:]
            if rest:
                numberOfThreads = int(rest[0])  # noqa: N806
            with _open(path, 'r') as f:
                g = f[key] if key else f
                if 'edges' in g:
                    ds = g['edges']
                    ds.n_threads = max(1, int(numberOfThreads))
                    edges = ds[:]
                else:
                    edges = np.zeros((0, 2), np.uint64)
                if 'nodes' in g:
                    ds = g['nodes']
                    ds.n_threads = max(1, int(numberOfThreads))
                    nodes = ds[:]
        else:
            raise TypeError('Graph(edges), Graph(path, key[, numberOfThreads]) or Graph(path_with_key[, n_threads])')
        self._uv = np.ascontiguousarray(edges.reshape(-1, 2).astype(np.uint64))
        self._nodes = np.unique(self._uv) if nodes is None else np.asarray(nodes, dtype=np.uint64)
        self._sorted = None

    @property
    def numberOfNodes(self):  # noqa: N802
        return int(self._nodes.shape[0])

    @property
    def numberOfEdges(self):  # noqa: N802
        return int(self._uv.shape[0])

    @property
    def maxNodeId(self):  # noqa: N802
        return int(self._nodes.max()) if self._nodes.size else 0

    @property
    def maxEdgeId(self):  # noqa: N802
        return self.numberOfEdges - 1

    def uvIds(self):  # noqa: N802
        return self._uv

    def nodes(self):
        return self._nodes

    def findEdges(self, uv):  # noqa: N802
        uv = np.asarray(uv, dtype=np.uint64).reshape(-1, 2)
        if self._sorted is None:
            order = np.lexsort((self._uv[:, 1], self._uv[:, 0]))
            self._sorted = (order, np.ascontiguousarray(self._uv[order]))
        order, srt = self._sorted
        pos = rag.map_edge_ids(srt, uv)
        return np.where(pos >= 0, order[np.maximum(pos, 0)], -1).astype(np.int64)

    def findEdge(self, u, v):  # noqa: N802
        return int(self.findEdges(np.array([[u, v]], dtype=np.uint64))[0])

    def extractSubgraphFromNodes(self, nodes, allowInvalidNodes=False):  # noqa: N802,N803
        """(inner_edges, outer_edges): ids of the edges with both / exactly one
        endpoint in ``nodes`` (multicut/solve_subproblems.py:154,
        lifted_multicut/solve_lifted_subproblems.py:170), ascending.  Without
        allowInvalidNodes a node id that is not in the graph raises, as nifty
        does."""
        nodes = np.asarray(nodes, dtype=np.uint64).reshape(-1)
        if not allowInvalidNodes and nodes.size:
            known = np.isin(nodes, self._nodes)
            if not known.all():
                raise RuntimeError('extractSubgraphFromNodes: node %d is not in the graph'
                                   % int(nodes[~known][0]))
        in_u = np.isin(self._uv[:, 0], nodes)
        in_v = np.isin(self._uv[:, 1], nodes)
        inner = np.flatnonzero(in_u & in_v).astype(np.int64)
        outer = np.flatnonzero(in_u ^ in_v).astype(np.int64)
        return inner, outer

    def flattenedNeighborhoods(self):  # noqa: N802
        """The node part of vigra's AdjacencyListGraph serialisation, as
        ilastik/carving.py:43 consumes it: for every node in ascending id
        order its degree, then (neighbour id, edge id) per neighbour in
        ascending neighbour order.  (Format restated from vigra's
        adjacency_list_graph.hxx serialize; no reference fixture pins it.)"""
        uv = self._uv
        E = uv.shape[0]
        eid = np.arange(E, dtype=np.uint64)
        # both directions of every edge, sorted by (node, neighbour)
        a = np.concatenate([uv[:, 0], uv[:, 1]])
        b = np.concatenate([uv[:, 1], uv[:, 0]])
        e = np.concatenate([eid, eid])
        order = np.lexsort((b, a))
        a, b, e = a[order], b[order], e[order]
        nodes = self._nodes
        deg = np.zeros(nodes.shape[0], dtype=np.uint64)
        if E:
            idx = np.searchsorted(nodes, a)
            np.add.at(deg, idx, 1)
        out = np.empty(nodes.shape[0] + 2 * a.shape[0], dtype=np.uint64)
        # layout: for node k at offset off[k]: deg, then 2*deg entries
        off = np.zeros(nodes.shape[0], dtype=np.int64)
        if nodes.shape[0] > 1:
            off[1:] = np.cumsum(1 + 2 * deg[:-1].astype(np.int64))
        out[off] = deg
        if E:
            start = np.repeat(off + 1, deg.astype(np.int64))
            rank = np.arange(a.shape[0]) - np.repeat(np.cumsum(deg.astype(np.int64)) - deg.astype(np.int64),
                                                     deg.astype(np.int64))
            out[start + 2 * rank] = b
            out[start + 2 * rank + 1] = e
        return out


# ---------------------------------------------------------------------------
# features
# ---------------------------------------------------------------------------

# the statistics companion is the library's own intermediate (written by the
# block jobs, read once by the merge jobs): uncompressed by default -- gzip,
# even at level 1, made its write the slowest part of the per-block feature
# stage (0.2 s of 0.62 s on configs[0]) and its decode the bulk of the merge
# read; CTG_STATS_COMPRESSION=gzip trades that time for ~3x less disk
STATS_COMPRESSION = os.environ.get('CTG_STATS_COMPRESSION', 'raw')


def _stats_dataset(fo, outKey, shape, chunks):  # noqa: N803
    comp = {'type': 'gzip', 'level': 1, 'useZlib': False} if STATS_COMPRESSION == 'gzip' else 'raw'
    return fo.require_dataset(outKey + STATS_SUFFIX, shape=shape, chunks=chunks, dtype='uint32',
                              compression=comp)


# A block's companion rows come in one of two widths, told apart by the chunk's
# element count over its edge count: STATS_WORDS (the sums + the 48-word wide
# record) or, when every histogram slot of the block fits 16 bits and the pad
# words are zero (always, for rows this library writes), STATS_WORDS_COMPACT:
# the sums, the 42 slots as u16 pairs, count|ADJ, min, max, pivot -- 116
# instead of 208 bytes per edge.
STATS_WORDS_COMPACT = 4 + rag.NSLOTS // 2 + 4


def encode_stats_words(sums, records, compact=True):
    """(E,2) float64 sums + (E,48) uint32 records -> (E,52) uint32 words, or
    (E,29) when the block's histograms fit 16-bit slots (``compact``)."""
    n = records.shape[0]
    recs = np.asarray(records, dtype=np.uint32).reshape(n, rag.WIDE_WORDS)
    sw = np.ascontiguousarray(sums, dtype=np.float64).view(np.uint32).reshape(n, 4)
    ns = rag.NSLOTS
    if compact and n and int(recs[:, :ns].max()) <= 0xFFFF and not recs[:, ns + 4:].any():
        out = np.empty((n, STATS_WORDS_COMPACT), dtype=np.uint32)
        out[:, :4] = sw
        out[:, 4:4 + ns // 2] = recs[:, 0:ns:2] | (recs[:, 1:ns:2] << np.uint32(16))
        out[:, 4 + ns // 2:] = recs[:, ns:ns + 4]
        return out
    out = np.empty((n, STATS_WORDS), dtype=np.uint32)
    out[:, :4] = sw
    out[:, 4:] = recs
    return out


def decode_stats_words(words, n_rows=None):
    """Inverse of encode_stats_words: (sums (E,2) f64, records (E,48) u32); the
    row width comes from the word count over ``n_rows`` (default: full rows)."""
    w = np.ascontiguousarray(words, dtype=np.uint32).ravel()
    width = STATS_WORDS if n_rows is None else (w.size // max(int(n_rows), 1) if n_rows else STATS_WORDS)
    if width not in (STATS_WORDS, STATS_WORDS_COMPACT) or (n_rows is not None and w.size != width * int(n_rows)):
        raise RuntimeError('statistics companion: %d words for %s rows' % (w.size, n_rows))
    w = w.reshape(-1, width)
    sums = np.ascontiguousarray(w[:, :4]).view(np.float64).reshape(-1, 2)
    if width == STATS_WORDS:
        return sums, np.ascontiguousarray(w[:, 4:])
    ns = rag.NSLOTS
    recs = np.zeros((w.shape[0], rag.WIDE_WORDS), dtype=np.uint32)
    h = w[:, 4:4 + ns // 2]
    recs[:, 0:ns:2] = h & np.uint32(0xFFFF)
    recs[:, 1:ns:2] = h >> np.uint32(16)
    recs[:, ns:ns + 4] = w[:, 4 + ns // 2:]
    return sums, recs


def _write_block_features(fo, outKey, pos, shape, chunks, feats, sums, records):  # noqa: N803
    fo[outKey].write_chunk(pos, feats.ravel(), True)
    _stats_dataset(fo, outKey, shape, chunks).write_chunk(pos, encode_stats_words(sums, records).ravel(), True)


# bytes of decoded input (labels + data) staged per ctg_rag_blocks call
# (512 MB: the two page-locked arenas a job pins cost ~0.2 s per GB to pin and
# again to release at process exit; a one-job process of configs[0] spent 0.94
# s pinning 2 GB batches, 0.30 s with 512 MB ones, at equal thread-mode time)
BATCH_BYTES = int(os.environ.get('CTG_BLOCK_BATCH_BYTES', str(512 << 20)))


def _batches(items, sizes, limit):
    out, cur, acc = [], [], 0
    for it, sz in zip(items, sizes):
        if cur and acc + sz > limit:
            out.append(cur)
            cur, acc = [], 0
        cur.append(it)
        acc += sz
    if cur:
        out.append(cur)
    return out


def _block_features(graphPath, subgraphKey, dataPath, dataKey, labelsPath, labelsKey, blockIds,  # noqa: N803
                    outPath, outKey, halo_lo, halo_hi, offsets, increaseRoi, data_dtype):  # noqa: N803
    """The job's blocks in batches of one ctg_rag_blocks call each: the ROIs
    (block + halo) are decoded straight into a page-locked arena while the
    previous batch runs on the GPU; per block the features of its stored
    sub-graph edges (rows in the order of the ``edges`` chunk) and the
    statistics companion are written as varlength chunks."""
    last_profile.clear()
    t = time.perf_counter()
    with _open(graphPath, 'r') as fg:
        g = fg[subgraphKey]
        blk, shape = _subgraph_blocking(g)
        ignore = bool(g.attrs.get('ignore_label', False))
        chunks = g['nodes'].chunks
        block_ids = [int(b) for b in blockIds]
        stored = g['edges'].read_chunks([blk.blockGridPosition(b) for b in block_ids])
    todo = [(b, e.reshape(-1, 2)) for b, e in zip(block_ids, stored) if e is not None]
    t = _prof('read', t)
    if not todo:
        return
    n_ch = 0 if offsets is None else len(offsets)
    lo = halo_lo if increaseRoi else [0, 0, 0]
    geo = []
    for b, eb in todo:
        block = blk.getBlock(b)
        rb = [max(x - h, 0) for x, h in zip(block.begin, lo)]
        re_ = [min(y + h, s_) for y, h, s_ in zip(block.end, halo_hi, shape)]
        gb = [max(x - 1, 0) for x in block.begin] if increaseRoi else list(block.begin)
        geo.append(dict(bid=b, edges=eb, rb=rb, re=re_, pos=blk.blockGridPosition(b),
                        shape=[y - x for x, y in zip(rb, re_)],
                        own=([x - r for x, r in zip(block.begin, rb)], [y - r for y, r in zip(block.end, rb)]),
                        graph=([x - r for x, r in zip(gb, rb)], [y - r for y, r in zip(block.end, rb)])))
    vox = [int(np.prod(x['shape'])) for x in geo]
    per_voxel = 8 + max(1, n_ch) * data_dtype.itemsize
    batches = _batches(list(range(len(geo))), [v * per_voxel for v in vox], BATCH_BYTES)
    max_vox = max(sum(vox[i] for i in bt) for bt in batches)
    # the first arena pair now; the second (double buffering) is pinned by the
    # reader thread while batch 0 runs on the GPU (pinning costs ~0.2 s/GB,
    # a large share of a short-lived job process)
    arena_bytes = (max_vox * 8, max_vox * max(1, n_ch) * data_dtype.itemsize)
    arenas = [(rag.host_arena(arena_bytes[0]), rag.host_arena(arena_bytes[1]))]
    _prof('setup', t)
    try:
        _block_batches(batches, arenas, arena_bytes, geo, vox, n_ch, data_dtype, dataPath, dataKey, labelsPath,
                       labelsKey, outPath, outKey, shape, chunks, offsets, ignore)
    finally:
        for pair in arenas:
            for a in pair:
                rag.release_arena(a)


def _block_batches(batches, arenas, arena_bytes, geo, vox, n_ch, data_dtype, dataPath, dataKey, labelsPath,  # noqa: N803
                   labelsKey, outPath, outKey, shape, chunks, offsets, ignore):  # noqa: N803

    with _open(dataPath, 'r') as fd, _open(labelsPath, 'r') as fl, _open(outPath) as fo:
        ds_data, ds_lab = fd[dataKey], fl[labelsKey]
        ds_out = fo[outKey]
        ds_st = _stats_dataset(fo, outKey, shape, chunks)

        def load(k):
            """decode batch k into arena k % 2 -> (label arena, data arena, descriptors)"""
            t0 = time.perf_counter()
            if k % 2 == len(arenas):
                arenas.append((rag.host_arena(arena_bytes[0]), rag.host_arena(arena_bytes[1])))
            la, da = arenas[k % 2]
            descs, reads, lo_, do_ = [], [], 0, 0
            for i in batches[k]:
                x = geo[i]
                v = vox[i]
                box = list(zip(x['rb'], x['re']))
                reads.append((ds_lab, box, la.view(np.uint64, v, lo_ * 8).reshape(x['shape'])))
                if n_ch:
                    dv = da.view(data_dtype, v * n_ch, do_ * data_dtype.itemsize).reshape([n_ch] + x['shape'])
                    reads.append((ds_data, [(0, n_ch)] + box, dv))
                else:
                    reads.append((ds_data, box, da.view(data_dtype, v, do_ * data_dtype.itemsize).reshape(x['shape'])))
                descs.append(dict(label_offset=lo_, data_offset=do_, shape=x['shape'], own=x['own'],
                                  graph=x['graph']))
                lo_ += v
                do_ += v * max(1, n_ch)
            # every ROI of the batch decoded at once (each over its chunks)
            list(io.map(lambda r: _read_into(r[0], r[1], r[2], 2), reads))
            _prof('load_thread', t0)
            return la.view(np.uint64, lo_), da.view(data_dtype, do_), descs

        def write(k, results):
            t0 = time.perf_counter()
            pos, feats, words = [], [], []
            for i, res in zip(batches[k], results):
                x = geo[i]
                eb = x['edges']
                if np.array_equal(res['edges'], eb):
                    f, sm, rc = res['features'], res['sums'], res['records']
                else:   # stored sub-graph from elsewhere: rows follow the stored edges
                    rows = rag.map_edge_ids(res['edges'], eb) if res['edges'].shape[0] else \
                        np.full(eb.shape[0], -1, np.int64)
                    hit = rows >= 0
                    f = np.zeros((eb.shape[0], N_FEATURES))
                    sm = np.zeros((eb.shape[0], 2))
                    rc = np.zeros((eb.shape[0], rag.WIDE_WORDS), np.uint32)
                    rc[:, 43] = ORD_POS_INF   # identities of the merge for edges without samples
                    rc[:, 44] = ORD_NEG_INF
                    f[hit], sm[hit], rc[hit] = res['features'][rows[hit]], res['sums'][rows[hit]], \
                        res['records'][rows[hit]]
                pos.append(x['pos'])
                feats.append(f.ravel())
                words.append(encode_stats_words(sm, rc).ravel())
            t0 = _prof('write_encode_thread', t0)
            ds_out.write_chunks(pos, feats, varlen=True)
            t0 = _prof('write_features_thread', t0)
            ds_st.write_chunks(pos, words, varlen=True)
            _prof('write_stats_thread', t0)

        with ThreadPoolExecutor(1) as reader, ThreadPoolExecutor(1) as writer, \
                ThreadPoolExecutor(max(1, IO_THREADS // 2)) as io:
            nxt = reader.submit(load, 0)
            pending = None
            for k in range(len(batches)):
                t = time.perf_counter()
                la, da, descs = nxt.result()
                _prof('read_wait', t)
                if k + 1 < len(batches):   # arena (k+1) % 2 held batch k-1, whose GPU call has returned
                    nxt = reader.submit(load, k + 1)
                t = time.perf_counter()
                results = rag.rag_blocks_arena(la, descs, da, offsets=offsets, ignore_label=ignore,
                                               keep_stats=True, nodes=False)
                t = _prof('compute', t)
                if pending is not None:
                    pending.result()
                    _prof('write_wait', t)
                pending = writer.submit(write, k, results)
            if pending is not None:
                t = time.perf_counter()
                pending.result()
                _prof('write_wait', t)


def extractBlockFeaturesFromBoundaryMaps_float32(graphPath, subgraphKey, dataPath, dataKey,  # noqa: N802,N803
                                                 labelsPath, labelsKey, blockIds, outPath, outKey,  # noqa: N803
                                                 increaseRoi=True):  # noqa: N803
    """Per-block 10 edge features of the block's sub-graph edges from a float32
    boundary map; every face counted once globally (owned by the block holding
    its upper voxel), both voxel values are samples."""
    _block_features(graphPath, subgraphKey, dataPath, dataKey, labelsPath, labelsKey, blockIds, outPath,
                    outKey, [1, 1, 1], [0, 0, 0], None, increaseRoi, np.dtype(np.float32))


def extractBlockFeaturesFromBoundaryMaps_uint8(graphPath, subgraphKey, dataPath, dataKey,  # noqa: N802,N803
                                               labelsPath, labelsKey, blockIds, outPath, outKey,  # noqa: N803
                                               increaseRoi=True):  # noqa: N803
    """uint8 boundary maps: samples are value/255 (SURVEY OPEN-7)."""
    _block_features(graphPath, subgraphKey, dataPath, dataKey, labelsPath, labelsKey, blockIds, outPath,
                    outKey, [1, 1, 1], [0, 0, 0], None, increaseRoi, np.dtype(np.uint8))


def extractBlockFeaturesFromAffinityMaps_float32(graphPath, subgraphKey, dataPath, dataKey,  # noqa: N802,N803
                                                 labelsPath, labelsKey, blockIds, outPath, outKey,  # noqa: N803
                                                 offsets):
    """Per-block features from channel-first affinities: sample aff[c,p] for
    every p in the block with L[p] != L[p+o_c] and (min,max) an edge of the
    block's sub-graph."""
    off = np.asarray(offsets, dtype=np.int64).reshape(-1, 3)
    halo_lo = [max(1, int(max(0, -off[:, a].min()))) for a in range(3)]
    halo_hi = [int(max(0, off[:, a].max())) for a in range(3)]
    _block_features(graphPath, subgraphKey, dataPath, dataKey, labelsPath, labelsKey, blockIds, outPath,
                    outKey, halo_lo, halo_hi, off.tolist(), True, np.dtype(np.float32))


def extractBlockFeaturesFromAffinityMaps_uint8(graphPath, subgraphKey, dataPath, dataKey,  # noqa: N802,N803
                                               labelsPath, labelsKey, blockIds, outPath, outKey,  # noqa: N803
                                               offsets):
    """uint8 affinities: samples are value/255 (SURVEY OPEN-7)."""
    off = np.asarray(offsets, dtype=np.int64).reshape(-1, 3)
    halo_lo = [max(1, int(max(0, -off[:, a].min()))) for a in range(3)]
    halo_hi = [int(max(0, off[:, a].max())) for a in range(3)]
    _block_features(graphPath, subgraphKey, dataPath, dataKey, labelsPath, labelsKey, blockIds, outPath,
                    outKey, halo_lo, halo_hi, off.tolist(), True, np.dtype(np.uint8))


def accumulateInput(graph, input, labels, ignoreLabel, withSize, minVal, maxVal):  # noqa: N802,N803,A002
    """ndist.accumulateInput (features/block_edge_features.py:159-168): the
    per-edge statistics of a filter response over the faces of ``labels``
    (both voxels of every boundary face, as the boundary-map features), for
    the edges of ``graph`` in its uvIds order.  Histogram range [minVal,
    maxVal] (the response's own min / max at the call site); columns mean,
    var, min, q10, q25, q50, q75, q90, max (+ count when ``withSize``); an
    edge of the graph with no face in ``labels`` gets a zero row.  One GPU
    face scan (libctg.so) per call.  Column set and empty-edge rows: nifty's
    accumulateInput is not in the image -- parity unpinned."""
    uv = graph.uvIds() if hasattr(graph, 'uvIds') else np.asarray(graph, dtype=np.uint64).reshape(-1, 2)
    uv = np.asarray(uv, dtype=np.uint64).reshape(-1, 2)
    lab = np.ascontiguousarray(np.asarray(labels, dtype=np.uint64))
    x = np.ascontiguousarray(np.asarray(input, dtype=np.float32))
    if lab.shape != x.shape:
        raise RuntimeError('accumulateInput: input shape %s != labels shape %s' % (x.shape, lab.shape))
    lo, hi = float(minVal), float(maxVal)
    if not hi > lo:                      # constant response: a unit range keeps the binning defined
        hi = lo + 1.0
    n_cols = N_FEATURES if withSize else N_FEATURES - 1
    out = np.zeros((uv.shape[0], n_cols), dtype=np.float64)
    if uv.shape[0] == 0 or lab.size == 0:
        return out
    r = rag.rag_features(lab, x, ignore_label=bool(ignoreLabel), hist_range=(lo, hi))
    if r['edges'].shape[0]:
        pos = rag.map_edge_ids(r['edges'], uv)
        hit = pos >= 0
        out[hit] = r['features'][pos[hit], :n_cols]
    return out


# mergeFeatureBlocks jobs of one workflow each read every block's edge_ids and
# feature chunks (merge_edge_features.py:127-147: the job's edge range is
# selected after reading).  Job threads that run at the same time share one
# decode: an entry lives only while a call that asked for it is still reading
# (a later call reads the files again), and its key carries every chunk file's
# (mtime, size).
_merge_cache = {}
_merge_cache_lock = threading.Lock()


def _chunk_stamp(ds, positions):
    out = []
    for pos in positions:
        try:
            st = os.stat(ds._chunk_path(pos))
            out.append((st.st_mtime_ns, st.st_size))
        except OSError:
            out.append(None)
    return tuple(out)


def _read_blocks_shared(ds_ids, ds_feat, positions, n_threads):
    pos_key = tuple(tuple(int(x) for x in p) for p in positions)
    key = (ds_ids.path, ds_feat.path, pos_key, _chunk_stamp(ds_ids, positions), _chunk_stamp(ds_feat, positions))
    with _merge_cache_lock:
        ent = _merge_cache.get(key)
        owner = ent is None
        if owner:
            ent = {'ev': threading.Event(), 'val': None, 'err': None, 'users': 0}
            _merge_cache[key] = ent
        ent['users'] += 1
    try:
        if owner:
            try:
                ent['val'] = (ds_ids.read_chunks(positions, n_threads), ds_feat.read_chunks(positions, n_threads))
            except Exception as e:   # every waiter re-raises
                ent['err'] = e
            finally:
                ent['ev'].set()
        else:
            ent['ev'].wait()
        if ent['err'] is not None:
            raise ent['err']
        return ent['val']
    finally:
        with _merge_cache_lock:
            ent['users'] -= 1
            if ent['users'] == 0 and _merge_cache.get(key) is ent:
                del _merge_cache[key]


def mergeFeatureBlocks(graphPath, subgraphKey, featuresPath, featuresKey, outPath, outKey,  # noqa: N802,N803
                       blockIds, edgeIdBegin, edgeIdEnd, numberOfThreads=1):  # noqa: N803
    """Combine the per-block feature rows of edges in [edgeIdBegin, edgeIdEnd)
    into rows of the (E, n_features) ``outKey`` dataset (10 columns, or
    9 k + 1 for the filter-feature branch).

    Blocks written by this library carry the mergeable statistics in the
    ``<featuresKey>_stats`` companion (uint32, 52 words per edge): counts and
    sums add, min/max elementwise, histograms add, and the quantiles are those
    of the merged histogram -- identical to the whole-volume features (SURVEY
    OPEN-3 default).  Reference-layout ``sub_features`` (10 float64 columns per
    row, no companion, e.g. written by nifty) are merged from the rows alone
    (``ctg_merge_feature_rows``): count sum, count-weighted mean, the exact
    pooled variance of the block (count, mean, var) triples, min/max over
    non-empty rows, and count-weighted quantiles (nifty-compatible; the exact
    merged quantiles need the histograms)."""
    begin, end = int(edgeIdBegin), int(edgeIdEnd)
    t = time.perf_counter()
    with _open(graphPath, 'r') as fg, _open(featuresPath, 'r') as ff:
        g = fg[subgraphKey]
        blk, _ = _subgraph_blocking(g)
        ds_ids = g['edge_ids']
        have_stats = featuresKey + STATS_SUFFIX in ff
        ds_feat = ff[featuresKey + STATS_SUFFIX] if have_stats else ff[featuresKey]
        n_features = int(ff[featuresKey].attrs.get('n_features', N_FEATURES))
        width = n_features   # (companion rows: per block, decode_stats_words)

        block_ids = [int(b) for b in blockIds]
        positions = [blk.blockGridPosition(b) for b in block_ids]
        all_ids, all_rows = _read_blocks_shared(ds_ids, ds_feat, positions, numberOfThreads)
        parts = []
        for b, ids, rows in zip(block_ids, all_ids, all_rows):
            if ids is None or rows is None:
                continue
            if have_stats:   # one canonical width for the concatenation
                if rows.size not in (ids.shape[0] * STATS_WORDS, ids.shape[0] * STATS_WORDS_COMPACT):
                    raise RuntimeError('mergeFeatureBlocks: block %d has %d edge ids but %d statistics words'
                                       % (b, ids.shape[0], rows.size))
                sm, rc = decode_stats_words(rows, ids.shape[0])
                rows = encode_stats_words(sm, rc, compact=False)
            rows = rows.reshape(-1, STATS_WORDS if have_stats else width)
            if rows.shape[0] != ids.shape[0]:
                raise RuntimeError('mergeFeatureBlocks: block %d has %d edge ids but %d feature rows'
                                   % (b, ids.shape[0], rows.shape[0]))
            sel = (ids >= begin) & (ids < end)
            if sel.any():
                parts.append((ids[sel], rows[sel]))
    t = _prof('merge_read', t)
    out = np.zeros((end - begin, N_FEATURES if have_stats else n_features), np.float64)
    if parts:
        ids = np.concatenate([p[0] for p in parts]).astype(np.uint64)
        rows = np.concatenate([p[1] for p in parts], axis=0)
        if have_stats:
            sums, recs = decode_stats_words(rows)
            keys = np.zeros((ids.shape[0], 2), np.uint64)
            keys[:, 1] = ids
            recs[:, 42] |= np.uint32(0x80000000)   # every block row is a graph edge
            merged = rag.merge_stats(keys, sums, recs)
            out[merged['edges'][:, 1].astype(np.int64) - begin] = merged['features']
        elif n_features == N_FEATURES:
            out = rag.merge_feature_rows(ids, rows, begin, end)
        else:
            # filter features (block_edge_features.py:226-233): groups of 9
            # statistics per (filter, sigma, channel) and the size column
            # last; each group merges as a 10-column row with that size
            if (n_features - 1) % (N_FEATURES - 1):
                raise RuntimeError('mergeFeatureBlocks: %d feature columns are not 9 k + 1' % n_features)
            size = rows[:, -1:]
            for g in range((n_features - 1) // (N_FEATURES - 1)):
                cols = slice(g * (N_FEATURES - 1), (g + 1) * (N_FEATURES - 1))
                m = rag.merge_feature_rows(ids, np.concatenate([rows[:, cols], size], axis=1), begin, end)
                out[:, cols] = m[:, :N_FEATURES - 1]
                out[:, -1] = m[:, -1]
    t = _prof('merge_compute', t)
    with _open(outPath) as fo:
        fo[outKey][begin:end, :] = out
    _prof('merge_write', t)
