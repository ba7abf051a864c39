"""Multi-GPU RAG + edge features: one process per GPU, z-slabs, RCCL exchange.

This is the MI355X replacement for the reference's block -> merge structure
at the scale of whole GPUs.  In the reference a volume is cut into blocks,
``initial_sub_graphs`` / ``block_edge_features`` run per block and
``merge_sub_graphs`` / ``merge_edge_features`` combine the per-block results
(graph/merge_sub_graphs.py:130-135, features/merge_edge_features.py:141-147).
Here every rank owns one z-slab that is resident in its HBM (288 GB per GPU
holds slabs of several Gvoxels; ``ctg_mgpu_slab`` gives the planes and the
halo below them), runs the single-launch face scan over the whole slab with
``keep_stats`` so that its per-edge partial statistics stay mergeable, and the
ranks combine their tables in ONE exchange step.  The global sorted edge table
is range-partitioned by the lower label ``u``; the device work between the
collectives is the C ABI's ``ctg_mgpu_*`` (cluster_tools_amd/csrc/ctg_mgpu.hip):

  1. ``ctg_mgpu_sample``  -> all_gather of every rank's u sample;
  2. ``ctg_mgpu_split``   -> splitters (exact integer weights: every rank gets
     the same ones) and the rows / node ids for every rank; all_gather of those
     counts -- read on the host: every segment size of the exchange is then
     known exactly on every rank (no capacity guess, no overflow retry);
  3. ``ctg_mgpu_pack``    -> one ``all_to_all_single`` of the rows (28 int64
     words: (u,v), (S1,S2), the 48-word wide record) and node ids that leave
     their rank, segment sizes from the count matrix;
  4. ``ctg_mgpu_merge``   -> this rank's shard: received rows merged with its
     own range (equal keys combined by Chan's rule, histograms added), every
     untouched own row kept as the local call computed it; with nothing
     received the own range IS the shard (no kernel, no copy);
  5. all_gather of the shard sizes (global offsets).

Host reads per call: the count matrix and the shard sizes (plus the library's
own result-size reads).  With spatially ordered labels (the reference's
block-offset watershed ids, the synthetic volumes) few rows leave their rank.

The exchange logic is backend-agnostic: ``HipBackend`` (libctg.so, the
product path) or, in the CPU tests, a numpy restatement of the four steps with
the same methods (tests/dist_helpers.py), which runs this module under gloo.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

ROW_WORDS = L.CTG_MGPU_ROW_WORDS     # int64 words per exchanged edge row
N_SAMPLES = L.CTG_MGPU_SAMPLES       # splitter sample per rank
MAX_WORLD = L.CTG_MGPU_MAX_WORLD


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class HipBackend:
    """The device steps of the exchange through libctg.so (ctg_mgpu_*).

    defer_stats (default): the local call writes no mergeable-statistics rows;
    ctg_mgpu_pack / ctg_mgpu_merge rebuild them from the call's records only
    for the rows that leave the rank and the own rows that meet a received key
    (CTG_DEFER_STATS; boundary maps without ignore_label -- the library writes
    the rows for every other call).  False: every row is written (CTG_KEEP_STATS)."""

    def __init__(self, defer_stats=True):
        self.defer_stats = defer_stats

    def local(self, labels, data, offsets, own_begin, own_end, ignore_label, hist_range):
        """This rank's partial table: a device-resident rag.Result with the
        mergeable statistics (affinities: non-adjacent pairs kept -- adjacency
        is only known globally, after the merge ORs the ADJ bits)."""
        from . import rag
        return rag.rag_features_handle(labels, data, offsets=offsets, own_begin=own_begin, own_end=own_end,
                                       ignore_label=ignore_label, hist_range=hist_range, keep_stats=True,
                                       no_adj_filter=offsets is not None, defer_stats=self.defer_stats)

    def sample(self, loc):
        meta = torch.empty(N_SAMPLES + 1, dtype=torch.int64, device='cuda')
        L.check(L.load().ctg_mgpu_sample(loc.handle, _vp(meta), _stream()), 'ctg_mgpu_sample')
        return meta

    def split(self, loc, meta_all, world):
        counts = torch.empty((world, 2), dtype=torch.int64, device='cuda')
        L.check(L.load().ctg_mgpu_split(loc.handle, _vp(meta_all.contiguous()), world, _vp(counts), _stream()),
                'ctg_mgpu_split')
        return counts

    def pack(self, loc, counts_all, world, rank, words):
        send = torch.empty(max(words, 1), dtype=torch.int64, device='cuda')
        ca = np.ascontiguousarray(counts_all, dtype=np.int64)
        L.check(L.load().ctg_mgpu_pack(loc.handle, ca.ctypes.data_as(ctypes.c_void_p), world, rank, _vp(send),
                                       _stream()), 'ctg_mgpu_pack')
        return send[:words]

    def merge(self, loc, recv, counts_all, world, rank, hist_range):
        from . import rag
        ca = np.ascontiguousarray(counts_all, dtype=np.int64)
        h = ctypes.c_void_p()
        L.check(L.load().ctg_mgpu_merge(loc.handle, _vp(recv), ca.ctypes.data_as(ctypes.c_void_p), world, rank,
                                        float(hist_range[0]), float(hist_range[1]), _stream(), ctypes.byref(h)),
                'ctg_mgpu_merge')
        return rag.Result(h, loc.device)


def _wire_device(device, group):
    """Where collectives run: RCCL ("nccl") moves HBM tensors over xGMI; a
    gloo group (CPU tests, and the multi-process GPU test on a one-GPU box)
    stages device tensors through host memory."""
    return torch.device('cpu') if dist.get_backend(group) == 'gloo' else device


def all_gather_flat(t, group=None):
    """all_gather of equal-size tensors into one flat tensor (rank-major, on
    t's device): one ``all_gather_into_tensor``, no per-rank outputs."""
    wire = _wire_device(t.device, group)
    tw = t.reshape(-1).to(wire)
    out = torch.empty(tw.numel() * dist.get_world_size(group), dtype=tw.dtype, device=wire)
    dist.all_gather_into_tensor(out, tw, group=group)
    return out.to(t.device)


# Every device -> host read of the exchange goes through _host(): the tests
# check the sequence (one count-matrix read and one shard-size read per call).
host_reads = []


def _host(t, where):
    host_reads.append(where)
    return t.cpu()


def segment_words(counts_all, world, rank):
    """int64 words this rank sends to / receives from every rank in the
    all_to_all (its own entries 0): rows x ROW_WORDS + node ids."""
    c = np.asarray(counts_all, dtype=np.int64).reshape(world, world, 2)
    w = c[:, :, 0] * ROW_WORDS + c[:, :, 1]
    send = w[rank].copy()
    recv = w[:, rank].copy()
    send[rank] = recv[rank] = 0
    return send.tolist(), recv.tolist()


class DistResult:
    """This rank's shard of the global (sorted) edge table + features + nodes.

    The shard sizes of every rank are all-gathered on the stream when the call
    returns; the host reads them (one read, ``_host(..., 'offsets')``) only when
    an offset, a global count or ``shard_sizes`` is first asked for, so a
    caller that works on its shard alone never waits for them."""

    def __init__(self, shard, sizes_all, rank, info):
        self.shard = shard            # rag.Result (HIP) or the test backend's shard
        self._sizes_all = sizes_all   # (world*2,) int64 tensor: (edges, nodes) of every rank
        self._rank = rank
        self._sizes = None
        self._info = info

    @property
    def shard_sizes(self):
        """[(edges, nodes)] of every rank."""
        if self._sizes is None:
            a = _host(self._sizes_all, 'offsets').reshape(-1, 2).tolist()
            self._sizes = [tuple(int(v) for v in row) for row in a]
            self._sizes_all = None
        return self._sizes

    @property
    def edge_offset(self):
        return sum(s[0] for s in self.shard_sizes[:self._rank])

    @property
    def n_edges_global(self):
        return sum(s[0] for s in self.shard_sizes)

    @property
    def node_offset(self):
        return sum(s[1] for s in self.shard_sizes[:self._rank])

    @property
    def n_nodes_global(self):
        return sum(s[1] for s in self.shard_sizes)

    @property
    def n_edges(self):
        return int(self.shard.n_edges)

    @property
    def node_shard(self):
        """(N_r,) int64 torch tensor (device for the HIP backend)."""
        return self.shard.nodes_torch()

    def info(self):
        return self._info

    def edges(self):
        """(E,2) uint64 numpy array."""
        return np.asarray(self.shard.edges()).astype(np.uint64)

    def features(self):
        """(E,10) float64 numpy array."""
        return np.asarray(self.shard.features())

    def edges_torch_i64(self):
        return self.shard.edges_torch_i64()

    def features_torch(self):
        return self.shard.features_torch()

    def free(self):
        self.shard.free()


def slab_plan(Z, world, rank, offsets=None):
    """(read_begin, own_begin, own_end) z planes of rank ``rank`` of ``world``
    over a volume of ``Z`` planes: ``ctg_mgpu_slab`` (include/ctg.h) -- owned
    planes [Z*r/W, Z*(r+1)/W), read from as many halo planes below as the faces
    / offsets reach down.  ``own_begin[0]`` of the local call is
    ``own_begin - read_begin``."""
    off = None if offsets is None else np.ascontiguousarray(np.asarray(offsets, dtype=np.int64).reshape(-1, 3))
    out = np.zeros(3, dtype=np.int64)
    L.check(L.load().ctg_mgpu_slab(int(Z), int(world), int(rank),
                                   None if off is None else off.ctypes.data_as(ctypes.c_void_p),
                                   0 if off is None else int(off.shape[0]),
                                   out.ctypes.data_as(ctypes.c_void_p)), 'ctg_mgpu_slab')
    return int(out[0]), int(out[1]), int(out[2])


def check_slab_halo(shape, offsets, own_begin, own_end, read_begin=None):
    """The slab layout gives every rank the planes below its owned range as a
    lower halo and nothing above it.  An affinity sample aff[c, p] needs the
    partner p + o_c: with a lower neighbour the halo must hold max(-o_z)
    planes -- or reach down to global plane 0 (``read_begin == 0``: the slab
    plan clips the halo there, ``ctg_mgpu_slab``) -- and positive z offsets
    have no upper halo at all; x / y are never split.  Raise instead of
    silently dropping samples."""
    if offsets is None:
        return
    off = np.asarray(offsets, dtype=np.int64).reshape(-1, 3)
    ob = int(own_begin[0]) if own_begin is not None else 0
    oe = int(own_end[0]) if own_end is not None else int(shape[0])
    need_lo = int(max(0, -off[:, 0].min())) if off.size else 0
    if ob > 0 and ob < need_lo and read_begin != 0:
        raise ValueError('slab halo of %d plane(s) below the owned range, but the affinity offsets reach %d '
                         'planes down: give each rank max(-offset_z) halo planes' % (ob, need_lo))
    if off.size and off[:, 0].max() > 0 and oe < int(shape[0]) + int(off[:, 0].max()):
        raise ValueError('positive z offsets need an upper halo, which the z-slab layout does not have')


def rag_features_distributed(labels, data=None, offsets=None, own_begin=None, own_end=None,
                             ignore_label=False, hist_range=(0.0, 1.0), group=None, backend=None,
                             read_begin=None):
    """Global RAG + edge features of a z-slab-partitioned volume.

    Every rank passes its slab (plus the halo planes below it, excluded via
    ``own_begin``); the call is collective.  ``read_begin``: the slab's first
    plane in the volume (``slab_plan``), needed only where a rank's halo is
    clipped at plane 0.  Returns a ``DistResult`` whose edge rows are rows
    [edge_offset, edge_offset + n_edges) of the global sorted edge table (same
    for nodes).
    """
    shape = tuple(labels.shape)
    if world_size_of(group) > 1:
        check_slab_halo(shape, offsets, own_begin, own_end, read_begin)
    debug = os.environ.get('CTG_DIST_DEBUG') == '1'   # per-phase wall times on stderr (synchronising)
    tdbg = [time.perf_counter()]

    def phase(name):
        if debug:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            tdbg.append(time.perf_counter())
            print('[dist r%d] %s %.3f ms' % (dist.get_rank(group), name, (tdbg[-1] - tdbg[-2]) * 1e3),
                  file=sys.stderr, flush=True)
    backend = backend or HipBackend()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world > MAX_WORLD:
        raise ValueError('at most %d ranks' % MAX_WORLD)
    loc = backend.local(labels, data, offsets, own_begin, own_end, ignore_label, hist_range)
    try:
        info = loc.info()
        phase('local')
        meta = backend.sample(loc)
        dev = meta.device
        wire = _wire_device(dev, group)
        meta_all = all_gather_flat(meta, group)
        counts = backend.split(loc, meta_all, world)
        counts_all = _host(all_gather_flat(counts, group), 'counts').numpy().reshape(world, world, 2)
        phase('splitters+counts')
        send_w, recv_w = segment_words(counts_all, world, rank)
        recv = None
        if _any_exchange(counts_all, world):   # the same decision on every rank: same count matrix
            send = backend.pack(loc, counts_all, world, rank, int(sum(send_w))) if sum(send_w) else \
                torch.empty(0, dtype=torch.int64, device=dev)
            recv = torch.empty(int(sum(recv_w)), dtype=torch.int64, device=wire)
            dist.all_to_all_single(recv, send.to(wire), output_split_sizes=recv_w, input_split_sizes=send_w,
                                   group=group)
            recv = recv.to(dev) if sum(recv_w) else None
        phase('exchange (%d words out, %d in)' % (sum(send_w), sum(recv_w)))
        shard = backend.merge(loc, recv, counts_all, world, rank, hist_range)
        phase('merge')
    finally:
        loc.free()
    # the global offsets: every rank's shard sizes, gathered now (collective
    # order), read by the host on first use (DistResult)
    ne, nn = int(shard.n_edges), int(shard.n_nodes)
    if wire.type == 'cuda':
        # built on the device by one kernel (no pageable host -> device copy,
        # which would wait for the stream)
        mine = torch.arange(2, dtype=torch.int64, device=wire) * (nn - ne) + ne
    else:
        mine = torch.tensor([ne, nn], dtype=torch.int64)
    sizes = all_gather_flat(mine, group)
    phase('offsets')
    return DistResult(shard, sizes, rank, info)


def _any_exchange(counts_all, world):
    c = np.asarray(counts_all).reshape(world, world, 2)
    off = c.sum(axis=2)
    return bool(off.sum() - np.trace(off) > 0)


def gather_to_host(res, root=0, group=None):
    """SURVEY §8(e) Output: the global (E,2) uint64 edges, (E,10) float64
    features and (N,) uint64 nodes on rank ``root`` (host memory, for the N5
    write of merge_edge_features.py:141-147 / merge_sub_graphs.py:130-135);
    collective, other ranks return None.  Shards travel to the root over the
    group's backend (RCCL: xGMI), then one copy to host."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    e = res.edges_torch_i64().reshape(-1, 2)
    f = res.features_torch().reshape(-1, 10)
    n = res.node_shard.reshape(-1)
    dev = e.device
    wire = _wire_device(dev, group)
    me = max(s[0] for s in res.shard_sizes)
    mn = max(s[1] for s in res.shard_sizes)
    # one padded buffer per rank: edges (2 words), features (10 words as int64 bits), nodes
    buf = torch.zeros(me * 12 + mn, dtype=torch.int64, device=dev)
    buf[:e.shape[0] * 2] = e.reshape(-1)
    buf[me * 2:me * 2 + f.shape[0] * 10] = f.reshape(-1).view(torch.int64)
    buf[me * 12:me * 12 + n.shape[0]] = n
    bw = buf.to(wire)
    parts = [torch.empty_like(bw) for _ in range(world)] if rank == root else None
    dist.gather(bw, parts, dst=root, group=group)
    if rank != root:
        return None
    edges, feats, nodes = [], [], []
    for p, (ne, nn) in zip(parts, res.shard_sizes):
        p = p.cpu()
        edges.append(p[:ne * 2].reshape(ne, 2))
        feats.append(p[me * 2:me * 2 + ne * 10].view(torch.float64).reshape(ne, 10))
        nodes.append(p[me * 12:me * 12 + nn])
    return (torch.cat(edges).numpy().view(np.uint64), torch.cat(feats).numpy(),
            torch.cat(nodes).numpy().view(np.uint64))


def write_global(res, graph_path, graph_key='graph', features_path=None, features_key='features', shape=None,
                 ignore_label=False, root=0, group=None, n_threads=8, timings=None):
    """SURVEY §8(e) Output: gather the shards on ``root`` (gather_to_host) and
    write what MergeSubGraphs / MergeEdgeFeatures write for the same volume:

    * ``graph_path/graph_key/{nodes,edges}`` (chunks min(262144, N) / (min(262144,
      E), 2), gzip) with attrs numberOfNodes / numberOfEdges
      (merge_sub_graphs.py:127-137, ndist.mergeSubgraphs), ``shape``
      (:137) and ``ignore_label`` (graph_workflow.py's sub-graph attrs, :63-68);
    * ``features_path/features_key`` (E, 10) float64, chunks (min(262144, E), 1),
      gzip (merge_edge_features.py:62-65, written per edge range at :141-147).

    Collective; the N5 write happens on ``root`` only (returns (E, N) there,
    None elsewhere).  ``timings`` (dict) receives 'gather_s' and 'write_s'."""
    from . import n5
    t0 = time.perf_counter()
    got = gather_to_host(res, root=root, group=group)
    t1 = time.perf_counter()
    if timings is not None:
        timings['gather_s'] = t1 - t0
    if got is None:
        return None
    edges, feats, nodes = got
    n_edges, n_nodes = int(edges.shape[0]), int(nodes.shape[0])
    with n5.file_reader(graph_path) as f:
        g = f.require_group(graph_key)
        ds_n = g.require_dataset('nodes', shape=(n_nodes,), chunks=(max(1, min(n_nodes, 262144)),),
                                 dtype='uint64', compression='gzip')
        ds_e = g.require_dataset('edges', shape=(n_edges, 2), chunks=(max(1, min(n_edges, 262144)), 2),
                                 dtype='uint64', compression='gzip')
        ds_n.n_threads = ds_e.n_threads = max(1, int(n_threads))
        if n_nodes:
            ds_n[:] = nodes
        if n_edges:
            ds_e[:] = edges
        g.attrs['numberOfNodes'] = n_nodes
        g.attrs['numberOfEdges'] = n_edges
        if shape is not None:
            g.attrs['shape'] = [int(v) for v in shape]
        g.attrs['ignore_label'] = bool(ignore_label)
    with n5.file_reader(features_path or graph_path) as f:
        ds_f = f.require_dataset(features_key, shape=(n_edges, 10), chunks=(max(1, min(n_edges, 262144)), 1),
                                 dtype='float64', compression='gzip')
        ds_f.n_threads = max(1, int(n_threads))
        if n_edges:
            ds_f[:] = feats
    if timings is not None:
        timings['write_s'] = time.perf_counter() - t1
    return n_edges, n_nodes


def world_size_of(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1
