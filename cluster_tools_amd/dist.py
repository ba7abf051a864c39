"""Multi-GPU RAG + edge features: one process per GPU, z-slabs, RCCL exchange.

This is the MI355X replacement for the reference's block -> merge structure
at the scale of whole GPUs.  In the reference a volume is cut into blocks,
``initial_sub_graphs`` / ``block_edge_features`` run per block and
``merge_sub_graphs`` / ``merge_edge_features`` combine the per-block results
(graph/merge_sub_graphs.py:130-135, features/merge_edge_features.py:141-147).
Here every rank owns one z-slab that is resident in its HBM (288 GB per GPU
holds slabs of several Gvoxels), reads one halo plane below it, and runs the
single-launch face scan over the whole slab with ``keep_stats`` so that its
per-edge partial statistics stay mergeable.  The only exchange step of the
path is the merge: edges are range-partitioned by their lower label ``u``
(splitters from an all-gathered sample, so the concatenation of the rank
shards is the globally sorted edge table); the rows that leave their rank
(28 x int64 per edge: (u,v), (sum, sumsq), the 48-word wide record) and the
node ids travel in ONE uniform-split ``all_to_all_single`` of fixed-capacity
segments whose layout, gather indices and true counts are computed on the
device (``ExchangePlan``: learned on the first call of a slab shape, reused
after, regrown when a call's counts overflow it).  Each rank then merges its
own rows with the received ones in one ``ctg_merge_stats`` call.  No count
matrix or split list is read on the host: the first host read of a call is
the merged result's size (with the overflow flag), then the shard offsets.
With spatially ordered labels (the reference's block-offset watershed ids,
the synthetic volumes) few rows leave their rank.  Scaling is weak:
per-rank slab size is fixed.

The exchange logic is backend-agnostic: ``HipBackend`` (libctg.so, the
product path) or, in the CPU tests, an oracle-backed numpy backend with the
same three methods, which lets the partition/exchange code run under gloo.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROW_WORDS = 28            # int64 words per exchanged edge row
WIDE_WORDS = 48           # u32 words of one wide statistics record
N_SAMPLES = 4096          # splitter sample per rank


class HipBackend:
    """Local partial tables and the merge on the GPU through libctg.so."""

    def local(self, labels, data, offsets, own_begin, own_end, ignore_label, hist_range):
        from . import rag
        # affinity partials keep non-adjacent pairs: adjacency is only known
        # globally, after the merge ORs the ADJ bits of all slabs
        r = rag.rag_features_handle(labels, data, offsets=offsets, own_begin=own_begin, own_end=own_end,
                                    ignore_label=ignore_label, hist_range=hist_range, keep_stats=True,
                                    no_adj_filter=offsets is not None)
        keys = r.edges_torch_i64()
        sums, recs = r.stats_torch()
        feats = r.features_torch()
        nodes = r.nodes_torch()
        info = r.info()
        r.free()
        return keys, sums, recs, nodes, info, feats

    def merge(self, keys, sums, recs, hist_range):
        """Merged (edges (E,2) int64, features (E,10) float64) tensors."""
        from . import rag
        m = rag.merge_stats_handle(keys, sums, recs, hist_range=hist_range)
        out = m.edges_torch_i64(), m.features_torch()
        m.free()
        return out

    def unique(self, values):
        from . import rag
        r = rag.unique_values_handle(values)
        out = r.nodes_torch()
        r.free()
        return out


def pack_rows(keys, sums, recs):
    """(E,2) int64 keys, (E,2) float64 sums, (E,48) int32 records -> (E,28) int64."""
    n = keys.shape[0]
    return torch.cat([keys.reshape(n, 2), sums.reshape(n, 2).view(torch.int64),
                      recs.reshape(n, WIDE_WORDS).view(torch.int64)], dim=1)


def unpack_rows(rows):
    rows = rows.reshape(-1, ROW_WORDS)
    keys = rows[:, :2].contiguous()
    sums = rows[:, 2:4].contiguous().view(torch.float64)
    recs = rows[:, 4:].contiguous().view(torch.int32)
    return keys, sums, recs


SIGN = -(1 << 63)         # xor with this maps uint64 order onto int64 order


def _ordered(k):
    """int64 view of uint64 labels -> int64 values in the same (unsigned) order."""
    return torch.bitwise_xor(k, SIGN)


def weighted_splitters_t(samples, counts, world):
    """Range splitters (world-1 values, torch) from per-rank samples of sorted keys.

    samples: (world, S) int64 tensor, row r an evenly spaced sample of rank r's
    sorted keys (meaningless where counts[r] == 0); counts: (world,) key
    totals.  Each sample of rank r stands for counts[r]/S keys.  Pure tensor
    arithmetic on the tensors' device (no host round trip), deterministic, so
    every rank computes the same splitters from the same gathered data.
    """
    S = samples.shape[1]
    dev = samples.device
    w = (counts.to(torch.float64) / S).repeat_interleave(S)
    v = samples.reshape(-1)
    keep = w > 0
    # dropped entries become +inf-weight-free sentinels at the end of the order
    v = torch.where(keep, v, torch.full_like(v, torch.iinfo(torch.int64).max))
    w = torch.where(keep, w, torch.zeros_like(w))
    order = torch.sort(v, stable=True).indices
    v, w = v[order], w[order]
    cw = torch.cumsum(w, 0)
    total = cw[-1]
    targets = total * torch.arange(1, world, device=dev, dtype=torch.float64) / world
    n_keep = keep.sum()
    idx = torch.searchsorted(cw, targets, side='left')
    idx = torch.minimum(idx, torch.clamp(n_keep - 1, min=0))
    out = v[idx]
    return torch.where(n_keep > 0, out, torch.zeros_like(out))


def weighted_splitters(samples, counts, world):
    """numpy front end of weighted_splitters_t (tests, host callers)."""
    t = weighted_splitters_t(torch.as_tensor(np.asarray(samples, dtype=np.int64)),
                             torch.as_tensor(np.asarray(counts, dtype=np.float64)), world)
    return t.numpy().astype(np.int64)


def split_counts_t(sorted_keys, splitters):
    """Rows per destination rank (tensor, on the keys' device) for a key column
    sorted ascending: rank k gets splitters[k-1] <= key < splitters[k]."""
    n = sorted_keys.shape[0]
    dev = sorted_keys.device
    if splitters.numel() == 0:
        return torch.tensor([n], dtype=torch.int64, device=dev)
    pos = torch.searchsorted(sorted_keys.contiguous(), splitters.to(dev), right=False)
    bounds = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), pos,
                        torch.full((1,), n, dtype=torch.int64, device=dev)])
    return bounds[1:] - bounds[:-1]


def split_counts(sorted_keys, splitters):
    """List front end of split_counts_t."""
    sp = torch.as_tensor(np.asarray(splitters, dtype=np.int64))
    return split_counts_t(sorted_keys, sp).cpu().tolist()


def _wire_device(device, group):
    """Where collectives run: RCCL ("nccl") moves HBM tensors over xGMI; a
    gloo group (CPU tests, and the multi-process GPU test on a one-GPU box)
    stages device tensors through host memory."""
    return torch.device('cpu') if dist.get_backend(group) == 'gloo' else device


def all_gather_tensor(t, group=None):
    """all_gather of equal-shape tensors -> list (on t's device)."""
    wire = _wire_device(t.device, group)
    tw = t.to(wire)
    out = [torch.empty_like(tw) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, tw, group=group)
    return [x.to(t.device) for x in out]


# Every device -> host read of the exchange goes through _host(): the count
# of reads per call (and where they happen) is what the tests check -- a call
# that reuses its ExchangePlan reads nothing before the result-size read.
host_reads = []


def _host(t, where):
    host_reads.append(where)
    return t.cpu()


class ExchangePlan:
    """Per-destination capacities of the uniform all_to_all (rows and node
    ids).  The first call of a (group, slab shape) learns them from the exact
    count matrix (one host read) with 50 % headroom; later calls reuse them
    and never read counts on the host: a call whose counts exceed a capacity
    notices it at the result-size read (the overflow flag rides along) and
    redoes the exchange with capacities learned from that call."""

    def __init__(self, cap_rows=0, cap_nodes=0, cap_own=None):
        self.cap_rows = int(cap_rows)
        self.cap_nodes = int(cap_nodes)
        # own rows merged with the received ones (this rank's; no collective
        # depends on it): None until the first call of the shape sizes it
        self.cap_own = cap_own

    @staticmethod
    def grow(x):
        return int(x) + int(x) // 2 + 64

    @staticmethod
    def from_counts(max_rows, max_nodes):
        return ExchangePlan(ExchangePlan.grow(max_rows), ExchangePlan.grow(max_nodes))


_plans = {}


def _plan_key(group, shape, offsets):
    return (id(group), dist.get_world_size(group), tuple(shape), None if offsets is None else
            tuple(map(tuple, np.asarray(offsets).reshape(-1, 3).tolist())))


NODE_EMPTY = -1           # node id of an empty slot: 2^64 - 1, last in unsigned order (never a real node id
                          # here: the volume's labels would need the full uint64 range)


def _uniform_exchange(keys, sums, recs, nodes, e_start, e_counts, n_start, n_counts, plan,
                      rank, group):
    """Rows and node ids to their owners in ONE uniform-split all_to_all_single.

    Destination d gets a fixed-size segment: [true row count, true node
    count, cap_rows rows of ROW_WORDS int64, cap_nodes node ids].  Empty
    slots hold a key (j, j) with a zero record (never an edge, no ADJ bit:
    the merge drops them) and node id NODE_EMPTY.  Segment layout, gather indices and the overflow flag are
    computed on the device; nothing is read on the host here.
    Returns (received rows, received node ids, overflow flag (device))."""
    world = dist.get_world_size(group)
    dev = keys.device
    wire = _wire_device(dev, group)
    cr, cn = plan.cap_rows, plan.cap_nodes
    n, nn = keys.shape[0], nodes.shape[0]
    j = torch.arange(cr, device=dev)
    src = e_start.reshape(-1, 1) + j.reshape(1, -1)                   # (world, cr)
    ok = j.reshape(1, -1) < e_counts.reshape(-1, 1)
    ok[rank] = False                                                  # this rank's own rows stay
    src = torch.clamp(src, max=max(n - 1, 0)).reshape(-1)
    if n:
        rows = pack_rows(keys.index_select(0, src), sums.index_select(0, src), recs.index_select(0, src))
    else:
        rows = torch.zeros((world * cr, ROW_WORDS), dtype=torch.int64, device=dev)
    ok = ok.reshape(-1, 1)
    # empty slot j: key (j, j) -- never an edge (u == v), and every empty slot
    # its own run (one shared key made one run of ~world * cap records, which
    # the merge's one-thread-per-edge reduce walked serially: 16-22 ms)
    empty = torch.zeros_like(rows)
    sl = torch.arange(rows.shape[0], device=dev, dtype=torch.int64)
    empty[:, 0] = sl
    empty[:, 1] = sl
    rows = torch.where(ok, rows, empty).reshape(world, cr * ROW_WORDS)
    jn = torch.arange(cn, device=dev)
    nsrc = torch.clamp(n_start.reshape(-1, 1) + jn.reshape(1, -1), max=max(nn - 1, 0)).reshape(-1)
    nok = jn.reshape(1, -1) < n_counts.reshape(-1, 1)
    nok[rank] = False
    nv = nodes.index_select(0, nsrc) if nn else torch.zeros(world * cn, dtype=torch.int64, device=dev)
    nv = torch.where(nok.reshape(-1), nv, torch.full_like(nv, NODE_EMPTY)).reshape(world, cn)
    hdr = torch.stack([e_counts, n_counts], dim=1).to(torch.int64)     # true counts: the receiver's check
    buf = torch.cat([hdr, rows, nv], dim=1).contiguous()
    out = torch.empty_like(buf, device=wire)
    dist.all_to_all_single(out, buf.to(wire), group=group)
    out = out.to(dev)
    got_e, got_n = out[:, 0].clone(), out[:, 1].clone()
    got_e[rank] = 0
    got_n[rank] = 0
    over = torch.logical_or((got_e > cr).any(), (got_n > cn).any()).to(torch.int64).reshape(1)
    # the row counts also size the next plan (max over this rank's senders)
    over = torch.cat([over, got_e.max().reshape(1), got_n.max().reshape(1)])
    rk = out[:, 2:2 + cr * ROW_WORDS].reshape(-1, ROW_WORDS)
    rn = out[:, 2 + cr * ROW_WORDS:].reshape(-1)
    return rk, rn, over


def _tensor(x, like):
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x).astype(np.int64) if np.asarray(x).dtype == np.uint64 else np.asarray(x),
                           device=like.device)


class DistResult:
    """This rank's shard of the global (sorted) edge table + features + nodes."""

    def __init__(self, merged, nodes, edge_offset, n_edges_global, node_offset, n_nodes_global, info):
        self.merged = merged          # backend merge result (rag.Result or dict)
        self.node_shard = nodes
        self.edge_offset = edge_offset
        self.n_edges_global = n_edges_global
        self.node_offset = node_offset
        self.n_nodes_global = n_nodes_global
        self._info = info

    @property
    def n_edges(self):
        return int(self.merged['edges'].shape[0])

    def info(self):
        return self._info

    def edges(self):
        """(E,2) uint64 numpy array."""
        e = self.merged['edges']
        if isinstance(e, torch.Tensor):
            e = e.cpu().numpy()
        return np.asarray(e).astype(np.uint64)

    def features(self):
        """(E,10) float64 numpy array."""
        f = self.merged['features']
        if isinstance(f, torch.Tensor):
            f = f.cpu().numpy()
        return np.asarray(f)

    def free(self):
        self.merged = {'edges': self.merged['edges'][:0], 'features': self.merged['features'][:0]}


def _exclusive_offsets(n_locals, group, device):
    """[(offset of this rank, total)] for each local count, one all_gather."""
    t = torch.tensor(list(n_locals), dtype=torch.int64, device=device)
    allc = _host(torch.stack(all_gather_tensor(t, group)), 'offsets').tolist()
    r = dist.get_rank(group)
    return [(sum(row[k] for row in allc[:r]), sum(row[k] for row in allc)) for k in range(len(n_locals))]


def slab_plan(Z, world, rank, offsets=None):
    """(read_begin, own_begin, own_end) z planes of rank ``rank`` of ``world``
    over a volume of ``Z`` planes: ``ctg_mgpu_slab`` (include/ctg.h) -- owned
    planes [Z*r/W, Z*(r+1)/W), read from as many halo planes below as the faces
    / offsets reach down.  ``own_begin[0]`` of the local call is
    ``own_begin - read_begin``."""
    from . import _lib
    import ctypes
    off = None if offsets is None else np.ascontiguousarray(np.asarray(offsets, dtype=np.int64).reshape(-1, 3))
    out = np.zeros(3, dtype=np.int64)
    _lib.check(_lib.load().ctg_mgpu_slab(int(Z), int(world), int(rank),
                                         None if off is None else off.ctypes.data_as(ctypes.c_void_p),
                                         0 if off is None else int(off.shape[0]),
                                         out.ctypes.data_as(ctypes.c_void_p)), 'ctg_mgpu_slab')
    return int(out[0]), int(out[1]), int(out[2])


def check_slab_halo(shape, offsets, own_begin, own_end):
    """The slab layout gives every rank the planes below its owned range as a
    lower halo and nothing above it.  An affinity sample aff[c, p] needs the
    partner p + o_c: with a lower neighbour (own_begin[0] > 0) the halo must
    hold max(-o_z) planes, and positive z offsets have no upper halo at all;
    x / y are never split.  Raise instead of silently dropping samples."""
    if offsets is None:
        return
    off = np.asarray(offsets, dtype=np.int64).reshape(-1, 3)
    ob = int(own_begin[0]) if own_begin is not None else 0
    oe = int(own_end[0]) if own_end is not None else int(shape[0])
    need_lo = int(max(0, -off[:, 0].min())) if off.size else 0
    if ob > 0 and ob < need_lo:
        raise ValueError('slab halo of %d plane(s) below the owned range, but the affinity offsets reach %d '
                         'planes down: give each rank max(-offset_z) halo planes' % (ob, need_lo))
    if off.size and off[:, 0].max() > 0 and oe < int(shape[0]) + int(off[:, 0].max()):
        raise ValueError('positive z offsets need an upper halo, which the z-slab layout does not have')


def rag_features_distributed(labels, data=None, offsets=None, own_begin=None, own_end=None,
                             ignore_label=False, hist_range=(0.0, 1.0), group=None, backend=None, plan=None):
    """Global RAG + edge features of a z-slab-partitioned volume.

    Every rank passes its slab (plus the halo planes below it, excluded via
    ``own_begin``); the call is collective.  Returns a ``DistResult`` whose
    edge rows are rows [edge_offset, edge_offset + n_edges) of the global
    sorted edge table (same for nodes).

    Device-resident exchange (RCCL moves HBM tensors; nothing is read on the
    host before the merged result's size):
      1. local partial table with mergeable statistics (one library call);
      2. one all_gather of splitter samples -> range splitters on u (device);
      3. per-destination row / node counts and gather indices (device);
      4. ONE uniform-split all_to_all_single of fixed-capacity segments
         (``ExchangePlan``) carrying rows, node ids and the true counts;
      5. one merge of this rank's own rows with the received ones
         (``ctg_merge_stats``: Chan's rule on the shifted sums, histograms add);
      6. one all_reduce of the overflow flag, read with the result size, and
         the all_gather of the shard sizes.
    A plan that proves too small (flag set on any rank) is regrown from the
    true counts and the exchange redone; the first call of a slab shape
    learns its plan that way.
    """
    shape = tuple(labels.shape)
    if world_size_of(group) > 1:
        check_slab_halo(shape, offsets, own_begin, own_end)
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
    keys, sums, recs, nodes, info, feats = backend.local(labels, data, offsets, own_begin, own_end,
                                                          ignore_label, hist_range)
    phase('local')
    dev = keys.device
    wire = _wire_device(dev, group)
    n = keys.shape[0]
    nodes = nodes.reshape(-1).to(torch.int64)
    # splitters on u (unsigned order) from an evenly spaced sample of the
    # sorted local keys
    ou = _ordered(keys[:, 0]) if n else keys[:, 0]
    if n > 0:
        idx = torch.div(torch.arange(N_SAMPLES, device=dev, dtype=torch.int64) * n, N_SAMPLES,
                        rounding_mode='floor')
        samp = ou.index_select(0, idx)
    else:
        samp = torch.zeros(N_SAMPLES, dtype=torch.int64, device=dev)
    meta = torch.cat([samp, torch.full((1,), n, dtype=torch.int64, device=dev)]).to(wire)
    g = torch.stack(all_gather_tensor(meta, group)).to(dev)
    splitters = weighted_splitters_t(g[:, :N_SAMPLES], g[:, N_SAMPLES], world)
    e_counts = split_counts_t(ou, splitters)
    n_counts = split_counts_t(_ordered(nodes), splitters)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    e_start = torch.cat([zero, torch.cumsum(e_counts, 0)[:-1]])
    n_start = torch.cat([zero, torch.cumsum(n_counts, 0)[:-1]])
    # this rank's own node ids stay in place; every other one is masked to an
    # empty slot (its rows were sent; its node ids travel with them)
    arn = torch.arange(nodes.shape[0], device=dev)
    own_n = (arn >= n_start[rank]) & (arn < n_start[rank] + n_counts[rank])
    own_nodes = torch.where(own_n, nodes, torch.full_like(nodes, NODE_EMPTY))
    own_lo = e_start[rank]
    own_hi = own_lo + e_counts[rank]
    phase('splitters+masks')

    key = _plan_key(group, shape, offsets)
    if plan is None:
        plan = _plans.get(key)
    learn = plan is None
    if learn:
        plan = ExchangePlan(0, 0)
    while True:
        rk, rn, over = _uniform_exchange(keys, sums, recs, nodes, e_start, e_counts, n_start, n_counts,
                                         plan, rank, group)
        over = over.to(wire)
        dist.all_reduce(over, op=dist.ReduceOp.MAX, group=group)
        phase('exchange (cap %d rows, %d nodes)' % (plan.cap_rows, plan.cap_nodes))
        if learn:
            # no plan yet: learn the capacities from the true counts now (the
            # only host read before the merge, first call of a shape only)
            ov = _host(over, 'plan')
            plan = ExchangePlan.from_counts(int(ov[1]), int(ov[2]))
            learn = False
            if int(ov[0]):
                continue
        rks, rss, rrs = unpack_rows(rk)
        # Own rows that can share a key with a received row: the received keys'
        # u values lie in this rank's range, and the own rows are sorted by u,
        # so they are the slice [lo, hi) of own rows with u between the
        # smallest and the largest received u.  Only that slice is merged with
        # the received rows; every other own row keeps the local call's
        # features.  (Empty slots are keyed (j, j).)
        real = rks[:, 0] != rks[:, 1]
        ru = _ordered(rks[:, 0])
        big = torch.iinfo(torch.int64).max
        umin = torch.where(real, ru, torch.full_like(ru, big)).min().reshape(1) if ru.numel() else \
            torch.full((1,), big, dtype=torch.int64, device=dev)
        umax = torch.where(real, ru, torch.full_like(ru, -big - 1)).max().reshape(1) if ru.numel() else \
            torch.full((1,), -big - 1, dtype=torch.int64, device=dev)
        lo = torch.searchsorted(ou.contiguous(), umin, right=False) if n else torch.zeros(1, dtype=torch.int64,
                                                                                           device=dev)
        hi = torch.searchsorted(ou.contiguous(), umax, right=True) if n else torch.zeros(1, dtype=torch.int64,
                                                                                          device=dev)
        lo = torch.clamp(torch.minimum(lo, own_hi), min=own_lo)
        hi = torch.maximum(torch.minimum(hi, own_hi), lo)
        while True:
            if plan.cap_own is None:   # first call of the shape: size the slice (this rank only)
                plan.cap_own = ExchangePlan.grow(int(_host(hi - lo, 'plan')[0]))
            c2 = plan.cap_own
            j = torch.arange(c2, device=dev, dtype=torch.int64)
            ok2 = (lo + j) < hi
            src = torch.clamp(lo + j, max=max(n - 1, 0))
            # empty slot: (j, j) -- never an edge; small j keeps every key below 2^32 (a larger one
            # sends ctg_merge_stats down its dense-relabel path); equal empty keys only merge empty runs
            slot_key = torch.stack([j, j], dim=1)
            k2 = torch.where(ok2.reshape(-1, 1), keys.index_select(0, src), slot_key) if n else slot_key
            s2 = torch.where(ok2.reshape(-1, 1), sums.reshape(n, 2).index_select(0, src),
                             torch.zeros((c2, 2), dtype=sums.dtype, device=dev)) if n else \
                torch.zeros((c2, 2), dtype=torch.float64, device=dev)
            r2 = torch.where(ok2.reshape(-1, 1), recs.reshape(n, WIDE_WORDS).index_select(0, src),
                             torch.zeros((c2, WIDE_WORDS), dtype=recs.dtype, device=dev)) if n else \
                torch.zeros((c2, WIDE_WORDS), dtype=torch.int32, device=dev)
            me, mf = backend.merge(torch.cat([k2, rks]), torch.cat([s2, rss]), torch.cat([r2, rrs]), hist_range)
            phase('merge (%d + %d rows)' % (c2, rks.shape[0]))
            # the result-size read: the merge has returned its size; the
            # overflow flags (the exchange's agreed by all ranks) and the slice
            # bounds come to the host with it
            ov = _host(torch.cat([over.to(dev), (hi - lo > c2).to(torch.int64).reshape(1), lo, hi,
                                  own_lo.reshape(1), own_hi.reshape(1)]), 'result')
            if int(ov[0]) or not int(ov[3]):
                break
            plan.cap_own = ExchangePlan.grow(int(ov[5] - ov[4]))   # this rank's slice only: no collective
        if int(ov[0]):
            cap_own = plan.cap_own
            plan = ExchangePlan.from_counts(int(ov[1]), int(ov[2]))
            plan.cap_own = cap_own
            continue
        break
    _plans[key] = plan
    lo_i, hi_i, olo, ohi = (int(x) for x in ov[4:8])
    me, mf = _tensor(me, keys), _tensor(mf, keys)
    loc_e = [keys[olo:lo_i], keys[hi_i:ohi]]
    loc_f = [feats[olo:lo_i], feats[hi_i:ohi]]
    if offsets is not None:
        # affinity partials keep non-adjacent pairs: a local-only key is an
        # edge when one of its samples proved adjacency (ADJ bit of its record)
        adj = [recs[olo:lo_i, 42] < 0, recs[hi_i:ohi, 42] < 0]
        loc_e = [x[m] for x, m in zip(loc_e, adj)]
        loc_f = [x[m] for x, m in zip(loc_f, adj)]
    # sorted by construction: own rows below the slice, the merged slice, own rows above it
    merged = {'edges': torch.cat([loc_e[0], me, loc_e[1]]), 'features': torch.cat([loc_f[0], mf, loc_f[1]])}
    n_loc = int(merged['edges'].shape[0])
    # nodes went to the same ranges in the all_to_all; one NODE_EMPTY is
    # appended so the sorted unique ids always end with exactly one of it
    node_shard = backend.unique(torch.cat([own_nodes, rn, torch.full((1,), NODE_EMPTY, dtype=torch.int64,
                                                                       device=dev)]))[:-1]
    phase('nodes')
    (e_off, e_tot), (n_off, n_tot) = _exclusive_offsets([n_loc, int(node_shard.shape[0])], group, dev)
    phase('offsets')
    return DistResult(merged, node_shard, e_off, e_tot, n_off, n_tot, info)


def world_size_of(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1
