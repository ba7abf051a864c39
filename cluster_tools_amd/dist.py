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
shards is the globally sorted edge table), the partial rows travel in one
``all_to_all_single`` (28 x int64 per edge: (u,v), (sum, sumsq), the 48-word
wide record).  Only rows that leave their rank are packed and shipped, and
only keys present on more than one rank are merged (``ctg_merge_stats``):
every other edge is complete in its slab and keeps the features of the local
call.  With spatially ordered labels (the reference's block-offset watershed
ids, the synthetic volumes) that is the few edges crossing a slab boundary.
Node lists take the same route.  Scaling is weak: per-rank slab size is fixed.

The exchange logic is backend-agnostic: ``HipBackend`` (libctg.so, the
product path) or, in the CPU tests, an oracle-backed numpy backend with the
same three methods, which lets the partition/exchange code run under gloo.
"""
from __future__ import annotations

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


def exchange(rows, send_counts, group=None, recv_counts=None):
    """all_to_all of variable-length row blocks; returns the received rows.
    With ``recv_counts`` (known from an earlier all_gather of the count
    matrix) no count exchange and no host round trip happen here."""
    world = dist.get_world_size(group)
    dev = rows.device
    wire = _wire_device(dev, group)
    if recv_counts is None:
        sc = torch.tensor(list(send_counts), dtype=torch.int64, device=wire)
        rc = torch.empty(world, dtype=torch.int64, device=wire)
        dist.all_to_all_single(rc, sc, group=group)
        recv_counts = rc.cpu().tolist()
    shape = (int(sum(recv_counts)),) + tuple(rows.shape[1:])
    out = torch.empty(shape, dtype=rows.dtype, device=wire)
    dist.all_to_all_single(out, rows.contiguous().to(wire), output_split_sizes=[int(c) for c in recv_counts],
                           input_split_sizes=[int(c) for c in send_counts], group=group)
    return out.to(dev)


def exchange_rows_nodes(rows, e_send, e_recv, nodes, n_send, n_recv, group=None):
    """One all_to_all for the edge rows (ROW_WORDS int64 each) and the node
    ids: destination d gets [its rows, its node ids] as one int64 segment
    (counts from the count matrix, known on every rank) -- one collective
    instead of two per step."""
    world = dist.get_world_size(group)
    dev = rows.device
    wire = _wire_device(dev, group)
    rows = rows.reshape(-1, ROW_WORDS)
    nodes = nodes.reshape(-1).to(torch.int64)
    parts, r0, n0 = [], 0, 0
    for d in range(world):
        parts.append(rows[r0:r0 + int(e_send[d])].reshape(-1))
        parts.append(nodes[n0:n0 + int(n_send[d])])
        r0 += int(e_send[d])
        n0 += int(n_send[d])
    buf = torch.cat(parts).to(wire)
    in_split = [int(e_send[d]) * ROW_WORDS + int(n_send[d]) for d in range(world)]
    out_split = [int(e_recv[d]) * ROW_WORDS + int(n_recv[d]) for d in range(world)]
    out = torch.empty(sum(out_split), dtype=torch.int64, device=wire)
    dist.all_to_all_single(out, buf, output_split_sizes=out_split, input_split_sizes=in_split, group=group)
    out = out.to(dev)
    rr, nr, o = [], [], 0
    for d in range(world):
        rr.append(out[o:o + int(e_recv[d]) * ROW_WORDS])
        o += int(e_recv[d]) * ROW_WORDS
        nr.append(out[o:o + int(n_recv[d])])
        o += int(n_recv[d])
    return torch.cat(rr).reshape(-1, ROW_WORDS), torch.cat(nr)


def all_gather_tensor(t, group=None):
    """all_gather of equal-shape tensors -> list (on t's device)."""
    wire = _wire_device(t.device, group)
    tw = t.to(wire)
    out = [torch.empty_like(tw) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, tw, group=group)
    return [x.to(t.device) for x in out]


def _pack_uv(k):
    """(E,2) int64 (u,v) -> one sortable int64 (labels < 2^31)."""
    return k[:, 0] * (1 << 32) + k[:, 1]


def _merge_sorted(ka, fa, kb, fb):
    """Merge two (u,v)-sorted row sets with disjoint keys (the local-only rows
    and the merged shared rows) by scatter, not a sort of the whole shard."""
    pa, pb = _pack_uv(ka), _pack_uv(kb)
    na, nb = pa.shape[0], pb.shape[0]
    dev = ka.device
    pos_a = torch.arange(na, device=dev) + torch.searchsorted(pb, pa)
    pos_b = torch.arange(nb, device=dev) + torch.searchsorted(pa, pb)
    k = torch.empty((na + nb,) + tuple(ka.shape[1:]), dtype=ka.dtype, device=dev)
    f = torch.empty((na + nb,) + tuple(fa.shape[1:]), dtype=fa.dtype, device=dev)
    k[pos_a] = ka
    k[pos_b] = kb
    f[pos_a] = fa
    f[pos_b] = fb
    return {'edges': k, 'features': f}


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
    allc = torch.stack(all_gather_tensor(t, group)).cpu().tolist()
    r = dist.get_rank(group)
    return [(sum(row[k] for row in allc[:r]), sum(row[k] for row in allc)) for k in range(len(n_locals))]


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
                             ignore_label=False, hist_range=(0.0, 1.0), group=None, backend=None):
    """Global RAG + edge features of a z-slab-partitioned volume.

    Every rank passes its slab (plus the halo planes below it, excluded via
    ``own_begin``); the call is collective.  Returns a ``DistResult`` whose
    edge rows are rows [edge_offset, edge_offset + n_edges) of the global
    sorted edge table (same for nodes).

    Collectives: one all_gather of the splitter samples, one all_gather of
    the (edge, node) send-count matrix -- the only host round trip before the
    data moves --, one all_to_all of the edge rows and node ids together, and
    the all_gather of the shard sizes.  Splitters and counts are computed on the
    wire device, so with RCCL nothing but the count matrix leaves HBM.
    """
    shape = tuple(labels.shape)
    if world_size_of(group) > 1:
        check_slab_halo(shape, offsets, own_begin, own_end)
    backend = backend or HipBackend()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    keys, sums, recs, nodes, info, feats = backend.local(labels, data, offsets, own_begin, own_end,
                                                         ignore_label, hist_range)
    dev = keys.device
    wire = _wire_device(dev, group)
    n = keys.shape[0]
    nodes = nodes.reshape(-1)
    # splitters on u (unsigned order) from an evenly spaced sample of the
    # sorted local keys; the signed min / max of every label ride along
    # (the packed (u,v) fast path needs 0 <= label < 2^31)
    ou = _ordered(keys[:, 0]) if n else keys[:, 0]
    if n > 0:
        idx = torch.div(torch.arange(N_SAMPLES, device=dev, dtype=torch.int64) * n, N_SAMPLES,
                        rounding_mode='floor')
        samp = ou.index_select(0, idx)
        lo = torch.minimum(keys.min(), nodes.min() if nodes.numel() else keys.min()).reshape(1)
        hi = torch.maximum(keys.max(), nodes.max() if nodes.numel() else keys.max()).reshape(1)
    else:
        samp = torch.zeros(N_SAMPLES, dtype=torch.int64, device=dev)
        z = nodes.min().reshape(1) if nodes.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
        lo = z
        hi = nodes.max().reshape(1) if nodes.numel() else z
    meta = torch.cat([samp, torch.tensor([n], dtype=torch.int64, device=dev), lo, hi]).to(wire)
    g = torch.stack(all_gather_tensor(meta, group))
    splitters = weighted_splitters_t(g[:, :N_SAMPLES], g[:, N_SAMPLES], world)
    packable = torch.logical_and(g[:, N_SAMPLES + 1].min() >= 0, g[:, N_SAMPLES + 2].max() < (1 << 31))
    onodes = _ordered(nodes)
    e_counts = split_counts_t(ou.to(wire), splitters)
    n_counts = split_counts_t(onodes.to(wire), splitters)
    mine = torch.cat([e_counts, n_counts, packable.reshape(1).to(torch.int64)])
    cm = torch.stack(all_gather_tensor(mine, group)).cpu()         # (world, 2*world + 1): the host round trip
    packable = bool(cm[:, 2 * world].min().item())
    e_send = cm[rank, :world].tolist()
    n_send = cm[rank, world:2 * world].tolist()
    e_recv_all = cm[:, rank].tolist()
    n_recv = cm[:, world + rank].tolist()

    if not packable:
        # general labels: every row goes to the owner of its u and is merged there
        rows = pack_rows(keys, sums, recs)
        recv, nrecv = exchange_rows_nodes(rows, e_send, e_recv_all, nodes, n_send, n_recv, group)
        rk, rs, rr = unpack_rows(recv)
        me, mf = backend.merge(rk, rs, rr, hist_range)
        merged = {'edges': me, 'features': mf}
    else:
        # rows of other owners leave; this rank's own block stays in place
        lo_i = sum(e_send[:rank])
        hi_i = lo_i + e_send[rank]
        send = list(e_send)
        send[rank] = 0
        recv_counts = list(e_recv_all)
        recv_counts[rank] = 0
        out_k = torch.cat([keys[:lo_i], keys[hi_i:]])
        out_rows = pack_rows(out_k, torch.cat([sums[:lo_i], sums[hi_i:]]), torch.cat([recs[:lo_i], recs[hi_i:]]))
        recv, nrecv = exchange_rows_nodes(out_rows, send, recv_counts, nodes, n_send, n_recv, group)
        lk, ls, lr, lf = keys[lo_i:hi_i], sums[lo_i:hi_i], recs[lo_i:hi_i], feats[lo_i:hi_i]
        if recv.shape[0] == 0:
            shared = torch.zeros(lk.shape[0], dtype=torch.bool, device=dev)
        else:
            rk, rs, rr = unpack_rows(recv)
            shared = torch.isin(_pack_uv(lk), _pack_uv(rk))
        # local-only keys are final; with affinities a key must have been seen
        # on a nearest-neighbour face (ADJ bit of its wide record)
        keep = ~shared
        if offsets is not None:
            keep &= lr[:, 42] < 0
        if recv.shape[0] == 0:
            merged = {'edges': lk[keep], 'features': lf[keep]}
        else:
            me, mf = backend.merge(torch.cat([rk, lk[shared]]), torch.cat([rs, ls[shared]]),
                                   torch.cat([rr, lr[shared]]), hist_range)
            me = _tensor(me, lk)
            mf = _tensor(mf, lf)
            merged = _merge_sorted(lk[keep], lf[keep], me, mf)
    n_loc = int(merged['edges'].shape[0])

    # nodes went to the same ranges in the rows' all_to_all
    node_shard = backend.unique(nrecv)

    (e_off, e_tot), (n_off, n_tot) = _exclusive_offsets([n_loc, int(node_shard.shape[0])], group, dev)
    return DistResult(merged, node_shard, e_off, e_tot, n_off, n_tot, info)


def world_size_of(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1
