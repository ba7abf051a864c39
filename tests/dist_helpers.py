"""Oracle-backed stand-in for dist.HipBackend, used by the gloo (CPU) tests of
the multi-GPU exchange logic.  Test infrastructure: it wraps oracle/ and the
wide-record layout of include/ctg.h (42 histogram slots, cnt|ADJ, ordered
min, ordered max, pad) so that the partition / all_to_all / merge code of
cluster_tools_amd/dist.py runs unchanged on CPU tensors.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import rag_oracle as O

WIDE = 48
ADJ = np.uint32(0x80000000)


def f2ord(x):
    b = np.asarray(x, dtype=np.float32).view(np.uint32)
    return np.where(b & np.uint32(0x80000000), ~b, b | np.uint32(0x80000000)).astype(np.uint32)


def ord2f(o):
    o = np.asarray(o, dtype=np.uint32)
    b = np.where(o & np.uint32(0x80000000), o & np.uint32(0x7FFFFFFF), ~o).astype(np.uint32)
    return b.view(np.float32)


def encode_stats(stats):
    """oracle _accumulate stats -> (sums (E,2) f64, records (E,48) u32): the
    shifted sums (S1, S2) about the pivot p = float32(mean) in word 45."""
    c = stats['count'].astype(np.float64)
    n = c.shape[0]
    with np.errstate(invalid='ignore', divide='ignore'):
        mean = np.where(c > 0, stats['sum'] / np.maximum(c, 1), 0.0)
    p = mean.astype(np.float32)
    sums = np.zeros((n, 2))
    sums[:, 0] = stats['sum'] - c * p.astype(np.float64)
    with np.errstate(invalid='ignore', divide='ignore'):
        sums[:, 1] = stats['m2'] + np.where(c > 0, sums[:, 0] ** 2 / np.maximum(c, 1), 0.0)
    rec = np.zeros((n, WIDE), dtype=np.uint32)
    rec[:, :O.NBINS + 2] = stats['hist'].astype(np.uint32)
    rec[:, 42] = stats['count'].astype(np.uint32) | ADJ
    rec[:, 43] = f2ord(stats['min'])
    rec[:, 44] = f2ord(stats['max'])
    rec[:, 45] = p.view(np.uint32)
    return sums, rec


def decode_stats(sums, rec):
    c = (rec[:, 42] & np.uint32(0x7FFFFFFF)).astype(np.int64)
    p = rec[:, 45].view(np.float32).astype(np.float64)
    s1 = sums[:, 0]
    with np.errstate(invalid='ignore', divide='ignore'):
        d = np.where(c > 0, s1 / np.maximum(c, 1), 0.0)
    mean = np.where(c > 0, p + d, 0.0)
    s = np.where(c > 0, mean * c, 0.0)
    m2 = sums[:, 1] - np.where(c > 0, s1 * d, 0.0)
    return dict(count=c, sum=s, mean=mean, m2=m2,
                min=ord2f(rec[:, 43]).astype(np.float64), max=ord2f(rec[:, 44]).astype(np.float64),
                hist=rec[:, :O.NBINS + 2].astype(np.int64))


SIGN = np.uint64(1 << 63)
S = 1024          # CTG_MGPU_SAMPLES
ROW = 28          # CTG_MGPU_ROW_WORDS


class Part:
    """A rank's partial table (the numpy twin of a CTG_KEEP_STATS result)."""

    def __init__(self, edges, feats, sums, rec, nodes, partial_adj):
        self.edges, self.feats, self.sums, self.rec, self.nodes = edges, feats, sums, rec, nodes
        self.partial_adj = partial_adj

    def info(self):
        return (0, 0)

    def free(self):
        pass


class NumpyShard:
    """The rag.Result accessors the distributed code and the tests use."""

    def __init__(self, edges, feats, nodes):
        self._e = np.ascontiguousarray(edges, dtype=np.uint64).reshape(-1, 2)
        self._f = np.ascontiguousarray(feats, dtype=np.float64).reshape(-1, O.N_FEATURES)
        self._n = np.ascontiguousarray(nodes, dtype=np.uint64).reshape(-1)

    n_edges = property(lambda self: self._e.shape[0])
    n_nodes = property(lambda self: self._n.shape[0])

    def edges(self):
        return self._e

    def features(self):
        return self._f

    def nodes(self):
        return self._n

    def edges_torch_i64(self):
        return torch.from_numpy(self._e.view(np.int64))

    def features_torch(self):
        return torch.from_numpy(self._f)

    def nodes_torch(self):
        return torch.from_numpy(self._n.view(np.int64))

    def free(self):
        pass


def splitters(meta_all, world):
    """Restatement of k_mgpu_splitters (ctg_mgpu.hip): sample j of rank r
    (value v) has the integer cumulative weight CW = sum_q count_q * c_q (c_q:
    samples of rank q at or before it in the (v, r, j) order); splitter k is
    the v whose interval (CW - count_r, CW] holds total * S * k / world."""
    m = np.asarray(meta_all, dtype=np.int64).reshape(world, S + 1)
    cnt = m[:, S].astype(np.uint64)
    total = int(cnt.sum())
    spl = np.zeros(max(world - 1, 0), dtype=np.uint64)
    for r in range(world):
        if cnt[r] == 0:
            continue
        v = m[r, :S]
        cw = np.zeros(S, dtype=object)
        for q in range(world):
            if cnt[q] == 0:
                continue
            row = m[q, :S]
            c = (np.searchsorted(row, v, side='right') if q < r else
                 np.searchsorted(row, v, side='left') if q > r else np.arange(1, S + 1))
            cw = cw + int(cnt[q]) * c.astype(object)
        for k in range(1, world):
            t = total * S * k
            hit = [(int(a) - int(cnt[r])) * world < t <= int(a) * world for a in cw]
            for j in np.nonzero(hit)[0]:
                spl[k - 1] = np.uint64(v[j]) ^ SIGN
    return spl


def split_counts(part, spl, world):
    """Restatement of k_mgpu_bounds: rows / node ids per rank's u range."""
    u = part.edges[:, 0] if part.edges.shape[0] else np.zeros(0, np.uint64)
    eb = [0] + [int(np.searchsorted(u, x, side='left')) for x in spl] + [u.shape[0]]
    nb = [0] + [int(np.searchsorted(part.nodes, x, side='left')) for x in spl] + [part.nodes.shape[0]]
    return np.array([[max(eb[d + 1] - eb[d], 0), max(nb[d + 1] - nb[d], 0)] for d in range(world)], np.int64)


class OracleBackend:
    """The four device steps of dist.py's exchange restated in numpy over the
    oracle's statistics (ctg_mgpu_sample / split / pack / merge)."""

    def local(self, labels, data, offsets, own_begin, own_end, ignore_label, hist_range):
        lab = np.asarray(labels)
        edges, feats, stats = O.boundary_features(lab, np.asarray(data), own_begin=own_begin,
                                                  ignore_label=ignore_label, lo=hist_range[0], hi=hist_range[1],
                                                  return_stats=True)
        sums, rec = encode_stats(stats)
        nodes = np.unique(edges.reshape(-1)).astype(np.uint64)
        return Part(edges.astype(np.uint64).reshape(-1, 2), np.ascontiguousarray(feats), sums, rec, nodes, False)

    def sample(self, part):
        E = part.edges.shape[0]
        meta = np.zeros(S + 1, dtype=np.int64)
        if E:
            idx = (np.arange(S, dtype=np.int64) * E) // S
            meta[:S] = (part.edges[idx, 0] ^ SIGN).view(np.int64)
        meta[S] = E
        return torch.from_numpy(meta)

    def split(self, part, meta_all, world):
        return torch.from_numpy(split_counts(part, splitters(meta_all.numpy(), world), world))

    def pack(self, part, counts_all, world, rank, words):
        c = np.asarray(counts_all).reshape(world, world, 2)[rank]
        e0 = np.concatenate([[0], np.cumsum(c[:, 0])])
        n0 = np.concatenate([[0], np.cumsum(c[:, 1])])
        out = []
        for d in range(world):
            if d == rank:
                continue
            a, b = e0[d], e0[d + 1]
            rows = np.concatenate([part.edges[a:b].view(np.int64), part.sums[a:b].view(np.int64),
                                   np.ascontiguousarray(part.rec[a:b]).view(np.int64)], axis=1)
            out.append(rows.reshape(-1))
            out.append(part.nodes[n0[d]:n0[d + 1]].view(np.int64))
        w = np.concatenate(out) if out else np.zeros(0, np.int64)
        assert w.shape[0] == words
        return torch.from_numpy(w)

    def merge(self, part, recv, counts_all, world, rank, hist_range):
        c = np.asarray(counts_all).reshape(world, world, 2)
        e_lo, n_lo = int(c[rank, :rank, 0].sum()), int(c[rank, :rank, 1].sum())
        e_cnt, n_cnt = int(c[rank, rank, 0]), int(c[rank, rank, 1])
        own_e, own_f = part.edges[e_lo:e_lo + e_cnt], part.feats[e_lo:e_lo + e_cnt]
        own_s, own_r = part.sums[e_lo:e_lo + e_cnt], part.rec[e_lo:e_lo + e_cnt]
        rk, rs, rr, rn = [], [], [], []
        w = recv.numpy() if recv is not None else np.zeros(0, np.int64)
        off = 0
        for q in range(world):
            if q == rank:
                continue
            nr, nn = int(c[q, rank, 0]), int(c[q, rank, 1])
            rows = w[off:off + nr * ROW].reshape(nr, ROW)
            rk.append(rows[:, :2].view(np.uint64))
            rs.append(rows[:, 2:4].copy().view(np.float64))
            rr.append(np.ascontiguousarray(rows[:, 4:]).view(np.uint32).reshape(nr, WIDE))
            rn.append(w[off + nr * ROW:off + nr * ROW + nn].view(np.uint64))
            off += nr * ROW + nn
        nodes = part.nodes[n_lo:n_lo + n_cnt]
        if rn and sum(x.shape[0] for x in rn):
            nodes = np.unique(np.concatenate([nodes] + rn))
        M = sum(x.shape[0] for x in rk)
        if M == 0 and not part.partial_adj:
            return NumpyShard(own_e, own_f, nodes)
        keys = np.concatenate([own_e] + rk)
        sums = np.concatenate([own_s] + rs)
        rec = np.concatenate([own_r] + rr)
        edges, inv = O._unique_pairs(keys, return_inverse=True)
        st = decode_stats(sums, rec)
        merged = O.merge_feature_stats([(inv, st)], edges.shape[0], hist_range[0], hist_range[1])
        feats = O.finalize_features(merged, hist_range[0], hist_range[1])
        touched = np.zeros(edges.shape[0], bool)
        touched[inv[e_cnt:]] = True
        keep_own = ~touched[inv[:e_cnt]]
        feats[inv[:e_cnt][keep_own]] = own_f[keep_own]     # untouched own rows: the local call's features
        adj = np.zeros(edges.shape[0], bool)
        np.logical_or.at(adj, inv, (rec[:, 42] & ADJ) != 0)
        keep = adj if part.partial_adj else np.ones(edges.shape[0], bool)
        return NumpyShard(edges[keep], feats[keep], nodes)
