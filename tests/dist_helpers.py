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


class OracleBackend:
    def local(self, labels, data, offsets, own_begin, own_end, ignore_label, hist_range):
        lab = np.asarray(labels)
        edges, feats, stats = O.boundary_features(lab, np.asarray(data), own_begin=own_begin,
                                                  ignore_label=ignore_label, lo=hist_range[0], hi=hist_range[1],
                                                  return_stats=True)
        sums, rec = encode_stats(stats)
        nodes = np.unique(edges.reshape(-1))
        return (torch.from_numpy(edges.astype(np.int64)), torch.from_numpy(sums),
                torch.from_numpy(rec.view(np.int32)), torch.from_numpy(nodes.astype(np.int64)), (0, 0),
                torch.from_numpy(np.ascontiguousarray(feats)))

    def merge(self, keys, sums, recs, hist_range):
        k = keys.numpy().astype(np.uint64)
        if k.shape[0] == 0:
            return torch.zeros((0, 2), dtype=torch.int64), torch.zeros((0, O.N_FEATURES), dtype=torch.float64)
        edges, inv = O._unique_pairs(k, return_inverse=True)
        rec = recs.numpy().view(np.uint32)
        st = decode_stats(sums.numpy(), rec)
        merged = O.merge_feature_stats([(inv, st)], edges.shape[0], hist_range[0], hist_range[1])
        feats = O.finalize_features(merged, hist_range[0], hist_range[1])
        # ctg_merge_stats keeps only keys with the ADJ bit on some row (need_adj):
        # the exchange's empty slots (keys (j, j), zero records) disappear here
        adj = np.zeros(edges.shape[0], bool)
        np.logical_or.at(adj, inv, (rec[:, 42] & ADJ) != 0)
        return (torch.from_numpy(edges[adj].astype(np.int64)),
                torch.from_numpy(np.ascontiguousarray(feats[adj])))

    def unique(self, values):
        """sorted unique ids in unsigned order (as ctg_unique_labels)"""
        u = np.unique(values.numpy().view(np.uint64))
        return torch.from_numpy(u.view(np.int64))
