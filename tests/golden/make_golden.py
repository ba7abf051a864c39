#!/usr/bin/env python
"""Generate the committed golden fixtures of the hot path.

The reference holds no golden vectors for this path and
nifty is not importable here, so the fixtures are:

* ``kats.json``: the hand-computed known-answer tests of SURVEY Appendix A.5
  (plus an affinity and an outlier KAT).  The expected numbers below are
  written by hand from the semantics (not produced by the oracle); this
  script asserts that the oracle reproduces them before writing them.
* ``volumes.npz``: small synthetic volumes (inputs) with the oracle's
  outputs for the cases the GPU parity tests replay: boundary float32 and
  uint8, ignore_label, owned sub-box, nearest-neighbour and long-range
  affinities, per-block sub-graphs.  Inputs for the long-range case are
  re-generated from ``cluster_tools_amd.synthetic`` (deterministic) and
  pinned by a SHA-256 of the arrays, which keeps the file small.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from cluster_tools_amd import synthetic as S  # noqa: E402
from oracle import rag_oracle as O  # noqa: E402

f32 = lambda x: float(np.float32(x))  # noqa: E731


def kats():
    """Hand-computed known answers.  Samples are float32."""
    out = []
    # KAT-1: one face, both voxel values are samples
    a, b = f32(0.2), f32(0.6)
    m = (a + b) / 2
    out.append(dict(name='kat1_sample_rule', labels=[[[1, 2]]], data=[[[0.2, 0.6]]],
                    edges=[[1, 2]], count=[2], mean=[m], var=[((a - m) ** 2 + (b - m) ** 2) / 2],
                    min=[a], max=[b]))
    # KAT-2: halo geometry, block shape (2,1,1)
    out.append(dict(name='kat2_halo', labels=[[[1]], [[1]], [[2]], [[2]]], block_shape=[2, 1, 1],
                    blocks=[dict(nodes=[1], edges=[], edge_ids=[]),
                            dict(nodes=[2], edges=[[1, 2]], edge_ids=[0])],
                    nodes=[1, 2], edges=[[1, 2]]))
    # KAT-3: halo-plane edge; features count the (1,2) face once
    D = [[[0.1, 0.3]], [[0.5, 0.7]]]
    d = [[f32(v) for v in row[0]] for row in D]
    pairs = {(1, 2): [d[0][0], d[0][1]], (1, 3): [d[0][0], d[1][0]], (2, 3): [d[0][1], d[1][1]]}
    out.append(dict(name='kat3_halo_plane', labels=[[[1, 2]], [[3, 3]]], data=D, block_shape=[1, 1, 2],
                    blocks=[dict(nodes=[1, 2], edges=[[1, 2]], edge_ids=[0]),
                            dict(nodes=[3], edges=[[1, 2], [1, 3], [2, 3]], edge_ids=[0, 1, 2])],
                    nodes=[1, 2, 3], edges=[[1, 2], [1, 3], [2, 3]],
                    count=[2, 2, 2], mean=[sum(v) / 2 for v in pairs.values()],
                    min=[min(v) for v in pairs.values()], max=[max(v) for v in pairs.values()]))
    # KAT-4: ignore label 0
    out.append(dict(name='kat4_ignore_label', labels=[[[0, 2]], [[3, 3]]], ignore_label=True,
                    edges=[[2, 3]], nodes=[0, 2, 3]))
    # KAT-5: quantiles of {0.05, 0.05, 0.95}, 40 bins on [0,1]
    x5, x95 = f32(0.05), f32(0.95)
    m_lo, m_hi = 40.0 * x5, 40.0 * x95      # keypoints in bin space: (m_lo,0) (3,2) (37,2) (m_hi,3)
    kp = [(m_lo, 0.0), (3.0, 2.0), (37.0, 2.0), (m_hi, 3.0)]

    def q(p):
        c = 3 * p
        for (t0, c0), (t1, c1) in zip(kp[:-1], kp[1:]):
            if c0 < c <= c1:
                return (t0 + (c - c0) / (c1 - c0) * (t1 - t0)) / 40.0
        raise AssertionError
    mean5 = (2 * x5 + x95) / 3
    out.append(dict(name='kat5_quantiles', labels=[[[1, 2]], [[1, 2]]], data=None,
                    samples=[0.05, 0.05, 0.95], count=[3], mean=[mean5],
                    var=[(2 * (x5 - mean5) ** 2 + (x95 - mean5) ** 2) / 3],
                    quantiles=[x5, q(0.1), q(0.25), q(0.5), q(0.75), q(0.9), x95]))
    # KAT-6: affinities, NN offsets: only the x channel at x=1 has q inside
    out.append(dict(name='kat6_affinity', labels=[[[1, 2]]], offsets=[[-1, 0, 0], [0, -1, 0], [0, 0, -1]],
                    affs=[[[[0.9, 0.8]]], [[[0.7, 0.6]]], [[[0.5, 0.25]]]],
                    edges=[[1, 2]], count=[1], mean=[0.25], min=[0.25], max=[0.25]))
    # KAT-7: histogram outliers: samples -0.5 and 1.5 on [0,1]
    out.append(dict(name='kat7_outliers', labels=[[[1, 2]]], data=[[[-0.5, 1.5]]],
                    edges=[[1, 2]], count=[2], mean=[0.5], var=[1.0], min=[-0.5], max=[1.5],
                    slots_left=1, slots_right=1))
    return out


def check_kats_with_oracle(ks):
    for k in ks:
        L = np.asarray(k['labels'], dtype=np.uint64)
        if k['name'] == 'kat5_quantiles':
            v = np.asarray(k['samples'], np.float32)
            st = O._accumulate(np.zeros(3, np.int64), v, 1, 0.0, 1.0)
            f = O.finalize_features(st, 0.0, 1.0)[0]
            np.testing.assert_allclose(f[2:9], k['quantiles'], rtol=0, atol=1e-12)
            np.testing.assert_allclose([f[0], f[1], f[9]], [k['mean'][0], k['var'][0], 3], rtol=1e-12)
            continue
        if 'offsets' in k:
            e, f = O.affinity_features(L, np.asarray(k['affs'], np.float32), k['offsets'])
        elif k.get('data') is not None:
            e, f = O.boundary_features(L, np.asarray(k['data'], np.float32))
        else:
            e = O.rag_edges(L, ignore_label=k.get('ignore_label', False))
            f = None
        np.testing.assert_array_equal(e, np.asarray(k['edges'], np.uint64).reshape(-1, 2))
        if f is not None:
            np.testing.assert_array_equal(f[:, 9], k['count'])
            np.testing.assert_allclose(f[:, 0], k['mean'], rtol=1e-12)
            np.testing.assert_allclose(f[:, 2], k['min'], rtol=1e-12)
            np.testing.assert_allclose(f[:, 8], k['max'], rtol=1e-12)
            if 'var' in k:
                np.testing.assert_allclose(f[:, 1], k['var'], rtol=1e-9, atol=1e-15)
        if 'blocks' in k:
            blocks = O.blocking_blocks(L.shape, k['block_shape'])
            sub_e = []
            for (pos, b, end), want in zip(blocks, k['blocks']):
                n, eb = O.block_subgraph(L, b, end)
                np.testing.assert_array_equal(n, want['nodes'])
                np.testing.assert_array_equal(eb, np.asarray(want['edges'], np.uint64).reshape(-1, 2))
                sub_e.append(eb)
            nodes, edges = O.merge_subgraphs([O.block_subgraph(L, b, e)[0] for _, b, e in blocks], sub_e)
            np.testing.assert_array_equal(nodes, k['nodes'])
            np.testing.assert_array_equal(edges, np.asarray(k['edges'], np.uint64).reshape(-1, 2))
            for eb, want in zip(sub_e, k['blocks']):
                np.testing.assert_array_equal(O.find_edges(edges, eb), want['edge_ids'])


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def volume_cases():
    out = {}
    # boundary float32
    lab, bnd = S.generate((12, 16, 14), cell=4, seed=11)
    e, f = O.boundary_features(lab, bnd)
    out.update(bf_labels=lab, bf_data=bnd, bf_edges=e, bf_feats=f, bf_nodes=O.unique_labels(lab))
    # boundary uint8 (value / 255)
    u8 = np.round(bnd * 255).astype(np.uint8)
    e, f = O.boundary_features(lab, u8)
    out.update(bu_data=u8, bu_edges=e, bu_feats=f)
    # ignore_label: label 0 on every fifth supervoxel
    lab0 = np.where(lab % 5 == 0, 0, lab).astype(np.uint64)
    e, f = O.boundary_features(lab0, bnd, ignore_label=True)
    out.update(ig_labels=lab0, ig_edges=e, ig_feats=f, ig_nodes=O.unique_labels(lab0))
    # owned sub-box (block with halo inside a larger array)
    ob, oe = (1, 2, 3), (10, 13, 12)
    e, f = O.boundary_features(lab, bnd, own_begin=ob, own_end=oe)
    out.update(ob_begin=np.array(ob), ob_end=np.array(oe), ob_edges=e, ob_feats=f)
    # nearest-neighbour affinities, 3 channels
    nn = np.asarray(S.NN_OFFSETS)
    affs = S.affinities_from_boundary(bnd, nn)
    e, f = O.affinity_features(lab, affs, nn)
    out.update(nn_offsets=nn, nn_affs=affs, nn_edges=e, nn_feats=f)
    # long-range affinities, 12 channels (inputs regenerated, pinned by hash)
    lr = np.asarray(S.LR_OFFSETS)
    lab2, bnd2 = S.generate((10, 32, 32), cell=4, seed=5)
    affs2 = S.affinities_from_boundary(bnd2, lr)
    e, f = O.affinity_features(lab2, affs2, lr)
    out.update(lr_offsets=lr, lr_sha=np.array(sha(lab2, affs2)), lr_edges=e, lr_feats=f)
    # per-block sub-graphs, block shape (4,8,8)
    bs = (4, 8, 8)
    blocks = O.blocking_blocks(lab.shape, bs)
    nodes_b, edges_b = [], []
    for _, b, en in blocks:
        n, eb = O.block_subgraph(lab, b, en)
        nodes_b.append(n)
        edges_b.append(eb)
    out['blk_shape'] = np.array(bs)
    out['blk_nodes_len'] = np.array([len(n) for n in nodes_b])
    out['blk_nodes'] = np.concatenate(nodes_b)
    out['blk_edges_len'] = np.array([len(e) for e in edges_b])
    out['blk_edges'] = np.concatenate(edges_b, axis=0)
    return out


def main():
    ks = kats()
    check_kats_with_oracle(ks)
    with open(os.path.join(HERE, 'kats.json'), 'w') as fh:
        json.dump(ks, fh, indent=1)
    vol = volume_cases()
    np.savez_compressed(os.path.join(HERE, 'volumes.npz'), **vol)
    print('wrote kats.json (%d KATs) and volumes.npz (%d arrays)' % (len(ks), len(vol)))


if __name__ == '__main__':
    main()
