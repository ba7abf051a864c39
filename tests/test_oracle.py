"""The oracle against the golden fixtures (CPU only).

* KATs (tests/golden/kats.json, hand-computed): numpy oracle and
  C oracle both reproduce them.
* volumes.npz: regenerating every case with the oracle reproduces the
  committed outputs (pins the oracle and the deterministic generator).
* numpy restatement == C restatement on synthetic volumes (two independent
  restatements of the same semantics).
* the reference tests' structural assertions (test_graph.py:27-115) hold for
  the oracle's per-block sub-graphs and merge.
"""
import json
import os

import numpy as np
import pytest

from cluster_tools_amd import synthetic as S
from oracle import c_oracle
from oracle import rag_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load_kats():
    with open(os.path.join(GOLD, 'kats.json')) as fh:
        return {k['name']: k for k in json.load(fh)}


@pytest.fixture(scope='module')
def vol():
    return dict(np.load(os.path.join(GOLD, 'volumes.npz')))


def _check_feats(f, k):
    np.testing.assert_array_equal(f[:, 9], k['count'])
    np.testing.assert_allclose(f[:, 0], k['mean'], rtol=1e-12)
    np.testing.assert_allclose(f[:, 2], k['min'], rtol=1e-12)
    np.testing.assert_allclose(f[:, 8], k['max'], rtol=1e-12)
    if 'var' in k:
        np.testing.assert_allclose(f[:, 1], k['var'], rtol=1e-9, atol=1e-15)


@pytest.mark.parametrize('impl', ['numpy', 'c'])
@pytest.mark.parametrize('name', ['kat1_sample_rule', 'kat3_halo_plane', 'kat7_outliers'])
def test_boundary_kats(impl, name):
    k = load_kats()[name]
    L = np.asarray(k['labels'], np.uint64)
    D = np.asarray(k['data'], np.float32)
    e, f = (O.boundary_features(L, D) if impl == 'numpy' else c_oracle.features(L, D))
    np.testing.assert_array_equal(e, np.asarray(k['edges'], np.uint64))
    _check_feats(f, k)


@pytest.mark.parametrize('impl', ['numpy', 'c'])
def test_affinity_kat(impl):
    k = load_kats()['kat6_affinity']
    L = np.asarray(k['labels'], np.uint64)
    A = np.asarray(k['affs'], np.float32)
    e, f = (O.affinity_features(L, A, k['offsets']) if impl == 'numpy'
            else c_oracle.features(L, A, offsets=k['offsets']))
    np.testing.assert_array_equal(e, np.asarray(k['edges'], np.uint64))
    _check_feats(f, k)


def test_quantile_kat():
    k = load_kats()['kat5_quantiles']
    st = O._accumulate(np.zeros(3, np.int64), np.asarray(k['samples'], np.float32), 1, 0.0, 1.0)
    f = O.finalize_features(st, 0.0, 1.0)[0]
    np.testing.assert_allclose(f[2:9], k['quantiles'], rtol=0, atol=1e-12)
    # the same samples as faces through the C oracle: L=[[1,2],[1,2]] gives
    # 2 x-faces -> 4 samples; check the KAT through vigra_quantiles directly
    slots = O.histogram_slots(np.asarray(k['samples'], np.float32), 0.0, 1.0)
    h = np.bincount(slots, minlength=42)
    q = O.vigra_quantiles(h, np.float32(0.05), np.float32(0.95), 3, 0.0, 1.0)
    np.testing.assert_allclose(q, k['quantiles'], rtol=0, atol=1e-12)


def test_outlier_slots():
    s = O.histogram_slots(np.array([-0.5, 0.0, 0.999, 1.0, 1.5, -0.01], np.float32), 0.0, 1.0)
    # -0.5 -> left, 0 -> bin 0, 0.999 -> bin 39, 1.0 -> bin 39 (m == nbins), 1.5 -> right,
    # -0.01 -> m = -0.4 truncates to 0 -> bin 0 (vigra's (int) cast)
    assert list(s) == [0, 1, 40, 40, 41, 1]


def test_graph_kats():
    ks = load_kats()
    for name in ('kat2_halo', 'kat3_halo_plane'):
        k = ks[name]
        L = np.asarray(k['labels'], np.uint64)
        blocks = O.blocking_blocks(L.shape, k['block_shape'])
        sub_n, sub_e = [], []
        for (_, b, e), want in zip(blocks, k['blocks']):
            n, eb = O.block_subgraph(L, b, e)
            np.testing.assert_array_equal(n, want['nodes'])
            np.testing.assert_array_equal(eb, np.asarray(want['edges'], np.uint64).reshape(-1, 2))
            sub_n.append(n)
            sub_e.append(eb)
        nodes, edges = O.merge_subgraphs(sub_n, sub_e)
        np.testing.assert_array_equal(nodes, k['nodes'])
        np.testing.assert_array_equal(edges, np.asarray(k['edges'], np.uint64))
        for eb, want in zip(sub_e, k['blocks']):
            np.testing.assert_array_equal(O.find_edges(edges, eb), want['edge_ids'])
    k = ks['kat4_ignore_label']
    L = np.asarray(k['labels'], np.uint64)
    np.testing.assert_array_equal(O.rag_edges(L, ignore_label=True), np.asarray(k['edges'], np.uint64))
    np.testing.assert_array_equal(O.unique_labels(L), k['nodes'])


def test_golden_volumes_reproduce(vol):
    lab, bnd = vol['bf_labels'], vol['bf_data']
    lab2, bnd2 = S.generate(lab.shape, cell=4, seed=11)
    np.testing.assert_array_equal(lab, lab2)
    np.testing.assert_array_equal(bnd, bnd2)
    e, f = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(e, vol['bf_edges'])
    np.testing.assert_array_equal(f, vol['bf_feats'])
    e, f = O.boundary_features(lab, vol['bu_data'])
    np.testing.assert_array_equal(e, vol['bu_edges'])
    np.testing.assert_array_equal(f, vol['bu_feats'])
    e, f = O.boundary_features(vol['ig_labels'], bnd, ignore_label=True)
    np.testing.assert_array_equal(e, vol['ig_edges'])
    np.testing.assert_array_equal(f, vol['ig_feats'])
    assert not (vol['ig_edges'] == 0).any() and (vol['ig_nodes'] == 0).any()
    e, f = O.boundary_features(lab, bnd, own_begin=tuple(vol['ob_begin']), own_end=tuple(vol['ob_end']))
    np.testing.assert_array_equal(e, vol['ob_edges'])
    np.testing.assert_array_equal(f, vol['ob_feats'])
    e, f = O.affinity_features(lab, vol['nn_affs'], vol['nn_offsets'])
    np.testing.assert_array_equal(e, vol['nn_edges'])
    np.testing.assert_array_equal(f, vol['nn_feats'])


def test_golden_long_range_inputs_pinned(vol):
    import hashlib
    lab2, bnd2 = S.generate((10, 32, 32), cell=4, seed=5)
    affs2 = S.affinities_from_boundary(bnd2, vol['lr_offsets'])
    h = hashlib.sha256()
    for a in (lab2, affs2):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == str(vol['lr_sha'])
    e, f = O.affinity_features(lab2, affs2, vol['lr_offsets'])
    np.testing.assert_array_equal(e, vol['lr_edges'])
    np.testing.assert_array_equal(f, vol['lr_feats'])


def test_golden_block_subgraphs(vol):
    lab = vol['bf_labels']
    blocks = O.blocking_blocks(lab.shape, tuple(vol['blk_shape']))
    no = np.concatenate([[0], np.cumsum(vol['blk_nodes_len'])])
    eo = np.concatenate([[0], np.cumsum(vol['blk_edges_len'])])
    sub_n, sub_e = [], []
    for i, (_, b, e) in enumerate(blocks):
        n, eb = O.block_subgraph(lab, b, e)
        np.testing.assert_array_equal(n, vol['blk_nodes'][no[i]:no[i + 1]])
        np.testing.assert_array_equal(eb, vol['blk_edges'][eo[i]:eo[i + 1]])
        # test_graph.py:70-77: Graph(edges).nodes() == unique(seg[outer.begin:inner.end])
        outer = tuple(slice(max(x - 1, 0), y) for x, y in zip(b, e))
        if len(eb):
            np.testing.assert_array_equal(np.unique(eb), np.unique(lab[outer]))
        sub_n.append(n)
        sub_e.append(eb)
    # test_graph.py:95-115: merged graph == whole-volume RAG
    nodes, edges = O.merge_subgraphs(sub_n, sub_e)
    np.testing.assert_array_equal(edges, O.rag_edges(lab))
    np.testing.assert_array_equal(nodes, O.unique_labels(lab))


@pytest.mark.parametrize('shape,cell,seed', [((9, 21, 17), 4, 2), ((16, 16, 40), 6, 7)])
def test_numpy_vs_c_oracle(shape, cell, seed):
    lab, bnd = S.generate(shape, cell=cell, seed=seed)
    e1, f1 = O.boundary_features(lab, bnd)
    e2, f2 = c_oracle.features(lab, bnd)
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_allclose(f1, f2, rtol=1e-12, atol=1e-14)
    e1, f1 = O.boundary_features(lab, bnd, own_begin=(1, 0, 0), ignore_label=True)
    e2, f2 = c_oracle.features(lab, bnd, own_begin=(1, 0, 0), ignore_label=True)
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_allclose(f1, f2, rtol=1e-12, atol=1e-14)
    lr = np.asarray(S.LR_OFFSETS)
    affs = S.affinities_from_boundary(bnd, lr)
    e1, f1 = O.affinity_features(lab, affs, lr)
    e2, f2 = c_oracle.features(lab, affs, offsets=lr)
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_allclose(f1, f2, rtol=1e-12, atol=1e-14)


def test_merge_of_partials_is_exact():
    """Splitting the faces into two owned halves and merging the statistics
    reproduces the whole-volume features (the mergeFeatureBlocks rule)."""
    lab, bnd = S.generate((14, 20, 18), cell=5, seed=4)
    e_all, f_all = O.boundary_features(lab, bnd)
    # z in [0,7) faces (upper voxel z<7) and [7,14)
    e1, _, s1 = O.boundary_features(lab[:7], bnd[:7], return_stats=True)
    e2, _, s2 = O.boundary_features(lab[6:], bnd[6:], own_begin=(1, 0, 0), return_stats=True)
    m = O.merge_feature_stats([(O.find_edges_fast(e_all, e1), s1), (O.find_edges_fast(e_all, e2), s2)],
                              e_all.shape[0])
    f = O.finalize_features(m, 0.0, 1.0)
    np.testing.assert_allclose(f, f_all, rtol=1e-10, atol=1e-13)
