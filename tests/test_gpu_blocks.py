"""ctg_rag_blocks: the batched per-block path (one launch for a job's blocks)
against the oracle's per-block semantics:

* nodes_b  = unique labels of the inner block (test_graph.py:53-60)
* edges_b  = RAG of labels[max(begin-1,0):end] (test_graph.py:70-84)
* features = the block's owned samples for every edge of edges_b, count 0
  for edges seen only on faces the block does not own; affinities counted
  only for pairs in edges_b (block_edge_features.py:127-145).
"""
import numpy as np
import pytest

from cluster_tools_amd import rag
from cluster_tools_amd import synthetic as S
from cluster_tools_amd.blocking import blocking
from oracle import rag_oracle as O

from test_gpu_parity import check_features

pytestmark = pytest.mark.gpu


def _block_geometry(shape, block, halo_lo=(1, 1, 1), halo_hi=(0, 0, 0)):
    """Per block: array box [rb, re) (the ROI the ndist call reads), own box
    and graph box in array coordinates, the inner and outer global boxes."""
    blk = blocking([0, 0, 0], list(shape), list(block))
    out = []
    for b in range(blk.numberOfBlocks):
        bb = blk.getBlock(b)
        rb = [max(x - h, 0) for x, h in zip(bb.begin, halo_lo)]
        re_ = [min(y + h, s) for y, h, s in zip(bb.end, halo_hi, shape)]
        gb = [max(x - 1, 0) for x in bb.begin]
        own = ([x - r for x, r in zip(bb.begin, rb)], [y - r for y, r in zip(bb.end, rb)])
        graph = ([g - r for g, r in zip(gb, rb)], [y - r for y, r in zip(bb.end, rb)])
        out.append(dict(rb=rb, re=re_, own=own, graph=graph,
                        inner=tuple(slice(x, y) for x, y in zip(bb.begin, bb.end)),
                        outer=tuple(slice(g, y) for g, y in zip(gb, bb.end)),
                        roi=tuple(slice(x, y) for x, y in zip(rb, re_))))
    return out


def _expected_boundary(lab, bnd, g, ignore_label=False):
    eb = O.rag_edges(lab[g['outer']], ignore_label=ignore_label)
    sl = g['roi']
    e_own, f_own = O.boundary_features(lab[sl], bnd[sl], own_begin=g['own'][0], own_end=g['own'][1],
                                       ignore_label=ignore_label)
    f = np.zeros((eb.shape[0], 10))
    if e_own.shape[0]:
        rows = O.find_edges(eb, e_own)
        f[rows] = f_own
    return eb, f


@pytest.mark.parametrize('ignore_label', [False, True])
@pytest.mark.parametrize('label_shift', [0, 1 << 40])
def test_blocks_graph_matches_per_block_oracle(gpu, ignore_label, label_shift):
    shape, block = (26, 41, 70), (8, 16, 32)
    lab, _ = S.generate(shape, cell=5, seed=41, with_boundary=False)
    if ignore_label:
        lab = np.where(lab % 5 == 0, 0, lab).astype(np.uint64)
    lab = lab + np.where(lab > 0, np.uint64(label_shift), np.uint64(0)) if label_shift else lab
    geo = _block_geometry(shape, block)
    res = rag.rag_blocks([lab[g['roi']] for g in geo], [g['own'] for g in geo], [g['graph'] for g in geo],
                         ignore_label=ignore_label)
    assert len(res) == len(geo)
    for g, r in zip(geo, res):
        np.testing.assert_array_equal(r['nodes'], np.unique(lab[g['inner']]))
        np.testing.assert_array_equal(r['edges'], O.rag_edges(lab[g['outer']], ignore_label=ignore_label))


def test_blocks_ignore_label_dense_relabel_without_zero(gpu):
    """ignore_label=True, no label 0 anywhere, labels above the block tag's
    range (2^(32 - tag_bits)) and above 2^32: the batched call relabels the
    arena densely; the smallest real label must not become the ignore label
    (its edges would be dropped).  Same for the whole-volume call."""
    shape, block = (26, 41, 70), (8, 16, 32)
    lab, bnd = S.generate(shape, cell=5, seed=45)
    for shift in (np.uint64(1) << np.uint64(29), np.uint64(1) << np.uint64(40)):
        big = lab + shift                           # no zeros
        geo = _block_geometry(shape, block)
        res = rag.rag_blocks([big[g['roi']] for g in geo], [g['own'] for g in geo], [g['graph'] for g in geo],
                             data=[bnd[g['roi']] for g in geo], ignore_label=True)
        for g, r in zip(geo, res):
            np.testing.assert_array_equal(r['nodes'], np.unique(big[g['inner']]))
            eb, f = _expected_boundary(big, bnd, g, ignore_label=True)
            np.testing.assert_array_equal(r['edges'], eb)
            check_features(r['features'], f)
        out = rag.rag_features(big, bnd, ignore_label=True)
        e_ref, f_ref = O.boundary_features(big, bnd, ignore_label=True)
        np.testing.assert_array_equal(out['edges'], e_ref)
        check_features(out['features'], f_ref)


@pytest.mark.parametrize('dtype', ['float32', 'uint8'])
def test_blocks_boundary_features(gpu, dtype):
    shape, block = (30, 37, 66), (10, 16, 32)
    lab, bnd = S.generate(shape, cell=5, seed=42)
    data = bnd if dtype == 'float32' else np.round(bnd * 255).astype(np.uint8)
    geo = _block_geometry(shape, block)
    res = rag.rag_blocks([lab[g['roi']] for g in geo], [g['own'] for g in geo], [g['graph'] for g in geo],
                         data=[data[g['roi']] for g in geo], keep_stats=True)
    for g, r in zip(geo, res):
        eb, f = _expected_boundary(lab, data, g)
        np.testing.assert_array_equal(r['edges'], eb)
        check_features(r['features'], f)
        assert r['sums'].shape == (eb.shape[0], 2) and r['records'].shape == (eb.shape[0], 48)


@pytest.mark.parametrize('offsets', [S.NN_OFFSETS, S.LR_OFFSETS])
def test_blocks_affinity_features(gpu, offsets):
    shape, block = (28, 40, 44), (9, 20, 22)
    lab, bnd = S.generate(shape, cell=5, seed=43)
    affs = S.affinities_from_boundary(bnd, offsets)
    off = np.asarray(offsets)
    halo_lo = [max(1, int(max(0, -off[:, a].min()))) for a in range(3)]
    halo_hi = [int(max(0, off[:, a].max())) for a in range(3)]
    geo = _block_geometry(shape, block, halo_lo, halo_hi)
    res = rag.rag_blocks([lab[g['roi']] for g in geo], [g['own'] for g in geo], [g['graph'] for g in geo],
                         data=[affs[(slice(None),) + g['roi']] for g in geo], offsets=offsets)
    for g, r in zip(geo, res):
        eb = O.rag_edges(lab[g['outer']])
        np.testing.assert_array_equal(r['edges'], eb)
        sl = g['roi']
        if eb.shape[0] == 0:
            continue
        e_b, f_b = O.affinity_features(lab[sl], affs[(slice(None),) + sl], offsets, own_begin=g['own'][0],
                                       own_end=g['own'][1], edge_list=eb)
        np.testing.assert_array_equal(e_b, eb)
        check_features(r['features'], f_b)


def test_blocks_single_block_equals_whole_call(gpu):
    """One block covering the volume with the whole volume as own and graph
    box is the plain ctg_rag_features call."""
    lab, bnd = S.generate((20, 33, 45), cell=6, seed=44)
    full = ((0, 0, 0), lab.shape)
    r = rag.rag_blocks([lab], [full], [full], data=[bnd])[0]
    ref = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(r['edges'], ref['edges'])
    np.testing.assert_array_equal(r['nodes'], np.unique(lab))
    np.testing.assert_array_equal(r['features'][:, 9], ref['features'][:, 9])
    np.testing.assert_allclose(r['features'], ref['features'], rtol=1e-12, atol=1e-15)


def test_blocks_empty_and_uniform_blocks(gpu):
    """Blocks with a single label (no edge), and a zero-size own box."""
    lab = np.zeros((12, 12, 12), np.uint64) + 7
    lab[6:, :, :] = 9
    geo = _block_geometry(lab.shape, (4, 12, 12))
    res = rag.rag_blocks([lab[g['roi']] for g in geo], [g['own'] for g in geo], [g['graph'] for g in geo])
    assert [r['edges'].shape[0] for r in res] == [0, 1, 0]    # only the block with the z=5|6 face
    assert [list(r['nodes']) for r in res] == [[7], [7, 9], [9]]


@pytest.mark.parametrize('packed', ['1', '0'])
def test_blocks_independent_of_workspace_history(gpu, monkeypatch, packed):
    """The same batched affinity call after a large call has grown the
    workspace (record buffer of 2^22+ slots: 23 slot bits, which with the 32
    tagged u bits and 9 v bits would fill the packed sort key to bit 63)
    gives the result of a fresh process."""
    monkeypatch.setenv('CTG_SORT_PACKED', packed)
    lt, bt = rag.synth_volume((512, 512, 512), cell=10, seed=1)
    rag.rag_features_handle(lt, bt).free()
    del lt, bt
    test_blocks_affinity_features(None, S.NN_OFFSETS)
    test_blocks_affinity_features(None, S.LR_OFFSETS)
