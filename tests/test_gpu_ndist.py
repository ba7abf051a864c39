"""The nifty.distributed mirror end to end on N5 containers (GPU).

Re-expresses the reference's hot-path tests without CREMI data, nifty or
luigi: the job bodies' call sequence of graph/initial_sub_graphs.py,
merge_sub_graphs.py, map_edge_ids.py, features/block_edge_features.py and
merge_edge_features.py, with the assertions of test/graph/test_graph.py:27-115
(per block and whole volume) and test/features/test_edge_features.py:32-77
(whole-volume features), checked against the oracle.
"""
import numpy as np
import pytest

from cluster_tools_amd import n5, ndist
from cluster_tools_amd import synthetic as S
from cluster_tools_amd.blocking import blocking
from oracle import rag_oracle as O

from test_gpu_parity import check_features

pytestmark = pytest.mark.gpu

SHAPE = (24, 40, 36)
BLOCK = (8, 16, 16)


def _setup(tmp_path, lab, data=None, ignore_label=False):
    p = str(tmp_path / 'data.n5')
    with n5.File(p) as f:
        f.create_dataset('seg', data=lab, chunks=BLOCK, compression='gzip')
        if data is not None:
            ch = BLOCK if data.ndim == 3 else (1,) + BLOCK
            f.create_dataset('bnd', data=data, chunks=ch, compression='gzip')
        # initial_sub_graphs.py:64-75 (the task creates the datasets)
        g = f.require_group('s0/sub_graphs')
        g.attrs['shape'] = list(lab.shape)
        g.attrs['ignore_label'] = bool(ignore_label)
        for k in ('nodes', 'edges', 'edge_ids'):
            g.require_dataset(k, shape=lab.shape, chunks=BLOCK, dtype='uint64', compression='gzip')
    return p


def _graph(p, ignore_label):
    blk = blocking([0, 0, 0], list(SHAPE), list(BLOCK))
    ids = list(range(blk.numberOfBlocks))
    for b in ids:
        bb = blk.getBlock(b)
        ndist.computeMergeableRegionGraph(p, 'seg', bb.begin, bb.end, p, 's0/sub_graphs', ignore_label,
                                          increaseRoi=True, serializeToVarlen=True)
    ndist.mergeSubgraphs(p, subgraphKey='s0/sub_graphs', blockIds=ids, outKey='graph', numberOfThreads=4,
                         serializeToVarlen=False)
    ndist.mapEdgeIds(p, 'graph', subgraphKey='s0/sub_graphs', blockIds=ids, numberOfThreads=4)
    return blk, ids


@pytest.mark.parametrize('ignore_label', [False, True])
def test_graph_workflow(gpu, tmp_path, ignore_label):
    lab, _ = S.generate(SHAPE, cell=5, seed=31, with_boundary=False)
    if ignore_label:
        lab = np.where(lab % 7 == 0, 0, lab).astype(np.uint64)
    p = _setup(tmp_path, lab, ignore_label=ignore_label)
    blk, ids = _graph(p, ignore_label)
    full = ndist.Graph(p, 'graph')
    with n5.File(p, 'r') as f:
        g = f['s0/sub_graphs']
        for b in ids:
            bb = blk.getBlock(b)
            pos = blk.blockGridPosition(b)
            inner = tuple(slice(x, y) for x, y in zip(bb.begin, bb.end))
            outer = tuple(slice(max(x - 1, 0), y) for x, y in zip(bb.begin, bb.end))
            nodes = g['nodes'].read_chunk(pos)
            np.testing.assert_array_equal(nodes, np.unique(lab[inner]))                  # test_graph.py:53-60
            edges = g['edges'].read_chunk(pos)
            ref = O.rag_edges(lab[outer], ignore_label=ignore_label)
            if edges is None:                                                              # :63-66
                assert ref.shape[0] == 0
                continue
            edges = edges.reshape(-1, 2)
            np.testing.assert_array_equal(edges, ref)                                     # :79-84
            if not ignore_label:
                np.testing.assert_array_equal(ndist.Graph(edges).nodes(), np.unique(lab[outer]))  # :70-77
            np.testing.assert_array_equal(g['edge_ids'].read_chunk(pos).astype(np.int64),
                                          full.findEdges(edges))                          # :89-93
        gr = f['graph']
        assert gr.attrs['numberOfEdges'] == full.numberOfEdges
    ref = O.rag_edges(lab, ignore_label=ignore_label)                                       # :95-115
    np.testing.assert_array_equal(full.uvIds(), ref)
    assert full.numberOfNodes == len(np.unique(lab))
    assert full.numberOfEdges == ref.shape[0]


def _features(p, ids, E, fn, *extra, **kw):
    with n5.File(p) as f:
        ds = f.require_dataset('s0/sub_features', shape=SHAPE, chunks=BLOCK, dtype='float64', compression='gzip')
        ds.attrs['n_features'] = 10
        f.require_dataset('features', shape=(E, 10), chunks=(min(262144, E), 1), dtype='float64',
                          compression='gzip')
    fn(p, 's0/sub_graphs', p, 'bnd', p, 'seg', ids, p, 's0/sub_features', *extra, **kw)
    # merge_edge_features.py:134-147: two jobs over edge-id ranges
    half = E // 2
    for b, e in ((0, half), (half, E)):
        ndist.mergeFeatureBlocks(p, 's0/sub_graphs', p, 's0/sub_features', p, 'features', blockIds=ids,
                                 edgeIdBegin=b, edgeIdEnd=e, numberOfThreads=2)
    with n5.File(p, 'r') as f:
        return f['features'][:]


@pytest.mark.parametrize('dtype', ['float32', 'uint8'])
def test_boundary_feature_workflow(gpu, tmp_path, dtype):
    lab, bnd = S.generate(SHAPE, cell=5, seed=32)
    data = bnd if dtype == 'float32' else np.round(bnd * 255).astype(np.uint8)
    p = _setup(tmp_path, lab, data)
    blk, ids = _graph(p, False)
    E = ndist.Graph(p, 'graph').numberOfEdges
    fn = (ndist.extractBlockFeaturesFromBoundaryMaps_float32 if dtype == 'float32'
          else ndist.extractBlockFeaturesFromBoundaryMaps_uint8)
    feats = _features(p, ids, E, fn, increaseRoi=True)
    e_ref, f_ref = O.boundary_features(lab, data)        # whole volume (test_edge_features.py:32-77)
    np.testing.assert_array_equal(ndist.Graph(p, 'graph').uvIds(), e_ref)
    check_features(feats, f_ref)


@pytest.mark.parametrize('offsets', [S.NN_OFFSETS, S.LR_OFFSETS])
def test_affinity_feature_workflow(gpu, tmp_path, offsets):
    lab, bnd = S.generate(SHAPE, cell=5, seed=33)
    affs = S.affinities_from_boundary(bnd, offsets)
    p = _setup(tmp_path, lab, affs)
    blk, ids = _graph(p, False)
    graph = ndist.Graph(p, 'graph')
    E = graph.numberOfEdges
    feats = _features(p, ids, E, ndist.extractBlockFeaturesFromAffinityMaps_float32, offsets)
    # oracle: per block, samples owned by the block and filtered by the
    # block's sub-graph (the ndist per-block semantics), merged over blocks
    off = np.asarray(offsets)
    halo_lo = [max(1, int(max(0, -off[:, a].min()))) for a in range(3)]
    halo_hi = [int(max(0, off[:, a].max())) for a in range(3)]
    parts = []
    with n5.File(p, 'r') as f:
        g = f['s0/sub_graphs']
        for b in ids:
            bb = blk.getBlock(b)
            pos = blk.blockGridPosition(b)
            eb = g['edges'].read_chunk(pos)
            if eb is None:
                continue
            eb = eb.reshape(-1, 2)
            rb = [max(x - h, 0) for x, h in zip(bb.begin, halo_lo)]
            re_ = [min(y + h, s) for y, h, s in zip(bb.end, halo_hi, SHAPE)]
            sl = tuple(slice(x, y) for x, y in zip(rb, re_))
            own_b = [x - r for x, r in zip(bb.begin, rb)]
            own_e = [y - r for y, r in zip(bb.end, rb)]
            e_b, _, st = O.affinity_features(lab[sl], affs[(slice(None),) + sl], offsets, own_begin=own_b,
                                             own_end=own_e, edge_list=eb, return_stats=True)
            parts.append((graph.findEdges(e_b), st))
    m = O.merge_feature_stats(parts, E)
    f_ref = O.finalize_features(m, 0.0, 1.0)
    check_features(feats, f_ref)
    if offsets == S.NN_OFFSETS:
        # nearest-neighbour offsets: every sample pair is adjacent and inside the
        # halo'd block, so the block path equals the whole-volume definition
        _, f_whole = O.affinity_features(lab, affs, offsets)
        check_features(feats, f_whole)


@pytest.mark.parametrize('serialize_edges', [False, True])
def test_serialize_merged_graph(gpu, tmp_path, serialize_edges):
    """Next-scale sub-graphs of the blockwise multicut (multicut/reduce_problem.py:247-258):
    nodes of every 2x block = the merged node labels of the scale-0 blocks inside it;
    with serializeEdges the mapped, self-loop-free, unique edges and their new ids."""
    lab, _ = S.generate(SHAPE, cell=5, seed=34, with_boundary=False)
    p = _setup(tmp_path, lab)
    blk, ids = _graph(p, False)
    full = ndist.Graph(p, 'graph')
    rng = np.random.default_rng(7)
    n_max = int(full.maxNodeId) + 1
    # a consecutive node labelling that merges nodes (reduce_problem.py:160-193)
    node_lab = np.unique(rng.integers(0, n_max // 3, n_max), return_inverse=True)[1].astype(np.uint64)
    new_uv_all = np.sort(node_lab[full.uvIds().astype(np.int64)], axis=1)
    live = new_uv_all[:, 0] != new_uv_all[:, 1]
    new_uv, inv = np.unique(new_uv_all[live], axis=0, return_inverse=True)
    edge_lab = np.full(full.numberOfEdges, np.iinfo(np.uint64).max, np.uint64)
    edge_lab[live] = inv.ravel()
    new_bs = [2 * b for b in BLOCK]
    nblk = blocking([0, 0, 0], list(SHAPE), new_bs)
    new_ids = list(range(nblk.numberOfBlocks))
    ndist.serializeMergedGraph(graphPath=p, graphBlockPrefix='s0/sub_graphs', shape=list(SHAPE),
                               blockShape=list(BLOCK), newBlockShape=new_bs, newBlockIds=new_ids,
                               nodeLabeling=node_lab, edgeLabeling=edge_lab, outPath=p,
                               graphOutPrefix='s1/sub_graphs', numberOfThreads=3,
                               serializeEdges=serialize_edges)
    with n5.File(p, 'r') as f:
        g = f['s1/sub_graphs']
        assert list(g['nodes'].chunks) == new_bs
        for b in new_ids:
            nb = nblk.getBlock(b)
            pos = nblk.blockGridPosition(b)
            inner = tuple(slice(x, y) for x, y in zip(nb.begin, nb.end))
            np.testing.assert_array_equal(g['nodes'].read_chunk(pos), np.unique(node_lab[np.unique(lab[inner])]))
            if not serialize_edges:
                continue
            parts = []
            for ob in blk.getBlockIdsOverlappingBoundingBox(nb.begin, nb.end):
                bb = blk.getBlock(int(ob))
                outer = tuple(slice(max(x - 1, 0), y) for x, y in zip(bb.begin, bb.end))
                e = O.rag_edges(lab[outer])
                if e.shape[0]:
                    parts.append(np.sort(node_lab[e.astype(np.int64)], axis=1))
            ref = np.concatenate(parts) if parts else np.zeros((0, 2), np.uint64)
            ref = ref[ref[:, 0] != ref[:, 1]]
            ref = np.unique(ref, axis=0) if ref.shape[0] else ref
            got = g['edges'].read_chunk(pos)
            if ref.shape[0] == 0:
                assert got is None
                continue
            got = got.reshape(-1, 2)
            np.testing.assert_array_equal(got, ref)
            rows = np.array([np.flatnonzero((new_uv == r).all(axis=1))[0] for r in ref], dtype=np.uint64)
            np.testing.assert_array_equal(g['edge_ids'].read_chunk(pos), rows)


def test_merge_subgraphs_next_scale_varlen(gpu, tmp_path):
    """n_scales=2: MergeSubGraphs at scale 1 (merge_sub_graphs.py:140-152,
    184-193) unites the 2x2x2 scale-0 blocks of every 2x block into one varlen
    chunk of s1/sub_graphs at that block's grid position.  The ids come in a
    shuffled order (the chunk position must not depend on it)."""
    lab, _ = S.generate(SHAPE, cell=5, seed=35, with_boundary=False)
    p = _setup(tmp_path, lab)
    blk, ids = _graph(p, False)
    bs1 = [2 * b for b in BLOCK]
    blk1 = blocking([0, 0, 0], list(SHAPE), bs1)
    with n5.File(p) as f:
        for k in ('nodes', 'edges'):   # merge_sub_graphs.py:42-50
            f.require_dataset('s1/sub_graphs/' + k, shape=SHAPE, chunks=bs1, compression='gzip', dtype='uint64')
    rng = np.random.default_rng(3)
    for b1 in range(blk1.numberOfBlocks):
        nb = blk1.getBlock(b1)
        old = blk.getBlockIdsInBoundingBox(roiBegin=nb.begin, roiEnd=nb.end, blockHalo=[0, 0, 0]).tolist()
        rng.shuffle(old)
        ndist.mergeSubgraphs(p, subgraphKey='s0/sub_graphs', blockIds=old, outKey='s1/sub_graphs',
                             serializeToVarlen=True)
    with n5.File(p, 'r') as f:
        g1 = f['s1/sub_graphs']
        for b1 in range(blk1.numberOfBlocks):
            nb = blk1.getBlock(b1)
            pos = blk1.blockGridPosition(b1)
            inner = tuple(slice(x, y) for x, y in zip(nb.begin, nb.end))
            np.testing.assert_array_equal(g1['nodes'].read_chunk(pos), np.unique(lab[inner]))
            # union of the scale-0 block sub-graphs = RAG faces with both voxels
            # in some old block's halo'd box
            parts = []
            for ob in blk.getBlockIdsInBoundingBox(nb.begin, nb.end).tolist():
                bb = blk.getBlock(int(ob))
                outer = tuple(slice(max(x - 1, 0), y) for x, y in zip(bb.begin, bb.end))
                e = O.rag_edges(lab[outer])
                if e.shape[0]:
                    parts.append(e)
            got = g1['edges'].read_chunk(pos)
            if not parts:
                assert got is None
                continue
            ref = np.unique(np.concatenate(parts), axis=0)
            np.testing.assert_array_equal(got.reshape(-1, 2), ref)


def test_merge_feature_blocks_reference_layout(gpu, tmp_path):
    """mergeFeatureBlocks on reference-layout sub_features (10 float64 columns,
    no statistics companion - what nifty writes): count / mean / pooled
    variance / min / max exact against the whole volume, quantiles exact for
    edges held by one block and count-weighted (within [min, max]) otherwise."""
    import shutil
    lab, bnd = S.generate(SHAPE, cell=5, seed=36)
    p = _setup(tmp_path, lab, bnd)
    blk, ids = _graph(p, False)
    E = ndist.Graph(p, 'graph').numberOfEdges
    exact = _features(p, ids, E, ndist.extractBlockFeaturesFromBoundaryMaps_float32, increaseRoi=True)
    shutil.rmtree(str(tmp_path / 'data.n5' / 's0' / 'sub_features_stats'))
    with n5.File(p) as f:
        f['features'][:] = np.zeros((E, 10))
    for b, e in ((0, E // 3), (E // 3, E)):
        ndist.mergeFeatureBlocks(p, 's0/sub_graphs', p, 's0/sub_features', p, 'features', blockIds=ids,
                                 edgeIdBegin=b, edgeIdEnd=e, numberOfThreads=2)
    with n5.File(p, 'r') as f:
        compat = f['features'][:]
        # edges with samples in exactly one block
        owners = np.zeros(E, np.int64)
        g = f['s0/sub_graphs']
        for b in ids:
            pos = blk.blockGridPosition(b)
            eid = g['edge_ids'].read_chunk(pos)
            rows = f['s0/sub_features'].read_chunk(pos)
            if eid is None:
                continue
            rows = rows.reshape(-1, 10)
            owners[eid[rows[:, 9] > 0].astype(np.int64)] += 1
    np.testing.assert_array_equal(compat[:, 9], exact[:, 9])
    np.testing.assert_allclose(compat[:, [0, 1]], exact[:, [0, 1]], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(compat[:, [2, 8]], exact[:, [2, 8]])
    one = owners == 1
    assert one.any() and (owners > 1).any()
    np.testing.assert_array_equal(compat[one, 3:8], exact[one, 3:8])
    assert np.all(compat[:, 3:8] >= compat[:, 2:3] - 1e-12) and np.all(compat[:, 3:8] <= compat[:, 8:9] + 1e-12)


def test_zarr_input_container(gpu, tmp_path):
    """Input labels in a zarr container (graph_workflow.py:17-20), sub-graphs
    in N5: the per-block graph equals the one from an N5 input."""
    lab, _ = S.generate(SHAPE, cell=5, seed=37, with_boundary=False)
    pz = str(tmp_path / 'in.zarr')
    with n5.file_reader(pz) as f:
        f.create_dataset('seg', data=lab, chunks=BLOCK, compression='gzip')
    pg = _setup(tmp_path, lab)
    blk = blocking([0, 0, 0], list(SHAPE), list(BLOCK))
    for b in range(blk.numberOfBlocks):
        bb = blk.getBlock(b)
        ndist.computeMergeableRegionGraph(pz, 'seg', bb.begin, bb.end, pg, 's0/sub_graphs', False,
                                          increaseRoi=True, serializeToVarlen=True)
    with n5.File(pg, 'r') as f:
        g = f['s0/sub_graphs']
        for b in range(blk.numberOfBlocks):
            bb = blk.getBlock(b)
            pos = blk.blockGridPosition(b)
            outer = tuple(slice(max(x - 1, 0), y) for x, y in zip(bb.begin, bb.end))
            ref = O.rag_edges(lab[outer])
            got = g['edges'].read_chunk(pos)
            if ref.shape[0] == 0:
                assert got is None
            else:
                np.testing.assert_array_equal(got.reshape(-1, 2), ref)


def test_graph_on_label_multiset_input(gpu, tmp_path):
    """test_graph.py:140-161: GraphWorkflow on a label-multiset dataset gives
    the graph of its argmax segmentation (per-block nodes / edges and the
    merged graph)."""
    from test_host import write_multiset_dataset
    lab, _ = S.generate(SHAPE, cell=5, seed=38, with_boundary=False)
    p = _setup(tmp_path, lab)
    with n5.File(p) as f:
        write_multiset_dataset(f, 'ms', lab, BLOCK)
    blk = blocking([0, 0, 0], list(SHAPE), list(BLOCK))
    ids = list(range(blk.numberOfBlocks))
    for b in ids:
        bb = blk.getBlock(b)
        ndist.computeMergeableRegionGraph(p, 'ms', bb.begin, bb.end, p, 's0/sub_graphs', False,
                                          increaseRoi=True, serializeToVarlen=True)
    ndist.mergeSubgraphs(p, subgraphKey='s0/sub_graphs', blockIds=ids, outKey='graph', numberOfThreads=2)
    with n5.File(p, 'r') as f:
        g = f['s0/sub_graphs']
        for b in ids:
            bb = blk.getBlock(b)
            pos = blk.blockGridPosition(b)
            np.testing.assert_array_equal(g['nodes'].read_chunk(pos),
                                          np.unique(lab[tuple(slice(x, y) for x, y in zip(bb.begin, bb.end))]))
    np.testing.assert_array_equal(ndist.Graph(p, 'graph').uvIds(), O.rag_edges(lab))


def test_number_of_nodes_literal_restatement(gpu, tmp_path):
    """test_graph.py:108-113 literally: on dense labels 0..max the merged
    graph's numberOfNodes equals gridRag's max + 1; per block (:79-81) the
    rag's max + 1 is >= the block graph's numberOfNodes.  With gaps in the
    labels numberOfNodes stays the distinct count."""
    lab, _ = S.generate(SHAPE, cell=5, seed=33, with_boundary=False)
    _, dense = np.unique(lab, return_inverse=True)
    dense = dense.reshape(lab.shape).astype(np.uint64)          # labels 0..n-1, every one present
    p = _setup(tmp_path, dense)
    blk, ids = _graph(p, False)
    full = ndist.Graph(p, 'graph')
    assert full.numberOfNodes == int(dense.max()) + 1               # :110-113
    with n5.File(p, 'r') as f:
        g = f['s0/sub_graphs']
        for b in ids:
            bb = blk.getBlock(b)
            edges = g['edges'].read_chunk(blk.blockGridPosition(b))
            if edges is None:
                continue
            outer = tuple(slice(max(x - 1, 0), y) for x, y in zip(bb.begin, bb.end))
            assert int(dense[outer].max()) + 1 >= ndist.Graph(edges.reshape(-1, 2)).numberOfNodes   # :79-81
    gapped = dense * 3 + 5                                          # same RAG, labels with gaps
    (tmp_path / 'gapped').mkdir()
    p2 = _setup(tmp_path / 'gapped', gapped)
    _graph(p2, False)
    g2 = ndist.Graph(p2, 'graph')
    assert g2.numberOfNodes == len(np.unique(gapped)) < int(gapped.max()) + 1
    assert g2.numberOfEdges == full.numberOfEdges
