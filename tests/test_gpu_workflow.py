"""GraphWorkflow + EdgeFeaturesWorkflow end to end (harness/workflow.py:
the reference's job bodies on job threads, N5 in -> N5 out), against the
whole-volume call: BASELINE configs[0] geometry (125 x 1250 x 1250 with
64 x 256 x 256 blocks, SURVEY 8(d)'s offline substitute) and small volumes
with boundary maps and affinities.

The merged graph equals the whole-volume RAG bit for bit (test_graph.py:95-115),
the merged features the whole-volume features (mean / var / min / max to
1e-5, counts and quantiles exact: the block statistics merge their
histograms), nodes = unique labels.
"""
import numpy as np
import pytest

from cluster_tools_amd import n5, rag
from harness import workflow
from cluster_tools_amd import synthetic as S
from oracle import rag_oracle as O

from test_gpu_parity import check_features

pytestmark = pytest.mark.gpu


def _write_inputs(path, lab, data, block, level=1):
    comp = {'type': 'gzip', 'level': level, 'useZlib': False}
    with n5.File(path) as f:
        ds = f.create_dataset('seg', shape=lab.shape, chunks=block, dtype='uint64', compression=comp)
        ds.n_threads = 16
        ds[:] = lab
        ch = block if data.ndim == 3 else (data.shape[0],) + tuple(block)
        ds = f.create_dataset('bnd', shape=data.shape, chunks=ch, dtype=data.dtype, compression=comp)
        ds.n_threads = 16
        ds[:] = data


def _run(tmp_path, lab, data, block, offsets=None, max_jobs=4, max_jobs_merge=2, mode='threads'):
    inp = str(tmp_path / 'in.n5')
    out = str(tmp_path / 'out.n5')
    _write_inputs(inp, lab, data, block)
    t = workflow.graph_workflow(inp, 'seg', out, 'graph', block, max_jobs=max_jobs, mode=mode)
    workflow.edge_features_workflow(inp, 'bnd', inp, 'seg', out, 'graph', out, 'features', block,
                                    max_jobs=max_jobs, max_jobs_merge=max_jobs_merge, offsets=offsets, timer=t,
                                    mode=mode)
    with n5.File(out, 'r') as f:
        g = f['graph']
        edges, nodes, feats = g['edges'][:], g['nodes'][:], f['features'][:]
        assert g.attrs['numberOfEdges'] == edges.shape[0] and g.attrs['numberOfNodes'] == nodes.shape[0]
        assert list(g.attrs['shape']) == list(lab.shape)
    return edges, nodes, feats, t


@pytest.mark.parametrize('dtype,mode', [('float32', 'threads'), ('uint8', 'threads'), ('float32', 'processes')])
def test_workflow_boundary_small(gpu, tmp_path, dtype, mode):
    """mode 'processes': every job a spawned process, as LocalTask runs them
    (3 job processes at a time beside the test process)."""
    lab, bnd = S.generate((40, 70, 90), cell=6, seed=51)
    data = bnd if dtype == 'float32' else np.round(bnd * 255).astype(np.uint8)
    edges, nodes, feats, _ = _run(tmp_path, lab, data, (16, 32, 32), max_jobs=3, mode=mode)
    e_ref, f_ref = O.boundary_features(lab, data)
    np.testing.assert_array_equal(edges, e_ref)
    np.testing.assert_array_equal(nodes, np.unique(lab))
    check_features(feats, f_ref)


def test_workflow_affinities_small(gpu, tmp_path):
    lab, bnd = S.generate((36, 60, 64), cell=6, seed=52)
    affs = S.affinities_from_boundary(bnd, S.NN_OFFSETS)
    edges, nodes, feats, _ = _run(tmp_path, lab, affs, (12, 32, 32), offsets=S.NN_OFFSETS)
    e_ref, f_ref = O.affinity_features(lab, affs, S.NN_OFFSETS)
    np.testing.assert_array_equal(edges, e_ref)
    check_features(feats, f_ref)


@pytest.mark.timeout(400)
def test_workflow_configs0_geometry(gpu, tmp_path):
    """BASELINE configs[0]: 125 x 1250 x 1250, 64 x 256 x 256 blocks (50
    blocks), N5 (gzip) in -> N5 out, against an independent torch
    recomputation of the whole volume (test_gpu_fullsize: every boundary
    face enumerated by torch comparisons; counts, two-pass moments, min / max,
    and the exact histograms of a 20 k-edge sample for the quantiles) -- not
    against the library's own whole-volume call."""
    torch = pytest.importorskip('torch')
    from test_gpu_fullsize import _check, _check_quantiles, _reference_boundary
    shape, block = (125, 1250, 1250), (64, 256, 256)
    lt, bt = rag.synth_volume(shape, cell=10, seed=0)
    ref, (inv, x) = _reference_boundary(lt, bt, with_samples=True)
    lab = lt.cpu().numpy().view(np.uint64)
    bnd = bt.cpu().numpy()
    del lt, bt
    torch.cuda.empty_cache()
    edges, nodes, feats, t = _run(tmp_path, lab, bnd, block, max_jobs=16, max_jobs_merge=4)
    np.testing.assert_array_equal(nodes, np.unique(lab))

    class _Read:   # the N5 outputs in the result-handle shape _check reads
        def edges_torch_i64(self):
            return torch.from_numpy(edges.view(np.int64)).cuda()

        def features_torch(self):
            return torch.from_numpy(feats).cuda()
    _check(_Read(), *ref)
    _check_quantiles(_Read().features_torch(), inv, x, seed=2)
    print('configs[0] stages (s):', {k: round(v, 3) for k, v in t.stages.items()})


def test_rag_blocks_concurrent_threads_are_deterministic(gpu):
    """Job threads share the library (calls are serialised per device): four
    threads running batched affinity / boundary calls at once give the same
    results as one thread, call after call."""
    from concurrent.futures import ThreadPoolExecutor
    lab, bnd = S.generate((36, 60, 64), cell=6, seed=53)
    affs = S.affinities_from_boundary(bnd, S.NN_OFFSETS)
    own = [((1, 1, 1), (13, 31, 33)), ((0, 0, 0), (12, 30, 32))]
    graph = [((0, 0, 0), (13, 31, 33)), ((0, 0, 0), (12, 30, 32))]
    arrays = [lab[11:24, 29:60, 31:64], lab[:12, :30, :32]]
    data = [affs[:, 11:24, 29:60, 31:64], affs[:, :12, :30, :32]]

    def run(i):
        if i % 2:
            return rag.rag_blocks(arrays, own, graph, data=[bnd[11:24, 29:60, 31:64], bnd[:12, :30, :32]])
        return rag.rag_blocks(arrays, own, graph, data=data, offsets=S.NN_OFFSETS, keep_stats=True)
    ref = [run(0), run(1)]
    with ThreadPoolExecutor(4) as ex:
        outs = list(ex.map(run, range(16)))
    def moments(d):   # (mean, M2) from the shifted sums about the record's pivot (word 45)
        n = (d['records'][:, 42] & 0x7FFFFFFF).astype(np.float64)
        p = d['records'][:, 45].view(np.float32).astype(np.float64)
        s1, s2 = d['sums'][:, 0], d['sums'][:, 1]
        dm = np.where(n > 0, s1 / np.maximum(n, 1), 0.0)
        return np.stack([p + dm, s2 - s1 * dm], axis=1)
    for i, o in enumerate(outs):
        for a, b in zip(o, ref[i % 2]):
            for k in a:
                if k == 'features':   # LDS f64 atomics: the summation order varies
                    np.testing.assert_allclose(a[k], b[k], rtol=1e-12, atol=1e-15)
                    np.testing.assert_array_equal(a[k][:, 2:], b[k][:, 2:])
                elif k == 'sums':     # ... and so does which sample became the pivot
                    np.testing.assert_allclose(moments(a), moments(b), rtol=1e-12, atol=1e-15)
                elif k == 'records':
                    np.testing.assert_array_equal(np.delete(a[k], 45, axis=1), np.delete(b[k], 45, axis=1))
                else:
                    np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize('max_jobs', [1, 4])
def test_workflow_affinities_repeatable(gpu, tmp_path, max_jobs):
    lab, bnd = S.generate((36, 60, 64), cell=6, seed=52)
    affs = S.affinities_from_boundary(bnd, S.NN_OFFSETS)
    e_ref, f_ref = O.affinity_features(lab, affs, S.NN_OFFSETS)
    for rep in range(3):
        d = tmp_path / ('r%d' % rep)
        d.mkdir()
        edges, nodes, feats, _ = _run(d, lab, affs, (12, 32, 32), offsets=S.NN_OFFSETS, max_jobs=max_jobs)
        np.testing.assert_array_equal(edges, e_ref)
        check_features(feats, f_ref)
