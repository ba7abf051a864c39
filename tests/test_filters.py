"""Filter-feature branch (features/block_edge_features.py:151-272).

CPU: the kernel rule (cluster_tools_amd.fastfilters.gaussian_taps) against its
numpy restatement (oracle/filter_oracle.py) and the moments that define it.
GPU (-m gpu): every filter vu.apply_filter can name (utils/volume_utils.py:
80-94) through libctg.so against the restatement; ndist.accumulateInput
against the oracle's boundary features with the response's own histogram
range; the EdgeFeaturesWorkflow filter branch end to end (N5 in -> N5 out,
9 k + 1 columns, merged over blocks).  fastfilters / vigra / nifty are not in
the image: parity against them is unpinned.
"""
import numpy as np
import pytest

from cluster_tools_amd import fastfilters as F
from oracle import filter_oracle as FO
from oracle import rag_oracle as O

FILTERS = ['gaussianSmoothing', 'gaussianGradientMagnitude', 'laplacianOfGaussian', 'hessianOfGaussianEigenvalues',
           'structureTensorEigenvalues', 'differenceOfGaussians']


@pytest.mark.parametrize('sigma', [0.7, 1.0, 1.6, 3.5])
def test_taps_moments(sigma):
    x = None
    for order in (0, 1, 2):
        t = F.gaussian_taps(sigma, order)
        np.testing.assert_allclose(t, FO.taps(sigma, order), rtol=0, atol=0)
        r = t.size // 2
        assert r == int(3.0 * sigma + 0.5 * order + 0.5)
        x = np.arange(-r, r + 1, dtype=np.float64)
        if order == 0:
            assert abs(t.sum() - 1.0) < 1e-12 and np.all(t > 0)
        elif order == 1:
            assert abs(np.sum(t * x) - 1.0) < 1e-12 and abs(t.sum()) < 1e-12   # d/dx x = 1, no DC
        else:
            assert abs(t.sum()) < 1e-12 and abs(np.sum(t * x * x / 2) - 1.0) < 1e-12


def test_oracle_filters_on_polynomials():
    """Away from the borders the restated filters differentiate exactly:
    gradient of a linear ramp, Laplacian of a quadratic."""
    z, y, x = np.meshgrid(np.arange(30.), np.arange(30.), np.arange(30.), indexing='ij')
    ramp = 0.5 * x + 0.25 * y
    inner = (slice(10, 20),) * 3
    np.testing.assert_allclose(FO.gaussianGradientMagnitude(ramp, 1.0)[inner], np.hypot(0.5, 0.25), rtol=1e-9)
    quad = 0.5 * (x * x + 2 * y * y + 3 * z * z)
    np.testing.assert_allclose(FO.laplacianOfGaussian(quad, 1.0)[inner], 6.0, rtol=1e-9)
    ev = FO.hessianOfGaussianEigenvalues(quad, 1.0)[inner]
    np.testing.assert_allclose(ev, np.broadcast_to([3.0, 2.0, 1.0], ev.shape), rtol=1e-9)


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize('name', FILTERS)
@pytest.mark.parametrize('shape,sigma', [((20, 24, 28), 1.0), ((9, 33, 17), 2.0), ((40, 36), 1.5),
                                         ((16, 20, 24), (1.0, 2.0, 0.5))])
def test_filters_match_restatement(gpu, name, shape, sigma):
    if isinstance(sigma, tuple) and len(sigma) != len(shape):
        pytest.skip('per-axis sigma of another rank')
    rng = np.random.default_rng(3)
    a = rng.random(shape).astype(np.float32)
    got = getattr(F, name)(a, sigma)
    ref = getattr(FO, name)(a.astype(np.float64), sigma)
    assert got.shape == ref.shape and got.dtype == np.float32
    scale = max(1.0, float(np.abs(ref).max()))
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-6 * scale)


@pytest.mark.gpu
def test_apply_filter_2d_slices_and_tensor_io(gpu):
    import torch
    rng = np.random.default_rng(4)
    a = rng.random((5, 30, 31)).astype(np.float32)
    got = F.apply_filter(a, 'gaussianGradientMagnitude', 1.2, apply_in_2d=True)
    ref = np.stack([FO.gaussianGradientMagnitude(s.astype(np.float64), 1.2) for s in a])
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-6)
    t = F.gaussianSmoothing(torch.from_numpy(a).cuda(), 1.0)
    assert t.is_cuda
    np.testing.assert_allclose(t.cpu().numpy(), FO.gaussianSmoothing(a.astype(np.float64), 1.0), rtol=2e-5,
                               atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize('with_size,ignore', [(True, False), (False, True)])
def test_accumulate_input(gpu, with_size, ignore):
    from cluster_tools_amd import ndist, synthetic as S
    lab, bnd = S.generate((20, 32, 40), cell=6, seed=5)
    resp = F.laplacianOfGaussian(bnd, 1.0)
    lo, hi = float(resp.min()), float(resp.max())
    e_ref, f_ref = O.boundary_features(lab, resp, ignore_label=ignore, lo=lo, hi=hi)
    # graph: every whole-volume edge (shuffled) plus one edge without faces
    rng = np.random.default_rng(0)
    uv = np.concatenate([e_ref[rng.permutation(e_ref.shape[0])], np.array([[10 ** 6, 10 ** 6 + 1]], np.uint64)])
    g = ndist.Graph(uv)
    out = ndist.accumulateInput(g, resp, lab, ignore, with_size, lo, hi)
    assert out.shape == (uv.shape[0], 10 if with_size else 9)
    assert np.all(out[-1] == 0)
    row = g.findEdges(e_ref)
    got = out[row]
    ref = f_ref if with_size else f_ref[:, :9]
    np.testing.assert_allclose(got[:, [0, 2, 8]], ref[:, [0, 2, 8]], rtol=1e-5, atol=1e-12)
    bound = (f_ref[:, 9] + 2) * np.finfo(np.float64).eps * np.maximum(f_ref[:, 2] ** 2, f_ref[:, 8] ** 2)
    assert np.all(np.abs(got[:, 1] - ref[:, 1]) <= np.maximum(1e-5 * np.abs(ref[:, 1]), bound))
    assert np.all(np.abs(got[:, 3:8] - ref[:, 3:8]) <= (hi - lo) / 40 + 1e-12)
    if with_size:
        np.testing.assert_array_equal(got[:, 9], ref[:, 9])


@pytest.mark.gpu
def test_workflow_filter_branch(gpu, tmp_path):
    from cluster_tools_amd import n5, synthetic as S
    from harness import workflow
    lab, bnd = S.generate((24, 48, 40), cell=7, seed=6)
    inp, out = str(tmp_path / 'in.n5'), str(tmp_path / 'out.n5')
    block = (12, 24, 20)
    with n5.File(inp) as f:
        f.create_dataset('seg', shape=lab.shape, chunks=block, dtype='uint64', compression='gzip')[:] = lab
        f.create_dataset('bnd', shape=bnd.shape, chunks=block, dtype='float32', compression='gzip')[:] = bnd
    workflow.graph_workflow(inp, 'seg', out, 'graph', block, max_jobs=2)
    filters, sigmas = ['gaussianSmoothing', 'hessianOfGaussianEigenvalues'], [1.0, 2.0]
    workflow.edge_features_workflow(inp, 'bnd', inp, 'seg', out, 'graph', out, 'features', block, max_jobs=2,
                                    max_jobs_merge=2, filters=filters, sigmas=sigmas, halo=(2, 4, 4))
    with n5.File(out, 'r') as f:
        feats = f['features'][:]
        edges = f['graph/edges'][:]
        n_features = f['s0/sub_features'].attrs['n_features']
    # 2 sigmas x (1 smoothing channel + 3 eigenvalue channels) x 9 statistics + size
    assert n_features == 2 * (1 + 3) * 9 + 1 and feats.shape == (edges.shape[0], n_features)
    # an edge whose faces all lie on a block's lower face plane is in that
    # block's sub-graph (lower halo) but its faces are in the previous block's
    # label box (inner + 1 on the upper side, block_edge_features.py:199-203):
    # the reference's geometry leaves such edges without samples
    size = feats[:, -1]
    has = size > 0
    assert has.mean() > 0.8
    assert np.all(feats[~has] == 0)
    # smoothing of a [0,1]-normalised input stays in [0,1]; min <= mean <= max per group
    for g in range((n_features - 1) // 9):
        grp = feats[has, 9 * g:9 * g + 9]
        assert np.all(grp[:, 2] <= grp[:, 0] + 1e-9) and np.all(grp[:, 0] <= grp[:, 8] + 1e-9)
        assert np.all(grp[:, 1] >= 0)
    sm = feats[has, :9]
    assert sm.min() >= -1e-6 and sm[:, [0, 2, 8]].max() <= 1 + 1e-6
