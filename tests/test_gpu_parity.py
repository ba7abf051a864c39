"""GPU parity: the HIP path (libctg.so, through the C ABI) against the oracle
and the committed golden fixtures.

Bars (north_star): graph outputs (edges, nodes, counts) bit-exact; mean, var,
min, max within 1e-5 relative; quantiles within one histogram bin width
(1/40 on [0,1]).
"""
import json
import os

import numpy as np
import pytest

from cluster_tools_amd import rag
from cluster_tools_amd import synthetic as S
from oracle import rag_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5
ATOL = 0.0
BIN = 1.0 / 40
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def check_features(f_gpu, f_ref):
    """north_star bars with no absolute slack: mean / var / min / max within
    1e-5 relative (the variance too: the GPU keeps shifted sums about a
    per-edge pivot), counts exact, quantiles within one bin."""
    assert f_gpu.shape == f_ref.shape
    np.testing.assert_array_equal(f_gpu[:, 9], f_ref[:, 9])            # count exact
    for c in (0, 1, 2, 8):                                               # mean var min max
        np.testing.assert_allclose(f_gpu[:, c], f_ref[:, c], rtol=RTOL, atol=ATOL)
    np.testing.assert_array_less(np.abs(f_gpu[:, 3:8] - f_ref[:, 3:8]), BIN + 1e-12)


@pytest.fixture(scope='module')
def vol():
    return dict(np.load(os.path.join(GOLD, 'volumes.npz')))


@pytest.fixture(scope='module')
def kats():
    with open(os.path.join(GOLD, 'kats.json')) as fh:
        return {k['name']: k for k in json.load(fh)}


# ------------------------------------------------------------------ KATs
@pytest.mark.parametrize('name', ['kat1_sample_rule', 'kat3_halo_plane', 'kat7_outliers'])
def test_kat_boundary(gpu, kats, name):
    k = kats[name]
    out = rag.rag_features(np.asarray(k['labels'], np.uint64), np.asarray(k['data'], np.float32))
    np.testing.assert_array_equal(out['edges'], np.asarray(k['edges'], np.uint64))
    f = out['features']
    np.testing.assert_array_equal(f[:, 9], k['count'])
    np.testing.assert_allclose(f[:, 0], k['mean'], rtol=1e-12)
    np.testing.assert_allclose(f[:, 2], k['min'], rtol=0)
    np.testing.assert_allclose(f[:, 8], k['max'], rtol=0)
    if 'var' in k:
        np.testing.assert_allclose(f[:, 1], k['var'], rtol=1e-9, atol=1e-15)


def test_kat_affinity(gpu, kats):
    k = kats['kat6_affinity']
    out = rag.rag_features(np.asarray(k['labels'], np.uint64), np.asarray(k['affs'], np.float32),
                           offsets=k['offsets'])
    np.testing.assert_array_equal(out['edges'], np.asarray(k['edges'], np.uint64))
    np.testing.assert_array_equal(out['features'][:, 9], k['count'])
    np.testing.assert_allclose(out['features'][:, 0], k['mean'], rtol=0)


def test_kat_ignore_label_and_halo_graph(gpu, kats):
    k = kats['kat4_ignore_label']
    out = rag.rag_features(np.asarray(k['labels'], np.uint64), ignore_label=True)
    np.testing.assert_array_equal(out['edges'], np.asarray(k['edges'], np.uint64))
    np.testing.assert_array_equal(out['nodes'], k['nodes'])
    k = kats['kat2_halo']
    L = np.asarray(k['labels'], np.uint64)
    # block 1 of KAT-2: ROI z in [1,4), owned faces = all of the ROI
    out = rag.rag_features(L[1:])
    np.testing.assert_array_equal(out['edges'], np.asarray(k['blocks'][1]['edges'], np.uint64))
    np.testing.assert_array_equal(rag.unique_labels(L, (2, 0, 0), (4, 1, 1)), k['blocks'][1]['nodes'])
    # block 0: one inner label, no edges
    out = rag.rag_features(L[:2])
    assert out['edges'].shape == (0, 2)
    np.testing.assert_array_equal(out['nodes'], [1])


# ------------------------------------------------------------- fixtures
def test_golden_boundary_f32(gpu, vol):
    out = rag.rag_features(vol['bf_labels'], vol['bf_data'])
    np.testing.assert_array_equal(out['edges'], vol['bf_edges'])
    np.testing.assert_array_equal(out['nodes'], vol['bf_nodes'])
    check_features(out['features'], vol['bf_feats'])


def test_fresh_process_small_calls(gpu):
    """The first calls of a fresh process size the sort / run buffers to their
    own record counts, so a kernel that reads past its valid range can leave
    the allocation (a node-marking lane re-read the unique-key table past its
    end; it faulted only when a small call came first in a process).  Small
    calls of growing size, each checked against the golden volume's edges."""
    import subprocess
    import sys
    code = (
        "import numpy as np\n"
        "from cluster_tools_amd import rag\n"
        "z = np.load(%r)\n"
        "for k in (1, 2, 3):\n"
        "    lab = np.tile(z['bf_labels'], (k, k, 1))\n"
        "    dat = np.tile(z['bf_data'], (k, k, 1))\n"
        "    out = rag.rag_features(lab, dat)\n"
        "    assert out['edges'].shape[0] > 0\n"
        "out = rag.rag_features(z['bf_labels'], z['bf_data'])\n"
        "assert (out['edges'] == z['bf_edges']).all()\n"
        "print('FRESH_OK')\n") % os.path.join(GOLD, 'volumes.npz')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, '-c', code], cwd=root, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and 'FRESH_OK' in r.stdout, r.stderr[-2000:]


def test_golden_boundary_u8(gpu, vol):
    out = rag.rag_features(vol['bf_labels'], vol['bu_data'])
    np.testing.assert_array_equal(out['edges'], vol['bu_edges'])
    check_features(out['features'], vol['bu_feats'])


def test_golden_ignore_label(gpu, vol):
    out = rag.rag_features(vol['ig_labels'], vol['bf_data'], ignore_label=True)
    np.testing.assert_array_equal(out['edges'], vol['ig_edges'])
    np.testing.assert_array_equal(out['nodes'], vol['ig_nodes'])   # nodes keep 0 (OPEN-2)
    check_features(out['features'], vol['ig_feats'])


def test_golden_owned_box(gpu, vol):
    out = rag.rag_features(vol['bf_labels'], vol['bf_data'], own_begin=tuple(vol['ob_begin']),
                           own_end=tuple(vol['ob_end']))
    np.testing.assert_array_equal(out['edges'], vol['ob_edges'])
    check_features(out['features'], vol['ob_feats'])


def test_golden_affinity_nn(gpu, vol):
    out = rag.rag_features(vol['bf_labels'], vol['nn_affs'], offsets=vol['nn_offsets'])
    np.testing.assert_array_equal(out['edges'], vol['nn_edges'])
    check_features(out['features'], vol['nn_feats'])


def test_golden_affinity_long_range(gpu, vol):
    lab, bnd = S.generate((10, 32, 32), cell=4, seed=5)
    affs = S.affinities_from_boundary(bnd, vol['lr_offsets'])
    out = rag.rag_features(lab, affs, offsets=vol['lr_offsets'])
    np.testing.assert_array_equal(out['edges'], vol['lr_edges'])
    check_features(out['features'], vol['lr_feats'])


def test_golden_block_subgraphs(gpu, vol):
    lab = vol['bf_labels']
    blocks = O.blocking_blocks(lab.shape, tuple(vol['blk_shape']))
    no = np.concatenate([[0], np.cumsum(vol['blk_nodes_len'])])
    eo = np.concatenate([[0], np.cumsum(vol['blk_edges_len'])])
    for i, (_, b, e) in enumerate(blocks):
        roi = [max(x - 1, 0) for x in b]
        sub = np.ascontiguousarray(lab[tuple(slice(r, y) for r, y in zip(roi, e))])
        out = rag.rag_features(sub)
        np.testing.assert_array_equal(out['edges'], vol['blk_edges'][eo[i]:eo[i + 1]])
        inner_b = [x - r for x, r in zip(b, roi)]
        inner_e = [y - r for y, r in zip(e, roi)]
        np.testing.assert_array_equal(rag.unique_labels(sub, inner_b, inner_e), vol['blk_nodes'][no[i]:no[i + 1]])


# --------------------------------------------------------- random volumes
@pytest.mark.parametrize("shape,cell", [((32, 48, 70), 6), ((40, 64, 64), 10), ((17, 130, 65), 5),
                                        ((3, 5, 200), 3), ((70, 2, 1), 2)])
def test_boundary_whole_volume(gpu, shape, cell):
    lab, bnd = S.generate(shape, cell=cell, seed=3)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    np.testing.assert_array_equal(out['nodes'], O.unique_labels(lab))
    check_features(out['features'], f_ref)


def test_graph_only(gpu):
    lab, _ = S.generate((33, 70, 90), cell=7, seed=1, with_boundary=False)
    out = rag.rag_features(lab)
    np.testing.assert_array_equal(out['edges'], O.rag_edges(lab))
    np.testing.assert_array_equal(out['nodes'], O.unique_labels(lab))


def test_label_bits_32(gpu):
    lab, bnd = S.generate((20, 40, 50), cell=5, seed=8)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(lab.astype(np.uint32), bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    np.testing.assert_array_equal(out['nodes'], O.unique_labels(lab))
    check_features(out['features'], f_ref)


def test_values_outside_range_and_custom_range(gpu):
    lab, bnd = S.generate((16, 30, 30), cell=5, seed=2)
    data = (bnd * 3.0 - 1.0).astype(np.float32)     # [-1, 2]: both outlier slots populated
    e_ref, f_ref = O.boundary_features(lab, data)
    out = rag.rag_features(lab, data)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)
    e_ref, f_ref = O.boundary_features(lab, data, lo=-1.0, hi=2.0)
    out = rag.rag_features(lab, data, hist_range=(-1.0, 2.0))
    np.testing.assert_array_equal(out['edges'], e_ref)
    f = out['features']
    np.testing.assert_array_equal(f[:, 9], f_ref[:, 9])
    np.testing.assert_array_less(np.abs(f[:, 3:8] - f_ref[:, 3:8]), 3.0 / 40 + 1e-12)


def test_single_label_and_empty(gpu):
    lab = np.full((5, 6, 7), 42, np.uint64)
    out = rag.rag_features(lab, np.zeros(lab.shape, np.float32))
    assert out['edges'].shape == (0, 2) and out['features'].shape == (0, 10)
    np.testing.assert_array_equal(out['nodes'], [42])
    out = rag.rag_features(np.zeros((0, 4, 4), np.uint64))
    assert out['edges'].shape == (0, 2) and out['nodes'].shape == (0,)


def test_many_edges_per_tile(gpu):
    """cell 2: dense supervoxels, the LDS edge table overflows into direct records."""
    lab, bnd = S.generate((24, 64, 128), cell=2, seed=6)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


def test_single_edge_past_u16_count(gpu, monkeypatch):
    """Labels alternate in x, so every x face of a 64x32x64 tile is the same edge
    (1,2): ~260 K samples per tile, all in two histogram slots.  Without the
    per-wave sample budget of the scan those u16 slots would wrap and q25 / q75
    would land 16 bins off."""
    monkeypatch.setenv('CTG_TILE_Z', '64')
    shape = (64, 64, 128)
    x = np.arange(shape[2])
    lab = np.broadcast_to((x % 2 + 1).astype(np.uint64), shape).copy()
    bnd = np.broadcast_to(np.where(x % 2, 0.7, 0.3).astype(np.float32), shape).copy()
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)
    assert out['features'][0, 9] > 4 * 65535
    offsets = S.NN_OFFSETS
    affs = np.stack([np.full(shape, 0.2 + 0.3 * c, np.float32) for c in range(len(offsets))])
    e_ref, f_ref = O.affinity_features(lab, affs, offsets)
    out = rag.rag_features(lab, affs, offsets=offsets)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


def test_salt_and_pepper_labels(gpu):
    """Random labels: almost every face is a boundary face with a new key."""
    rng = np.random.default_rng(1)
    lab = rng.integers(0, 50, size=(12, 40, 70)).astype(np.uint64)
    bnd = rng.random(lab.shape).astype(np.float32)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)
    lab = rng.integers(0, 100000, size=(12, 40, 70)).astype(np.uint64)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


@pytest.mark.parametrize('offsets', [S.NN_OFFSETS, S.LR_OFFSETS])
def test_affinity_random_volumes(gpu, offsets):
    lab, bnd = S.generate((20, 60, 60), cell=6, seed=12)
    affs = S.affinities_from_boundary(bnd, offsets)
    e_ref, f_ref = O.affinity_features(lab, affs, offsets)
    out = rag.rag_features(lab, affs, offsets=offsets)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)
    # uint8 affinities
    a8 = np.round(affs * 255).astype(np.uint8)
    e_ref, f_ref = O.affinity_features(lab, a8, offsets)
    out = rag.rag_features(lab, a8, offsets=offsets)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


@pytest.mark.parametrize('offsets', [
    [[-1, 0, 0], [0, -1, 0], [0, 0, -3]],                 # one nearest-neighbour channel missing
    [[0, 0, -1], [-1, 0, 0], [0, -1, 0], [0, 0, -9]],      # nearest-neighbour channels in another order
    [[-2, 0, 0], [0, -3, 0]],                              # long-range channels only
    [[0, 0, -1], [-1, 0, 0], [0, -1, 0]],                  # the three nearest-neighbour channels permuted
])
def test_affinity_channel_sets(gpu, offsets):
    """Channel sets with and without the three nearest-neighbour offsets: the
    scan pushes adjacency markers only when they are not all present."""
    lab, bnd = S.generate((18, 50, 70), cell=6, seed=21)
    affs = S.affinities_from_boundary(bnd, offsets)
    e_ref, f_ref = O.affinity_features(lab, affs, offsets)
    out = rag.rag_features(lab, affs, offsets=offsets)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


def test_affinity_without_marker_skip_is_identical(gpu, monkeypatch):
    """CTG_SKIP_ADJ=0 forces the adjacency markers: same edges, same features."""
    lab, bnd = S.generate((18, 50, 70), cell=6, seed=22)
    for offs in (S.NN_OFFSETS, S.LR_OFFSETS):
        affs = S.affinities_from_boundary(bnd, offs)
        a = rag.rag_features(lab, affs, offsets=offs)
        monkeypatch.setenv('CTG_SKIP_ADJ', '0')
        b = rag.rag_features(lab, affs, offsets=offs)
        monkeypatch.delenv('CTG_SKIP_ADJ')
        np.testing.assert_array_equal(a['edges'], b['edges'])
        np.testing.assert_array_equal(a['nodes'], b['nodes'])
        np.testing.assert_array_equal(a['features'][:, 9], b['features'][:, 9])
        np.testing.assert_allclose(a['features'], b['features'], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('shape', [(1, 7, 5), (3, 1, 130), (2, 33, 1), (5, 9, 65), (7, 40, 129)])
@pytest.mark.parametrize('offsets', [S.NN_OFFSETS, S.LR_OFFSETS])
def test_affinity_odd_shapes(gpu, shape, offsets):
    """Single planes, single rows / columns, ragged x tiles (65, 129 columns)
    and y tiles (40 rows): the face-form modes and the channel loop against
    the oracle."""
    lab, bnd = S.generate(shape, cell=3, seed=31)
    affs = S.affinities_from_boundary(bnd, offsets)
    e_ref, f_ref = O.affinity_features(lab, affs, offsets)
    out = rag.rag_features(lab, affs, offsets=offsets)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


@pytest.mark.parametrize('offsets', [S.NN_OFFSETS, S.LR_OFFSETS])
def test_nearest_neighbour_faces_equal_channel_loop(gpu, monkeypatch, offsets):
    """The face-scan forms of the affinity scan (MODE_AFF_NN for the three
    nearest-neighbour channels, MODE_AFF_MIX beside long-range channels) give
    the channel loop's result (CTG_NN3=0): same edges, nodes and counts,
    features to rounding (the samples fold in another order)."""
    lab, bnd = S.generate((20, 66, 70), cell=5, seed=23)
    affs = S.affinities_from_boundary(bnd, offsets)
    a = rag.rag_features(lab, affs, offsets=offsets)
    monkeypatch.setenv('CTG_NN3', '0')
    b = rag.rag_features(lab, affs, offsets=offsets)
    monkeypatch.delenv('CTG_NN3')
    np.testing.assert_array_equal(a['edges'], b['edges'])
    np.testing.assert_array_equal(a['nodes'], b['nodes'])
    np.testing.assert_array_equal(a['features'][:, 9], b['features'][:, 9])
    np.testing.assert_allclose(a['features'], b['features'], rtol=1e-12, atol=1e-12)


def test_record_regions_overflow(gpu, monkeypatch):
    """Smallest record buffer (CTG_REC_FRESH: 64 regions of 1024 slots) on
    random labels: the regions overflow and the scan re-runs with a larger
    buffer; the result must still match the oracle."""
    rng = np.random.default_rng(5)
    lab = rng.integers(0, 200000, size=(16, 48, 96)).astype(np.uint64)
    bnd = rng.random(lab.shape).astype(np.float32)
    monkeypatch.setenv('CTG_REC_FRESH', '1')
    out = rag.rag_features(lab, bnd)
    monkeypatch.delenv('CTG_REC_FRESH')
    e_ref, f_ref = O.boundary_features(lab, bnd)
    assert e_ref.shape[0] > 64 * 1024
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)


def test_affinity_edge_list_filter(gpu):
    """no_adj_filter + an explicit edge list = the ndist per-block semantics."""
    lab, bnd = S.generate((16, 40, 40), cell=5, seed=13)
    offs = S.LR_OFFSETS
    affs = S.affinities_from_boundary(bnd, offs)
    ob, oe = (1, 1, 1), (12, 30, 33)
    edge_list = O.rag_edges(lab[:12, :30, :33])      # some block's sub-graph edges
    e_ref, f_ref = O.affinity_features(lab, affs, offs, own_begin=ob, own_end=oe, edge_list=edge_list)
    out = rag.rag_features(lab, affs, offsets=offs, own_begin=ob, own_end=oe, no_adj_filter=True)
    rows = rag.map_edge_ids(out['edges'], e_ref)
    hit = rows >= 0
    f = np.zeros_like(f_ref)
    f[hit] = out['features'][rows[hit]]
    check_features(f, f_ref)


# --------------------------------------------------------------- helpers
def test_synth_matches_numpy(gpu):
    import torch
    shape, gshape = (9, 33, 47), (30, 33, 47)
    lab_t, bnd_t = rag.synth_volume(shape, cell=6, seed=4, z_offset=11, global_shape=gshape)
    lab, bnd = S.generate(shape, cell=6, seed=4, z_offset=11, global_shape=gshape)
    np.testing.assert_array_equal(lab_t.cpu().numpy().view(np.uint64), lab)
    np.testing.assert_array_equal(bnd_t.cpu().numpy(), bnd)
    affs_t = rag.synth_affinities(bnd_t, S.LR_OFFSETS)
    np.testing.assert_array_equal(affs_t.cpu().numpy(), S.affinities_from_boundary(bnd, S.LR_OFFSETS))
    torch.cuda.synchronize()


def test_device_tensors_in_and_out(gpu):
    import torch
    lab_t, bnd_t = rag.synth_volume((24, 50, 70), cell=6, seed=9)
    r = rag.rag_features_handle(lab_t, bnd_t)
    e_t, f_t = r.edges_torch_i64(), r.features_torch()
    r.free()
    lab, bnd = S.generate((24, 50, 70), cell=6, seed=9)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(e_t.cpu().numpy().view(np.uint64), e_ref)
    check_features(f_t.cpu().numpy(), f_ref)
    assert e_t.is_cuda and f_t.is_cuda and torch.cuda.current_device() == e_t.device.index


def test_merge_stats_of_slabs_equals_whole(gpu):
    lab, bnd = S.generate((30, 40, 44), cell=5, seed=14)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    a = rag.rag_features(lab[:13], bnd[:13], keep_stats=True)
    b = rag.rag_features(lab[12:], bnd[12:], own_begin=(1, 0, 0), keep_stats=True)
    keys = np.concatenate([a['edges'], b['edges']])
    sums = np.concatenate([a['sums'], b['sums']])
    recs = np.concatenate([a['records'], b['records']])
    m = rag.merge_stats(keys, sums, recs)
    np.testing.assert_array_equal(m['edges'], e_ref)
    check_features(m['features'], f_ref)


def test_unique_and_map_helpers(gpu):
    rng = np.random.default_rng(3)
    v = rng.integers(0, 2 ** 40, size=5000).astype(np.uint64)
    r = rag.unique_values_handle(v)
    np.testing.assert_array_equal(r.nodes(), np.unique(v))
    r.free()
    pairs = np.sort(rng.integers(0, 300, size=(4000, 2)), axis=1).astype(np.uint64)
    pairs = pairs[pairs[:, 0] != pairs[:, 1]]
    e, n = rag.unique_pairs(pairs)
    np.testing.assert_array_equal(e, O._unique_pairs(pairs))
    np.testing.assert_array_equal(n, np.unique(pairs))
    q = np.concatenate([e[::7], np.array([[1000, 1001], [0, 0]], np.uint64)])
    ids = rag.map_edge_ids(e, q)
    np.testing.assert_array_equal(ids, O.find_edges(e, q))
    assert ids[-1] == -1 and ids[-2] == -1
    lab = rng.integers(0, 60, size=(9, 10, 11)).astype(np.uint64)
    np.testing.assert_array_equal(rag.unique_labels(lab, (2, 3, 4), (7, 9, 10)), np.unique(lab[2:7, 3:9, 4:10]))


@pytest.mark.parametrize('defer', [False, True])
def test_hip_backend_slabs_merge(gpu, defer):
    """The multi-GPU data path (local partials -> ctg_mgpu_split / pack ->
    exchanged rows -> ctg_mgpu_merge) for 2 and 3 z-slabs on one GPU
    (tests/exchange_sim.py) == the oracle's whole-volume features; with the
    statistics rows written by the local calls (CTG_KEEP_STATS) and rebuilt
    from the records by the exchange (CTG_DEFER_STATS) -- the two agree to
    the f64 summation order (record slots come from the scan's flush atomics,
    so two calls may sum an edge's records in a different order)."""
    from cluster_tools_amd import dist as cdist
    from tests.exchange_sim import simulate
    shape = (40, 48, 56)
    lab, bnd = rag.synth_volume(shape, cell=6, seed=21)
    e_ref, f_ref = O.boundary_features(lab.cpu().numpy().view(np.uint64), bnd.cpu().numpy())
    for world in (2, 3):
        shards = simulate(cdist.HipBackend(defer_stats=defer), lab, bnd, world, fresh=defer)
        e = np.concatenate([x.edges() for x in shards])
        f = np.concatenate([x.features() for x in shards])
        np.testing.assert_array_equal(e, e_ref)
        check_features(f, f_ref)
        if defer:
            eager = simulate(cdist.HipBackend(defer_stats=False), lab, bnd, world)
            np.testing.assert_array_equal(np.concatenate([x.edges() for x in eager]), e)
            np.testing.assert_allclose(np.concatenate([x.features() for x in eager]), f, rtol=1e-12, atol=1e-15)


def test_deferred_stats_stale_after_another_call(gpu):
    """A CTG_DEFER_STATS table serves ctg_mgpu_pack only while its records are
    the device's latest: after another call, pack refuses it (CTG_ERR_STALE)
    instead of reading overwritten records; a rank with nothing to send or
    receive never needs them."""
    from cluster_tools_amd import _lib
    from cluster_tools_amd import dist as cdist
    from tests.exchange_sim import simulate
    lab, bnd = rag.synth_volume((40, 48, 56), cell=6, seed=21)
    with pytest.raises(_lib.CtgError, match='overwritten'):
        simulate(cdist.HipBackend(defer_stats=True), lab, bnd, 2)
    shards = simulate(cdist.HipBackend(defer_stats=True), lab, bnd, 1)   # world 1: no rows move
    assert shards[0].n_edges > 0


def test_hip_backend_affinity_slabs_merge(gpu):
    """The same with long-range affinities (halo = max(-o_z) planes from the
    slab plan): per-slab partials keep non-adjacent pairs, the merge keeps the
    keys whose ADJ bit some slab proved."""
    from cluster_tools_amd import dist as cdist
    from tests.exchange_sim import simulate
    shape = (30, 40, 40)
    lab, bnd = rag.synth_volume(shape, cell=5, seed=22)
    offs = [[-1, 0, 0], [0, -1, 0], [0, 0, -1], [-2, 0, 0], [0, -3, 0], [0, 0, -3]]
    affs = rag.synth_affinities(bnd, offs)
    e_ref, f_ref = O.affinity_features(lab.cpu().numpy().view(np.uint64), affs.cpu().numpy(), offs)
    for world in (2, 3):
        # (long-range partials keep the written rows: CTG_DEFER_STATS falls back)
        shards = simulate(cdist.HipBackend(), lab, affs, world, offsets=offs)
        np.testing.assert_array_equal(np.concatenate([x.edges() for x in shards]), e_ref)
        check_features(np.concatenate([x.features() for x in shards]), f_ref)


# ------------------------------------------------------- labels >= 2^32
BIG = np.uint64(1) << np.uint64(40)


def test_labels_above_2_32(gpu):
    """Labels >= 2^32 take the dense-relabelling path."""
    lab, bnd = S.generate((18, 40, 44), cell=5, seed=15)
    big = lab * np.uint64(977) + BIG          # sparse, huge ids; same partition
    e_ref, f_ref = O.boundary_features(lab, bnd)
    out = rag.rag_features(big, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref * np.uint64(977) + BIG)
    np.testing.assert_array_equal(out['nodes'], O.unique_labels(lab) * np.uint64(977) + BIG)
    check_features(out['features'], f_ref)
    g = rag.rag_features(big)
    np.testing.assert_array_equal(g['edges'], e_ref * np.uint64(977) + BIG)
    offs = S.NN_OFFSETS
    affs = S.affinities_from_boundary(bnd, offs)
    e_ref, f_ref = O.affinity_features(lab, affs, offs)
    out = rag.rag_features(big, affs, offsets=offs)
    np.testing.assert_array_equal(out['edges'], e_ref * np.uint64(977) + BIG)
    check_features(out['features'], f_ref)


def test_merge_and_pairs_above_2_32(gpu):
    lab, bnd = S.generate((20, 30, 30), cell=5, seed=16)
    big = lab + BIG
    e_ref, f_ref = O.boundary_features(lab, bnd)
    a = rag.rag_features(big[:9], bnd[:9], keep_stats=True)
    b = rag.rag_features(big[8:], bnd[8:], own_begin=(1, 0, 0), keep_stats=True)
    m = rag.merge_stats(np.concatenate([a['edges'], b['edges']]), np.concatenate([a['sums'], b['sums']]),
                        np.concatenate([a['records'], b['records']]))
    np.testing.assert_array_equal(m['edges'], e_ref + BIG)
    check_features(m['features'], f_ref)
    e, n = rag.unique_pairs(np.concatenate([a['edges'], b['edges']]))
    np.testing.assert_array_equal(e, e_ref + BIG)
    np.testing.assert_array_equal(n, np.unique(e_ref) + BIG)


def test_variance_constant_and_near_constant_edges(gpu):
    """Edges whose samples are all equal have variance exactly 0; near-constant
    edges (spread 1e-3 around 0.75, and around 1000) meet rtol 1e-5 against
    the two-pass oracle."""
    rng = np.random.default_rng(11)
    lab = np.zeros((24, 40, 72), np.uint64)
    lab[:, :, 36:] = 1
    lab[:, 20:, :] += 2          # labels 0..3: four edges, two per data regime
    bnd = np.full(lab.shape, 0.75, np.float32)
    bnd[:, 20:, :] = (0.75 + 1e-3 * rng.random((24, 20, 72))).astype(np.float32)
    out = rag.rag_features(lab, bnd)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    f = out['features']
    const = f[:, 2] == f[:, 8]
    assert const.any() and (~const).any()
    assert np.all(f[const, 1] == 0.0)
    np.testing.assert_allclose(f[~const, 1], f_ref[~const, 1], rtol=RTOL, atol=0)
    np.testing.assert_allclose(f[:, 0], f_ref[:, 0], rtol=1e-12, atol=0)
    # spread 1e-3 around 1000 (outside the histogram range): var / mean^2 ~ 1e-13,
    # where power sums (sum x^2 - sum x * mean) lose every digit; the pivoted
    # sums keep rtol 1e-5, in the scan and through the statistics merge
    big = (1000.0 + 1e-3 * rng.random(lab.shape)).astype(np.float32)
    out = rag.rag_features(lab, big, keep_stats=True)
    e_ref, f_ref = O.boundary_features(lab, big)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)
    assert np.all(f_ref[:, 1] > 0)
    a = rag.rag_features(lab[:11], big[:11], keep_stats=True)
    b = rag.rag_features(lab[10:], big[10:], own_begin=(1, 0, 0), keep_stats=True)
    m = rag.merge_stats(np.concatenate([a['edges'], b['edges']]), np.concatenate([a['sums'], b['sums']]),
                        np.concatenate([a['records'], b['records']]))
    np.testing.assert_array_equal(m['edges'], e_ref)
    check_features(m['features'], f_ref)


def test_bucket_sort_skewed_keys(gpu, monkeypatch):
    """The record sort's MSD bucket pass (ctg_sort.hip) on a skewed key set:
    every third plane is background label 0, adjacent to nearly every cell, so
    one bucket holds a large share of the records (the segmented sort's
    large-segment path).  Same result as the plain radix sort and the oracle."""
    lab, bnd = S.generate((48, 64, 80), cell=4, seed=9)
    lab = lab.copy()
    lab[::3] = 0
    out = rag.rag_features(lab, bnd)
    monkeypatch.setenv('CTG_BUCKET_SORT', '0')
    ref = rag.rag_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], ref['edges'])
    np.testing.assert_array_equal(out['nodes'], ref['nodes'])
    np.testing.assert_array_equal(out['features'][:, 9], ref['features'][:, 9])
    np.testing.assert_allclose(out['features'], ref['features'], rtol=1e-12, atol=1e-15)
    e_o, f_o = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_o)
    check_features(out['features'], f_o)


def _same_result(out, ref, exact_sums=False):
    np.testing.assert_array_equal(out['edges'], ref['edges'])
    np.testing.assert_array_equal(out['nodes'], ref['nodes'])
    np.testing.assert_array_equal(out['features'][:, [2, 8, 9]], ref['features'][:, [2, 8, 9]])
    np.testing.assert_allclose(out['features'], ref['features'], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize('shape,cell,seed', [((48, 96, 130), 5, 11), ((64, 128, 128), 3, 12), ((9, 70, 300), 7, 13)])
def test_group_sort_matches_other_paths(gpu, monkeypatch, shape, cell, seed):
    """The group sort of (key, slot) records (ctg_sort.hip k_gs_*: bucket
    passes over the record regions, per-bucket LDS counting sort + in-group
    ranks, decoupled look-back for the run index) against the onesweep pair
    sort (CTG_GROUP_SORT=0, CTG_BUCKET_SORT_PAIRS=0) and the oracle."""
    lab, bnd = S.generate(shape, cell=cell, seed=seed)
    monkeypatch.setenv('CTG_SORT_PACKED', '0')   # small volumes would pack key + slot into one word
    out = rag.rag_features(lab, bnd)
    monkeypatch.setenv('CTG_GROUP_SORT', '0')
    monkeypatch.setenv('CTG_BUCKET_SORT_PAIRS', '0')
    ref = rag.rag_features(lab, bnd)
    _same_result(out, ref)
    e_o, f_o = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_o)
    check_features(out['features'], f_o)


@pytest.mark.parametrize('case', ['boundary', 'ignore', 'graph', 'affinity_lr', 'far_labels'])
def test_group_sort_cases(gpu, monkeypatch, case):
    """The group sort path (run table and node bitmap from its run pass:
    ctg_sort.hip k_gs_runs, node window in LDS) against the onesweep path
    (CTG_GROUP_SORT=0) and the oracle: boundary maps, ignore_label (kept-edge
    compaction), graph only, long-range affinities (adjacency filter), and
    labels spread so that a bucket's node window does not fit LDS (global node
    atomics)."""
    lab, bnd = S.generate((40, 72, 100), cell=5, seed=41)
    kw = {}
    data = bnd
    if case == 'ignore':
        lab = lab.copy()
        lab[::4, ::3] = 0
        kw['ignore_label'] = True
    elif case == 'graph':
        data = None
    elif case == 'affinity_lr':
        kw['offsets'] = S.LR_OFFSETS
        data = S.affinities_from_boundary(bnd, S.LR_OFFSETS)
    elif case == 'far_labels':
        lab = lab * np.uint64(40503) % np.uint64(1 << 29)   # ids scattered over 2^29
    monkeypatch.setenv('CTG_SORT_PACKED', '0')
    out = rag.rag_features(lab, data, **kw)
    monkeypatch.setenv('CTG_GROUP_SORT', '0')
    monkeypatch.setenv('CTG_BUCKET_SORT_PAIRS', '0')
    ref = rag.rag_features(lab, data, **kw)
    np.testing.assert_array_equal(out['edges'], ref['edges'])
    np.testing.assert_array_equal(out['nodes'], ref['nodes'])
    if data is not None:
        np.testing.assert_array_equal(out['features'][:, [2, 8, 9]], ref['features'][:, [2, 8, 9]])
        np.testing.assert_allclose(out['features'], ref['features'], rtol=1e-12, atol=1e-15)
    if case in ('boundary', 'ignore', 'far_labels'):
        e_o, f_o = O.boundary_features(lab, bnd, ignore_label=case == 'ignore')
        np.testing.assert_array_equal(out['edges'], e_o)
        check_features(out['features'], f_o)


def test_group_sort_one_label_group(gpu, monkeypatch):
    """Every record of one bucket in one in-bucket group (label 1 under a
    plane of ~10 K cells: keys (1, v) only differ in v), and labels >= 2^20 so
    the group bits are u's: the in-group rank pass over a ~10 K-item group."""
    lab2, bnd2 = S.generate((1, 512, 512), cell=5, seed=3)
    lab = np.empty((2, 512, 512), np.uint64)
    lab[0] = 1
    lab[1] = lab2[0] + np.uint64(1 << 20)
    bnd = np.concatenate([np.full((1, 512, 512), 0.3, np.float32), bnd2])
    monkeypatch.setenv('CTG_SORT_PACKED', '0')
    out = rag.rag_features(lab, bnd)
    monkeypatch.setenv('CTG_GROUP_SORT', '0')
    monkeypatch.setenv('CTG_BUCKET_SORT_PAIRS', '0')
    ref = rag.rag_features(lab, bnd)
    _same_result(out, ref)
    e_o, f_o = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_o)
    check_features(out['features'], f_o)


def test_group_sort_oversized_bucket_falls_back(gpu, monkeypatch):
    """Background label 1 on every other plane of a 64 x 1024 x 1024 volume:
    the (1, v) records of ~250 K cells crowd one bucket far past the LDS
    capacity, so the host takes the onesweep path; same result as forcing it."""
    lab, bnd = S.generate((64, 1024, 1024), cell=6, seed=5)
    lab = lab + np.uint64(1)
    lab[::2] = 1
    monkeypatch.setenv('CTG_SORT_PACKED', '0')
    out = rag.rag_features(lab, bnd)
    monkeypatch.setenv('CTG_GROUP_SORT', '0')
    monkeypatch.setenv('CTG_BUCKET_SORT_PAIRS', '0')
    ref = rag.rag_features(lab, bnd)
    _same_result(out, ref)
    assert np.all(out['edges'][:, 0][out['edges'][:, 1] > 1] >= 1)


@pytest.mark.parametrize('shape,cell,quant', [((40, 80, 96), 5, None), ((48, 64, 128), 4, 4), ((32, 96, 70), 9, 2),
                                              ((24, 130, 200), 3, None)])
def test_narrow_tile_matches_wide_tile(gpu, monkeypatch, shape, cell, quant):
    """The narrow-tile scan (CTG_NARROW_ROWS=1: 2-row waves, 16-plane tiles,
    one staged entry per lane -- the configs[4] kernel, otherwise only reached
    at 1024^3) against the wide-tile scan and the oracle, on small volumes.
    quant: the boundary map rounded to that many levels (histogram slots
    with many samples)."""
    lab, bnd = S.generate(shape, cell=cell, seed=21)
    if quant:
        bnd = (np.round(bnd * quant) / quant).astype(np.float32)
    monkeypatch.setenv('CTG_NARROW_ROWS', '1')
    out = rag.rag_features(lab, bnd)
    monkeypatch.setenv('CTG_NARROW_ROWS', '0')
    ref = rag.rag_features(lab, bnd)
    _same_result(out, ref)
    e_o, f_o = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_o)
    check_features(out['features'], f_o)


def test_heavy_and_light_edges(gpu):
    """The features-only reduce keeps each edge's histogram as 21 u16-pair
    words while its count stays below 2^16; an edge past that (here the
    131072-sample face between two 256 x 256 slabs) is listed and redone with
    the wide histogram.  Heavy and light edges together, against the oracle:
    every column, quantiles included."""
    small, _ = S.generate((4, 256, 256), cell=6, seed=31)
    lab = np.empty((12, 256, 256), np.uint64)
    lab[:4] = small + np.uint64(10)
    lab[4:8] = 1
    lab[8:] = 2
    rng = np.random.default_rng(31)
    bnd = rng.random(lab.shape, dtype=np.float32)
    out = rag.rag_features(lab, bnd)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    np.testing.assert_array_equal(out['edges'], e_ref)
    check_features(out['features'], f_ref)
    k = int(np.flatnonzero((e_ref[:, 0] == 1) & (e_ref[:, 1] == 2))[0])
    assert out['features'][k, 9] == 2 * 256 * 256 and out['features'][:, 9].max() == 2 * 256 * 256


def test_single_edge_many_records(gpu, monkeypatch):
    """One edge with a record from every tile: two planes of two labels over
    4096 x 4096 (8192 (1, 2) records, all in one bucket and one in-bucket
    group of the group sort; packed keys take the bucket sort).  One edge,
    every face counted, exact statistics."""
    lab = np.ones((2, 4096, 4096), np.uint64)
    lab[1] = 2
    bnd = np.zeros(lab.shape, np.float32)
    bnd[0] = 0.25
    bnd[1] = 0.75
    for packed in ('1', '0'):
        monkeypatch.setenv('CTG_SORT_PACKED', packed)
        out = rag.rag_features(lab, bnd)
        assert out['edges'].tolist() == [[1, 2]]
        f = out['features'][0]
        assert f[9] == 2 * 4096 * 4096 and f[0] == 0.5 and f[2] == 0.25 and f[8] == 0.75
        assert abs(f[1] - 0.0625) < 1e-12