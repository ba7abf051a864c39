"""Multi-rank logic of cluster_tools_amd/dist.py on CPU (gloo, world sizes 1-8).

Each rank holds one z-slab (+ the halo plane below it) of a synthetic volume,
builds its partial table with the oracle-backed backend, and the real
partition / all_to_all / merge code of dist.py produces the rank shards.
Their concatenation must equal the whole-volume oracle: bit-exact edges and
nodes, features within 1e-9 (same float64 statistics, merged by Chan's rule).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from cluster_tools_amd import dist as cdist
from cluster_tools_amd import synthetic
from oracle import rag_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


BIG = 1 << 33   # labels >= 2^31: the exchange falls back to merging every row
HUGE = (1 << 63) + 5   # labels >= 2^63: negative in the int64 views on the wire


def _volume(shape, cell, big):
    lab, bnd = synthetic.generate(shape, cell=cell, seed=3)
    if big == 'flat_top':
        # the top half is one label: the upper ranks own no edge at all
        lab[shape[0] // 2:] = lab.max() + 1
    elif big == 'huge':
        lab = lab + np.uint64(HUGE)
    elif big:
        lab = lab + np.uint64(BIG)
    return lab, bnd


def _worker(rank, world, port, shape, cell, outdir, ignore_label, big=False):
    import torch.distributed as dist
    from tests.dist_helpers import OracleBackend
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    lab, bnd = _volume(shape, cell, big)
    Z = shape[0]
    z0 = [Z * r // world for r in range(world + 1)]
    halo = 1 if rank > 0 else 0
    sl = slice(z0[rank] - halo, z0[rank + 1])
    res = cdist.rag_features_distributed(np.ascontiguousarray(lab[sl]), np.ascontiguousarray(bnd[sl]),
                                         own_begin=(halo, 0, 0), ignore_label=ignore_label,
                                         backend=OracleBackend())
    np.save(os.path.join(outdir, 'e%d.npy' % rank), np.asarray(res.edges()))
    np.save(os.path.join(outdir, 'f%d.npy' % rank), np.asarray(res.features()))
    np.save(os.path.join(outdir, 'n%d.npy' % rank), res.node_shard.numpy())
    np.save(os.path.join(outdir, 'o%d.npy' % rank),
            np.array([res.edge_offset, res.n_edges_global, res.node_offset, res.n_nodes_global]))
    dist.destroy_process_group()


@pytest.mark.parametrize('world,shape,cell,ignore,big', [
    (1, (20, 24, 22), 5, False, False),   # the exchange with itself (bench.py --dist-path at N=1)
    (2, (24, 40, 36), 6, False, False),
    (3, (30, 33, 29), 5, True, False),
    (2, (20, 30, 28), 5, False, True),
    (4, (32, 30, 28), 5, False, False),
    (4, (32, 24, 20), 5, False, 'flat_top'),
    (4, (24, 20, 22), 5, False, 'huge'),
    (8, (40, 24, 20), 5, False, False),
    (8, (32, 20, 18), 4, True, True),
])
def test_distributed_matches_whole_volume(tmp_path, world, shape, cell, ignore, big):
    mp.spawn(_worker, args=(world, _free_port(), shape, cell, str(tmp_path), ignore, big), nprocs=world, join=True)
    lab, bnd = _volume(shape, cell, big)
    e_ref, f_ref = O.boundary_features(lab, bnd, ignore_label=ignore)
    nodes_ref = O.unique_labels(O.rag_edges(lab))  # endpoints of the unfiltered RAG
    es = [np.load(tmp_path / ('e%d.npy' % r)) for r in range(world)]
    fs = [np.load(tmp_path / ('f%d.npy' % r)) for r in range(world)]
    ns = [np.load(tmp_path / ('n%d.npy' % r)) for r in range(world)]
    offs = [np.load(tmp_path / ('o%d.npy' % r)) for r in range(world)]
    e = np.concatenate(es).astype(np.uint64)
    f = np.concatenate(fs)
    n = np.concatenate(ns).astype(np.uint64)
    np.testing.assert_array_equal(e, e_ref)
    np.testing.assert_allclose(f, f_ref, rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(n, nodes_ref)
    # offsets are the exclusive prefix of the shard sizes, totals agree
    acc_e = acc_n = 0
    for r in range(world):
        assert offs[r][0] == acc_e and offs[r][2] == acc_n
        acc_e += len(es[r])
        acc_n += len(ns[r])
        assert offs[r][1] == e_ref.shape[0] and offs[r][3] == nodes_ref.shape[0]
    # every shard is non-empty for these sizes (splitters balance the ranks)
    if big != 'flat_top':
        assert all(len(x) > 0 for x in es)


def _meta(keys_per_rank):
    """meta rows (CTG_MGPU_SAMPLES evenly spaced u of sorted keys, + count) as ctg_mgpu_sample writes them."""
    from tests.dist_helpers import S
    rows = []
    for k in keys_per_rank:
        k = np.sort(np.asarray(k, dtype=np.uint64))
        m = np.zeros(S + 1, np.int64)
        if k.size:
            m[:S] = (k[(np.arange(S) * k.size) // S] ^ np.uint64(1 << 63)).view(np.int64)
        m[S] = k.size
        rows.append(m)
    return np.stack(rows)


def test_splitters_balance_and_agree():
    """The integer-weight splitter rule (restated from k_mgpu_splitters)
    balances skewed ranks and is a pure function of the gathered samples."""
    from tests.dist_helpers import splitters
    rng = np.random.default_rng(0)
    keys = [rng.integers(r * 1000, r * 1000 + 1500, size=n).astype(np.uint64) for r, n in enumerate([5000, 100, 9000])]
    sp = splitters(_meta(keys), 3)
    assert sp.shape == (2,) and sp[0] <= sp[1]
    allk = np.sort(np.concatenate(keys))
    owner = np.searchsorted(sp, allk, side='right')
    frac = np.bincount(owner, minlength=3) / allk.size
    assert np.all(np.abs(frac - 1 / 3) < 0.05)
    np.testing.assert_array_equal(sp, splitters(_meta(keys), 3))


def test_splitters_empty_ranks():
    from tests.dist_helpers import splitters
    assert list(splitters(_meta([[], [], [], []]), 4)) == [0, 0, 0]
    sp = splitters(_meta([[5] * 10, []]), 2)
    assert list(sp) == [5]
    # labels >= 2^63: unsigned order survives the int64 samples
    big = np.uint64(1 << 63)
    sp = splitters(_meta([np.arange(100, dtype=np.uint64) + big, np.arange(100, dtype=np.uint64)]), 2)
    assert sp[0] < big


def test_segment_words():
    c = np.zeros((3, 3, 2), np.int64)
    c[0, 1] = (2, 5)
    c[2, 1] = (1, 0)
    c[1, 1] = (7, 7)
    send, recv = cdist.segment_words(c, 3, 1)
    assert send == [0, 0, 0] and recv == [2 * cdist.ROW_WORDS + 5, 0, cdist.ROW_WORDS]
    assert cdist._any_exchange(c, 3)
    diag = np.zeros((3, 3, 2), np.int64)
    for r in range(3):
        diag[r, r] = (4, 4)
    assert not cdist._any_exchange(diag, 3)


def test_exchange_in_one_process_matches_whole_volume():
    """The four exchange steps of every rank simulated in one process (the
    collectives replaced by stacking / slicing; tests/exchange_sim.py): the
    shards concatenate to the whole-volume oracle."""
    from tests.dist_helpers import OracleBackend
    from tests.exchange_sim import simulate
    shape = (30, 26, 24)
    lab, bnd = _volume(shape, 5, False)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    n_ref = O.unique_labels(O.rag_edges(lab))
    for world in (1, 2, 3, 5):
        shards = simulate(OracleBackend(), lab, bnd, world)
        e = np.concatenate([s.edges() for s in shards])
        f = np.concatenate([s.features() for s in shards])
        n = np.concatenate([s.nodes() for s in shards])
        np.testing.assert_array_equal(e, e_ref)
        np.testing.assert_allclose(f, f_ref, rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(n, n_ref)


def test_slab_halo_checked_against_offsets():
    """dist.py refuses affinity offsets that reach past the slab's halo
    instead of silently dropping the samples whose partner lies below it --
    unless the slab plan clipped the halo at plane 0 (tiny slabs)."""
    lr = synthetic.LR_OFFSETS
    cdist.check_slab_halo((40, 8, 8), lr, (27, 0, 0), None)        # enough halo planes
    cdist.check_slab_halo((40, 8, 8), lr, (0, 0, 0), None)         # bottom slab: no neighbour below
    cdist.check_slab_halo((40, 8, 8), None, (1, 0, 0), None)       # boundary maps: 1 plane
    cdist.check_slab_halo((40, 8, 8), synthetic.NN_OFFSETS, (1, 0, 0), None)
    with pytest.raises(ValueError, match='halo'):
        cdist.check_slab_halo((40, 8, 8), lr, (1, 0, 0), None)
    with pytest.raises(ValueError, match='upper halo'):
        cdist.check_slab_halo((40, 8, 8), [[2, 0, 0]], (1, 0, 0), None)
    # 16 planes over 8 ranks, offset -4: rank 1 owns [2, 4) and reads from plane 0
    for r in range(8):
        rd, own, end = cdist.slab_plan(16, 8, r, [[-4, 0, 0]])
        cdist.check_slab_halo((end - rd, 8, 8), [[-4, 0, 0]], (own - rd, 0, 0), None, read_begin=rd)


def _reads_worker(rank, world, port, outdir):
    """Two calls with different slab shapes (Z = 100, then 101 over W = 3: the
    slabs differ between the ranks and between the calls); the host reads of
    every call are recorded."""
    import torch.distributed as dist
    from tests.dist_helpers import OracleBackend
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    reads = []
    for Z in (100, 101):
        lab, bnd = _volume((Z, 14, 12), 4, False)
        rd, own, end = cdist.slab_plan(Z, world, rank)
        del cdist.host_reads[:]
        res = cdist.rag_features_distributed(np.ascontiguousarray(lab[rd:end]), np.ascontiguousarray(bnd[rd:end]),
                                             own_begin=(own - rd, 0, 0), backend=OracleBackend())
        reads.append('|'.join(cdist.host_reads))   # the call itself: the count matrix only
        _ = (res.edge_offset, res.n_edges_global, res.node_offset, res.shard_sizes)
        reads.append('|'.join(cdist.host_reads))   # the shard sizes, once, on first use
        np.save(os.path.join(outdir, 'e%d_%d.npy' % (Z, rank)), res.edges())
        np.save(os.path.join(outdir, 'f%d_%d.npy' % (Z, rank)), res.features())
    np.save(os.path.join(outdir, 'reads%d.npy' % rank), np.array(reads))
    dist.destroy_process_group()


def test_changing_slab_shapes_and_host_reads(tmp_path):
    """No state is carried between calls (a capacity plan cached
    per slab shape could disagree between ranks): Z = 100 then Z = 101 over 3
    ranks both equal the whole-volume oracle; every call reads exactly the
    count matrix on the host, and the shard sizes once when first used."""
    world = 3
    mp.spawn(_reads_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for Z in (100, 101):
        lab, bnd = _volume((Z, 14, 12), 4, False)
        e_ref, f_ref = O.boundary_features(lab, bnd)
        e = np.concatenate([np.load(tmp_path / ('e%d_%d.npy' % (Z, r))) for r in range(world)])
        f = np.concatenate([np.load(tmp_path / ('f%d_%d.npy' % (Z, r))) for r in range(world)])
        np.testing.assert_array_equal(e, e_ref)
        np.testing.assert_allclose(f, f_ref, rtol=1e-9, atol=1e-12)
    for r in range(world):
        assert list(np.load(tmp_path / ('reads%d.npy' % r))) == ['counts', 'counts|offsets'] * 2


def test_mgpu_slab_plan_c_abi():
    """ctg_mgpu_slab (include/ctg.h; host-only, no device): owned ranges tile
    [0, Z) in rank order, the halo below reaches as far as the faces / offsets
    (1 plane for boundary maps, max(-o_z) for long-range offsets, none on rank
    0), and positive z offsets are refused when the volume is split."""
    from cluster_tools_amd import _lib
    from cluster_tools_amd import synthetic as S
    for Z, world in [(1024, 1), (2048, 8), (101, 4), (7, 7)]:
        for offs, down in [(None, 1), (S.NN_OFFSETS, 1), (S.LR_OFFSETS, 4)]:
            plans = [cdist.slab_plan(Z, world, r, offs) for r in range(world)]
            assert plans[0][:2] == (0, 0) and plans[-1][2] == Z
            for r, (rd, own, end) in enumerate(plans):
                assert own == Z * r // world and end == Z * (r + 1) // world and end > own
                assert own - rd == (min(down, own) if r else 0)
    with pytest.raises(_lib.CtgError, match='upper halo'):
        cdist.slab_plan(64, 2, 0, [[1, 0, 0]])
    assert cdist.slab_plan(64, 1, 0, [[1, 0, 0]]) == (0, 0, 64)
    with pytest.raises(_lib.CtgError):
        cdist.slab_plan(4, 8, 0)
    with pytest.raises(_lib.CtgError):
        cdist.slab_plan(64, 2, 2)


def _gather_worker(rank, world, port, shape, cell, outdir, big):
    import torch.distributed as dist
    from tests.dist_helpers import OracleBackend
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    lab, bnd = _volume(shape, cell, big)
    Z = shape[0]
    z0 = [Z * r // world for r in range(world + 1)]
    halo = 1 if rank > 0 else 0
    sl = slice(z0[rank] - halo, z0[rank + 1])
    res = cdist.rag_features_distributed(np.ascontiguousarray(lab[sl]), np.ascontiguousarray(bnd[sl]),
                                         own_begin=(halo, 0, 0), backend=OracleBackend())
    root = world - 1   # not rank 0: the root argument is honoured
    got = cdist.gather_to_host(res, root=root)
    assert (got is None) == (rank != root)
    if got is not None:
        e, f, n = got
        np.save(os.path.join(outdir, 'ge.npy'), e)
        np.save(os.path.join(outdir, 'gf.npy'), f)
        np.save(os.path.join(outdir, 'gn.npy'), n)
    t = {}
    w = cdist.write_global(res, os.path.join(outdir, 'out.n5'), 'graph', os.path.join(outdir, 'feat.n5'),
                           'features', shape=shape, ignore_label=False, root=0, timings=t)
    assert (w is None) == (rank != 0) and 'gather_s' in t
    dist.destroy_process_group()


@pytest.mark.parametrize('world,shape,cell,big', [
    (2, (24, 40, 36), 6, False),
    (3, (30, 33, 29), 5, 'huge'),
    (4, (32, 24, 20), 5, 'flat_top'),   # the upper ranks' shards are empty
])
def test_gather_to_host_and_n5_write(tmp_path, world, shape, cell, big):
    """SURVEY §8(e) Output: gather_to_host puts the global tables on the root
    (any rank), and write_global writes graph/{nodes,edges} with the
    MergeSubGraphs attrs and the (E, 10) features dataset with
    merge_edge_features.py's chunks; both equal the whole-volume oracle."""
    mp.spawn(_gather_worker, args=(world, _free_port(), shape, cell, str(tmp_path), big), nprocs=world, join=True)
    lab, bnd = _volume(shape, cell, big)
    e_ref, f_ref = O.boundary_features(lab, bnd)
    nodes_ref = O.unique_labels(O.rag_edges(lab))
    e = np.load(tmp_path / 'ge.npy')
    np.testing.assert_array_equal(e, e_ref)
    np.testing.assert_allclose(np.load(tmp_path / 'gf.npy'), f_ref, rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(np.load(tmp_path / 'gn.npy'), nodes_ref)
    from cluster_tools_amd import n5
    with n5.file_reader(str(tmp_path / 'out.n5'), 'r') as f:
        g = f['graph']
        assert g.attrs['numberOfEdges'] == e_ref.shape[0] and g.attrs['numberOfNodes'] == nodes_ref.shape[0]
        assert list(g.attrs['shape']) == list(shape) and g.attrs['ignore_label'] is False
        assert tuple(g['edges'].chunks) == (min(262144, e_ref.shape[0]), 2)
        np.testing.assert_array_equal(g['edges'][:], e_ref)
        np.testing.assert_array_equal(g['nodes'][:], nodes_ref)
    with n5.file_reader(str(tmp_path / 'feat.n5'), 'r') as f:
        ds = f['features']
        assert tuple(ds.shape) == (e_ref.shape[0], 10) and tuple(ds.chunks) == (min(262144, e_ref.shape[0]), 1)
        np.testing.assert_allclose(ds[:], f_ref, rtol=1e-9, atol=1e-12)
