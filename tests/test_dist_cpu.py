"""Multi-rank logic of cluster_tools_amd/dist.py on CPU (gloo, world_size 2 and 3).

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


def test_weighted_splitters_balance():
    rng = np.random.default_rng(0)
    keys = [np.sort(rng.integers(r * 1000, r * 1000 + 1500, size=n)) for r, n in enumerate([5000, 100, 9000])]
    S = 64
    samples = np.stack([k[(np.arange(S) * len(k)) // S] for k in keys])
    sp = cdist.weighted_splitters(samples, [len(k) for k in keys], 3)
    assert sp.shape == (2,) and sp[0] <= sp[1]
    allk = np.sort(np.concatenate(keys))
    owner = np.searchsorted(sp, allk, side='right')
    frac = np.bincount(owner, minlength=3) / allk.size
    assert np.all(np.abs(frac - 1 / 3) < 0.05)


def test_weighted_splitters_empty_ranks():
    sp = cdist.weighted_splitters(np.zeros((4, 8), np.int64), [0, 0, 0, 0], 4)
    assert sp.shape == (3,)
    sp = cdist.weighted_splitters(np.array([[5] * 8, [0] * 8]), [10, 0], 2)
    assert list(sp) == [5]


def test_split_counts_and_rows_roundtrip():
    k = torch.tensor([1, 1, 2, 5, 5, 5, 9], dtype=torch.int64)
    assert cdist.split_counts(k, np.array([2, 6])) == [2, 4, 1]
    assert cdist.split_counts(k, np.array([0, 100])) == [0, 7, 0]
    assert cdist.split_counts(k, np.array([], np.int64)) == [7]
    n = 5
    keys = torch.arange(2 * n, dtype=torch.int64).reshape(n, 2)
    sums = torch.rand(n, 2, dtype=torch.float64)
    recs = torch.randint(-2 ** 31, 2 ** 31 - 1, (n, 48), dtype=torch.int32)
    rows = cdist.pack_rows(keys, sums, recs)
    assert rows.shape == (n, cdist.ROW_WORDS)
    k2, s2, r2 = cdist.unpack_rows(rows)
    assert torch.equal(k2, keys) and torch.equal(s2, sums) and torch.equal(r2, recs)


def test_slab_halo_checked_against_offsets():
    """dist.py refuses affinity offsets that reach past the slab's halo
    instead of silently dropping the samples whose partner lies below it."""
    lr = synthetic.LR_OFFSETS
    cdist.check_slab_halo((40, 8, 8), lr, (27, 0, 0), None)        # enough halo planes
    cdist.check_slab_halo((40, 8, 8), lr, (0, 0, 0), None)         # bottom slab: no neighbour below
    cdist.check_slab_halo((40, 8, 8), None, (1, 0, 0), None)       # boundary maps: 1 plane
    cdist.check_slab_halo((40, 8, 8), synthetic.NN_OFFSETS, (1, 0, 0), None)
    with pytest.raises(ValueError, match='halo'):
        cdist.check_slab_halo((40, 8, 8), lr, (1, 0, 0), None)
    with pytest.raises(ValueError, match='upper halo'):
        cdist.check_slab_halo((40, 8, 8), [[2, 0, 0]], (1, 0, 0), None)


def test_device_splitters_match_numpy_restatement():
    rng = np.random.default_rng(5)
    for world in (2, 4, 8):
        counts = rng.integers(0, 5000, world)
        counts[rng.integers(0, world)] = 0
        S = 32
        samples = np.sort(rng.integers(-2 ** 62, 2 ** 62, (world, S)), axis=1)
        sp = cdist.weighted_splitters(samples, counts, world)
        # restatement: weighted quantiles of the kept samples
        w = np.repeat(counts / S, S)
        v = samples.reshape(-1)
        v, w = v[w > 0], w[w > 0]
        o = np.argsort(v, kind='stable')
        v, w = v[o], w[o]
        cw = np.cumsum(w)
        idx = np.minimum(np.searchsorted(cw, cw[-1] * np.arange(1, world) / world, side='left'), v.size - 1)
        np.testing.assert_array_equal(sp, v[idx])


def _plan_worker(rank, world, port, outdir):
    """Four calls on the same slab: the first learns the ExchangePlan, the
    second reuses it (no host read before the result-size read), the third
    starts from exchange capacities too small for its counts (overflow ->
    regrow -> redo), the fourth from a too small merge slice (redone locally)."""
    import torch.distributed as dist
    from tests.dist_helpers import OracleBackend
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    shape = (8 * world, 30, 28)
    lab, bnd = _volume(shape, 5, False)
    z0 = [shape[0] * r // world for r in range(world + 1)]
    halo = 1 if rank > 0 else 0
    sl = slice(z0[rank] - halo, z0[rank + 1])
    args = (np.ascontiguousarray(lab[sl]), np.ascontiguousarray(bnd[sl]))
    outs, reads = [], []
    for call, plan in enumerate([None, None, cdist.ExchangePlan(1, 1), cdist.ExchangePlan(1 << 16, 1 << 16, 1)]):
        del cdist.host_reads[:]
        res = cdist.rag_features_distributed(*args, own_begin=(halo, 0, 0), backend=OracleBackend(), plan=plan)
        reads.append(list(cdist.host_reads))
        outs.append((np.asarray(res.edges()), np.asarray(res.features()), res.node_shard.numpy()))
    for a in outs[1:]:
        for x, y in zip(a, outs[0]):
            np.testing.assert_array_equal(x, y)
    np.save(os.path.join(outdir, 'reads%d.npy' % rank), np.array(['|'.join(r) for r in reads]))
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_exchange_plan_reuse_and_overflow(tmp_path, world):
    mp.spawn(_plan_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        reads = list(np.load(tmp_path / ('reads%d.npy' % r)))
        # (the shard offsets are read after the result size)
        assert reads[0] == 'plan|plan|result|offsets'      # first call of the shape: learns its capacities
        assert reads[1] == 'result|offsets'                # plan reused: nothing read before the result size
        # exchange capacity too small: overflow seen with the result, exchange redone
        # (the merge slice sized on the truncated exchange may need a local redo too)
        assert reads[2].startswith('plan|result|result') and reads[2].endswith('|offsets')
        assert 'plan' not in reads[2][5:]
        # merge-slice capacity too small: this rank redoes its merge alone (no collective)
        assert reads[3].startswith('result|') and reads[3].endswith('|offsets')


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
