"""The multi-GPU path of cluster_tools_amd/dist.py end to end on the GPU box:
two processes, each running the HIP backend (libctg.so) on its z-slab of one
synthetic volume on cuda:0, exchange through a gloo group (the one-GPU box has
no second device for RCCL; dist.py stages device tensors through host memory
for gloo and keeps them in HBM for RCCL).  The rank shards must concatenate to
the single-call whole-volume result: bit-exact edges and nodes, features
within 1e-9 (the same float64 statistics, merged in a different order).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip('torch')
mp = pytest.importorskip('torch.multiprocessing')

SHAPE = (96, 160, 192)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, affinity):
    import torch.distributed as dist
    from cluster_tools_amd import dist as cdist
    from cluster_tools_amd import rag
    from cluster_tools_amd import synthetic
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    Z = SHAPE[0]
    z0 = [Z * r // world for r in range(world + 1)]
    offs = synthetic.NN_OFFSETS if affinity else None
    halo = 1 if rank > 0 else 0
    lab, bnd = rag.synth_volume((z0[rank + 1] - z0[rank] + halo,) + SHAPE[1:], cell=7, seed=9,
                                z_offset=z0[rank] - halo, global_shape=SHAPE)
    data = rag.synth_affinities(bnd, offs) if affinity else bnd
    res = cdist.rag_features_distributed(lab, data, offsets=offs, own_begin=(halo, 0, 0))
    np.save(os.path.join(outdir, 'e%d.npy' % rank), res.edges())
    np.save(os.path.join(outdir, 'f%d.npy' % rank), res.features())
    np.save(os.path.join(outdir, 'n%d.npy' % rank), res.node_shard.cpu().numpy())
    np.save(os.path.join(outdir, 'o%d.npy' % rank), np.array([res.edge_offset, res.n_edges_global]))
    dist.destroy_process_group()


@pytest.mark.parametrize('affinity', [False, True])
def test_two_rank_slabs_equal_whole_volume(tmp_path, affinity):
    from cluster_tools_amd import rag
    from cluster_tools_amd import synthetic
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), affinity), nprocs=world, join=True)
    lab, bnd = rag.synth_volume(SHAPE, cell=7, seed=9)
    offs = synthetic.NN_OFFSETS if affinity else None
    data = rag.synth_affinities(bnd, offs) if affinity else bnd
    ref = rag.rag_features(lab.cpu().numpy().view(np.uint64), data.cpu().numpy(), offsets=offs)
    e = np.concatenate([np.load(tmp_path / ('e%d.npy' % r)) for r in range(world)])
    f = np.concatenate([np.load(tmp_path / ('f%d.npy' % r)) for r in range(world)])
    n = np.concatenate([np.load(tmp_path / ('n%d.npy' % r)) for r in range(world)]).astype(np.uint64)
    np.testing.assert_array_equal(e, ref['edges'])
    np.testing.assert_allclose(f, ref['features'], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(n, ref['nodes'])
    o = [np.load(tmp_path / ('o%d.npy' % r)) for r in range(world)]
    assert o[0][0] == 0 and o[1][0] == len(np.load(tmp_path / 'e0.npy'))
    assert o[0][1] == o[1][1] == ref['edges'].shape[0]


def _rccl_worker(rank, world, port, outdir, affinity):
    """One rank over RCCL ("nccl"): the exchange's collectives (all_gather of
    the splitter samples, the uniform all_to_all_single, the overflow
    all_reduce, the shard-size all_gather) run on HBM tensors through RCCL --
    the code path the driver's 8-GPU scaling run takes, at world 1."""
    import torch.distributed as dist
    from cluster_tools_amd import dist as cdist
    from cluster_tools_amd import rag
    from cluster_tools_amd import synthetic
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world,
                            device_id=torch.device('cuda', 0))
    assert cdist._wire_device(torch.device('cuda', 0), None).type == 'cuda'
    offs = synthetic.NN_OFFSETS if affinity else None
    lab, bnd = rag.synth_volume(SHAPE, cell=7, seed=9)
    data = rag.synth_affinities(bnd, offs) if affinity else bnd
    for _ in range(2):   # two calls: no state is carried between them
        del cdist.host_reads[:]
        res = cdist.rag_features_distributed(lab, data, offsets=offs, own_begin=(0, 0, 0))
    np.save(os.path.join(outdir, 'e.npy'), res.edges())
    np.save(os.path.join(outdir, 'f.npy'), res.features())
    np.save(os.path.join(outdir, 'n.npy'), res.node_shard.cpu().numpy())
    calls_reads = list(cdist.host_reads)
    assert res.edge_offset == 0 and res.n_edges_global == res.n_edges   # the lazy shard-size read
    np.save(os.path.join(outdir, 'reads.npy'), np.array(calls_reads + list(cdist.host_reads)))
    # SURVEY §8(e) Output over RCCL: the shards gathered in HBM on the root, then the N5 write
    e, f, n = cdist.gather_to_host(res, root=0)
    np.save(os.path.join(outdir, 'ge.npy'), e)
    np.save(os.path.join(outdir, 'gf.npy'), f)
    np.save(os.path.join(outdir, 'gn.npy'), n)
    t = {}
    assert cdist.write_global(res, os.path.join(outdir, 'out.n5'), shape=SHAPE, timings=t) == (len(e), len(n))
    assert t['gather_s'] >= 0 and t['write_s'] >= 0
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('affinity', [False, True])
def test_rccl_world1_exchange_equals_single_call(tmp_path, affinity):
    from cluster_tools_amd import rag
    from cluster_tools_amd import synthetic
    mp.spawn(_rccl_worker, args=(1, _free_port(), str(tmp_path), affinity), nprocs=1, join=True)
    lab, bnd = rag.synth_volume(SHAPE, cell=7, seed=9)
    offs = synthetic.NN_OFFSETS if affinity else None
    data = rag.synth_affinities(bnd, offs) if affinity else bnd
    ref = rag.rag_features(lab.cpu().numpy().view(np.uint64), data.cpu().numpy(), offsets=offs)
    np.testing.assert_array_equal(np.load(tmp_path / 'e.npy'), ref['edges'])
    np.testing.assert_allclose(np.load(tmp_path / 'f.npy'), ref['features'], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(np.load(tmp_path / 'n.npy').astype(np.uint64), ref['nodes'])
    # one count-matrix read per call; the shard sizes when first asked for
    assert list(np.load(tmp_path / 'reads.npy')) == ['counts', 'counts', 'offsets']
    np.testing.assert_array_equal(np.load(tmp_path / 'ge.npy'), ref['edges'])
    np.testing.assert_allclose(np.load(tmp_path / 'gf.npy'), ref['features'], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(np.load(tmp_path / 'gn.npy'), ref['nodes'])
    from cluster_tools_amd import n5
    with n5.file_reader(str(tmp_path / 'out.n5'), 'r') as fh:
        np.testing.assert_array_equal(fh['graph/edges'][:], ref['edges'])
        np.testing.assert_array_equal(fh['graph/nodes'][:], ref['nodes'])
        assert fh['graph'].attrs['numberOfEdges'] == ref['edges'].shape[0]
        np.testing.assert_allclose(fh['features'][:], ref['features'], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize('affinity', [False, True, 'lr'])
def test_mgpu_exchange_simulated_in_one_process(affinity):
    """ctg_mgpu_sample / split / pack / merge of every rank in one process
    (tests/exchange_sim.py: the collectives replaced by their data movement)
    at world sizes 1-5: the shards concatenate to the single-call result --
    edges and nodes bit-exact, features within 1e-9 -- and the HIP split
    equals the numpy restatement of the splitter rule on the same samples."""
    from cluster_tools_amd import dist as cdist
    from cluster_tools_amd import rag
    from cluster_tools_amd import synthetic
    from tests.dist_helpers import splitters, split_counts, Part
    from tests.exchange_sim import simulate
    # 'lr': test_mws.py's 12 long-range offsets -- slabs with 4 halo planes, and
    # non-adjacent pairs kept by every rank until the merged ADJ bits decide
    offs = synthetic.LR_OFFSETS if affinity == 'lr' else synthetic.NN_OFFSETS if affinity else None
    lab, bnd = rag.synth_volume(SHAPE, cell=7, seed=9)
    data = rag.synth_affinities(bnd, offs) if affinity else bnd
    ref = rag.rag_features(lab.cpu().numpy().view(np.uint64), data.cpu().numpy(), offsets=offs)
    backend = cdist.HipBackend(defer_stats=affinity != 'lr')
    for world in (1, 2, 3, 5):
        # deferred statistics: each rank's records re-made before its pack / merge
        shards = simulate(backend, lab, data, world, offsets=offs, fresh=backend.defer_stats)
        e = np.concatenate([x.edges() for x in shards])
        f = np.concatenate([x.features() for x in shards])
        n = np.concatenate([x.nodes() for x in shards])
        np.testing.assert_array_equal(e, ref['edges'])
        np.testing.assert_allclose(f, ref['features'], rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(n, ref['nodes'])
        for x in shards:
            x.free()
    # the split kernel against its restatement: a world-3 sample of this table
    loc = backend.local(lab, data, offs, (0, 0, 0), None, False, (0.0, 1.0))
    rng = np.random.default_rng(1)
    meta = backend.sample(loc).cpu().numpy()
    metas = [meta]
    for _ in range(2):
        m = np.sort(rng.choice(meta[:-1], size=meta.shape[0] - 1))
        metas.append(np.concatenate([m, [int(rng.integers(1, 10 ** 6))]]))
    meta_all = np.stack(metas).astype(np.int64)
    got = backend.split(loc, torch.from_numpy(meta_all).cuda(), 3).cpu().numpy()
    part = Part(loc.edges(), None, None, None, loc.nodes(), False)
    np.testing.assert_array_equal(got, split_counts(part, splitters(meta_all, 3), 3))
    loc.free()
