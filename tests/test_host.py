"""Host-side pieces of the drop-in (CPU only): the N5 codec,
the nifty.tools.blocking mirror, blocks_in_volume, the synthetic generator."""
import gzip
import json
import struct
import zlib

import numpy as np
import pytest

from cluster_tools_amd import blocking as B
from cluster_tools_amd import n5
from cluster_tools_amd import synthetic as S
from oracle import rag_oracle as O


# ---------------------------------------------------------------- N5 codec
def test_n5_roundtrip_and_layout(tmp_path):
    p = str(tmp_path / 'c.n5')
    data = np.arange(5 * 7 * 9, dtype=np.uint64).reshape(5, 7, 9) * 3
    with n5.File(p) as f:
        ds = f.create_dataset('a/b', shape=data.shape, chunks=(2, 4, 4), dtype='uint64', compression='gzip')
        ds[:] = data
        ds.attrs['foo'] = [1, 2]
    with open(tmp_path / 'c.n5' / 'attributes.json') as fh:
        assert json.load(fh)['n5'].startswith('2.')
    with open(tmp_path / 'c.n5' / 'a' / 'b' / 'attributes.json') as fh:
        meta = json.load(fh)
    assert meta['dimensions'] == [9, 7, 5] and meta['blockSize'] == [4, 4, 2]    # reversed axes
    assert meta['dataType'] == 'uint64' and meta['compression']['type'] == 'gzip' and meta['foo'] == [1, 2]
    # chunk (z=1, y=0, x=2) lives at <ds>/2/0/1; big-endian header + gzip payload
    raw = (tmp_path / 'c.n5' / 'a' / 'b' / '2' / '0' / '1').read_bytes()
    mode, nd = struct.unpack('>HH', raw[:4])
    dims = struct.unpack('>III', raw[4:16])
    assert (mode, nd, dims) == (0, 3, (1, 4, 2))
    payload = gzip.decompress(raw[16:])
    np.testing.assert_array_equal(np.frombuffer(payload, '>u8').reshape(2, 4, 1), data[2:4, 0:4, 8:9])
    with n5.File(p, 'r') as f:
        ds = f['a/b']
        np.testing.assert_array_equal(ds[:], data)
        np.testing.assert_array_equal(ds[1:4, 2:7, 3:8], data[1:4, 2:7, 3:8])
        assert ds.attrs['foo'] == [1, 2]


def test_n5_varlen_chunks_and_missing(tmp_path):
    with n5.File(str(tmp_path / 'v.n5')) as f:
        ds = f.create_dataset('s', shape=(10, 10, 10), chunks=(5, 5, 5), dtype='uint64', compression='gzip')
        assert ds.read_chunk((0, 0, 0)) is None          # block_edge_features.py:181-185
        vals = np.array([3, 1, 4, 1, 5, 9, 2, 6], dtype=np.uint64)
        ds.write_chunk((1, 0, 1), vals, True)
        np.testing.assert_array_equal(ds.read_chunk((1, 0, 1)), vals)
        raw = (tmp_path / 'v.n5' / 's' / '1' / '0' / '1').read_bytes()
        mode, nd = struct.unpack('>HH', raw[:4])
        assert mode == 1 and nd == 3
        (n,) = struct.unpack('>I', raw[16:20])
        assert n == vals.size
        ds.write_chunk((0, 1, 0), np.zeros(0, np.uint64), True)
        assert ds.read_chunk((0, 1, 0)).size == 0


def test_n5_reads_zlib_and_raw(tmp_path):
    with n5.File(str(tmp_path / 'z.n5')) as f:
        ds = f.create_dataset('r', shape=(4, 4), chunks=(4, 4), dtype='float32', compression='raw')
        x = np.random.default_rng(0).random((4, 4)).astype(np.float32)
        ds[:] = x
        np.testing.assert_array_equal(ds[:], x)
        dz = f.create_dataset('z', shape=(3,), chunks=(3,), dtype='int32', compression='gzip')
        # a zlib-wrapped payload (z5 with useZlib) must decode too
        hdr = struct.pack('>HHI', 0, 1, 3)
        body = zlib.compress(np.array([7, -1, 5], '>i4').tobytes())
        (tmp_path / 'z.n5' / 'z' / '0').write_bytes(hdr + body)
        np.testing.assert_array_equal(dz[:], [7, -1, 5])


# ---------------------------------------------------------------- blocking
def test_blocking_c_order_and_blocks():
    b = B.blocking([0, 0, 0], [10, 9, 7], [4, 4, 4])
    assert b.blocksPerAxis == [3, 3, 2] and b.numberOfBlocks == 18
    assert b.blockGridPosition(1) == [0, 0, 1]           # last axis fastest
    assert b.blockGridPosition(2) == [0, 1, 0]
    blk = b.getBlock(17)
    assert blk.begin == [8, 8, 4] and blk.end == [10, 9, 7]
    ref = O.blocking_blocks((10, 9, 7), (4, 4, 4))
    for i, (pos, bg, en) in enumerate(ref):
        g = b.getBlock(i)
        assert tuple(g.begin) == bg and tuple(g.end) == en and tuple(b.blockGridPosition(i)) == pos
        assert b.gridPositionToBlockId(list(pos)) == i


def test_blocking_halo_and_bounding_boxes():
    b = B.blocking([0, 0, 0], [10, 9, 7], [4, 4, 4])
    h = b.getBlockWithHalo(2, [1, 1, 1])
    assert h.innerBlock.begin == [0, 4, 0] and h.outerBlock.begin == [0, 3, 0] and h.outerBlock.end == [5, 9, 5]
    assert h.innerBlockLocal.begin == [0, 1, 0]
    ids = b.getBlockIdsOverlappingBoundingBox([3, 0, 0], [5, 4, 4])
    assert list(ids) == [0, 6]
    assert list(b.getBlockIdsInBoundingBox([0, 0, 0], [8, 8, 7])) == [0, 1, 2, 3, 6, 7, 8, 9]
    with pytest.raises(IndexError):
        b.getBlock(18)


def test_blocks_in_volume():
    assert B.blocks_in_volume((10, 9, 7), (4, 4, 4)) == list(range(18))
    assert B.blocks_in_volume((10, 9, 7), (4, 4, 4), [4, 4, 4], [None, None, None]) == [9, 11, 15, 17]


# ---------------------------------------------------------------- synthetic
def test_synthetic_deterministic_and_slab_consistent():
    a, ba = S.generate((12, 20, 16), cell=5, seed=9)
    b, bb = S.generate((12, 20, 16), cell=5, seed=9)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(ba, bb)
    # a z-slab generated with z_offset equals the slab of the whole volume
    s, bs = S.generate((5, 20, 16), cell=5, seed=9, z_offset=6, global_shape=(12, 20, 16))
    np.testing.assert_array_equal(s, a[6:11])
    np.testing.assert_array_equal(bs, ba[6:11])
    assert ba.min() >= 0.0 and ba.max() <= 1.0
    c, _ = S.generate((12, 20, 16), cell=5, seed=10)
    assert (c != a).any()


def test_synthetic_edge_density():
    lab, _ = S.generate((40, 40, 40), cell=10, seed=0, with_boundary=False)
    n_nodes = O.unique_labels(lab).size
    n_edges = O.rag_edges(lab).shape[0]
    assert 40 <= n_nodes <= 130 and 4 * n_nodes <= n_edges <= 12 * n_nodes


def test_graph_subgraph_and_neighborhoods():
    """ndist.Graph.extractSubgraphFromNodes / flattenedNeighborhoods against
    a direct restatement over python sets."""
    from cluster_tools_amd import ndist
    uv = np.array([[1, 2], [1, 5], [2, 3], [3, 5], [5, 9]], dtype=np.uint64)
    g = ndist.Graph(uv)
    inner, outer = g.extractSubgraphFromNodes([1, 2, 3])
    np.testing.assert_array_equal(inner, [0, 2])
    np.testing.assert_array_equal(outer, [1, 3])
    with pytest.raises(RuntimeError):
        g.extractSubgraphFromNodes([1, 4])
    inner, outer = g.extractSubgraphFromNodes([1, 4], allowInvalidNodes=True)
    assert inner.size == 0 and list(outer) == [0, 1]
    flat = g.flattenedNeighborhoods()
    ref = []
    for n in [1, 2, 3, 5, 9]:
        nb = sorted((int(b if a == n else a), e) for e, (a, b) in enumerate(uv.tolist()) if n in (a, b))
        ref.append(len(nb))
        for other, e in nb:
            ref += [other, e]
    np.testing.assert_array_equal(flat, np.array(ref, dtype=np.uint64))


def test_blocking_neighbor_ids():
    from cluster_tools_amd.blocking import blocking
    b = blocking([0, 0, 0], [10, 20, 30], [5, 10, 10])   # 2 x 2 x 3 blocks
    assert b.numberOfBlocks == 12
    bid = b.gridPositionToBlockId([1, 0, 1])
    assert b.getNeighborId(bid, 0, True) == b.gridPositionToBlockId([0, 0, 1])
    assert b.getNeighborId(bid, 0, False) == -1
    assert b.getNeighborId(bid, 1, True) == -1
    assert b.getNeighborId(bid, 2, False) == b.gridPositionToBlockId([1, 0, 2])


def test_bench_cpu_baseline_chunks_cover_the_slab():
    """bench.py's CPU baseline: z-chunks with a halo plane, faces owned by the
    upper voxel, so the chunk edge sets together are the slab's RAG."""
    import os
    import sys
    torch = pytest.importorskip('torch')
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    lab, bnd = S.generate((24, 40, 56), cell=6, seed=4)
    v, info = bench.cpu_baseline(torch.from_numpy(lab.view(np.int64)), torch.from_numpy(bnd), 24, 3)
    assert v > 0 and info['threads'] == 3
    from oracle import c_oracle
    whole, _ = c_oracle.features(lab, bnd)
    parts = []
    for z0, z1 in ((0, 8), (8, 16), (16, 24)):
        h = 1 if z0 else 0
        e, _ = c_oracle.features(lab[z0 - h:z1], bnd[z0 - h:z1], own_begin=(h, 0, 0))
        parts.append(e)
    u = np.unique(np.concatenate(parts), axis=0)
    np.testing.assert_array_equal(u, whole)
    assert '3 z-chunks on 3 worker processes' in info['sample']
