"""Host-side pieces of the drop-in (CPU only): the N5 codec,
the nifty.tools.blocking mirror, blocks_in_volume, the synthetic generator."""
import gzip
import os
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


# ---------------------------------------------------------------- zarr, Graph forms, companion layout
@pytest.mark.parametrize('codec', ['gzip', 'raw'])
def test_zarr_roundtrip_and_layout(tmp_path, codec):
    """zarr v2 input containers (graph_workflow.py:17-20 accepts zr / zarr):
    C-order metadata, 'i.j.k' chunk keys, edge chunks stored at full shape."""
    p = str(tmp_path / 'c.zarr')
    data = (np.arange(5 * 7 * 9, dtype=np.uint64).reshape(5, 7, 9) * 7) % 1000
    with n5.file_reader(p) as f:
        ds = f.create_dataset('vol/seg', data=data, chunks=(2, 4, 4), compression=codec)
        ds.attrs['resolution'] = [1, 2, 3]
    root = tmp_path / 'c.zarr'
    assert json.loads((root / '.zgroup').read_text())['zarr_format'] == 2
    assert json.loads((root / 'vol' / '.zgroup').read_text())['zarr_format'] == 2
    meta = json.loads((root / 'vol' / 'seg' / '.zarray').read_text())
    assert meta['shape'] == [5, 7, 9] and meta['chunks'] == [2, 4, 4] and meta['dtype'] == '<u8'
    assert json.loads((root / 'vol' / 'seg' / '.zattrs').read_text()) == {'resolution': [1, 2, 3]}
    raw = (root / 'vol' / 'seg' / '2.1.2').read_bytes()         # last chunk in every axis
    if codec == 'gzip':
        raw = gzip.decompress(raw)
    full = np.frombuffer(raw, '<u8').reshape(2, 4, 4)
    np.testing.assert_array_equal(full[:1, :3, :1], data[4:5, 4:7, 8:9])
    with n5.file_reader(p, 'r') as f:
        ds = f['vol/seg']
        np.testing.assert_array_equal(ds[:], data)
        np.testing.assert_array_equal(ds[1:4, 2:7, 3:8], data[1:4, 2:7, 3:8])
        assert ds.attrs['resolution'] == [1, 2, 3]
    assert not os.path.exists(str(root / 'attributes.json'))


def test_zarr_blosc_raises_and_other_formats_rejected(tmp_path):
    p = tmp_path / 'b.zarr' / 'x'
    p.mkdir(parents=True)
    (tmp_path / 'b.zarr' / '.zgroup').write_text('{"zarr_format": 2}')
    (p / '.zarray').write_text(json.dumps({'zarr_format': 2, 'shape': [4], 'chunks': [4], 'dtype': '<u8',
                                           'compressor': {'id': 'blosc', 'cname': 'lz4'}, 'fill_value': 0,
                                           'order': 'C', 'filters': None}))
    (p / '0').write_bytes(b'\x00' * 8)
    with n5.file_reader(str(tmp_path / 'b.zarr'), 'r') as f:
        with pytest.raises(ValueError, match='blosc'):
            f['x'][:]
        assert (f['x'].read_chunk((1,)) is None)
    with pytest.raises(ValueError):
        n5.file_reader(str(tmp_path / 'a.h5'))


def test_graph_constructor_forms(tmp_path):
    """ndist.Graph(path, key), Graph(path_with_key) (ilastik/carving.py:28),
    Graph(path_with_key, n_threads) (edges_from_skeletons.py:146), keyword
    numberOfThreads (solve_subproblems.py:250); numberOfNodes semantics."""
    from cluster_tools_amd import ndist
    p = str(tmp_path / 'problem.n5')
    nodes = np.array([0, 1, 2, 3, 4, 5], dtype=np.uint64)
    uv = np.array([[0, 1], [1, 2], [2, 5], [3, 4]], dtype=np.uint64)
    with n5.File(p) as f:
        g = f.require_group('s0/graph')
        g.create_dataset('nodes', data=nodes, chunks=(4,))
        g.create_dataset('edges', data=uv, chunks=(3, 2))
    forms = [ndist.Graph(p, 's0/graph'), ndist.Graph(p, 's0/graph', numberOfThreads=3),
             ndist.Graph(os.path.join(p, 's0/graph')), ndist.Graph(os.path.join(p, 's0', 'graph'), 4),
             ndist.Graph(os.path.join(p, 's0', 'graph'), numberOfThreads=2)]
    for gr in forms:
        np.testing.assert_array_equal(gr.uvIds(), uv)
        np.testing.assert_array_equal(gr.nodes(), nodes)
        # test_graph.py:113 literally: dense 0..max labels -> numberOfNodes == seg.max() + 1
        assert gr.numberOfNodes == int(nodes.max()) + 1
        assert gr.numberOfEdges == 4 and gr.maxNodeId == 5 and gr.maxEdgeId == 3
    # non-dense labels: numberOfNodes counts distinct nodes (test_graph.py:78-80
    # "number of nodes in nifty can be larger" for gridRag's max+1)
    sparse = ndist.Graph(np.array([[2, 7], [7, 40]], dtype=np.uint64))
    assert sparse.numberOfNodes == 3 and sparse.maxNodeId == 40
    with pytest.raises(ValueError):
        ndist.Graph(str(tmp_path / 'not_a_container' / 'graph'))
    with pytest.raises(TypeError):
        ndist.Graph()


def test_stats_companion_words_roundtrip():
    from cluster_tools_amd import ndist
    rng = np.random.default_rng(1)
    sums = rng.random((7, 2))
    recs = rng.integers(0, 2 ** 32, (7, 48), dtype=np.uint64).astype(np.uint32)
    w = ndist.encode_stats_words(sums, recs)
    assert w.dtype == np.uint32 and w.shape == (7, 52) and w.nbytes == 7 * 208
    s2, r2 = ndist.decode_stats_words(w.ravel())
    np.testing.assert_array_equal(s2, sums)
    np.testing.assert_array_equal(r2, recs)


def test_stats_companion_compact_rows():
    """Blocks whose histogram slots fit 16 bits (and whose pad words are zero,
    as the library writes them) store 29-word rows; decode detects the width
    from the word count and restores the 48-word records exactly; a block with
    a slot above 65535 keeps the 52-word rows."""
    from cluster_tools_amd import ndist
    rng = np.random.default_rng(2)
    n = 9
    sums = rng.random((n, 2))
    recs = np.zeros((n, 48), np.uint32)
    recs[:, :42] = rng.integers(0, 65536, (n, 42))
    recs[:, 42] = rng.integers(1, 2 ** 31, n) | np.uint32(0x80000000)
    recs[:, 43:46] = rng.integers(0, 2 ** 32, (n, 3), dtype=np.uint64).astype(np.uint32)
    w = ndist.encode_stats_words(sums, recs)
    assert w.shape == (n, ndist.STATS_WORDS_COMPACT) == (n, 29)
    s2, r2 = ndist.decode_stats_words(w.ravel(), n)
    np.testing.assert_array_equal(s2, sums)
    np.testing.assert_array_equal(r2, recs)
    recs[3, 17] = 65536
    w = ndist.encode_stats_words(sums, recs)
    assert w.shape == (n, ndist.STATS_WORDS)
    s2, r2 = ndist.decode_stats_words(w.ravel(), n)
    np.testing.assert_array_equal(r2, recs)
    with pytest.raises(RuntimeError):
        ndist.decode_stats_words(w.ravel()[:-1], n)


def test_blocks_in_volume_block_list_path(tmp_path):
    lp = tmp_path / 'blocks.json'
    lp.write_text(json.dumps([1, 9, 11, 12]))
    assert B.blocks_in_volume((10, 9, 7), (4, 4, 4), block_list_path=str(lp)) == [1, 9, 11, 12]
    ids = B.blocks_in_volume((10, 9, 7), (4, 4, 4), [4, 4, 4], [None, None, None], block_list_path=str(lp))
    assert ids == [9, 11]
    ids, blk = B.blocks_in_volume((10, 9, 7), (4, 4, 4), return_blocking=True)
    assert blk.numberOfBlocks == 18 and ids == list(range(18))
    with pytest.raises(AssertionError):
        B.blocks_in_volume((10, 9, 7), (4, 4, 4), block_list_path=str(tmp_path / 'missing.json'))


# ---------------------------------------------------------------- native chunk codec (ctg_io_*)
def _with_codec(monkeypatch, native):
    monkeypatch.setattr(n5, '_NATIVE', None)
    if native:
        monkeypatch.delenv('CTG_IO_PYTHON', raising=False)
    else:
        monkeypatch.setenv('CTG_IO_PYTHON', '1')


@pytest.mark.parametrize('ext,comp,dtype', [('n5', 'gzip', 'uint64'), ('n5', 'raw', 'float32'),
                                            ('n5', 'gzip', 'uint8'), ('zarr', 'gzip', 'uint64'),
                                            ('zarr', 'raw', 'float32')])
@pytest.mark.parametrize('writer', ['native', 'python'])
def test_native_codec_matches_python(tmp_path, monkeypatch, ext, comp, dtype, writer):
    """libctg.so's threaded chunk codec and the Python codec read each other's
    chunks (edge chunks, missing chunks, boxes not aligned to chunks)."""
    rng = np.random.default_rng(2)
    data = rng.integers(0, 255, (19, 23, 30)).astype(dtype)
    p = str(tmp_path / ('c.' + ext))
    _with_codec(monkeypatch, writer == 'native')
    assert (n5._native() is not None) == (writer == 'native')
    with n5.file_reader(p) as f:
        ds = f.create_dataset('d', shape=data.shape, chunks=(4, 8, 7), dtype=dtype, compression=comp)
        ds[:16, :, :] = data[:16]          # chunk-aligned box: batched writer
        ds[16:, :, :] = data[16:]          # unaligned box: read-modify-write
        ds.n_threads = 3
    for reader in ('native', 'python'):
        _with_codec(monkeypatch, reader == 'native')
        with n5.file_reader(p, 'r') as f:
            ds = f['d']
            np.testing.assert_array_equal(ds[:], data)
            np.testing.assert_array_equal(ds[3:17, 5:21, 2:29], data[3:17, 5:21, 2:29])
            np.testing.assert_array_equal(ds[7, 2:9, :], data[7, 2:9, :])
    # a missing chunk reads as zeros
    _with_codec(monkeypatch, True)
    import shutil
    if ext == 'n5':
        os.remove(str(tmp_path / "c.n5" / "d" / "0" / "0" / "0"))     # chunk (0,0,0) = <x>/<y>/<z>
    else:
        os.remove(str(tmp_path / 'c.zarr' / 'd' / '0.0.0'))
    with n5.file_reader(p, 'r') as f:
        assert not f['d'][:4, :8, :7].any()
        np.testing.assert_array_equal(f['d'][4:, :, :], data[4:])


def test_native_varlen_batches(tmp_path, monkeypatch):
    _with_codec(monkeypatch, True)
    p = str(tmp_path / 'v.n5')
    rng = np.random.default_rng(3)
    with n5.File(p) as f:
        ds = f.create_dataset('s', shape=(10, 10, 10), chunks=(5, 5, 5), dtype='uint64', compression='gzip')
        pos = [(0, 0, 0), (1, 0, 1), (1, 1, 1), (0, 1, 0)]
        vals = [rng.integers(0, 2 ** 63, n, dtype=np.uint64) for n in (0, 7, 1000, 3)]
        ds.write_chunks(pos, vals, varlen=True, n_threads=4)
        got = ds.read_chunks(pos + [(1, 1, 0)], n_threads=4)
        assert got[-1] is None
        for a, b in zip(got, vals):
            np.testing.assert_array_equal(a, b)
        # python reader on native-written varlen chunks and vice versa
        _with_codec(monkeypatch, False)
        for pp, v in zip(pos, vals):
            np.testing.assert_array_equal(ds.read_chunk(pp), v)
        ds.write_chunk((0, 0, 1), vals[2], True)
        _with_codec(monkeypatch, True)
        np.testing.assert_array_equal(ds.read_chunks([(0, 0, 1)])[0], vals[2])
        # a default-mode chunk is not a varlength chunk
        f.create_dataset('d', data=np.ones((4, 4, 4), np.uint64), chunks=(2, 2, 2))
        with pytest.raises(OSError):
            f['d'].read_chunks([(0, 0, 0)])


def test_native_chunk_cache_sees_rewrites_and_threads(tmp_path, monkeypatch):
    """ctg_io_read_box's decoded-chunk cache: re-reads after a native or a
    Python rewrite of a chunk return the new data; concurrent overlapping
    reads (the halo of neighbouring blocks) agree."""
    from concurrent.futures import ThreadPoolExecutor
    _with_codec(monkeypatch, True)
    p = str(tmp_path / 'c.n5')
    rng = np.random.default_rng(4)
    data = rng.integers(0, 2 ** 40, (24, 40, 40), dtype=np.uint64)
    with n5.File(p) as f:
        ds = f.create_dataset('d', shape=data.shape, chunks=(8, 16, 16), dtype='uint64', compression='gzip')
        ds[:] = data
        np.testing.assert_array_equal(ds[:], data)
        boxes = [(slice(max(z - 1, 0), z + 8), slice(max(y - 1, 0), y + 16), slice(max(x - 1, 0), x + 16))
                 for z in range(0, 24, 8) for y in range(0, 40, 16) for x in range(0, 40, 16)]
        with ThreadPoolExecutor(8) as ex:
            outs = list(ex.map(lambda b: ds[b], boxes * 3))
        for b, o in zip(boxes * 3, outs):
            np.testing.assert_array_equal(o, data[b])
        new = data[:8, :16, :16] + np.uint64(7)
        ds.write_chunks([(0, 0, 0)], [new])                       # native write drops the entry
        np.testing.assert_array_equal(ds[:8, :16, :16], new)
        _with_codec(monkeypatch, False)
        ds.write_chunk((0, 0, 0), new + np.uint64(1))             # python write: the file stamp changes
        _with_codec(monkeypatch, True)
        np.testing.assert_array_equal(ds[:8, :16, :16], new + np.uint64(1))
    n5._native().ctg_io_cache_clear()


def test_native_readahead_follows_the_job_stride(tmp_path, monkeypatch):
    """a job walks every n_jobs-th block (block_list[k::n_jobs]),
    so the readahead queues the boxes one stride, two strides, ... past the last
    read (the step between this thread's last two reads of the dataset), not
    the C-order successors, which belong to another job; it looks kAhead (8)
    boxes ahead (one block = one gzip chunk decodes on one thread, so a single
    box of lookahead paced a job at one decode per call), stops at the grid's
    end and skips chunks already decoded or in flight."""
    import ctypes
    import time
    _with_codec(monkeypatch, True)
    lib = n5._native()
    p = str(tmp_path / 's.n5')
    nb = 24
    data = np.arange(8 * 16 * 16 * nb, dtype=np.uint64).reshape(8, 16, 16 * nb)
    with n5.File(p) as f:
        ds = f.create_dataset('d', shape=data.shape, chunks=(8, 16, 16), dtype='uint64', compression='gzip')
        ds[:] = data
        lib.ctg_io_cache_clear()

        def stats():
            out = np.zeros(3, np.int64)
            lib.ctg_io_cache_stats(out.ctypes.data_as(ctypes.c_void_p))
            return out

        def settle(before, n):
            for _ in range(300):   # the readahead pool works in the background
                s = stats()
                if s[2] - before[2] >= n:
                    break
                time.sleep(0.01)
            time.sleep(0.05)
            return stats()

        def read(i):
            np.testing.assert_array_equal(ds[:, :, 16 * i:16 * i + 16], data[:, :, 16 * i:16 * i + 16])

        s0 = stats()
        read(0)                  # no history: the C-order successors 1..8 are queued
        s1 = settle(s0, 8)
        assert s1[1] - s0[1] == 1 and s1[2] - s0[2] == 8
        read(3)                  # a hit; stride 3: 6 (known), 9, 12, 15, 18, 21 queued (24 leaves the grid)
        s2 = settle(s1, 5)
        assert s2[0] - s1[0] == 1 and s2[1] == s1[1] and s2[2] - s1[2] == 5
        for i in (6, 9, 12, 15, 18, 21):   # every one served by the readahead, nothing more queued
            read(i)
        time.sleep(0.1)
        s3 = stats()
        assert s3[0] - s2[0] == 6 and s3[1] == s2[1] and s3[2] == s2[2]
        read(10)                 # never queued along the stride: decoded by the caller
        assert stats()[1] - s3[1] == 1
    lib.ctg_io_cache_clear()


def test_native_writer_follows_the_declared_stream_type(tmp_path, monkeypatch):
    """N5 gzip with "useZlib": true and zarr "zlib" get zlib streams from the
    native writer (plain zlib.decompress reads them), N5 / zarr "gzip" get gzip
    streams (magic 1f 8b), as numcodecs / z5 readers of that metadata expect."""
    import json
    import zlib
    _with_codec(monkeypatch, True)
    data = np.arange(4 * 8 * 8, dtype=np.uint64).reshape(4, 8, 8)
    cases = [('n5', {'type': 'gzip', 'level': 3, 'useZlib': True}, 'zlib'),
             ('n5', {'type': 'gzip', 'level': 3, 'useZlib': False}, 'gzip'),
             ('zarr', {'type': 'gzip', 'level': 3, 'useZlib': True}, 'zlib'),
             ('zarr', {'type': 'gzip', 'level': 3, 'useZlib': False}, 'gzip')]
    for i, (ext, comp, stream) in enumerate(cases):
        p = str(tmp_path / ('s%d.%s' % (i, ext)))
        with n5.file_reader(p) as f:
            ds = f.create_dataset('d', shape=data.shape, chunks=(4, 8, 8), dtype='uint64', compression=comp)
            ds[:] = data                                    # aligned: the native batched writer
        if ext == 'n5':
            with open(os.path.join(p, 'd', '0', '0', '0'), 'rb') as fh:
                buf = fh.read()[4 + 4 * 3:]
            raw_dt = '>u8'
        else:
            assert json.load(open(os.path.join(p, 'd', '.zarray')))['compressor']['id'] == stream
            with open(os.path.join(p, 'd', '0.0.0'), 'rb') as fh:
                buf = fh.read()
            raw_dt = '<u8'
        if stream == 'zlib':
            raw = zlib.decompress(buf)
        else:
            assert buf[:2] == b'\x1f\x8b'
            raw = zlib.decompress(buf, 16 + zlib.MAX_WBITS)
        np.testing.assert_array_equal(np.frombuffer(raw, dtype=raw_dt).reshape(data.shape), data)


def test_native_cache_sees_same_size_raw_rewrite(tmp_path, monkeypatch):
    """Uncompressed chunks keep their size on rewrite and a quick rewrite may
    keep the mtime: the decoded-chunk cache keys on the inode (rewrites are
    renames) and the Python writer drops the entry."""
    _with_codec(monkeypatch, True)
    p = str(tmp_path / 'r.n5')
    data = np.arange(8 * 8 * 8, dtype=np.uint32).reshape(8, 8, 8)
    with n5.File(p) as f:
        ds = f.create_dataset('d', shape=data.shape, chunks=(8, 8, 8), dtype='uint32', compression='raw')
        ds[:] = data
        for k in range(1, 6):
            np.testing.assert_array_equal(ds[:], data + k - 1)
            ds.write_chunk((0, 0, 0), data + k)             # python writer, same size
        np.testing.assert_array_equal(ds[:], data + 5)
    n5._native().ctg_io_cache_clear()


def test_zarr_fill_value_and_big_endian(tmp_path, monkeypatch):
    """zarr: missing chunks read as the array's fill_value on both codecs;
    a '>u8' array written by the native writer lands big-endian on disk."""
    import json
    for native in (True, False):
        _with_codec(monkeypatch, native)
        p = str(tmp_path / ('z%d.zarr' % native))
        data = np.arange(6 * 8 * 10, dtype=np.uint64).reshape(6, 8, 10) * np.uint64(1 << 33)
        with n5.file_reader(p) as f:
            f.create_dataset('d', shape=data.shape, chunks=(3, 8, 5), dtype='>u8', compression='raw')
        meta_p = os.path.join(p, 'd', '.zarray')
        meta = json.load(open(meta_p))
        meta['fill_value'] = 7
        json.dump(meta, open(meta_p, 'w'))
        with n5.file_reader(p) as f:
            ds = f['d']
            ds[:3] = data[:3]                               # chunks (1, *, *) stay missing
            got = ds[:]
            np.testing.assert_array_equal(got[:3], data[:3])
            assert np.all(got[3:] == 7)
        with open(os.path.join(p, 'd', '0.0.0'), 'rb') as fh:
            raw = np.frombuffer(fh.read(), dtype='>u8').reshape(3, 8, 5)
        np.testing.assert_array_equal(raw, data[:3, :, :5])


def serialize_argmax_multiset(labels):
    """A label multiset of one label per voxel in the imglib2 / paintera N5
    serialisation (test-side writer, the restated format of n5.Dataset.
    _read_multiset_chunk): int32 n, n x int64 argmax, n x int32 list offsets,
    lists (int32 size, size x (int64 id, int32 count)), big-endian."""
    flat = np.asarray(labels, dtype=np.uint64).ravel()
    uniq, inv = np.unique(flat, return_inverse=True)
    lists = b''.join(struct.pack('>iqi', 1, int(u), 1) for u in uniq)
    offsets = (inv * 16).astype('>i4')
    head = struct.pack('>i', flat.size)
    return np.frombuffer(head + flat.astype('>i8').tobytes() + offsets.tobytes() + lists, dtype=np.uint8)


def write_multiset_dataset(group, key, labels, chunks):
    ds = group.create_dataset(key, shape=labels.shape, chunks=chunks, dtype='uint8', compression='gzip')
    ds.attrs['isLabelMultiset'] = True
    ds.attrs['maxId'] = int(labels.max())
    blk = B.blocking([0, 0, 0], list(labels.shape), list(chunks))
    for b in range(blk.numberOfBlocks):
        bb = blk.getBlock(b)
        sl = tuple(slice(x, y) for x, y in zip(bb.begin, bb.end))
        if labels[sl].sum() == 0:      # create_multiset.py:118-121 skips empty blocks
            continue
        ds.write_chunk(blk.blockGridPosition(b), serialize_argmax_multiset(labels[sl]), True)


def test_label_multiset_reads_as_argmax(tmp_path):
    lab, _ = S.generate((20, 30, 26), cell=5, seed=12, with_boundary=False)
    lab[:8, :10, :10] = 0                                    # an empty (unwritten) chunk
    with n5.File(str(tmp_path / 'm.n5')) as f:
        write_multiset_dataset(f, 'ms', lab, (8, 10, 10))
    with n5.File(str(tmp_path / 'm.n5'), 'r') as f:
        ds = f['ms']
        assert ds.is_label_multiset and ds.dtype == np.uint64
        np.testing.assert_array_equal(ds[:], lab)
        np.testing.assert_array_equal(ds[3:17, 4:29, 1:25], lab[3:17, 4:29, 1:25])


def _square_job(x):
    if x < 0:
        raise ValueError('negative job %d' % x)
    return x * x


def test_harness_job_processes_order_and_failure():
    """harness.workflow's process mode (LocalTask's model, cluster_tasks.py:
    528-550): one spawned process per job, results in job order, a failing
    job fails the task with its traceback."""
    from harness import workflow
    assert workflow._run_jobs(_square_job, [3, 1, 2], 'processes') == [9, 1, 4]
    assert workflow._run_jobs(_square_job, [3, 1, 2], 'threads') == [9, 1, 4]
    with pytest.raises(RuntimeError, match='negative job -1'):
        workflow._run_jobs(_square_job, [2, -1], 'processes')
    with pytest.raises(ValueError):
        workflow._run_jobs(_square_job, [1], 'fibers')


@pytest.mark.parametrize('dtype', ['uint8', 'int16', 'uint16', 'float32', 'uint32', 'float64', 'uint64', 'int64'])
def test_native_codec_byte_swaps_every_width(tmp_path, monkeypatch, dtype):
    """N5 payloads are big-endian: the native codec's word-wise swaps (2 / 4 /
    8 bytes) agree with numpy's '>' dtypes, for box reads, varlen chunks and
    raw / gzip payloads."""
    _with_codec(monkeypatch, True)
    rng = np.random.default_rng(11)
    info = np.iinfo(dtype) if np.dtype(dtype).kind in 'iu' else None
    data = (rng.integers(info.min, info.max, (9, 20, 17), dtype=dtype, endpoint=True) if info is not None
            else rng.standard_normal((9, 20, 17)).astype(dtype))
    for comp in ('raw', 'gzip'):
        p = str(tmp_path / ('%s_%s.n5' % (dtype, comp)))
        with n5.File(p) as f:
            ds = f.create_dataset('d', shape=data.shape, chunks=(4, 8, 8), dtype=dtype, compression=comp)
            ds[:] = data                                        # native aligned writer
            np.testing.assert_array_equal(ds[:], data)          # native box reader
            np.testing.assert_array_equal(ds[1:8, 3:19, 2:15], data[1:8, 3:19, 2:15])
            with open(os.path.join(p, 'd', '0', '0', '0'), 'rb') as fh:
                buf = fh.read()[4 + 4 * 3:]
            raw = zlib.decompress(buf, 16 + zlib.MAX_WBITS) if comp == 'gzip' else buf
            np.testing.assert_array_equal(np.frombuffer(raw, dtype=np.dtype(dtype).newbyteorder('>')).reshape(4, 8, 8),
                                          data[:4, :8, :8])
            flat = data.ravel()[:1000]
            ds.write_chunks([(0, 0, 1)], [flat], varlen=True)   # varlen chunk, native writer and reader
            np.testing.assert_array_equal(ds.read_chunks([(0, 0, 1)])[0], flat)
    n5._native().ctg_io_cache_clear()
