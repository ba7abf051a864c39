"""Minimal N5 container codec (the subset of z5py the hot path uses).

The reference's hot-path tasks read and write N5 through z5py / elf
(utils/volume_utils.py:21-22); z5py is not installed in this image, so the
ndist mirror needs its own codec.  Format (N5 spec 2.0, as written by z5):

* group / dataset = directory with ``attributes.json``; the root carries
  ``{"n5": "2.0.0"}``.  Dataset metadata ``dimensions``, ``blockSize`` are in
  REVERSED (F) axis order relative to the numpy/z5py shape; ``dataType`` is a
  numpy-style name, ``compression`` is ``{"type": "gzip", ...}`` or
  ``{"type": "raw"}``.  User attributes live in the same JSON object.
* chunk at grid position (i0, ..., in) is the file ``<ds>/in/.../i0``.
* chunk = big-endian header: uint16 mode (0 default, 1 varlength), uint16
  ndim, ndim x uint32 chunk dims (reversed), and for mode 1 a uint32 element
  count; then the (gzip/zlib or raw) payload of BIG-ENDIAN elements.
* ``read_chunk`` of a missing chunk returns None (test_graph.py:63-66,
  block_edge_features.py:181-185); ``write_chunk(pos, data, True)`` writes a
  varlength chunk (block_edge_features.py:236).

zarr v2 containers (``.zr`` / ``.zarr``, accepted by graph_workflow.py:17-20
and features_workflow.py:24-29 for the input volumes) are read and written by
the same classes: ``.zgroup`` / ``.zarray`` / ``.zattrs`` metadata in C axis
order, chunk keys ``i.j.k`` (or ``i/j/k`` with dimension_separator "/"),
edge chunks stored at full chunk shape, missing chunks = fill_value, and the
gzip / zlib / uncompressed codecs.  Blosc (zarr's default codec) needs the
c-blosc library, which this image does not have: such arrays raise on access.
"""
from __future__ import annotations

import json
import os
import struct
import threading
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_ATTR = 'attributes.json'
_lock = threading.Lock()


def _read_json(path, name=_ATTR):
    p = os.path.join(path, name)
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def _write_json(path, d, name=_ATTR):
    os.makedirs(path, exist_ok=True)
    tmp = os.path.join(path, name + '.tmp%d_%d' % (os.getpid(), threading.get_ident()))
    with open(tmp, 'w') as f:
        json.dump(d, f)
    os.replace(tmp, os.path.join(path, name))


_ZGROUP, _ZARRAY, _ZATTRS = '.zgroup', '.zarray', '.zattrs'


def is_container_root(path):
    """True for the root directory of an N5 or zarr container."""
    if not os.path.isdir(path):
        return False
    if path.rstrip('/').lower().endswith(('.n5', '.zr', '.zarr')):
        return True
    return 'n5' in _read_json(path)


def _is_zarr_path(path):
    return path.rstrip('/').split('.')[-1].lower() in ('zr', 'zarr')


class Attributes:
    """dict-like view of the user attributes (N5: inside attributes.json,
    zarr: .zattrs)."""
    _RESERVED = ('dimensions', 'blockSize', 'dataType', 'compression', 'n5')

    def __init__(self, path, name=_ATTR):
        self.path = path
        self.name = name

    def _load(self):
        return _read_json(self.path, self.name)

    def __getitem__(self, k):
        return self._load()[k]

    def get(self, k, default=None):
        return self._load().get(k, default)

    def __setitem__(self, k, v):
        if isinstance(v, np.generic):
            v = v.item()
        if isinstance(v, np.ndarray):
            v = v.tolist()
        if isinstance(v, tuple):
            v = list(v)
        with _lock:
            d = self._load()
            d[k] = v
            _write_json(self.path, d, self.name)

    def __contains__(self, k):
        return k in self._load()

    def keys(self):
        return [k for k in self._load() if k not in self._RESERVED]

    def items(self):
        d = self._load()
        return [(k, d[k]) for k in d if k not in self._RESERVED]


def _normalize_compression(compression):
    if compression in (None, 'raw'):
        return {'type': 'raw'}
    if compression == 'gzip':
        return {'type': 'gzip', 'level': 5, 'useZlib': False}
    if isinstance(compression, dict):
        return compression
    raise ValueError('unsupported compression %r' % (compression,))


_NATIVE = None


def _native():
    """libctg.so's chunk codec (ctg_io_*), or None when the library is not
    built (the pure-Python codec below is then used; it is also the reference
    the native one is tested against)."""
    global _NATIVE
    if _NATIVE is None:
        if os.environ.get('CTG_IO_PYTHON'):
            _NATIVE = False
        else:
            try:
                from . import _lib
                _NATIVE = _lib.load()
            except Exception:
                _NATIVE = False
    return _NATIVE or None


def _replace_file(path, buf):
    """Atomic chunk write (tmp file + rename), then drop the native codec's
    cached decode of that chunk (ctg_io_read_box would otherwise keep serving
    it if the rewrite kept size and mtime)."""
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + '.tmp%d_%d' % (os.getpid(), threading.get_ident())
    with open(tmp, 'wb') as f:
        f.write(buf)
    os.replace(tmp, path)
    lib = _native()
    if lib is not None:
        lib.ctg_io_cache_drop(path.encode())


def _io_threads(n_threads):
    return max(1, int(n_threads) if n_threads and n_threads > 1 else min(16, os.cpu_count() or 1))


def _i64(vals):
    import ctypes
    vals = [int(v) for v in vals]
    return (ctypes.c_int64 * max(1, len(vals)))(*vals)


def _decompress(buf):
    if len(buf) >= 2 and buf[0] == 0x1F and buf[1] == 0x8B:
        return zlib.decompress(buf, 16 + zlib.MAX_WBITS)
    return zlib.decompress(buf)


class Dataset:
    def __init__(self, path):
        self.path = path
        meta = _read_json(path)
        if 'dimensions' not in meta:
            raise KeyError('%s is not an N5 dataset' % path)
        self.shape = tuple(int(s) for s in meta['dimensions'][::-1])
        self.chunks = tuple(int(s) for s in meta['blockSize'][::-1])
        self.dtype = np.dtype(meta['dataType'])
        self.compression = meta.get('compression', {'type': 'raw'})
        self.attrs = Attributes(path)
        self.n_threads = 1
        # paintera / imglib2 label multisets (uint8 varlen chunks, attribute
        # isLabelMultiset): read as their per-voxel argmax labels (uint64)
        self.is_label_multiset = bool(meta.get('isLabelMultiset', False))
        if self.is_label_multiset:
            self.dtype = np.dtype('uint64')

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def size(self):
        return int(np.prod(self.shape))

    def __len__(self):
        return self.shape[0]

    # --- chunk level -----------------------------------------------------
    def _chunk_path(self, pos):
        return os.path.join(self.path, *[str(int(p)) for p in pos[::-1]])

    def chunk_exists(self, pos):
        return os.path.exists(self._chunk_path(pos))

    # --- native fast paths (ctg_io_*) ------------------------------------
    _FORMAT = 0        # CTG_IO_N5

    def _big_endian(self):
        return 1

    def _ctype(self):
        """CTG_IO_RAW / CTG_IO_GZIP / CTG_IO_ZLIB (N5 gzip with "useZlib": zlib
        streams), None for codecs the native path lacks."""
        c = self.compression.get('type', 'raw')
        if c == 'gzip':
            return 2 if self.compression.get('useZlib', False) else 1
        return {'raw': 0}.get(c)

    def _level(self):
        lv = self.compression.get('level', 5)
        return 5 if lv is None or lv < 0 else int(lv)

    def read_box_native(self, bb, n_threads=None, out=None):
        """C-order box [(b, e), ...] through ctg_io_read_box (into ``out`` if
        given: a C-contiguous native-endian array of the box's shape, e.g. a
        view of a page-locked staging arena), or None without the library."""
        lib = _native()
        ct = self._ctype()
        if lib is None or ct is None or self.is_label_multiset:
            return None
        import ctypes
        shape = tuple(e - b for b, e in bb)
        if out is None:
            out = np.empty(shape, dtype=self.dtype.newbyteorder('='))
        elif tuple(out.shape) != shape or out.dtype != self.dtype.newbyteorder('=') or not out.flags.c_contiguous:
            raise ValueError('read_box_native: out must be a C-contiguous %s array of shape %s'
                             % (self.dtype, shape))
        fv = getattr(self, 'fill_value', 0)
        fill = None
        if fv:   # missing chunks read as the array's fill value (zarr), else zeros
            fill = np.array([fv], dtype=self.dtype.newbyteorder('='))
        rc = lib.ctg_io_read_box(self.path.encode(), self._FORMAT, self.dtype.itemsize, self._big_endian(),
                                 self.ndim, _i64(self.shape), _i64(self.chunks), ct, _i64([b for b, _ in bb]),
                                 _i64([e for _, e in bb]), out.ctypes.data_as(ctypes.c_void_p),
                                 _io_threads(n_threads or self.n_threads),
                                 None if fill is None else fill.ctypes.data_as(ctypes.c_void_p))
        if rc != 0:
            msg = lib.ctg_last_error()
            raise OSError(msg.decode() if msg else 'ctg_io_read_box failed')
        return out

    def write_chunks(self, positions, datas, varlen=False, n_threads=None):
        """Write many chunks at once (native thread pool when available).
        Default-mode chunks must have their grid cell's shape."""
        positions = [tuple(int(p) for p in pos) for pos in positions]
        # native byte order: the codec swaps to the stored order itself (_big_endian)
        datas = [np.ascontiguousarray(np.asarray(d, dtype=self.dtype.newbyteorder('='))) for d in datas]
        lib = _native()
        ct = self._ctype()
        if lib is None or ct is None or not positions:
            for pos, d in zip(positions, datas):
                self.write_chunk(pos, d, varlen)
            return
        import ctypes
        nd = self.ndim
        shapes = []
        for pos, d in zip(positions, datas):
            cs = self._chunk_shape(pos)
            if not varlen and self._FORMAT == 0 and tuple(d.shape) != tuple(cs):
                raise ValueError('chunk %s has shape %s, expected %s' % (pos, d.shape, cs))
            shapes.append(cs)
        n = len(positions)
        ptrs = (ctypes.c_void_p * n)(*[d.ctypes.data for d in datas])
        counts = _i64([d.size for d in datas])
        rc = lib.ctg_io_write_chunks(self.path.encode(), self._FORMAT, self.dtype.itemsize, self._big_endian(), nd,
                                     n, _i64([x for pos in positions for x in pos]),
                                     _i64([x for cs in shapes for x in cs]), ptrs, counts, int(bool(varlen)), ct,
                                     self._level(), _io_threads(n_threads or self.n_threads))
        if rc != 0:
            msg = lib.ctg_last_error()
            raise OSError(msg.decode() if msg else 'ctg_io_write_chunks failed')

    def read_chunks(self, positions, n_threads=None):
        """Varlength chunks at many grid positions (None where missing)."""
        positions = [tuple(int(p) for p in pos) for pos in positions]
        lib = _native()
        ct = self._ctype()
        if lib is None or ct is None or self._FORMAT != 0 or not positions:
            return [self.read_chunk(pos) for pos in positions]
        import ctypes
        n = len(positions)
        outs = (ctypes.c_void_p * n)()
        counts = (ctypes.c_int64 * n)()
        rc = lib.ctg_io_read_varlen(self.path.encode(), self.dtype.itemsize, self.ndim, n,
                                    _i64([x for pos in positions for x in pos]), ct, outs, counts,
                                    _io_threads(n_threads or self.n_threads))
        if rc != 0:
            msg = lib.ctg_last_error()
            raise OSError(msg.decode() if msg else 'ctg_io_read_varlen failed')
        res = []
        dt = self.dtype.newbyteorder('=')
        for i in range(n):
            if counts[i] < 0:
                res.append(None)
                continue
            if counts[i]:
                # one copy out of the native buffer (a bytes() round trip would make two)
                buf = (ctypes.c_char * (int(counts[i]) * dt.itemsize)).from_address(outs[i])
                res.append(np.frombuffer(buf, dtype=dt).copy())
            else:
                res.append(np.zeros(0, dt))
            lib.ctg_io_free(outs[i])
        return res

    def _encode(self, arr, varlen, shape):
        be = np.ascontiguousarray(arr).astype(self.dtype.newbyteorder('>'), copy=False).tobytes()
        hdr = struct.pack('>HH', 1 if varlen else 0, len(shape))
        hdr += struct.pack('>' + 'I' * len(shape), *[int(s) for s in shape[::-1]])
        if varlen:
            hdr += struct.pack('>I', int(arr.size))
        ctype = self.compression.get('type', 'raw')
        if ctype == 'gzip':
            level = self.compression.get('level', 5)
            level = 5 if level is None or level < 0 else level
            if self.compression.get('useZlib', False):
                payload = zlib.compress(be, level)
            else:
                co = zlib.compressobj(level, zlib.DEFLATED, 16 + zlib.MAX_WBITS)
                payload = co.compress(be) + co.flush()
        elif ctype == 'raw':
            payload = be
        else:
            raise ValueError('unsupported compression %s' % ctype)
        return hdr + payload

    def write_chunk(self, pos, data, varlen=False):
        pos = tuple(int(p) for p in pos)
        data = np.asarray(data, dtype=self.dtype)
        if varlen:
            shape = self._chunk_shape(pos)
            buf = self._encode(data.ravel(), True, shape)
        else:
            shape = data.shape
            buf = self._encode(data, False, shape)
        _replace_file(self._chunk_path(pos), buf)

    def _read_multiset_chunk(self, pos):
        """argmax labels of a label-multiset chunk, or None if missing.

        Serialisation (imglib2 / paintera N5 label multisets, written by
        elf.label_multiset.serialize_multiset, label_multisets/create_multiset.py:
        123-131), all big-endian: int32 n = voxels of the chunk, n x int64
        argmax label per voxel, n x int32 byte offset of the voxel's entry list,
        then the entry lists (int32 length, length x (int64 id, int32 count)).
        The graph only needs the argmax (test_graph.py:140-161 compares the
        multiset graph with the graph of the argmax segmentation).  Parity
        unpinned: neither elf nor a fixture of the format is available here."""
        p = self._chunk_path(pos)
        if not os.path.exists(p):
            return None
        with open(p, 'rb') as f:
            buf = f.read()
        mode, nd = struct.unpack_from('>HH', buf, 0)
        off = 4 + 4 * nd + (4 if mode == 1 else 0)
        ctype = self.compression.get('type', 'raw')
        raw = _decompress(buf[off:]) if ctype == 'gzip' else buf[off:]
        shape = self._chunk_shape(tuple(int(x) for x in pos))
        n_vox = int(np.prod(shape))
        (n,) = struct.unpack_from('>i', raw, 0)
        if n != n_vox or len(raw) < 4 + 12 * n:
            raise ValueError('label multiset chunk %s: %d argmax entries for a %s chunk' % (p, n, shape))
        return np.frombuffer(raw, dtype='>i8', count=n, offset=4).astype(np.uint64).reshape(shape)

    def read_chunk(self, pos):
        """Chunk data (varlen chunks as 1-D arrays) or None if missing."""
        if self.is_label_multiset:
            return self._read_multiset_chunk(pos)
        p = self._chunk_path(pos)
        if not os.path.exists(p):
            return None
        with open(p, 'rb') as f:
            buf = f.read()
        mode, nd = struct.unpack_from('>HH', buf, 0)
        off = 4
        dims = struct.unpack_from('>' + 'I' * nd, buf, off)[::-1]
        off += 4 * nd
        n = None
        if mode == 1:
            (n,) = struct.unpack_from('>I', buf, off)
            off += 4
        payload = buf[off:]
        ctype = self.compression.get('type', 'raw')
        raw = _decompress(payload) if ctype == 'gzip' else payload
        arr = np.frombuffer(raw, dtype=self.dtype.newbyteorder('>')).astype(self.dtype)
        if mode == 1:
            return arr[:n]
        return arr.reshape(dims)

    def _chunk_shape(self, pos):
        return tuple(min(c, s - p * c) for p, c, s in zip(pos, self.chunks, self.shape))

    # --- array level -----------------------------------------------------
    def _norm_index(self, index):
        if not isinstance(index, tuple):
            index = (index,)
        if any(i is Ellipsis for i in index):
            k = index.index(Ellipsis)
            index = index[:k] + (slice(None),) * (self.ndim - len(index) + 1) + index[k + 1:]
        index = index + (slice(None),) * (self.ndim - len(index))
        bb, squeeze = [], []
        for ax, (i, s) in enumerate(zip(index, self.shape)):
            if isinstance(i, slice):
                b, e, st = i.indices(s)
                assert st == 1, 'strided N5 access is not supported'
                bb.append((b, max(b, e)))
            else:
                i = int(i)
                i = i + s if i < 0 else i
                bb.append((i, i + 1))
                squeeze.append(ax)
        return bb, tuple(squeeze)

    def _chunks_in(self, bb):
        rng = [range(b // c, (e + c - 1) // c) if e > b else range(0) for (b, e), c in zip(bb, self.chunks)]
        return np.stack(np.meshgrid(*rng, indexing='ij'), -1).reshape(-1, len(bb)) if all(len(r) for r in rng) \
            else np.zeros((0, len(bb)), dtype=np.int64)

    def __getitem__(self, index):
        bb, squeeze = self._norm_index(index)
        nat = self.read_box_native(bb)
        if nat is not None:
            return nat.squeeze(axis=squeeze) if squeeze else nat
        out = np.full(tuple(e - b for b, e in bb), getattr(self, 'fill_value', 0), dtype=self.dtype)

        def one(pos):
            data = self.read_chunk(pos)
            if data is None:
                return
            cb = [p * c for p, c in zip(pos, self.chunks)]
            src, dst = [], []
            for (b, e), c0, cs in zip(bb, cb, data.shape):
                lo, hi = max(b, c0), min(e, c0 + cs)
                src.append(slice(lo - c0, hi - c0))
                dst.append(slice(lo - b, hi - b))
            out[tuple(dst)] = data[tuple(src)]

        chunks = [tuple(int(x) for x in p) for p in self._chunks_in(bb)]
        if self.n_threads > 1 and len(chunks) > 1:
            with ThreadPoolExecutor(self.n_threads) as ex:
                list(ex.map(one, chunks))
        else:
            for c in chunks:
                one(c)
        return out.squeeze(axis=squeeze) if squeeze else out

    def __setitem__(self, index, value):
        bb, _ = self._norm_index(index)
        shape = tuple(e - b for b, e in bb)
        value = np.broadcast_to(np.asarray(value, dtype=self.dtype), shape)
        aligned = all(b % c == 0 and (e % c == 0 or e == s) for (b, e), c, s in zip(bb, self.chunks, self.shape))
        if aligned and _native() is not None and self._ctype() is not None and all(x > 0 for x in shape):
            pos_list = [tuple(int(x) for x in p) for p in self._chunks_in(bb)]
            datas = []
            for pos in pos_list:
                cs = self._chunk_shape(pos)
                src = tuple(slice(p * c - b, p * c - b + n) for p, c, (b, _), n in zip(pos, self.chunks, bb, cs))
                datas.append(value[src])
            self.write_chunks(pos_list, datas)
            return

        def one(pos):
            cb = [p * c for p, c in zip(pos, self.chunks)]
            cshape = self._chunk_shape(pos)
            src, dst, full = [], [], True
            for (b, e), c0, cs in zip(bb, cb, cshape):
                lo, hi = max(b, c0), min(e, c0 + cs)
                src.append(slice(lo - b, hi - b))
                dst.append(slice(lo - c0, hi - c0))
                full &= (lo == c0 and hi == c0 + cs)
            if full:
                chunk = np.ascontiguousarray(value[tuple(src)])
            else:
                chunk = self.read_chunk(pos)
                if chunk is None or chunk.shape != cshape:
                    chunk = np.zeros(cshape, dtype=self.dtype)
                else:
                    chunk = chunk.copy()
                chunk[tuple(dst)] = value[tuple(src)]
            self.write_chunk(pos, chunk)

        chunks = [tuple(int(x) for x in p) for p in self._chunks_in(bb)]
        if self.n_threads > 1 and len(chunks) > 1:
            with ThreadPoolExecutor(self.n_threads) as ex:
                list(ex.map(one, chunks))
        else:
            for c in chunks:
                one(c)


_ZARR_CODECS = ('gzip', 'zlib')


class ZarrArray(Dataset):
    """A zarr v2 array with the Dataset interface (C axis order)."""

    def __init__(self, path):
        self.path = path
        meta = _read_json(path, _ZARRAY)
        if 'shape' not in meta:
            raise KeyError('%s is not a zarr array' % path)
        if meta.get('order', 'C') != 'C':
            raise ValueError('zarr array %s: only C order is supported' % path)
        if meta.get('filters'):
            raise ValueError('zarr array %s: filters are not supported' % path)
        self.shape = tuple(int(x) for x in meta['shape'])
        self.chunks = tuple(int(x) for x in meta['chunks'])
        self.dtype = np.dtype(meta['dtype'])
        self.fill_value = meta.get('fill_value', 0) or 0
        self.compressor = meta.get('compressor')
        self.sep = meta.get('dimension_separator', '.')
        self.attrs = Attributes(path, _ZATTRS)
        self.n_threads = 1
        self.is_label_multiset = False

    @property
    def _FORMAT(self):  # noqa: N802
        return 2 if self.sep == '/' else 1   # CTG_IO_ZARR_SLASH / CTG_IO_ZARR_DOT

    def _big_endian(self):
        return 1 if self.dtype.byteorder == '>' else 0

    def _ctype(self):
        c = self.compressor
        if c is None:
            return 0
        # CTG_IO_GZIP / CTG_IO_ZLIB; other codecs: the Python path raises
        return {'gzip': 1, 'zlib': 2}.get(c.get('id'))

    def _level(self):
        lv = (self.compressor or {}).get('level', 5)
        return 5 if lv is None or lv < 0 else int(lv)

    def write_chunks(self, positions, datas, varlen=False, n_threads=None):
        if varlen:
            raise ValueError('zarr has no varlength chunks (the sub-graph datasets are N5)')
        full = []
        for d in datas:
            d = np.asarray(d, dtype=self.dtype)
            f = np.full(self.chunks, self.fill_value, dtype=self.dtype)
            f[tuple(slice(0, n) for n in d.shape)] = d
            full.append(f)
        Dataset.write_chunks(self, positions, full, False, n_threads)

    def _codec(self):
        c = self.compressor
        if c is None:
            return None
        cid = c.get('id')
        if cid not in _ZARR_CODECS:
            raise ValueError('zarr array %s: compressor %r is not available in this image (gzip, zlib or none '
                             'are supported)' % (self.path, cid))
        return cid

    def _chunk_path(self, pos):
        return os.path.join(self.path, self.sep.join(str(int(p)) for p in pos))

    def write_chunk(self, pos, data, varlen=False):
        if varlen:
            raise ValueError('zarr has no varlength chunks (the sub-graph datasets are N5)')
        pos = tuple(int(p) for p in pos)
        data = np.asarray(data, dtype=self.dtype)
        full = np.full(self.chunks, self.fill_value, dtype=self.dtype)
        full[tuple(slice(0, n) for n in data.shape)] = data
        raw = np.ascontiguousarray(full).tobytes()
        cid = self._codec()
        level = (self.compressor or {}).get('level', 5)
        if cid == 'gzip':
            co = zlib.compressobj(level, zlib.DEFLATED, 16 + zlib.MAX_WBITS)
            raw = co.compress(raw) + co.flush()
        elif cid == 'zlib':
            raw = zlib.compress(raw, level)
        _replace_file(self._chunk_path(pos), raw)

    def read_chunk(self, pos):
        p = self._chunk_path(pos)
        if not os.path.exists(p):
            return None
        with open(p, 'rb') as f:
            buf = f.read()
        raw = _decompress(buf) if self._codec() else buf
        arr = np.frombuffer(raw, dtype=self.dtype).reshape(self.chunks)
        cs = self._chunk_shape(tuple(int(x) for x in pos))
        return np.ascontiguousarray(arr[tuple(slice(0, n) for n in cs)])


class Group:
    def __init__(self, path, mode='a', zarr=False):
        self.path = path
        self.mode = mode
        self.zarr = zarr
        self.attrs = Attributes(path, _ZATTRS if zarr else _ATTR)

    def __contains__(self, key):
        return os.path.isdir(os.path.join(self.path, key))

    def __getitem__(self, key):
        p = os.path.join(self.path, key)
        if not os.path.isdir(p):
            raise KeyError(key)
        if self.zarr:
            if os.path.exists(os.path.join(p, _ZARRAY)):
                return ZarrArray(p)
            return Group(p, self.mode, True)
        meta = _read_json(p)
        if 'dimensions' in meta:
            return Dataset(p)
        return Group(p, self.mode)

    def keys(self):
        return sorted(d for d in os.listdir(self.path) if os.path.isdir(os.path.join(self.path, d)))

    def _make_group_dirs(self, p):
        if self.zarr:
            # every intermediate level is a zarr group
            rel = os.path.relpath(p, self.path).split(os.sep)
            cur = self.path
            for part in rel:
                cur = os.path.join(cur, part)
                os.makedirs(cur, exist_ok=True)
                if not os.path.exists(os.path.join(cur, _ZGROUP)):
                    _write_json(cur, {'zarr_format': 2}, _ZGROUP)
        else:
            os.makedirs(p, exist_ok=True)
            _write_json(p, _read_json(p))

    def require_group(self, key):
        p = os.path.join(self.path, key)
        if not os.path.isdir(p):
            if self.mode == 'r':
                raise ValueError('read-only container')
            self._make_group_dirs(p)
        return Group(p, self.mode, self.zarr)

    create_group = require_group

    def create_dataset(self, key, shape=None, chunks=None, dtype=None, compression='gzip', data=None, **kw):
        if data is not None:
            data = np.asarray(data)
            shape = data.shape if shape is None else shape
            dtype = data.dtype if dtype is None else dtype
        shape = tuple(int(s) for s in shape)
        chunks = tuple(int(c) for c in (chunks if chunks is not None else shape))
        chunks = tuple(max(1, c) for c in chunks)
        p = os.path.join(self.path, key)
        parent = os.path.dirname(p)
        if parent != self.path and not os.path.isdir(parent):
            self._make_group_dirs(parent)
        if self.zarr:
            comp = _normalize_compression(compression)
            zc = None if comp['type'] == 'raw' else {'id': 'zlib' if comp.get('useZlib') else 'gzip',
                                                     'level': comp.get('level', 5)}
            os.makedirs(p, exist_ok=True)
            _write_json(p, {'zarr_format': 2, 'shape': list(shape), 'chunks': list(chunks),
                            'dtype': np.dtype(dtype).str, 'compressor': zc, 'fill_value': 0, 'order': 'C',
                            'filters': None}, _ZARRAY)
            ds = ZarrArray(p)
        else:
            meta = _read_json(p)
            meta.update({'dimensions': list(shape[::-1]), 'blockSize': list(chunks[::-1]),
                         'dataType': np.dtype(dtype).name, 'compression': _normalize_compression(compression)})
            _write_json(p, meta)
            ds = Dataset(p)
        if data is not None:
            ds[...] = data
        return ds

    def require_dataset(self, key, shape, chunks=None, dtype=None, compression='gzip', **kw):
        p = os.path.join(self.path, key)
        exists = os.path.exists(os.path.join(p, _ZARRAY)) if self.zarr else \
            (os.path.isdir(p) and 'dimensions' in _read_json(p))
        if exists:
            ds = ZarrArray(p) if self.zarr else Dataset(p)
            if tuple(ds.shape) != tuple(int(s) for s in shape):
                raise ValueError('shape mismatch for existing dataset %s' % key)
            return ds
        return self.create_dataset(key, shape=shape, chunks=chunks, dtype=dtype, compression=compression)


class File(Group):
    """z5py.File-like N5 (or, for a .zr / .zarr path, zarr v2) container
    (context manager)."""

    def __init__(self, path, mode='a', use_zarr_format=None):
        zarr = _is_zarr_path(path) if use_zarr_format is None else bool(use_zarr_format)
        if mode != 'r':
            os.makedirs(path, exist_ok=True)
            if zarr:
                if not os.path.exists(os.path.join(path, _ZGROUP)):
                    _write_json(path, {'zarr_format': 2}, _ZGROUP)
            else:
                meta = _read_json(path)
                if 'n5' not in meta:
                    meta['n5'] = '2.0.0'
                    _write_json(path, meta)
        elif not os.path.isdir(path):
            raise OSError('no %s container at %s' % ('zarr' if zarr else 'N5', path))
        super().__init__(path, mode, zarr)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def close(self):
        pass


def file_reader(path, mode='a'):
    """vu.file_reader (utils/volume_utils.py:21-22) for the formats the hot path
    accepts (graph_workflow.py:17-20): N5 (.n5) and zarr (.zr / .zarr)."""
    ending = path.rstrip('/').split('.')[-1].lower()
    if ending not in ('n5', 'zr', 'zarr'):
        raise ValueError('only N5 and zarr containers are supported, got %s' % path)
    return File(path, mode)
