"""Array-level API over libctg.so: RAG + edge features of a label volume.

Inputs are numpy arrays (host memory, results come back as numpy) or torch
CUDA tensors (device memory, results stay resident as torch tensors).  This is
the layer that ``cluster_tools_amd.ndist`` (the ``nifty.distributed`` mirror)
calls after reading blocks from N5.
"""
from __future__ import annotations

import ctypes
import sys
import threading

import numpy as np

from . import _lib as L

N_FEATURES = L.CTG_N_FEATURES
NBINS = L.CTG_NBINS
WIDE_WORDS = L.CTG_WIDE_RECORD_WORDS
NSLOTS = NBINS + 2   # histogram slots of a wide record: left outliers, the bins, right outliers


def _is_torch(x):
    """x is a torch tensor -- without importing torch: a process that never
    imported it holds no tensors (a drop-in job process would otherwise pay
    torch's ~1.4 s import on its first library call)."""
    torch = sys.modules.get('torch')
    return torch is not None and isinstance(x, torch.Tensor)


def _ptr(x):
    if x is None:
        return None
    if _is_torch(x):
        return ctypes.c_void_p(x.data_ptr())
    return x.ctypes.data_as(ctypes.c_void_p)


def _shape_arr(vals):
    return (ctypes.c_int64 * 3)(*[int(v) for v in vals])


class Result:
    """Owning wrapper around a ``ctg_result*`` handle (device-resident)."""

    def __init__(self, handle, device):
        self.handle = handle
        self.device = device

    def __del__(self):
        self.free()

    def free(self):
        if getattr(self, 'handle', None) and L is not None:
            L.load().ctg_free(self.handle)
            self.handle = None

    @property
    def n_edges(self):
        return int(L.load().ctg_result_num_edges(self.handle))

    @property
    def n_nodes(self):
        return int(L.load().ctg_result_num_nodes(self.handle))

    def info(self):
        a, b = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.load().ctg_result_info(self.handle, ctypes.byref(a), ctypes.byref(b)), 'ctg_result_info')
        return int(a.value), int(b.value)

    # --- host copies
    def edges(self):
        out = np.empty((self.n_edges, 2), dtype=np.uint64)
        L.check(L.load().ctg_result_copy_edges(self.handle, _ptr(out), L.CTG_MEM_HOST), 'copy_edges')
        return out

    def nodes(self):
        out = np.empty(self.n_nodes, dtype=np.uint64)
        L.check(L.load().ctg_result_copy_nodes(self.handle, _ptr(out), L.CTG_MEM_HOST), 'copy_nodes')
        return out

    def features(self):
        out = np.empty((self.n_edges, N_FEATURES), dtype=np.float64)
        L.check(L.load().ctg_result_copy_features(self.handle, _ptr(out), L.CTG_MEM_HOST), 'copy_features')
        return out

    def stats(self):
        """(sums (E,2) float64, records (E,48) uint32) wide statistics."""
        s = np.empty((self.n_edges, 2), dtype=np.float64)
        r = np.empty((self.n_edges, WIDE_WORDS), dtype=np.uint32)
        L.check(L.load().ctg_result_copy_stats(self.handle, _ptr(s), _ptr(r), L.CTG_MEM_HOST), 'copy_stats')
        return s, r

    # --- device copies (torch)
    def _torch_copy(self, shape, dtype, fn):
        import torch
        t = torch.empty(shape, dtype=dtype, device='cuda:%d' % self.device)
        L.check(fn(self.handle, ctypes.c_void_p(t.data_ptr()), L.CTG_MEM_DEVICE), 'device copy')
        return t

    def edges_torch(self):
        import torch
        t = self._torch_copy((self.n_edges, 2), torch.int64, L.load().ctg_result_copy_edges)
        return t.view(torch.uint64) if hasattr(torch, 'uint64') else t

    def nodes_torch(self):
        import torch
        return self._torch_copy((self.n_nodes,), torch.int64, L.load().ctg_result_copy_nodes)

    def edges_torch_i64(self):
        """(E,2) int64 view of the uint64 edge table (labels < 2^63)."""
        import torch
        return self._torch_copy((self.n_edges, 2), torch.int64, L.load().ctg_result_copy_edges)

    def features_torch(self):
        import torch
        return self._torch_copy((self.n_edges, N_FEATURES), torch.float64, L.load().ctg_result_copy_features)

    def stats_torch(self):
        import torch
        s = torch.empty((self.n_edges, 2), dtype=torch.float64, device='cuda:%d' % self.device)
        r = torch.empty((self.n_edges, WIDE_WORDS), dtype=torch.int32, device='cuda:%d' % self.device)
        L.check(L.load().ctg_result_copy_stats(self.handle, ctypes.c_void_p(s.data_ptr()),
                                               ctypes.c_void_p(r.data_ptr()), L.CTG_MEM_DEVICE), 'copy_stats')
        return s, r


def _current_stream(tensor_input):
    if not tensor_input:
        return None
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check_offsets(offsets):
    off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int32).reshape(-1, 3))
    if off.shape[0] > L.CTG_MAX_CHANNELS:
        raise ValueError('at most %d affinity channels are supported' % L.CTG_MAX_CHANNELS)
    return off


def rag_features_handle(labels, data=None, offsets=None, own_begin=None, own_end=None, ignore_label=False,
                        hist_range=(0.0, 1.0), keep_stats=False, stream=None, no_adj_filter=False,
                        defer_stats=False):
    """Run the hot path and return the device-resident ``Result`` handle.

    labels: (Z,Y,X) uint64/uint32 numpy array or CUDA tensor (int64/int32 views
    of unsigned labels are accepted for torch); data: None, (Z,Y,X) boundary
    map or (C,Z,Y,X) affinities (float32 or uint8); offsets: C x 3 for
    affinities.  keep_stats keeps the mergeable wide records; no_adj_filter
    (affinities) keeps sampled pairs that are not edges of this array's RAG;
    defer_stats (with keep_stats, for the multi-GPU exchange only:
    CTG_DEFER_STATS) writes no statistics rows -- the exchange rebuilds the
    rows it needs from this call's records, valid until the next call.
    """
    lib = L.load()
    dev = L.init_device()
    on_dev = _is_torch(labels)
    if on_dev:
        import torch
        assert labels.is_cuda and labels.is_contiguous(), 'labels must be a contiguous CUDA tensor'
        label_bits = labels.element_size() * 8
        shape = tuple(labels.shape)
        if data is not None:
            assert _is_torch(data) and data.is_cuda and data.is_contiguous()
            kind = L.CTG_DATA_U8 if data.dtype == torch.uint8 else L.CTG_DATA_F32
            if kind == L.CTG_DATA_F32:
                assert data.dtype == torch.float32
    else:
        labels = np.asarray(labels)
        if labels.dtype not in (np.uint64, np.uint32, np.int64, np.int32):
            labels = labels.astype(np.uint64)
        labels = np.ascontiguousarray(labels)
        label_bits = labels.dtype.itemsize * 8
        shape = labels.shape
        if data is not None:
            data = np.asarray(data)
            if data.dtype == np.uint8:
                kind = L.CTG_DATA_U8
            else:
                kind = L.CTG_DATA_F32
                data = data.astype(np.float32, copy=False)
            data = np.ascontiguousarray(data)
    if len(shape) != 3:
        raise ValueError('labels must be 3-D, got shape %s' % (shape,))
    n_ch = 0
    off_ptr = None
    off = None
    if data is None:
        kind = L.CTG_DATA_NONE
    elif offsets is not None:
        off = _check_offsets(offsets)
        n_ch = off.shape[0]
        if tuple(data.shape) != (n_ch,) + tuple(shape):
            raise ValueError('affinities must be (C,Z,Y,X) = %s, got %s' % ((n_ch,) + tuple(shape),
                                                                           tuple(data.shape)))
        off_ptr = off.ctypes.data_as(ctypes.c_void_p)
    else:
        if tuple(data.shape) != tuple(shape):
            raise ValueError('boundary map shape %s != labels shape %s' % (tuple(data.shape), tuple(shape)))
    flags = ((L.CTG_KEEP_STATS if keep_stats else 0) | (L.CTG_NO_ADJ_FILTER if no_adj_filter else 0) |
             (L.CTG_DEFER_STATS if keep_stats and defer_stats else 0))
    sh = _shape_arr(shape)
    ob = _shape_arr(own_begin) if own_begin is not None else None
    oe = _shape_arr(own_end) if own_end is not None else None
    if stream is None:
        stream = _current_stream(on_dev)
    h = ctypes.c_void_p()
    rc = lib.ctg_rag_features(_ptr(labels), label_bits, _ptr(data), kind, n_ch, off_ptr, sh, ob, oe,
                              int(bool(ignore_label)), float(hist_range[0]), float(hist_range[1]),
                              flags, L.CTG_MEM_DEVICE if on_dev else L.CTG_MEM_HOST,
                              stream, ctypes.byref(h))
    L.check(rc, 'ctg_rag_features')
    return Result(h, dev)


def rag_features(labels, data=None, offsets=None, own_begin=None, own_end=None, ignore_label=False,
                 hist_range=(0.0, 1.0), keep_stats=False, no_adj_filter=False):
    """Host convenience: returns dict(edges, nodes, features[, sums, records])."""
    r = rag_features_handle(labels, data, offsets, own_begin, own_end, ignore_label, hist_range, keep_stats,
                            no_adj_filter=no_adj_filter)
    out = dict(edges=r.edges(), nodes=r.nodes())
    if data is not None:
        out['features'] = r.features()
        if keep_stats:
            out['sums'], out['records'] = r.stats()
    out['n_records'], out['n_direct'] = r.info()
    r.free()
    return out


_arena_pool = []
_arena_lock = threading.Lock()
ARENA_POOL_BYTES = 8 << 30


def _leak_arenas_at_exit():
    """Interpreter exit: drop the pooled page-locked arenas without unpinning
    them one by one (hipHostFree ~0.2 s per GB in a drop-in job process that
    is about to end; process teardown releases the pages).  CTG_EXIT_FREE=1
    keeps the explicit frees."""
    import os
    if os.environ.get('CTG_EXIT_FREE') == '1':
        return
    with _arena_lock:
        for a in _arena_pool:
            a.ptr = None
        _arena_pool.clear()


import atexit  # noqa: E402
atexit.register(_leak_arenas_at_exit)


def host_arena(nbytes):
    """A page-locked arena of at least ``nbytes`` from the process pool
    (pinning GBs of host memory costs ~0.2 s/GB: arenas are kept for the next
    batch / call); give it back with release_arena."""
    with _arena_lock:
        best = None
        for a in _arena_pool:
            if a.nbytes >= nbytes and (best is None or a.nbytes < best.nbytes):
                best = a
        if best is not None:
            _arena_pool.remove(best)
            return best
    return HostArena(nbytes)


def release_arena(arena):
    with _arena_lock:
        _arena_pool.append(arena)
        _arena_pool.sort(key=lambda a: -a.nbytes)
        while sum(a.nbytes for a in _arena_pool) > ARENA_POOL_BYTES and len(_arena_pool) > 1:
            _arena_pool.pop().free()


class HostArena:
    """Page-locked host buffer (ctg_host_alloc) viewed as a numpy array: the
    staging area of batched block inputs (decoded N5 ROIs go straight in)."""

    def __init__(self, nbytes):
        self.nbytes = int(max(nbytes, 64))
        lib = L.load()
        L.init_device()
        self.ptr = lib.ctg_host_alloc(self.nbytes)
        if not self.ptr:
            L.check(-3, 'ctg_host_alloc')
        self.buf = (ctypes.c_char * self.nbytes).from_address(self.ptr)

    def view(self, dtype, count, offset_bytes=0):
        return np.frombuffer(self.buf, dtype=dtype, count=int(count), offset=int(offset_bytes))

    def free(self):
        if getattr(self, 'ptr', None):
            L.load().ctg_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


def _desc(blocks):
    arr = (L.BlockDesc * len(blocks))()
    for d, b in zip(arr, blocks):
        d.label_offset = int(b['label_offset'])
        d.data_offset = int(b.get('data_offset', 0))
        for k in range(3):
            d.shape[k] = int(b['shape'][k])
            d.own_begin[k] = int(b['own'][0][k])
            d.own_end[k] = int(b['own'][1][k])
            d.graph_begin[k] = int(b['graph'][0][k])
            d.graph_end[k] = int(b['graph'][1][k])
    return arr


def rag_blocks_arena(labels, blocks, data=None, offsets=None, ignore_label=False, hist_range=(0.0, 1.0),
                     keep_stats=False, nodes=True):
    """ctg_rag_blocks over arenas that already hold the block arrays.

    labels: 1-D uint64/uint32 array (host, ideally a HostArena view);
    data: None or 1-D float32/uint8 array; blocks: list of dicts with
    label_offset, data_offset, shape, own=(begin, end), graph=(begin, end).
    Returns one dict per block: nodes, edges[, features, sums, records]."""
    lib = L.load()
    dev = L.init_device()
    on_dev = _is_torch(labels)
    if on_dev:   # device-resident arenas (torch CUDA tensors, int64/int32 views of the labels)
        import torch
        assert labels.is_cuda and labels.is_contiguous() and labels.element_size() in (4, 8)
        label_bits = labels.element_size() * 8
        n_lab = labels.numel()
        if data is not None:
            assert _is_torch(data) and data.is_cuda and data.is_contiguous()
            assert data.dtype in (torch.float32, torch.uint8)
    else:
        labels = np.asarray(labels)
        if labels.dtype not in (np.uint64, np.uint32):
            raise ValueError('labels arena must be uint64 or uint32')
        label_bits = labels.dtype.itemsize * 8
        n_lab = labels.size
    kind = L.CTG_DATA_NONE
    n_ch = 0
    off_ptr = None
    n_dat = 0
    if data is not None:
        if on_dev:
            import torch
            kind = L.CTG_DATA_U8 if data.dtype == torch.uint8 else L.CTG_DATA_F32
            n_dat = data.numel()
        else:
            data = np.asarray(data)
            kind = L.CTG_DATA_U8 if data.dtype == np.uint8 else L.CTG_DATA_F32
            if kind == L.CTG_DATA_F32 and data.dtype != np.float32:
                raise ValueError('data arena must be float32 or uint8')
            n_dat = data.size
        if offsets is not None:
            off = _check_offsets(offsets)
            n_ch = off.shape[0]
            off_ptr = off.ctypes.data_as(ctypes.c_void_p)
    desc = _desc(blocks)
    flags = (L.CTG_KEEP_STATS if keep_stats else 0) | (0 if nodes else L.CTG_NO_NODES)
    h = ctypes.c_void_p()
    rc = lib.ctg_rag_blocks(_ptr(labels), label_bits, _ptr(data), kind, n_ch, off_ptr,
                            ctypes.cast(desc, ctypes.c_void_p), len(blocks), n_lab, n_dat,
                            int(bool(ignore_label)), float(hist_range[0]), float(hist_range[1]), flags,
                            L.CTG_MEM_DEVICE if on_dev else L.CTG_MEM_HOST, _current_stream(on_dev),
                            ctypes.byref(h))
    L.check(rc, 'ctg_rag_blocks')
    r = Result(h, dev)
    nb = len(blocks)
    eoff = np.zeros(nb + 1, np.int64)
    noff = np.zeros(nb + 1, np.int64)
    L.check(lib.ctg_result_block_offsets(r.handle, _ptr(eoff), _ptr(noff)), 'ctg_result_block_offsets')
    edges, nodes = r.edges(), r.nodes()
    feats = r.features() if data is not None else None
    sums = recs = None
    if keep_stats and data is not None:
        sums, recs = r.stats()
    r.free()
    out = []
    for b in range(nb):
        e0, e1, n0, n1 = eoff[b], eoff[b + 1], noff[b], noff[b + 1]
        d = dict(edges=edges[e0:e1], nodes=nodes[n0:n1])
        if feats is not None:
            d['features'] = feats[e0:e1]
        if sums is not None:
            d['sums'], d['records'] = sums[e0:e1], recs[e0:e1]
        out.append(d)
    return out


def rag_blocks(arrays, own, graph, data=None, offsets=None, ignore_label=False, hist_range=(0.0, 1.0),
               keep_stats=False):
    """Convenience front end of rag_blocks_arena: per-block label arrays
    (and data arrays: (Z,Y,X) boundary maps or (C,Z,Y,X) affinities) with
    their own / graph boxes ((begin, end) in array coordinates)."""
    lab = [np.ascontiguousarray(np.asarray(a)) for a in arrays]
    dt = np.uint32 if all(a.dtype == np.uint32 for a in lab) else np.uint64
    lab_arena = np.concatenate([a.astype(dt, copy=False).ravel() for a in lab]) if lab else np.zeros(0, dt)
    blocks, lo, do = [], 0, 0
    dat_arena = None
    if data is not None:
        dd = [np.ascontiguousarray(np.asarray(x)) for x in data]
        ddt = np.uint8 if all(x.dtype == np.uint8 for x in dd) else np.float32
        dat_arena = np.concatenate([x.astype(ddt, copy=False).ravel() for x in dd])
    for i, a in enumerate(lab):
        blocks.append(dict(label_offset=lo, data_offset=do, shape=a.shape, own=own[i], graph=graph[i]))
        lo += a.size
        if data is not None:
            do += data[i].size
    return rag_blocks_arena(lab_arena, blocks, dat_arena, offsets, ignore_label, hist_range, keep_stats)


def unique_labels(labels, begin=None, end=None):
    """Sorted unique labels of labels[begin:end] (uint64 numpy array)."""
    lib = L.load()
    L.init_device()
    on_dev = _is_torch(labels)
    if not on_dev:
        labels = np.ascontiguousarray(np.asarray(labels).astype(np.uint64, copy=False))
    shape = tuple(labels.shape)
    h = ctypes.c_void_p()
    rc = lib.ctg_unique_labels(_ptr(labels), _shape_arr(shape),
                               _shape_arr(begin) if begin is not None else None,
                               _shape_arr(end) if end is not None else None,
                               L.CTG_MEM_DEVICE if on_dev else L.CTG_MEM_HOST,
                               _current_stream(on_dev), ctypes.byref(h))
    L.check(rc, 'ctg_unique_labels')
    r = Result(h, L.init_device())
    nodes = r.nodes()
    r.free()
    return nodes


def merge_stats_handle(keys, sums, records, hist_range=(0.0, 1.0), keep_stats=False, stream=None):
    """Device-resident merge of partial statistics: keys (n,2), sums (n,2)
    float64, records (n,48) 32-bit words; numpy (host) or CUDA tensors."""
    lib = L.load()
    dev = L.init_device()
    on_dev = _is_torch(keys)
    if on_dev:
        for t in (keys, sums, records):
            assert _is_torch(t) and t.is_cuda and t.is_contiguous(), 'merge inputs must be contiguous CUDA tensors'
        n = keys.shape[0]
        assert keys.element_size() == 8 and keys.numel() == 2 * n
        assert sums.element_size() == 8 and sums.numel() == 2 * n
        assert records.element_size() == 4 and records.numel() == WIDE_WORDS * n
    else:
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1, 2))
        sums = np.ascontiguousarray(np.asarray(sums, dtype=np.float64).reshape(-1, 2))
        records = np.ascontiguousarray(np.asarray(records, dtype=np.uint32).reshape(-1, WIDE_WORDS))
        n = keys.shape[0]
        assert sums.shape[0] == n and records.shape[0] == n
    if stream is None:
        stream = _current_stream(on_dev)
    h = ctypes.c_void_p()
    rc = lib.ctg_merge_stats(_ptr(keys), _ptr(sums), _ptr(records), n, float(hist_range[0]),
                             float(hist_range[1]), int(bool(keep_stats)),
                             L.CTG_MEM_DEVICE if on_dev else L.CTG_MEM_HOST, stream, ctypes.byref(h))
    L.check(rc, 'ctg_merge_stats')
    return Result(h, dev)


def unique_values_handle(values, stream=None):
    """Sorted unique values of a uint64 list (numpy or CUDA int64 tensor) -> Result (nodes)."""
    lib = L.load()
    dev = L.init_device()
    on_dev = _is_torch(values)
    if not on_dev:
        values = np.ascontiguousarray(np.asarray(values, dtype=np.uint64).reshape(-1))
    else:
        assert values.is_cuda and values.is_contiguous() and values.element_size() == 8
    if stream is None:
        stream = _current_stream(on_dev)
    h = ctypes.c_void_p()
    L.check(lib.ctg_unique_values(_ptr(values), int(values.shape[0]),
                                  L.CTG_MEM_DEVICE if on_dev else L.CTG_MEM_HOST, stream, ctypes.byref(h)),
            'ctg_unique_values')
    return Result(h, dev)


def merge_stats(keys, sums, records, hist_range=(0.0, 1.0), keep_stats=False):
    """Combine partial statistics tables (wide records) -> dict(edges, features[, sums, records])."""
    r = merge_stats_handle(keys, sums, records, hist_range, keep_stats)
    out = dict(edges=r.edges(), features=r.features())
    if keep_stats:
        out['sums'], out['records'] = r.stats()
    r.free()
    return out


def merge_feature_rows(ids, rows, id_begin, id_end):
    """Reference-layout (n,10) feature rows of global edge ids -> the merged
    (id_end - id_begin, 10) rows (ctg_merge_feature_rows)."""
    lib = L.load()
    L.init_device()
    ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64).reshape(-1))
    rows = np.ascontiguousarray(np.asarray(rows, dtype=np.float64).reshape(-1, N_FEATURES))
    if rows.shape[0] != ids.shape[0]:
        raise ValueError('ids and rows differ in length')
    out = np.zeros((int(id_end) - int(id_begin), N_FEATURES), dtype=np.float64)
    L.check(lib.ctg_merge_feature_rows(_ptr(ids), _ptr(rows), ids.shape[0], int(id_begin), int(id_end), _ptr(out),
                                       L.CTG_MEM_HOST, None), 'ctg_merge_feature_rows')
    return out


def unique_pairs(pairs):
    """Sorted unique rows of an (n,2) uint64 pair list -> (edges, nodes)."""
    lib = L.load()
    dev = L.init_device()
    p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint64).reshape(-1, 2))
    h = ctypes.c_void_p()
    L.check(lib.ctg_unique_pairs(_ptr(p), p.shape[0], L.CTG_MEM_HOST, None, ctypes.byref(h)), 'ctg_unique_pairs')
    r = Result(h, dev)
    out = r.edges(), r.nodes()
    r.free()
    return out


def map_edge_ids(global_edges, query):
    """Row of every query (u,v) in the sorted global edge table (-1 if absent)."""
    lib = L.load()
    L.init_device()
    g = np.ascontiguousarray(np.asarray(global_edges, dtype=np.uint64).reshape(-1, 2))
    q = np.ascontiguousarray(np.asarray(query, dtype=np.uint64).reshape(-1, 2))
    out = np.empty(q.shape[0], dtype=np.int64)
    rc = lib.ctg_map_edge_ids(_ptr(g), g.shape[0], _ptr(q), q.shape[0], _ptr(out), L.CTG_MEM_HOST, None)
    L.check(rc, 'ctg_map_edge_ids')
    return out


def synth_volume(shape, cell=10, seed=0, z_offset=0, global_shape=None, label_offset=0, noise_amp=0.1,
                 with_boundary=True, device=None):
    """Generate the synthetic volume directly in HBM (torch tensors)."""
    import torch
    lib = L.load()
    dev = L.init_device(device)
    labels = torch.empty(tuple(shape), dtype=torch.int64, device='cuda:%d' % dev)
    bnd = torch.empty(tuple(shape), dtype=torch.float32, device='cuda:%d' % dev) if with_boundary else None
    gs = _shape_arr(global_shape) if global_shape is not None else None
    rc = lib.ctg_synth_volume(_ptr(labels), _ptr(bnd), _shape_arr(shape), int(z_offset), gs, int(cell),
                              int(seed), int(label_offset), float(noise_amp),
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    L.check(rc, 'ctg_synth_volume')
    return labels, bnd


def synth_affinities(boundary, offsets):
    import torch
    lib = L.load()
    off = _check_offsets(offsets)
    shape = tuple(boundary.shape)
    affs = torch.empty((off.shape[0],) + shape, dtype=torch.float32, device=boundary.device)
    rc = lib.ctg_synth_affinities(_ptr(boundary), _ptr(affs), _shape_arr(shape), off.shape[0],
                                  off.ctypes.data_as(ctypes.c_void_p),
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    L.check(rc, 'ctg_synth_affinities')
    return affs


def trim_cache():
    """Return the library's cached device memory (workspace + pool) to HIP."""
    L.init_device()
    L.check(L.load().ctg_trim(), 'ctg_trim')


def set_profiling(on=True):
    L.check(L.load().ctg_set_profiling(int(bool(on))), 'ctg_set_profiling')


def last_timings():
    """Device ms of the last rag call: scan, pack, sort, segment, reduce, nodes, total, and narrow (the
    uint64 -> u32 label pass of long-range affinity calls, before the scan; 0 when it did not run)."""
    buf = (ctypes.c_double * 8)()
    L.check(L.load().ctg_last_timings(buf, 8), 'ctg_last_timings')
    return dict(zip(['scan', 'pack', 'sort', 'segment', 'reduce', 'nodes', 'total', 'narrow'], list(buf)))
