"""ctypes wrapper of oracle/libctg_oracle.so (scalar C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def load():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, 'libctg_oracle.so')
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(['make', '-C', _HERE, '-s'])
        lib = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        lib.ctgo_features.restype = ctypes.c_int
        lib.ctgo_features.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_int64, vp, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(vp), ctypes.POINTER(vp)]
        lib.ctgo_free.argtypes = [vp]
        lib.ctgo_free.restype = None
        _lib = lib
    return _lib


def features(labels, data=None, offsets=None, own_begin=None, ignore_label=False, lo=0.0, hi=1.0):
    """Returns (edges (E,2) uint64, features (E,10) float64)."""
    lib = load()
    labels = np.ascontiguousarray(labels, dtype=np.uint64)
    Z, Y, X = labels.shape
    mode = 0
    dptr = None
    optr = None
    n_ch = 0
    off = None
    if data is not None:
        if data.dtype == np.uint8:
            data = data.astype(np.float32) / np.float32(255)
        data = np.ascontiguousarray(data, dtype=np.float32)
        dptr = data.ctypes.data_as(ctypes.c_void_p)
        if offsets is not None:
            mode = 2
            off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int32).reshape(-1, 3))
            n_ch = off.shape[0]
            optr = off.ctypes.data_as(ctypes.c_void_p)
        else:
            mode = 1
    own = (ctypes.c_int64 * 3)(*own_begin) if own_begin is not None else None
    n = ctypes.c_int64()
    ep = ctypes.c_void_p()
    fp = ctypes.c_void_p()
    rc = lib.ctgo_features(labels.ctypes.data_as(ctypes.c_void_p), dptr, mode, n_ch, optr, Z, Y, X, own,
                           int(bool(ignore_label)), float(lo), float(hi), ctypes.byref(n), ctypes.byref(ep),
                           ctypes.byref(fp))
    if rc != 0:
        raise MemoryError('ctgo_features failed')
    E = n.value
    edges = np.ctypeslib.as_array(ctypes.cast(ep, ctypes.POINTER(ctypes.c_uint64)), shape=(max(E, 1) * 2,))
    edges = edges[:2 * E].reshape(E, 2).copy()
    feats = np.ctypeslib.as_array(ctypes.cast(fp, ctypes.POINTER(ctypes.c_double)), shape=(max(E, 1) * 10,))
    feats = feats[:10 * E].reshape(E, 10).copy()
    lib.ctgo_free(ep)
    lib.ctgo_free(fp)
    return edges, feats


def chunk_job(args):
    """One z-chunk of a slab stored as .npy files (bench.py's CPU baseline):
    (labels_path, data_path, z0, z1, halo) -> (n_edges, seconds of the C call).
    The chunk is read from the memory-mapped files before the clock starts."""
    import time
    lp, dp, z0, z1, halo = args
    lab = np.ascontiguousarray(np.load(lp, mmap_mode='r')[z0 - halo:z1])
    dat = np.ascontiguousarray(np.load(dp, mmap_mode='r')[z0 - halo:z1])
    load()
    t0 = time.perf_counter()
    e, _ = features(lab, dat, own_begin=(halo, 0, 0))
    return int(e.shape[0]), time.perf_counter() - t0


def block_job(args):
    """configs[0] CPU baseline (bench.py): the per-block job bodies of the
    reference's local target on the scalar C restatement, with the same gzip
    N5 I/O -- for every block of the job: read the labels and boundary ROIs
    (block + lower halo, increaseRoi, initial_sub_graphs.py:124-129 /
    block_edge_features.py:127-134) from the N5 input, compute the RAG and the
    10 features of the block's owned faces, write the block's varlength
    ``nodes`` / ``edges`` / ``sub_features`` chunks (gzip).  One
    single-threaded job per worker process, as LocalTask runs it
    (cluster_tasks.py:528-550).  args = (input path, output path, block shape,
    block ids) -> (n_edges, seconds of the job body)."""
    import time
    import numpy as np
    from cluster_tools_amd import n5
    from cluster_tools_amd.blocking import blocking
    inp, out, block_shape, block_ids = args
    load()
    t0 = time.perf_counter()
    n_edges = 0
    with n5.File(inp, 'r') as f, n5.File(out) as fo:
        ds_l, ds_d = f['seg'], f['bnd']
        shape = list(ds_l.shape)
        blk = blocking([0, 0, 0], shape, list(block_shape))
        g_nodes, g_edges, g_feat = fo['s0/sub_graphs/nodes'], fo['s0/sub_graphs/edges'], fo['s0/sub_features']
        for b in block_ids:
            bb = blk.getBlock(b)
            rb = [max(x - 1, 0) for x in bb.begin]
            sl = tuple(slice(x, y) for x, y in zip(rb, bb.end))
            lab = np.ascontiguousarray(ds_l[sl], dtype=np.uint64)
            dat = np.ascontiguousarray(ds_d[sl], dtype=np.float32)
            own = tuple(x - r for x, r in zip(bb.begin, rb))
            e, ft = features(lab, dat, own_begin=own)
            inner = lab[tuple(slice(o, None) for o in own)]
            pos = blk.blockGridPosition(b)
            g_nodes.write_chunk(pos, np.unique(inner), True)
            if e.shape[0]:
                g_edges.write_chunk(pos, e.ravel(), True)
                g_feat.write_chunk(pos, ft.ravel(), True)
            n_edges += e.shape[0]
    return n_edges, time.perf_counter() - t0
