"""CPU oracle for the RAG + edge-feature hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``cluster_tools_amd``) never calls it.

This is a numpy restatement of the semantics that the reference's hot path
obtains from ``nifty.distributed`` (C++, not vendored under /root/reference;
pinned as ``nifty >=v1.0.7`` in ``conda-recipe/meta.yaml:30``).  Because the
library itself is absent, the restatement follows the reference's call sites
and the assertions of its own tests:

* per-block sub-graphs      -- graph/initial_sub_graphs.py:116-131 (call),
                               test/graph/test_graph.py:42-84 (semantics)
* merged global graph       -- graph/merge_sub_graphs.py:127-137,
                               test/graph/test_graph.py:95-115
* per-block edge ids        -- graph/map_edge_ids.py:101-120,
                               test/graph/test_graph.py:86-93
* boundary/affinity features -- features/block_edge_features.py:113-148,
                               test/features/test_edge_features.py:32-77,97,126
* feature merge             -- features/merge_edge_features.py:110-149

Parity status (see DESIGN.md "Oracle"): the graph is pinned by the reference
tests' assertions plus hand-computed known-answer tests (tests/golden).  The
10 feature columns are pinned only partially: count/mean/variance follow the
reference test's assertions; quantiles follow vigra's
``StandardQuantiles<UserRangeHistogram<40>>`` algorithm restated in
``vigra_quantiles`` (parity unpinned: no fixture from the reference exists).
"""
from __future__ import annotations

import numpy as np

NBINS = 40
QUANTILES = (0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0)
N_FEATURES = 10  # mean, var, q0(min), q10, q25, q50, q75, q90, q100(max), count


# ----------------------------------------------------------------------------
# faces
# ----------------------------------------------------------------------------

def _own_end(shape, own_end):
    return tuple(shape) if own_end is None else tuple(min(int(e), int(s)) for e, s in zip(own_end, shape))


def _face_slices(shape, axis, own_begin, own_end=None):
    """Slices (lower, upper) selecting every face (p, p+e_axis) whose upper
    voxel q = p + e_axis lies in the owned box [own_begin, own_end).

    own_begin = (0,0,0) selects every face of the array (whole-volume RAG as in
    nifty.graph.rag.gridRag, test_graph.py:79,108).  A 1-voxel own_begin on an
    axis is the "increaseRoi" halo geometry of initial_sub_graphs.py:124-129;
    own_end < shape is a block inside a larger (halo) array
    (block_edge_features.py:189-211 geometry twin).
    """
    end = _own_end(shape, own_end)
    up, lo = [], []
    for ax in range(3):
        b = own_begin[ax]
        e = max(end[ax], b)
        if ax == axis:
            b = max(b, 1)
            e = max(e, b)
            up.append(slice(b, e))
            lo.append(slice(b - 1, e - 1))
        else:
            up.append(slice(b, e))
            lo.append(slice(b, e))
    return tuple(lo), tuple(up)


def _pairs_view(u, v):
    uv = np.empty((u.size, 2), dtype=np.uint64)
    uv[:, 0] = u
    uv[:, 1] = v
    return uv


def _unique_pairs(uv, return_inverse=False):
    """Lexicographically sorted unique rows of an (n,2) uint64 array."""
    if uv.shape[0] == 0:
        out = np.zeros((0, 2), dtype=np.uint64)
        return (out, np.zeros(0, dtype=np.int64)) if return_inverse else out
    order = np.lexsort((uv[:, 1], uv[:, 0]))
    s = uv[order]
    head = np.ones(s.shape[0], dtype=bool)
    head[1:] = (s[1:, 0] != s[:-1, 0]) | (s[1:, 1] != s[:-1, 1])
    uniq = s[head]
    if not return_inverse:
        return uniq
    seg = np.cumsum(head) - 1
    inv = np.empty(uv.shape[0], dtype=np.int64)
    inv[order] = seg
    return uniq, inv


def face_keys(labels, own_begin=(0, 0, 0), ignore_label=False, own_end=None):
    """All boundary faces as canonical (u<v) keys, per axis.

    Returns list of (key_uv (n,2), lower_index_slices, upper_index_slices, mask).
    """
    labels = np.asarray(labels)
    assert labels.ndim == 3
    out = []
    for axis in range(3):
        lo, up = _face_slices(labels.shape, axis, own_begin, own_end)
        a = labels[lo]
        b = labels[up]
        mask = a != b
        if ignore_label:
            mask &= (a != 0) & (b != 0)
        u = np.minimum(a[mask], b[mask]).astype(np.uint64)
        v = np.maximum(a[mask], b[mask]).astype(np.uint64)
        out.append((_pairs_view(u, v), lo, up, mask))
    return out


# ----------------------------------------------------------------------------
# graph
# ----------------------------------------------------------------------------

def rag_edges(labels, own_begin=(0, 0, 0), ignore_label=False, own_end=None):
    """Sorted unique (u<v) label pairs over forward faces.

    Equals ``nrag.gridRag(seg).uvIds()`` (test_graph.py:79-84, 108-115) for
    own_begin = 0 and ignore_label False.  With ``ignore_label`` every edge that
    contains label 0 is dropped (initial_sub_graphs.py:38-43,147 config key).
    """
    parts = [k for k, _, _, _ in face_keys(labels, own_begin, ignore_label, own_end)]
    uv = np.concatenate(parts, axis=0) if parts else np.zeros((0, 2), np.uint64)
    return _unique_pairs(uv)


def unique_labels(labels):
    return np.unique(np.asarray(labels).astype(np.uint64, copy=False))


def block_subgraph(labels, block_begin, block_end, ignore_label=False):
    """Per-block output of ndist.computeMergeableRegionGraph(increaseRoi=True).

    nodes = unique labels of the INNER block  (test_graph.py:53-60)
    edges = RAG of seg[max(begin-1,0):end]   (test_graph.py:42-51,70-84)
    """
    roi_begin = [max(b - 1, 0) for b in block_begin]
    inner = tuple(slice(b, e) for b, e in zip(block_begin, block_end))
    outer = tuple(slice(b, e) for b, e in zip(roi_begin, block_end))
    nodes = unique_labels(labels[inner])
    edges = rag_edges(labels[outer], (0, 0, 0), ignore_label)
    return nodes, edges


def blocking_blocks(shape, block_shape):
    """nifty.tools.blocking([0,0,0], shape, block_shape) in C order (block id ->
    (begin, end)); block ids enumerate the grid with the last axis fastest."""
    grid = [(s + b - 1) // b for s, b in zip(shape, block_shape)]
    blocks = []
    for gz in range(grid[0]):
        for gy in range(grid[1]):
            for gx in range(grid[2]):
                pos = (gz, gy, gx)
                begin = tuple(p * b for p, b in zip(pos, block_shape))
                end = tuple(min(bg + b, s) for bg, b, s in zip(begin, block_shape, shape))
                blocks.append((pos, begin, end))
    return blocks


def merge_subgraphs(sub_nodes, sub_edges):
    """ndist.mergeSubgraphs: sorted union (merge_sub_graphs.py:127-137)."""
    nodes = np.unique(np.concatenate([n for n in sub_nodes if n is not None] or
                                     [np.zeros(0, np.uint64)]).astype(np.uint64))
    es = [e for e in sub_edges if e is not None and len(e)]
    edges = _unique_pairs(np.concatenate(es, axis=0)) if es else np.zeros((0, 2), np.uint64)
    return nodes, edges


def find_edges(global_edges, uv):
    """ndist.Graph.findEdges (test_graph.py:92): row index of every uv in the
    sorted global edge table, -1 if absent."""
    ge = np.asarray(global_edges, dtype=np.uint64)
    uv = np.asarray(uv, dtype=np.uint64).reshape(-1, 2)
    if ge.shape[0] == 0:
        return np.full(uv.shape[0], -1, dtype=np.int64)
    # lexicographic search: search on u then on v within the u-run
    lo = np.searchsorted(ge[:, 0], uv[:, 0], side='left')
    hi = np.searchsorted(ge[:, 0], uv[:, 0], side='right')
    out = np.full(uv.shape[0], -1, dtype=np.int64)
    for i in range(uv.shape[0]):
        j = lo[i] + np.searchsorted(ge[lo[i]:hi[i], 1], uv[i, 1])
        if j < hi[i] and ge[j, 1] == uv[i, 1]:
            out[i] = j
    return out


# ----------------------------------------------------------------------------
# vigra histogram + quantiles
# ----------------------------------------------------------------------------

def histogram_slots(values, lo, hi, nbins=NBINS):
    """vigra RangeHistogramBase::update binning (UserRangeHistogram).

    m = scale * (x - offset), scale = nbins/(hi-lo), offset = lo, in double;
    index = (m == nbins) ? nbins-1 : (int)m   -- C truncation toward zero;
    index < 0 -> left outlier, index >= nbins -> right outlier.
    Returns slot in [0, nbins+2): 0 = left outliers, 1+k = bin k,
    nbins+1 = right outliers.
    """
    x = np.asarray(values, dtype=np.float64)
    scale = float(nbins) / (float(hi) - float(lo))
    m = scale * (x - float(lo))
    idx = np.trunc(m)
    idx = np.where(m == float(nbins), float(nbins - 1), idx)
    slot = np.empty(x.shape, dtype=np.int64)
    left = idx < 0
    right = idx >= nbins
    mid = ~(left | right)
    slot[left] = 0
    slot[right] = nbins + 1
    slot[mid] = idx[mid].astype(np.int64) + 1
    return slot


def vigra_quantiles(hist_slots, vmin, vmax, count, lo, hi,
                    quantiles=QUANTILES, nbins=NBINS):
    """RangeHistogramBase::computeStandardQuantiles restated.

    hist_slots: length nbins+2 (left outliers, bins..., right outliers).
    Keypoints live in mapped (bin) space and are mapped back with
    x = t / scale + offset.
    """
    res = np.zeros(len(quantiles), dtype=np.float64)
    if count == 0:
        return res
    scale = float(nbins) / (float(hi) - float(lo))
    offset = float(lo)

    def mapf(t):
        return scale * (t - offset)

    left = float(hist_slots[0])
    right = float(hist_slots[nbins + 1])
    h = hist_slots[1:nbins + 1]
    keypoints = [mapf(float(vmin))]
    cumhist = [0.0]
    if left > 0.0:
        keypoints.append(0.0)
        cumhist.append(left)
    cumulative = left
    for k in range(nbins):
        if h[k] > 0:
            if keypoints[-1] <= k:
                keypoints.append(float(k))
                cumhist.append(cumulative)
            cumulative += float(h[k])
            keypoints.append(float(k + 1))
            cumhist.append(cumulative)
    if right > 0.0:
        if keypoints[-1] != nbins:
            keypoints.append(float(nbins))
            cumhist.append(cumulative)
        keypoints.append(mapf(float(vmax)))
        cumhist.append(float(count))
    else:
        keypoints[-1] = mapf(float(vmax))
        cumhist[-1] = float(count)

    q = 0
    end = len(quantiles)
    if quantiles[0] == 0.0:
        res[0] = float(vmin)
        q += 1
    if quantiles[end - 1] == 1.0:
        res[end - 1] = float(vmax)
        end -= 1
    point = 0
    if q < end:
        qcount = float(count) * quantiles[q]
    while q < end:
        if cumhist[point] < qcount and cumhist[point + 1] >= qcount:
            t = (qcount - cumhist[point]) / (cumhist[point + 1] - cumhist[point]) * \
                (keypoints[point + 1] - keypoints[point])
            res[q] = (1.0 / scale) * (t + keypoints[point]) + offset  # mapItemInverse
            q += 1
            if q < len(quantiles):
                qcount = float(count) * quantiles[q]
        else:
            point += 1
    return res


# ----------------------------------------------------------------------------
# features
# ----------------------------------------------------------------------------

def _accumulate(inv, values, n_edges, lo, hi, nbins=NBINS):
    """Per-edge statistics of samples (inv = edge row of each sample)."""
    values = np.asarray(values, dtype=np.float32).astype(np.float64)
    count = np.bincount(inv, minlength=n_edges).astype(np.int64)
    ssum = np.bincount(inv, weights=values, minlength=n_edges)
    with np.errstate(invalid='ignore', divide='ignore'):
        mean = np.where(count > 0, ssum / np.maximum(count, 1), 0.0)
    dev = values - mean[inv]
    m2 = np.bincount(inv, weights=dev * dev, minlength=n_edges)
    var = np.where(count > 0, m2 / np.maximum(count, 1), 0.0)
    vmin = np.full(n_edges, np.inf)
    vmax = np.full(n_edges, -np.inf)
    np.minimum.at(vmin, inv, values)
    np.maximum.at(vmax, inv, values)
    vmin[count == 0] = 0.0
    vmax[count == 0] = 0.0
    slots = histogram_slots(values, lo, hi, nbins)
    hist = np.bincount(inv * (nbins + 2) + slots,
                       minlength=n_edges * (nbins + 2)).reshape(n_edges, nbins + 2)
    return dict(count=count, sum=ssum, mean=mean, var=var, m2=m2,
                min=vmin, max=vmax, hist=hist)


def finalize_features(stats, lo, hi, nbins=NBINS):
    """(E,10) float64: mean, var, q0..q100 (q0=min, q100=max), count.

    Column contract: test_edge_features.py:58-59,71-77; probs_to_costs.py:205-207.
    """
    n = stats['count'].shape[0]
    out = np.zeros((n, N_FEATURES), dtype=np.float64)
    for e in range(n):
        c = int(stats['count'][e])
        if c == 0:
            continue
        q = vigra_quantiles(stats['hist'][e], stats['min'][e], stats['max'][e], c,
                            lo, hi, QUANTILES, nbins)
        out[e, 0] = stats['mean'][e]
        out[e, 1] = stats['var'][e]
        out[e, 2:9] = q
        out[e, 9] = c
    return out


def as_samples(data):
    """uint8 maps are sampled as value/255 in float32 (SURVEY OPEN-7 default)."""
    data = np.asarray(data)
    if data.dtype == np.uint8:
        return data.astype(np.float32) / np.float32(255.0)
    return data.astype(np.float32, copy=False)


def boundary_features(labels, data, own_begin=(0, 0, 0), ignore_label=False,
                      lo=0.0, hi=1.0, nbins=NBINS, return_stats=False, own_end=None):
    """RAG + boundary-map edge features, whole-volume semantics.

    Every boundary face (p, q=p+e_a) whose upper voxel lies in the owned box
    contributes BOTH voxel values D[p] and D[q] as samples (SURVEY OPEN-1,
    'both'; consistent with the count assertion of test_edge_features.py:52
    against nrag.accumulateEdgeMeanAndLength).
    Returns (edges (E,2) uint64, features (E,10) float64).
    """
    labels = np.asarray(labels)
    data = as_samples(data)
    assert data.shape == labels.shape
    keys, vals = [], []
    for uv, lo_sl, up_sl, mask in face_keys(labels, own_begin, ignore_label, own_end):
        a = data[lo_sl][mask]
        b = data[up_sl][mask]
        keys.append(uv)
        keys.append(uv)
        vals.append(a)
        vals.append(b)
    uv = np.concatenate(keys, axis=0)
    v = np.concatenate(vals).astype(np.float32)
    edges, inv = _unique_pairs(uv, return_inverse=True)
    stats = _accumulate(inv, v, edges.shape[0], lo, hi, nbins)
    feats = finalize_features(stats, lo, hi, nbins)
    if return_stats:
        return edges, feats, stats
    return edges, feats


def affinity_features(labels, affs, offsets, own_begin=(0, 0, 0), ignore_label=False,
                      lo=0.0, hi=1.0, nbins=NBINS, return_stats=False, own_end=None, edge_list=None):
    """RAG + affinity-map edge features.

    affs is channel-first (C,Z,Y,X) (block_edge_features.py:136,215).  For
    channel c with offset o_c and voxel p in the owned box, q = p + o_c inside
    the array: if L[p] != L[q] and (min,max) is an edge of the RAG (faces with
    upper voxel in the owned box), sample affs[c, p].  Pairs that are not RAG
    edges (long-range, non-adjacent) are skipped.  With ``edge_list`` (a
    block's sub-graph edges, the ndist per-block call) the output rows are
    that list and it is the adjacency filter.
    """
    labels = np.asarray(labels)
    affs = as_samples(affs)
    assert affs.ndim == 4 and affs.shape[1:] == labels.shape
    assert affs.shape[0] == len(offsets)
    if edge_list is None:
        edges = rag_edges(labels, own_begin, ignore_label, own_end)
    else:
        edges = _unique_pairs(np.asarray(edge_list, dtype=np.uint64).reshape(-1, 2))
    shape = labels.shape
    end = _own_end(shape, own_end)
    keys, vals = [], []
    for c, off in enumerate(offsets):
        psl, qsl = [], []
        for ax in range(3):
            o = int(off[ax])
            b = own_begin[ax]
            p0 = max(b, -o)
            p1 = min(end[ax], shape[ax] - o)
            if p1 <= p0:
                p0 = p1 = 0
            psl.append(slice(p0, p1))
            qsl.append(slice(p0 + o, p1 + o))
        lp = labels[tuple(psl)]
        lq = labels[tuple(qsl)]
        mask = lp != lq
        if ignore_label:
            mask &= (lp != 0) & (lq != 0)
        u = np.minimum(lp[mask], lq[mask]).astype(np.uint64)
        v = np.maximum(lp[mask], lq[mask]).astype(np.uint64)
        keys.append(_pairs_view(u, v))
        vals.append(affs[c][tuple(psl)][mask])
    uv = np.concatenate(keys, axis=0) if keys else np.zeros((0, 2), np.uint64)
    val = np.concatenate(vals).astype(np.float32) if vals else np.zeros(0, np.float32)
    idx = find_edges_fast(edges, uv)
    keep = idx >= 0
    stats = _accumulate(idx[keep], val[keep], edges.shape[0], lo, hi, nbins)
    feats = finalize_features(stats, lo, hi, nbins)
    if return_stats:
        return edges, feats, stats
    return edges, feats


def find_edges_fast(global_edges, uv):
    """Vectorised findEdges via a combined sort key (labels < 2**32 only,
    falls back to ``find_edges`` otherwise)."""
    ge = np.asarray(global_edges, dtype=np.uint64)
    uv = np.asarray(uv, dtype=np.uint64).reshape(-1, 2)
    if uv.shape[0] == 0:
        return np.zeros(0, dtype=np.int64)
    if ge.shape[0] == 0:
        return np.full(uv.shape[0], -1, dtype=np.int64)
    mx = max(int(ge.max()), int(uv.max()))
    if mx >= 2 ** 32:
        return find_edges(ge, uv)
    gk = (ge[:, 0] << np.uint64(32)) | ge[:, 1]
    qk = (uv[:, 0] << np.uint64(32)) | uv[:, 1]
    pos = np.searchsorted(gk, qk)
    pos_c = np.minimum(pos, gk.size - 1)
    hit = gk[pos_c] == qk
    return np.where(hit, pos_c, -1).astype(np.int64)


def merge_feature_stats(parts, n_edges, lo=0.0, hi=1.0, nbins=NBINS):
    """Exact cross-block / cross-GPU combine of partial statistics.

    parts: iterable of (edge_ids, stats) with stats as returned by
    ``_accumulate`` restricted to those edges.  count adds, mean is
    count-weighted, M2 combines by Chan's formula, min/max elementwise over
    non-empty partials, histograms add (OPEN-3 default).
    """
    count = np.zeros(n_edges, np.int64)
    ssum = np.zeros(n_edges)
    vmin = np.full(n_edges, np.inf)
    vmax = np.full(n_edges, -np.inf)
    hist = np.zeros((n_edges, nbins + 2), np.int64)
    for ids, st in parts:
        ids = np.asarray(ids, dtype=np.int64)
        ne = st['count'] > 0
        np.add.at(count, ids, st['count'])
        np.add.at(ssum, ids, st['sum'])
        np.minimum.at(vmin, ids[ne], st['min'][ne])
        np.maximum.at(vmax, ids[ne], st['max'][ne])
        np.add.at(hist, ids, st['hist'])
    with np.errstate(invalid='ignore', divide='ignore'):
        mean = np.where(count > 0, ssum / np.maximum(count, 1), 0.0)
    m2 = np.zeros(n_edges)
    for ids, st in parts:
        ids = np.asarray(ids, dtype=np.int64)
        d = st['mean'] - mean[ids]
        np.add.at(m2, ids, st['m2'] + st['count'] * d * d)
    var = np.where(count > 0, m2 / np.maximum(count, 1), 0.0)
    vmin[count == 0] = 0.0
    vmax[count == 0] = 0.0
    return dict(count=count, sum=ssum, mean=mean, var=var, m2=m2, min=vmin,
                max=vmax, hist=hist)
