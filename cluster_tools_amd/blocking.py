"""Mirror of ``nifty.tools.blocking`` (the regular block grid the hot-path
tasks use: initial_sub_graphs.py:150-152, merge_edge_features.py:134,
utils/volume_utils.py:42-57, test/graph/test_graph.py:35-53).

Block ids enumerate the grid in C order (last axis fastest); the N5 chunk of
block b is ``begin // block_shape`` (multicut/solve_subproblems.py:203-204).
"""
from __future__ import annotations

import itertools

import numpy as np


class Block:
    def __init__(self, begin, end):
        self.begin = [int(b) for b in begin]
        self.end = [int(e) for e in end]

    @property
    def shape(self):
        return [e - b for b, e in zip(self.begin, self.end)]

    def __repr__(self):
        return 'Block(begin=%s, end=%s)' % (self.begin, self.end)


class BlockWithHalo:
    def __init__(self, outer, inner, inner_local):
        self.outerBlock = outer
        self.innerBlock = inner
        self.innerBlockLocal = inner_local


class blocking:  # noqa: N801  (nifty's spelling)
    def __init__(self, roiBegin, roiEnd, blockShape):  # noqa: N803
        self.roiBegin = [int(b) for b in roiBegin]
        self.roiEnd = [int(e) for e in roiEnd]
        self.blockShape = [int(s) for s in blockShape]
        self.blocksPerAxis = [max(0, (e - b + s - 1) // s) for b, e, s in
                              zip(self.roiBegin, self.roiEnd, self.blockShape)]
        self.numberOfBlocks = int(np.prod(self.blocksPerAxis)) if self.blocksPerAxis else 0
        strides = [1] * len(self.blocksPerAxis)
        for ax in range(len(strides) - 2, -1, -1):
            strides[ax] = strides[ax + 1] * self.blocksPerAxis[ax + 1]
        self._strides = strides

    def blockGridPosition(self, block_id):  # noqa: N802
        pos = []
        for s in self._strides:
            pos.append(block_id // s)
            block_id %= s
        return pos

    def gridPositionToBlockId(self, pos):  # noqa: N802
        return int(sum(p * s for p, s in zip(pos, self._strides)))

    def getNeighborId(self, block_id, axis, lower):  # noqa: N802
        """Id of the neighbouring block along ``axis`` (the lower one if
        ``lower``), -1 past the grid (mutex_watershed/two_pass_mws.py:241)."""
        pos = self.blockGridPosition(block_id)
        pos[axis] += -1 if lower else 1
        if not 0 <= pos[axis] < self.blocksPerAxis[axis]:
            return -1
        return self.gridPositionToBlockId(pos)

    def getBlock(self, block_id):  # noqa: N802
        if not 0 <= block_id < self.numberOfBlocks:
            raise IndexError('block id %d out of range' % block_id)
        pos = self.blockGridPosition(block_id)
        begin = [rb + p * s for rb, p, s in zip(self.roiBegin, pos, self.blockShape)]
        end = [min(b + s, re) for b, s, re in zip(begin, self.blockShape, self.roiEnd)]
        return Block(begin, end)

    def getBlockWithHalo(self, block_id, halo):  # noqa: N802
        inner = self.getBlock(block_id)
        ob = [max(b - h, rb) for b, h, rb in zip(inner.begin, halo, self.roiBegin)]
        oe = [min(e + h, re) for e, h, re in zip(inner.end, halo, self.roiEnd)]
        outer = Block(ob, oe)
        local = Block([b - o for b, o in zip(inner.begin, ob)], [e - o for e, o in zip(inner.end, ob)])
        return BlockWithHalo(outer, inner, local)

    def getBlockIdsOverlappingBoundingBox(self, roiBegin, roiEnd, blockHalo=None):  # noqa: N802,N803
        ranges = []
        for ax in range(len(self.blockShape)):
            b = max(int(roiBegin[ax]), self.roiBegin[ax]) - self.roiBegin[ax]
            e = min(int(roiEnd[ax]), self.roiEnd[ax]) - self.roiBegin[ax]
            if e <= b:
                return np.zeros(0, dtype=np.uint64)
            ranges.append(range(b // self.blockShape[ax], (e - 1) // self.blockShape[ax] + 1))
        ids = [self.gridPositionToBlockId(p) for p in itertools.product(*ranges)]
        return np.array(sorted(ids), dtype=np.uint64)

    def getBlockIdsInBoundingBox(self, roiBegin, roiEnd, blockHalo=None):  # noqa: N802,N803
        """Blocks fully inside [roiBegin, roiEnd) (used by the multi-scale merge,
        merge_sub_graphs.py:144-146)."""
        cand = self.getBlockIdsOverlappingBoundingBox(roiBegin, roiEnd)
        keep = []
        for bid in cand:
            blk = self.getBlock(int(bid))
            if all(b >= rb and e <= re for b, e, rb, re in zip(blk.begin, blk.end, roiBegin, roiEnd)):
                keep.append(int(bid))
        return np.array(keep, dtype=np.uint64)


def blocks_in_volume(shape, block_shape, roi_begin=None, roi_end=None, block_list_path=None,
                     return_blocking=False):
    """vu.blocks_in_volume (utils/volume_utils.py:31-73): all block ids, those
    overlapping an ROI, those listed in a JSON file, or the intersection."""
    import json
    import os
    assert len(shape) == len(block_shape)
    assert (roi_begin is None) == (roi_end is None)
    if block_list_path is not None and not os.path.exists(block_list_path):
        raise AssertionError("Was given block_list_path %s that doesn't exist" % block_list_path)
    b = blocking([0] * len(shape), list(shape), list(block_shape))
    if roi_begin is None and block_list_path is None:
        ids = list(range(b.numberOfBlocks))
    else:
        ids = None
        if roi_begin is not None:
            roi_end = [s if e is None else e for e, s in zip(roi_end, shape)]
            ids = b.getBlockIdsOverlappingBoundingBox(list(roi_begin), list(roi_end)).tolist()
        if block_list_path is not None:
            with open(block_list_path) as f:
                listed = json.load(f)
            ids = listed if ids is None else np.intersect1d(listed, ids).tolist()
    return (ids, b) if return_blocking else ids
