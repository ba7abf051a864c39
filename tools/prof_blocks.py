"""Batched per-block calls (ctg_rag_blocks) on the configs[0] geometry with
device-resident arenas, for rocprofv3: 50 blocks of 64x256x256 (+ halo) of a
125x1250x1250 synthetic volume; graph call + feature call, a few times."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cluster_tools_amd import rag  # noqa: E402
from cluster_tools_amd.blocking import blocking  # noqa: E402

shape, block = (125, 1250, 1250), (64, 256, 256)
lt, bt = rag.synth_volume(shape, cell=10)
blk = blocking([0, 0, 0], list(shape), list(block))
descs, sls, lo = [], [], 0
for b in range(blk.numberOfBlocks):
    bb = blk.getBlock(b)
    rb = [max(x - 1, 0) for x in bb.begin]
    shp = [y - x for x, y in zip(rb, bb.end)]
    descs.append(dict(label_offset=lo, data_offset=lo, shape=shp,
                      own=([x - r for x, r in zip(bb.begin, rb)], [y - r for y, r in zip(bb.end, rb)]),
                      graph=([0, 0, 0], shp)))
    sls.append(tuple(slice(x, y) for x, y in zip(rb, bb.end)))
    lo += int(np.prod(shp))
la = torch.cat([lt[s].reshape(-1) for s in sls])
da = torch.cat([bt[s].reshape(-1) for s in sls])
del lt, bt
# algorithmic bytes of the feature call's face scan: every block array (+ halo)
# read once, 8 B label + 4 B sample per voxel (bench.py --config 0)
print('feature_scan_bytes=%d' % (lo * 12), flush=True)
rag.set_profiling(True)
for i in range(int(os.environ.get('CTG_PROF_ITERS', '4'))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rag.rag_blocks_arena(la, descs)
    t1 = time.perf_counter()
    g = rag.last_timings()
    rag.rag_blocks_arena(la, descs, da, keep_stats=True)
    t2 = time.perf_counter()
    f = rag.last_timings()
    print('graph %.2f ms %s | features %.2f ms %s' % ((t1 - t0) * 1e3, {k: round(v, 3) for k, v in g.items()},
                                                      (t2 - t1) * 1e3, {k: round(v, 3) for k, v in f.items()}),
          flush=True)
