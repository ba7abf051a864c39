"""Every rank's exchange steps of cluster_tools_amd/dist.py in ONE process:
the collectives are replaced by their data movement (all_gather = stack,
all_to_all = slicing the senders' segments), so the device steps
(ctg_mgpu_sample / split / pack / merge, or their numpy restatement in
tests/dist_helpers.py) are tested at any world size without processes or a
process group.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np
import torch

from cluster_tools_amd import dist as cdist


def simulate(backend, labels, data, world, offsets=None, hist_range=(0.0, 1.0), fresh=False):
    """Shards (one per rank) of the volume ``labels`` / ``data`` (numpy for
    the numpy backend, CUDA tensors for the HIP backend) split into the z-slabs
    of ``ctg_mgpu_slab``.

    fresh: re-run a rank's local call right before its pack and its merge.
    A CTG_DEFER_STATS table rebuilds its statistics from the records of the
    device's latest call, and every rank shares this process's one device, so
    without it the earlier ranks' tables are stale (CTG_ERR_STALE); the local
    call is deterministic, so the fresh table is the same table."""
    Z = labels.shape[0]

    def local(r):
        rd, own, end = cdist.slab_plan(Z, world, r, offsets)
        if offsets is None:
            d = data[rd:end]
        else:
            d = data[:, rd:end]
        if isinstance(labels, np.ndarray):
            lab_s, d = np.ascontiguousarray(labels[rd:end]), np.ascontiguousarray(d)
        else:
            lab_s, d = labels[rd:end].contiguous(), d.contiguous()
        return backend.local(lab_s, d, offsets, (own - rd, 0, 0), None, False, hist_range)

    def refresh(r):
        if fresh:
            locs[r].free()
            locs[r] = local(r)

    locs = [local(r) for r in range(world)]
    meta_all = torch.stack([backend.sample(x) for x in locs])
    counts_all = torch.stack([backend.split(x, meta_all, world) for x in locs]).cpu().numpy()
    sends, words = [], []
    for r in range(world):
        sw, _ = cdist.segment_words(counts_all, world, r)
        words.append(sw)
        if sum(sw):
            refresh(r)
        sends.append(backend.pack(locs[r], counts_all, world, r, int(sum(sw))) if sum(sw) else None)
    shards = []
    for r in range(world):
        parts = []
        for q in range(world):
            if q == r or not words[q][r]:
                continue
            a = int(sum(words[q][:r]))
            parts.append(sends[q][a:a + words[q][r]])
        recv = torch.cat(parts) if parts else None
        refresh(r)
        shards.append(backend.merge(locs[r], recv, counts_all, world, r, hist_range))
    for x in locs:
        x.free()
    return shards
