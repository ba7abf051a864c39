"""Deterministic synthetic supervoxel volumes (host twin of the HIP generator).

BASELINE.json configs 2-5 quote synthetic "watershed-like" volumes: jittered
grid Voronoi cells (uint64 labels) plus a float32 boundary map that is high on
cell faces.  Everything here is integer / correctly-rounded double arithmetic
so that the HIP generator in ``csrc/ctg_synth.hip`` produces bit-identical
volumes (checked by tests/test_gpu_parity.py).

Geometry (all integer, positions in 1/256 voxel units):
  cell c = (cz, cy, cx) of size ``cell`` voxels, grid over the GLOBAL shape;
  seed_c = 256*cell*c + (splitmix64(seed ^ id*3+k) mod 256*cell) per axis;
  label(p) = 1 + linear id of the nearest seed among the 3x3x3 cells around
  floor(p/cell) (strict '<', scan order z,y,x -> smallest id wins ties)
  + label_offset;
  boundary(p) = float32(clamp(K/(K+D2-D1) + noise, 0, 1)) with D1 <= D2 the two
  smallest squared distances, K = 4 voxel^2, noise = (h16/65536 - 0.5)*noise_amp.
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1
K_FIX = 4 * 256 * 256


def splitmix64_np(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over='ignore'):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def cell_grid(global_shape, cell):
    return tuple((s + cell - 1) // cell for s in global_shape)


def seed_positions(global_shape, cell, seed):
    """(ncz, ncy, ncx, 3) int64 seed coordinates in 1/256 voxel units."""
    ncz, ncy, ncx = cell_grid(global_shape, cell)
    cid = np.arange(ncz * ncy * ncx, dtype=np.uint64)
    out = np.empty((cid.size, 3), dtype=np.int64)
    span = np.uint64(256 * cell)
    cz = (cid // np.uint64(ncy * ncx)).astype(np.int64)
    cy = ((cid // np.uint64(ncx)) % np.uint64(ncy)).astype(np.int64)
    cx = (cid % np.uint64(ncx)).astype(np.int64)
    base = (cz, cy, cx)
    with np.errstate(over='ignore'):
        for k in range(3):
            h = splitmix64_np(np.uint64(seed) ^ (cid * np.uint64(3) + np.uint64(k)))
            out[:, k] = base[k] * 256 * cell + (h % span).astype(np.int64)
    return out.reshape(ncz, ncy, ncx, 3)


def generate(shape, cell=10, seed=0, z_offset=0, global_shape=None,
             label_offset=0, noise_amp=0.1, with_boundary=True):
    """Labels (uint64) and boundary (float32) for the sub-volume
    z in [z_offset, z_offset + shape[0]) of the global volume."""
    shape = tuple(int(s) for s in shape)
    if global_shape is None:
        global_shape = (z_offset + shape[0],) + shape[1:]
    ncz, ncy, ncx = cell_grid(global_shape, cell)
    seeds = seed_positions(global_shape, cell, seed)
    z = np.arange(z_offset, z_offset + shape[0], dtype=np.int64)
    y = np.arange(shape[1], dtype=np.int64)
    x = np.arange(shape[2], dtype=np.int64)
    Z, Y, X = np.meshgrid(z, y, x, indexing='ij')
    pz, py, px = Z * 256 + 128, Y * 256 + 128, X * 256 + 128
    cz0, cy0, cx0 = Z // cell, Y // cell, X // cell
    big = np.int64(1) << np.int64(62)
    d1 = np.full(shape, big, dtype=np.int64)
    d2 = np.full(shape, big, dtype=np.int64)
    best = np.zeros(shape, dtype=np.int64)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                cz, cy, cx = cz0 + dz, cy0 + dy, cx0 + dx
                valid = ((cz >= 0) & (cz < ncz) & (cy >= 0) & (cy < ncy) &
                         (cx >= 0) & (cx < ncx))
                czc = np.clip(cz, 0, ncz - 1)
                cyc = np.clip(cy, 0, ncy - 1)
                cxc = np.clip(cx, 0, ncx - 1)
                s = seeds[czc, cyc, cxc]
                d = ((pz - s[..., 0]) ** 2 + (py - s[..., 1]) ** 2 +
                     (px - s[..., 2]) ** 2)
                d = np.where(valid, d, big)
                cid = (czc * ncy + cyc) * ncx + cxc
                closer = d < d1
                second = (~closer) & (d < d2)
                d2 = np.where(closer, d1, np.where(second, d, d2))
                best = np.where(closer, cid, best)
                d1 = np.where(closer, d, d1)
    labels = (best.astype(np.uint64) + np.uint64(1) + np.uint64(label_offset))
    if not with_boundary:
        return labels, None
    g = (d2 - d1).astype(np.float64)
    val = float(K_FIX) / (float(K_FIX) + g)
    vid = ((Z * global_shape[1] + Y) * global_shape[2] + X).astype(np.uint64)
    h = splitmix64_np(vid ^ np.uint64((int(seed) * 0x632BE59BD9B4E019) & MASK64))
    noise = ((h & np.uint64(0xFFFF)).astype(np.float64) / 65536.0 - 0.5) * noise_amp
    val = np.clip(val + noise, 0.0, 1.0).astype(np.float32)
    return labels, val


def affinities_from_boundary(boundary, offsets):
    """(C,Z,Y,X) float32: aff[c,p] = max(B[p], B[p+o_c]) (B[p] if p+o_c is
    outside the volume) -- a deterministic, exact stand-in for CNN affinities."""
    b = np.asarray(boundary, dtype=np.float32)
    out = np.empty((len(offsets),) + b.shape, dtype=np.float32)
    for c, off in enumerate(offsets):
        shifted = b.copy()
        src, dst = [], []
        for ax, o in enumerate(off):
            n = b.shape[ax]
            o = int(o)
            if o >= 0:
                dst.append(slice(0, max(n - o, 0)))
                src.append(slice(o, n))
            else:
                dst.append(slice(-o, n))
                src.append(slice(0, max(n + o, 0)))
        shifted[tuple(dst)] = b[tuple(src)]
        out[c] = np.maximum(b, shifted)
    return out


NN_OFFSETS = [[-1, 0, 0], [0, -1, 0], [0, 0, -1]]  # test_edge_features.py:26
LR_OFFSETS = [[-1, 0, 0], [0, -1, 0], [0, 0, -1],   # test/mutex_watershed/test_mws.py:26-29
              [-2, 0, 0], [0, -3, 0], [0, 0, -3],
              [-3, 0, 0], [0, -9, 0], [0, 0, -9],
              [-4, 0, 0], [0, -27, 0], [0, 0, -27]]
