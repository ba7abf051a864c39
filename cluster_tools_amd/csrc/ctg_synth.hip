// Device twin of cluster_tools_amd/synthetic.py: jittered-grid Voronoi
// supervoxels (uint64) + a float32 boundary map, bit-identical to the host
// generator (integer geometry, correctly rounded double division, no FMA:
// the library is built with -ffp-contract=off).  Used by bench.py to build the
// BASELINE.json synthetic volumes directly in HBM.
#include <algorithm>

#include "ctg_internal.h"

namespace ctg {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct SynthParams {
    int64_t shape[3];
    int64_t gshape[3];
    int64_t ncell[3];
    int64_t z_offset;
    int cell;
    uint64_t seed;
    uint64_t label_offset;
    double noise_amp;
};

__device__ __forceinline__ int64_t seed_coord(const SynthParams& P, uint64_t cid, int k, int64_t c) {
    const uint64_t span = (uint64_t)(256 * P.cell);
    const uint64_t h = splitmix64(P.seed ^ (cid * 3ull + (uint64_t)k));
    return c * 256 * P.cell + (int64_t)(h % span);
}

__device__ __forceinline__ void synth_voxel(const SynthParams& P, int64_t i, uint64_t* __restrict__ labels,
                                            float* __restrict__ boundary) {
    const int64_t X = P.shape[2], Y = P.shape[1];
    const int64_t x = i % X, y = (i / X) % Y, zl = i / (X * Y);
    const int64_t z = zl + P.z_offset;
    const int64_t pz = z * 256 + 128, py = y * 256 + 128, px = x * 256 + 128;
    const int64_t cz0 = z / P.cell, cy0 = y / P.cell, cx0 = x / P.cell;
    const int64_t big = (int64_t)1 << 62;
    int64_t d1 = big, d2 = big, best = 0;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                const int64_t cz = cz0 + dz, cy = cy0 + dy, cx = cx0 + dx;
                const bool valid = cz >= 0 && cz < P.ncell[0] && cy >= 0 && cy < P.ncell[1] && cx >= 0 &&
                                   cx < P.ncell[2];
                const int64_t czc = min(max(cz, (int64_t)0), P.ncell[0] - 1);
                const int64_t cyc = min(max(cy, (int64_t)0), P.ncell[1] - 1);
                const int64_t cxc = min(max(cx, (int64_t)0), P.ncell[2] - 1);
                const int64_t cid = (czc * P.ncell[1] + cyc) * P.ncell[2] + cxc;
                const int64_t sz = seed_coord(P, (uint64_t)cid, 0, czc);
                const int64_t sy = seed_coord(P, (uint64_t)cid, 1, cyc);
                const int64_t sx = seed_coord(P, (uint64_t)cid, 2, cxc);
                int64_t d = (pz - sz) * (pz - sz) + (py - sy) * (py - sy) + (px - sx) * (px - sx);
                if (!valid) d = big;
                if (d < d1) {
                    d2 = d1;
                    d1 = d;
                    best = cid;
                } else if (d < d2) {
                    d2 = d;
                }
            }
    labels[i] = (uint64_t)best + 1ull + P.label_offset;
    if (boundary) {
        const double K = 4.0 * 256.0 * 256.0;
        const double g = (double)(d2 - d1);
        double val = K / (K + g);
        const uint64_t vid = (uint64_t)((z * P.gshape[1] + y) * P.gshape[2] + x);
        const uint64_t h = splitmix64(vid ^ (P.seed * 0x632BE59BD9B4E019ull));
        const double noise = ((double)(h & 0xFFFFull) / 65536.0 - 0.5) * P.noise_amp;
        val = val + noise;
        val = val < 0.0 ? 0.0 : (val > 1.0 ? 1.0 : val);
        boundary[i] = (float)val;
    }
}

__global__ __launch_bounds__(256) void k_synth(SynthParams P, uint64_t* __restrict__ labels,
                                               float* __restrict__ boundary) {
    const int64_t n = P.shape[0] * P.shape[1] * P.shape[2];
    // grid-stride: a launch covers at most 2^32 work-items (2048^3 volumes)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        synth_voxel(P, i, labels, boundary);
}

__global__ void k_synth_aff(const float* __restrict__ b, float* __restrict__ out, int64_t Z, int64_t Y, int64_t X,
                            int oz, int oy, int ox) {
    const int64_t n = Z * Y * X;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = i % X, y = (i / X) % Y, z = i / (X * Y);
        const int64_t qz = z + oz, qy = y + oy, qx = x + ox;
        float v = b[i];
        if (qz >= 0 && qz < Z && qy >= 0 && qy < Y && qx >= 0 && qx < X) v = fmaxf(v, b[(qz * Y + qy) * X + qx]);
        out[i] = v;
    }
}

hipError_t launch_synth(uint64_t* labels, float* boundary, const int64_t* shape, int64_t z_offset,
                        const int64_t* gshape, int cell, uint64_t seed, uint64_t label_offset, double noise_amp,
                        hipStream_t s) {
    SynthParams P;
    for (int k = 0; k < 3; ++k) {
        P.shape[k] = shape[k];
        P.gshape[k] = gshape[k];
        P.ncell[k] = (gshape[k] + cell - 1) / cell;
    }
    P.z_offset = z_offset;
    P.cell = cell;
    P.seed = seed;
    P.label_offset = label_offset;
    P.noise_amp = noise_amp;
    const int64_t n = shape[0] * shape[1] * shape[2];
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1 << 20)), dim3(256), 0, s, P, labels, boundary);
    return hipGetLastError();
}

hipError_t launch_synth_aff(const float* b, float* out, const int64_t* shape, int n_channels, const int32_t* off,
                            hipStream_t s) {
    const int64_t n = shape[0] * shape[1] * shape[2];
    if (n == 0) return hipSuccess;
    for (int c = 0; c < n_channels; ++c) {
        hipLaunchKernelGGL(k_synth_aff, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1 << 20)), dim3(256), 0, s, b, out + (size_t)c * n,
                           shape[0], shape[1], shape[2], off[3 * c], off[3 * c + 1], off[3 * c + 2]);
    }
    return hipGetLastError();
}

}  // namespace ctg
