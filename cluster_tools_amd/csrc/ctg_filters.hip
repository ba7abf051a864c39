// Filter responses of the filter-feature branch (gfx950).
//
// The reference's BlockEdgeFeatures task, when configured with `filters` /
// `sigmas`, smooths the block input with fastfilters / vigra
// (utils/volume_utils.py:80-94, features/block_edge_features.py:151-168) and
// accumulates every response channel over the block's RAG edges with
// ndist.accumulateInput.  The filters are separable Gaussian-derivative
// convolutions plus a per-voxel combine (gradient magnitude, Laplacian, the
// eigenvalues of the Hessian / structure tensor), i.e. HBM-bound streaming
// work: one pass per axis reads and writes 4 B per voxel.
//
//   k_conv_axis     out[p] = sum_k taps[k] * in[reflect(p + (k - R) e_axis)]
//                   (vigra BORDER_TREATMENT_REFLECT: mirror without repeating
//                   the edge voxel).  One thread per voxel, x fastest, so every
//                   tap of a wave is one coalesced row read (L2 serves the
//                   2R+1 overlapping reads of neighbouring outputs).
//   k_combine       elementwise: |g| (1..3 components), sums, products, a - b
//   k_sym_eig       eigenvalues of the symmetric 2x2 / 3x3 matrix per voxel,
//                   descending (vigra's order), closed form in f64
#include "ctg_internal.h"

namespace ctg {

constexpr int FILT_THREADS = 256;
constexpr int MAX_TAPS = 257;

struct Taps {
    float w[MAX_TAPS];
};

__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
    // mirror at both borders without repeating the border voxel; n == 1 -> 0
    if (n == 1) return 0;
    const int64_t period = 2 * (n - 1);
    i %= period;
    if (i < 0) i += period;
    return i < n ? i : period - i;
}

__global__ __launch_bounds__(FILT_THREADS) void k_conv_axis(const float* __restrict__ in, float* __restrict__ out,
                                                            int64_t n0, int64_t n1, int64_t n2, int axis, Taps T,
                                                            int radius) {
    const int64_t V = n0 * n1 * n2;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < V; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i2 = p % n2, i1 = (p / n2) % n1, i0 = p / (n1 * n2);
        const int64_t n = axis == 0 ? n0 : (axis == 1 ? n1 : n2);
        const int64_t c = axis == 0 ? i0 : (axis == 1 ? i1 : i2);
        const int64_t stride = axis == 0 ? n1 * n2 : (axis == 1 ? n2 : 1);
        const int64_t base = p - c * stride;
        double acc = 0.0;
        for (int k = -radius; k <= radius; ++k)
            acc += (double)T.w[k + radius] * (double)in[base + reflect_idx(c + k, n) * stride];
        out[p] = (float)acc;
    }
}

// op 0: sqrt(a^2 + b^2 + c^2) (absent components null)   op 1: a + b + c
// op 2: a * b                                               op 3: a - b
__global__ __launch_bounds__(FILT_THREADS) void k_combine(int op, const float* __restrict__ a,
                                                          const float* __restrict__ b, const float* __restrict__ c,
                                                          float* __restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float x = a[i], y = b ? b[i] : 0.f, z = c ? c[i] : 0.f;
        float r;
        if (op == 0) r = sqrtf(x * x + y * y + z * z);
        else if (op == 1) r = x + y + z;
        else if (op == 2) r = x * y;
        else r = x - y;
        out[i] = r;
    }
}

// eigenvalues (descending) of the symmetric matrix with upper-triangle
// components comp[k] (planes of n voxels): 2x2 (a00, a01, a11) or 3x3
// (a00, a01, a02, a11, a12, a22); out is (n, dim) channel-last
__global__ __launch_bounds__(FILT_THREADS) void k_sym_eig(const float* __restrict__ comp, int dim, int64_t n,
                                                          float* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (dim == 2) {
            const double a = comp[i], b = comp[n + i], d = comp[2 * n + i];
            const double m = 0.5 * (a + d), r = sqrt(0.25 * (a - d) * (a - d) + b * b);
            out[2 * i] = (float)(m + r);
            out[2 * i + 1] = (float)(m - r);
            continue;
        }
        const double a00 = comp[i], a01 = comp[n + i], a02 = comp[2 * n + i];
        const double a11 = comp[3 * n + i], a12 = comp[4 * n + i], a22 = comp[5 * n + i];
        const double p1 = a01 * a01 + a02 * a02 + a12 * a12;
        double e0, e1, e2;
        if (p1 == 0.0) {   // diagonal
            e0 = a00;
            e1 = a11;
            e2 = a22;
        } else {
            // trigonometric solution of the characteristic cubic (Smith 1961)
            const double q = (a00 + a11 + a22) / 3.0;
            const double b00 = a00 - q, b11 = a11 - q, b22 = a22 - q;
            const double p2 = b00 * b00 + b11 * b11 + b22 * b22 + 2.0 * p1;
            const double p = sqrt(p2 / 6.0);
            const double det = b00 * (b11 * b22 - a12 * a12) - a01 * (a01 * b22 - a12 * a02) +
                               a02 * (a01 * a12 - b11 * a02);
            double r = det / (2.0 * p * p * p);
            r = fmin(1.0, fmax(-1.0, r));
            const double phi = acos(r) / 3.0;
            e0 = q + 2.0 * p * cos(phi);
            e2 = q + 2.0 * p * cos(phi + 2.0943951023931953);   // + 2 pi / 3
            e1 = 3.0 * q - e0 - e2;
        }
        // descending order
        double t;
        if (e0 < e1) { t = e0; e0 = e1; e1 = t; }
        if (e1 < e2) { t = e1; e1 = e2; e2 = t; }
        if (e0 < e1) { t = e0; e0 = e1; e1 = t; }
        out[3 * i] = (float)e0;
        out[3 * i + 1] = (float)e1;
        out[3 * i + 2] = (float)e2;
    }
}

static unsigned grid_for(int64_t n) {
    const int64_t b = (n + FILT_THREADS - 1) / FILT_THREADS;
    return (unsigned)(b < 1 ? 1 : (b > 65536 * 8 ? 65536 * 8 : b));
}

}  // namespace ctg

using namespace ctg;

extern "C" {

int ctg_filter_conv_axis(const float* in, float* out, const int64_t* shape, int ndim, int axis, const float* taps,
                         int n_taps, void* stream) {
    if (!in || !out || !shape || !taps || ndim < 1 || ndim > 3 || axis < 0 || axis >= ndim || n_taps < 1 ||
        n_taps > MAX_TAPS || (n_taps & 1) == 0 || in == out) {
        set_error("ctg_filter_conv_axis: bad arguments (odd tap count <= 257, distinct in/out, axis < ndim <= 3)");
        return CTG_ERR_ARG;
    }
    int64_t s[3] = {1, 1, 1};
    for (int k = 0; k < ndim; ++k) s[3 - ndim + k] = shape[k];
    const int ax = 3 - ndim + axis;
    for (int k = 0; k < 3; ++k)
        if (s[k] <= 0) return CTG_OK;
    Taps T;
    for (int k = 0; k < n_taps; ++k) T.w[k] = taps[k];
    hipLaunchKernelGGL(k_conv_axis, dim3(grid_for(s[0] * s[1] * s[2])), dim3(FILT_THREADS), 0, (hipStream_t)stream, in,
                       out, s[0], s[1], s[2], ax, T, n_taps / 2);
    CTG_CHECK(hipGetLastError());
    return CTG_OK;
}

int ctg_filter_combine(int op, const float* a, const float* b, const float* c, float* out, int64_t n, void* stream) {
    if (op < 0 || op > 3 || !a || !out || n < 0 || (op >= 2 && !b)) {
        set_error("ctg_filter_combine: bad arguments");
        return CTG_ERR_ARG;
    }
    if (n == 0) return CTG_OK;
    hipLaunchKernelGGL(k_combine, dim3(grid_for(n)), dim3(FILT_THREADS), 0, (hipStream_t)stream, op, a, b, c, out, n);
    CTG_CHECK(hipGetLastError());
    return CTG_OK;
}

int ctg_sym_eigenvalues(const float* comps, int dim, int64_t n, float* out, void* stream) {
    if (!comps || !out || (dim != 2 && dim != 3) || n < 0) {
        set_error("ctg_sym_eigenvalues: bad arguments (dim 2 or 3)");
        return CTG_ERR_ARG;
    }
    if (n == 0) return CTG_OK;
    hipLaunchKernelGGL(k_sym_eig, dim3(grid_for(n)), dim3(FILT_THREADS), 0, (hipStream_t)stream, comps, dim, n, out);
    CTG_CHECK(hipGetLastError());
    return CTG_OK;
}

}  // extern "C"
