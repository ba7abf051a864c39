// Record reduction: sort (tile, edge) records by edge key, combine each run into
// one edge row and finalise the 10 nifty edge features.
//
//   records --pack--> (u<<nb)|v sort keys --radix sort (rocPRIM, 2*nb bits)-->
//   run-length encode --> one thread per edge: sum counts/sums, min/max,
//   42-slot histogram in registers --> mean, population variance and the vigra
//   StandardQuantiles<UserRangeHistogram<40>> quantiles (0,.1,.25,.5,.75,.9,1).
//
// Column contract (E,10): mean, var, min, q10, q25, q50, q75, q90, max, count
// (features/block_edge_features.py:146-147, features/merge_edge_features.py:62-65,
// costs/probs_to_costs.py:205-207).
#include "ctg_internal.h"

namespace ctg {

__global__ void k_pack_keys(int64_t n, const uint64_t* __restrict__ key, int nb, uint64_t* __restrict__ sk,
                            uint32_t* __restrict__ idx) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = key[i];
    sk[i] = ((k >> 32) << nb) | (k & 0xFFFFFFFFull);
    idx[i] = (uint32_t)i;
}

// pack (u,v) pairs given as two u64 (merge inputs); flags labels >= 2^32
__global__ void k_pack_pairs(int64_t n, const uint64_t* __restrict__ uv, int nb, uint64_t* __restrict__ sk,
                             uint32_t* __restrict__ idx) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sk[i] = (uv[2 * i] << nb) | uv[2 * i + 1];
    idx[i] = (uint32_t)i;
}

__global__ void k_max_pairs(int64_t n, const uint64_t* __restrict__ uv, unsigned long long* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long m = 0;
    if (i < n) m = max(uv[2 * i], uv[2 * i + 1]);
    // wave reduction then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        unsigned lo = __shfl_xor((unsigned)m, o, 64), hi = __shfl_xor((unsigned)(m >> 32), o, 64);
        unsigned long long other = ((unsigned long long)hi << 32) | lo;
        m = max(m, other);
    }
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// ---------------------------------------------------------------------------
// vigra computeStandardQuantiles as a single streaming walk over the bins
// ---------------------------------------------------------------------------
struct QuantileWalk {
    static constexpr int NQ = 7;
    double count, scale, inv_scale, offset;
    double res[NQ];
    int q, qend;
    double qcount;
    bool have_prev, have_pend;
    double prev_kp, prev_ch, pend_kp, pend_ch;

    __device__ __forceinline__ static double qv(int i) {
        // 0.0 and 1.0 handled exactly (min/max), the rest by interpolation
        return i == 1 ? 0.1 : i == 2 ? 0.25 : i == 3 ? 0.5 : i == 4 ? 0.75 : i == 5 ? 0.9 : (i == 0 ? 0.0 : 1.0);
    }
    __device__ void init(double cnt, double sc, double off) {
        count = cnt;
        scale = sc;
        inv_scale = 1.0 / sc;
        offset = off;
        for (int i = 0; i < NQ; ++i) res[i] = 0.0;
        q = 1;  // quantile 0.0 -> minimum
        qend = NQ - 1;  // quantile 1.0 -> maximum
        qcount = count * qv(q);
        have_prev = have_pend = false;
    }
    __device__ void consume(double kp, double ch) {
        if (!have_prev) {
            prev_kp = kp;
            prev_ch = ch;
            have_prev = true;
            return;
        }
        while (q < qend && prev_ch < qcount && ch >= qcount) {
            double t = (qcount - prev_ch) / (ch - prev_ch) * (kp - prev_kp);
            res[q] = inv_scale * (t + prev_kp) + offset;
            ++q;
            qcount = count * qv(q);
        }
        prev_kp = kp;
        prev_ch = ch;
    }
    __device__ void gen(double kp, double ch) {
        if (have_pend) consume(pend_kp, pend_ch);
        pend_kp = kp;
        pend_ch = ch;
        have_pend = true;
    }
    __device__ double last_kp() const { return pend_kp; }
};

template <bool WIDE>
__device__ __forceinline__ void load_record(const RecordBuf& R, uint32_t i, uint32_t (&h)[NSLOTS], uint32_t& cnt,
                                            uint32_t& flags, uint32_t& mn, uint32_t& mx) {
    if constexpr (!WIDE) {
        const uint4* p = (const uint4*)(R.hist + (size_t)i * NREC_WORDS);
        uint32_t w[NREC_WORDS];
#pragma unroll
        for (int j = 0; j < NREC_WORDS / 4; ++j) {
            uint4 v = p[j];
            w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
        }
#pragma unroll
        for (int j = 0; j < HWORDS; ++j) {
            h[2 * j] += w[j] & 0xFFFFu;
            h[2 * j + 1] += w[j] >> 16;
        }
        cnt += w[21] & ~ADJ_FLAG;
        flags |= w[21] & ADJ_FLAG;
        mn = min(mn, w[22]);
        mx = max(mx, w[23]);
    } else {
        const uint4* p = (const uint4*)(R.hist + (size_t)i * WREC_WORDS);
        uint32_t w[WREC_WORDS];
#pragma unroll
        for (int j = 0; j < WREC_WORDS / 4; ++j) {
            uint4 v = p[j];
            w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
        }
#pragma unroll
        for (int j = 0; j < NSLOTS; ++j) h[j] += w[j];
        cnt += w[42] & ~ADJ_FLAG;
        flags |= w[42] & ADJ_FLAG;
        mn = min(mn, w[43]);
        mx = max(mx, w[44]);
    }
}

template <bool WIDE, bool STATS>
__global__ __launch_bounds__(256) void k_reduce_edges(int64_t E, const uint64_t* __restrict__ uniq,
                                                      const uint32_t* __restrict__ runs,
                                                      const uint32_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ perm, RecordBuf R, int nb,
                                                      int need_adj, int ignore_label, double scale, double offset,
                                                      ReduceOut O) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const uint64_t sk = uniq[e];
    const uint64_t u = sk >> nb, v = sk & ((1ull << nb) - 1ull);
    O.edges[2 * e] = u;
    O.edges[2 * e + 1] = v;
    uint32_t flags = 0;
    if constexpr (!STATS) {
        if (need_adj) {
            const uint32_t b = offs[e], n = runs[e];
            for (uint32_t r = b; r < b + n; ++r) {
                const uint32_t i = perm[r];
                flags |= R.hist[(size_t)i * (WIDE ? WREC_WORDS : NREC_WORDS) + (WIDE ? 42 : 21)] & ADJ_FLAG;
            }
        } else {
            flags = ADJ_FLAG;
        }
        if (O.keep) O.keep[e] = ((flags & ADJ_FLAG) || !need_adj) && !(ignore_label && u == 0) ? 1u : 0u;
        return;
    } else {
        uint32_t h[NSLOTS];
#pragma unroll
        for (int j = 0; j < NSLOTS; ++j) h[j] = 0;
        uint32_t cnt = 0, mn = ORD_POS_INF, mx = ORD_NEG_INF;
        double sum = 0.0, sq = 0.0;
        const uint32_t b = offs[e], n = runs[e];
        for (uint32_t r = b; r < b + n; ++r) {
            const uint32_t i = perm[r];
            load_record<WIDE>(R, i, h, cnt, flags, mn, mx);
            const double2 s = R.sums[i];
            sum += s.x;
            sq += s.y;
        }
        if (!need_adj) flags |= ADJ_FLAG;
        const bool keep = (flags & ADJ_FLAG) && !(ignore_label && u == 0);
        if (O.keep) O.keep[e] = keep ? 1u : 0u;
        if (O.wstats) {
            uint4* p = (uint4*)(O.wstats + (size_t)e * WREC_WORDS);
            uint32_t w[WREC_WORDS];
#pragma unroll
            for (int j = 0; j < NSLOTS; ++j) w[j] = h[j];
            w[42] = cnt | (flags & ADJ_FLAG);
            w[43] = mn;
            w[44] = mx;
            w[45] = w[46] = w[47] = 0;
#pragma unroll
            for (int j = 0; j < WREC_WORDS / 4; ++j) p[j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
            O.wsums[e] = make_double2(sum, sq);
        }
        if (!O.feats) return;
        double f[N_FEATURES];
#pragma unroll
        for (int j = 0; j < N_FEATURES; ++j) f[j] = 0.0;
        if (cnt > 0) {
            const double c = (double)cnt;
            const double mean = sum / c;
            double var = (sq - sum * mean) / c;
            if (var < 0.0) var = 0.0;
            const double vmin = (double)ord2f(mn), vmax = (double)ord2f(mx);
            QuantileWalk W;
            W.init(c, scale, offset);
            const double left = (double)h[0], right = (double)h[NSLOTS - 1];
            W.gen(scale * (vmin - offset), 0.0);
            if (left > 0.0) W.gen(0.0, left);
            double cum = left;
#pragma unroll
            for (int k = 0; k < NBINS; ++k) {
                const uint32_t hk = h[k + 1];
                if (hk > 0) {
                    if (W.last_kp() <= (double)k) W.gen((double)k, cum);
                    cum += (double)hk;
                    W.gen((double)(k + 1), cum);
                }
            }
            if (right > 0.0) {
                if (W.last_kp() != (double)NBINS) W.gen((double)NBINS, cum);
                W.gen(scale * (vmax - offset), c);
                W.consume(W.pend_kp, W.pend_ch);
            } else {
                W.consume(scale * (vmax - offset), c);  // replaces the last keypoint
            }
            f[0] = mean;
            f[1] = var;
            f[2] = vmin;
#pragma unroll
            for (int j = 1; j < 6; ++j) f[2 + j] = W.res[j];
            f[8] = vmax;
            f[9] = c;
        }
        double* o = O.feats + (size_t)e * N_FEATURES;
#pragma unroll
        for (int j = 0; j < N_FEATURES; ++j) o[j] = f[j];
    }
}

__global__ void k_compact(int64_t E, const uint32_t* __restrict__ keep, const uint32_t* __restrict__ pos,
                          ReduceOut in, ReduceOut out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E || !keep[e]) return;
    const uint32_t p = pos[e];
    out.edges[2 * (size_t)p] = in.edges[2 * e];
    out.edges[2 * (size_t)p + 1] = in.edges[2 * e + 1];
    if (in.feats)
        for (int j = 0; j < N_FEATURES; ++j) out.feats[(size_t)p * N_FEATURES + j] = in.feats[(size_t)e * N_FEATURES + j];
    if (in.wstats) {
        const uint4* s = (const uint4*)(in.wstats + (size_t)e * WREC_WORDS);
        uint4* d = (uint4*)(out.wstats + (size_t)p * WREC_WORDS);
        for (int j = 0; j < WREC_WORDS / 4; ++j) d[j] = s[j];
        out.wsums[p] = in.wsums[e];
    }
}

// endpoints of every unique key -> node candidates (u32, labels < 2^32 here)
__global__ void k_endpoints(int64_t E, const uint64_t* __restrict__ uniq, int nb, uint32_t* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const uint64_t sk = uniq[e];
    out[2 * e] = (uint32_t)(sk >> nb);
    out[2 * e + 1] = (uint32_t)(sk & ((1ull << nb) - 1ull));
}

__global__ void k_u32_to_u64(int64_t n, const uint32_t* __restrict__ in, uint64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// lexicographic binary search of (u,v) queries in a sorted (u,v) table
__global__ void k_find_edges(const uint64_t* __restrict__ ge, int64_t n, const uint64_t* __restrict__ q,
                             int64_t m, int64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t qu = q[2 * i], qv = q[2 * i + 1];
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const uint64_t mu = ge[2 * mid], mv = ge[2 * mid + 1];
        if (mu < qu || (mu == qu && mv < qv)) lo = mid + 1;
        else hi = mid;
    }
    out[i] = (lo < n && ge[2 * lo] == qu && ge[2 * lo + 1] == qv) ? lo : -1;
}

hipError_t launch_pack_keys(int64_t n, const uint64_t* key, int nb, uint64_t* sk, uint32_t* idx, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, key, nb, sk, idx);
    return hipGetLastError();
}
hipError_t launch_pack_pairs(int64_t n, const uint64_t* uv, int nb, uint64_t* sk, uint32_t* idx, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, uv, nb, sk, idx);
    return hipGetLastError();
}
hipError_t launch_max_pairs(int64_t n, const uint64_t* uv, unsigned long long* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_max_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, uv, out);
    return hipGetLastError();
}
hipError_t launch_reduce(int64_t E, const uint64_t* uniq, const uint32_t* runs, const uint32_t* offs,
                         const uint32_t* perm, const RecordBuf& R, int wide, int stats, int nb, int need_adj,
                         int ignore_label, double scale, double offset, const ReduceOut& O, hipStream_t s) {
    if (E == 0) return hipSuccess;
    dim3 g((unsigned)((E + 255) / 256)), b(256);
    if (wide) {
        if (stats) hipLaunchKernelGGL((k_reduce_edges<true, true>), g, b, 0, s, E, uniq, runs, offs, perm, R, nb, need_adj, ignore_label, scale, offset, O);
        else hipLaunchKernelGGL((k_reduce_edges<true, false>), g, b, 0, s, E, uniq, runs, offs, perm, R, nb, need_adj, ignore_label, scale, offset, O);
    } else {
        if (stats) hipLaunchKernelGGL((k_reduce_edges<false, true>), g, b, 0, s, E, uniq, runs, offs, perm, R, nb, need_adj, ignore_label, scale, offset, O);
        else hipLaunchKernelGGL((k_reduce_edges<false, false>), g, b, 0, s, E, uniq, runs, offs, perm, R, nb, need_adj, ignore_label, scale, offset, O);
    }
    return hipGetLastError();
}
hipError_t launch_compact(int64_t E, const uint32_t* keep, const uint32_t* pos, const ReduceOut& in,
                          const ReduceOut& out, hipStream_t s) {
    if (E == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, E, keep, pos, in, out);
    return hipGetLastError();
}
hipError_t launch_endpoints(int64_t E, const uint64_t* uniq, int nb, uint32_t* out, hipStream_t s) {
    if (E == 0) return hipSuccess;
    hipLaunchKernelGGL(k_endpoints, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, E, uniq, nb, out);
    return hipGetLastError();
}
hipError_t launch_u32_to_u64(int64_t n, const uint32_t* in, uint64_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_u32_to_u64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, in, out);
    return hipGetLastError();
}
hipError_t launch_find_edges(const uint64_t* ge, int64_t n, const uint64_t* q, int64_t m, int64_t* out,
                             hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_find_edges, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, ge, n, q, m, out);
    return hipGetLastError();
}

}  // namespace ctg
