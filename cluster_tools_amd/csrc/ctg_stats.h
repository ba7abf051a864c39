// Per-edge statistics shared by the record reduction (ctg_reduce.hip) and the
// multi-GPU merge (ctg_mgpu.hip): the re-pivoting moment sums, vigra's
// StandardQuantiles over the 42-slot histogram, and the 10-column feature row
// (mean, var, min, q10, q25, q50, q75, q90, max, count --
// features/merge_edge_features.py:62-65, costs/probs_to_costs.py:205-207).
#pragma once
#include "ctg_internal.h"

namespace ctg {

// ---------------------------------------------------------------------------
// vigra computeStandardQuantiles as a single streaming walk over the bins
// ---------------------------------------------------------------------------
// The keypoints (mapped value, cumulative count) are generated in order; the
// last generated point is held back one step because vigra replaces the final
// keypoint by (mapped max, count) when there are no right outliers.  Each
// interior quantile q (0.1 .. 0.9) is interpolated on the first segment with
// cum(a) < q*count <= cum(b) and written straight to out[q] (global memory:
// no dynamically indexed register arrays, no scratch).
__host__ __device__ __forceinline__ double qv5(int i) {
    return i == 0 ? 0.1 : i == 1 ? 0.25 : i == 2 ? 0.5 : i == 3 ? 0.75 : 0.9;
}

// HL: a pointer to the NSLOTS bins, or the thread's register array itself
// (the bin walk is fully unrolled, so the array is never indexed dynamically
// and stays in registers - no LDS copy, no scratch)
template <typename HL>
__host__ __device__ __forceinline__ void vigra_quantiles(const HL& hl, double count, double vmin, double vmax, double scale,
                                                double offset, double* __restrict__ out) {
    const double inv = 1.0 / scale;
    int q = 0;
    double qc = count * qv5(0);
    bool have_prev = false, have_pend = false;
    double pkp = 0.0, pch = 0.0, kp_pend = 0.0, ch_pend = 0.0;
    auto consume = [&](double kp, double ch) {
        if (!have_prev) {
            pkp = kp;
            pch = ch;
            have_prev = true;
            return;
        }
        while (q < 5 && pch < qc && ch >= qc) {
            const double t = (qc - pch) / (ch - pch) * (kp - pkp);
            out[q] = inv * (t + pkp) + offset;
            ++q;
            qc = count * qv5(q);
        }
        pkp = kp;
        pch = ch;
    };
    auto gen = [&](double kp, double ch) {
        if (have_pend) consume(kp_pend, ch_pend);
        kp_pend = kp;
        ch_pend = ch;
        have_pend = true;
    };
    gen(scale * (vmin - offset), 0.0);
    const double left = (double)hl[0], right = (double)hl[NSLOTS - 1];
    if (left > 0.0) gen(0.0, left);
    double cum = left;
#pragma unroll
    for (int k = 0; k < NBINS; ++k) {
        const uint32_t hk = hl[k + 1];
        if (hk > 0) {
            if (kp_pend <= (double)k) gen((double)k, cum);
            cum += (double)hk;
            gen((double)(k + 1), cum);
        }
    }
    if (right > 0.0) {
        if (kp_pend != (double)NBINS) gen((double)NBINS, cum);
        gen(scale * (vmax - offset), count);
        consume(kp_pend, ch_pend);
    } else {
        consume(scale * (vmax - offset), count);  // replaces the last keypoint
    }
}

// The same quantiles without walking the keypoint list: the keypoints' counts
// are 0, left, then per non-empty bin k (cum before k, a duplicate point at
// x = k) and (cum after k, at x = k + 1), then for right outliers
// (cum, at x = 40) and (count, at x = mapped max); the last point is replaced
// by (mapped max, count) when there are no right outliers.  Quantile q
// interpolates on the segment ending at the first keypoint whose count
// reaches q*count, so one integer pass over the 40 bins finds, per q, the
// crossing bin and the counts on both sides (count >= q*count <=> count >=
// ceil(q*count) for integer counts), and the f64 arithmetic runs only at the
// five crossings.  Same segment endpoints and the same interpolation formula
// as vigra_quantiles, hence the same bits (tools/quantile_fuzz.hip).
template <typename HL>
__host__ __device__ __forceinline__ void vigra_quantiles_cross(const HL& hl, double count, double vmin, double vmax,
                                                               double scale, double offset,
                                                               double* __restrict__ out) {
    const double inv = 1.0 / scale;
    const double p0 = scale * (vmin - offset), pe = scale * (vmax - offset);
    const uint32_t left = hl[0], right = hl[NSLOTS - 1];
    uint32_t T[5], kq[5], cb[5], ca[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        T[q] = (uint32_t)ceil(count * qv5(q));
        kq[q] = 0;
        cb[q] = left;
        ca[q] = 0xFFFFFFFFu;
    }
    uint32_t cum = left;
#pragma unroll
    for (int k = 0; k < NBINS; ++k) {
        const uint32_t nc = cum + (uint32_t)hl[k + 1];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const bool below = nc < T[q];
            cb[q] = below ? nc : cb[q];
            kq[q] = below ? (uint32_t)(k + 1) : kq[q];
            ca[q] = (!below && nc < ca[q]) ? nc : ca[q];
        }
        cum = nc;
    }
    // cum = left + every bin = count - right
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const double qc = count * qv5(q);
        double pkp, pch, kp, ch;
        if (left >= T[q]) {                 // segment P0 -> (0, left)
            pkp = p0;
            pch = 0.0;
            const bool last = cum == left && right == 0;
            kp = last ? pe : 0.0;
            ch = last ? count : (double)left;
        } else if (kq[q] < (uint32_t)NBINS) {   // inside bin kq
            const bool first = cb[q] == left;   // no non-empty bin before kq
            pkp = (first && left == 0 && !(p0 <= (double)kq[q])) ? p0 : (double)kq[q];
            pch = (double)cb[q];
            const bool last = ca[q] == cum && right == 0;
            kp = last ? pe : (double)(kq[q] + 1);
            ch = last ? count : (double)ca[q];
        } else {                            // right-outlier segment (40, count - right) -> (mapped max, count)
            pkp = (double)NBINS;
            pch = (double)cum;
            kp = pe;
            ch = count;
        }
        const double t = (qc - pch) / (ch - pch) * (kp - pkp);
        out[q] = inv * (t + pkp) + offset;
    }
}

// Shifted sums of one edge about the pivot p0 of its first non-empty record:
// a record (n, S1, S2 about its own pivot p) is re-pivoted by d = p - p0,
//   sum(x - p0) = S1 + n d,   sum((x - p0)^2) = S2 + d (2 S1 + n d),
// where every term is bounded by the edge's sample spread (both pivots are
// samples of the edge), so the variance keeps its relative accuracy however
// large the samples are against their spread (Chan et al.'s pairwise update,
// in sums form).
// Branch-free: until a record with samples arrives (records without samples
// carry zero sums), p0 follows the latest pivot, so d = 0 for the first one.
struct Moments {
    uint32_t n = 0;
    double p0 = 0.0, S1 = 0.0, S2 = 0.0;
    __device__ __forceinline__ void add(uint32_t ni, double s1, double s2, uint32_t pbits) {
        const double p = (double)__uint_as_float(pbits);
        p0 = n == 0 ? p : p0;
        const double d = p - p0, nd = (double)ni * d;
        S1 += s1 + nd;
        S2 += s2 + d * (2.0 * s1 + nd);
        n += ni;
    }
};

// one narrow 128-byte record body at p: (S1, S2), the 24 record words, the pivot
__device__ __forceinline__ void add_narrow(const uint4* p, uint32_t (&h)[NSLOTS], uint32_t& cnt, uint32_t& flags,
                                           uint32_t& mn, uint32_t& mx, Moments& mo) {
    const double2 sw = *reinterpret_cast<const double2*>(p);
    uint32_t w[NREC_WORDS];
#pragma unroll
    for (int j = 0; j < NREC_WORDS / 4; ++j) {
        uint4 v = p[1 + j];
        w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
    }
    const uint32_t piv = p[7].x;
#pragma unroll
    for (int j = 0; j < HWORDS; ++j) {
        h[2 * j] += w[j] & 0xFFFFu;
        h[2 * j + 1] += w[j] >> 16;
    }
    const uint32_t n = w[21] & ~ADJ_FLAG;
    cnt += n;
    flags |= w[21] & ADJ_FLAG;
    mn = min(mn, w[22]);
    mx = max(mx, w[23]);
    mo.add(n, sw.x, sw.y, piv);
}

// An edge's combined statistics from its run e of sorted narrow records (the
// reduce's accumulation, k_reduce_edges): CTG_DEFER_STATS rows on demand.
__device__ __forceinline__ void edge_from_records(const DeferredStats& D, int64_t e, uint32_t (&h)[NSLOTS],
                                                  uint32_t& cnt, uint32_t& flags, uint32_t& mn, uint32_t& mx,
                                                  Moments& mo) {
    const uint32_t b = D.offs[e], n = D.runs[e];
    for (uint32_t r = b; r < b + n; ++r)
        add_narrow(reinterpret_cast<const uint4*>(D.hist + (size_t)D.perm(r) * NREC_STRIDE), h, cnt, flags, mn, mx,
                   mo);
}

// the mergeable wide statistics record of an edge (48 words: 42 slots,
// count | ADJ, ordered min, ordered max, pivot bits, pad); its (S1, S2) are
// mo.S1 / mo.S2 about the pivot mo.p0
__device__ __forceinline__ void wide_row(const uint32_t (&h)[NSLOTS], uint32_t cnt, uint32_t flags, uint32_t mn,
                                         uint32_t mx, const Moments& mo, uint32_t (&w)[WREC_WORDS]) {
#pragma unroll
    for (int j = 0; j < NSLOTS; ++j) w[j] = h[j];
    w[42] = cnt | (flags & ADJ_FLAG);
    w[43] = mn;
    w[44] = mx;
    w[WREC_PIV] = __float_as_uint((float)mo.p0);   // a sample: exact in f32
    w[46] = w[47] = 0;
}

// The 10 feature columns of one edge from its combined statistics (count, the
// 42-slot histogram, ordered min / max, shifted sums about mo.p0) as five
// column pairs in registers; an edge without samples gets a zero row.
// the 42 u16 slots of a histogram kept as 21 u16-pair words (the narrow
// record's own packing), read slot by slot (constant slots after unrolling)
struct PackedHist {
    const uint32_t* w;
    __device__ __forceinline__ uint32_t operator[](int k) const { return (w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu; }
};

template <typename HL>
__device__ __forceinline__ void finalize_vals(const HL& h, uint32_t cnt, uint32_t mn, uint32_t mx,
                                              const Moments& mo, double scale, double offset, double2 (&r)[5],
                                              bool quantiles = true) {
    if (cnt == 0) {
#pragma unroll
        for (int j = 0; j < N_FEATURES / 2; ++j) r[j] = make_double2(0.0, 0.0);
        return;
    }
    const double sum = mo.S1, sq = mo.S2;   // about the pivot mo.p0
    const double c = (double)cnt;
    const double dm = sum / c;
    const double mean = mo.p0 + dm;
    // population variance from the sums about the pivot (a sample of the
    // edge): the cancellation in S2 - S1 * (S1 / n) is bounded by the
    // samples' spread, not by their magnitude; an edge whose samples are
    // all equal (min == max) has variance exactly 0, as the two-pass rule
    double var = (sq - sum * dm) / c;
    if (var < 0.0 || mn == mx) var = 0.0;
    const double vmin = (double)ord2f(mn), vmax = (double)ord2f(mx);
    double qv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};   // registers (constant indices after unrolling)
    if (quantiles) vigra_quantiles_cross(h, c, vmin, vmax, scale, offset, qv);
    r[0] = make_double2(mean, var);
    r[1] = make_double2(vmin, qv[0]);
    r[2] = make_double2(qv[1], qv[2]);
    r[3] = make_double2(qv[3], qv[4]);
    r[4] = make_double2(vmax, c);
}

// the same row stored at o (16-B aligned: five 16-B stores)
__device__ __forceinline__ void finalize_row(const uint32_t (&h)[NSLOTS], uint32_t cnt, uint32_t mn, uint32_t mx,
                                             const Moments& mo, double scale, double offset, double* __restrict__ o,
                                             bool quantiles = true) {
    double2 r[5];
    finalize_vals(h, cnt, mn, mx, mo, scale, offset, r, quantiles);
    double2* o2 = reinterpret_cast<double2*>(o);
#pragma unroll
    for (int j = 0; j < N_FEATURES / 2; ++j) o2[j] = r[j];
}

// one wide statistics record (48 words: 42 slots, count|ADJ, ordered min,
// ordered max, pivot bits, pad) and its (S1, S2) into an edge's accumulators
__device__ __forceinline__ void add_wide(const uint32_t (&w)[WREC_WORDS], double s1, double s2,
                                         uint32_t (&h)[NSLOTS], uint32_t& cnt, uint32_t& flags, uint32_t& mn,
                                         uint32_t& mx, Moments& mo) {
#pragma unroll
    for (int j = 0; j < NSLOTS; ++j) h[j] += w[j];
    const uint32_t n = w[42] & ~ADJ_FLAG;
    cnt += n;
    flags |= w[42] & ADJ_FLAG;
    mn = min(mn, w[43]);
    mx = max(mx, w[44]);
    mo.add(n, s1, s2, w[WREC_PIV]);
}

}  // namespace ctg
