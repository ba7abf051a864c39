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
#include <algorithm>
#include <cstdlib>

#include "ctg_internal.h"
#include "ctg_stats.h"

namespace ctg {

__global__ void k_pack_keys(int64_t n, const uint64_t* __restrict__ key, int nb, uint64_t* __restrict__ sk,
                            uint32_t* __restrict__ idx) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = key[i];
    sk[i] = ((k >> 32) << nb) | (k & 0xFFFFFFFFull);
    idx[i] = (uint32_t)i;
}

// scan records: region r holds pre.off[r+1]-pre.off[r] keys from slot r*rcap;
// packed densely in region order, idx = the record's slot.  ib > 0: the slot
// rides in the low ib bits of the sort key itself ((key << ib) | slot, sorted
// on bits [ib, ib + 2nb)) and no separate index array is written.
__global__ void k_pack_regions(const uint64_t* __restrict__ key, int64_t rcap, RegionPrefix pre, int nb, int ib,
                               uint64_t* __restrict__ sk, uint32_t* __restrict__ idx) {
    const int r = blockIdx.y;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = pre.off[r];
    if (i >= pre.off[r + 1] - b) return;
    const uint64_t src = (uint64_t)r * (uint64_t)rcap + i;
    const uint64_t k = key[src];
    const uint64_t pk = ((k >> 32) << nb) | (k & 0xFFFFFFFFull);
    if (ib) {
        sk[b + i] = (pk << ib) | src;
    } else {
        sk[b + i] = pk;
        idx[b + i] = (uint32_t)src;
    }
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

template <bool WIDE>
__device__ __forceinline__ void load_record(const RecordBuf& R, uint32_t i, uint32_t (&h)[NSLOTS], uint32_t& cnt,
                                            uint32_t& flags, uint32_t& mn, uint32_t& mx, Moments& mo) {
    if constexpr (!WIDE) {
        add_narrow((const uint4*)(R.hist + (size_t)i * NREC_STRIDE), h, cnt, flags, mn, mx, mo);
    } else {
        const uint4* p = (const uint4*)(R.hist + (size_t)i * WREC_WORDS);
        uint32_t w[WREC_WORDS];
#pragma unroll
        for (int j = 0; j < WREC_WORDS / 4; ++j) {
            uint4 v = p[j];
            w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
        }
        const double2 s2 = R.sums[i];
        add_wide(w, s2.x, s2.y, h, cnt, flags, mn, mx, mo);
    }
}

// an edge's records: sorted positions [b, b + n); the next slot index is loaded
// while this record's body is in flight (one global latency per record, not two)
template <bool WIDE>
__device__ __forceinline__ void accumulate_run(const Perm& perm, const RecordBuf& R, uint32_t b, uint32_t n,
                                               uint32_t (&h)[NSLOTS], uint32_t& cnt, uint32_t& flags, uint32_t& mn,
                                               uint32_t& mx, Moments& mo) {
    uint32_t i = n ? perm(b) : 0u;
    for (uint32_t r = b; r < b + n; ++r) {
        const uint32_t nxt = r + 1 < b + n ? perm(r + 1) : 0u;
        load_record<WIDE>(R, i, h, cnt, flags, mn, mx, mo);
        i = nxt;
    }
}

// per-edge epilogue of the reduce: keep flag, mergeable stats row; the feature
// row is returned in registers (k_reduce_edges stages it for coalesced stores)
__device__ __forceinline__ void reduce_epilogue(int64_t e, uint64_t u, uint32_t (&h)[NSLOTS], uint32_t cnt,
                                                uint32_t flags, uint32_t mn, uint32_t mx, const Moments& mo,
                                                uint64_t umask, int need_adj, int ignore_label, double scale,
                                                double offset, const ReduceOut& O, double2 (&row)[5]) {
    const double sum = mo.S1, sq = mo.S2;   // about the pivot mo.p0
    // need_adj: 0 every record is an edge (boundary maps), 1 keep edges seen
    // on a nearest-neighbour face, 2 keep all and carry the flag (partials)
    if (need_adj == 0) flags |= ADJ_FLAG;
    const bool keep = (need_adj == 2 || (flags & ADJ_FLAG)) && !(ignore_label && (u & umask) == 0);
    if (O.keep) O.keep[e] = keep ? 1u : 0u;
    if (O.wstats) {
        uint4* p = (uint4*)(O.wstats + (size_t)e * WREC_WORDS);
        uint32_t w[WREC_WORDS];
        wide_row(h, cnt, flags, mn, mx, mo, w);
#pragma unroll
        for (int j = 0; j < WREC_WORDS / 4; ++j) p[j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
        O.wsums[e] = make_double2(sum, sq);
    }
    if (!O.feats) return;
#ifdef CTG_DIAG
    finalize_vals(h, cnt, mn, mx, mo, scale, offset, row, !(O.ablate & 1));
#else
    finalize_vals(h, cnt, mn, mx, mo, scale, offset, row);
#endif
}

// A wave's 64 feature rows (80 B each, lane = edge) go out through LDS: lane l
// writes its five 16-B column pairs to stage[5 l + j], then store k of the
// wave writes pairs [64 k, 64 k + 64) of the wave's contiguous 5120-B block --
// five fully coalesced stores instead of five 64-lane scatters at an 80-B
// stride.  Rows at or past `n` (the tail wave) are not stored.
__device__ __forceinline__ void store_rows_staged(double2* __restrict__ stage, const double2 (&row)[5],
                                                  double2* __restrict__ out, int64_t e0, int64_t n) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < N_FEATURES / 2; ++j) stage[5 * lane + j] = row[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const int64_t lim = (min(n - e0, (int64_t)64)) * (N_FEATURES / 2);
    double2* o = out + e0 * (N_FEATURES / 2);
#pragma unroll
    for (int k = 0; k < N_FEATURES / 2; ++k) {
        const int q = 64 * k + lane;
        if (q < lim) o[q] = stage[q];
    }
}

template <bool WIDE, bool STATS>
__global__ __launch_bounds__(256) void k_reduce_edges(int64_t E, const uint32_t* __restrict__ dE,
                                                      const uint64_t* __restrict__ uniq,
                                                      const uint32_t* __restrict__ runs,
                                                      const uint32_t* __restrict__ offs,
                                                      Perm perm, RecordBuf R, int nb, uint64_t umask,
                                                      int need_adj, int ignore_label, double scale, double offset,
                                                      ReduceOut O) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e == 0 && O.count_out) *O.count_out = *dE;
    const int64_t En = min(E, (int64_t)*dE);
    if constexpr (!STATS) {
        if (e >= En) return;
        const uint64_t sk = uniq[e];
        const uint64_t u = sk >> nb, v = sk & ((1ull << nb) - 1ull);
        O.edges[2 * e] = u;
        O.edges[2 * e + 1] = v;
        uint32_t flags = 0;
        if (need_adj) {
            const uint32_t b = offs[e], n = runs[e];
            for (uint32_t r = b; r < b + n; ++r) {
                const uint32_t i = perm(r);
                flags |= R.hist[(size_t)i * (WIDE ? WREC_WORDS : NREC_STRIDE) + (WIDE ? 42 : NREC_OFF + 21)] & ADJ_FLAG;
            }
        } else {
            flags = ADJ_FLAG;
        }
        if (O.keep) O.keep[e] = ((flags & ADJ_FLAG) || need_adj != 1) && !(ignore_label && (u & umask) == 0) ? 1u : 0u;
        return;
    } else {
        __shared__ double2 stage[256 / 64][64 * (N_FEATURES / 2)];
        const int64_t e0 = e - (threadIdx.x & 63);   // the wave's first edge
        if (e0 >= En) return;                       // (uniform per wave)
        double2 row[5];
        if (e < En) {
            const uint64_t sk = uniq[e];
            const uint64_t u = sk >> nb, v = sk & ((1ull << nb) - 1ull);
            O.edges[2 * e] = u;
            O.edges[2 * e + 1] = v;
            uint32_t flags = 0;
            uint32_t h[NSLOTS];
#pragma unroll
            for (int j = 0; j < NSLOTS; ++j) h[j] = 0;
            uint32_t cnt = 0, mn = ORD_POS_INF, mx = ORD_NEG_INF;
            Moments mo;
            const uint32_t b = offs[e], n = runs[e];
#ifdef CTG_DIAG   // diagnostic ablation (CTG_REDUCE_ABLATE, variant builds only)
            if (O.ablate & 2) {
                cnt = n;
                h[1] = n;
                mn = mx = 0x3F800000u ^ 0x80000000u;
                mo.add(n, 0.0, 0.0, 0u);
            } else
#endif
            {
                accumulate_run<WIDE>(perm, R, b, n, h, cnt, flags, mn, mx, mo);
            }
            reduce_epilogue(e, u, h, cnt, flags, mn, mx, mo, umask, need_adj, ignore_label, scale, offset, O, row);
        }
        if (!O.feats) return;
#ifdef CTG_DIAG
        if (O.ablate & 4) {   // keep the values live without the row stores
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < 5; ++j) t += row[j].x + row[j].y;
            if (t == -1.0) O.feats[0] = t;
            return;
        }
#endif
        store_rows_staged(stage[threadIdx.x >> 6], row, reinterpret_cast<double2*>(O.feats), e0, En);
    }
}

// one narrow record into a packed histogram: its 21 u16-pair words are added
// as they are (no slot can wrap while the edge's count stays below 2^16)
__device__ __forceinline__ void add_narrow_packed(const uint4* p, uint32_t (&hp)[HWORDS], uint32_t& cnt,
                                                  uint32_t& flags, uint32_t& mn, uint32_t& mx, Moments& mo) {
    const double2 sw = *reinterpret_cast<const double2*>(p);
    uint32_t w[NREC_WORDS];
#pragma unroll
    for (int j = 0; j < NREC_WORDS / 4; ++j) {
        const uint4 v = p[1 + j];
        w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
    }
    const uint32_t piv = p[7].x;
#pragma unroll
    for (int j = 0; j < HWORDS; ++j) hp[j] += w[j];
    const uint32_t n = w[21] & ~ADJ_FLAG;
    cnt += n;
    flags |= w[21] & ADJ_FLAG;
    mn = min(mn, w[22]);
    mx = max(mx, w[23]);
    mo.add(n, sw.x, sw.y, piv);
}

// Features-only reduce of narrow records (no mergeable statistics rows): the
// histogram stays packed, 21 u16-pair words instead of 42 slots (configs[4]
// reduce 5.35 -> 5.17 ms; squeezed to 96 VGPRs for a fifth wave per SIMD it
// spills and takes 7.05 ms).  An edge with more than 65535 samples (a slot
// could have wrapped) is listed in `heavy` and redone by k_reduce_heavy with
// the wide histogram; its row here is not used.
#ifndef CTG_REDUCE_MINB
#define CTG_REDUCE_MINB 4   // workgroups of 4 waves per CU (5 fits 96 VGPRs only by spilling: slower)
#endif
#ifndef CTG_REDUCE_PACKED
#define CTG_REDUCE_PACKED 1   // 0: features-only calls take k_reduce_edges too (variant builds)
#endif
__global__ __launch_bounds__(256, CTG_REDUCE_MINB) void k_reduce_packed(int64_t E, const uint32_t* __restrict__ dE,
                                                          const uint64_t* __restrict__ uniq,
                                                          const uint32_t* __restrict__ runs,
                                                          const uint32_t* __restrict__ offs, Perm perm, RecordBuf R,
                                                          int nb, uint64_t umask, int need_adj, int ignore_label,
                                                          double scale, double offset, ReduceOut O,
                                                          uint32_t* __restrict__ heavy, uint32_t* __restrict__ n_heavy) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e == 0 && O.count_out) *O.count_out = *dE;
    const int64_t En = min(E, (int64_t)*dE);
    __shared__ double2 stage[256 / 64][64 * (N_FEATURES / 2)];
    const int64_t e0 = e - (threadIdx.x & 63);
    if (e0 >= En) return;
    double2 row[5];
    if (e < En) {
        const uint64_t sk = uniq[e];
        const uint64_t u = sk >> nb, v = sk & ((1ull << nb) - 1ull);
        O.edges[2 * e] = u;
        O.edges[2 * e + 1] = v;
        uint32_t hp[HWORDS];
#pragma unroll
        for (int j = 0; j < HWORDS; ++j) hp[j] = 0;
        uint32_t cnt = 0, flags = 0, mn = ORD_POS_INF, mx = ORD_NEG_INF;
        Moments mo;
        const uint32_t b = offs[e], n = runs[e];
        uint32_t i = n ? perm(b) : 0u;
        for (uint32_t r = b; r < b + n; ++r) {
            const uint32_t nxt = r + 1 < b + n ? perm(r + 1) : 0u;
            add_narrow_packed(reinterpret_cast<const uint4*>(R.hist + (size_t)i * NREC_STRIDE), hp, cnt, flags, mn,
                              mx, mo);
            i = nxt;
        }
        if (cnt > 0xFFFFu) {
            heavy[atomicAdd(n_heavy, 1u)] = (uint32_t)e;
        } else {
            if (need_adj == 0) flags |= ADJ_FLAG;
            if (O.keep)
                O.keep[e] = ((need_adj == 2 || (flags & ADJ_FLAG)) && !(ignore_label && (u & umask) == 0)) ? 1u : 0u;
            finalize_vals(PackedHist{hp}, cnt, mn, mx, mo, scale, offset, row);
        }
    }
    store_rows_staged(stage[threadIdx.x >> 6], row, reinterpret_cast<double2*>(O.feats), e0, En);
}

// the listed edges of k_reduce_packed, with the wide histogram (grid-stride)
__global__ __launch_bounds__(256) void k_reduce_heavy(const uint32_t* __restrict__ heavy,
                                                      const uint32_t* __restrict__ n_heavy,
                                                      const uint32_t* __restrict__ runs,
                                                      const uint32_t* __restrict__ offs, Perm perm, RecordBuf R,
                                                      const uint64_t* __restrict__ uniq, int nb, uint64_t umask,
                                                      int need_adj, int ignore_label, double scale, double offset,
                                                      ReduceOut O) {
    const uint32_t nh = *n_heavy;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nh; k += gridDim.x * blockDim.x) {
        const int64_t e = heavy[k];
        uint32_t h[NSLOTS];
#pragma unroll
        for (int j = 0; j < NSLOTS; ++j) h[j] = 0;
        uint32_t cnt = 0, flags = 0, mn = ORD_POS_INF, mx = ORD_NEG_INF;
        Moments mo;
        accumulate_run<false>(perm, R, offs[e], runs[e], h, cnt, flags, mn, mx, mo);
        double2 row[5];
        reduce_epilogue(e, uniq[e] >> nb, h, cnt, flags, mn, mx, mo, umask, need_adj, ignore_label, scale, offset, O,
                        row);
        double2* o = reinterpret_cast<double2*>(O.feats + (size_t)e * N_FEATURES);
#pragma unroll
        for (int j = 0; j < N_FEATURES / 2; ++j) o[j] = row[j];
    }
}

// 16 threads per edge (one per 8-B feature / 16-B stats word): the copies of
// consecutive kept rows are coalesced
__global__ void k_compact(int64_t E, const uint32_t* __restrict__ dE, const uint32_t* __restrict__ keep,
                          const uint32_t* __restrict__ pos, ReduceOut in, ReduceOut out, uint32_t* __restrict__ kept) {
    const int64_t n = min(E, (int64_t)*dE);
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i0 == 0) *kept = n ? pos[n - 1] + keep[n - 1] : 0u;   // kept edge count
    for (int64_t i = i0; i < n * 16; i += (int64_t)gridDim.x * blockDim.x) {   // bound by the device count
        const int64_t e = i >> 4;
        const int j = (int)(i & 15);
        if (!keep[e]) continue;
        const size_t p = pos[e];
        if (j < 2) out.edges[2 * p + j] = in.edges[2 * e + j];
        if (in.feats && j < N_FEATURES) out.feats[p * N_FEATURES + j] = in.feats[(size_t)e * N_FEATURES + j];
        if (in.wstats && j < WREC_WORDS / 4) {
            reinterpret_cast<uint4*>(out.wstats)[p * (WREC_WORDS / 4) + j] =
                reinterpret_cast<const uint4*>(in.wstats)[(size_t)e * (WREC_WORDS / 4) + j];
            if (j == 0) out.wsums[p] = in.wsums[e];
        }
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

// one thread per label of the bitmap: a set bit's rank among the set bits
// before it is its node position, so consecutive nodes are stored by
// consecutive lanes (a per-word expansion loop stores 32 scattered u64 per lane)
__global__ void k_bits_to_nodes(int64_t W, const uint32_t* __restrict__ bits, const uint32_t* __restrict__ off,
                                uint64_t* __restrict__ nodes, uint32_t* __restrict__ dN) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * 32) return;
    const int64_t w = i >> 5;
    const uint32_t b = bits[w], k = (uint32_t)(i & 31);
    if (i == W * 32 - 1) *dN = off[w] + __popc(b);   // node count
    if ((b >> k) & 1u) nodes[off[w] + __popc(b & ((1u << k) - 1u))] = (uint64_t)i;
}

// Nodes as a bitmap over [0, max label], built per chunk of the sorted key
// table in LDS (u is sorted, so only run heads mark it; every v marks its
// bit).  A chunk of
// NODE_CHUNK consecutive edges covers a narrow u range and, for spatially
// ordered label ids, a narrow v window above it: the workgroup marks its
// nodes in an LDS window and ORs the non-zero words into the global bitmap
// with coalesced atomics (one 256-B wave-instruction per 64 words), instead of
// one scattered global atomic per edge.  A chunk whose v window does not fit
// the LDS bitmap falls back to per-edge global atomics.
constexpr int NODE_CHUNK = 2048;
constexpr int NODE_WORDS = 8192;   // 32 KB LDS window = 262144 labels

__global__ __launch_bounds__(256) void k_mark_nodes_win(int64_t E, const uint32_t* __restrict__ dE,
                                                        const uint64_t* __restrict__ uniq, int nb,
                                                        uint32_t* __restrict__ bits) {
    constexpr int PER = NODE_CHUNK / 256;
    __shared__ uint32_t bm[NODE_WORDS];
    __shared__ uint32_t red[4];
    const int tid = threadIdx.x, lane = tid & 63;
    E = min(E, (int64_t)*dE);
    const int64_t e0 = (int64_t)blockIdx.x * NODE_CHUNK;
    if (e0 >= E) return;
    const int64_t e1 = min(E, e0 + NODE_CHUNK);
    const uint64_t vmask = (1ull << nb) - 1ull;
    // each key is read once: kept in registers for the window bound and the marks
    uint64_t sk[PER];
    uint32_t vmax = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int64_t e = e0 + tid + 256 * k;
        sk[k] = e < e1 ? uniq[e] : 0ull;
        vmax = max(vmax, (uint32_t)(sk[k] & vmask));
    }
    const uint32_t base = (uint32_t)(uniq[e0] >> nb) & ~31u;   // v > u >= u(e0)
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if (lane == 0) red[tid >> 6] = vmax;
    __syncthreads();
    vmax = max(max(red[0], red[1]), max(red[2], red[3]));
    const uint32_t nw = ((vmax - base) >> 5) + 1;
    const bool win = nw <= (uint32_t)NODE_WORDS;
    if (win) {   // clear only the window this chunk uses
        for (uint32_t w = tid; w < nw; w += 256) bm[w] = 0u;
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int64_t e = e0 + tid + 256 * k;
        const uint32_t u = (uint32_t)(sk[k] >> nb), v = (uint32_t)(sk[k] & vmask);
        // u is sorted: only a run head marks it (the previous key is the
        // previous lane's, or a reload for the wave's first lane)
        uint32_t up = (uint32_t)__shfl_up((int)u, 1, 64);
        // (only lanes holding an edge: past e1 the index can leave uniq's
        // allocation, which is sized by this call's records)
        if (lane == 0 && e < e1) up = e > 0 ? (uint32_t)(uniq[e - 1] >> nb) : ~u;
        if (e < e1) {
            if (win) {
                if (up != u) atomicOr(&bm[(u - base) >> 5], 1u << ((u - base) & 31));
                atomicOr(&bm[(v - base) >> 5], 1u << ((v - base) & 31));
            } else {
                if (up != u) atomicOr(&bits[u >> 5], 1u << (u & 31));
                atomicOr(&bits[v >> 5], 1u << (v & 31));
            }
        }
    }
    if (!win) return;
    __syncthreads();
    for (uint32_t w = tid; w < nw; w += 256) {
        const uint32_t b = bm[w];
        if (b) atomicOr(&bits[(base >> 5) + w], b);
    }
}

hipError_t launch_mark_nodes(int64_t E, const uint32_t* dE, const uint64_t* uniq, int nb, uint32_t* bits,
                             hipStream_t s) {
    if (E == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mark_nodes_win, dim3((unsigned)((E + NODE_CHUNK - 1) / NODE_CHUNK)), dim3(256), 0, s,
                           E, dE, uniq, nb, bits);
    return hipGetLastError();
}
hipError_t launch_bits_to_nodes(int64_t W, const uint32_t* bits, const uint32_t* off, uint64_t* nodes, uint32_t* dN,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_bits_to_nodes, dim3((unsigned)((W * 32 + 255) / 256)), dim3(256), 0, s, W, bits, off, nodes, dN);
    return hipGetLastError();
}

__global__ void k_u32_to_u64(int64_t n, const uint32_t* __restrict__ in, uint64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// owner-blocked Bloom filter of the RAG edges (labels < 2^32; ctg_internal.h):
// u -> v into u's block and v -> u into v's block, the long-range affinity
// prefilter of the face scan
__global__ void k_build_bloom(const uint64_t* __restrict__ edges, int64_t E, unsigned long long* words,
                              uint32_t block_mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const uint32_t u = (uint32_t)edges[2 * i], v = (uint32_t)edges[2 * i + 1];
    const uint64_t hu = bloom_hash(((uint64_t)u << 32) | v), hv = bloom_hash(((uint64_t)v << 32) | u);
    atomicOr(&words[bloom_word(bloom_block(u, block_mask), hu)], (unsigned long long)bloom_bits(hu));
    atomicOr(&words[bloom_word(bloom_block(v, block_mask), hv)], (unsigned long long)bloom_bits(hv));
}

hipError_t launch_build_bloom(const uint64_t* edges, int64_t E, unsigned long long* words, uint32_t block_mask,
                              hipStream_t s) {
    hipError_t e = hipMemsetAsync(words, 0, ((size_t)block_mask + 1) * 64, s);
    if (e != hipSuccess || E == 0) return e;
    hipLaunchKernelGGL(k_build_bloom, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, edges, E, words,
                       block_mask);
    return hipGetLastError();
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

// labels >= 2^32: dense relabelling through the sorted unique label table U
// (monotone, so sorted dense edges stay sorted after mapping back)
template <typename OutT>
__global__ void k_remap_dense(const uint64_t* __restrict__ L, int64_t V, const uint64_t* __restrict__ U, int64_t n,
                              OutT* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t x = L[i];
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (U[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        out[i] = (OutT)lo;
    }
}

__global__ void k_gather_labels(const uint64_t* __restrict__ U, uint64_t* __restrict__ x, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = U[x[i]];
}

hipError_t launch_remap_dense(const uint64_t* L, int64_t V, const uint64_t* U, int64_t n, uint32_t* out,
                              hipStream_t s) {
    if (V == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((V + 255) / 256, 256 * 64);
    hipLaunchKernelGGL(k_remap_dense<uint32_t>, dim3((unsigned)blocks), dim3(256), 0, s, L, V, U, n, out);
    return hipGetLastError();
}

hipError_t launch_remap_dense64(const uint64_t* L, int64_t V, const uint64_t* U, int64_t n, uint64_t* out,
                                hipStream_t s) {
    if (V == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((V + 255) / 256, 256 * 64);
    hipLaunchKernelGGL(k_remap_dense<uint64_t>, dim3((unsigned)blocks), dim3(256), 0, s, L, V, U, n, out);
    return hipGetLastError();
}

hipError_t launch_gather_labels(const uint64_t* U, uint64_t* x, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_labels, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U, x, n);
    return hipGetLastError();
}

// Reference-layout feature rows (10 float64 columns, no histograms) of the
// same edge from several blocks -> one row (mergeFeatureBlocks without the
// statistics companion, features/merge_edge_features.py:141-147).  The rows
// are sorted by edge (key = id - begin); the head of every run combines its
// rows in sorted order: count sum, count-weighted mean, exact pooled variance
// sum(c * (var + (mean_i - mean)^2)) / N, min / max over non-empty rows and
// count-weighted quantiles.
__global__ void k_merge_feature_rows(int64_t n, const uint32_t* __restrict__ key, const uint32_t* __restrict__ idx,
                                     const double* __restrict__ rows, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = key[i];
    if (i > 0 && key[i - 1] == k) return;
    int64_t j1 = i;
    while (j1 < n && key[j1] == k) ++j1;
    double N = 0.0, S = 0.0, q[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    double mn = INFINITY, mx = -INFINITY;
    int n_rows = 0;
    const double* only = nullptr;
    for (int64_t j = i; j < j1; ++j) {
        const double* r = rows + (size_t)idx[j] * N_FEATURES;
        const double c = r[9];
        if (!(c > 0.0)) continue;
        ++n_rows;
        only = r;
        N += c;
        S += c * r[0];
        mn = fmin(mn, r[2]);
        mx = fmax(mx, r[8]);
#pragma unroll
        for (int t = 0; t < 5; ++t) q[t] += c * r[3 + t];
    }
    double* o = out + (size_t)k * N_FEATURES;
    if (N == 0.0) return;   // rows stay zero (pre-filled)
    if (n_rows == 1) {      // one non-empty block: its row is the edge's row, bit for bit
        for (int t = 0; t < N_FEATURES; ++t) o[t] = only[t];
        return;
    }
    const double mean = S / N;
    double M2 = 0.0;
    for (int64_t j = i; j < j1; ++j) {
        const double* r = rows + (size_t)idx[j] * N_FEATURES;
        const double c = r[9];
        if (!(c > 0.0)) continue;
        const double d = r[0] - mean;
        M2 += c * (r[1] + d * d);
    }
    o[0] = mean;
    o[1] = M2 / N;
    o[2] = mn;
#pragma unroll
    for (int t = 0; t < 5; ++t) o[3 + t] = q[t] / N;
    o[8] = mx;
    o[9] = N;
}

// ids outside [begin, end) raise *bad (the host reports them)
__global__ void k_row_keys(int64_t n, const uint64_t* __restrict__ ids, uint64_t begin, uint64_t end,
                           uint32_t* __restrict__ key, uint32_t* __restrict__ idx, uint32_t* __restrict__ bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t id = ids[i];
    const bool ok = id >= begin && id < end;
    if (!ok) atomicOr(bad, 1u);
    key[i] = ok ? (uint32_t)(id - begin) : 0u;
    idx[i] = (uint32_t)i;
}

hipError_t launch_row_keys(int64_t n, const uint64_t* ids, uint64_t begin, uint64_t end, uint32_t* key,
                           uint32_t* idx, uint32_t* bad, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_row_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, ids, begin, end, key, idx,
                       bad);
    return hipGetLastError();
}

hipError_t launch_merge_feature_rows(int64_t n, const uint32_t* key, const uint32_t* idx, const double* rows,
                                     double* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_merge_feature_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, key, idx, rows,
                       out);
    return hipGetLastError();
}

// batched blocks: row range of every block in a table sorted by its tagged
// first column (tag = block << shift), then the tag bits are cleared
__global__ void k_block_bounds(int64_t n, const uint64_t* __restrict__ col, int stride, int n_blocks, int shift,
                               int64_t* __restrict__ bounds) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > n_blocks) return;
    const uint64_t key = (uint64_t)b << shift;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (col[mid * stride] < key) lo = mid + 1;
        else hi = mid;
    }
    bounds[b] = b == n_blocks ? n : lo;
}

__global__ void k_clear_bits(int64_t n, uint64_t* __restrict__ col, int stride, uint64_t mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) col[i * stride] &= mask;
}

hipError_t launch_block_bounds(int64_t n, const uint64_t* col, int stride, int n_blocks, int shift, int64_t* bounds,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_block_bounds, dim3((unsigned)((n_blocks + 1 + 255) / 256)), dim3(256), 0, s, n, col, stride,
                       n_blocks, shift, bounds);
    return hipGetLastError();
}

hipError_t launch_clear_bits(int64_t n, uint64_t* col, int stride, uint64_t mask, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_clear_bits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, col, stride, mask);
    return hipGetLastError();
}

hipError_t launch_pack_keys(int64_t n, const uint64_t* key, int nb, uint64_t* sk, uint32_t* idx, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, key, nb, sk, idx);
    return hipGetLastError();
}
hipError_t launch_pack_regions(const uint64_t* key, int64_t rcap, const RegionPrefix& pre, int nb, int ib,
                               uint64_t* sk, uint32_t* idx, hipStream_t s) {
    uint32_t mx = 0;
    for (int r = 0; r < NREG; ++r) mx = std::max(mx, pre.off[r + 1] - pre.off[r]);
    if (mx == 0) return hipSuccess;
    if ((uint64_t)rcap * NREG > (1ull << 32)) return hipErrorInvalidValue;   // slots index as u32
    hipLaunchKernelGGL(k_pack_regions, dim3((mx + 255) / 256, NREG), dim3(256), 0, s, key, rcap, pre, nb, ib, sk,
                       idx);
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
hipError_t launch_reduce(int64_t E, const uint32_t* dE, const uint64_t* uniq, const uint32_t* runs,
                         const uint32_t* offs, const uint32_t* perm32, const uint64_t* perm64, int ib,
                         const RecordBuf& R, int wide, int stats, int nb, uint64_t umask, int need_adj,
                         int ignore_label, double scale, double offset, const ReduceOut& O, hipStream_t s,
                         uint32_t* heavy, uint32_t* n_heavy) {
    if (E == 0) return hipSuccess;
    const Perm perm{perm32, perm64, ib};
    dim3 g((unsigned)((E + 255) / 256)), b(256);
    if (CTG_REDUCE_PACKED && !wide && stats && O.feats && !O.wstats && !O.ablate && heavy && n_heavy) {
        // features only: the packed-histogram kernel, then its heavy edges
        hipError_t e = hipMemsetAsync(n_heavy, 0, 4, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_reduce_packed, g, b, 0, s, E, dE, uniq, runs, offs, perm, R, nb, umask, need_adj,
                           ignore_label, scale, offset, O, heavy, n_heavy);
        hipLaunchKernelGGL(k_reduce_heavy, dim3((unsigned)std::min<int64_t>((E + 255) / 256, 1024)), b, 0, s, heavy,
                           n_heavy, runs, offs, perm, R, uniq, nb, umask, need_adj, ignore_label, scale, offset, O);
        return hipGetLastError();
    }
    if (wide) {
        if (stats) hipLaunchKernelGGL((k_reduce_edges<true, true>), g, b, 0, s, E, dE, uniq, runs, offs, perm, R, nb, umask, need_adj, ignore_label, scale, offset, O);
        else hipLaunchKernelGGL((k_reduce_edges<true, false>), g, b, 0, s, E, dE, uniq, runs, offs, perm, R, nb, umask, need_adj, ignore_label, scale, offset, O);
    } else {
        if (stats) hipLaunchKernelGGL((k_reduce_edges<false, true>), g, b, 0, s, E, dE, uniq, runs, offs, perm, R, nb, umask, need_adj, ignore_label, scale, offset, O);
        else hipLaunchKernelGGL((k_reduce_edges<false, false>), g, b, 0, s, E, dE, uniq, runs, offs, perm, R, nb, umask, need_adj, ignore_label, scale, offset, O);
    }
    return hipGetLastError();
}
hipError_t launch_compact(int64_t E, const uint32_t* dE, const uint32_t* keep, const uint32_t* pos,
                          const ReduceOut& in, const ReduceOut& out, uint32_t* dkept, hipStream_t s) {
    if (E == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3((unsigned)std::min<int64_t>((E * 16 + 255) / 256, 16384)), dim3(256), 0, s, E, dE, keep, pos, in, out,
                       dkept);
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
