// Multi-GPU combine of the z-slab partial tables: the device
// side of one rank's exchange step, between RCCL collectives that the host
// layer (cluster_tools_amd/dist.py) issues over torch.distributed.
//
// The reference combines per-block results in two tasks --
// graph/merge_sub_graphs.py:130-135 (ndist.mergeSubgraphs) and
// features/merge_edge_features.py:141-147 (ndist.mergeFeatureBlocks) -- by
// re-reading every block's chunks.  Here every rank holds the sorted partial
// table of its slab (edges, 10 features and the mergeable wide statistics of
// each edge, CTG_KEEP_STATS) and the global table is range-partitioned by the
// lower label u:
//
//   ctg_mgpu_sample  an evenly spaced sample of this rank's u column
//                    (all-gathered by the host)
//   ctg_mgpu_split   range splitters from the gathered samples (exact integer
//                    weights, so every rank derives the same ones) and the
//                    rows / node ids this rank sends to every rank
//                    (all-gathered by the host: every rank then knows every
//                    segment size of the all_to_all)
//   ctg_mgpu_pack    the rows and node ids for the other ranks, one segment
//                    per destination, in one launch
//   ctg_mgpu_merge   after the all_to_all: the received rows are merged with
//                    this rank's own range -- stats of equal keys combined
//                    (Chan's rule on the shifted sums, histograms added),
//                    features re-finalised only for those keys, every other
//                    own row kept as the local call computed it.  With nothing
//                    received the own range IS the shard (no kernel, no copy).
#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "ctg_internal.h"
#include "ctg_stats.h"

namespace ctg {

constexpr int MS = CTG_MGPU_SAMPLES;
constexpr int ROW = CTG_MGPU_ROW_WORDS;       // int64 words per exchanged row
constexpr uint64_t SIGN = 1ull << 63;         // u ^ SIGN: unsigned order as int64 order

// ---------------------------------------------------------------------------
// sample and split
// ---------------------------------------------------------------------------
__global__ void k_mgpu_sample(const uint64_t* __restrict__ edges, int64_t E, int64_t* __restrict__ meta) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < MS) meta[i] = E ? (int64_t)(edges[2 * ((int64_t)i * E / MS)] ^ SIGN) : 0;
    if (i == MS) meta[MS] = E;
}

__device__ __forceinline__ int lower_i64(const int64_t* a, int n, int64_t v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int upper_i64(const int64_t* a, int n, int64_t v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Splitters: sample j of rank r (value v, sorted per rank) stands for
// count_r / MS rows.  In the total order (v, r, j) its cumulative weight,
// scaled by MS to integers, is CW = sum_r' count_r' * c_r', with c_r' the
// samples of rank r' at or before it (r' < r: <= v; r' > r: < v; r' = r: j+1).
// Splitter k (1..W-1) is the v of the one sample whose weight interval
// (CW - count_r, CW] holds total * MS * k / W -- exact integer arithmetic, so
// every rank finds the same splitters from the same gathered samples, and no
// atomics are needed (the crossing sample writes its splitter alone).
__global__ void k_mgpu_splitters(const int64_t* __restrict__ meta_all, int world, uint64_t* __restrict__ spl) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= world * MS) return;
    const int r = e / MS, j = e % MS;
    const uint64_t cnt_r = (uint64_t)meta_all[(int64_t)r * (MS + 1) + MS];
    if (cnt_r == 0) return;
    const int64_t v = meta_all[(int64_t)r * (MS + 1) + j];
    uint64_t cw = 0, total = 0;
    for (int q = 0; q < world; ++q) {
        const int64_t* row = meta_all + (int64_t)q * (MS + 1);
        const uint64_t cq = (uint64_t)row[MS];
        total += cq;
        if (cq == 0) continue;
        const int c = q < r ? upper_i64(row, MS, v) : q > r ? lower_i64(row, MS, v) : j + 1;
        cw += cq * (uint64_t)c;
    }
    const uint64_t lo = (cw - cnt_r) * (uint64_t)world, hi = cw * (uint64_t)world;
    for (int k = 1; k < world; ++k) {
        const uint64_t t = total * (uint64_t)MS * (uint64_t)k;
        if (lo < t && t <= hi) spl[k - 1] = (uint64_t)v ^ SIGN;
    }
}

// first row of a sorted (u,v) table (stride words per row) whose u >= x
__device__ __forceinline__ int64_t lower_u(const uint64_t* col, int stride, int64_t n, uint64_t x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (col[mid * stride] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// rows / node ids of this rank that fall in every rank's u range
// [spl[d-1], spl[d]) -> counts[2d], counts[2d+1]
__global__ void k_mgpu_bounds(const uint64_t* __restrict__ edges, int64_t E, const uint64_t* __restrict__ nodes,
                              int64_t N, const uint64_t* __restrict__ spl, int world, int64_t* __restrict__ counts) {
    const int d = threadIdx.x;
    if (d >= world) return;
    const int64_t e0 = d == 0 ? 0 : lower_u(edges, 2, E, spl[d - 1]);
    const int64_t e1 = d == world - 1 ? E : lower_u(edges, 2, E, spl[d]);
    const int64_t n0 = d == 0 ? 0 : lower_u(nodes, 1, N, spl[d - 1]);
    const int64_t n1 = d == world - 1 ? N : lower_u(nodes, 1, N, spl[d]);
    counts[2 * d] = max(e1 - e0, (int64_t)0);
    counts[2 * d + 1] = max(n1 - n0, (int64_t)0);
}

// ---------------------------------------------------------------------------
// pack: one segment per destination, rows then node ids
// ---------------------------------------------------------------------------
struct Segs {   // destination segments of the send buffer (host-computed)
    int64_t e_start[CTG_MGPU_MAX_WORLD], e_cnt[CTG_MGPU_MAX_WORLD];
    int64_t n_start[CTG_MGPU_MAX_WORLD], n_cnt[CTG_MGPU_MAX_WORLD];
    int64_t w_off[CTG_MGPU_MAX_WORLD + 1];   // word offset of segment i
    int n;
};

// a row = (u, v, S1 bits, S2 bits, the 48-word wide record as 24 u64)
__global__ void k_mgpu_pack(Segs S, const uint64_t* __restrict__ edges, const double2* __restrict__ sums,
                            const uint64_t* __restrict__ wide64, const uint64_t* __restrict__ nodes,
                            uint64_t* __restrict__ out) {
    const int64_t total = S.w_off[S.n];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        int s = 0;
        while (s + 1 < S.n && S.w_off[s + 1] <= i) ++s;
        const int64_t off = i - S.w_off[s];
        uint64_t val;
        if (off < S.e_cnt[s] * ROW) {
            const int64_t r = S.e_start[s] + off / ROW;
            const int w = (int)(off % ROW);
            if (w < 2) val = edges[2 * r + w];
            else if (!wide64) continue;   // CTG_DEFER_STATS: k_mgpu_pack_deferred writes the statistics
            else if (w < 4) {
                const double2 sm = sums[r];
                val = (uint64_t)__double_as_longlong(w == 2 ? sm.x : sm.y);
            } else {
                val = wide64[r * (WREC_WORDS / 2) + (w - 4)];
            }
        } else {
            val = nodes[S.n_start[s] + (off - S.e_cnt[s] * ROW)];
        }
        out[i] = val;
    }
}

// CTG_DEFER_STATS: one thread per row to send -- its statistics rebuilt from
// its records (words 2..27 of the row; k_mgpu_pack writes the key words).
// Boundary maps only: every key is an edge (the reduce's need_adj 0 sets ADJ).
__global__ __launch_bounds__(256) void k_mgpu_pack_deferred(Segs S, DeferredStats D, uint64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int s = 0;
    int64_t before = 0;
    while (s < S.n && i >= before + S.e_cnt[s]) before += S.e_cnt[s++];
    if (s >= S.n) return;
    const int64_t a = i - before, r = S.e_start[s] + a;
    uint32_t h[NSLOTS];
#pragma unroll
    for (int j = 0; j < NSLOTS; ++j) h[j] = 0;
    uint32_t cnt = 0, flags = ADJ_FLAG, mn = ORD_POS_INF, mx = ORD_NEG_INF;
    Moments mo;
    edge_from_records(D, r, h, cnt, flags, mn, mx, mo);
    uint32_t w[WREC_WORDS];
    wide_row(h, cnt, flags, mn, mx, mo, w);
    uint64_t* o = out + S.w_off[s] + a * ROW;
    o[2] = (uint64_t)__double_as_longlong(mo.S1);
    o[3] = (uint64_t)__double_as_longlong(mo.S2);
#pragma unroll
    for (int t = 0; t < WREC_WORDS / 2; ++t) o[4 + t] = (uint64_t)w[2 * t] | ((uint64_t)w[2 * t + 1] << 32);
}

// ---------------------------------------------------------------------------
// merge
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool key_lt(uint64_t au, uint64_t av, uint64_t bu, uint64_t bv) {
    return au < bu || (au == bu && av < bv);
}

struct RecvSegs {   // received segments (sources in rank order, own skipped)
    int64_t row0[CTG_MGPU_MAX_WORLD + 1];   // first global received row of segment i
    int64_t w_off[CTG_MGPU_MAX_WORLD];      // word offset of segment i in the receive buffer
    int n;
};

__device__ __forceinline__ const uint64_t* recv_row(const RecvSegs& S, const uint64_t* recv, int s, int64_t a) {
    return recv + S.w_off[s] + a * ROW;
}

// rows of segment q with key < (u,v) (lower) or <= (upper)
__device__ __forceinline__ int64_t seg_rank(const RecvSegs& S, const uint64_t* recv, int q, uint64_t u, uint64_t v,
                                            bool upper) {
    int64_t lo = 0, hi = S.row0[q + 1] - S.row0[q];
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const uint64_t* p = recv_row(S, recv, q, mid);
        const bool before = upper ? !key_lt(u, v, p[0], p[1]) : key_lt(p[0], p[1], u, v);
        if (before) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Received rows in one sorted order without a sort: every source's segment is
// sorted, so row a of segment s lands at a + (rows of the other segments that
// precede it; ties go to the lower source).  order[pos] = global row index.
__global__ void k_mgpu_order(RecvSegs S, const uint64_t* __restrict__ recv, uint32_t* __restrict__ order,
                             uint64_t* __restrict__ skeys) {
    const int64_t M = S.row0[S.n];
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    int s = 0;
    while (s + 1 < S.n && S.row0[s + 1] <= j) ++s;
    const int64_t a = j - S.row0[s];
    const uint64_t* p = recv_row(S, recv, s, a);
    const uint64_t u = p[0], v = p[1];
    int64_t pos = a;
    for (int q = 0; q < S.n; ++q)
        if (q != s) pos += seg_rank(S, recv, q, u, v, q < s);
    order[pos] = (uint32_t)j;
    skeys[2 * pos] = u;
    skeys[2 * pos + 1] = v;
}

__global__ void k_mgpu_heads(int64_t M, const uint64_t* __restrict__ skeys, uint32_t* __restrict__ head) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= M) return;
    head[p] = (p == 0 || skeys[2 * p] != skeys[2 * p - 2] || skeys[2 * p + 1] != skeys[2 * p - 1]) ? 1u : 0u;
}

// first sorted position of every run (rid = exclusive scan of the heads); K
// (the unique received keys) in *nK
__global__ void k_mgpu_runs(int64_t M, const uint32_t* __restrict__ head, const uint32_t* __restrict__ rid,
                            uint32_t* __restrict__ run0, uint32_t* __restrict__ nK) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= M) return;
    if (head[p]) run0[rid[p]] = (uint32_t)p;
    if (p == M - 1) {
        const uint32_t K = rid[p] + head[p];
        *nK = K;
        run0[K] = (uint32_t)M;
    }
}

// position of (u,v) in a sorted (u,v) table of n rows: lower bound
__device__ __forceinline__ int64_t lower_uv(const uint64_t* t, int64_t n, uint64_t u, uint64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (key_lt(t[2 * mid], t[2 * mid + 1], u, v)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

struct MergeIO {
    // own range of the local table (rows [0, n_own) after offsetting)
    const uint64_t* own_edges;
    const double* own_feats;
    const uint32_t* own_wide;
    const double2* own_sums;
    DeferredStats defer;  // on: own rows' statistics from the records (own row i = run own_row0 + i)
    int64_t own_row0;
    int64_t n_own;
    // received rows, sorted order and runs
    const uint64_t* recv;
    const uint32_t* order;
    const uint64_t* skeys;
    const uint32_t* run0;
    const uint32_t* nK;
    // per unique received key k
    uint64_t* mkeys;      // (K,2)
    double* mfeats;       // (K,10)
    uint32_t* mkeep;      // keep (ADJ proved, or every key for boundary maps)
    uint32_t* mnew;       // key absent from the own range
    int64_t* mins;        // own rows with a smaller key
    uint32_t* touched;    // (n_own) 1 + k of the received key that matches own row i, 0 none
    int partial_adj;      // keys need the ADJ bit (affinity partials)
    double scale, offset;
};

// One thread per unique received key: its own-range match (binary search),
// the combined statistics of the own row and every received row of the key,
// and the re-finalised feature row.
__global__ __launch_bounds__(256) void k_mgpu_combine(RecvSegs S, MergeIO io) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= (int64_t)*io.nK) return;
    const uint32_t p0 = io.run0[k], p1 = io.run0[k + 1];
    const uint64_t u = io.skeys[2 * (int64_t)p0], v = io.skeys[2 * (int64_t)p0 + 1];
    const int64_t ins = lower_uv(io.own_edges, io.n_own, u, v);
    const bool found = ins < io.n_own && io.own_edges[2 * ins] == u && io.own_edges[2 * ins + 1] == v;
    uint32_t h[NSLOTS];
#pragma unroll
    for (int j = 0; j < NSLOTS; ++j) h[j] = 0;
    uint32_t cnt = 0, flags = 0, mn = ORD_POS_INF, mx = ORD_NEG_INF;
    Moments mo;
    uint32_t w[WREC_WORDS];
    if (found && io.defer.on) {   // the own row's records (boundary maps: every key an edge)
        flags = ADJ_FLAG;
        edge_from_records(io.defer, io.own_row0 + ins, h, cnt, flags, mn, mx, mo);
        io.touched[ins] = (uint32_t)k + 1u;
    } else if (found) {
        const uint4* q = reinterpret_cast<const uint4*>(io.own_wide + ins * WREC_WORDS);
#pragma unroll
        for (int j = 0; j < WREC_WORDS / 4; ++j) {
            const uint4 x = q[j];
            w[4 * j] = x.x; w[4 * j + 1] = x.y; w[4 * j + 2] = x.z; w[4 * j + 3] = x.w;
        }
        const double2 sm = io.own_sums[ins];
        add_wide(w, sm.x, sm.y, h, cnt, flags, mn, mx, mo);
        io.touched[ins] = (uint32_t)k + 1u;
    }
    for (uint32_t p = p0; p < p1; ++p) {
        const uint32_t j = io.order[p];
        int s = 0;
        while (s + 1 < S.n && S.row0[s + 1] <= (int64_t)j) ++s;
        const uint64_t* r = recv_row(S, io.recv, s, (int64_t)j - S.row0[s]);
#pragma unroll
        for (int t = 0; t < WREC_WORDS / 2; ++t) {
            const uint64_t x = r[4 + t];
            w[2 * t] = (uint32_t)x;
            w[2 * t + 1] = (uint32_t)(x >> 32);
        }
        add_wide(w, __longlong_as_double((long long)r[2]), __longlong_as_double((long long)r[3]), h, cnt, flags,
                 mn, mx, mo);
    }
    io.mkeys[2 * k] = u;
    io.mkeys[2 * k + 1] = v;
    io.mkeep[k] = (!io.partial_adj || (flags & ADJ_FLAG)) ? 1u : 0u;
    io.mnew[k] = found ? 0u : 1u;
    io.mins[k] = ins;
    finalize_row(h, cnt, mn, mx, mo, io.scale, io.offset, io.mfeats + k * N_FEATURES);
}

// merged-order slot of every own row and every new received key, and its keep
// flag: own row i -> i + (new keys below it); new key k -> (own rows below it)
// + (new keys before it).  nrank = exclusive scan of mnew.
__global__ void k_mgpu_slots(MergeIO io, const uint32_t* __restrict__ nrank, uint32_t* __restrict__ keep,
                             int64_t n_slots) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t K = (int64_t)*io.nK;
    const uint32_t n_new = K ? nrank[K - 1] + io.mnew[K - 1] : 0u;
    // slots past the merged table (the buffer is sized by the bound n_own + M)
    if (i >= io.n_own + (int64_t)n_new && i < n_slots) keep[i] = 0u;
    if (i < io.n_own) {
        const uint64_t u = io.own_edges[2 * i], v = io.own_edges[2 * i + 1];
        const int64_t b = K ? lower_uv(io.mkeys, K, u, v) : 0;
        const int64_t slot = i + (b < K ? (int64_t)nrank[b] : (int64_t)n_new);
        const uint32_t t = io.touched[i];
        const uint32_t kp = t ? io.mkeep[t - 1]
                              : ((!io.partial_adj || (io.own_wide[i * WREC_WORDS + 42] & ADJ_FLAG)) ? 1u : 0u);
        keep[slot] = kp;
    } else if (i < io.n_own + K) {
        const int64_t k = i - io.n_own;
        if (io.mnew[k]) keep[io.mins[k] + nrank[k]] = io.mkeep[k];
    }
}

// rows to their final positions (fpos = exclusive scan of keep over the slots)
__global__ void k_mgpu_scatter(MergeIO io, const uint32_t* __restrict__ nrank, const uint32_t* __restrict__ keep,
                               const uint32_t* __restrict__ fpos, int64_t n_slots, uint64_t* __restrict__ out_e,
                               double* __restrict__ out_f, uint32_t* __restrict__ n_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t K = (int64_t)*io.nK;
    if (i == 0) *n_out = n_slots ? fpos[n_slots - 1] + keep[n_slots - 1] : 0u;
    const uint32_t n_new = K ? nrank[K - 1] + io.mnew[K - 1] : 0u;
    const uint64_t* ke;
    const double* kf;
    int64_t slot;
    if (i < io.n_own) {
        const uint64_t u = io.own_edges[2 * i], v = io.own_edges[2 * i + 1];
        const int64_t b = K ? lower_uv(io.mkeys, K, u, v) : 0;
        slot = i + (b < K ? (int64_t)nrank[b] : (int64_t)n_new);
        const uint32_t t = io.touched[i];
        ke = io.own_edges + 2 * i;
        kf = t ? io.mfeats + (int64_t)(t - 1) * N_FEATURES : io.own_feats + i * N_FEATURES;
    } else if (i < io.n_own + K) {
        const int64_t k = i - io.n_own;
        if (!io.mnew[k]) return;
        slot = io.mins[k] + nrank[k];
        ke = io.mkeys + 2 * k;
        kf = io.mfeats + k * N_FEATURES;
    } else {
        return;
    }
    if (!keep[slot]) return;
    const int64_t f = fpos[slot];
    out_e[2 * f] = ke[0];
    out_e[2 * f + 1] = ke[1];
    const double2* s2 = reinterpret_cast<const double2*>(kf);
    double2* d2 = reinterpret_cast<double2*>(out_f + f * N_FEATURES);
#pragma unroll
    for (int j = 0; j < N_FEATURES / 2; ++j) d2[j] = s2[j];
}

// node ids of the own range and every received segment -> one list
__global__ void k_mgpu_node_list(RecvSegs S, const uint64_t* __restrict__ recv, const int64_t* __restrict__ rn,
                                 const int64_t* __restrict__ rn_off, const uint64_t* __restrict__ own, int64_t n_own,
                                 uint64_t* __restrict__ out, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    if (i < n_own) {
        out[i] = own[i];
        return;
    }
    int s = 0;
    while (s + 1 < S.n && rn_off[s + 1] <= i - n_own) ++s;
    const int64_t a = i - n_own - rn_off[s];
    const int64_t rows = S.row0[s + 1] - S.row0[s];
    out[i] = recv[S.w_off[s] + rows * ROW + a];
}

// ---------------------------------------------------------------------------
// launchers (called from ctg_api.hip)
// ---------------------------------------------------------------------------
hipError_t mgpu_sample(const uint64_t* edges, int64_t E, int64_t* meta, hipStream_t s) {
    hipLaunchKernelGGL(k_mgpu_sample, dim3((MS + 1 + 255) / 256), dim3(256), 0, s, edges, E, meta);
    return hipGetLastError();
}

hipError_t mgpu_split(const uint64_t* edges, int64_t E, const uint64_t* nodes, int64_t N, const int64_t* meta_all,
                      int world, uint64_t* spl, int64_t* counts, hipStream_t s) {
    if (world > 1) {
        hipError_t e = hipMemsetAsync(spl, 0, (size_t)(world - 1) * 8, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_mgpu_splitters, dim3((world * MS + 255) / 256), dim3(256), 0, s, meta_all, world, spl);
    }
    hipLaunchKernelGGL(k_mgpu_bounds, dim3(1), dim3(CTG_MGPU_MAX_WORLD), 0, s, edges, E, nodes, N, spl, world,
                       counts);
    return hipGetLastError();
}

hipError_t mgpu_pack(const ctg_result* r, const int64_t* counts_all, int world, int rank, int64_t* send,
                     hipStream_t s) {
    Segs S;
    std::memset(&S, 0, sizeof(S));
    const int64_t* mine = counts_all + (int64_t)rank * world * 2;   // [dst][rows, nodes] of this rank
    int64_t e0 = 0, n0 = 0, w = 0;
    for (int d = 0; d < world; ++d) {
        const int64_t ec = mine[2 * d], nc = mine[2 * d + 1];
        if (d != rank && (ec || nc)) {
            S.e_start[S.n] = e0;
            S.e_cnt[S.n] = ec;
            S.n_start[S.n] = n0;
            S.n_cnt[S.n] = nc;
            S.w_off[S.n] = w;
            w += ec * ROW + nc;
            ++S.n;
        }
        e0 += ec;
        n0 += nc;
    }
    S.w_off[S.n] = w;
    if (w == 0) return hipSuccess;
    const bool defer = r->defer.on && !r->stats;
    const int64_t blocks = std::min<int64_t>((w + 255) / 256, 8192);
    hipLaunchKernelGGL(k_mgpu_pack, dim3((unsigned)blocks), dim3(256), 0, s, S, r->edges, r->stat_sums,
                       defer ? nullptr : reinterpret_cast<const uint64_t*>(r->stats), r->nodes,
                       reinterpret_cast<uint64_t*>(send));
    if (defer) {
        int64_t rows = 0;
        for (int i = 0; i < S.n; ++i) rows += S.e_cnt[i];
        if (rows > 0)
            hipLaunchKernelGGL(k_mgpu_pack_deferred, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, S,
                               r->defer, reinterpret_cast<uint64_t*>(send));
    }
    return hipGetLastError();
}


// exclusive prefix sum of n u32 (rocPRIM, the workspace's temp buffer)
static hipError_t excl_scan(Workspace& w, const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t tb = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, tb, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    ensure(&w.temp, w.temp_bytes, tb + 256);
    if (!w.temp) return hipErrorOutOfMemory;
    tb = w.temp_bytes;
    return rocprim::exclusive_scan(w.temp, tb, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
}

static unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>((n + 255) / 256, 1); }

// ctg_mgpu_merge (include/ctg.h): this rank's shard of the global table.
hipError_t mgpu_merge(ctg_result* L, const int64_t* recv, const int64_t* counts_all, int world, int rank,
                      double hist_lo, double hist_hi, hipStream_t s, ctg_result* r, int* lib_rc) {
    Workspace& w = ws(r->device);
    *lib_rc = CTG_OK;
    // own range: rows / node ids this rank kept for itself
    const int64_t* mine = counts_all + (int64_t)rank * world * 2;
    int64_t e_lo = 0, n_lo = 0;
    for (int d = 0; d < rank; ++d) {
        e_lo += mine[2 * d];
        n_lo += mine[2 * d + 1];
    }
    const int64_t e_cnt = mine[2 * rank], n_cnt = mine[2 * rank + 1];
    // received segments, sources in rank order
    RecvSegs S;
    std::memset(&S, 0, sizeof(S));
    int64_t rn[CTG_MGPU_MAX_WORLD], rn_off[CTG_MGPU_MAX_WORLD + 1];
    int64_t M = 0, NM = 0, words = 0;
    for (int q = 0; q < world; ++q) {
        const int64_t* c = counts_all + ((int64_t)q * world + rank) * 2;
        if (q == rank || (c[0] == 0 && c[1] == 0)) continue;
        S.row0[S.n] = M;
        S.w_off[S.n] = words;
        rn[S.n] = c[1];
        rn_off[S.n] = NM;
        M += c[0];
        NM += c[1];
        words += c[0] * ROW + c[1];
        ++S.n;
    }
    S.row0[S.n] = M;
    rn_off[S.n] = NM;
    const uint64_t* rv = reinterpret_cast<const uint64_t*>(recv);
    std::vector<void*> tmp;
    auto alloc = [&](size_t bytes) {
        void* p = dev_alloc(std::max<size_t>(bytes, 16));
        tmp.push_back(p);
        return p;
    };
    struct Release {
        std::vector<void*>& t;
        ~Release() {
            for (void* p : t) dev_free(p);   // stream-ordered reuse
        }
    } release{tmp};
    hipError_t e = hipSuccess;

    // nodes: the own range, or the own range and every received id, unique
    if (NM == 0) {
        r->nodes = L->nodes + n_lo;
        r->n_nodes = n_cnt;
        r->owned.push_back(L->nodes);
        L->nodes = nullptr;
    } else {
        const int64_t total = n_cnt + NM;
        uint64_t* list = (uint64_t*)alloc((size_t)total * 8);
        if (!list) return hipErrorOutOfMemory;
        int64_t* rnd = (int64_t*)alloc((size_t)(2 * CTG_MGPU_MAX_WORLD + 1) * 8);
        if (!rnd) return hipErrorOutOfMemory;
        e = hipMemcpyAsync(rnd, rn, (size_t)S.n * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(rnd + CTG_MGPU_MAX_WORLD, rn_off, (size_t)(S.n + 1) * 8, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_mgpu_node_list, dim3(grid_of(total)), dim3(256), 0, s, S, rv, rnd,
                           rnd + CTG_MGPU_MAX_WORLD, L->nodes + n_lo, n_cnt, list, total);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        ctg_result* U = nullptr;
        const int rc = ctg_unique_values(list, total, CTG_MEM_DEVICE, s, &U);
        if (rc) {   // its status and message pass through
            *lib_rc = rc;
            return hipErrorUnknown;
        }
        r->nodes = U->nodes;
        r->n_nodes = U->n_nodes;
        r->owned.push_back(U->nodes);
        U->nodes = nullptr;
        ctg_free(U);
    }

    // edges and features
    if (M == 0 && !L->partial_adj) {   // nothing received, nothing to drop: the own range is the shard
        r->edges = L->edges + 2 * e_lo;
        r->features = L->features ? L->features + 10 * e_lo : nullptr;
        r->n_edges = e_cnt;
        r->owned.push_back(L->edges);
        r->owned.push_back(L->features);
        L->edges = nullptr;
        L->features = nullptr;
        return hipSuccess;
    }
    // needs a CTG_KEEP_STATS partial table (rows, or CTG_DEFER_STATS records)
    if ((!L->stats && !L->defer.on) || !L->features) return hipErrorInvalidValue;
    // row indices, run heads and output positions below are u32
    if (M >= (1ll << 32) || e_cnt + M >= (1ll << 32) || NM >= (1ll << 32)) {
        set_error("ctg_mgpu_merge: more than 2^32 rows in one shard (split the slab over more ranks)");
        *lib_rc = CTG_ERR_UNSUPPORTED;
        return hipErrorNotSupported;
    }
    MergeIO io{};
    io.own_edges = L->edges + 2 * e_lo;
    io.own_feats = L->features + 10 * e_lo;
    io.own_wide = L->stats ? L->stats + WREC_WORDS * e_lo : nullptr;
    io.own_sums = L->stat_sums ? L->stat_sums + e_lo : nullptr;
    if (!L->stats) io.defer = L->defer;
    io.own_row0 = e_lo;
    io.n_own = e_cnt;
    io.recv = rv;
    io.partial_adj = L->partial_adj;
    io.scale = (double)NBINS / (hist_hi - hist_lo);
    io.offset = hist_lo;
    const int64_t Mb = std::max<int64_t>(M, 1);
    uint32_t* order = (uint32_t*)alloc(Mb * 4);
    uint64_t* skeys = (uint64_t*)alloc(Mb * 16);
    uint32_t* head = (uint32_t*)alloc(Mb * 4);
    uint32_t* rid = (uint32_t*)alloc(Mb * 4);
    uint32_t* run0 = (uint32_t*)alloc((Mb + 1) * 4);
    uint64_t* mkeys = (uint64_t*)alloc(Mb * 16);
    double* mfeats = (double*)alloc(Mb * N_FEATURES * 8);
    uint32_t* mkeep = (uint32_t*)alloc(Mb * 4);
    uint32_t* mnew = (uint32_t*)alloc(Mb * 4);
    uint32_t* nrank = (uint32_t*)alloc(Mb * 4);
    int64_t* mins = (int64_t*)alloc(Mb * 8);
    uint32_t* touched = (uint32_t*)alloc(std::max<int64_t>(e_cnt, 1) * 4);
    const int64_t n_slots = e_cnt + M;
    uint32_t* keep = (uint32_t*)alloc(std::max<int64_t>(n_slots, 1) * 4);
    uint32_t* fpos = (uint32_t*)alloc(std::max<int64_t>(n_slots, 1) * 4);
    uint32_t* nK = w.small + 20;
    uint32_t* n_out = w.small + 21;
    if (!order || !skeys || !head || !rid || !run0 || !mkeys || !mfeats || !mkeep || !mnew || !nrank || !mins ||
        !touched || !keep || !fpos)
        return hipErrorOutOfMemory;
    io.order = order;
    io.skeys = skeys;
    io.run0 = run0;
    io.nK = nK;
    io.mkeys = mkeys;
    io.mfeats = mfeats;
    io.mkeep = mkeep;
    io.mnew = mnew;
    io.mins = mins;
    io.touched = touched;
    if ((e = hipMemsetAsync(nK, 0, 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(mnew, 0, Mb * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(touched, 0, std::max<int64_t>(e_cnt, 1) * 4, s)) != hipSuccess) return e;
    if (M > 0) {
        hipLaunchKernelGGL(k_mgpu_order, dim3(grid_of(M)), dim3(256), 0, s, S, rv, order, skeys);
        hipLaunchKernelGGL(k_mgpu_heads, dim3(grid_of(M)), dim3(256), 0, s, M, skeys, head);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = excl_scan(w, head, rid, M, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_mgpu_runs, dim3(grid_of(M)), dim3(256), 0, s, M, head, rid, run0, nK);
        hipLaunchKernelGGL(k_mgpu_combine, dim3(grid_of(M)), dim3(256), 0, s, S, io);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = excl_scan(w, mnew, nrank, M, s)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_mgpu_slots, dim3(grid_of(n_slots)), dim3(256), 0, s, io, nrank, keep, n_slots);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = excl_scan(w, keep, fpos, n_slots, s)) != hipSuccess) return e;
    r->edges = (uint64_t*)dev_alloc((size_t)std::max<int64_t>(n_slots, 1) * 16);
    r->features = (double*)dev_alloc((size_t)std::max<int64_t>(n_slots, 1) * N_FEATURES * 8);
    r->owned.push_back(r->edges);
    r->owned.push_back(r->features);
    if (!r->edges || !r->features) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(k_mgpu_scatter, dim3(grid_of(n_slots)), dim3(256), 0, s, io, nrank, keep, fpos, n_slots,
                       r->edges, r->features, n_out);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(w.small_host + 21, n_out, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    r->n_edges = n_slots ? w.small_host[21] : 0;
    return hipSuccess;
}

}  // namespace ctg
