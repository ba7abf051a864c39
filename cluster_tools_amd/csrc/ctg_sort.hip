// Record-key sort for the back half (gfx950): MSD bucket pass + segmented sort.
//
// The scan's record keys (packed (u,v) with the record slot in the low ib
// bits) come out of the face scan grouped by tile, and the reduction only
// needs them grouped by key and ordered by (u,v).  rocPRIM's onesweep sorts
// the 57-bit words of the 512^3 step in 4 passes of 10 bits, each a launch
// with its own look-back state and buffer fills (~150 us at 2 M records: the
// passes are launch- and latency-bound at that size).  Here:
//
//   k_bucket_hist    histogram of the top BB key bits (LDS per workgroup)
//   k_bucket_scan    exclusive scan of the 2^BB counts (one workgroup)
//   k_bucket_scatter every key to its bucket (per-workgroup LDS ranks, one
//                    global reservation per (workgroup, bucket))
//   rocprim::segmented_radix_sort_keys over the buckets, on the key bits below
//                    the bucket bits only (the slot bits need no order)
//
// BB is chosen so a bucket averages ~1 K keys (LDS-sized segments); any skew
// (e.g. one label adjacent to many: background) is handled by the segmented
// sort's large-segment path, so there is no size precondition.  (The scan's
// (key, slot) records take the group sort further below.)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "ctg_internal.h"

namespace ctg {

constexpr int BK_THREADS = 256;
constexpr int BK_CHUNK = 4096;   // keys per workgroup in the histogram / scatter
constexpr int BK_MAX_BITS = 12;  // at most 4096 buckets (LDS counters)
static_assert(5 * (1 << BK_MAX_BITS) + 2 <= BK_SMALL_WORDS, "bucket-sort scratch (ctg_internal.h)");

__global__ __launch_bounds__(BK_THREADS) void k_bucket_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                            uint32_t nbk, uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[1 << BK_MAX_BITS];
    for (uint32_t i = threadIdx.x; i < nbk; i += BK_THREADS) h[i] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * BK_CHUNK, b1 = min(n, b0 + BK_CHUNK);
    for (int64_t i = b0 + threadIdx.x; i < b1; i += BK_THREADS) atomicAdd(&h[(uint32_t)(keys[i] >> shift)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbk; i += BK_THREADS)
        if (h[i]) atomicAdd(&counts[i], h[i]);
}

// offs[0..nbk] exclusive prefix of counts; cursor[i] = 0
__global__ __launch_bounds__(1024) void k_bucket_scan(const uint32_t* __restrict__ counts, uint32_t nbk,
                                                      uint32_t* __restrict__ offs, uint32_t* __restrict__ cursor) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (nbk + 1023) / 1024;
    const uint32_t t = threadIdx.x, i0 = t * per;
    uint32_t s = 0;
    for (uint32_t i = i0; i < min(nbk, i0 + per); ++i) s += counts[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan of the thread sums
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0u;
    for (uint32_t i = i0; i < min(nbk, i0 + per); ++i) {
        offs[i] = run;
        run += counts[i];
        cursor[i] = 0u;
    }
    if (t == 1023) offs[nbk] = part[1023];
}

__global__ __launch_bounds__(BK_THREADS) void k_bucket_scatter(const uint64_t* __restrict__ keys, int64_t n,
                                                               int shift, uint32_t nbk,
                                                               const uint32_t* __restrict__ offs,
                                                               uint32_t* __restrict__ cursor,
                                                               uint64_t* __restrict__ out) {
    constexpr int PER = BK_CHUNK / BK_THREADS;
    __shared__ uint32_t h[1 << BK_MAX_BITS];
    __shared__ uint32_t base[1 << BK_MAX_BITS];
    for (uint32_t i = threadIdx.x; i < nbk; i += BK_THREADS) h[i] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * BK_CHUNK;
    uint64_t k[PER];
    uint32_t rank[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = b0 + j * BK_THREADS + threadIdx.x;
        k[j] = i < n ? keys[i] : 0ull;
        rank[j] = i < n ? atomicAdd(&h[(uint32_t)(k[j] >> shift)], 1u) : 0u;   // order within a bucket: any
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbk; i += BK_THREADS)
        base[i] = h[i] ? offs[i] + atomicAdd(&cursor[i], h[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = b0 + j * BK_THREADS + threadIdx.x;
        if (i < n) out[base[(uint32_t)(k[j] >> shift)] + rank[j]] = k[j];
    }
}

// (key, value) pairs to their buckets (as k_bucket_scatter)
__global__ __launch_bounds__(BK_THREADS) void k_bucket_scatter_pairs(const uint64_t* __restrict__ keys,
                                                                     const uint32_t* __restrict__ vals, int64_t n,
                                                                     int shift, uint32_t nbk,
                                                                     const uint32_t* __restrict__ offs,
                                                                     uint32_t* __restrict__ cursor,
                                                                     uint64_t* __restrict__ kout,
                                                                     uint32_t* __restrict__ vout) {
    constexpr int PER = BK_CHUNK / BK_THREADS;
    __shared__ uint32_t h[1 << BK_MAX_BITS];
    __shared__ uint32_t base[1 << BK_MAX_BITS];
    for (uint32_t i = threadIdx.x; i < nbk; i += BK_THREADS) h[i] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * BK_CHUNK;
    uint64_t k[PER];
    uint32_t rank[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = b0 + j * BK_THREADS + threadIdx.x;
        k[j] = i < n ? keys[i] : 0ull;
        rank[j] = i < n ? atomicAdd(&h[(uint32_t)(k[j] >> shift)], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbk; i += BK_THREADS)
        base[i] = h[i] ? offs[i] + atomicAdd(&cursor[i], h[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = b0 + j * BK_THREADS + threadIdx.x;
        if (i < n) {
            const uint32_t d = base[(uint32_t)(k[j] >> shift)] + rank[j];
            kout[d] = k[j];
            vout[d] = vals[i];
        }
    }
}

static int bucket_bits(int64_t n, int key_bits) {
    int bb = 1;
    while (bb < BK_MAX_BITS && (n >> (bb + 10)) > 0) ++bb;   // ~1 K keys per bucket
    return std::min(bb, key_bits);
}

// (keys, vals) sorted by key bits [0, hi_bit) into (kout, vout); ktmp / vtmp: n each
hipError_t bucket_sort_pairs(const uint64_t* keys, const uint32_t* vals, uint64_t* ktmp, uint32_t* vtmp,
                             uint64_t* kout, uint32_t* vout, int64_t n, int hi_bit, uint32_t* small, void** temp,
                             size_t* temp_bytes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (n > 0xFFFFFFFFll || hi_bit > 64 || hi_bit <= 0) return hipErrorInvalidValue;
    const int bb = bucket_bits(n, hi_bit);
    const int shift = hi_bit - bb;
    const uint32_t nbk = 1u << bb;
    uint32_t* counts = small;
    uint32_t* offs = small + (1 << BK_MAX_BITS);
    uint32_t* cursor = small + 2 * (1 << BK_MAX_BITS) + 1;
    hipError_t e = hipMemsetAsync(counts, 0, nbk * 4, s);
    if (e != hipSuccess) return e;
    const unsigned nwg = (unsigned)((n + BK_CHUNK - 1) / BK_CHUNK);
    hipLaunchKernelGGL(k_bucket_hist, dim3(nwg), dim3(BK_THREADS), 0, s, keys, n, shift, nbk, counts);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(1024), 0, s, counts, nbk, offs, cursor);
    hipLaunchKernelGGL(k_bucket_scatter_pairs, dim3(nwg), dim3(BK_THREADS), 0, s, keys, vals, n, shift, nbk, offs,
                       cursor, ktmp, vtmp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (shift <= 0) {
        e = hipMemcpyAsync(kout, ktmp, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
        return e != hipSuccess ? e : hipMemcpyAsync(vout, vtmp, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    }
    size_t need = 0;
    e = rocprim::segmented_radix_sort_pairs(nullptr, need, ktmp, kout, vtmp, vout, (unsigned)n, nbk, offs, offs + 1,
                                            0u, (unsigned)shift, s);
    if (e != hipSuccess) return e;
    ensure(temp, *temp_bytes, need + 256);
    size_t have = *temp_bytes;
    return rocprim::segmented_radix_sort_pairs(*temp, have, ktmp, kout, vtmp, vout, (unsigned)n, nbk, offs, offs + 1,
                                               0u, (unsigned)shift, s);
}

// ---------------------------------------------------------------------------
// Runs of equal keys after bucket_sort_keys (the back half's "segment" step):
// runs never cross buckets, so heads are counted per bucket (one workgroup
// each), the bucket counts scanned (k_bucket_scan), and every bucket writes
// its unique keys, run offsets and run lengths at its base -- three light
// launches instead of rocPRIM's run-length encode and exclusive scan.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool is_head(const uint64_t* k, uint32_t i, uint32_t b0, int ib) {
    return i == b0 || (k[i] >> ib) != (k[i - 1] >> ib);
}

__global__ __launch_bounds__(BK_THREADS) void k_run_heads_count(const uint64_t* __restrict__ keys, int ib,
                                                                const uint32_t* __restrict__ offs,
                                                                uint32_t* __restrict__ hc) {
    __shared__ uint32_t red[BK_THREADS / 64];
    const uint32_t b = blockIdx.x, b0 = offs[b], b1 = offs[b + 1];
    uint32_t c = 0;
    for (uint32_t i = b0 + threadIdx.x; i < b1; i += BK_THREADS) c += is_head(keys, i, b0, ib) ? 1u : 0u;
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < BK_THREADS / 64; ++w) t += red[w];
        hc[b] = t;
    }
}

__global__ __launch_bounds__(BK_THREADS) void k_run_heads_write(const uint64_t* __restrict__ keys, int ib,
                                                                uint32_t nbk, const uint32_t* __restrict__ offs,
                                                                const uint32_t* __restrict__ ho,
                                                                uint64_t* __restrict__ uniq, uint32_t* __restrict__ runs,
                                                                uint32_t* __restrict__ roffs, uint32_t* __restrict__ dE) {
    __shared__ uint32_t wsum[BK_THREADS / 64];
    const uint32_t b = blockIdx.x, b0 = offs[b], b1 = offs[b + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (b == 0 && threadIdx.x == 0) *dE = ho[nbk];
    uint32_t base = ho[b];
    for (uint32_t c0 = b0; c0 < b1; c0 += BK_THREADS) {
        const uint32_t i = c0 + threadIdx.x;
        const bool h = i < b1 && is_head(keys, i, b0, ib);
        const uint64_t m = __ballot(h);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < BK_THREADS / 64; ++w) {
            before += w < wv ? wsum[w] : 0u;
            total += wsum[w];
        }
        if (h) {
            const uint32_t e = base + before + r;
            const uint64_t k = keys[i] >> ib;
            uint32_t j = i + 1;
            while (j < b1 && (keys[j] >> ib) == k) ++j;   // runs are short (~2 records per edge)
            uniq[e] = k;
            roffs[e] = i;
            runs[e] = j - i;
        }
        base += total;
        __syncthreads();
    }
}

// (sorted keys of bucket_sort_keys with the same n / lo_bit / hi_bit) ->
// uniq keys (>> lo_bit), run lengths, run offsets, *dE = number of runs
hipError_t bucket_runs(const uint64_t* sorted, int64_t n, int lo_bit, int hi_bit, uint32_t* small, uint64_t* uniq,
                       uint32_t* runs, uint32_t* roffs, uint32_t* dE, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int bb = bucket_bits(n, hi_bit - lo_bit);
    const uint32_t nbk = 1u << bb;
    // small layout (BK_SMALL_WORDS): counts [0, M), bucket offsets [M, 2M+1),
    // cursors [2M+1, 3M+1) -- free now, they hold the head counts --, head
    // offsets [3M+1, 4M+2), scratch for the scan's cursor output [4M+2, 5M+2)
    constexpr uint32_t M = 1u << BK_MAX_BITS;
    const uint32_t* offs = small + M;
    uint32_t* hc = small + 2 * M + 1;
    uint32_t* ho = small + 3 * M + 1;
    hipLaunchKernelGGL(k_run_heads_count, dim3(nbk), dim3(BK_THREADS), 0, s, sorted, lo_bit, offs, hc);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(1024), 0, s, hc, nbk, ho, small + 4 * M + 2);
    hipLaunchKernelGGL(k_run_heads_write, dim3(nbk), dim3(BK_THREADS), 0, s, sorted, lo_bit, nbk, offs, ho, uniq,
                       runs, roffs, dE);
    return hipGetLastError();
}

// keys (n, packed: key bits [lo_bit, hi_bit), slot bits below) -> sorted by
// the key bits into out (order among equal keys: any).  tmp: n u64;
// small: 3 * 4096 + 1 u32; temp / temp_bytes: the caller's growable scratch.
hipError_t bucket_sort_keys(const uint64_t* keys, uint64_t* tmp, uint64_t* out, int64_t n, int lo_bit, int hi_bit,
                            uint32_t* small, void** temp, size_t* temp_bytes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (n > 0xFFFFFFFFll || hi_bit > 64 || lo_bit < 0 || hi_bit <= lo_bit) return hipErrorInvalidValue;
    const int bb = bucket_bits(n, hi_bit - lo_bit);
    const int shift = hi_bit - bb;
    const uint32_t nbk = 1u << bb;
    uint32_t* counts = small;
    uint32_t* offs = small + (1 << BK_MAX_BITS);
    uint32_t* cursor = small + 2 * (1 << BK_MAX_BITS) + 1;
    hipError_t e = hipMemsetAsync(counts, 0, nbk * 4, s);
    if (e != hipSuccess) return e;
    const unsigned nwg = (unsigned)((n + BK_CHUNK - 1) / BK_CHUNK);
    hipLaunchKernelGGL(k_bucket_hist, dim3(nwg), dim3(BK_THREADS), 0, s, keys, n, shift, nbk, counts);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(1024), 0, s, counts, nbk, offs, cursor);
    hipLaunchKernelGGL(k_bucket_scatter, dim3(nwg), dim3(BK_THREADS), 0, s, keys, n, shift, nbk, offs, cursor, tmp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (shift <= lo_bit) {   // the buckets are the keys: already grouped and ordered
        return hipMemcpyAsync(out, tmp, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
    }
    size_t need = 0;
    e = rocprim::segmented_radix_sort_keys(nullptr, need, tmp, out, (unsigned)n, nbk, offs, offs + 1,
                                           (unsigned)lo_bit, (unsigned)shift, s);
    if (e != hipSuccess) return e;
    ensure(temp, *temp_bytes, need + 256);
    size_t have = *temp_bytes;
    return rocprim::segmented_radix_sort_keys(*temp, have, tmp, out, (unsigned)n, nbk, offs, offs + 1,
                                              (unsigned)lo_bit, (unsigned)shift, s);
}

// ---------------------------------------------------------------------------
// Group sort: the face scan's (key, slot) records -> runs of equal keys, for
// record sets whose key and slot do not pack into one 63-bit sort word
// (configs[2], [3], [4]: 44-48 key bits + 25-28 slot bits).
//
//   k_gs_hist     bucket histogram of the packed key's bits above `shift`,
//                 read straight from the scan's 64 record regions (no pack
//                 pass); only buckets up to the largest label are launched
//   k_gs_scan     bucket offsets, the largest bucket (the host checks it
//                 against the LDS capacity), cursors reset
//   k_gs_scatter  item = (key bits below the bucket bits) << ib | slot to its
//                 bucket (LDS ranks, one global reservation per workgroup and
//                 bucket)
//   k_gs_sort     one workgroup per bucket: an LDS counting sort by the top
//                 GS_GB bits of the bucket-local key (its u offset for the
//                 usual label densities: one group per label u), each item's
//                 rank in its group by one compare pass over the group (~15
//                 records per u); writes the slot permutation, the sorted
//                 packed keys (in place) and the bucket's run count
//   k_gs_scan     run offsets of the buckets
//   k_gs_runs     one workgroup per bucket: run heads of the sorted keys ->
//                 run table (unique key, first sorted position, length)
//
// No inter-workgroup dependency inside a launch (a single-pass look-back
// needs an ordered ticket per workgroup, and one counter serves only ~88
// tickets per microsecond).  A bucket above GS_CAP items (a label adjacent to
// very many) makes the host take the onesweep path instead.
// ---------------------------------------------------------------------------
constexpr int GS_THREADS = 512;               // k_gs_sort / k_gs_runs (three workgroups per CU)
constexpr int GS_IPT = 16;
constexpr int GS_CAP = GS_THREADS * GS_IPT;   // items of one bucket in LDS
constexpr int GS_TARGET = 3072;               // records per bucket aimed at
constexpr int GS_PASS_THREADS = 1024;         // bucket passes
constexpr int GS_CHUNK = GS_PASS_THREADS * GS_IPT; // records per workgroup of the bucket passes
constexpr int GS_BB_MAX = 16;                 // 64 K buckets
constexpr int GS_M = 1 << GS_BB_MAX;
constexpr uint32_t GS_HALF = 8192;            // LDS bucket counters per window pass of the bucket kernels (32 KB:
                                              // two 1024-thread workgroups per CU; a workgroup's bucket range
                                              // is usually far narrower, a wider one takes several passes)
constexpr int GS_GB = 11;                     // group bits of the in-bucket counting sort
constexpr int GS_NG = 1 << GS_GB;
constexpr uint64_t GS_HEAD = 1ull << 63;      // sorted key of a run head (keys use at most 63 bits)
static_assert(GS_SMALL_WORDS >= 5 * GS_M + 8, "group-sort scratch (ctg_internal.h)");
static_assert(GS_NG % GS_THREADS == 0 && GS_CAP / 32 <= GS_THREADS, "group-sort geometry");

// small (GS_SMALL_WORDS u32): counts [0, M), offsets [M, 2M + 1), cursors
// [2M + 1, 3M + 1), misc [3M + 1, 3M + 8): largest bucket, run total; run
// counts [3M + 8, 4M + 8), run offsets [4M + 8, 5M + 8)
struct GsLayout {
    uint32_t* counts;
    uint32_t* offs;
    uint32_t* cursor;
    uint32_t* misc;
    uint32_t* rcount;
    uint32_t* roff;
    __host__ __device__ explicit GsLayout(uint32_t* small)
        : counts(small), offs(small + GS_M), cursor(small + 2 * GS_M + 1), misc(small + 3 * GS_M + 1),
          rcount(small + 3 * GS_M + 8), roff(small + 4 * GS_M + 8) {}
};

struct GsParams {
    const uint64_t* key;   // the scan's record keys, (u << 32) | v
    int64_t rcap;          // slots per region
    RegionPrefix pre;      // records per region (exclusive prefix)
    int nb;                // bits of v in the packed key (u << nb) | v
    int shift;             // bucket = packed key >> shift
    int ib;                // slot bits of an item
    uint32_t nbk;
};

__device__ __forceinline__ uint64_t gs_packed(uint64_t k, int nb) { return ((k >> 32) << nb) | (k & 0xFFFFFFFFull); }

// The workgroup's bucket range [lo, hi] (hi < lo: no item).  A region chunk's
// records were flushed by tiles scanned at about the same time, so they span a
// few hundred of the (up to 64 K) buckets: the counter passes below zero, count
// and reserve only that window instead of every bucket.
__device__ __forceinline__ void gs_bucket_range(const uint32_t (&bk)[GS_IPT], uint32_t* red, uint32_t& lo,
                                                uint32_t& hi) {
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {
        if (bk[q] != 0xFFFFFFFFu) {
            mn = min(mn, bk[q]);
            mx = max(mx, bk[q]);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    }
    if (threadIdx.x == 0) {
        red[0] = 0xFFFFFFFFu;
        red[1] = 0u;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&red[0], mn);
        atomicMax(&red[1], mx);
    }
    __syncthreads();
    lo = red[0];
    hi = red[1];
}

__global__ __launch_bounds__(GS_PASS_THREADS) void k_gs_hist(GsParams P, uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t h[];   // min(nbk, GS_HALF) counters
    const int r = blockIdx.y;
    const uint32_t cnt = P.pre.off[r + 1] - P.pre.off[r];
    const uint32_t c0 = blockIdx.x * GS_CHUNK;
    if (c0 >= cnt) return;
    const uint64_t* src = P.key + (int64_t)r * P.rcap;
    // every load issued before the first use (clamped index, no branch around it)
    uint32_t bk[GS_IPT];
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {
        const uint32_t j = c0 + q * GS_PASS_THREADS + threadIdx.x;
        const uint64_t k = src[min(j, cnt - 1)];
        const uint32_t b = (uint32_t)(gs_packed(k, P.nb) >> P.shift);
        bk[q] = j < cnt && b < P.nbk ? b : 0xFFFFFFFFu;   // (the bucket loop's bound, as before the window)
    }
    __shared__ uint32_t red[2];
    uint32_t lo, hi;
    gs_bucket_range(bk, red, lo, hi);
    // [lo, hi] in windows of at most GS_HALF counters
    for (uint32_t h0 = lo; h0 <= hi && lo <= hi; h0 += GS_HALF) {
        const uint32_t hn = min(GS_HALF, hi + 1 - h0);
        for (uint32_t i = threadIdx.x; i < hn; i += GS_PASS_THREADS) h[i] = 0;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < GS_IPT; ++q)
            if (bk[q] - h0 < hn) atomicAdd(&h[bk[q] - h0], 1u);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < hn; i += GS_PASS_THREADS)
            if (h[i]) atomicAdd(&counts[h0 + i], h[i]);
        __syncthreads();
    }
}

// one workgroup, exclusive scan of in[0, n) into out[0, n] (out[n] = total),
// four entries per thread and 4096 per round; optionally the largest entry
// into *mx_out and cursor[0, n) = 0
__global__ __launch_bounds__(1024) void k_gs_scan(const uint32_t* __restrict__ in, uint32_t n,
                                                  uint32_t* __restrict__ out, uint32_t* __restrict__ cursor,
                                                  uint32_t* __restrict__ mx_out) {
    __shared__ uint32_t wtmp[16];
    __shared__ uint32_t mx;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) mx = 0;
    uint32_t carry = 0, m = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += 4096) {
        const uint32_t i0 = c0 + 4 * t;
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = i0 + k < n ? in[i0 + k] : 0u;
        m = max(m, max(max(v[0], v[1]), max(v[2], v[3])));
        const uint32_t x = v[0] + v[1] + v[2] + v[3];
        uint32_t s = x;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)s, o, 64);
            s += lane >= o ? y : 0u;
        }
        if (lane == 63) wtmp[wv] = s;
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint32_t u = wtmp[w];
            before += w < wv ? u : 0u;
            total += u;
        }
        __syncthreads();
        uint32_t ex = carry + before + s - x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (i0 + k < n) {
                out[i0 + k] = ex;
                if (cursor) cursor[i0 + k] = 0u;
            }
            ex += v[k];
        }
        carry += total;
    }
    atomicMax(&mx, m);
    __syncthreads();
    if (t == 0) {
        out[n] = carry;
        if (mx_out) *mx_out = mx;
    }
}

__global__ __launch_bounds__(GS_PASS_THREADS) void k_gs_scatter(GsParams P, const uint32_t* __restrict__ offs,
                                                                uint32_t* __restrict__ cursor,
                                                                uint64_t* __restrict__ items) {
    extern __shared__ uint32_t h[];   // bucket counters, then the workgroup's bucket bases (per pass)
    const int r = blockIdx.y;
    const uint32_t cnt = P.pre.off[r + 1] - P.pre.off[r];
    const uint32_t c0 = blockIdx.x * GS_CHUNK;
    if (c0 >= cnt) return;
    const uint64_t* src = P.key + (int64_t)r * P.rcap;
    const uint64_t rmask = (1ull << P.shift) - 1ull;
    uint64_t it[GS_IPT];
    uint32_t bk[GS_IPT], rk[GS_IPT];
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) it[q] = src[min(c0 + q * GS_PASS_THREADS + threadIdx.x, cnt - 1)];
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {
        const uint32_t j = c0 + q * GS_PASS_THREADS + threadIdx.x;
        const uint64_t pk = gs_packed(it[q], P.nb);
        const uint32_t b = (uint32_t)(pk >> P.shift);
        bk[q] = j < cnt && b < P.nbk ? b : 0xFFFFFFFFu;
        it[q] = ((pk & rmask) << P.ib) | ((uint64_t)r * (uint64_t)P.rcap + j);
    }
    __shared__ uint32_t red[2];
    uint32_t lo, hi;
    gs_bucket_range(bk, red, lo, hi);
    for (uint32_t h0 = lo; h0 <= hi && lo <= hi; h0 += GS_HALF) {
        const uint32_t hn = min(GS_HALF, hi + 1 - h0);
        for (uint32_t i = threadIdx.x; i < hn; i += GS_PASS_THREADS) h[i] = 0;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < GS_IPT; ++q)
            if (bk[q] - h0 < hn) rk[q] = atomicAdd(&h[bk[q] - h0], 1u);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < hn; i += GS_PASS_THREADS)
            if (h[i]) h[i] = offs[h0 + i] + atomicAdd(&cursor[h0 + i], h[i]);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < GS_IPT; ++q)
            if (bk[q] - h0 < hn) items[h[bk[q] - h0] + rk[q]] = it[q];
        __syncthreads();
    }
}

// exclusive scan in place of a[0, GS_NG) (GS_NG / GS_THREADS consecutive
// entries per thread); returns the total
__device__ __forceinline__ uint32_t gs_block_scan(uint32_t* a, uint32_t* wtmp) {
    constexpr int PER = GS_NG / GS_THREADS;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t x[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        x[k] = a[PER * t + k];
        sum += x[k];
    }
    uint32_t s = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)s, o, 64);
        s += lane >= o ? y : 0u;
    }
    if (lane == 63) wtmp[wv] = s;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < GS_THREADS / 64; ++w) {
        const uint32_t v = wtmp[w];
        before += w < wv ? v : 0u;
        total += v;
    }
    uint32_t ex = before + s - sum;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        a[PER * t + k] = ex;
        ex += x[k];
    }
    __syncthreads();
    return total;
}

__device__ __forceinline__ unsigned long long gs_stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
// CTG_GS_DIAG: per-phase s_memtime sums of k_gs_sort (thread 0 of each workgroup)
#define GS_STAMP(k)                                             \
    do {                                                        \
        if (diag && threadIdx.x == 0) {                         \
            const unsigned long long now_ = gs_stamp();         \
            atomicAdd(&diag[k], now_ - t_prev);                 \
            t_prev = now_;                                      \
        }                                                       \
    } while (0)

// per bucket: sort by the bucket-local key, write the slot permutation and
// the sorted packed keys (in place of the items), count the runs.
// Arrival order only feeds the group counting sort; the in-group ranks are
// taken in group order (lanes of a wave on consecutive positions read the
// same group entries: broadcasts, not bank conflicts).
__global__ __launch_bounds__(GS_THREADS) void k_gs_sort(uint64_t* __restrict__ items, uint32_t* __restrict__ small,
                                                        int shift, int ib, uint32_t* __restrict__ perm,
                                                        unsigned long long* diag) {
    unsigned long long t_prev = diag ? gs_stamp() : 0ull;
    __shared__ uint32_t grem[GS_CAP + 8];         // low key bits by group position, then sorted (+ read pad)
    __shared__ uint16_t gidx[GS_CAP];             // group position -> arrival index
    __shared__ uint32_t goff[GS_NG + 1];          // group counts -> offsets
    __shared__ uint32_t hm[GS_CAP / 32];          // group starts, then every run head
    __shared__ uint32_t wtmp[GS_THREADS / 64];
    GsLayout L(small);
    const int t = threadIdx.x;
    const uint32_t b = blockIdx.x;
    for (int i = t; i <= GS_NG; i += GS_THREADS) goff[i] = 0u;
    for (int i = t; i < GS_CAP / 32; i += GS_THREADS) hm[i] = 0u;
    __syncthreads();
    const uint32_t b0 = L.offs[b], n = L.offs[b + 1] - b0;   // n <= GS_CAP (host-checked)
    if (n == 0) {
        if (t == 0) L.rcount[b] = 0u;
        return;
    }
    const int lo = shift - min(GS_GB, shift);                // <= 32 (host-checked)
    const uint64_t lmask = (1ull << lo) - 1ull;
    const uint32_t smask = ib >= 32 ? 0xFFFFFFFFu : ((1u << ib) - 1u);
    uint32_t va[GS_IPT], vb[GS_IPT];   // arrival phase: low bits, group << 16 | arrival rank
    {
        uint64_t it[GS_IPT];   // every load before the first use (see k_gs_hist)
#pragma unroll
        for (int q = 0; q < GS_IPT; ++q) it[q] = items[b0 + min((uint32_t)(q * GS_THREADS + t), n - 1)];
#pragma unroll
        for (int q = 0; q < GS_IPT; ++q) {
            const uint64_t rem = it[q] >> ib;
            va[q] = (uint32_t)(rem & lmask);
            const uint32_t g = (uint32_t)(rem >> lo);
            vb[q] = 0xFFFFFFFFu;
            if (q * GS_THREADS + t < n) vb[q] = (g << 16) | atomicAdd(&goff[g], 1u);
        }
    }
    __syncthreads();
    GS_STAMP(0);
    gs_block_scan(goff, wtmp);
    if (t == 0) goff[GS_NG] = n;
    __syncthreads();
    GS_STAMP(1);
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q)
        if (vb[q] != 0xFFFFFFFFu) {
            const uint32_t p = goff[vb[q] >> 16] + (vb[q] & 0xFFFFu);
            grem[p] = va[q];
            gidx[p] = (uint16_t)(q * GS_THREADS + t);
        }
    for (int g = t; g < GS_NG; g += GS_THREADS) {   // group starts
        const uint32_t p = goff[g];
        if (goff[g + 1] > p) atomicOr(&hm[p >> 5], 1u << (p & 31));
    }
    __syncthreads();
    GS_STAMP(2);
    // group order: position p ranks among its group [s0, s1) (bounds from the
    // group-start bits); va = the key bits, vb = the final position
    const uint32_t wlast = (n - 1) >> 5;
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {
        const uint32_t p = q * GS_THREADS + t;
        vb[q] = 0xFFFFFFFFu;
        if (p < n) {
            const uint32_t x = grem[p];
            uint32_t w = p >> 5;
            uint32_t m = hm[w] & (0xFFFFFFFFu >> (31 - (p & 31)));   // starts at or below p (p itself at most)
            while (!m) m = hm[--w];
            const uint32_t s0 = (w << 5) + 31 - __clz(m);
            w = p >> 5;
            m = (p & 31) == 31 ? 0u : (hm[w] & (0xFFFFFFFEu << (p & 31)));   // starts above p
            while (!m && w < wlast) m = hm[++w];
            const uint32_t s1 = m ? (w << 5) + __ffs(m) - 1 : n;
            uint32_t rk = 0;
            for (uint32_t j = s0; j < s1; ++j) {
                const uint32_t y = grem[j];
                rk += (y < x || (y == x && j < p)) ? 1u : 0u;
            }
            va[q] = x;
            vb[q] = (s0 + rk) | ((uint32_t)gidx[p] << 16);   // final position | arrival index
        }
    }
    __syncthreads();
    GS_STAMP(3);
    uint32_t gg[GS_IPT];   // the group of each position (from the re-read item)
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {
        const uint32_t a = vb[q] == 0xFFFFFFFFu ? 0u : (vb[q] >> 16);
        const uint64_t it = items[b0 + min(a, n - 1)];   // the slot and the group: an L2 re-read
        gg[q] = (uint32_t)((it >> ib) >> lo);
        if (vb[q] != 0xFFFFFFFFu) {
            const uint32_t f = vb[q] & 0xFFFFu;
            grem[f] = va[q];
            perm[b0 + f] = (uint32_t)it & smask;
        }
    }
    __syncthreads();   // every item read (and grem sorted) before the keys overwrite the items
    GS_STAMP(4);
    const uint64_t bkey = (uint64_t)b << shift;
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q)
        if (vb[q] != 0xFFFFFFFFu) {
            const uint32_t f = vb[q] & 0xFFFFu;
            // run heads: group starts (already marked) or a new key inside the group
            const bool head = ((hm[f >> 5] >> (f & 31)) & 1u) || grem[f - (f > 0 ? 1 : 0)] != va[q] || f == 0;
            items[b0 + f] = bkey | ((uint64_t)gg[q] << lo) | va[q] | (head ? GS_HEAD : 0ull);
            if (head) atomicOr(&hm[f >> 5], 1u << (f & 31));
        }
    __syncthreads();
    GS_STAMP(5);
    uint32_t c = t < GS_CAP / 32 ? (uint32_t)__popc(hm[t]) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
    if ((t & 63) == 0) wtmp[t >> 6] = c;
    __syncthreads();
    if (t == 0) {
        uint32_t T = 0;
        for (int w = 0; w < GS_THREADS / 64; ++w) T += wtmp[w];
        L.rcount[b] = T;
    }
    GS_STAMP(6);
}

struct GsRuns {
    uint64_t* uniq;    // run -> packed key
    uint32_t* runs;    // run -> length
    uint32_t* roffs;   // run -> first sorted position
    uint32_t* dE;      // number of runs
};

// per bucket: the sorted keys (head bit set by k_gs_sort) -> run table at the
// bucket's run offset
__global__ __launch_bounds__(GS_THREADS) void k_gs_runs(const uint64_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ small, uint32_t nbk, GsRuns O) {
    __shared__ uint32_t hm[GS_CAP / 32];
    __shared__ uint32_t hpre[GS_CAP / 32];
    __shared__ uint32_t wtmp[GS_THREADS / 64];
    GsLayout L(const_cast<uint32_t*>(small));
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t b0 = L.offs[b], n = L.offs[b + 1] - b0;
    if (b == 0 && t == 0) *O.dE = L.roff[nbk];
    if (n == 0) return;
    uint64_t k[GS_IPT];
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) k[q] = keys[b0 + min((uint32_t)(q * GS_THREADS + t), n - 1)];
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {   // positions q * 1024 + 64 * wv + lane: one ballot = two words
        const uint64_t m = __ballot(q * GS_THREADS + t < n && (k[q] & GS_HEAD));
        if (lane == 0) {
            const uint32_t w = (q * GS_THREADS + 64 * wv) >> 5;
            hm[w] = (uint32_t)m;
            hm[w + 1] = (uint32_t)(m >> 32);
        }
    }
    __syncthreads();
    const uint32_t hc = t < GS_CAP / 32 ? (uint32_t)__popc(hm[t]) : 0u;
    uint32_t s = hc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)s, o, 64);
        s += lane >= o ? y : 0u;
    }
    if (lane == 63) wtmp[wv] = s;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wv; ++w) before += wtmp[w];
    if (t < GS_CAP / 32) hpre[t] = before + s - hc;
    __syncthreads();
    const uint32_t E0 = L.roff[b];
#pragma unroll
    for (int q = 0; q < GS_IPT; ++q) {
        const uint32_t p = q * GS_THREADS + t;
        if (p < n && (k[q] & GS_HEAD)) {
            const uint32_t w = p >> 5, bit = p & 31;
            const uint32_t e = E0 + hpre[w] + (uint32_t)__popc(hm[w] & ((1u << bit) - 1u));
            uint32_t np = p + 1;
            while (np < n && !((hm[np >> 5] >> (np & 31)) & 1u)) ++np;   // runs are short
            O.uniq[e] = k[q] & ~GS_HEAD;
            O.roffs[e] = b0 + p;
            O.runs[e] = np - p;
        }
    }
}

// Records of the face scan (keys in NREG regions) -> perm / uniq / runs / roffs
// / *dE as the reduction reads them.  *done = false (nothing written): the
// geometry does not fit or some bucket exceeds GS_CAP; the caller sorts
// another way.  One host read (the largest bucket).
hipError_t group_sort_runs(const uint64_t* key, int64_t rcap, const RegionPrefix& pre, int64_t n, int nb, int ub,
                           int ib, uint64_t max_label, uint32_t* small, uint32_t* host_word, uint64_t* items,
                           uint32_t* perm, uint64_t* uniq, uint32_t* runs, uint32_t* roffs, uint32_t* dE,
                           bool* done, hipStream_t s) {
    *done = false;
    if (n <= 0 || n > 0xFFFFFFFFll) return hipSuccess;
    const int kb = ub + nb;
    if (kb > 63) return hipSuccess;
    // buckets of 2^shift packed keys up to the largest key (u, v <= max_label):
    // the largest shift whose buckets average at most GS_TARGET records, and
    // at most GS_M buckets
    const uint64_t max_pk = (std::min<uint64_t>(max_label, (1ull << ub) - 1ull) << nb) | max_label;
    int shift = kb;
    while (shift > 0 && ((max_pk >> (shift - 1)) + 1) <= (uint64_t)GS_M &&
           (double)n / (double)((max_pk >> shift) + 1) > (double)GS_TARGET)
        --shift;
    while (((max_pk >> shift) + 1) > (uint64_t)GS_M) ++shift;
    if (shift + ib > 64 || shift - std::min(GS_GB, shift) > 32) return hipSuccess;
    GsParams P;
    P.key = key;
    P.rcap = rcap;
    P.pre = pre;
    P.nb = nb;
    P.shift = shift;
    P.ib = ib;
    P.nbk = (uint32_t)((max_pk >> shift) + 1);
    GsLayout L(small);
    uint32_t mx = 0;
    for (int r = 0; r < NREG; ++r) mx = std::max(mx, pre.off[r + 1] - pre.off[r]);
    const dim3 grid((mx + GS_CHUNK - 1) / GS_CHUNK, NREG);
    hipError_t e = hipMemsetAsync(L.counts, 0, P.nbk * 4, s);
    if (e != hipSuccess) return e;
    const size_t lds = std::min<uint32_t>(P.nbk, GS_HALF) * 4;
    hipLaunchKernelGGL(k_gs_hist, grid, dim3(GS_PASS_THREADS), lds, s, P, L.counts);
    hipLaunchKernelGGL(k_gs_scan, dim3(1), dim3(1024), 0, s, L.counts, P.nbk, L.offs, L.cursor, L.misc);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(host_word, L.misc, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (*host_word > (uint32_t)GS_CAP) return hipSuccess;   // skewed: a bucket does not fit LDS
    hipLaunchKernelGGL(k_gs_scatter, grid, dim3(GS_PASS_THREADS), lds, s, P, L.offs, L.cursor, items);
#ifdef CTG_DIAG   // per-phase s_memtime sums of k_gs_sort (variant builds, CTG_GS_DIAG set)
    static unsigned long long* diag = nullptr;
    static const bool want_diag = getenv("CTG_GS_DIAG") != nullptr;
    if (want_diag && !diag) hipMalloc(&diag, 64);
    if (diag) hipMemsetAsync(diag, 0, 64, s);
#else
    unsigned long long* diag = nullptr;
#endif
    hipLaunchKernelGGL(k_gs_sort, dim3(P.nbk), dim3(GS_THREADS), 0, s, items, small, shift, ib, perm, diag);
#ifdef CTG_DIAG
    if (diag) {
        unsigned long long h[8];
        hipMemcpyAsync(h, diag, 64, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        fprintf(stderr, "gs_sort nbk %u n %lld stamps load %llu scan %llu scatter %llu rank %llu perm %llu keys %llu count %llu\n",
                P.nbk, (long long)n, h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
    }
#endif
    hipLaunchKernelGGL(k_gs_scan, dim3(1), dim3(1024), 0, s, L.rcount, P.nbk, L.roff, nullptr, nullptr);
    const GsRuns O{uniq, runs, roffs, dE};
    hipLaunchKernelGGL(k_gs_runs, dim3(P.nbk), dim3(GS_THREADS), 0, s, items, small, P.nbk, O);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    *done = true;
    return hipSuccess;
}

}  // namespace ctg
