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
// sort's large-segment path, so there is no size precondition.
#include <algorithm>

#include <rocprim/block/block_radix_sort.hpp>
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

// ---------------------------------------------------------------------------
// In-LDS bucket sort: after the MSD bucket pass, one workgroup per bucket
// sorts it in LDS (rocPRIM's block radix sort: 1024 threads x 8 items), so
// the keys make one HBM round trip after the bucket scatter.  A bucket of
// more than LS_CAP items is first split by its next key bits into
// sub-buckets (LDS histogram, scattered into the output range), each then
// sorted in LDS in place; a sub-bucket still above LS_CAP (heavy skew: one
// label adjacent to very many) raises *flag and the caller re-sorts with
// rocPRIM's device sort.  (key, value) pairs travel as one 64-bit item:
// (key bits below the bucket / sub-bucket bits) << 32 | value -- at most 32
// key bits remain, the sub-bucket split guarantees it.
// ---------------------------------------------------------------------------
constexpr int LS_IPT = 8;
constexpr int LS_MAX_SUB_BITS = 10;
template <int TH>
struct LsShared {
    typename rocprim::block_radix_sort<uint64_t, TH, LS_IPT>::storage_type sort;
    uint32_t cnt[1 << LS_MAX_SUB_BITS];          // sub-bucket counts, then cursors
    uint32_t off[(1 << LS_MAX_SUB_BITS) + 1];    // sub-bucket offsets
};

// item -> (key, value) and back; KEYS: the item is the key itself
template <bool PAIRS>
__device__ __forceinline__ uint64_t ls_item(uint64_t k, uint32_t v, int rem) {
    return PAIRS ? ((k & ((1ull << rem) - 1ull)) << 32) | v : k;
}

// sort items [i0, i0 + n) of (kin, vin) by key bits [lo, hi) of the item
// into (kout, vout) at the same positions; prefix = the key bits above `rem`
template <bool PAIRS, int TH>
__device__ void ls_sort_range(LsShared<TH>& sh, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                              uint32_t* vout, uint32_t i0, uint32_t n, int rem, uint64_t prefix, int lo_bit) {
    uint64_t it[LS_IPT];
    const uint32_t t = threadIdx.x;
    using LdsSort = rocprim::block_radix_sort<uint64_t, TH, LS_IPT>;
#pragma unroll
    for (int j = 0; j < LS_IPT; ++j) {
        const uint32_t i = t * LS_IPT + j;
        it[j] = i < n ? ls_item<PAIRS>(kin[i0 + i], PAIRS ? vin[i0 + i] : 0u, rem) : ~0ull;
    }
    // PAIRS: sort on the item bits [32, 32 + rem); KEYS: on [lo_bit, rem)
    const unsigned b0 = PAIRS ? 32u : (unsigned)lo_bit, b1 = PAIRS ? 32u + (unsigned)rem : (unsigned)rem;
    if (b1 > b0) LdsSort().sort(it, sh.sort, b0, b1);
#pragma unroll
    for (int j = 0; j < LS_IPT; ++j) {
        const uint32_t i = t * LS_IPT + j;
        if (i < n) {
            if constexpr (PAIRS) {
                kout[i0 + i] = prefix | (it[j] >> 32);
                vout[i0 + i] = (uint32_t)it[j];
            } else {
                kout[i0 + i] = it[j];
            }
        }
    }
    __syncthreads();   // the shared storage is reused by the next range
}

// one workgroup per bucket of the MSD pass (offs: bucket ranges in kin);
// key bits [lo_bit, shift) are sorted (KEYS: slot bits below lo_bit ride along)
template <bool PAIRS, int TH>
__global__ __launch_bounds__(TH) void k_bucket_lds_sort(const uint64_t* __restrict__ kin,
                                                                const uint32_t* __restrict__ vin,
                                                                uint64_t* __restrict__ kout,
                                                                uint32_t* __restrict__ vout,
                                                                const uint32_t* __restrict__ offs, int lo_bit,
                                                                int shift, uint32_t* __restrict__ flag) {
    constexpr uint32_t LS_CAP = TH * LS_IPT;
    __shared__ LsShared<TH> sh;
    const uint32_t b = blockIdx.x, b0 = offs[b], n = offs[b + 1] - b0;
    if (n == 0) return;
    const uint64_t bucket_prefix = (uint64_t)b << shift;
    // sub-bucket bits: enough for ~LS_CAP / 2 items per sub-bucket, and (pairs)
    // enough that at most 32 key bits remain below them
    int sb = 0;
    while (sb < LS_MAX_SUB_BITS && sb < shift - lo_bit && (n >> sb) > LS_CAP / 2) ++sb;
    if (n <= LS_CAP) sb = 0;
    if (PAIRS) sb = max(sb, shift - 32);
    if (sb > LS_MAX_SUB_BITS || (sb > 0 && sb > shift - lo_bit)) {
        if (threadIdx.x == 0) atomicOr(flag, 1u);
        return;
    }
    if (sb == 0) {
        ls_sort_range<PAIRS, TH>(sh, kin, vin, kout, vout, b0, n, shift, bucket_prefix, lo_bit);
        return;
    }
    // split by key bits [shift - sb, shift) into kout / vout (order within a
    // sub-bucket: any), then sort every sub-bucket in place
    const int rem = shift - sb;
    const uint32_t nsub = 1u << sb, smask = nsub - 1u;
    for (uint32_t i = threadIdx.x; i < nsub; i += TH) sh.cnt[i] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += TH)
        atomicAdd(&sh.cnt[(uint32_t)(kin[b0 + i] >> rem) & smask], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive prefix (nsub <= 1024: one thread is enough)
        uint32_t acc = 0;
        for (uint32_t i = 0; i < nsub; ++i) {
            sh.off[i] = acc;
            acc += sh.cnt[i];
            sh.cnt[i] = 0;
        }
        sh.off[nsub] = acc;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += TH) {
        const uint64_t k = kin[b0 + i];
        const uint32_t sbk = (uint32_t)(k >> rem) & smask;
        const uint32_t d = b0 + sh.off[sbk] + atomicAdd(&sh.cnt[sbk], 1u);
        kout[d] = k;
        if constexpr (PAIRS) vout[d] = vin[b0 + i];
    }
    __syncthreads();
    for (uint32_t q = 0; q < nsub; ++q) {
        const uint32_t s0 = sh.off[q], m = sh.off[q + 1] - s0;   // uniform
        if (m > LS_CAP) {
            if (threadIdx.x == 0) atomicOr(flag, 1u);
            return;
        }
        if (m > 1)   // (a single item is in place already)
            ls_sort_range<PAIRS, TH>(sh, kout, vout, kout, vout, b0 + s0, m, rem,
                                     bucket_prefix | ((uint64_t)q << rem), lo_bit);
    }
}

// the in-LDS sort of every bucket of an MSD pass (offs: nbk + 1 bucket bounds
// in kin); *flag (device u32) set -> some sub-bucket exceeded the LDS capacity
template <bool PAIRS>
static hipError_t bucket_lds_sort(const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout,
                                  const uint32_t* offs, uint32_t nbk, int64_t n, int lo_bit, int shift,
                                  uint32_t* flag, hipStream_t s) {
    hipError_t e = hipMemsetAsync(flag, 0, 4, s);
    if (e != hipSuccess) return e;
    if (n / nbk <= 1024)   // small buckets: 256-thread workgroups (2 K items each in LDS)
        hipLaunchKernelGGL((k_bucket_lds_sort<PAIRS, 256>), dim3(nbk), dim3(256), 0, s, kin, vin, kout, vout, offs,
                           lo_bit, shift, flag);
    else
        hipLaunchKernelGGL((k_bucket_lds_sort<PAIRS, 1024>), dim3(nbk), dim3(1024), 0, s, kin, vin, kout, vout,
                           offs, lo_bit, shift, flag);
    return hipGetLastError();
}

// CTG_LDS_SORT (read per call: tests and A/B switch it): 1 in-LDS bucket sort
// for keys and pairs, 0 rocPRIM's segmented sort of the buckets; unset: the
// in-LDS sort for (key, slot) pairs (2048^3: sort 1.80 -> 1.54 ms), rocPRIM's
// for packed keys (512^3: 0.074 vs 0.113 ms in LDS; profiles/r4/g)
static bool lds_sort_on(bool pairs) {
    const char* e = getenv("CTG_LDS_SORT");
    if (e) return e[0] == '1';
    return pairs;
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
    if (lds_sort_on(true)) {
        uint32_t* flag = small + 5 * (1 << BK_MAX_BITS) + 8;
        e = bucket_lds_sort<true>(ktmp, vtmp, kout, vout, offs, nbk, n, 0, shift, flag, s);
        if (e != hipSuccess) return e;
        uint32_t f = 0;
        if ((e = hipMemcpyAsync(&f, flag, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (!f) return hipSuccess;   // (else: skewed buckets -- the segmented sort below redoes all)
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
    if (lds_sort_on(false)) {
        uint32_t* flag = small + 5 * (1 << BK_MAX_BITS) + 8;
        e = bucket_lds_sort<false>(tmp, nullptr, out, nullptr, offs, nbk, n, lo_bit, shift, flag, s);
        if (e != hipSuccess) return e;
        uint32_t f = 0;
        if ((e = hipMemcpyAsync(&f, flag, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (!f) return hipSuccess;   // (else: skewed buckets -- the segmented sort below redoes all)
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

}  // namespace ctg
