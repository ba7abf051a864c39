// C ABI of libctg.so (include/ctg.h): host orchestration of the face scan,
// the record sort/reduction and the result handles.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <cstdio>
#include <map>
#include <mutex>

#include "ctg_internal.h"

namespace ctg {
hipError_t launch_face_scan(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s);
int scan_tile_rows();
int scan_tile_rows_narrow();
hipError_t launch_density(const void* L, int label_bits, const int64_t* shape, int n_rows, uint32_t* out,
                          hipStream_t s);
hipError_t launch_unique_tiles(const uint64_t* L, const int64_t* shape, const int64_t* b, const int64_t* e,
                               uint64_t* out, unsigned long long* count, int64_t cap, hipStream_t s);
hipError_t launch_pack_keys(int64_t n, const uint64_t* key, int nb, uint64_t* sk, uint32_t* idx, hipStream_t s);
hipError_t launch_pack_regions(const uint64_t* key, int64_t rcap, const RegionPrefix& pre, int nb, int ib, uint64_t* sk,
                               uint32_t* idx, hipStream_t s);
hipError_t launch_pack_pairs(int64_t n, const uint64_t* uv, int nb, uint64_t* sk, uint32_t* idx, hipStream_t s);
hipError_t bucket_sort_keys(const uint64_t* keys, uint64_t* tmp, uint64_t* out, int64_t n, int lo_bit, int hi_bit,
                            uint32_t* small, void** temp, size_t* temp_bytes, hipStream_t s);
hipError_t bucket_runs(const uint64_t* sorted, int64_t n, int lo_bit, int hi_bit, uint32_t* small, uint64_t* uniq,
                       uint32_t* runs, uint32_t* roffs, uint32_t* dE, hipStream_t s);
hipError_t bucket_sort_pairs(const uint64_t* keys, const uint32_t* vals, uint64_t* ktmp, uint32_t* vtmp,
                             uint64_t* kout, uint32_t* vout, int64_t n, int hi_bit, uint32_t* small, void** temp,
                             size_t* temp_bytes, hipStream_t s);
hipError_t group_sort_runs(const uint64_t* key, int64_t rcap, const RegionPrefix& pre, int64_t n, int nb, int ub,
                           int ib, uint64_t max_label, uint32_t* small, uint32_t* host_word, uint64_t* items,
                           uint32_t* perm, uint64_t* uniq, uint32_t* runs, uint32_t* roffs, uint32_t* dE,
                           bool* done, hipStream_t s);
hipError_t launch_max_pairs(int64_t n, const uint64_t* uv, unsigned long long* out, hipStream_t s);
hipError_t launch_reduce(int64_t E, const uint32_t* dE, const uint64_t* uniq, const uint32_t* runs,
                         const uint32_t* offs, const uint32_t* perm32, const uint64_t* perm64, int ib,
                         const RecordBuf& R, int wide, int stats, int nb, uint64_t umask, int need_adj,
                         int ignore_label, double scale, double offset, const ReduceOut& O, hipStream_t s, uint32_t* heavy = nullptr,
                         uint32_t* n_heavy = nullptr);
hipError_t launch_unique_blocks(const void* L, int label_bits, const BlockGeom* blocks, const uint32_t* tile_prefix,
                                int n_blocks, int64_t n_tiles, uint64_t* out, unsigned long long* count, int64_t cap,
                                hipStream_t s);
int unique_tile_y();
hipError_t launch_block_bounds(int64_t n, const uint64_t* col, int stride, int n_blocks, int shift, int64_t* bounds,
                               hipStream_t s);
hipError_t launch_clear_bits(int64_t n, uint64_t* col, int stride, uint64_t mask, hipStream_t s);
hipError_t launch_compact(int64_t E, const uint32_t* dE, const uint32_t* keep, const uint32_t* pos,
                          const ReduceOut& in, const ReduceOut& out, uint32_t* dkept, hipStream_t s);
hipError_t launch_endpoints(int64_t E, const uint64_t* uniq, int nb, uint32_t* out, hipStream_t s);
hipError_t launch_u32_to_u64(int64_t n, const uint32_t* in, uint64_t* out, hipStream_t s);
hipError_t launch_mark_nodes(int64_t E, const uint32_t* dE, const uint64_t* uniq, int nb, uint32_t* bits,
                             hipStream_t s);
hipError_t launch_bits_to_nodes(int64_t W, const uint32_t* bits, const uint32_t* off, uint64_t* nodes, uint32_t* dN,
                                hipStream_t s);
hipError_t launch_build_bloom(const uint64_t* edges, int64_t E, unsigned long long* words, uint32_t mask,
                              hipStream_t s);
hipError_t launch_find_edges(const uint64_t* ge, int64_t n, const uint64_t* q, int64_t m, int64_t* out,
                             hipStream_t s);
hipError_t launch_synth(uint64_t* labels, float* boundary, const int64_t* shape, int64_t z_offset,
                        const int64_t* gshape, int cell, uint64_t seed, uint64_t label_offset, double noise_amp,
                        hipStream_t s);
hipError_t launch_remap_dense(const uint64_t* L, int64_t V, const uint64_t* U, int64_t n, uint32_t* out,
                              hipStream_t s);
hipError_t launch_gather_labels(const uint64_t* U, uint64_t* x, int64_t n, hipStream_t s);
hipError_t launch_remap_dense64(const uint64_t* L, int64_t V, const uint64_t* U, int64_t n, uint64_t* out,
                                hipStream_t s);
hipError_t launch_synth_aff(const float* b, float* out, const int64_t* shape, int n_channels, const int32_t* off,
                            hipStream_t s);
hipError_t launch_row_keys(int64_t n, const uint64_t* ids, uint64_t begin, uint64_t end, uint32_t* key,
                           uint32_t* idx, uint32_t* bad, hipStream_t s);
hipError_t launch_merge_feature_rows(int64_t n, const uint32_t* key, const uint32_t* idx, const double* rows,
                                     double* out, hipStream_t s);

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// ---------------------------------------------------------------------------
// caching device allocator: results and scratch are recycled between calls so
// steady-state calls do no hipMalloc/hipFree
// ---------------------------------------------------------------------------
static std::mutex g_mu;
static std::multimap<size_t, void*> g_pool[64];

static int cur_dev() {
    int d = 0;
    hipGetDevice(&d);
    return d;
}

static size_t round_up(size_t b) {
    size_t r = 256;
    while (r < b) r = r < (1u << 20) ? r * 2 : r + (r >> 2);
    return r;
}

static void* dmalloc(size_t bytes) {
    if (bytes == 0) bytes = 256;
    bytes = round_up(bytes);
    const int d = cur_dev();
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto& pool = g_pool[d & 63];
        auto it = pool.lower_bound(bytes);
        if (it != pool.end() && it->first <= bytes * 2) {
            void* p = it->second;
            pool.erase(it);
            return p;
        }
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes + 64) != hipSuccess) {
        // release cached blocks and retry once
        std::lock_guard<std::mutex> g(g_mu);
        for (auto& kv : g_pool[d & 63]) hipFree(kv.second);
        g_pool[d & 63].clear();
        if (hipMalloc(&p, bytes + 64) != hipSuccess) return nullptr;
    }
    return p;
}

static std::map<void*, size_t> g_sizes;
static void* dalloc(size_t bytes) {
    bytes = round_up(bytes == 0 ? 256 : bytes);
    void* p = dmalloc(bytes);
    if (p) {
        std::lock_guard<std::mutex> g(g_mu);
        g_sizes[p] = bytes;
    }
    return p;
}
static void dfree(void* p) {
    if (!p) return;
    const int d = cur_dev();
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_sizes.find(p);
    size_t b = it == g_sizes.end() ? 256 : it->second;
    g_pool[d & 63].emplace(b, p);
}

void* dev_alloc(size_t bytes) { return dalloc(bytes); }
void dev_free(void* p) { dfree(p); }

void ensure(void** p, size_t& have, size_t need) {
    if (need <= have && *p) return;
    if (*p) dfree(*p);
    size_t n = std::max(need, have + have / 2);
    *p = dalloc(n);
    have = *p ? n : 0;
}

static Workspace g_ws[64];
Workspace& ws(int device) { return g_ws[device & 63]; }

// One workspace per device: calls that use it are serialised per device, so
// job threads may call the library concurrently (ctypes drops the GIL) --
// their N5 decode overlaps, their GPU work queues.  Recursive: the dense
// relabel and adjacency paths re-enter the C ABI.
static std::recursive_mutex g_dev_mu[64];
struct DevLock {
    std::lock_guard<std::recursive_mutex> g;
    DevLock() : g(g_dev_mu[cur_dev() & 63]) {}
};
int current_device() { return cur_dev(); }

static hipError_t ws_init(Workspace& w) {
    if (w.counters) return hipSuccess;
    hipError_t e = hipMalloc(&w.counters, sizeof(Counters));
    if (e != hipSuccess) return e;
    e = hipHostMalloc(&w.counters_host, sizeof(Counters), hipHostMallocDefault);
    if (e != hipSuccess) return e;
    e = hipMalloc(&w.small, 64 * sizeof(unsigned int));
    if (e != hipSuccess) return e;
    e = hipMalloc(&w.bsort, BK_SMALL_WORDS * sizeof(uint32_t));   // bucket sort scratch
    if (e != hipSuccess) return e;
    e = hipMalloc(&w.gsort, GS_SMALL_WORDS * sizeof(uint32_t));   // group sort scratch
    if (e != hipSuccess) return e;
    // the splitters stay in workspace memory: k_mgpu_bounds still reads them
    // after ctg_mgpu_split returns (a pool block freed there could be handed
    // to a call on another stream while that kernel runs)
    e = hipMalloc(&w.mgpu_spl, CTG_MGPU_MAX_WORLD * sizeof(uint64_t));
    if (e != hipSuccess) return e;
    e = hipHostMalloc(&w.small_host, 64 * sizeof(unsigned int), hipHostMallocDefault);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 10; ++i) hipEventCreate(&w.ev[i]);
    w.events = true;
    return hipSuccess;
}

static void free_records(Workspace& w) {
    dfree(w.rec.key);
    dfree(w.rec.sums);
    dfree(w.rec.hist);
    w.rec = RecordBuf{};
}

hipError_t ensure_records(Workspace& w, int64_t need, int wide) {
    ++w.gen;   // a scan is about to overwrite the records
    if (need <= w.rec.cap && w.rec.key) return hipSuccess;
    free_records(w);
    const int words = wide ? WREC_WORDS : NREC_STRIDE;
    w.rec.key = (uint64_t*)dalloc((size_t)need * 8);
    w.rec.sums = wide ? (double2*)dalloc((size_t)need * 16) : nullptr;
    w.rec.hist = (uint32_t*)dalloc((size_t)need * words * 4);
    if (!w.rec.key || (wide && !w.rec.sums) || !w.rec.hist) return hipErrorOutOfMemory;
    w.rec.cap = need;
    w.rec.rcap = need / NREG;
    return hipSuccess;
}

static int bits_for(uint64_t v) {
    int b = 1;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

struct Ev {
    Workspace& w;
    hipStream_t s;
    void mark(int i) {
        if (w.profiling) hipEventRecord(w.ev[i], s);
    }
};

// rocPRIM call with the shared temp buffer: size query (t == nullptr), grow, run.
// CALL must use the names ``t`` (void*) and ``tbytes`` (size_t&).
#define ROCPRIM_CALL(w, CALL)                                     \
    do {                                                          \
        void* t = nullptr;                                        \
        size_t tbytes = 0;                                        \
        hipError_t e_ = (CALL);                                   \
        if (e_ != hipSuccess) return e_;                          \
        ensure(&(w).temp, (w).temp_bytes, tbytes + 256);          \
        if (!(w).temp) return hipErrorOutOfMemory;                \
        t = (w).temp;                                             \
        tbytes = (w).temp_bytes;                                  \
        e_ = (CALL);                                              \
        if (e_ != hipSuccess) return e_;                          \
    } while (0)

// Record sort: (u,v) keys packed to 2*nb bits (34 at 1.3e5 labels).  rocPRIM's
// gfx950 default sorts 8 bits per onesweep pass (5 passes at 34 bits, each a
// launch with its own decoupled look-back); 10-bit digits cut that to 4 (34 bits)
// and the sort from 0.185 to 0.151 ms at 512^3 (11+ bits exceed the LDS of the
// histogram kernel).
#ifndef CTG_SORT_BITS
#define CTG_SORT_BITS 10
#endif
#ifndef CTG_SORT_BLOCK
#define CTG_SORT_BLOCK 1024
#endif
#ifndef CTG_SORT_IPT
#define CTG_SORT_IPT 8
#endif
#if CTG_SORT_BITS
using RecordSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 16>,
                                        rocprim::kernel_config<CTG_SORT_BLOCK, CTG_SORT_IPT>, CTG_SORT_BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;
#else
using RecordSortConfig = rocprim::default_config;
#endif
// The wide digits pay off for small sorts (launch / look-back bound: 1.9 M
// records at 512^3: 0.185 -> 0.151 ms; 27.8 M at 2048^3: 1.88 -> 1.49 ms) and
// lose for very large ones (298 M records of configs[4]:
// 14.1 -> 18.7 ms, the 1024-way scatter coalesces worse), so they are used up
// to this many records.
static bool sort_packed() {
    const char* e = getenv("CTG_SORT_PACKED");   // read per call: tests switch it
    return !(e && e[0] == '0');
}
static bool bucket_sort() {
    const char* e = getenv("CTG_BUCKET_SORT");   // read per call: A/B and tests switch it
    return !(e && e[0] == '0');
}
// The pair path's bucket sort pays up to ~30 M records (1024^3 3-channel: 1.09 -> 1.00 ms at
// 15.6 M; 2048^3: equal at 28 M) and loses on configs[4]'s 190 M (9.5 -> 12.8 ms: buckets of
// ~46 K records go to the segmented sort's slower large-segment path); CTG_BUCKET_SORT_PAIRS=0/1 forces it.
static bool bucket_sort_pairs_on(int64_t n) {
    const char* e = getenv("CTG_BUCKET_SORT_PAIRS");
    if (e) return e[0] == '1';
    // up to ~32 M records (configs[4]'s 138 M: onesweep 6.7 ms against 9.3 ms for the bucket pass with
    // the in-LDS sort of ~34 K-record buckets split into sub-buckets; profiles/r4/g)
    return n <= (int64_t)(32 << 20);
}
// CTG_GROUP_SORT=0: the (key, slot) scan records take the bucket / onesweep paths
static bool group_sort_on() {
    const char* e = getenv("CTG_GROUP_SORT");   // read per call: tests switch it
    return !(e && e[0] == '0');
}
static int64_t sort_wide_digits_max() { return (int64_t)(64 << 20); }

// ---------------------------------------------------------------------------
// shared back half: records (n, with keys (u<<32|v) or (u,v) pairs) -> result
// ---------------------------------------------------------------------------
struct ReduceJob {
    int64_t n;                 // records
    const uint64_t* keys;      // packed (u<<32)|v, or null if pairs given
    const uint64_t* pairs;     // (u,v) pairs
    RecordBuf R;
    int wide, stats, need_adj, ignore_label, keep_stats;
    uint64_t max_v;
    double scale, offset;
    int64_t single_label_nodes;  // >=0: no edges -> nodes = this label; -1: none
    const uint64_t* single_label_ptr;  // device pointer to a label to use if E == 0
    const RegionPrefix* regions;       // keys in NREG regions of R (scan records), or null: dense
    int ub = 0;                        // bits of the key's u field (0: = bits of the largest label)
    uint64_t umask = ~0ull;            // label bits of u (batched blocks: below the block tag)
    int skip_nodes = 0;                // batched blocks: nodes come from the per-block unique pass
    int defer_stats = 0;               // CTG_DEFER_STATS (with keep_stats)
};

static hipError_t reduce_records(Workspace& w, const ReduceJob& J, hipStream_t s, ctg_result* res) {
    // Device-resident counts: the run count E_all, the kept edge count E and
    // the node count N stay in w.small[0..2] until one read-back at the end;
    // every kernel in between bounds itself by them, and buffers are sized by
    // the record count n (an upper bound), so the back half issues no
    // host synchronisation (except on the rare node path for labels >= 2^30).
    Ev ev{w, s};
    ++w.gen;   // the sort / run buffers are about to be overwritten
    const int64_t n = J.n;
    const int nb = bits_for(J.max_v);
    const int ub = J.ub ? J.ub : nb;
    if (nb > 32 || ub > 32) return hipErrorInvalidValue;
    if (n == 0) {
        res->n_edges = 0;
        res->edges = (uint64_t*)dalloc(16);
        res->features = J.stats ? (double*)dalloc(N_FEATURES * 8) : nullptr;
        if (J.keep_stats && J.stats) {
            res->stats = (uint32_t*)dalloc(WREC_WORDS * 4);
            res->stat_sums = (double2*)dalloc(16);
        }
        res->nodes = (uint64_t*)dalloc(8);
        res->n_nodes = 0;
        if (J.single_label_ptr) {
            hipError_t e = hipMemcpyAsync(res->nodes, J.single_label_ptr, 8, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return e;
            res->n_nodes = 1;
        }
        for (int i = 2; i <= 6; ++i) ev.mark(i);
        return hipStreamSynchronize(s);
    }
    // sort buffers
    if (n > w.sort_cap) {
        dfree(w.sk_in); dfree(w.sk_out); dfree(w.idx_in); dfree(w.idx_out);
        dfree(w.uniq); dfree(w.runs); dfree(w.offs); dfree(w.keep); dfree(w.pos);
        const int64_t cap = std::max<int64_t>(n, w.sort_cap + w.sort_cap / 2);
        w.sk_in = (uint64_t*)dalloc(cap * 8); w.sk_out = (uint64_t*)dalloc(cap * 8);
        w.idx_in = (uint32_t*)dalloc(cap * 4); w.idx_out = (uint32_t*)dalloc(cap * 4);
        w.uniq = (uint64_t*)dalloc(cap * 8); w.runs = (uint32_t*)dalloc(cap * 4);
        w.offs = (uint32_t*)dalloc(cap * 4); w.keep = (uint32_t*)dalloc(cap * 4);
        w.pos = (uint32_t*)dalloc(cap * 4);
        if (!w.sk_in || !w.sk_out || !w.idx_in || !w.idx_out || !w.uniq || !w.runs || !w.offs || !w.keep || !w.pos)
            return hipErrorOutOfMemory;
        w.sort_cap = cap;
    }
    uint32_t* dE_all = w.small;
    uint32_t* dE = w.small + 1;
    uint32_t* dN = w.small + 2;
    hipError_t e;
    // Scan records whose slot fits beside the 2*nb key bits sort as bare u64
    // keys (slot in the low ib bits): 16 instead of 24 bytes per record and
    // pass; the reduction reads the slots from the sorted keys (CTG_SORT_PACKED=0 disables).
    const int ib = J.regions ? bits_for((uint64_t)std::max<int64_t>(J.R.cap - 1, 1)) : 0;
    // at most 63 bits: with the record slot packed up to bit 63 exactly, the
    // sorted order came out wrong (tests/test_gpu_blocks.py::
    // test_blocks_independent_of_workspace_history), so one bit stays free
    const bool packed = J.keys && J.regions && sort_packed() && ub + nb + ib <= 63 && n <= sort_wide_digits_max();
    // the bucket passes need keys spread over their top bits: block-tagged keys
    // (ctg_rag_blocks, J.ub set) put the block id there and fill a few huge
    // buckets (configs[0] device time 3.9 -> 6.7 ms), so they keep onesweep
    const bool spread = J.ub == 0;
    // (key, slot) scan records: the group sort reads the record regions itself
    // (no pack pass) and writes the run table and the slot permutation
    bool grouped = false;
    if (J.keys && J.regions && !packed && spread && group_sort_on()) {
        ev.mark(2);   // (phases: the whole group sort is "sort")
        e = group_sort_runs(J.keys, J.R.rcap, *J.regions, n, nb, ub, ib, J.max_v, w.gsort, w.small_host + 16, w.sk_out,
                            w.idx_out, w.uniq, w.runs, w.offs, dE_all, &grouped, s);
        if (e != hipSuccess) return e;
        if (grouped) ev.mark(3);
    }
    if (grouped) {
    } else if (J.keys && J.regions)
        e = launch_pack_regions(J.keys, J.R.rcap, *J.regions, nb, packed ? ib : 0, w.sk_in, w.idx_in, s);
    else if (J.keys) e = launch_pack_keys(n, J.keys, nb, w.sk_in, w.idx_in, s);
    else e = launch_pack_pairs(n, J.pairs, nb, w.sk_in, w.idx_in, s);
    if (e != hipSuccess) return e;
    if (!grouped) ev.mark(2);
    bool have_offs = grouped;     // run offsets already written (bucket / group path)
    bool pairs_done = grouped;    // pair sort + runs done by the bucket / group path
    if (grouped) {
    } else if (packed && spread && bucket_sort()) {
        // MSD bucket pass + segmented sort of the key bits (ctg_sort.hip):
        // 4 fused launches instead of 4 onesweep passes with their fills
        e = bucket_sort_keys(w.sk_in, w.uniq, w.sk_out, n, ib, ib + ub + nb, w.bsort, &w.temp, &w.temp_bytes, s);
        if (e != hipSuccess) return e;
        ev.mark(3);
        // runs from the buckets: unique keys, lengths and offsets in one go
        e = bucket_runs(w.sk_out, n, ib, ib + ub + nb, w.bsort, w.uniq, w.runs, w.offs, dE_all, s);
        if (e != hipSuccess) return e;
        have_offs = true;
    } else if (packed) {
        ROCPRIM_CALL(w, rocprim::radix_sort_keys<RecordSortConfig>(t, tbytes, w.sk_in, w.sk_out, (size_t)n,
                                                                   (unsigned)ib, (unsigned)(ib + ub + nb), s));
        ev.mark(3);
        auto key_only = rocprim::make_transform_iterator(w.sk_out, [ib] __device__(uint64_t k) { return k >> ib; });
        ROCPRIM_CALL(w, rocprim::run_length_encode(t, tbytes, key_only, (unsigned)n, w.uniq, w.runs, dE_all, s));
    } else if (spread && bucket_sort_pairs_on(n)) {
        // tmp buffers: w.uniq (keys) and w.keep (values) are free until the
        // run-length pass / the reduction
        e = bucket_sort_pairs(w.sk_in, w.idx_in, w.uniq, w.keep, w.sk_out, w.idx_out, n, ub + nb, w.bsort, &w.temp,
                              &w.temp_bytes, s);
        if (e != hipSuccess) return e;
        ev.mark(3);
        // runs never cross the MSD buckets: unique keys, lengths and offsets per bucket
        e = bucket_runs(w.sk_out, n, 0, ub + nb, w.bsort, w.uniq, w.runs, w.offs, dE_all, s);
        if (e != hipSuccess) return e;
        have_offs = true;
        pairs_done = true;
    } else if (n <= sort_wide_digits_max()) {
        ROCPRIM_CALL(w, rocprim::radix_sort_pairs<RecordSortConfig>(t, tbytes, w.sk_in, w.sk_out, w.idx_in,
                                                                    w.idx_out, (size_t)n, 0u, (unsigned)(ub + nb), s));
    } else {
        ROCPRIM_CALL(w, rocprim::radix_sort_pairs(t, tbytes, w.sk_in, w.sk_out, w.idx_in, w.idx_out, (size_t)n, 0u,
                                                  (unsigned)(ub + nb), s));
    }
    if (!packed && !pairs_done) {
        ev.mark(3);
        ROCPRIM_CALL(w, rocprim::run_length_encode(t, tbytes, w.sk_out, (unsigned)n, w.uniq, w.runs, dE_all, s));
    }
    // offsets over the n-bound: entries past E_all are never read
    if (!have_offs)
        ROCPRIM_CALL(w, rocprim::exclusive_scan(t, tbytes, w.runs, w.offs, 0u, (size_t)n, rocprim::plus<uint32_t>(),
                                                s));
    ev.mark(4);

    // outputs (uncompacted), sized by the bound n
    const bool may_drop = J.need_adj || J.ignore_label;
    // CTG_DEFER_STATS: result row e is run e of the records (no compaction),
    // whose statistics the exchange rebuilds where it needs them
    const bool defer = J.defer_stats && J.keep_stats && J.stats && !J.wide && !may_drop;
    ReduceOut O{};
    O.edges = (uint64_t*)dalloc(n * 16);
    O.feats = J.stats ? (double*)dalloc(n * N_FEATURES * 8) : nullptr;
    O.keep = may_drop ? w.keep : nullptr;
    if (J.keep_stats && J.stats && !defer) {
        O.wstats = (uint32_t*)dalloc(n * WREC_WORDS * 4);
        O.wsums = (double2*)dalloc(n * 16);
    }
    if (!O.edges || (J.stats && !O.feats)) return hipErrorOutOfMemory;
    O.count_out = may_drop ? nullptr : dE;   // no compaction: the kernel copies the count
#ifdef CTG_DIAG   // diagnostic reduce ablations exist only in diagnostic builds (make variant EXTRA=-DCTG_DIAG)
    {
        static const int ablate = [] { const char* v = getenv("CTG_REDUCE_ABLATE"); return v ? atoi(v) : 0; }();
        O.ablate = ablate;
    }
#else
    O.ablate = 0;
#endif
    // features-only narrow reduce: edges past 2^16 samples are listed for the
    // wide-histogram kernel (w.small[40]: their count)
    uint32_t* heavy = (!J.wide && J.stats && !O.wstats) ? (uint32_t*)dalloc(n * 4) : nullptr;
    e = launch_reduce(n, dE_all, w.uniq, w.runs, w.offs, packed ? nullptr : w.idx_out, packed ? w.sk_out : nullptr,
                      packed ? ib : 0, J.R, J.wide, J.stats, nb, J.umask, J.need_adj, J.ignore_label, J.scale, J.offset,
                      O, s, heavy, heavy ? w.small + 40 : nullptr);
    dfree(heavy);   // stream-ordered reuse
    if (e != hipSuccess) return e;
    if (may_drop) {
        ROCPRIM_CALL(w, rocprim::exclusive_scan(t, tbytes, w.keep, w.pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
        ReduceOut C2{};
        C2.edges = (uint64_t*)dalloc(n * 16);
        C2.feats = O.feats ? (double*)dalloc(n * N_FEATURES * 8) : nullptr;
        if (O.wstats) {
            C2.wstats = (uint32_t*)dalloc(n * WREC_WORDS * 4);
            C2.wsums = (double2*)dalloc(n * 16);
        }
        e = launch_compact(n, dE_all, w.keep, w.pos, O, C2, dE, s);
        if (e != hipSuccess) return e;
        dfree(O.edges); dfree(O.feats); dfree(O.wstats); dfree(O.wsums);   // stream-ordered reuse
        O = C2;
    }
    ev.mark(5);
    res->edges = O.edges;
    res->features = O.feats;
    res->stats = O.wstats;
    if (defer) {
        res->defer.on = 1;
        res->defer.offs = w.offs;
        res->defer.runs = w.runs;
        res->defer.perm = Perm{packed ? nullptr : w.idx_out, packed ? w.sk_out : nullptr, packed ? ib : 0};
        res->defer.hist = J.R.hist;
        res->defer.gen = w.gen;
    }
    res->stat_sums = O.wsums;

    // nodes = unique endpoints of every unique key (before filtering)
    uint32_t counts[3] = {0, 0, 0};
    if (J.skip_nodes) {
        res->nodes = (uint64_t*)dalloc(8);
        e = hipMemcpyAsync(w.small_host, w.small, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        counts[0] = w.small_host[0];
        counts[1] = w.small_host[1];
    } else if (J.max_v < (1ull << 30)) {
        // bitmap over [0, max label]: one pass over the sorted key table
        const int64_t W = (int64_t)(J.max_v >> 5) + 1;
        uint32_t* bits = (uint32_t*)dalloc(W * 4);
        uint32_t* off = (uint32_t*)dalloc(W * 4);
        res->nodes = (uint64_t*)dalloc(std::min<int64_t>(W * 32, 2 * n) * 8);
        if (!bits || !off || !res->nodes) return hipErrorOutOfMemory;
        e = hipMemsetAsync(bits, 0, W * 4, s);
        if (e != hipSuccess) return e;
        e = launch_mark_nodes(n, dE_all, w.uniq, nb, bits, s);
        if (e != hipSuccess) return e;
        // word offsets = exclusive scan of the words' popcounts (read through the scan's input iterator)
        // (tried: the scan and the expansion in one workgroup for small label ranges -- 0.053 -> 0.115 ms
        // at 512^3, the serial per-thread expansion loses to the wide launch)
        auto popc = rocprim::make_transform_iterator(bits, [] __device__(uint32_t b) { return (uint32_t)__popc(b); });
        ROCPRIM_CALL(w, rocprim::exclusive_scan(t, tbytes, popc, off, 0u, (size_t)W, rocprim::plus<uint32_t>(), s));
        e = launch_bits_to_nodes(W, bits, off, res->nodes, dN, s);
        if (e != hipSuccess) return e;
        e = hipMemcpyAsync(w.small_host, w.small, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        for (int i = 0; i < 3; ++i) counts[i] = w.small_host[i];
        dfree(bits); dfree(off);
    } else {
        e = hipMemcpyAsync(w.small_host, w.small, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        counts[0] = w.small_host[0];
        counts[1] = w.small_host[1];
        const int64_t E_all = counts[0];
        uint32_t* ep = (uint32_t*)dalloc(std::max<int64_t>(E_all, 1) * 8);
        uint32_t* ep2 = (uint32_t*)dalloc(std::max<int64_t>(E_all, 1) * 8);
        uint32_t* nodes32 = (uint32_t*)dalloc(std::max<int64_t>(E_all, 1) * 8);
        if (!ep || !ep2 || !nodes32) return hipErrorOutOfMemory;
        e = launch_endpoints(E_all, w.uniq, nb, ep, s);
        if (e != hipSuccess) return e;
        ROCPRIM_CALL(w, rocprim::radix_sort_keys(t, tbytes, ep, ep2, (size_t)(2 * E_all), 0u, (unsigned)nb, s));
        ROCPRIM_CALL(w, rocprim::unique(t, tbytes, ep2, nodes32, dN, (size_t)(2 * E_all),
                                        rocprim::equal_to<uint32_t>(), s));
        e = hipMemcpyAsync(w.small_host + 2, dN, 4, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        counts[2] = w.small_host[2];
        res->nodes = (uint64_t*)dalloc(std::max<int64_t>(counts[2], 1) * 8);
        e = launch_u32_to_u64(counts[2], nodes32, res->nodes, s);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        dfree(ep); dfree(ep2); dfree(nodes32);
    }
    res->n_edges = counts[1];
    res->n_nodes = counts[2];
    if (counts[0] == 0) {   // no edge at all: the owned origin voxel's label is the only node
        res->n_nodes = 0;
        if (J.single_label_ptr) {
            e = hipMemcpyAsync(res->nodes, J.single_label_ptr, 8, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return e;
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            res->n_nodes = 1;
        }
    }
    ev.mark(6);
    return hipSuccess;
}

}  // namespace ctg

using namespace ctg;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int ctg_version(void) { return 1; }

const char* ctg_last_error(void) { return g_err.c_str(); }

int ctg_mgpu_slab(int64_t Z, int world_size, int rank, const int64_t* offsets, int n_channels, int64_t* out) {
    if (Z <= 0 || world_size <= 0 || rank < 0 || rank >= world_size || !out || n_channels < 0 ||
        (n_channels > 0 && !offsets)) {
        set_error("ctg_mgpu_slab: invalid arguments");
        return CTG_ERR_ARG;
    }
    if (world_size > Z) {
        set_error("ctg_mgpu_slab: more ranks than z planes");
        return CTG_ERR_ARG;
    }
    int64_t down = 1, up = 0;   // planes a face / partner reaches below and above a voxel
    for (int c = 0; c < n_channels; ++c) {
        down = std::max<int64_t>(down, -offsets[3 * c]);
        up = std::max<int64_t>(up, offsets[3 * c]);
    }
    if (up > 0 && world_size > 1) {
        set_error("ctg_mgpu_slab: positive z offsets need an upper halo, which the z-slab layout does not have");
        return CTG_ERR_UNSUPPORTED;
    }
    const int64_t z0 = Z * rank / world_size, z1 = Z * (rank + 1) / world_size;
    out[0] = z0 - std::min(down, z0);
    out[1] = z0;
    out[2] = z1;
    return CTG_OK;
}

static bool mgpu_args(const ctg_result* r, int world, const char* who) {
    if (!r || world <= 0 || world > CTG_MGPU_MAX_WORLD) {
        set_error(std::string(who) + ": bad arguments (world size must be 1.." +
                  std::to_string(CTG_MGPU_MAX_WORLD) + ")");
        return false;
    }
    return true;
}

int ctg_mgpu_sample(const ctg_result* local, int64_t* meta, void* stream) {
    DevLock dev_lock;
    if (!mgpu_args(local, 1, "ctg_mgpu_sample") || !meta) return CTG_ERR_ARG;
    CTG_CHECK(mgpu_sample(local->edges, local->n_edges, meta, (hipStream_t)stream));
    return CTG_OK;
}

int ctg_mgpu_split(const ctg_result* local, const int64_t* meta_all, int world_size, int64_t* counts, void* stream) {
    DevLock dev_lock;
    if (!mgpu_args(local, world_size, "ctg_mgpu_split") || !meta_all || !counts) return CTG_ERR_ARG;
    Workspace& w = ws(cur_dev());
    CTG_CHECK(ws_init(w));
    CTG_CHECK(mgpu_split(local->edges, local->n_edges, local->nodes, local->n_nodes, meta_all, world_size,
                         w.mgpu_spl, counts, (hipStream_t)stream));
    return CTG_OK;
}

int ctg_mgpu_pack(const ctg_result* local, const int64_t* counts_all, int world_size, int rank, int64_t* send,
                  void* stream) {
    DevLock dev_lock;
    if (!mgpu_args(local, world_size, "ctg_mgpu_pack") || !counts_all || rank < 0 || rank >= world_size)
        return CTG_ERR_ARG;
    const int64_t* mine = counts_all + (int64_t)rank * world_size * 2;
    int64_t rows = 0, nodes = 0, words = 0;
    for (int d = 0; d < world_size; ++d) {
        rows += mine[2 * d];
        nodes += mine[2 * d + 1];
        if (d != rank) words += mine[2 * d] * CTG_MGPU_ROW_WORDS + mine[2 * d + 1];
    }
    if (rows != local->n_edges || nodes != local->n_nodes) {
        set_error("ctg_mgpu_pack: counts do not cover this rank's table");
        return CTG_ERR_ARG;
    }
    if (words > 0 && (!send || (!(local->stats && local->stat_sums) && !local->defer.on))) {
        set_error("ctg_mgpu_pack: rows to send need a CTG_KEEP_STATS table and a send buffer");
        return CTG_ERR_ARG;
    }
    if (words > 0 && local->defer.on && local->defer.gen != ws(local->device).gen) {
        set_error("ctg_mgpu_pack: the CTG_DEFER_STATS table's records were overwritten by a later call");
        return CTG_ERR_STALE;
    }
    CTG_CHECK(mgpu_pack(local, counts_all, world_size, rank, send, (hipStream_t)stream));
    return CTG_OK;
}

int ctg_mgpu_merge(ctg_result* local, const int64_t* recv, const int64_t* counts_all, int world_size, int rank,
                   double hist_lo, double hist_hi, void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!mgpu_args(local, world_size, "ctg_mgpu_merge") || !counts_all || !out || rank < 0 || rank >= world_size ||
        !(hist_hi > hist_lo))
        return CTG_ERR_ARG;
    *out = nullptr;
    if (!local->owned.empty()) {   // a shard's arrays are interior pointers of its owned blocks
        set_error("ctg_mgpu_merge: the local table is itself a merge shard; pass the rank's local call");
        return CTG_ERR_ARG;
    }
    int64_t rows = 0, nodes = 0, recv_words = 0;
    for (int d = 0; d < world_size; ++d) {
        rows += counts_all[((int64_t)rank * world_size + d) * 2];
        nodes += counts_all[((int64_t)rank * world_size + d) * 2 + 1];
        if (d != rank)
            recv_words += counts_all[((int64_t)d * world_size + rank) * 2] * CTG_MGPU_ROW_WORDS +
                          counts_all[((int64_t)d * world_size + rank) * 2 + 1];
    }
    if (rows != local->n_edges || nodes != local->n_nodes) {
        set_error("ctg_mgpu_merge: counts do not cover this rank's table");
        return CTG_ERR_ARG;
    }
    if (recv_words > 0 && !recv) {
        set_error("ctg_mgpu_merge: null receive buffer");
        return CTG_ERR_ARG;
    }
    if (recv_words > 0 && local->defer.on && local->defer.gen != ws(local->device).gen) {
        set_error("ctg_mgpu_merge: the CTG_DEFER_STATS table's records were overwritten by a later call");
        return CTG_ERR_STALE;
    }
    Workspace& w = ws(cur_dev());
    CTG_CHECK(ws_init(w));
    ctg_result* r = new ctg_result();
    r->device = cur_dev();
    int lib_rc = CTG_OK;
    const hipError_t e = mgpu_merge(local, recv, counts_all, world_size, rank, hist_lo, hist_hi,
                                    (hipStream_t)stream, r, &lib_rc);
    if (lib_rc != CTG_OK) {   // the message is set already
        ctg_free(r);
        return lib_rc;
    }
    if (e != hipSuccess) {
        set_error(std::string("ctg_mgpu_merge: ") + hipGetErrorString(e));
        ctg_free(r);
        return e == hipErrorOutOfMemory ? CTG_ERR_NOMEM : CTG_ERR_HIP;
    }
    local->n_edges = 0;
    local->n_nodes = 0;
    *out = r;
    return CTG_OK;
}

int ctg_device_count(int* count) {
    CTG_CHECK(hipGetDeviceCount(count));
    return CTG_OK;
}

int ctg_init(int device) {
    int n = 0;
    std::lock_guard<std::recursive_mutex> init_lock(g_dev_mu[device & 63]);
    CTG_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) {
        set_error("ctg_init: invalid device " + std::to_string(device));
        return CTG_ERR_ARG;
    }
    CTG_CHECK(hipSetDevice(device));
    CTG_CHECK(ws_init(ws(device)));
    return CTG_OK;
}

int ctg_trim(void) {
    DevLock dev_lock;
    // hand every cached device block of the current device back to HIP: the
    // workspace (records, sort scratch, staging) and the allocator's pool
    const int d = cur_dev();
    Workspace& w = ws(d);
    CTG_CHECK(hipDeviceSynchronize());
    free_records(w);
    dfree(w.sk_in); dfree(w.sk_out); dfree(w.idx_in); dfree(w.idx_out);
    dfree(w.uniq); dfree(w.runs); dfree(w.offs); dfree(w.keep); dfree(w.pos);
    w.sk_in = w.sk_out = w.uniq = nullptr;
    w.idx_in = w.idx_out = w.runs = w.offs = w.keep = w.pos = nullptr;
    w.sort_cap = 0;
    dfree(w.temp);
    w.temp = nullptr;
    w.temp_bytes = 0;
    for (int i = 0; i < 2; ++i) {
        dfree(w.stage[i]);
        w.stage[i] = nullptr;
        w.stage_bytes[i] = 0;
    }
    std::lock_guard<std::mutex> g(g_mu);
    for (auto& kv : g_pool[d & 63]) {
        g_sizes.erase(kv.second);
        CTG_CHECK(hipFree(kv.second));
    }
    g_pool[d & 63].clear();
    return CTG_OK;
}

int ctg_set_profiling(int on) {
    ws(cur_dev()).profiling = on;
    return CTG_OK;
}

int ctg_last_timings(double* ms, int n) {
    Workspace& w = ws(cur_dev());
    for (int i = 0; i < n && i < 8; ++i) ms[i] = w.last_ms[i];
    return CTG_OK;
}

static int stage_in(Workspace& w, int slot, const void* src, size_t bytes, int mem, hipStream_t s,
                    const void** dev) {
    if (mem == CTG_MEM_DEVICE || src == nullptr) {
        *dev = src;
        return CTG_OK;
    }
    ensure(&w.stage[slot], w.stage_bytes[slot], bytes);
    if (!w.stage[slot]) {
        set_error("out of device memory staging input");
        return CTG_ERR_NOMEM;
    }
    CTG_CHECK(hipMemcpyAsync(w.stage[slot], src, bytes, hipMemcpyHostToDevice, s));
    *dev = w.stage[slot];
    return CTG_OK;
}

// (u,v) pair lists with labels >= 2^32 (merge / union inputs): the sort packs
// (u,v) into one 64-bit key, so the endpoints are replaced by their rank in
// the sorted unique endpoint table (monotone) and mapped back afterwards.
struct DensePairs {
    ctg_result* U = nullptr;
    uint64_t* dense = nullptr;
    int build(const uint64_t* dk, int64_t n, hipStream_t s) {
        int rc = ctg_unique_values(dk, 2 * n, CTG_MEM_DEVICE, s, &U);
        if (rc) return rc;
        dense = (uint64_t*)dalloc((size_t)n * 16);
        if (!dense) {
            set_error("out of device memory for the dense endpoint relabelling");
            return CTG_ERR_NOMEM;
        }
        CTG_CHECK(launch_remap_dense64(dk, 2 * n, U->nodes, U->n_nodes, dense, s));
        return CTG_OK;
    }
    hipError_t map_back(ctg_result* r, hipStream_t s) {
        if (!U) return hipSuccess;
        hipError_t e = launch_gather_labels(U->nodes, r->edges, 2 * r->n_edges, s);
        if (e == hipSuccess) e = launch_gather_labels(U->nodes, r->nodes, r->n_nodes, s);
        return e;
    }
    ~DensePairs() {
        if (dense) dfree(dense);   // stream-ordered reuse
        if (U) ctg_free(U);
    }
};

// The dense relabellings below map a label to its rank in the sorted unique
// label table U.  The reduce recognises the ignore label as dense id 0, so with
// ignore_label set the table must start with label 0 even where the array
// holds no 0 -- else the smallest real label would become 0 and its edges
// would be dropped.  Puts a 0 in front of U->nodes when U[0] != 0.
static int keep_zero_first(ctg_result* U, hipStream_t s) {
    uint64_t first = 0;
    if (U->n_nodes > 0) {
        CTG_CHECK(hipMemcpyAsync(&first, U->nodes, 8, hipMemcpyDeviceToHost, s));
        CTG_CHECK(hipStreamSynchronize(s));
    }
    if (U->n_nodes > 0 && first == 0) return CTG_OK;
    uint64_t* t = (uint64_t*)dalloc((size_t)(U->n_nodes + 1) * 8);
    if (!t) {
        set_error("out of device memory for the dense relabelling table");
        return CTG_ERR_NOMEM;
    }
    CTG_CHECK(hipMemsetAsync(t, 0, 8, s));
    if (U->n_nodes)
        CTG_CHECK(hipMemcpyAsync(t + 1, U->nodes, (size_t)U->n_nodes * 8, hipMemcpyDeviceToDevice, s));
    dfree(U->nodes);   // stream-ordered reuse
    U->nodes = t;
    U->n_nodes += 1;
    return CTG_OK;
}

// Labels >= 2^32: the face keys pack (u,v) as 32+32 bits, so the
// array is relabelled densely through its sorted unique labels (a monotone
// map: sorted dense edges stay sorted), scanned as 32-bit labels, and the
// edge and node tables are mapped back.
static int rag_dense_relabel(const void* dl, const void* dd, int data_kind, int n_channels, const int32_t* offsets,
                             const int64_t* shape, const int64_t* own_begin, const int64_t* own_end,
                             int ignore_label, double hist_lo, double hist_hi, int flags, void* stream,
                             ctg_result** out) {
    hipStream_t s = (hipStream_t)stream;
    ctg_result* U = nullptr;
    int rc = ctg_unique_labels((const uint64_t*)dl, shape, nullptr, nullptr, CTG_MEM_DEVICE, stream, &U);
    if (rc) return rc;
    if (ignore_label && (rc = keep_zero_first(U, s)) != CTG_OK) {
        ctg_free(U);
        return rc;
    }
    if (U->n_nodes > 0xFFFFFFFFll) {
        ctg_free(U);
        set_error("ctg_rag_features: more than 2^32 distinct labels in one array");
        return CTG_ERR_UNSUPPORTED;
    }
    const int64_t V = shape[0] * shape[1] * shape[2];
    uint32_t* dense = (uint32_t*)dalloc((size_t)V * 4);
    if (!dense) {
        ctg_free(U);
        set_error("ctg_rag_features: out of device memory for the dense relabelling");
        return CTG_ERR_NOMEM;
    }
    CTG_CHECK(launch_remap_dense((const uint64_t*)dl, V, U->nodes, U->n_nodes, dense, s));
    ctg_result* r = nullptr;
    rc = ctg_rag_features(dense, 32, dd, data_kind, n_channels, offsets, shape, own_begin, own_end, ignore_label,
                          hist_lo, hist_hi, flags, CTG_MEM_DEVICE, stream, &r);
    dfree(dense);   // stream-ordered: later users of the block run after the scan
    if (rc) {
        ctg_free(U);
        return rc;
    }
    CTG_CHECK(launch_gather_labels(U->nodes, r->edges, 2 * r->n_edges, s));
    CTG_CHECK(launch_gather_labels(U->nodes, r->nodes, r->n_nodes, s));
    CTG_CHECK(hipStreamSynchronize(s));
    ctg_free(U);
    *out = r;
    return CTG_OK;
}

// One face scan with its record bookkeeping: the record buffer grows and the
// scan re-runs when a region overflowed.  *overflow = labels that do not fit
// the key's u / v fields (the caller relabels densely).
static int scan_records(Workspace& w, const ScanParams& P, int64_t V, hipStream_t s, Ev& ev, RegionPrefix& pre,
                        bool* overflow, const char* who) {
    *overflow = false;
    if (getenv("CTG_REC_FRESH")) {   // test hook: start from the smallest record buffer
        CTG_CHECK(hipStreamSynchronize(s));
        free_records(w);
    }
    int64_t need = std::max<int64_t>(w.rec.cap, std::max<int64_t>(1 << 16, V / 24));
    need = (need + NREG - 1) / NREG * NREG;
    for (int attempt = 0; attempt < 4; ++attempt) {
        CTG_CHECK(ensure_records(w, need, 0));
        CTG_CHECK(hipMemsetAsync(w.counters, 0, sizeof(Counters), s));
        ev.mark(0);   // (re-recorded here: the scan phase brackets the scan launch alone)
        CTG_CHECK(launch_face_scan(P, w.rec, w.counters, s));
        ev.mark(1);
        CTG_CHECK(hipMemcpyAsync(w.counters_host, w.counters, sizeof(Counters), hipMemcpyDeviceToHost, s));
        CTG_CHECK(hipStreamSynchronize(s));
        if (w.counters_host->label_overflow) {
            *overflow = true;
            return CTG_OK;
        }
        unsigned long long tot = 0, mx = 0;
        for (int r = 0; r < NREG; ++r) {
            pre.off[r] = (uint32_t)tot;
            tot += w.counters_host->rcount[r];
            mx = std::max(mx, w.counters_host->rcount[r]);
        }
        pre.off[NREG] = (uint32_t)tot;
        w.counters_host->n_records = tot;
        if (tot >= (1ull << 32)) {
            set_error(std::string(who) + ": more than 2^32 records");
            return CTG_ERR_NOMEM;
        }
        if ((int64_t)mx <= w.rec.rcap) break;
        need = ((int64_t)(mx * 5 / 4) + 1024) * NREG;
        if (attempt == 3) {
            set_error(std::string(who) + ": record buffer overflow");
            return CTG_ERR_NOMEM;
        }
    }
    if (P.ablate & 256)   // diagnostic s_memtime stamps, summed over waves
        fprintf(stderr, "stamps total %llu fold %llu flush %llu wait %llu\n", w.counters_host->pad[2],
                w.counters_host->pad[3], w.counters_host->pad[4], w.counters_host->pad[5]);
    w.last_records = (int64_t)w.counters_host->n_records;
    w.last_direct = (int64_t)w.counters_host->n_direct;
    return CTG_OK;
}

int ctg_rag_features(const void* labels, int label_bits, const void* data, int data_kind, int n_channels,
                     const int32_t* offsets, const int64_t* shape, const int64_t* own_begin,
                     const int64_t* own_end, int ignore_label,
                     double hist_lo, double hist_hi, int flags, int mem, void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!out || !shape || !labels) {
        set_error("ctg_rag_features: null argument");
        return CTG_ERR_ARG;
    }
    *out = nullptr;
    if (label_bits != 32 && label_bits != 64) {
        set_error("ctg_rag_features: label_bits must be 32 or 64");
        return CTG_ERR_ARG;
    }
    if (n_channels < 0 || n_channels > CTG_MAX_CHANNELS || (n_channels > 0 && !offsets)) {
        set_error("ctg_rag_features: bad channel/offset arguments");
        return CTG_ERR_ARG;
    }
    if (data && data_kind != CTG_DATA_F32 && data_kind != CTG_DATA_U8) {
        set_error("ctg_rag_features: data_kind must be CTG_DATA_F32 or CTG_DATA_U8");
        return CTG_ERR_ARG;
    }
    if (!(hist_hi > hist_lo)) {
        set_error("ctg_rag_features: hist_hi must be > hist_lo");
        return CTG_ERR_ARG;
    }
    for (int k = 0; k < 3; ++k)
        if (shape[k] < 0 || (own_begin && (own_begin[k] < 0)) || (own_end && own_end[k] < 0)) {
            set_error("ctg_rag_features: negative shape/own_begin/own_end");
            return CTG_ERR_ARG;
        }
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    const int64_t V = shape[0] * shape[1] * shape[2];
    const size_t lbytes = (size_t)V * (label_bits / 8);
    const size_t dbytes = data ? (size_t)V * (n_channels > 0 ? n_channels : 1) * (data_kind == CTG_DATA_U8 ? 1 : 4) : 0;
    const void* dl = nullptr;
    const void* dd = nullptr;
    int rc = stage_in(w, 0, labels, lbytes, mem, s, &dl);
    if (rc) return rc;
    rc = stage_in(w, 1, data, dbytes, mem, s, &dd);
    if (rc) return rc;

    ScanParams P;
    std::memset(&P, 0, sizeof(P));
    P.labels = dl;
    P.data = dd;
    P.label_bits = label_bits;
    P.data_kind = data ? data_kind : CTG_DATA_NONE;
    P.n_channels = data ? n_channels : 0;
    for (int c = 0; c < P.n_channels; ++c)
        for (int k = 0; k < 3; ++k) P.offsets[c][k] = offsets[3 * c + k];
    for (int k = 0; k < 3; ++k) {
        P.shape[k] = shape[k];
        P.own_begin[k] = own_begin ? own_begin[k] : 0;
        P.own_end[k] = own_end ? std::min(own_end[k], shape[k]) : shape[k];
    }
    P.scale = (double)NBINS / (hist_hi - hist_lo);
    P.offset = hist_lo;
    P.fast40 = (hist_lo == 0.0 && P.scale == 40.0) ? 1 : 0;
    // flush decisions every check_planes planes (overflow safety does not
    // depend on it: ctg_scan.hip's per-wave sample budget bounds every count)
    P.check_planes = 8;
    // planes per workgroup of the narrow-tile launch (fragmented volumes):
    // shallower tiles split fewer edges at table flushes (profiles/r4/tz)
    constexpr int NARROW_TILE_Z = 16;
    // planes per workgroup: 32, fewer where that leaves < ~1024 workgroups,
    // 64 (128) where even 64 (128)-plane tiles give >= 32 K workgroups (A/B with the 5/8
    // table fill, 32 vs 64 planes: 512^3 step 1.027 -> 1.014 ms, configs[4]
    // 32.2 -> 30.0 ms with records 148 M -> 134 M; 2048^3 scan 30.4 vs 30.9 ms
    // favours 64)
    {
        const int64_t rows = scan_tile_rows();
        const int64_t cols = ((shape[2] + TILE_X - 1) / TILE_X) * ((shape[1] + rows - 1) / rows);
        int tz = cols * ((shape[0] + 63) / 64) >= 32768 ? 64 : 32;
        // 128 where even 128-plane tiles leave >= 32 K workgroups (2048^3: scan
        // 29.76 -> 29.35 ms, records 28.1 M -> 27.3 M, step 33.65 -> 33.08 ms;
        // profiles/r4/ablate)
        if (cols * ((shape[0] + 127) / 128) >= 32768) tz = 128;
        while (tz > 8 && cols * ((shape[0] + tz - 1) / tz) < 1024) tz /= 2;
        // narrow tiles 16 planes deep, deeper where that would launch more than
        // 64 K workgroups: both widths are launched and one exits at once, and
        // at 2048^3 the exiting launch of 16-plane narrow tiles (524 K
        // workgroups) cost 0.22 ms per call
        {
            const int64_t rn = scan_tile_rows_narrow();
            const int64_t cols_n = ((shape[2] + TILE_X - 1) / TILE_X) * ((shape[1] + rn - 1) / rn);
            int tzn = std::min(tz, NARROW_TILE_Z);
            while (tzn < tz && cols_n * ((shape[0] + tzn - 1) / tzn) > 65536) tzn *= 2;
            P.tile_z_narrow = tzn;
        }
        if (const char* t = getenv("CTG_TILE_Z")) P.tile_z_narrow = tz = std::max(1, atoi(t));   // tests
        P.tile_z = tz;
    }
#ifdef CTG_DIAG   // scan ablations (variant builds only)
    {
        const char* ab = getenv("CTG_ABLATE");
        P.ablate = ab ? atoi(ab) : 0;
    }
#endif
    P.xcd_remap = 1;
    // boundary maps of fragmented volumes (configs[4]: cell 5) scan with
    // 2-row waves: the sampled x-face density decides on the device (cell 10
    // ~ 0.10, cell 5 ~ 0.20 changes per pair; threshold 0.14), without a host
    // round trip.  The probe and the second launch cost ~0.1 ms, so volumes
    // below 2^28 voxels (~645^3, steps of ~2 ms) keep the wide tiles.
    // CTG_NARROW_ROWS=0/1 forces a width.
    if (data && n_channels == 0 && (V >= (1ll << 28) || getenv("CTG_NARROW_ROWS"))) {
        const char* nr = getenv("CTG_NARROW_ROWS");
        if (nr) {
            P.narrow_rows = atoi(nr) ? 1 : 0;
        } else {
            CTG_CHECK(hipMemsetAsync(w.small + 4, 0, 8, s));
            CTG_CHECK(launch_density(dl, label_bits, shape, 512, w.small + 4, s));
            P.narrow_rows = 2;
            P.density = w.small + 4;
        }
    }

    // Long-range affinity channels: a sample counts only if its
    // (u,v) is a RAG edge.  Filtering in the scan (against the edge set of a
    // graph-only pass) keeps the non-adjacent pairs - most long-range pairs -
    // out of the edge tables and records.  Labels >= 2^32 skip it here: the
    // dense-relabel path re-enters with 32-bit labels and filters there.
    unsigned long long* bloom = nullptr;
    ctg_result* adj_graph = nullptr;
    bool long_range = false;
    for (int c = 0; c < P.n_channels; ++c)
        long_range |= std::abs(P.offsets[c][0]) + std::abs(P.offsets[c][1]) + std::abs(P.offsets[c][2]) > 1;

    if (data) w.last_ms[7] = 0.0;   // the narrowing pass of earlier builds: no longer run
    if (long_range && !(flags & CTG_NO_ADJ_FILTER) && V > 0) {
        rc = ctg_rag_features(dl, label_bits, nullptr, CTG_DATA_NONE, 0, nullptr, shape, own_begin, own_end, 0,
                              hist_lo, hist_hi, 0, CTG_MEM_DEVICE, stream, &adj_graph);
        if (rc) return rc;
        uint64_t mx = 0;
        if (adj_graph->n_edges > 0) {
            // largest label of the sorted edge table: the v of some row; the
            // max over all v equals the last node
            CTG_CHECK(hipMemcpyAsync(&mx, adj_graph->nodes + adj_graph->n_nodes - 1, 8, hipMemcpyDeviceToHost, s));
            CTG_CHECK(hipStreamSynchronize(s));
        }
        if ((mx >> 32) == 0) {
            // Bloom prefilter, 24 bits per stored direction (48 per edge; 32: +3 %
            // records, 12-channel scan +0.5 ms, profiles/r4/tz): one
            // load per long-range sample (vs. a probe chain in a set 4x the
            // size); the reduce drops its false positives (keys no
            // nearest-neighbour sample flagged)
            const int64_t bits = adj_graph->n_edges * 48;
            uint32_t blocks = 128;   // 64-B blocks
            while ((int64_t)blocks * 512 < bits) blocks *= 2;
            bloom = (unsigned long long*)dalloc((size_t)blocks * 64);
            if (!bloom) {
                ctg_free(adj_graph);
                set_error("ctg_rag_features: out of memory (adjacency filter)");
                return CTG_ERR_NOMEM;
            }
            hipError_t e = launch_build_bloom(adj_graph->edges, adj_graph->n_edges, bloom, blocks - 1, s);
            if (e != hipSuccess) {
                dfree(bloom);
                ctg_free(adj_graph);
                set_error(std::string("ctg_rag_features: ") + hipGetErrorString(e));
                return CTG_ERR_HIP;
            }
            P.bloom = bloom;
            P.bloom_mask = blocks - 1;
        }
    }
    {
        bool nn[3] = {false, false, false};
        for (int c = 0; c < P.n_channels; ++c) {
            const int* o = P.offsets[c];
            if (std::abs(o[0]) + std::abs(o[1]) + std::abs(o[2]) > 1) P.lr_mask |= 1u << c;
            for (int a = 0; a < 3; ++a)
                nn[a] |= o[a] == -1 && o[(a + 1) % 3] == 0 && o[(a + 2) % 3] == 0;
        }
        // every nearest-neighbour face yields a sample of its channel (the
        // adjacency proof), so no separate markers are pushed
        P.skip_adj_marks = P.n_channels > 0 && nn[0] && nn[1] && nn[2] && !(flags & CTG_NO_ADJ_FILTER) &&
                           (!long_range || P.bloom != nullptr);
        if (const char* sa = getenv("CTG_SKIP_ADJ")) P.skip_adj_marks = P.skip_adj_marks && atoi(sa);
        // exactly the three nearest-neighbour channels (any order), every
        // sample an adjacency proof: the face-scan form of the affinity scan
        // (MODE_AFF_NN, ctg_scan.hip); CTG_NN3=0 keeps the channel loop
        if (P.n_channels == 3 && !long_range && P.skip_adj_marks) {
            int ch[3] = {-1, -1, -1};
            for (int c = 0; c < 3; ++c)
                for (int a = 0; a < 3; ++a)
                    if (P.offsets[c][a] == -1 && P.offsets[c][(a + 1) % 3] == 0 && P.offsets[c][(a + 2) % 3] == 0)
                        ch[a] = c;
            const char* e = getenv("CTG_NN3");
            if (ch[0] >= 0 && ch[1] >= 0 && ch[2] >= 0 && !(e && e[0] == '0')) {
                P.nn3 = 1;
                for (int a = 0; a < 3; ++a) P.nn_ch[a] = ch[a];
            }
        }
        // long-range calls with the Bloom filter: the nearest-neighbour
        // channels as faces (their samples flag adjacency), the rest looped
        if (long_range && P.bloom != nullptr && P.skip_adj_marks) {
            int ch[3] = {-1, -1, -1};
            for (int c = 0; c < P.n_channels; ++c)
                for (int a = 0; a < 3; ++a)
                    if (ch[a] < 0 && P.offsets[c][a] == -1 && P.offsets[c][(a + 1) % 3] == 0 &&
                        P.offsets[c][(a + 2) % 3] == 0)
                        ch[a] = c;
            const char* e = getenv("CTG_NN3");
            if (ch[0] >= 0 && ch[1] >= 0 && ch[2] >= 0 && !(e && e[0] == '0')) {
                P.nn_mix = 1;
                for (int a = 0; a < 3; ++a) P.nn_ch[a] = ch[a];
                P.n_loop = 0;
                for (int c = 0; c < P.n_channels; ++c)
                    if (c != ch[0] && c != ch[1] && c != ch[2]) P.loop_ch[P.n_loop++] = c;
            }
        }
    }
    struct AdjRelease {   // the set and its graph live until the scan is done
        unsigned long long*& set;
        ctg_result*& g;
        hipStream_t s;
        ~AdjRelease() {
            if (set) {
                hipStreamSynchronize(s);
                dfree(set);
            }
            if (g) ctg_free(g);
        }
    } adj_release{bloom, adj_graph, s};

    Ev ev{w, s};
    ev.mark(0);
    if (V == 0) {
        ctg_result* r = new ctg_result();
        r->device = dev;
        r->edges = (uint64_t*)dalloc(16);
        r->nodes = (uint64_t*)dalloc(8);
        *out = r;
        return CTG_OK;
    }
    RegionPrefix pre{};
    const bool stats = P.data_kind != CTG_DATA_NONE;
    bool overflow = false;
    rc = scan_records(w, P, V, s, ev, pre, &overflow, "ctg_rag_features");
    if (rc) return rc;
    if (overflow) {
        if (label_bits != 64) {
            set_error("ctg_rag_features: internal label overflow on 32-bit labels");
            return CTG_ERR_HIP;
        }
        return rag_dense_relabel(dl, dd, data_kind, n_channels, offsets, shape, own_begin, own_end, ignore_label,
                                 hist_lo, hist_hi, flags, stream, out);
    }
    const int64_t n = (int64_t)w.counters_host->n_records;

    ctg_result* r = new ctg_result();
    r->device = dev;
    r->n_records = n;
    r->n_direct = w.last_direct;
    ReduceJob J{};
    J.n = n;
    J.keys = w.rec.key;
    J.regions = &pre;
    J.R = w.rec;
    J.wide = 0;
    J.stats = stats;
    J.need_adj = P.n_channels > 0 && !P.skip_adj_marks ? ((flags & CTG_NO_ADJ_FILTER) ? 2 : 1) : 0;
    if (P.bloom) J.need_adj = 1;   // drop the Bloom filter's false positives
    J.ignore_label = ignore_label;
    J.keep_stats = (flags & CTG_KEEP_STATS) ? 1 : 0;
    J.defer_stats = (flags & CTG_DEFER_STATS) ? 1 : 0;
    J.max_v = w.counters_host->max_v;
    J.scale = P.scale;
    J.offset = P.offset;
    // single-label array: the owned origin voxel is the only node
    const int64_t o0 = own_begin ? own_begin[0] : 0, o1 = own_begin ? own_begin[1] : 0,
                  o2 = own_begin ? own_begin[2] : 0;
    const bool has_owned = o0 < P.own_end[0] && o1 < P.own_end[1] && o2 < P.own_end[2];
    J.single_label_ptr = (label_bits == 64 && has_owned)
                             ? (const uint64_t*)dl + ((o0 * shape[1] + o1) * shape[2] + o2)
                             : nullptr;
    hipError_t e = reduce_records(w, J, s, r);
    if (e == hipSuccess && label_bits == 32 && r->n_records == 0 && has_owned) {
        // 32-bit labels: widen the single label
        uint32_t l32 = 0;
        e = hipMemcpyAsync(&l32, (const uint32_t*)dl + ((o0 * shape[1] + o1) * shape[2] + o2), 4,
                           hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        uint64_t l64 = l32;
        if (e == hipSuccess) e = hipMemcpy(r->nodes, &l64, 8, hipMemcpyHostToDevice);
        r->n_nodes = 1;
    }
    if (e != hipSuccess) {
        set_error(std::string("ctg_rag_features: ") + hipGetErrorString(e));
        ctg_free(r);
        return CTG_ERR_HIP;
    }
    if (w.profiling) {
        CTG_CHECK(hipStreamSynchronize(s));
        float ms = 0.f;
        const int a[6] = {0, 1, 2, 3, 4, 5};
        for (int i = 0; i < 6; ++i) {
            hipEventElapsedTime(&ms, w.ev[a[i]], w.ev[a[i] + 1]);
            w.last_ms[i] = ms;
        }
        hipEventElapsedTime(&ms, w.ev[0], w.ev[6]);
        w.last_ms[6] = ms;
    }
    r->partial_adj = J.need_adj == 2 ? 1 : 0;
    *out = r;
    return CTG_OK;
}

// ---------------------------------------------------------------------------
// batched per-block sub-graphs / features (the ndist per-block calls)
// ---------------------------------------------------------------------------
static int bits_u(int64_t v) { return v <= 0 ? 0 : bits_for((uint64_t)v); }

// the per-block nodes of a batched call: unique labels of every own box
static int block_nodes(Workspace& w, const void* dl, int label_bits, const BlockGeom* dgeom, int n_blocks,
                       const std::vector<uint32_t>& uprefix, int64_t own_voxels, hipStream_t s, ctg_result* r) {
    const int64_t n_tiles = uprefix.back();
    uint32_t* dprefix = (uint32_t*)dalloc((n_blocks + 1) * 4);
    if (!dprefix) return CTG_ERR_NOMEM;
    CTG_CHECK(hipMemcpyAsync(dprefix, uprefix.data(), (n_blocks + 1) * 4, hipMemcpyHostToDevice, s));
    int64_t cap = std::max<int64_t>(1, std::min<int64_t>(own_voxels, std::max<int64_t>(1 << 16, own_voxels / 8)));
    for (int attempt = 0; attempt < 3; ++attempt) {
        uint64_t* cand = (uint64_t*)dalloc(cap * 8);
        uint64_t* sorted = (uint64_t*)dalloc(cap * 8);
        uint64_t* nodes = (uint64_t*)dalloc(cap * 8);
        int64_t* bounds = (int64_t*)dalloc((n_blocks + 1) * 8);
        if (!cand || !sorted || !nodes || !bounds) return CTG_ERR_NOMEM;
        CTG_CHECK(hipMemsetAsync(w.counters, 0, sizeof(Counters), s));
        CTG_CHECK(launch_unique_blocks(dl, label_bits, dgeom, dprefix, n_blocks, n_tiles, cand,
                                       &w.counters->n_records, cap, s));
        CTG_CHECK(hipMemcpyAsync(w.counters_host, w.counters, sizeof(Counters), hipMemcpyDeviceToHost, s));
        CTG_CHECK(hipStreamSynchronize(s));
        const int64_t m = (int64_t)w.counters_host->n_records;
        if (m > cap) {
            dfree(cand); dfree(sorted); dfree(nodes); dfree(bounds);
            cap = m + 1024;
            continue;
        }
        const unsigned kb = 32u + (unsigned)bits_u(n_blocks - 1);
        size_t tb = 0;
        CTG_CHECK(rocprim::radix_sort_keys(nullptr, tb, cand, sorted, (size_t)m, 0u, kb, s));
        ensure(&w.temp, w.temp_bytes, tb + 256);
        tb = w.temp_bytes;
        CTG_CHECK(rocprim::radix_sort_keys(w.temp, tb, cand, sorted, (size_t)m, 0u, kb, s));
        tb = 0;
        CTG_CHECK(rocprim::unique(nullptr, tb, sorted, nodes, w.small + 2, (size_t)m, rocprim::equal_to<uint64_t>(), s));
        ensure(&w.temp, w.temp_bytes, tb + 256);
        tb = w.temp_bytes;
        CTG_CHECK(rocprim::unique(w.temp, tb, sorted, nodes, w.small + 2, (size_t)m, rocprim::equal_to<uint64_t>(), s));
        CTG_CHECK(hipMemcpyAsync(w.small_host + 2, w.small + 2, 4, hipMemcpyDeviceToHost, s));
        CTG_CHECK(hipStreamSynchronize(s));
        const int64_t N = w.small_host[2];
        CTG_CHECK(launch_block_bounds(N, nodes, 1, n_blocks, 32, bounds, s));
        r->node_off.assign(n_blocks + 1, 0);
        CTG_CHECK(hipMemcpyAsync(r->node_off.data(), bounds, (n_blocks + 1) * 8, hipMemcpyDeviceToHost, s));
        CTG_CHECK(launch_clear_bits(N, nodes, 1, 0xFFFFFFFFull, s));
        CTG_CHECK(hipStreamSynchronize(s));
        dfree(r->nodes);
        r->nodes = nodes;
        r->n_nodes = N;
        dfree(cand); dfree(sorted); dfree(bounds); dfree(dprefix);
        return CTG_OK;
    }
    set_error("ctg_rag_blocks: node candidate buffer overflow");
    return CTG_ERR_NOMEM;
}

int ctg_rag_blocks(const void* labels, int label_bits, const void* data, int data_kind, int n_channels,
                   const int32_t* offsets, const ctg_block_desc* blocks, int n_blocks, int64_t labels_len,
                   int64_t data_len, int ignore_label, double hist_lo, double hist_hi, int flags, int mem,
                   void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!out || !labels || !blocks || n_blocks < 1 || n_blocks > (1 << 20) || labels_len < 0 ||
        (label_bits != 32 && label_bits != 64) || (data && data_kind != CTG_DATA_F32 && data_kind != CTG_DATA_U8) ||
        n_channels < 0 || n_channels > CTG_MAX_CHANNELS || (n_channels > 0 && !offsets) || !(hist_hi > hist_lo)) {
        set_error("ctg_rag_blocks: bad arguments");
        return CTG_ERR_ARG;
    }
    *out = nullptr;
    const int nch = data ? std::max(1, n_channels) : 0;
    int64_t own_voxels = 0, voxels = 0, zmax = 1;
    for (int b = 0; b < n_blocks; ++b) {
        const ctg_block_desc& d = blocks[b];
        int64_t V = 1;
        for (int k = 0; k < 3; ++k) {
            V *= d.shape[k];
            if (d.shape[k] < 0 || d.shape[k] > 0x7FFFFFFF || d.own_begin[k] < 0 || d.own_end[k] > d.shape[k] ||
                d.graph_begin[k] < 0 || d.graph_end[k] > d.shape[k]) {
                set_error("ctg_rag_blocks: block " + std::to_string(b) + ": box outside its array");
                return CTG_ERR_ARG;
            }
        }
        if (d.label_offset < 0 || d.label_offset + V > labels_len ||
            (data && (d.data_offset < 0 || d.data_offset + V * nch > data_len))) {
            set_error("ctg_rag_blocks: block " + std::to_string(b) + ": array outside the arena");
            return CTG_ERR_ARG;
        }
        int64_t ov = 1;
        for (int k = 0; k < 3; ++k) ov *= std::max<int64_t>(0, d.own_end[k] - d.own_begin[k]);
        own_voxels += ov;
        voxels += V;
        zmax = std::max(zmax, d.shape[0]);
    }
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    const void* dl = nullptr;
    const void* dd = nullptr;
    int rc = stage_in(w, 0, labels, (size_t)labels_len * (label_bits / 8), mem, s, &dl);
    if (rc) return rc;
    rc = stage_in(w, 1, data, data ? (size_t)data_len * (data_kind == CTG_DATA_U8 ? 1 : 4) : 0, mem, s, &dd);
    if (rc) return rc;

    ScanParams P;
    std::memset(&P, 0, sizeof(P));
    P.labels = dl;
    P.data = dd;
    P.label_bits = label_bits;
    P.data_kind = data ? data_kind : CTG_DATA_NONE;
    P.n_channels = data ? n_channels : 0;
    for (int c = 0; c < P.n_channels; ++c)
        for (int k = 0; k < 3; ++k) P.offsets[c][k] = offsets[3 * c + k];
    for (int c = 0; c < P.n_channels; ++c) {
        const int* o = P.offsets[c];
        if (std::abs(o[0]) + std::abs(o[1]) + std::abs(o[2]) > 1) P.lr_mask |= 1u << c;
    }
    P.scale = (double)NBINS / (hist_hi - hist_lo);
    P.offset = hist_lo;
    P.fast40 = (hist_lo == 0.0 && P.scale == 40.0) ? 1 : 0;
    P.check_planes = 8;
    P.tile_z = (int)std::min<int64_t>(zmax, 128);   // one tile deep for the usual <= 128-plane blocks
    if (const char* t = getenv("CTG_TILE_Z")) P.tile_z = std::max(1, atoi(t));
    P.xcd_remap = 1;
    const int tag_bits = bits_u(n_blocks - 1);
    P.tag_shift = 32 - tag_bits;
    P.label_hi_mask = tag_bits ? ~((1u << P.tag_shift) - 1u) : 0u;
    P.n_blocks = n_blocks;
    // per-block geometry and the tile prefixes of the scan / node launches
    const int rows = scan_tile_rows(), uty = unique_tile_y();
    std::vector<BlockGeom> geom(n_blocks);
    std::vector<uint32_t> prefix(n_blocks + 1, 0), uprefix(n_blocks + 1, 0);
    for (int b = 0; b < n_blocks; ++b) {
        const ctg_block_desc& d = blocks[b];
        BlockGeom& g = geom[b];
        g.label_offset = d.label_offset;
        g.data_offset = data ? d.data_offset : 0;
        for (int k = 0; k < 3; ++k) {
            g.shape[k] = (int32_t)d.shape[k];
            g.own_begin[k] = (int32_t)d.own_begin[k];
            g.own_end[k] = (int32_t)d.own_end[k];
            g.graph_begin[k] = (int32_t)d.graph_begin[k];
            g.graph_end[k] = (int32_t)d.graph_end[k];
        }
        g.ntx = (int32_t)((d.shape[2] + TILE_X - 1) / TILE_X);
        g.nty = (int32_t)((d.shape[1] + rows - 1) / rows);
        g.ntz = (int32_t)((d.shape[0] + P.tile_z - 1) / P.tile_z);
        const int64_t nt = (int64_t)g.ntx * g.nty * g.ntz;
        int64_t ut = 1;
        const int64_t oe[3] = {std::max<int64_t>(0, d.own_end[0] - d.own_begin[0]),
                               std::max<int64_t>(0, d.own_end[1] - d.own_begin[1]),
                               std::max<int64_t>(0, d.own_end[2] - d.own_begin[2])};
        ut = ((oe[2] + 63) / 64) * ((oe[1] + uty - 1) / uty) * ((oe[0] + 15) / 16);
        if ((int64_t)prefix[b] + nt > 0x7FFFFFFFll || (int64_t)uprefix[b] + ut > 0x7FFFFFFFll) {
            set_error("ctg_rag_blocks: too many tiles in one call");
            return CTG_ERR_ARG;
        }
        prefix[b + 1] = prefix[b] + (uint32_t)nt;
        uprefix[b + 1] = uprefix[b] + (uint32_t)ut;
    }
    P.batch_tiles = prefix[n_blocks];
    BlockGeom* dgeom = (BlockGeom*)dalloc(sizeof(BlockGeom) * n_blocks);
    uint32_t* dprefix = (uint32_t*)dalloc((n_blocks + 1) * 4);
    if (!dgeom || !dprefix) {
        set_error("ctg_rag_blocks: out of device memory");
        return CTG_ERR_NOMEM;
    }
    CTG_CHECK(hipMemcpyAsync(dgeom, geom.data(), sizeof(BlockGeom) * n_blocks, hipMemcpyHostToDevice, s));
    CTG_CHECK(hipMemcpyAsync(dprefix, prefix.data(), (n_blocks + 1) * 4, hipMemcpyHostToDevice, s));
    P.blocks = dgeom;
    P.tile_prefix = dprefix;
    struct Release {
        BlockGeom* g;
        uint32_t* p;
        hipStream_t s;
        ~Release() {
            hipStreamSynchronize(s);
            dfree(g);
            dfree(p);
        }
    } release{dgeom, dprefix, s};

    Ev ev{w, s};
    ev.mark(0);
    RegionPrefix pre{};
    bool overflow = false;
    rc = P.batch_tiles ? scan_records(w, P, voxels, s, ev, pre, &overflow, "ctg_rag_blocks") : CTG_OK;
    if (rc) return rc;
    if (overflow) {
        // labels too large for the tagged keys: relabel the arena densely
        // (monotone, so sorted dense tables stay sorted after mapping back)
        const uint64_t* l64 = (const uint64_t*)dl;
        uint64_t* wide = nullptr;
        if (label_bits == 32) {
            wide = (uint64_t*)dalloc(std::max<int64_t>(labels_len, 1) * 8);
            if (!wide) return CTG_ERR_NOMEM;
            CTG_CHECK(launch_u32_to_u64(labels_len, (const uint32_t*)dl, wide, s));
            l64 = wide;
        }
        ctg_result* U = nullptr;
        rc = ctg_unique_values(l64, labels_len, CTG_MEM_DEVICE, stream, &U);
        if (rc) return rc;
        if (ignore_label && (rc = keep_zero_first(U, s)) != CTG_OK) {
            ctg_free(U);
            return rc;
        }
        if (U->n_nodes > (int64_t)(1ull << P.tag_shift)) {
            ctg_free(U);
            set_error("ctg_rag_blocks: too many distinct labels for one batch of blocks: call with fewer blocks");
            return CTG_ERR_UNSUPPORTED;
        }
        uint32_t* dense = (uint32_t*)dalloc(std::max<int64_t>(labels_len, 1) * 4);
        if (!dense) {
            ctg_free(U);
            return CTG_ERR_NOMEM;
        }
        CTG_CHECK(launch_remap_dense(l64, labels_len, U->nodes, U->n_nodes, dense, s));
        ctg_result* r = nullptr;
        rc = ctg_rag_blocks(dense, 32, dd, data_kind, n_channels, offsets, blocks, n_blocks, labels_len, data_len,
                            ignore_label, hist_lo, hist_hi, flags, CTG_MEM_DEVICE, stream, &r);
        dfree(dense);
        if (wide) dfree(wide);
        if (rc) {
            ctg_free(U);
            return rc;
        }
        CTG_CHECK(launch_gather_labels(U->nodes, r->edges, 2 * r->n_edges, s));
        CTG_CHECK(launch_gather_labels(U->nodes, r->nodes, r->n_nodes, s));
        CTG_CHECK(hipStreamSynchronize(s));
        ctg_free(U);
        *out = r;
        return CTG_OK;
    }
    const int64_t n = P.batch_tiles ? (int64_t)w.counters_host->n_records : 0;
    ctg_result* r = new ctg_result();
    r->device = dev;
    r->n_records = n;
    r->n_direct = P.batch_tiles ? (int64_t)w.counters_host->n_direct : 0;
    ReduceJob J{};
    J.n = n;
    J.keys = w.rec.key;
    J.regions = &pre;
    J.R = w.rec;
    J.stats = P.data_kind != CTG_DATA_NONE;
    // boundary / graph: every key is a face of the block's graph box;
    // affinities: keep the keys of the block's sub-graph (ADJ marks)
    J.need_adj = P.n_channels > 0 ? 1 : 0;
    J.ignore_label = ignore_label;
    J.keep_stats = (flags & CTG_KEEP_STATS) ? 1 : 0;
    J.max_v = P.batch_tiles ? w.counters_host->max_v : 0;
    J.scale = P.scale;
    J.offset = P.offset;
    J.ub = tag_bits ? 32 : 0;
    J.umask = tag_bits ? (1ull << P.tag_shift) - 1ull : ~0ull;
    J.skip_nodes = 1;
    hipError_t e = reduce_records(w, J, s, r);
    if (e == hipSuccess) {
        r->edge_off.assign(n_blocks + 1, 0);
        r->edge_off[n_blocks] = r->n_edges;
        if (tag_bits && r->n_edges) {
            int64_t* bounds = (int64_t*)dalloc((n_blocks + 1) * 8);
            e = bounds ? launch_block_bounds(r->n_edges, r->edges, 2, n_blocks, P.tag_shift, bounds, s)
                       : hipErrorOutOfMemory;
            if (e == hipSuccess)
                e = hipMemcpyAsync(r->edge_off.data(), bounds, (n_blocks + 1) * 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = launch_clear_bits(r->n_edges, r->edges, 2, J.umask, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            dfree(bounds);
        }
    }
    if (e != hipSuccess) {
        set_error(std::string("ctg_rag_blocks: ") + hipGetErrorString(e));
        ctg_free(r);
        return CTG_ERR_HIP;
    }
    if (flags & CTG_NO_NODES) {
        r->node_off.assign(n_blocks + 1, 0);
        rc = CTG_OK;
    } else {
        rc = block_nodes(w, dl, label_bits, dgeom, n_blocks, uprefix, own_voxels, s, r);
    }
    if (rc) {
        ctg_free(r);
        return rc;
    }
    if (w.profiling && P.batch_tiles) {   // same phase split as ctg_rag_features ([5] = reduce end -> nodes)
        CTG_CHECK(hipStreamSynchronize(s));
        float ms = 0.f;
        for (int i = 0; i < 6; ++i) {
            hipEventElapsedTime(&ms, w.ev[i], w.ev[i + 1]);
            w.last_ms[i] = ms;
        }
        hipEventElapsedTime(&ms, w.ev[0], w.ev[6]);
        w.last_ms[6] = ms;
    }
    r->partial_adj = J.need_adj == 2 ? 1 : 0;
    *out = r;
    return CTG_OK;
}

void* ctg_host_alloc(int64_t bytes) {
    void* p = nullptr;
    if (bytes <= 0) bytes = 64;
    if (hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault) != hipSuccess) {
        set_error("ctg_host_alloc: hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

void ctg_host_free(void* p) {
    if (p) hipHostFree(p);
}

int ctg_result_num_blocks(const ctg_result* r) { return r ? (int)std::max<size_t>(r->edge_off.size(), 1) - 1 : -1; }

int ctg_result_block_offsets(const ctg_result* r, int64_t* edge_off, int64_t* node_off) {
    if (!r || r->edge_off.empty()) {
        set_error("ctg_result_block_offsets: not a batched-blocks result");
        return CTG_ERR_ARG;
    }
    const size_t nb = r->edge_off.size();
    if (edge_off) std::memcpy(edge_off, r->edge_off.data(), nb * 8);
    if (node_off) {
        if (r->node_off.size() == nb) std::memcpy(node_off, r->node_off.data(), nb * 8);
        else std::memset(node_off, 0, nb * 8);
    }
    return CTG_OK;
}

int ctg_unique_labels(const uint64_t* labels, const int64_t* shape, const int64_t* begin, const int64_t* end,
                      int mem, void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!labels || !shape || !out) {
        set_error("ctg_unique_labels: null argument");
        return CTG_ERR_ARG;
    }
    *out = nullptr;
    int64_t b[3], e[3];
    for (int k = 0; k < 3; ++k) {
        b[k] = begin ? begin[k] : 0;
        e[k] = end ? end[k] : shape[k];
        if (b[k] < 0 || e[k] > shape[k] || b[k] > e[k]) {
            set_error("ctg_unique_labels: box outside the array");
            return CTG_ERR_ARG;
        }
    }
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    const int64_t V = shape[0] * shape[1] * shape[2];
    const void* dl = nullptr;
    int rc = stage_in(w, 0, labels, (size_t)V * 8, mem, s, &dl);
    if (rc) return rc;
    ctg_result* r = new ctg_result();
    r->device = dev;
    const int64_t nb = (e[0] - b[0]) * (e[1] - b[1]) * (e[2] - b[2]);
    if (nb == 0) {
        r->nodes = (uint64_t*)dalloc(8);
        r->edges = (uint64_t*)dalloc(16);
        *out = r;
        return CTG_OK;
    }
    int64_t cap = std::min<int64_t>(nb, std::max<int64_t>(1 << 16, nb / 8));
    for (int attempt = 0; attempt < 3; ++attempt) {
        uint64_t* cand = (uint64_t*)dalloc(cap * 8);
        uint64_t* sorted = (uint64_t*)dalloc(cap * 8);
        r->nodes = (uint64_t*)dalloc(cap * 8);
        CTG_CHECK(hipMemsetAsync(w.counters, 0, sizeof(Counters), s));
        CTG_CHECK(launch_unique_tiles((const uint64_t*)dl, shape, b, e, cand, &w.counters->n_records, cap, s));
        CTG_CHECK(hipMemcpyAsync(w.counters_host, w.counters, sizeof(Counters), hipMemcpyDeviceToHost, s));
        CTG_CHECK(hipStreamSynchronize(s));
        const int64_t m = (int64_t)w.counters_host->n_records;
        if (m > cap) {
            dfree(cand); dfree(sorted); dfree(r->nodes); r->nodes = nullptr;
            cap = std::min<int64_t>(nb, m + 1024);
            continue;
        }
        size_t tb = 0;
        CTG_CHECK(rocprim::radix_sort_keys(nullptr, tb, cand, sorted, (size_t)m, 0u, 64u, s));
        ensure(&w.temp, w.temp_bytes, tb + 256);
        tb = w.temp_bytes;
        CTG_CHECK(rocprim::radix_sort_keys(w.temp, tb, cand, sorted, (size_t)m, 0u, 64u, s));
        tb = 0;
        CTG_CHECK(rocprim::unique(nullptr, tb, sorted, r->nodes, w.small + 2, (size_t)m,
                                  rocprim::equal_to<uint64_t>(), s));
        ensure(&w.temp, w.temp_bytes, tb + 256);
        tb = w.temp_bytes;
        CTG_CHECK(rocprim::unique(w.temp, tb, sorted, r->nodes, w.small + 2, (size_t)m,
                                  rocprim::equal_to<uint64_t>(), s));
        CTG_CHECK(hipMemcpyAsync(w.small_host + 2, w.small + 2, 4, hipMemcpyDeviceToHost, s));
        CTG_CHECK(hipStreamSynchronize(s));
        r->n_nodes = w.small_host[2];
        dfree(cand);
        dfree(sorted);
        r->edges = (uint64_t*)dalloc(16);
        *out = r;
        return CTG_OK;
    }
    set_error("ctg_unique_labels: candidate buffer overflow");
    ctg_free(r);
    return CTG_ERR_NOMEM;
}

int ctg_unique_values(const uint64_t* values, int64_t n, int mem, void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!out || n < 0 || (n > 0 && !values)) {
        set_error("ctg_unique_values: bad arguments");
        return CTG_ERR_ARG;
    }
    *out = nullptr;
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    ctg_result* r = new ctg_result();
    r->device = dev;
    r->edges = (uint64_t*)dalloc(16);
    r->nodes = (uint64_t*)dalloc(std::max<int64_t>(n, 1) * 8);
    if (n == 0) {
        *out = r;
        return CTG_OK;
    }
    uint64_t* in = (uint64_t*)values;
    uint64_t* sorted = (uint64_t*)dalloc(n * 8);
    if (mem == CTG_MEM_HOST) in = (uint64_t*)dalloc(n * 8);
    if (!in || !sorted || !r->nodes) {
        set_error("ctg_unique_values: out of device memory");
        ctg_free(r);
        return CTG_ERR_NOMEM;
    }
    if (mem == CTG_MEM_HOST) CTG_CHECK(hipMemcpyAsync(in, values, n * 8, hipMemcpyHostToDevice, s));
    size_t tb = 0;
    CTG_CHECK(rocprim::radix_sort_keys(nullptr, tb, in, sorted, (size_t)n, 0u, 64u, s));
    ensure(&w.temp, w.temp_bytes, tb + 256);
    tb = w.temp_bytes;
    CTG_CHECK(rocprim::radix_sort_keys(w.temp, tb, in, sorted, (size_t)n, 0u, 64u, s));
    tb = 0;
    CTG_CHECK(rocprim::unique(nullptr, tb, sorted, r->nodes, w.small + 2, (size_t)n,
                              rocprim::equal_to<uint64_t>(), s));
    ensure(&w.temp, w.temp_bytes, tb + 256);
    tb = w.temp_bytes;
    CTG_CHECK(rocprim::unique(w.temp, tb, sorted, r->nodes, w.small + 2, (size_t)n,
                              rocprim::equal_to<uint64_t>(), s));
    CTG_CHECK(hipMemcpyAsync(w.small_host + 2, w.small + 2, 4, hipMemcpyDeviceToHost, s));
    CTG_CHECK(hipStreamSynchronize(s));
    r->n_nodes = w.small_host[2];
    dfree(sorted);
    if (mem == CTG_MEM_HOST) dfree(in);
    *out = r;
    return CTG_OK;
}

int ctg_merge_stats(const uint64_t* keys, const double* sums, const uint32_t* records, int64_t n, double hist_lo,
                    double hist_hi, int keep_stats, int mem, void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!out || n < 0 || (n > 0 && (!keys || !sums || !records))) {
        set_error("ctg_merge_stats: bad arguments");
        return CTG_ERR_ARG;
    }
    *out = nullptr;
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    ctg_result* r = new ctg_result();
    r->device = dev;
    if (n == 0) {
        r->edges = (uint64_t*)dalloc(16);
        r->nodes = (uint64_t*)dalloc(8);
        *out = r;
        return CTG_OK;
    }
    // inputs to device (merge buffers are separate from the scan records)
    uint64_t* dk = (uint64_t*)keys;
    double2* ds = (double2*)sums;
    uint32_t* dr = (uint32_t*)records;
    bool owned = false;
    if (mem == CTG_MEM_HOST) {
        dk = (uint64_t*)dalloc(n * 16);
        ds = (double2*)dalloc(n * 16);
        dr = (uint32_t*)dalloc(n * WREC_WORDS * 4);
        if (!dk || !ds || !dr) {
            set_error("ctg_merge_stats: out of device memory");
            return CTG_ERR_NOMEM;
        }
        CTG_CHECK(hipMemcpyAsync(dk, keys, n * 16, hipMemcpyHostToDevice, s));
        CTG_CHECK(hipMemcpyAsync(ds, sums, n * 16, hipMemcpyHostToDevice, s));
        CTG_CHECK(hipMemcpyAsync(dr, records, n * WREC_WORDS * 4, hipMemcpyHostToDevice, s));
        owned = true;
    }
    CTG_CHECK(hipMemsetAsync(w.counters, 0, sizeof(Counters), s));
    CTG_CHECK(launch_max_pairs(n, dk, &w.counters->max_v, s));
    CTG_CHECK(hipMemcpyAsync(w.counters_host, w.counters, sizeof(Counters), hipMemcpyDeviceToHost, s));
    CTG_CHECK(hipStreamSynchronize(s));
    DensePairs dp;
    if (w.counters_host->max_v >> 32) {
        int rc = dp.build(dk, n, s);
        if (rc) {
            delete r;
            return rc;
        }
    }
    ReduceJob J{};
    J.n = n;
    J.pairs = dp.U ? dp.dense : dk;
    J.R.key = nullptr;
    J.R.sums = ds;
    J.R.hist = dr;
    J.R.cap = n;
    J.wide = 1;
    J.stats = 1;
    J.need_adj = 1;
    J.ignore_label = 0;
    J.keep_stats = keep_stats;
    J.max_v = dp.U ? (uint64_t)std::max<int64_t>(dp.U->n_nodes - 1, 0) : w.counters_host->max_v;
    J.scale = (double)NBINS / (hist_hi - hist_lo);
    J.offset = hist_lo;
    hipError_t e = reduce_records(w, J, s, r);
    if (e == hipSuccess) e = dp.map_back(r, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (owned) {
        dfree(dk);
        dfree(ds);
        dfree(dr);
    }
    if (e != hipSuccess) {
        set_error(std::string("ctg_merge_stats: ") + hipGetErrorString(e));
        ctg_free(r);
        return CTG_ERR_HIP;
    }
    *out = r;
    return CTG_OK;
}

int ctg_merge_feature_rows(const uint64_t* ids, const double* rows, int64_t n, int64_t id_begin, int64_t id_end,
                           double* out, int mem, void* stream) {
    DevLock dev_lock;
    if (n < 0 || id_end < id_begin || (n > 0 && (!ids || !rows)) || (id_end > id_begin && !out)) {
        set_error("ctg_merge_feature_rows: bad arguments");
        return CTG_ERR_ARG;
    }
    if (id_end - id_begin > 0xFFFFFFFFll || n > 0xFFFFFFFFll) {
        set_error("ctg_merge_feature_rows: more than 2^32 edges or rows in one call");
        return CTG_ERR_UNSUPPORTED;
    }
    const int64_t E = id_end - id_begin;
    if (E == 0) return CTG_OK;
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    const bool host = mem == CTG_MEM_HOST;
    const uint64_t* di = ids;
    const double* dr = rows;
    double* dout = out;
    void* owned[3] = {nullptr, nullptr, nullptr};
    if (host) {
        owned[0] = dalloc(std::max<int64_t>(n, 1) * 8);
        owned[1] = dalloc(std::max<int64_t>(n, 1) * N_FEATURES * 8);
        owned[2] = dalloc(E * N_FEATURES * 8);
        if (!owned[0] || !owned[1] || !owned[2]) {
            set_error("ctg_merge_feature_rows: out of device memory");
            return CTG_ERR_NOMEM;
        }
        if (n) {
            CTG_CHECK(hipMemcpyAsync(owned[0], ids, n * 8, hipMemcpyHostToDevice, s));
            CTG_CHECK(hipMemcpyAsync(owned[1], rows, n * N_FEATURES * 8, hipMemcpyHostToDevice, s));
        }
        di = (const uint64_t*)owned[0];
        dr = (const double*)owned[1];
        dout = (double*)owned[2];
    }
    CTG_CHECK(hipMemsetAsync(dout, 0, E * N_FEATURES * 8, s));
    if (n) {
        uint32_t* k_in = (uint32_t*)dalloc(n * 4);
        uint32_t* k_out = (uint32_t*)dalloc(n * 4);
        uint32_t* i_in = (uint32_t*)dalloc(n * 4);
        uint32_t* i_out = (uint32_t*)dalloc(n * 4);
        if (!k_in || !k_out || !i_in || !i_out) {
            set_error("ctg_merge_feature_rows: out of device memory");
            return CTG_ERR_NOMEM;
        }
        CTG_CHECK(hipMemsetAsync(w.small + 3, 0, 4, s));
        CTG_CHECK(launch_row_keys(n, di, (uint64_t)id_begin, (uint64_t)id_end, k_in, i_in, w.small + 3, s));
        const unsigned kb = (unsigned)bits_for((uint64_t)std::max<int64_t>(E - 1, 1));
        size_t tb = 0;
        CTG_CHECK(rocprim::radix_sort_pairs(nullptr, tb, k_in, k_out, i_in, i_out, (size_t)n, 0u, kb, s));
        ensure(&w.temp, w.temp_bytes, tb + 256);
        tb = w.temp_bytes;
        CTG_CHECK(rocprim::radix_sort_pairs(w.temp, tb, k_in, k_out, i_in, i_out, (size_t)n, 0u, kb, s));
        CTG_CHECK(launch_merge_feature_rows(n, k_out, i_out, dr, dout, s));
        CTG_CHECK(hipMemcpyAsync(w.small_host + 3, w.small + 3, 4, hipMemcpyDeviceToHost, s));
        dfree(k_in); dfree(k_out); dfree(i_in); dfree(i_out);
    }
    if (host) CTG_CHECK(hipMemcpyAsync(out, dout, E * N_FEATURES * 8, hipMemcpyDeviceToHost, s));
    CTG_CHECK(hipStreamSynchronize(s));
    for (void* p : owned) dfree(p);
    if (n && w.small_host[3]) {
        set_error("ctg_merge_feature_rows: an edge id lies outside [id_begin, id_end)");
        return CTG_ERR_ARG;
    }
    return CTG_OK;
}

int ctg_unique_pairs(const uint64_t* pairs, int64_t n, int mem, void* stream, ctg_result** out) {
    DevLock dev_lock;
    if (!out || n < 0 || (n > 0 && !pairs)) {
        set_error("ctg_unique_pairs: bad arguments");
        return CTG_ERR_ARG;
    }
    *out = nullptr;
    const int dev = cur_dev();
    Workspace& w = ws(dev);
    CTG_CHECK(ws_init(w));
    hipStream_t s = (hipStream_t)stream;
    ctg_result* r = new ctg_result();
    r->device = dev;
    if (n == 0) {
        r->edges = (uint64_t*)dalloc(16);
        r->nodes = (uint64_t*)dalloc(8);
        *out = r;
        return CTG_OK;
    }
    uint64_t* dk = (uint64_t*)pairs;
    if (mem == CTG_MEM_HOST) {
        dk = (uint64_t*)dalloc(n * 16);
        if (!dk) {
            set_error("ctg_unique_pairs: out of device memory");
            delete r;
            return CTG_ERR_NOMEM;
        }
        CTG_CHECK(hipMemcpyAsync(dk, pairs, n * 16, hipMemcpyHostToDevice, s));
    }
    CTG_CHECK(hipMemsetAsync(w.counters, 0, sizeof(Counters), s));
    CTG_CHECK(launch_max_pairs(n, dk, &w.counters->max_v, s));
    CTG_CHECK(hipMemcpyAsync(w.counters_host, w.counters, sizeof(Counters), hipMemcpyDeviceToHost, s));
    CTG_CHECK(hipStreamSynchronize(s));
    DensePairs dp;
    if (w.counters_host->max_v >> 32) {
        int rc = dp.build(dk, n, s);
        if (rc) {
            if (mem == CTG_MEM_HOST) dfree(dk);
            delete r;
            return rc;
        }
    }
    ReduceJob J{};
    J.n = n;
    J.pairs = dp.U ? dp.dense : dk;
    J.stats = 0;
    J.need_adj = 0;
    J.max_v = dp.U ? (uint64_t)std::max<int64_t>(dp.U->n_nodes - 1, 0) : w.counters_host->max_v;
    J.scale = 1.0;
    J.offset = 0.0;
    hipError_t e = reduce_records(w, J, s, r);
    if (e == hipSuccess) e = dp.map_back(r, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (mem == CTG_MEM_HOST) dfree(dk);
    if (e != hipSuccess) {
        set_error(std::string("ctg_unique_pairs: ") + hipGetErrorString(e));
        ctg_free(r);
        return CTG_ERR_HIP;
    }
    *out = r;
    return CTG_OK;
}

int ctg_map_edge_ids(const uint64_t* global_edges, int64_t n_global, const uint64_t* query, int64_t n_query,
                     int64_t* out_ids, int mem, void* stream) {
    DevLock dev_lock;
    if (n_global < 0 || n_query < 0 || (n_query > 0 && (!query || !out_ids))) {
        set_error("ctg_map_edge_ids: bad arguments");
        return CTG_ERR_ARG;
    }
    if (n_query == 0) return CTG_OK;
    hipStream_t s = (hipStream_t)stream;
    if (mem == CTG_MEM_DEVICE) {
        CTG_CHECK(launch_find_edges(global_edges, n_global, query, n_query, out_ids, s));
        return CTG_OK;
    }
    uint64_t* g = (uint64_t*)dalloc(std::max<int64_t>(n_global, 1) * 16);
    uint64_t* q = (uint64_t*)dalloc(n_query * 16);
    int64_t* o = (int64_t*)dalloc(n_query * 8);
    if (!g || !q || !o) {
        set_error("ctg_map_edge_ids: out of device memory");
        return CTG_ERR_NOMEM;
    }
    if (n_global) CTG_CHECK(hipMemcpyAsync(g, global_edges, n_global * 16, hipMemcpyHostToDevice, s));
    CTG_CHECK(hipMemcpyAsync(q, query, n_query * 16, hipMemcpyHostToDevice, s));
    CTG_CHECK(launch_find_edges(g, n_global, q, n_query, o, s));
    CTG_CHECK(hipMemcpyAsync(out_ids, o, n_query * 8, hipMemcpyDeviceToHost, s));
    CTG_CHECK(hipStreamSynchronize(s));
    dfree(g);
    dfree(q);
    dfree(o);
    return CTG_OK;
}

int64_t ctg_result_num_edges(const ctg_result* r) { return r ? r->n_edges : -1; }
int64_t ctg_result_num_nodes(const ctg_result* r) { return r ? r->n_nodes : -1; }

static int copy_out(void* dst, const void* src, size_t bytes, int mem) {
    if (bytes == 0) return CTG_OK;
    if (!dst || !src) {
        set_error("copy: null pointer");
        return CTG_ERR_ARG;
    }
    CTG_CHECK(hipMemcpy(dst, src, bytes, mem == CTG_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    return CTG_OK;
}

int ctg_result_copy_edges(const ctg_result* r, uint64_t* dst, int mem) {
    return copy_out(dst, r->edges, (size_t)r->n_edges * 16, mem);
}
int ctg_result_copy_nodes(const ctg_result* r, uint64_t* dst, int mem) {
    return copy_out(dst, r->nodes, (size_t)r->n_nodes * 8, mem);
}
int ctg_result_copy_features(const ctg_result* r, double* dst, int mem) {
    if (!r->features && r->n_edges) {
        set_error("result has no features (graph-only call)");
        return CTG_ERR_ARG;
    }
    return copy_out(dst, r->features, (size_t)r->n_edges * N_FEATURES * 8, mem);
}
int ctg_result_copy_stats(const ctg_result* r, double* sums_dst, uint32_t* records_dst, int mem) {
    if (!r->stats && r->n_edges) {
        set_error("result has no statistics (call with keep_stats=1 and data)");
        return CTG_ERR_ARG;
    }
    int rc = copy_out(sums_dst, r->stat_sums, (size_t)r->n_edges * 16, mem);
    if (rc) return rc;
    return copy_out(records_dst, r->stats, (size_t)r->n_edges * WREC_WORDS * 4, mem);
}
const uint64_t* ctg_result_device_edges(const ctg_result* r) { return r ? r->edges : nullptr; }
const double* ctg_result_device_features(const ctg_result* r) { return r ? r->features : nullptr; }
int ctg_result_info(const ctg_result* r, int64_t* n_records, int64_t* n_direct) {
    if (!r) return CTG_ERR_ARG;
    if (n_records) *n_records = r->n_records;
    if (n_direct) *n_direct = r->n_direct;
    return CTG_OK;
}

void ctg_free(ctg_result* r) {
    if (!r) return;
    int d = cur_dev();
    if (r->device >= 0 && r->device != d) hipSetDevice(r->device);
    if (!r->owned.empty()) {   // the handle's arrays point into these (ctg_mgpu_merge)
        for (void* p : r->owned) dfree(p);
    } else {
        dfree(r->edges);
        dfree(r->nodes);
        dfree(r->features);
    }
    dfree(r->stats);
    dfree(r->stat_sums);
    if (r->device >= 0 && r->device != d) hipSetDevice(d);
    delete r;
}

int ctg_synth_volume(uint64_t* labels, float* boundary, const int64_t* shape, int64_t z_offset,
                     const int64_t* global_shape, int cell, uint64_t seed, uint64_t label_offset, double noise_amp,
                     void* stream) {
    if (!labels || !shape || cell <= 0) {
        set_error("ctg_synth_volume: bad arguments");
        return CTG_ERR_ARG;
    }
    int64_t g[3] = {z_offset + shape[0], shape[1], shape[2]};
    if (global_shape)
        for (int k = 0; k < 3; ++k) g[k] = global_shape[k];
    CTG_CHECK(launch_synth(labels, boundary, shape, z_offset, g, cell, seed, label_offset, noise_amp,
                           (hipStream_t)stream));
    return CTG_OK;
}

int ctg_synth_affinities(const float* boundary, float* affs, const int64_t* shape, int n_channels,
                         const int32_t* offsets, void* stream) {
    if (!boundary || !affs || !shape || !offsets || n_channels <= 0) {
        set_error("ctg_synth_affinities: bad arguments");
        return CTG_ERR_ARG;
    }
    CTG_CHECK(launch_synth_aff(boundary, affs, shape, n_channels, offsets, (hipStream_t)stream));
    return CTG_OK;
}

}  // extern "C"
