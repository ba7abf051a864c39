// Internal definitions shared by the ctg (cluster-tools graph) HIP sources.
// gfx950 / CDNA4 only.  See DESIGN.md for the data layout and the pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <string>
#include <vector>

#include "../../include/ctg.h"

namespace ctg {

// ---------------------------------------------------------------------------
// fixed geometry of the face-scan tiles and the LDS edge table
// ---------------------------------------------------------------------------
constexpr int WAVE = 64;
#ifndef CTG_SCAN_THREADS
#define CTG_SCAN_THREADS 512
#endif
constexpr int SCAN_THREADS = CTG_SCAN_THREADS;   // 8 waves per workgroup (1024: 16 waves, one per CU)
constexpr int TILE_X = 64;             // one wave row
constexpr int TILE_Y = 8;
// LDS edge-table entries: a multiple of 4 (4-slot buckets), at most one per
// thread in a flush; a power of two or not (the home bucket is a multiply-high)
#ifndef CTG_TABLE_CAP
#define CTG_TABLE_CAP SCAN_THREADS
#endif
constexpr int TABLE_CAP = CTG_TABLE_CAP;
static_assert(TABLE_CAP % 4 == 0 && TABLE_CAP <= SCAN_THREADS, "table capacity");
constexpr int NBINS = 40;              // vigra UserRangeHistogram<40> (nifty default)
constexpr int NSLOTS = NBINS + 2;      // left outliers, 40 bins, right outliers
constexpr int HWORDS = 21;             // 42 u16 slots packed in 21 u32 words
constexpr int NREC_WORDS = 24;         // narrow record: 21 hist words + cnt + min + max
// narrow records live in 128-byte bodies (one cache line each, so the
// reduction's gather touches exactly one line per record):
//   words 0..3 (sum f64, sum of squares f64), 4..27 the NREC_WORDS, 28..31 zero
constexpr int NREC_STRIDE = 32;
constexpr int NREC_OFF = 4;
constexpr int NREC_PIV = 28;           // word 28: the pivot (f32 bits) the two sums are taken about
constexpr int WREC_WORDS = 48;         // wide record: 42 u32 slots + cnt + min + max + pivot + pad
constexpr int WREC_PIV = 45;
// Statistics are kept as shifted sums about a per-entry pivot p (the entry's
// first sample): S1 = sum(x - p), S2 = sum((x - p)^2).  The variance
// (S2 - S1^2/n)/n then cancels only the spread of the samples, not their
// magnitude, and records / partial tables combine by re-pivoting
// (Moments::add, ctg_reduce.hip).  A pivot word of 0 is the plain power sums.
constexpr uint32_t PIV_EMPTY = 0xFFFFFFFFu;   // table entry without a pivot yet (a NaN no sample carries)
constexpr uint32_t ADJ_FLAG = 0x80000000u;  // record/edge came from a nearest-neighbour face
constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr int N_FEATURES = 10;

// order-preserving float <-> u32 mapping for LDS/global atomicMin/Max
__host__ __device__ inline uint32_t f2ord(float f) {
    uint32_t b;
    __builtin_memcpy(&b, &f, 4);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__host__ __device__ inline float ord2f(uint32_t o) {
    uint32_t b = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    float f;
    __builtin_memcpy(&f, &b, 4);
    return f;
}
constexpr uint32_t ORD_POS_INF = 0xFF800000u;  // f2ord(+inf)
constexpr uint32_t ORD_NEG_INF = 0x007FFFFFu;  // f2ord(-inf)

// vigra RangeHistogramBase::update binning -> slot in [0, NSLOTS)
__host__ __device__ inline int hist_slot(double x, double scale, double offset) {
    double m = scale * (x - offset);
    if (m == (double)NBINS) return NBINS;          // index nbins-1 -> slot nbins
    if (!(m < (double)NBINS)) return (m != m) ? 0 : NBINS + 1;  // right outlier (NaN -> left)
    if (m <= -1.0) return 0;                          // (int)m < 0 -> left outlier
    return (int)m + 1;                                // trunc toward zero, as (int)m
}

__host__ __device__ inline uint32_t hash_key(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return (uint32_t)k;
}

// Blocked Bloom filter of RAG edge keys (the long-range affinity prefilter),
// blocked by OWNER label: an edge (u, v) is stored twice, as u -> v in the
// 64-B block of u and as v -> u in the block of v; a probe from a voxel of
// label a for partner b tests a -> b: 4 bits of ONE 64-bit word of a's block.
// A wave's probes then touch one cache line per distinct own label (a few per
// row) instead of one per distinct pair, and the line of a label stays hot in
// L2 over every channel and plane that label's cell spans.
__host__ __device__ inline uint64_t bloom_hash(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 29;
    k *= 0xc4ceb9fe1a85ec53ull;
    return k ^ (k >> 32);
}
// h: bloom_hash((owner << 32) | other)
__host__ __device__ inline uint64_t bloom_bits(uint64_t h) {
    return (1ull << (h & 63)) | (1ull << ((h >> 6) & 63)) | (1ull << ((h >> 12) & 63)) | (1ull << ((h >> 18) & 63));
}
// word of the owner's block (block_mask = blocks - 1, 8 words per block)
__host__ __device__ inline uint32_t bloom_block(uint32_t owner, uint32_t block_mask) {
    return ((uint32_t)(bloom_hash(owner) >> 24) & block_mask) * 8u;
}
__host__ __device__ inline uint32_t bloom_word(uint32_t block, uint64_t h) { return block + ((uint32_t)(h >> 40) & 7u); }

// ---------------------------------------------------------------------------
// records: the face scan flushes one record per (tile, edge)
// ---------------------------------------------------------------------------
// The scan reserves record slots from NREG region counters (region r owns
// slots [r*rcap, (r+1)*rcap)) instead of one global counter: same-address
// device atomics serialize (~25 ns each), and one counter per flush across
// every workgroup of the chip was a measurable queue.
constexpr int NREG = 64;

struct RegionPrefix {          // exclusive prefix of the region counts (host-computed)
    uint32_t off[NREG + 1];
};

struct RecordBuf {
    uint64_t* key = nullptr;      // (u << 32) | v
    double2* sums = nullptr;      // wide records: (sum, sum of squares); compact: unused (in the body)
    uint32_t* hist = nullptr;     // narrow: NREC_STRIDE-word bodies; wide: WREC_WORDS per record
    int64_t cap = 0;
    int64_t rcap = 0;             // slots per region (cap / NREG)
};

// one array of a batched call (ctg_rag_blocks): the host's ctg_block_desc
// in device memory plus the tile bookkeeping of the launch
struct BlockGeom {
    int64_t label_offset;    // element offset of the array in the labels arena
    int64_t data_offset;     // element offset in the data arena (affinities: channel 0 of C x V)
    int32_t shape[3];
    int32_t own_begin[3], own_end[3];
    int32_t graph_begin[3], graph_end[3];
    int32_t ntx, nty, ntz;   // tiles along x, y, z
};

struct ScanParams {
    const void* labels;
    const void* data;          // boundary (Z,Y,X) or affinities (C,Z,Y,X); may be null
    int label_bits;            // 64 or 32
    int data_kind;             // CTG_DATA_*
    int n_channels;            // 0 -> boundary map
    int offsets[CTG_MAX_CHANNELS][3];
    int64_t shape[3];
    int64_t own_begin[3];
    int64_t own_end[3];
    double scale, offset;      // histogram mapping
    double u8_scale;           // uint8 -> float factor (1/255)
    int tile_z;                // z-planes per workgroup
    int tile_z_narrow;         // z-planes per workgroup of the narrow-tile launch (0: tile_z)
    int check_planes;          // planes between flush decisions
    int fast40;                // histogram range [0,1) x 40 bins: exact f32 binning
    int ablate;                // diagnostic: 8 loads only, 32 staging without fold
    // long-range affinity channels: samples whose (u,v) fails this blocked
    // Bloom filter of the RAG edge keys ((u << 32) | v) are dropped in the scan
    // (bloom_mask = blocks - 1, 8 words a block); the reduce drops the false positives, keeping
    // only keys that nearest-neighbour samples (MARK_ONE_ADJ) flagged
    const unsigned long long* bloom;
    uint32_t bloom_mask;
    int64_t ntiles[3];         // tiles along x, y, z (set by the launcher)
    int xcd_remap;             // 1: XCD-contiguous tile order (see k_face_scan)
    // affinities: the three nearest-neighbour channels are present, so every
    // RAG edge gets a sample of one of them and the scan pushes no adjacency
    // markers (with a Bloom filter those samples carry the flag instead)
    int skip_adj_marks;
    // the three nearest-neighbour channels alone (whole array, no long-range
    // channel, adjacency proven by every sample): scanned as faces, like a
    // boundary map, the sample of face (p - e_a, p) being aff[nn_ch[a], p]
    int nn3;
    int nn_ch[3];              // channel of the offset -e_a, a = z, y, x
    // long-range calls (Bloom-filtered): the three nearest-neighbour channels
    // as faces (their samples are the adjacency proofs), the other channels
    // loop_ch[0 .. n_loop) in the channel loop
    int nn_mix;
    int n_loop;
    int loop_ch[CTG_MAX_CHANNELS];
    uint32_t lr_mask;          // bit c: channel c is long-range (|offset|_1 > 1)
    int narrow_rows;           // boundary maps: 1 2-row waves (fragmented volumes, see ctg_scan.hip),
                               // 2 decided on the device from density[] (no host round trip)
    const uint32_t* density;   // sampled x-face changes / pairs (k_density), for narrow_rows == 2
    // batched blocks (ctg_rag_blocks): workgroup w scans a tile of array b with
    // tile_prefix[b] <= w < tile_prefix[b+1]; keys carry b in the bits of u
    // from tag_shift up, so labels must stay below 2^tag_shift (else the label
    // overflow flag is raised and the host relabels densely)
    const BlockGeom* blocks;
    const uint32_t* tile_prefix;
    int n_blocks;
    int64_t batch_tiles;       // tile_prefix[n_blocks]: the launch's workgroups
    int tag_shift;             // 32: no tag (n_blocks == 1)
    uint32_t label_hi_mask;    // bits a narrowed label must not have (overflow flag)
};

struct Counters {               // device-side counters, zeroed per call
    unsigned long long n_records;
    unsigned long long n_direct;     // faces emitted past a full LDS table
    unsigned long long label_overflow;  // labels >= 2^32 seen by the 32-bit key path
    unsigned long long max_v;        // largest label in any key
    unsigned long long pad[8];      // diagnostics (ablation checks, s_memtime stamps)
    unsigned long long rcount[NREG];  // records reserved per region (may exceed rcap: overflow)
};

// record slot of sorted position r: a u32 index array, or the low ib bits of
// the packed sort keys (keys-only record sort, no unpack pass)
struct Perm {
    const uint32_t* p32;
    const uint64_t* p64;
    int ib;
    __device__ __forceinline__ uint32_t operator()(uint32_t r) const {
        return p64 ? (uint32_t)(p64[r] & ((1ull << ib) - 1ull)) : p32[r];
    }
};

// CTG_DEFER_STATS: what a result needs to rebuild an edge's mergeable
// statistics from its records -- run e of the sorted records is slots
// perm(offs[e] .. offs[e] + runs[e]) of the narrow record bodies `hist` --
// valid while the workspace's generation is still `gen`
struct DeferredStats {
    int on = 0;
    const uint32_t* offs = nullptr;
    const uint32_t* runs = nullptr;
    Perm perm{nullptr, nullptr, 0};
    const uint32_t* hist = nullptr;
    uint64_t gen = 0;
};

struct ReduceOut {
    uint64_t* edges;      // 2E
    double* feats;        // 10E or null
    uint32_t* keep;       // E or null
    uint32_t* wstats;     // WREC_WORDS*E or null
    double2* wsums;       // E or null
    uint32_t* count_out;  // null, or receives the edge count (no compaction follows)
    int ablate;           // diagnostics (CTG_REDUCE_ABLATE): 1 no quantiles, 2 no record loads, 4 no feature stores
};

constexpr int BK_SMALL_WORDS = 5 * 4096 + 16;   // bucket sort: counts, offsets, cursors, run heads
constexpr int GS_SMALL_WORDS = 5 * 65536 + 8;    // group sort: counts, offsets, cursors, misc, look-back state

struct Workspace {
    int device = -1;
    // bumped by every call that overwrites the records or the sort / run
    // buffers (a CTG_DEFER_STATS handle compares it)
    uint64_t gen = 1;
    RecordBuf rec;
    // sort / reduce scratch
    uint64_t* sk_in = nullptr; uint64_t* sk_out = nullptr;
    uint32_t* idx_in = nullptr; uint32_t* idx_out = nullptr;
    int64_t sort_cap = 0;
    uint64_t* uniq = nullptr; uint32_t* runs = nullptr; uint32_t* offs = nullptr;
    uint32_t* keep = nullptr; uint32_t* pos = nullptr;
    int64_t edge_cap = 0;
    void* temp = nullptr; size_t temp_bytes = 0;
    Counters* counters = nullptr;        // device
    Counters* counters_host = nullptr;   // pinned
    unsigned int* small = nullptr;       // device scalars (run counts etc.)
    unsigned int* small_host = nullptr;
    uint32_t* bsort = nullptr;           // device: bucket-sort scratch, BK_SMALL_WORDS u32 (ctg_sort.hip)
    uint32_t* gsort = nullptr;           // device: group-sort scratch, GS_SMALL_WORDS u32 (ctg_sort.hip)
    uint64_t* mgpu_spl = nullptr;        // device: the exchange's splitters, CTG_MGPU_MAX_WORLD u64
    // host->device staging of volumes
    void* stage[2] = {nullptr, nullptr};
    size_t stage_bytes[2] = {0, 0};
    // timing
    hipEvent_t ev[10];   // 0..6 phases of a call; 8, 9 bracket the label narrowing (prep)
    bool events = false;
    double last_ms[8] = {0};   // scan, pack, sort, segment, reduce, nodes, total, narrow
    int64_t last_records = 0, last_direct = 0;
    int profiling = 0;
};

Workspace& ws(int device);
int current_device();
void set_error(const std::string& msg);
void ensure(void** p, size_t& have, size_t need);
hipError_t ensure_records(Workspace& w, int64_t need, int wide);
// the library's caching device allocator (stream-ordered reuse, ctg_api.hip)
void* dev_alloc(size_t bytes);
void dev_free(void* p);

}  // namespace ctg

// result handle (opaque in the C ABI)
struct ctg_result {
    int device = -1;
    // batched blocks (ctg_rag_blocks): rows [edge_off[b], edge_off[b+1]) of the
    // edge / feature tables and [node_off[b], node_off[b+1]) of the node table
    // belong to block b
    std::vector<int64_t> edge_off, node_off;
    int64_t n_edges = 0;
    int64_t n_nodes = 0;
    uint64_t* edges = nullptr;      // device (E,2)
    uint64_t* nodes = nullptr;      // device (N,)
    double* features = nullptr;     // device (E,10) or null
    uint32_t* stats = nullptr;      // device wide records (E, WREC_WORDS) or null
    double2* stat_sums = nullptr;   // device (E,) (sum, sumsq) or null
    int64_t n_records = 0;
    int64_t n_direct = 0;
    // affinity partial table (CTG_NO_ADJ_FILTER): a key is an edge only where
    // some record carries the ADJ bit (decided after a merge)
    int partial_adj = 0;
    // CTG_DEFER_STATS: statistics rows rebuilt from the records on demand
    ctg::DeferredStats defer;
    // allocations this handle frees instead of the five pointers above, which
    // then point into them (a multi-GPU shard that is a range of its rank's
    // local table: ctg_mgpu_merge)
    std::vector<void*> owned;
};

namespace ctg {
hipError_t mgpu_sample(const uint64_t* edges, int64_t E, int64_t* meta, hipStream_t s);
hipError_t mgpu_split(const uint64_t* edges, int64_t E, const uint64_t* nodes, int64_t N, const int64_t* meta_all,
                      int world, uint64_t* spl, int64_t* counts, hipStream_t s);
hipError_t mgpu_pack(const ctg_result* r, const int64_t* counts_all, int world, int rank, int64_t* send,
                     hipStream_t s);
// *lib_rc: a library status (with its message set) when a nested C-ABI call
// failed, or CTG_ERR_UNSUPPORTED for a shard past the u32 row indices
hipError_t mgpu_merge(ctg_result* local, const int64_t* recv, const int64_t* counts_all, int world, int rank,
                      double hist_lo, double hist_hi, hipStream_t s, ctg_result* out, int* lib_rc);
}  // namespace ctg

#define CTG_CHECK(expr)                                                        \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            ctg::set_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
            return CTG_ERR_HIP;                                                \
        }                                                                      \
    } while (0)
