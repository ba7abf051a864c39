// Face scan: the O(V) hot loop of the RAG + edge-feature path (gfx950).
//
// Replaces the per-face std::set / findEdge loop of nifty.distributed, called
// at graph/initial_sub_graphs.py:124-129 (graph) and
// features/block_edge_features.py:127-145 (features): one launch computes the
// edge set AND the per-edge statistics of a whole z-slab.
//
// Geometry.  A workgroup (8 waves) owns a 64 (x) x 8*ROWS (y) x tile_z (z)
// tile.  Each wave holds ROWS rows (+ the y-halo row) of one z-plane in
// registers, lane = x, and walks z with the next plane's loads in flight while
// it works on the current plane, so every label / sample is read from HBM once
// (plus the halo row).  Labels are reduced to their low 32 bits on load; any
// non-zero high half raises an overflow flag and the host re-runs the call on
// a dense relabelling (ctg_api.hip), so the loop compares and packs u32.
//
// Faces.  For a row, the x face (x, x+1) takes its neighbour with one DPP
// wave_shl (lane 63 from the x-halo register), the y face compares with the
// next row register, the z face with the prefetched plane.  The active lanes
// of one site (row x axis) append (u, v, sample a, sample b) to the wave's LDS
// stage at ballot/mbcnt positions; a full stage is folded with one face per
// lane into the workgroup's LDS edge table (open addressing, 4-slot home
// buckets read with two ds_read_b128): per edge the sample count, f64 sum and
// sum of squares, order-preserving min / max and the 42-slot vigra histogram
// (u16 slots in u32 words).
//
// Overflow safety without returning atomics.  A histogram slot never exceeds
// its entry's count, and an entry's count never exceeds the samples the eight
// waves folded since the last table flush.  Each wave keeps a sample budget of
// 65535 / 8 per flush interval: before a fold batch that would pass it, the
// wave forces a flush.  So no u16 slot can wrap, and every statistics update
// is a fire-and-forget LDS atomic.  Table fill only sets a per-lane "need
// flush" flag; the wave then raises the workgroup's flush request, which every
// wave polls after each fold batch and plane (see k_face_scan).
#include <type_traits>

#include "ctg_internal.h"

#ifndef CTG_ROWS
#define CTG_ROWS 4
#endif

namespace ctg {

enum { MODE_GRAPH = 0, MODE_BOUNDARY = 1, MODE_AFFINITY = 2, MODE_AFF_NN = 3, MODE_AFF_MIX = 4 };

// y rows per wave, held in registers: 4, or 2 for highly fragmented volumes
// (the workgroup's tile cross-section, hence its live edge set, halves: the
// table then holds it and flushes -- records -- drop by ~40 % at cell 5)
constexpr int ROWS_WIDE = CTG_ROWS;
#ifndef CTG_ROWS_NARROW
#define CTG_ROWS_NARROW 2
#endif
constexpr int ROWS_NARROW = CTG_ROWS_NARROW;
#ifndef CTG_AFF_ROWS
#define CTG_AFF_ROWS CTG_ROWS
#endif
constexpr int ROWS_AFF = CTG_AFF_ROWS;   // affinity maps: rows per wave (the channel loop's registers scale with it)
constexpr int WAVES = SCAN_THREADS / WAVE;                // 8
constexpr int WG_ROWS = ROWS_WIDE * WAVES;                // tile y extent (the default kernel)
#ifndef CTG_AFF_G
#define CTG_AFF_G 2   // (3: 12-channel scan 42.6 -> 42.1 ms, but its register spills add 26 GB of reads and 11 GB of writes)
#endif
// affinity channels whose gathers / sample loads / Bloom probes are issued
// together (x ROWS rows): the channel loop is bound by memory round trips
constexpr int AFF_G = CTG_AFF_G;
#ifndef CTG_NPER
#define CTG_NPER 2
#endif
constexpr int NPER = CTG_NPER;                            // staged entries folded per lane
// the narrow-tile boundary kernel (configs[4]'s fragmented volumes) folds one
// staged entry per lane: its scan 15.3 -> 14.5 ms, records +5 %, step -1.5 %
// (A/B of CTG_NPER=1 builds); every other kernel keeps NPER
#ifndef CTG_NPER_NARROW
#define CTG_NPER_NARROW 1
#endif
// u16 histogram slots: a table entry holds at most 65535 samples.  Each wave
// folds at most this many samples between two table flushes (it requests a
// flush before a batch would exceed it), so no entry can pass the bound.
constexpr uint32_t WAVE_SAMPLE_BUDGET = 65535u / WAVES;
// flush past 5/8 of the table: more live entries per flush interval, fewer
// records (A/B over the BASELINE workloads, tools/ab_run.sh: 256 -> 320 cut
// configs[4]'s records 191 M -> 148 M and its step 36.7 -> 32.2 ms, equal at
// 512^3; 384+ lengthens the probe chains and slows the scan)
#ifndef CTG_FILL_SOFT
#define CTG_FILL_SOFT (TABLE_CAP * 5 / 8)
#endif
constexpr uint32_t FILL_SOFT = CTG_FILL_SOFT;
// (the inserting lane compares the returned fill count: non-returning
// increments checked at every poll measured slower, 2048^3 scan 29.38 -> 29.92 ms)
constexpr uint32_t MARK_ADJ = 0xFFFFFFFFu;                // stage entry: nearest-neighbour face, no sample
constexpr uint32_t MARK_ONE = 0xFFFFFFFEu;                // stage entry: one affinity sample in .z
constexpr uint32_t MARK_ONE_ADJ = 0xFFFFFFFDu;            // ... of a nearest-neighbour face (Bloom-filtered calls)

struct __align__(16) Table {
    uint64_t key[TABLE_CAP];
    double sum[TABLE_CAP];
    double sq[TABLE_CAP];
    // hist words 0..20, 21 cnt|ADJ, 22 min, 23 max, 24 pivot (the entry's
    // first sample, claimed by CAS); odd row stride (25 words) so atomics to
    // different entries spread over the LDS banks
    uint32_t w[TABLE_CAP][NREC_WORDS + 1];
    uint16_t compact[(TABLE_CAP + WAVE - 1) / WAVE * WAVE];   // per-wave flush ranks
    uint32_t wave_cnt[WAVES];
    uint32_t used;
    uint32_t flush_req;   // a wave asked for a flush; every wave joins at its next poll
    uint32_t live;        // waves still walking their planes
    uint32_t ncompact;
    unsigned long long base;
    unsigned long long maxv;
};

__device__ __forceinline__ void entry_reset(Table& T, int e) {
    T.key[e] = EMPTY_KEY;
    T.sum[e] = 0.0;
    T.sq[e] = 0.0;
#pragma unroll
    for (int j = 0; j < HWORDS + 1; ++j) T.w[e][j] = 0u;
    T.w[e][22] = ORD_POS_INF;
    T.w[e][23] = ORD_NEG_INF;
    T.w[e][24] = PIV_EMPTY;
}

// pivot bits of a sample: its own bits, NaN -> 0 (never PIV_EMPTY)
__device__ __forceinline__ uint32_t pivot_bits(float a) { return a == a ? __float_as_uint(a) : 0u; }

// home bucket: four slots starting at a multiple of 4, read by two ds_read_b128
// Two full-rate 24-bit multiplies (v_mul_u32_u24) instead of 32-bit ones and a
// 64-bit multiply-add: bits 14.. of the product sum mix every one of the low
// 24 bits of u and v; labels that differ only above bit 24 share buckets,
// which costs probes, never correctness.
constexpr bool TABLE_POW2 = (TABLE_CAP & (TABLE_CAP - 1)) == 0;
// hash -> first slot of a 4-slot bucket (any table size: multiply-high)
__device__ __forceinline__ uint32_t bucket_of(uint32_t h) {
    if constexpr (TABLE_POW2) return h & (TABLE_CAP - 4);
    else return __umulhi(h, (uint32_t)(TABLE_CAP / 4)) * 4u;
}
__device__ __forceinline__ uint32_t home_bucket(uint32_t u, uint32_t v) {
    const uint32_t p = (u & 0xFFFFFFu) * 0x9E3779u + ((v ^ (u >> 24)) & 0xFFFFFFu) * 0x85EBCBu;
    return TABLE_POW2 ? bucket_of(p >> 12) : bucket_of(p << 8);
}

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for every
// outstanding global load (vmcnt(0)), which would drain the next plane's
// prefetch at every flush decision; nothing in the scan needs global-memory
// ordering between waves (records are consumed by later kernels).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Flush by waves: every wave writes out the live entries among its own 64
// table slots (entry tid) - its own record range from one global atomic, its
// own 128-byte bodies, its own resets - so the flush needs two workgroup
// barriers (table stable / table empty) instead of a workgroup-wide
// compaction with one serial record reservation.  (Tried: keeping entries
// touched in the planes the waves still work on across a flush -- at a
// 512-entry table nearly every live entry is that recent, and records did not
// drop.)
template <int MODE>
__device__ __noinline__ void table_flush_waves(Table& T, RecordBuf R, Counters* C) {
    lds_barrier();
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1), wv = tid >> 6;
    if (tid == 0) {   // no wave inserts or polls between the two barriers
        T.used = 0;
        T.flush_req = 0;
    }
    // entry tid (threads past TABLE_CAP own none)
    const uint64_t k = tid < TABLE_CAP ? T.key[tid] : EMPTY_KEY;
    const bool out = k != EMPTY_KEY;
    const uint64_t m = __ballot(out);
    if (m) {
        const uint32_t n = (uint32_t)__popcll(m);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        uint32_t mv = out ? (uint32_t)k : 0u;
        for (int o = 32; o > 0; o >>= 1) mv = max(mv, (uint32_t)__shfl_xor((int)mv, o, WAVE));
        const int reg = (blockIdx.x * WAVES + wv) & (NREG - 1);
        unsigned long long b = 0;
        if (lane == 0) {
            b = atomicAdd(&C->rcount[reg], (unsigned long long)n);
            if (mv) atomicMax(&T.maxv, (unsigned long long)mv);
        }
        const unsigned long long base = ((unsigned long long)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
        const unsigned long long rcap = (unsigned long long)R.rcap, slot0 = (unsigned long long)reg * rcap + base;
        uint16_t* cw = T.compact + wv * WAVE;
        if (out) {
            if (base + rank < rcap) R.key[slot0 + rank] = k;
            cw[rank] = (uint16_t)tid;
        }
        __builtin_amdgcn_wave_barrier();
        if (MODE != MODE_GRAPH) {
            // 16-byte pieces of the 128-byte bodies: piece q of record r (eight
            // consecutive lanes per record; n * 8 is a multiple of 8, so a
            // record's lanes are active together).  The sample count is not
            // kept in the table (one atomic less per face): it is the sum of
            // the 42 u16 histogram slots, reduced over the record's lanes here.
            for (uint32_t f = lane; f < n * 8; f += WAVE) {
                const uint32_t r = f >> 3, q = f & 7;
                const int e = cw[r];
                uint4 val = make_uint4(0u, 0u, 0u, 0u);
                if (q == 0) {
                    const double2 sq2 = make_double2(T.sum[e], T.sq[e]);
                    val = *reinterpret_cast<const uint4*>(&sq2);
                } else if (q < 7) {
                    const uint32_t* w = &T.w[e][4 * (q - 1)];
                    val = make_uint4(w[0], w[1], w[2], w[3]);
                } else {   // word 28: the pivot (none: adjacency-only entry, no samples)
                    const uint32_t pv = T.w[e][24];
                    val.x = pv == PIV_EMPTY ? 0u : pv;
                }
                // histogram words 0..20 sit in pieces 1..5 and piece 6's .x
                auto h2 = [](uint32_t v) { return (v & 0xFFFFu) + (v >> 16); };
                uint32_t c = (q >= 1 && q <= 5) ? h2(val.x) + h2(val.y) + h2(val.z) + h2(val.w)
                                                : (q == 6 ? h2(val.x) : 0u);
                c += (uint32_t)__shfl_xor((int)c, 1, WAVE);
                c += (uint32_t)__shfl_xor((int)c, 2, WAVE);
                c += (uint32_t)__shfl_xor((int)c, 4, WAVE);
                if (q == 6) val.y |= c;   // word 21: count | ADJ
                if (base + r < rcap) reinterpret_cast<uint4*>(R.hist + (slot0 + r) * NREC_STRIDE)[q] = val;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (out) entry_reset(T, tid);
    }
    lds_barrier();
}

// One record straight to HBM: a key that found no room in the table.
// sa / sb: histogram slots of the samples (-1: none); s / q / mn / mx: the
// shifted sum, sum of squares (about the pivot bits piv) and ordered min / max
// this record carries.
__device__ __noinline__ void emit_direct(RecordBuf R, Counters* C, uint64_t key, uint32_t cnt_flag, int sa, int sb,
                                         double s, double q, uint32_t mn, uint32_t mx, uint32_t piv,
                                         bool with_stats) {
    const int reg = blockIdx.x & (NREG - 1);
    const unsigned long long j = atomicAdd(&C->rcount[reg], 1ull);
    atomicAdd(&C->n_direct, 1ull);
    atomicMax(&C->max_v, (unsigned long long)(key & 0xFFFFFFFFull));
    if (j >= (unsigned long long)R.rcap) return;
    const unsigned long long i = (unsigned long long)reg * (unsigned long long)R.rcap + j;
    R.key[i] = key;
    if (!with_stats) return;
    uint32_t* b = R.hist + i * NREC_STRIDE;
    reinterpret_cast<double2*>(b)[0] = make_double2(s, q);
    for (int j = 0; j < HWORDS; ++j) {
        uint32_t v = 0;
        if (sa >= 0 && (sa >> 1) == j) v += 1u << ((sa & 1) * 16);
        if (sb >= 0 && (sb >> 1) == j) v += 1u << ((sb & 1) * 16);
        b[NREC_OFF + j] = v;
    }
    b[NREC_OFF + 21] = cnt_flag;
    b[NREC_OFF + 22] = mn;
    b[NREC_OFF + 23] = mx;
    b[NREC_PIV] = piv;
    for (int j = NREC_PIV + 1; j < NREC_STRIDE; ++j) b[j] = 0u;
}

// affinity samples are read once: a non-temporal load keeps them from
// evicting the label lines the long-range partner gathers re-read from L2
// (CTG_NT_AFF=0: ordinary loads)
#ifndef CTG_NT_AFF
#define CTG_NT_AFF 1
#endif
template <typename DataT>
__device__ __forceinline__ float load_val_stream(const DataT* p, int64_t i) {
    if constexpr (CTG_NT_AFF == 0) {
        if constexpr (sizeof(DataT) == 1) return __fdiv_rn((float)p[i], 255.0f);
        else return p[i];
    } else if constexpr (sizeof(DataT) == 1) {
        return __fdiv_rn((float)__builtin_nontemporal_load(p + i), 255.0f);
    } else {
        return __builtin_nontemporal_load(p + i);
    }
}

template <typename DataT>
__device__ __forceinline__ float load_val(const DataT* p, int64_t i) {
    if constexpr (sizeof(DataT) == 1) {
        return __fdiv_rn((float)p[i], 255.0f);
    } else {
        return p[i];
    }
}

// low 32 bits of label i (a 4-B gather for 64-bit labels; little-endian)
template <typename LabelT>
__device__ __forceinline__ uint32_t load_lo(const LabelT* L, int64_t i) {
    if constexpr (sizeof(LabelT) == 8) return reinterpret_cast<const uint32_t*>(L)[2 * i];
    else return (uint32_t)L[i];
}

// vigra RangeHistogramBase binning of one sample -> slot in [0, NSLOTS)
// (hist_slot's rule, ctg_internal.h), branch-free on the f64 value the sums
// use anyway: m = scale * (x - offset); FAST40 (offset 0, scale 40) skips the
// subtraction -- 40 * x is exact in f64 for every float x, so the slot is the
// double-precision rule's.  Selects instead of branches: no exec-mask
// juggling in the fold.
template <bool FAST40>
__device__ __forceinline__ int sample_slot(double dx, double scale, double offset) {
    const double m = FAST40 ? dx * 40.0 : scale * (dx - offset);
    int s = (int)m + 1;                              // trunc toward zero (v_cvt_i32_f64 saturates)
    s = m <= -1.0 ? 0 : s;                           // left outlier
    s = !(m < (double)NBINS) ? NBINS + 1 : s;        // right outlier
    s = m != m ? 0 : s;                              // NaN -> left
    return m == (double)NBINS ? NBINS : s;           // index nbins-1
}

// 2-sample histogram add: one atomic when both samples share a word
__device__ __forceinline__ void hist_add2(Table& T, int e, int sa, int sb) {
    const uint32_t ia = 1u << ((sa & 1) * 16), ib = 1u << ((sb & 1) * 16);
    const bool same = (sa >> 1) == (sb >> 1);
    atomicAdd(&T.w[e][sa >> 1], same ? ia + ib : ia);
    if (!same) atomicAdd(&T.w[e][sb >> 1], ib);
}

// probe/insert past the home bucket (a key missing from its bucket); -1 when
// the table is too full.  INSERT_OVER is or-ed into the slot when this insert
// took the table past FILL_SOFT (a flag, not a reference: a bool& argument of
// an out-of-line call would live in scratch memory).
constexpr int INSERT_OVER = 0x10000;
#ifndef CTG_PROBE_BUCKETS
#define CTG_PROBE_BUCKETS 16   // buckets (of 4 slots) a key may walk past its home bucket
#endif
__device__ __noinline__ int table_insert(Table& T, uint32_t h, int empty, uint64_t key) {
    // Probe order is linear from the home bucket's start, so a key never sits
    // beyond an empty slot; a lost race or a full bucket walks on.  Whole
    // buckets are read at a time (two ds_read_b128, as the home-bucket probe):
    // one LDS round trip per 4 slots instead of one per slot.
    uint32_t b = h;
    int j0 = empty >= 0 ? empty : 4;   // first slot of bucket b still to look at
#pragma unroll 1
    for (int i = 0; i <= CTG_PROBE_BUCKETS;) {
        if (j0 >= 4) {
            b = TABLE_POW2 ? ((b + 4) & (TABLE_CAP - 1)) : (b + 4 >= (uint32_t)TABLE_CAP ? 0u : b + 4);
            j0 = 0;
            ++i;
            continue;
        }
        const uint4 b01 = *reinterpret_cast<const uint4*>(&T.key[b]);
        const uint4 b23 = *reinterpret_cast<const uint4*>(&T.key[b + 2]);
        const uint64_t kk[4] = {((uint64_t)b01.y << 32) | b01.x, ((uint64_t)b01.w << 32) | b01.z,
                                ((uint64_t)b23.y << 32) | b23.x, ((uint64_t)b23.w << 32) | b23.z};
        uint32_t km = 0, em = 0;   // slots (>= j0) holding the key / empty, as bit masks
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            km |= (kk[j] == key ? 1u : 0u) << j;
            em |= (kk[j] == EMPTY_KEY ? 1u : 0u) << j;
        }
        const uint32_t live = ~((1u << j0) - 1u);
        km &= live;
        em &= live;
        if ((km | em) == 0) {
            j0 = 4;
            continue;
        }
        const int first = __builtin_ctz(km | em);
        if ((km >> first) & 1u) return (int)(b + first);
        const uint64_t old = atomicCAS((unsigned long long*)&T.key[b + first], (unsigned long long)EMPTY_KEY,
                                       (unsigned long long)key);
        if (old == EMPTY_KEY)
            return (int)(b + first) | (atomicAdd(&T.used, 1u) + 1u > FILL_SOFT ? INSERT_OVER : 0);
        if (old == key) return (int)(b + first);
        j0 = first + 1;   // lost the slot to another key: re-read the rest of the bucket
    }
    return -1;
}

// slot of key in its 4-slot home bucket (b01, b23 = the bucket's keys), -1 if
// absent; `empty` = first empty slot of the bucket or -1
__device__ __forceinline__ int bucket_match(const uint4& b01, const uint4& b23, uint32_t h, uint64_t key,
                                            int& empty) {
    const uint64_t kk[4] = {((uint64_t)b01.y << 32) | b01.x, ((uint64_t)b01.w << 32) | b01.z,
                            ((uint64_t)b23.y << 32) | b23.x, ((uint64_t)b23.w << 32) | b23.z};
    int s = -1;
    empty = -1;
#pragma unroll
    for (int j = 3; j >= 0; --j) {
        s = kk[j] == key ? (int)h + j : s;
        empty = kk[j] == EMPTY_KEY ? j : empty;
    }
    return s;
}

// statistics of one staged entry into table slot s (s < 0: direct record);
// pv: the slot's pivot word as read by the batch (PIV_EMPTY: none yet); cur:
// its ordered (min, max) as read by the batch
template <int MODE, bool FAST40, bool BATCH, typename StageT>
__device__ __forceinline__ void fold_stats(Table& T, const StageT& e, int s, uint32_t pv, uint2 cur, RecordBuf R,
                                           Counters* C, double scale, double offset, bool& need, int ablate) {
    constexpr bool BND = MODE == MODE_BOUNDARY;
    constexpr bool AFF = MODE == MODE_AFFINITY || MODE == MODE_AFF_MIX;
    const uint64_t key = ((uint64_t)e.x << 32) | e.y;
    if constexpr (MODE == MODE_GRAPH) {
        if (s < 0) emit_direct(R, C, key, 0u, -1, -1, 0.0, 0.0, 0u, 0u, 0u, false);
        return;
    } else {
        // adjacency-only entries: a nearest-neighbour face of an affinity map, or
        // (batched blocks) a boundary face of the block's sub-graph that the
        // block does not own -- the key is inserted, no sample counted
        const bool adj = (AFF || BATCH) && e.w == MARK_ADJ && (AFF || e.z == MARK_ADJ);
        const uint32_t nnf = (AFF && e.w == MARK_ONE_ADJ) ? ADJ_FLAG : 0u;   // sample that proves adjacency
        // affinity entries carry one sample (.w a marker) or, for two
        // neighbouring lanes of one long-range channel with the same key, two
        // samples (.w the second; the push never pairs a marker-valued sample)
        const bool two = BND || (AFF && e.w < MARK_ONE_ADJ);
        const float a = __uint_as_float(e.z);
        const float b = two ? __uint_as_float(e.w) : a;
        const uint32_t n = adj ? 0u : (two ? 2u : 1u);
        const double da = (double)a, db = (double)b;
        const int sa = adj ? -1 : sample_slot<FAST40>(da, scale, offset);
        const int sb = (two && !adj) ? sample_slot<FAST40>(db, scale, offset) : -1;
        const uint32_t mn = f2ord(fminf(a, b)), mx = f2ord(fmaxf(a, b));
        const uint32_t mine = pivot_bits(a);
        if (s < 0) {   // a direct record is its own entry: pivot = its first sample
            const double ea = da - (double)__uint_as_float(mine), eb = db - (double)__uint_as_float(mine);
            emit_direct(R, C, key, n | (adj ? ADJ_FLAG : nnf), sa, sb, adj ? 0.0 : (two ? ea + eb : ea),
                        adj ? 0.0 : (two ? ea * ea + eb * eb : ea * ea), adj ? ORD_POS_INF : mn,
                        adj ? ORD_NEG_INF : mx, adj ? 0u : mine, true);
            return;
        }
        if (adj) {
            atomicOr(&T.w[s][21], ADJ_FLAG);
            return;
        }
        if (ablate & 64) {   // diagnostic: probe only
            if (s == 0x7FFFFFF) atomicAdd(&C->pad[1], 1ull);
            return;
        }
        // fire-and-forget updates: the per-wave sample budget (k_face_scan)
        // keeps every count, hence every u16 histogram slot, below 2^16.  The
        // ones that do not need the pivot go first, so the batch's pivot reads
        // land behind them.
        if (mn < cur.x) atomicMin(&T.w[s][22], mn);
        if (mx > cur.y) atomicMax(&T.w[s][23], mx);
        // word 21 carries only the ADJ flag in the table; the count is the
        // histogram's sum, filled in by the flush
        if (nnf) atomicOr(&T.w[s][21], ADJ_FLAG);
        if (!(ablate & 128)) {   // diagnostic 128: no histogram
            if constexpr (BND) hist_add2(T, s, sa, sb);
            else if (two) hist_add2(T, s, sa, sb);
            else atomicAdd(&T.w[s][sa >> 1], 1u << ((sa & 1) * 16));
        }
        // the entry's pivot: the first sample that claims the empty pivot word
        // (a CAS, so every lane of every wave agrees on it; the word is reset
        // only inside a flush, between two workgroup barriers)
        if (pv == PIV_EMPTY) {
            const uint32_t old = atomicCAS(&T.w[s][24], PIV_EMPTY, mine);
            pv = old == PIV_EMPTY ? mine : old;
        }
        const double dp = (double)__uint_as_float(pv);
        const double ea = da - dp, eb = db - dp;
        atomicAdd(&T.sum[s], two ? ea + eb : ea);
        atomicAdd(&T.sq[s], two ? ea * ea + eb * eb : ea * ea);
    }
}

// lane pairs (2i, 2i+1) / (i, i^2) exchange a value (DPP quad_perm [1,0,3,2] / [2,3,0,1])
__device__ __forceinline__ uint32_t dpp_x1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_x2(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xf, 0xf, false);
}
template <int X>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = X == 1 ? dpp_x1((uint32_t)b) : dpp_x2((uint32_t)b);
    const uint32_t hi = X == 1 ? dpp_x1((uint32_t)(b >> 32)) : dpp_x2((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Boundary-map fold with same-key lanes combined first.  Faces of one site
// arrive in x order, so runs of lanes hold the same key (a cell pair's y / z
// boundary spans several voxels along x); their LDS atomics to one entry
// serialise in the LDS banks.  Within each aligned lane pair, lanes that
// resolved to the same table slot add their shifted sums and fold their min /
// max with one DPP exchange, and only the pair's first lane issues the sum /
// sum-of-squares / min / max atomics (the histogram adds stay per lane: two
// samples rarely share a slot word with their neighbours').  Pairs only: a
// second (quad) stage cost more issue than its saved atomics (scan 2048^3
// 29.92 -> 29.43 ms, 512^3 0.756 -> 0.710, configs[4] 14.63 -> 14.23;
// profiles/r4/e).
#ifndef CTG_PAIR_FOLD
#define CTG_PAIR_FOLD 1
#endif

// (affinity maps: not grouped -- measured slower, configs[3] 12-channel scan
// 45.8 -> 49.9 ms, 3-channel 8.98 -> 9.84 ms: the channel loop's entries
// rarely share a slot within a quad, and the exchanges lengthen every fold)
template <int MODE, bool FAST40, bool BATCH, typename StageT, int NPER>
__device__ __forceinline__ void fold_grouped(Table& T, const StageT (&e)[NPER], const int (&slot)[NPER],
                                             const uint32_t (&pv)[NPER], const uint2 (&mm)[NPER], int lane,
                                             RecordBuf R, Counters* C, double scale, double offset, int ablate) {
    constexpr bool BND = MODE == MODE_BOUNDARY;
    constexpr bool AFF = MODE == MODE_AFFINITY || MODE == MODE_AFF_MIX;
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        const int sl = slot[i];
        if (sl == -1) {   // table full: a direct record, no grouping (rare)
            bool dummy = false;
            fold_stats<MODE, FAST40, BATCH, StageT>(T, e[i], -1, PIV_EMPTY, make_uint2(ORD_POS_INF, ORD_NEG_INF), R, C,
                                                    scale, offset, dummy, 0);
        }
        // adjacency-only entries (fold_stats' rule): the flag, no samples, no group
        const bool adj = (AFF || BATCH) && e[i].w == MARK_ADJ && (AFF || e[i].z == MARK_ADJ);
        if (sl >= 0 && adj) atomicOr(&T.w[sl][21], ADJ_FLAG);
        const bool v = sl >= 0 && !adj;
        if (ablate & 64) {   // diagnostic: probe only (slot and pivot resolved, no statistics)
            if (v && pv[i] == 0x12345u) atomicAdd(&C->pad[1], 1ull);
            continue;
        }
        // affinity entries carry one sample (.w a marker) or two (.w the second)
        const bool two = BND || (AFF && e[i].w < MARK_ONE_ADJ);
        const float a = __uint_as_float(e[i].z);
        const float b = two ? __uint_as_float(e[i].w) : a;
        const double da = (double)a, db = (double)b;
        if (v && !(ablate & 128)) {   // (diagnostic 128: no histogram)
            const int sa = sample_slot<FAST40>(da, scale, offset);
            if (two) hist_add2(T, sl, sa, sample_slot<FAST40>(db, scale, offset));
            else atomicAdd(&T.w[sl][sa >> 1], 1u << ((sa & 1) * 16));
        }
        // the entry's pivot: the first sample that claims the empty word (CAS)
        uint32_t p = pv[i];
        if (v && p == PIV_EMPTY) {
            const uint32_t mine = pivot_bits(a);
            const uint32_t old = atomicCAS(&T.w[sl][24], PIV_EMPTY, mine);
            p = old == PIV_EMPTY ? mine : old;
        }
        const double dp = (double)__uint_as_float(p);
        const double ea = da - dp, eb = two ? db - dp : 0.0;
        double sm = ea + eb, sq = ea * ea + eb * eb;
        uint32_t mn = f2ord(fminf(a, b)), mx = f2ord(fmaxf(a, b));
        // a nearest-neighbour sample proves adjacency (long-range calls with the Bloom filter)
        uint32_t nnf = (AFF && v && e[i].w == MARK_ONE_ADJ) ? 1u : 0u;
        // groups: every lane active here (no divergent branch encloses this);
        // a lane without a slot gets a key no other lane has
        // (diagnostic 1024: no grouping -- every lane its own atomics)
        const uint32_t key = (v && !(ablate & 1024)) ? (uint32_t)sl : 0x80000000u | (uint32_t)lane;
        const bool g1 = dpp_x1(key) == key;
        {
            const double s1 = dpp_f64<1>(sm), q1 = dpp_f64<1>(sq);
            const uint32_t mn1 = dpp_x1(mn), mx1 = dpp_x1(mx), f1 = AFF ? dpp_x1(nnf) : 0u;
            sm = g1 ? sm + s1 : sm;
            sq = g1 ? sq + q1 : sq;
            mn = g1 ? min(mn, mn1) : mn;
            mx = g1 ? max(mx, mx1) : mx;
            nnf = g1 ? nnf | f1 : nnf;
        }
        const bool lead = !(g1 && (lane & 1));
        if (v && lead && !(ablate & 2048)) {   // (diagnostic 2048: no moment / min / max atomics)
            if (!(ablate & 8192)) {            // (diagnostic 8192: no min / max atomics)
                if (mn < mm[i].x) atomicMin(&T.w[sl][22], mn);
                if (mx > mm[i].y) atomicMax(&T.w[sl][23], mx);
            }
            if (AFF && nnf) atomicOr(&T.w[sl][21], ADJ_FLAG);
            if (!(ablate & 4096)) {            // (diagnostic 4096: no f64 sum atomics)
                atomicAdd(&T.sum[sl], sm);
                atomicAdd(&T.sq[sl], sq);
            }
        }
    }
}

// Fold the wave's nb staged entries into the LDS edge table: NPER entries per
// lane (lane, lane+64, ...), their stage reads and home-bucket reads issued
// together so the LDS round trips of the entries overlap.
template <int MODE, bool FAST40, bool BATCH, typename StageT, int NPER>
__device__ __forceinline__ void fold_batch(Table& T, const StageT* __restrict__ stage, int nb, int lane, RecordBuf R,
                                           Counters* C, double scale, double offset, bool& need, int ablate) {
    StageT e[NPER];
    uint32_t h[NPER];
    uint4 b01[NPER], b23[NPER];
#pragma unroll
    for (int i = 0; i < NPER; ++i) e[i] = stage[lane + WAVE * i];   // past nb: stale, ignored
    if (ablate & 32) {   // diagnostic: staging only, no fold
#pragma unroll
        for (int i = 0; i < NPER; ++i)
            if (lane + WAVE * i < nb && e[i].x == 0x12345u && e[i].y == 0x6789u) atomicAdd(&C->pad[1], 1ull);
        return;
    }
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        h[i] = home_bucket(e[i].x, e[i].y);
        b01[i] = *reinterpret_cast<const uint4*>(&T.key[h[i]]);
        b23[i] = *reinterpret_cast<const uint4*>(&T.key[h[i] + 2]);
    }
    int slot[NPER];
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        const bool valid = lane + WAVE * i < nb;
        int s = -1;
        if (valid) {
            const uint64_t key = ((uint64_t)e[i].x << 32) | e[i].y;
            int empty;
            s = bucket_match(b01[i], b23[i], h[i], key, empty);
            if (s < 0) {
                // not in the home bucket: claim its first empty slot with one CAS
                if (empty >= 0) {
                    const uint64_t old = atomicCAS((unsigned long long*)&T.key[h[i] + empty],
                                                   (unsigned long long)EMPTY_KEY, (unsigned long long)key);
                    if (old == EMPTY_KEY) {
                        if (atomicAdd(&T.used, 1u) + 1u > FILL_SOFT) need = true;
                        s = (int)h[i] + empty;
                    } else if (old == key) {
                        s = (int)h[i] + empty;
                    }
                }
                if (s < 0) {
                    s = table_insert(T, h[i], empty, key);
                    need |= s < 0 || (s & INSERT_OVER) != 0;
                    s = s < 0 ? s : (s & (INSERT_OVER - 1));
                }
            }
        }
        slot[i] = valid ? s : -2;   // -2: nothing to fold
    }
    // the entries' pivot words, read together (one LDS round trip for the batch)
    uint32_t pv[NPER];
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        pv[i] = PIV_EMPTY;
        if (MODE != MODE_GRAPH && slot[i] >= 0)
            pv[i] = __hip_atomic_load(&T.w[slot[i]][24], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // ... and their ordered min / max, in the same round trip: the min / max
    // atomics are issued only by lanes whose values extend the entry's range
    // (values only move outward, so a stale read can only ask for an atomic
    // that changes nothing, never skip one that would).  Unconditional, they
    // were ~1/3 of the 2048^3 scan's LDS bank-conflict cycles.
    uint2 mm[NPER];
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        mm[i] = make_uint2(ORD_POS_INF, ORD_NEG_INF);
        if (MODE != MODE_GRAPH && slot[i] >= 0)
            mm[i] = make_uint2(__hip_atomic_load(&T.w[slot[i]][22], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP),
                               __hip_atomic_load(&T.w[slot[i]][23], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    }
#if CTG_PAIR_FOLD
    // grouped atomics: whole-array boundary maps and nearest-neighbour
    // affinity faces (single-sample entries)
    if constexpr ((MODE == MODE_BOUNDARY || MODE == MODE_AFF_NN) && !BATCH) {
        fold_grouped<MODE, FAST40, BATCH, StageT, NPER>(T, e, slot, pv, mm, lane, R, C, scale, offset, ablate);
        return;
    }
#endif
#pragma unroll
    for (int i = 0; i < NPER; ++i)
        if (slot[i] != -2)
            fold_stats<MODE, FAST40, BATCH, StageT>(T, e[i], slot[i], pv[i], mm[i], R, C, scale, offset, need,
                                                    ablate);
}

// diagnostic time stamp (volatile: never merged or moved across other code)
__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// lane pairs (2i, 2i+1) exchange a value (DPP quad_perm [1,0,3,2])
__device__ __forceinline__ uint32_t swap1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xf, 0xf, false);
}

// x-neighbour of every lane: lane i gets lane i+1 (DPP wave_shl:1), lane 63
// gets `edge` (the x-halo value)
__device__ __forceinline__ uint32_t shl1(uint32_t v, uint32_t edge) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x130, 0xf, 0xf, false);
}

#define FLUSH_TABLE table_flush_waves

template <typename LabelT, typename DataT, int MODE, bool FAST40, bool BATCH, int ROWS>
#ifndef CTG_SCAN_MIN_WAVES
#define CTG_SCAN_MIN_WAVES 4   // waves per SIMD the register budget must allow
#endif
__global__ __launch_bounds__(SCAN_THREADS, CTG_SCAN_MIN_WAVES) void k_face_scan(ScanParams P, RecordBuf R, Counters* C) {
    constexpr bool BND = MODE == MODE_BOUNDARY;
    constexpr bool AFF = MODE == MODE_AFFINITY || MODE == MODE_AFF_MIX;
    constexpr bool NN3 = MODE == MODE_AFF_NN;   // nearest-neighbour affinities scanned as faces (P.nn3)
    constexpr bool MIX = MODE == MODE_AFF_MIX;  // ... and the long-range channels in the loop (P.nn_mix)
    constexpr bool NNF = NN3 || MIX;            // faces carry the nearest-neighbour channels' samples
    constexpr uint32_t NN_MARK = MIX ? MARK_ONE_ADJ : MARK_ONE;   // MIX: each such sample proves adjacency
    constexpr bool STATS = MODE != MODE_GRAPH;
    using StageT = typename std::conditional<STATS, uint4, uint2>::type;
    __shared__ Table T;
    constexpr int NP = (ROWS == ROWS_NARROW && ROWS_NARROW != ROWS_WIDE && MODE == MODE_BOUNDARY && !BATCH)
                           ? CTG_NPER_NARROW : NPER;   // staged entries folded per lane
    constexpr int STAGE_CAP = WAVE * NP;               // stage entries per wave
    __shared__ StageT stage_all[WAVES][STAGE_CAP];
    if constexpr (!BATCH) {
        // narrow_rows == 2: both tile widths are launched back to back and the
        // sampled face density picks the one that works (the other exits here)
        if (P.narrow_rows == 2) {
            const bool narrow = (uint64_t)P.density[0] * 100u > (uint64_t)P.density[1] * 14u;
            if (narrow != (ROWS == ROWS_NARROW)) return;
        }
    }
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    StageT* stage = stage_all[wave];
    for (int e = tid; e < TABLE_CAP; e += SCAN_THREADS) entry_reset(T, e);
    if (tid == 0) {
        T.used = 0;
        T.ncompact = 0;
        T.maxv = 0;
        T.flush_req = 0;
        T.live = WAVES;
    }
    __syncthreads();

    // XCD-aware tile order: the hardware deals workgroups round-robin over the
    // 8 XCDs (block b and b+8 share one), so block b takes tile t(b) with each
    // XCD owning one contiguous run of tiles (x fastest, then y, then z).  The
    // workgroups an XCD runs at a time are then x / y neighbours, and the
    // x-halo column and y-halo row one tile reads are the rows its neighbour
    // streams through the same L2, not a second HBM read.
    uint32_t t;
    {
        const uint32_t nwg = gridDim.x, id = blockIdx.x;
        t = id;
        if (P.xcd_remap) {
            const uint32_t q = nwg / 8, rm = nwg % 8, xcd = id % 8, j = id / 8;
            t = xcd < rm ? xcd * (q + 1) + j : rm * (q + 1) + (xcd - rm) * q + j;
        }
    }
    // geometry: the whole array, or (ctg_rag_blocks) the array of the block
    // whose tile range holds t.  Faces with both voxels in the graph box are
    // pushed (sub-graph edges); those owned by the block -- upper voxel in the
    // own box -- carry samples, the others go in as adjacency-only entries.
    constexpr bool batch = BATCH;   // compile-time: the whole-array kernel carries none of this
    int Z, Y, X;
    int obz, oez, oby, oey, obx, oex;
    int gbz, gez, gby, gey, gbx, gex;
    uint32_t ntx, nty, tag = 0;
    int64_t l_off = 0, d_off = 0;
    if constexpr (BATCH) {
        int lo = 0, hi = P.n_blocks;   // tile_prefix[lo] <= t < tile_prefix[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (P.tile_prefix[mid] <= t) lo = mid;
            else hi = mid;
        }
        const BlockGeom& G = P.blocks[lo];
        t -= P.tile_prefix[lo];
        Z = G.shape[0]; Y = G.shape[1]; X = G.shape[2];
        obz = G.own_begin[0]; oez = G.own_end[0]; oby = G.own_begin[1]; oey = G.own_end[1];
        obx = G.own_begin[2]; oex = G.own_end[2];
        gbz = G.graph_begin[0]; gez = G.graph_end[0]; gby = G.graph_begin[1]; gey = G.graph_end[1];
        gbx = G.graph_begin[2]; gex = G.graph_end[2];
        ntx = (uint32_t)G.ntx;
        nty = (uint32_t)G.nty;
        l_off = G.label_offset;
        d_off = G.data_offset;
        tag = P.tag_shift < 32 ? (uint32_t)lo << P.tag_shift : 0u;
    } else {
        Z = (int)P.shape[0]; Y = (int)P.shape[1]; X = (int)P.shape[2];
        obz = (int)P.own_begin[0]; oez = (int)P.own_end[0];
        oby = (int)P.own_begin[1]; oey = (int)P.own_end[1];
        obx = (int)P.own_begin[2]; oex = (int)P.own_end[2];
        gbz = gez = gby = gey = gbx = gex = 0;
        ntx = (uint32_t)P.ntiles[0];
        nty = (uint32_t)P.ntiles[1];
    }
    const int64_t sz = (int64_t)Y * X;
    const int tx = (int)(t % ntx);
    const int ty = (int)((t / ntx) % nty);
    const int tz = (int)(t / (ntx * nty));
    const int x0 = tx * TILE_X;
    const int x = x0 + lane;
    const int yw = ty * (ROWS * WAVES) + wave * ROWS;   // first row of this wave (uniform)
    const int z0 = tz * P.tile_z;
    const int z1 = min(z0 + P.tile_z, Z);
    const LabelT* L = (const LabelT*)P.labels + l_off;
    const DataT* D = (const DataT*)P.data + d_off;
    const double scale = P.scale, offset = P.offset;
#ifdef CTG_DIAG
    const int ablate = P.ablate;   // diagnostic builds only (make variant EXTRA=-DCTG_DIAG)
#else
    constexpr int ablate = 0;      // product kernels carry no diagnostic branches
#endif
    const uint32_t hi_mask = BATCH ? P.label_hi_mask : 0u;
    // lane masks (x is per lane): faces are owned by their upper voxel
    const bool inx = x < X;
    const bool own_x_lo = x >= obx && x < oex;
    const bool lane_xf = inx && x + 1 < X && x + 1 >= obx && x + 1 < oex;   // x face (x, x+1)
    const bool lane_yz = inx && own_x_lo;                                    // y / z faces, samples at p
    // graph membership (batched): both voxels inside the graph box
    const bool g_x_lo = batch && inx && x >= gbx && x < gex;
    const bool glane_xf = g_x_lo && x + 1 < gex;
    const bool glane_yz = g_x_lo;
    // the same lane sets as wave masks (uniform)
    const uint64_t m_xf = __builtin_amdgcn_ballot_w64(lane_xf), m_yz = __builtin_amdgcn_ballot_w64(lane_yz);
    const uint64_t m_gxf = __builtin_amdgcn_ballot_w64(glane_xf), m_gyz = __builtin_amdgcn_ballot_w64(glane_yz);
    // row masks (uniform): bit r for row y = yw + r
    uint32_t row_x = 0, row_y = 0, grow_x = 0, grow_y = 0;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const int y = yw + r;
        if (y < Y && y >= oby && y < oey) row_x |= 1u << r;
        if (y + 1 < Y && y + 1 >= oby && y + 1 < oey) row_y |= 1u << r;
        if (batch && y < Y && y >= gby && y < gey) grow_x |= 1u << r;
        if (batch && y + 1 < gey && y >= gby) grow_y |= 1u << r;
    }
    // adjacency markers of nearest-neighbour faces (affinities); batched
    // blocks always push them (the block's sub-graph is the edge filter)
    const bool adj_marks = AFF && (batch || !P.skip_adj_marks);
    const int xh = x0 + TILE_X;              // x of the lane-63 neighbour

    // plane buffers: rows 0..ROWS-1 of this wave + the y-halo row; the x-halo
    // voxel of row r lives in lane r of XL / XD
    // the prefetched plane keeps full labels: narrowing (and the overflow OR of
    // the high halves) happens when the plane is consumed, never right behind
    // the load, so no s_waitcnt lands in the prefetch
    uint32_t Lc[ROWS + 1];
    LabelT Ln[ROWS + 1];
    float Dc[ROWS + 1], Dn[ROWS + 1];
    // NN3: Dc / Dn hold the x channel; the y channel's rows (sample of face
    // (y, y+1) = row r + 1) and the prefetched plane's z channel (sample of
    // face (z, z+1) = plane z + 1)
    float Dyc[ROWS + 1], Dyn[ROWS + 1], Dzn[ROWS];
    uint32_t XLc = 0;
    LabelT XLn = 0;
    float XDc = 0.f, XDn = 0.f;
    uint32_t ovf = 0;   // OR of the high halves of every 64-bit label loaded

    auto narrow = [&](LabelT l) -> uint32_t {
        if constexpr (sizeof(LabelT) == 8) ovf |= (uint32_t)(l >> 32);
        if constexpr (BATCH) ovf |= (uint32_t)l & hi_mask;   // batched blocks: the tag bits must be free
        return (uint32_t)l;
    };
    // Loads are unconditional: rows past Y and lanes past X read the clamped
    // row / column (valid memory; every face and sample of such a row or lane
    // is masked by row_x / row_y / lane_xf / lane_yz), so no exec-mask
    // branches and no default moves sit between the loads.
    const int xcl = min(x, X - 1);
    const int xhc = min(xh, X - 1);
    const int64_t csz = (int64_t)Z * sz;   // channel stride (NN3)
    auto load_plane = [&](int z, LabelT (&Lb)[ROWS + 1], float (&Db)[ROWS + 1], LabelT& XL, float& XD,
                          float (&Dyb)[ROWS + 1], float (&Dzb)[ROWS], bool with_z) {
        const LabelT* Lz = L + (int64_t)z * sz + (int64_t)yw * X;
        const DataT* Dz = BND ? D + (int64_t)z * sz + (int64_t)yw * X
                              : NN3 ? D + (int64_t)P.nn_ch[2] * csz + (int64_t)z * sz + (int64_t)yw * X : nullptr;
        const int rmax = Y - 1 - yw;   // last valid row offset (uniform; < 0 only for waves past Y)
#pragma unroll
        for (int r = 0; r <= ROWS; ++r) {
            const int rr = min(r, rmax);
            Lb[r] = Lz[(int64_t)rr * X + xcl];
            if constexpr (BND || NN3) Db[r] = load_val<DataT>(Dz, (int64_t)rr * X + xcl);
            else Db[r] = 0.f;
        }
        if constexpr (NN3) {
            const DataT* Ay = D + (int64_t)P.nn_ch[1] * csz + (int64_t)z * sz + (int64_t)yw * X;
            const DataT* Az = D + (int64_t)P.nn_ch[0] * csz + (int64_t)z * sz + (int64_t)yw * X;
#pragma unroll
            for (int r = 1; r <= ROWS; ++r) Dyb[r] = load_val_stream<DataT>(Ay, (int64_t)min(r, rmax) * X + xcl);
            if (with_z) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) Dzb[r] = load_val_stream<DataT>(Az, (int64_t)min(r, rmax) * X + xcl);
            }
        }
        // x-halo: lane r < ROWS holds row r's voxel at x = x0 + 64 (lanes past
        // ROWS repeat row ROWS - 1; only lanes < ROWS are read)
        const int hr = min(min(lane, ROWS - 1), rmax);
        XL = Lz[(int64_t)hr * X + xhc];
        if constexpr (BND || NN3) XD = load_val<DataT>(Dz, (int64_t)hr * X + xhc);
        else XD = 0.f;
    };

    // Flushes on demand: a wave whose fold found the table past FILL_SOFT (or
    // an entry near its count bound) raises T.flush_req; every wave polls it
    // after each fold batch and at each plane end, and all eight then run
    // table_flush together (its barriers are the only workgroup barriers).
    // Waves done with their planes keep polling until the last one is done,
    // so a request never waits for a wave that has left the loop.
    bool need = false;
    int nbuf = 0;         // staged entries (wave-uniform)
    uint32_t wsamp = 0;   // samples this wave folded since the last flush (wave-uniform)
    // diagnostic 256: s_memtime stamps per wave (fold, flush, prefetch wait, total)
    const bool stamps = (ablate & 256) != 0;
    uint64_t t_fold = 0, t_flush = 0, t_wait = 0;
    const uint64_t t_start = stamps ? stamp_now() : 0;
    auto poll = [&]() {
        if (__ballot(need)) {
            if (lane == 0) atomicOr(&T.flush_req, 1u);
            need = false;
        }
        const uint32_t fr = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(&T.flush_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (fr) {
            const uint64_t t0 = stamps ? stamp_now() : 0;
            FLUSH_TABLE<MODE>(T, R, C);
            wsamp = 0;
            if (stamps) t_flush += stamp_now() - t0;
        }
    };
    auto flush_stage = [&]() {
        if (nbuf) {
            if constexpr (STATS) {
                // per-wave sample budget: flush first if this batch would pass it
                const uint32_t add = (BND || AFF) ? 2u * (uint32_t)nbuf : (uint32_t)nbuf;   // AFF: paired entries
                if (wsamp + add > WAVE_SAMPLE_BUDGET) {
                    need = true;
                    poll();
                }
                wsamp += add;
            }
            const uint64_t t0 = stamps ? stamp_now() : 0;
            fold_batch<MODE, FAST40, BATCH, StageT, NP>(T, stage, nbuf, lane, R, C, scale, offset, need, ablate);
            nbuf = 0;
            if (stamps) t_fold += stamp_now() - t0;
            poll();   // after every fold batch (only at plane ends: slower)
        }
    };
    // append the active lanes of one site to the stage
    // (the ballot is taken at the call site, PUSH below: through a bool
    // parameter the compiler rebuilds the lane mask with a cndmask + compare)
    auto push_m = [&](uint64_t m, bool act, uint32_t a, uint32_t b, uint32_t za, uint32_t zb) {
        // no early-out on an empty ballot: at ~15 % face density a site is
        // almost never empty, and k = 0 makes the rest a no-op
        const int k = __popcll(m);
        if (nbuf + k > STAGE_CAP) flush_stage();
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (act) {
            const uint32_t lo_l = BATCH ? (min(a, b) | tag) : min(a, b);
            if constexpr (STATS) stage[nbuf + rank] = make_uint4(lo_l, max(a, b), za, zb);
            else stage[nbuf + rank] = make_uint2(lo_l, max(a, b));
        }
        nbuf += k;
    };
    // PUSH(face compare, uniform 64-bit mask of the lanes whose face counts,
    // per-lane membership, entry...): the ballot of the bare compare is the
    // v_cmp result itself; and-ing the uniform lane mask is one scalar op
#define PUSH(cmp, lanes, member, ...)                                      \
    do {                                                                   \
        const bool c_ = (cmp);                                             \
        push_m(__builtin_amdgcn_ballot_w64(c_) & (lanes), c_ && (member), __VA_ARGS__); \
    } while (0)

    if (z0 < z1) {
        load_plane(z0, Ln, Dc, XLn, XDc, Dyc, Dzn, false);
#pragma unroll
        for (int r = 0; r <= ROWS; ++r) Lc[r] = narrow(Ln[r]);
        XLc = narrow(XLn);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): nothing in flight when the plane loop starts
    for (int z = z0; z < z1; ++z) {
        const bool hz = z + 1 < Z;
        // prefetch of plane z + 1, unconditional (the last plane re-reads
        // itself; its z faces are masked by hz): in flight during the x / y
        // faces, consumed by the z faces (z, z+1) at the end of the plane.
        // (Tried: z faces (z-1, z) against the previous plane, so nothing in
        // a plane waits for the prefetch -- 0.006 ms faster at 512^3, but the
        // changed face order raised records by 23 % at cell 5.)
        load_plane(hz ? z + 1 : z, Ln, Dn, XLn, XDn, Dyn, Dzn, true);
        const bool zlo = z >= obz && z < oez;
        const bool zup = hz && z + 1 >= obz && z + 1 < oez;      // face (z, z+1): upper voxel in the own box
        const bool zg = batch && z >= gbz && z < gez;            // graph box planes (batched)
        const bool gzup = zg && z + 1 < gez;
        // this plane's face sites as scalar bit masks (bit r = row r): owned x /
        // y / z faces and (batched) graph-box faces -- tested with scalar bit
        // tests, not carried as per-lane booleans
        const uint32_t s_xo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(zlo ? row_x : 0u));
        const uint32_t s_yo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(zlo ? row_y : 0u));
        const uint32_t s_zo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(zup ? row_x : 0u));
        const uint32_t s_xg = (uint32_t)__builtin_amdgcn_readfirstlane((int)(zg ? grow_x : 0u));
        const uint32_t s_yg = (uint32_t)__builtin_amdgcn_readfirstlane((int)(zg ? grow_y : 0u));
        const uint32_t s_zg = (uint32_t)__builtin_amdgcn_readfirstlane((int)(gzup ? grow_x : 0u));
        if constexpr (MIX) {
            // the channel loop holds most registers: the nearest-neighbour
            // channels of this plane are loaded here, not prefetched with the
            // labels, and die before the loop (x channel rows + x-halo, y
            // channel rows 1..ROWS); the z channel is loaded before the z faces
            const int rmax = Y - 1 - yw;
            const DataT* Ax = D + (int64_t)P.nn_ch[2] * csz + (int64_t)z * sz + (int64_t)yw * X;
            const DataT* Ay = D + (int64_t)P.nn_ch[1] * csz + (int64_t)z * sz + (int64_t)yw * X;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) Dc[r] = load_val_stream<DataT>(Ax, (int64_t)min(r, rmax) * X + xcl);
            XDc = load_val<DataT>(Ax, (int64_t)min(min(lane, ROWS - 1), rmax) * X + xhc);
#pragma unroll
            for (int r = 1; r <= ROWS; ++r) Dyc[r] = load_val_stream<DataT>(Ay, (int64_t)min(r, rmax) * X + xcl);
        }
        if (ablate & 8) {   // diagnostic: loads only
            uint32_t chk = 0;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) chk ^= Lc[r] ^ (uint32_t)Ln[r] ^ __float_as_uint(Dc[r] + Dn[r]);
            if (chk == 0x9E3779B9u && XLc == 7u) atomicAdd(&C->pad[0], 1ull);
        } else {
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const uint32_t lc = Lc[r];
                // x face (x, x+1); lane 63 takes its neighbour from the x-halo
                const uint32_t lx = shl1(lc, (uint32_t)__builtin_amdgcn_readlane((int)XLc, r));
                // owned faces carry samples; (batched) sub-graph faces the block
                // does not own go in as adjacency-only entries
                const bool xo = (s_xo >> r) & 1u, xg = BATCH && ((s_xg >> r) & 1u);
                if ((xo || xg) && (!AFF || adj_marks || NNF)) {
                    const float dx = (BND || NNF) ? __uint_as_float(shl1(__float_as_uint(Dc[r]),
                                                                         (uint32_t)__builtin_amdgcn_readlane(
                                                                             (int)__float_as_uint(XDc), r)))
                                                  : 0.f;
                    const bool own = xo && lane_xf;
                    if constexpr (NNF) {   // aff[x channel] of the upper voxel x + 1
                        PUSH(lc != lx, m_xf, own, lc, lx, __float_as_uint(dx), NN_MARK);
                    } else {
                        PUSH(lc != lx, (xo ? m_xf : 0ull) | (xg ? m_gxf : 0ull), own || (xg && glane_xf), lc, lx,
                             (own || !BATCH) ? __float_as_uint(Dc[r]) : MARK_ADJ,
                             (AFF || (BATCH && !own)) ? MARK_ADJ : __float_as_uint(dx));
                    }
                }
                // y face (y, y+1)
                const bool yo = (s_yo >> r) & 1u, yg = BATCH && ((s_yg >> r) & 1u);
                if ((yo || yg) && (!AFF || adj_marks || NNF)) {
                    const bool own = yo && lane_yz;
                    if constexpr (NNF) {   // aff[y channel] of the upper voxel, row r + 1
                        PUSH(lc != Lc[r + 1], m_yz, own, lc, Lc[r + 1], __float_as_uint(Dyc[r + 1]), NN_MARK);
                    } else {
                        PUSH(lc != Lc[r + 1], (yo ? m_yz : 0ull) | (yg ? m_gyz : 0ull), own || (yg && glane_yz), lc,
                             Lc[r + 1],
                             (own || !BATCH) ? __float_as_uint(Dc[r]) : MARK_ADJ,
                             (AFF || (BATCH && !own)) ? MARK_ADJ : __float_as_uint(Dc[r + 1]));
                    }
                }
            }
            // affinity samples aff[c, p] for q = p + o_c, p in the owned box:
            // per channel, the gathers / sample loads of all ROWS rows are in
            // flight together, then their Bloom probes (long-range channels)
            if constexpr (AFF) {
                if (zlo && row_x) {
                    const int64_t iz = (int64_t)z * sz + (int64_t)yw * X + x;
                    const int n_loop = MIX ? P.n_loop : P.n_channels;
                    for (int c0 = 0; c0 < n_loop; c0 += AFF_G) {
                        constexpr int K = AFF_G * ROWS;   // (channel, row) sites of the group
                        uint32_t lq[K];
                        float av[K];
                        bool act[K];
#pragma unroll
                        for (int j = 0; j < AFF_G; ++j) {
                            const bool has = c0 + j < n_loop;
                            const int c = MIX ? (has ? P.loop_ch[c0 + j] : 0) : c0 + j;
                            const int qz = has ? z + P.offsets[c][0] : -1, oy = has ? P.offsets[c][1] : 0;
                            const int qx = has ? x + P.offsets[c][2] : -1;
                            const bool okzx = lane_yz && qz >= 0 && qz < Z && qx >= 0 && qx < X;
#pragma unroll
                            for (int r = 0; r < ROWS; ++r) {
                                const int k = j * ROWS + r;
                                const int qy = yw + r + oy;
                                act[k] = (row_x >> r & 1u) && okzx && qy >= 0 && qy < Y;
                                lq[k] = Lc[r];
                                av[k] = 0.f;
                                if (act[k]) {
                                    // the low half only: every label's high half is
                                    // checked where its own tile loads it
                                    lq[k] = load_lo(L, (int64_t)qz * sz + (int64_t)qy * X + qx);
                                    av[k] = load_val_stream<DataT>(D, (int64_t)c * Z * sz + iz + (int64_t)r * X);
                                }
                            }
                        }
#pragma unroll
                        for (int k = 0; k < K; ++k) act[k] = act[k] && lq[k] != Lc[k % ROWS];
                        // long-range channels: only pairs that are RAG edges
                        // (MIX: every loop channel is long-range)
                        const uint32_t glr = MIX ? (1u << AFF_G) - 1u : (P.lr_mask >> c0) & ((1u << AFF_G) - 1u);
                        if (glr && P.bloom != nullptr && !(ablate & 512)) {
                            uint64_t hb[K];
                            unsigned long long wb[K];
                            uint32_t blk[ROWS];   // the own label's block (owner-blocked filter)
#pragma unroll
                            for (int r = 0; r < ROWS; ++r) blk[r] = bloom_block(Lc[r], P.bloom_mask);
#pragma unroll
                            for (int k = 0; k < K; ++k) {
                                hb[k] = bloom_hash(((uint64_t)Lc[k % ROWS] << 32) | lq[k]);
                                wb[k] = (act[k] && (glr >> (k / ROWS) & 1u)) ? P.bloom[bloom_word(blk[k % ROWS], hb[k])]
                                                                             : ~0ull;
                            }
#pragma unroll
                            for (int k = 0; k < K; ++k)
                                act[k] = act[k] && (wb[k] & bloom_bits(hb[k])) == bloom_bits(hb[k]);
                        }
#pragma unroll
                        for (int j = 0; j < AFF_G; ++j) {
                            if (c0 + j >= n_loop) break;
                            const uint32_t mk = (P.bloom != nullptr && !(glr >> j & 1u)) ? MARK_ONE_ADJ : MARK_ONE;
                            // (nearest-neighbour channels unpaired: A/B nn1024 scan 8.6 -> 9.4 ms paired)
                            if (mk == MARK_ONE && P.bloom != nullptr) {
                                // long-range (or unfiltered) channel: lanes 2i, 2i+1 with the
                                // same key fold as one two-sample entry (along x a cell pair
                                // spans runs of lanes), ~halving this channel's fold work
#pragma unroll
                                for (int r = 0; r < ROWS; ++r) {
                                    const int k = j * ROWS + r;
                                    const uint32_t sv = __float_as_uint(av[k]);
                                    const uint32_t nq = swap1(lq[k]), ns = swap1(sv), nact = swap1(act[k] ? 1u : 0u);
                                    const bool pair = act[k] && nact && nq == lq[k] && ns < MARK_ONE_ADJ &&
                                                      sv < MARK_ONE_ADJ;   // Lc[r] is equal on the pair unless a face
                                    const bool lead = (lane & 1) == 0;
                                    const bool same_c = swap1(Lc[r]) == Lc[r];
                                    const bool pr = pair && same_c;
                                    PUSH(act[k] && !(pr && !lead), ~0ull, true, Lc[r], lq[k], sv,
                                         (pr && lead) ? ns : MARK_ONE);
                                }
                            } else {
#pragma unroll
                                for (int r = 0; r < ROWS; ++r)
                                    PUSH(act[j * ROWS + r], ~0ull, true, Lc[r], lq[j * ROWS + r],
                                         __float_as_uint(av[j * ROWS + r]), mk);
                            }
                        }
                    }
                }
            }
            if constexpr (MIX) {   // the z channel of plane z + 1 (upper voxels of the z faces)
                const int rmax = Y - 1 - yw;
                const DataT* Az = D + (int64_t)P.nn_ch[0] * csz + (int64_t)(hz ? z + 1 : z) * sz + (int64_t)yw * X;
#pragma unroll
                for (int r = 0; r < ROWS; ++r) Dzn[r] = load_val_stream<DataT>(Az, (int64_t)min(r, rmax) * X + xcl);
            }
            // z faces (z, z+1): plane z against the prefetched plane
            if (stamps) {   // diagnostic: how long the prefetched plane keeps this wave waiting
                const uint64_t tw = stamp_now();
                __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
                t_wait += stamp_now() - tw;
            }
            if ((s_zo | s_zg) && (!AFF || adj_marks || NNF)) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    const bool zo = (s_zo >> r) & 1u, zgr = BATCH && ((s_zg >> r) & 1u);
                    if (zo || zgr) {
                        const bool own = zo && lane_yz;
                        const uint32_t ln = (uint32_t)Ln[r];
                        if constexpr (NNF) {   // aff[z channel] of the upper voxel, plane z + 1
                            PUSH(Lc[r] != ln, m_yz, own, Lc[r], ln, __float_as_uint(Dzn[r]), NN_MARK);
                        } else {
                            PUSH(Lc[r] != ln, (zo ? m_yz : 0ull) | (zgr ? m_gyz : 0ull), own || (zgr && glane_yz),
                                 Lc[r], ln, (own || !BATCH) ? __float_as_uint(Dc[r]) : MARK_ADJ,
                                 (AFF || (BATCH && !own)) ? MARK_ADJ : __float_as_uint(Dn[r]));
                        }
                    }
                }
            }
        }
        // staged entries stay staged across planes (raw faces are valid for
        // whatever table they are folded into later)
        poll();
        // the prefetched plane has landed by now (it had the whole plane's work
        // to do so): wait for it here, before the next plane's loads are
        // issued -- a wait placed after them (where the compiler would put it
        // on first use) would drain the new prefetch too
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
#pragma unroll
        for (int r = 0; r <= ROWS; ++r) {
            Lc[r] = narrow(Ln[r]);
            Dc[r] = Dn[r];
            if constexpr (NN3) {
                if (r >= 1) Dyc[r] = Dyn[r];   // (row 0 of the y channel is never a sample)
            }
        }
        XLc = narrow(XLn);
        XDc = XDn;
    }
#undef PUSH
    if (__ballot(ovf != 0) && lane == 0) atomicAdd(&C->label_overflow, 1ull);
    flush_stage();
    poll();
    if (lane == 0) atomicSub(&T.live, 1u);
    while (true) {
        const uint32_t fr = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(&T.flush_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (fr) {
            FLUSH_TABLE<MODE>(T, R, C);
            continue;
        }
        const uint32_t lv = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(&T.live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (lv == 0) break;
        __builtin_amdgcn_s_sleep(2);
    }
    FLUSH_TABLE<MODE>(T, R, C);
    if (tid == 0 && T.maxv) atomicMax(&C->max_v, T.maxv);   // after the final flush's barrier
    if (stamps && lane == 0) {
        atomicAdd(&C->pad[2], (unsigned long long)(stamp_now() - t_start));
        atomicAdd(&C->pad[3], (unsigned long long)t_fold);
        atomicAdd(&C->pad[4], (unsigned long long)t_flush);
        atomicAdd(&C->pad[5], (unsigned long long)t_wait);
    }
}

// ---------------------------------------------------------------------------
// launcher
// ---------------------------------------------------------------------------
template <typename LabelT, typename DataT, int MODE, int NR>
static hipError_t launch_scan_r(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    ScanParams Q = P;
    int64_t nwg = P.batch_tiles;
    if (!P.blocks) {
        if (NR == ROWS_NARROW && ROWS_NARROW != ROWS_WIDE && P.tile_z_narrow > 0) Q.tile_z = P.tile_z_narrow;
        Q.ntiles[0] = (P.shape[2] + TILE_X - 1) / TILE_X;
        Q.ntiles[1] = (P.shape[1] + NR * WAVES - 1) / (NR * WAVES);
        Q.ntiles[2] = (P.shape[0] + Q.tile_z - 1) / Q.tile_z;
        nwg = Q.ntiles[0] * Q.ntiles[1] * Q.ntiles[2];
    }
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    dim3 grid((unsigned)nwg);
    constexpr unsigned pad = 0;   // dynamic LDS
    if (P.blocks) {
        if (P.fast40)
            hipLaunchKernelGGL((k_face_scan<LabelT, DataT, MODE, true, true, NR>), grid, dim3(SCAN_THREADS), pad, s, Q,
                               R, C);
        else
            hipLaunchKernelGGL((k_face_scan<LabelT, DataT, MODE, false, true, NR>), grid, dim3(SCAN_THREADS), pad, s,
                               Q, R, C);
    } else if (P.fast40) {
        hipLaunchKernelGGL((k_face_scan<LabelT, DataT, MODE, true, false, NR>), grid, dim3(SCAN_THREADS), pad, s, Q,
                           R, C);
    } else {
        hipLaunchKernelGGL((k_face_scan<LabelT, DataT, MODE, false, false, NR>), grid, dim3(SCAN_THREADS), pad, s, Q,
                           R, C);
    }
    return hipGetLastError();
}

// the narrow-tile kernel exists for whole-array boundary maps (the
// fragmentation-bound configs[4] path); every other mode uses the wide one
template <typename LabelT, typename DataT, int MODE>
static hipError_t launch_scan_t(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    if constexpr (MODE == MODE_BOUNDARY) {
        if (P.narrow_rows == 2 && !P.blocks) {
            const hipError_t e = launch_scan_r<LabelT, DataT, MODE, ROWS_WIDE>(P, R, C, s);
            return e != hipSuccess ? e : launch_scan_r<LabelT, DataT, MODE, ROWS_NARROW>(P, R, C, s);
        }
        if (P.narrow_rows == 1 && !P.blocks) return launch_scan_r<LabelT, DataT, MODE, ROWS_NARROW>(P, R, C, s);
    }
    // (batched blocks keep the wide tile: their tile counts come from scan_tile_rows())
    if constexpr (MODE == MODE_AFFINITY || MODE == MODE_AFF_MIX)
        if (!P.blocks) return launch_scan_r<LabelT, DataT, MODE, ROWS_AFF>(P, R, C, s);
    return launch_scan_r<LabelT, DataT, MODE, ROWS_WIDE>(P, R, C, s);
}

template <typename LabelT>
static hipError_t launch_scan_l(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    if (P.data_kind == CTG_DATA_NONE || P.data == nullptr)
        return launch_scan_t<LabelT, float, MODE_GRAPH>(P, R, C, s);
    const bool aff = P.n_channels > 0;
    const bool nn3 = aff && P.nn3 && !P.blocks;
    const bool mix = aff && P.nn_mix && !P.blocks;
    if (P.data_kind == CTG_DATA_U8)
        return nn3 ? launch_scan_t<LabelT, uint8_t, MODE_AFF_NN>(P, R, C, s)
               : mix ? launch_scan_t<LabelT, uint8_t, MODE_AFF_MIX>(P, R, C, s)
               : aff ? launch_scan_t<LabelT, uint8_t, MODE_AFFINITY>(P, R, C, s)
                     : launch_scan_t<LabelT, uint8_t, MODE_BOUNDARY>(P, R, C, s);
    return nn3 ? launch_scan_t<LabelT, float, MODE_AFF_NN>(P, R, C, s)
           : mix ? launch_scan_t<LabelT, float, MODE_AFF_MIX>(P, R, C, s)
           : aff ? launch_scan_t<LabelT, float, MODE_AFFINITY>(P, R, C, s)
                 : launch_scan_t<LabelT, float, MODE_BOUNDARY>(P, R, C, s);
}

hipError_t launch_face_scan(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    if (P.label_bits == 32) return launch_scan_l<uint32_t>(P, R, C, s);
    return launch_scan_l<uint64_t>(P, R, C, s);
}

// Fragmentation probe: label changes along x on a sample of rows (a boundary
// face density estimate) -- the host picks the narrow-tile scan above a
// threshold.  One workgroup per sampled row; counts in out[0] (changes) and
// out[1] (pairs).
template <typename LabelT>
__global__ __launch_bounds__(256) void k_density(const LabelT* __restrict__ L, int64_t Z, int64_t Y, int64_t X,
                                                 uint32_t* __restrict__ out) {
    const int64_t i = blockIdx.x;
    const int64_t z = (i * 7919) % Z, y = (i * 104729 + 17) % Y;
    const LabelT* row = L + (z * Y + y) * X;
    uint32_t ch = 0, pairs = 0;
    for (int64_t x = threadIdx.x; x + 1 < X; x += 256) {
        ch += row[x] != row[x + 1];
        ++pairs;
    }
    for (int o = 32; o > 0; o >>= 1) {
        ch += __shfl_xor(ch, o, 64);
        pairs += __shfl_xor(pairs, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], ch);
        atomicAdd(&out[1], pairs);
    }
}

hipError_t launch_density(const void* L, int label_bits, const int64_t* shape, int n_rows, uint32_t* out,
                          hipStream_t s) {
    if (label_bits == 32)
        hipLaunchKernelGGL(k_density<uint32_t>, dim3(n_rows), dim3(256), 0, s, (const uint32_t*)L, shape[0], shape[1],
                           shape[2], out);
    else
        hipLaunchKernelGGL(k_density<uint64_t>, dim3(n_rows), dim3(256), 0, s, (const uint64_t*)L, shape[0], shape[1],
                           shape[2], out);
    return hipGetLastError();
}

int scan_tile_rows() { return WG_ROWS; }
int scan_tile_rows_narrow() { return ROWS_NARROW * WAVES; }

// ---------------------------------------------------------------------------
// unique labels of a box (per-block ``nodes``): LDS hash set per tile
// ---------------------------------------------------------------------------
constexpr int UNIQ_THREADS = 256;  // 4 waves: the unique-label scan walks 4 planes per step
constexpr int USET_CAP = 2048;

__global__ __launch_bounds__(UNIQ_THREADS) void k_unique_tiles(const uint64_t* L, int64_t Y, int64_t X,
                                                                int64_t bz, int64_t by, int64_t bx,
                                                                int64_t ez, int64_t ey, int64_t ex,
                                                                uint64_t* out, unsigned long long* count,
                                                                int64_t cap) {
    __shared__ uint64_t set[USET_CAP];
    __shared__ uint32_t used;
    __shared__ unsigned long long base;
    __shared__ uint32_t wpos;
    const int tid = threadIdx.x;
    for (int e = tid; e < USET_CAP; e += UNIQ_THREADS) set[e] = EMPTY_KEY;
    if (tid == 0) used = 0;
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t x = bx + (int64_t)blockIdx.x * 64 + lane;
    const int64_t y0 = by + (int64_t)blockIdx.y * TILE_Y;
    const int64_t z0 = bz + (int64_t)blockIdx.z * 16;
    for (int zs = 0; zs < 16; zs += 4) {
        const int64_t z = z0 + zs + wave;
        if (z < ez) {
            for (int dy = 0; dy < TILE_Y; ++dy) {
                const int64_t y = y0 + dy;
                if (y >= ey) break;
                uint64_t l = (x < ex) ? L[(z * Y + y) * X + x] : EMPTY_KEY;
                uint32_t lo = (uint32_t)l, hi = (uint32_t)(l >> 32);
                uint32_t plo = __shfl_up(lo, 1, 64), phi = __shfl_up(hi, 1, 64);
                uint64_t prev = ((uint64_t)phi << 32) | plo;
                const bool head = (x < ex) && (lane == 0 || prev != l);
                if (head) {
                    uint32_t h = hash_key(l) & (USET_CAP - 1);
                    for (int p = 0; p < USET_CAP; ++p) {
                        uint64_t cur = set[h];
                        if (cur == l) break;
                        if (cur == EMPTY_KEY) {
                            uint64_t old = atomicCAS((unsigned long long*)&set[h], (unsigned long long)EMPTY_KEY,
                                                     (unsigned long long)l);
                            if (old == EMPTY_KEY) {
                                atomicAdd(&used, 1u);
                                break;
                            }
                            if (old == l) break;
                        }
                        h = (h + 1) & (USET_CAP - 1);
                    }
                }
            }
        }
        __syncthreads();
        if (used > USET_CAP / 2 || zs + 4 >= 16) {
            if (tid == 0) {
                base = atomicAdd(count, (unsigned long long)used);
                wpos = 0;
            }
            __syncthreads();
            // compaction order is irrelevant (sorted afterwards)
            for (int e = tid; e < USET_CAP; e += UNIQ_THREADS) {
                uint64_t k = set[e];
                if (k != EMPTY_KEY) {
                    uint32_t r = atomicAdd(&wpos, 1u);
                    if (base + r < (unsigned long long)cap) out[base + r] = k;
                    set[e] = EMPTY_KEY;
                }
            }
            __syncthreads();
            if (tid == 0) used = 0;
            __syncthreads();
        }
    }
}

// Per-block node lists of a batched call (ctg_rag_blocks): the unique labels
// of every block's own box (its inner block, test_graph.py:53-60), one LDS set
// per 64 x 8 x 16 tile, emitted as (block << 32) | label candidates; sorting
// and de-duplicating them leaves each block's sorted nodes contiguous.
template <typename LabelT>
__global__ __launch_bounds__(UNIQ_THREADS) void k_unique_blocks(const LabelT* __restrict__ L,
                                                                 const BlockGeom* __restrict__ blocks,
                                                                 const uint32_t* __restrict__ tile_prefix,
                                                                 int n_blocks, uint64_t* __restrict__ out,
                                                                 unsigned long long* count, int64_t cap) {
    __shared__ uint64_t set[USET_CAP];
    __shared__ uint32_t used;
    __shared__ unsigned long long base;
    __shared__ uint32_t wpos;
    const int tid = threadIdx.x;
    for (int e = tid; e < USET_CAP; e += UNIQ_THREADS) set[e] = EMPTY_KEY;
    if (tid == 0) used = 0;
    uint32_t t = blockIdx.x;
    int lo = 0, hi = n_blocks;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tile_prefix[mid] <= t) lo = mid;
        else hi = mid;
    }
    const BlockGeom& G = blocks[lo];
    t -= tile_prefix[lo];
    const int bz = G.own_begin[0], by = G.own_begin[1], bx = G.own_begin[2];
    const int ez = G.own_end[0], ey = G.own_end[1], ex = G.own_end[2];
    const uint32_t ntx = (uint32_t)(ex - bx + 63) / 64, nty = (uint32_t)(ey - by + TILE_Y - 1) / TILE_Y;
    const int64_t Y = G.shape[1], X = G.shape[2];
    const LabelT* Lb = L + G.label_offset;
    const uint64_t tag = (uint64_t)lo << 32;
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t x = bx + (int64_t)(t % ntx) * 64 + lane;
    const int64_t y0 = by + (int64_t)((t / ntx) % nty) * TILE_Y;
    const int64_t z0 = bz + (int64_t)(t / (ntx * nty)) * 16;
    for (int zs = 0; zs < 16; zs += 4) {
        const int64_t z = z0 + zs + wave;
        if (z < ez) {
            for (int dy = 0; dy < TILE_Y; ++dy) {
                const int64_t y = y0 + dy;
                if (y >= ey) break;
                const uint64_t l = (x < ex) ? (tag | (uint32_t)Lb[(z * Y + y) * X + x]) : EMPTY_KEY;
                uint32_t plo = __shfl_up((uint32_t)l, 1, 64), phi = __shfl_up((uint32_t)(l >> 32), 1, 64);
                const uint64_t prev = ((uint64_t)phi << 32) | plo;
                const bool head = (x < ex) && (lane == 0 || prev != l);
                if (head) {
                    uint32_t h = hash_key(l) & (USET_CAP - 1);
                    for (int p = 0; p < USET_CAP; ++p) {
                        const uint64_t cur = set[h];
                        if (cur == l) break;
                        if (cur == EMPTY_KEY) {
                            const uint64_t old = atomicCAS((unsigned long long*)&set[h],
                                                           (unsigned long long)EMPTY_KEY, (unsigned long long)l);
                            if (old == EMPTY_KEY) {
                                atomicAdd(&used, 1u);
                                break;
                            }
                            if (old == l) break;
                        }
                        h = (h + 1) & (USET_CAP - 1);
                    }
                }
            }
        }
        __syncthreads();
        if (used > USET_CAP / 2 || zs + 4 >= 16) {
            if (tid == 0) {
                base = atomicAdd(count, (unsigned long long)used);
                wpos = 0;
            }
            __syncthreads();
            for (int e = tid; e < USET_CAP; e += UNIQ_THREADS) {
                const uint64_t k = set[e];
                if (k != EMPTY_KEY) {
                    const uint32_t r = atomicAdd(&wpos, 1u);
                    if (base + r < (unsigned long long)cap) out[base + r] = k;
                    set[e] = EMPTY_KEY;
                }
            }
            __syncthreads();
            if (tid == 0) used = 0;
            __syncthreads();
        }
    }
}

hipError_t launch_unique_blocks(const void* L, int label_bits, const BlockGeom* blocks, const uint32_t* tile_prefix,
                                int n_blocks, int64_t n_tiles, uint64_t* out, unsigned long long* count, int64_t cap,
                                hipStream_t s) {
    if (n_tiles <= 0) return hipSuccess;
    if (label_bits == 32)
        hipLaunchKernelGGL(k_unique_blocks<uint32_t>, dim3((unsigned)n_tiles), dim3(UNIQ_THREADS), 0, s,
                           (const uint32_t*)L, blocks, tile_prefix, n_blocks, out, count, cap);
    else
        hipLaunchKernelGGL(k_unique_blocks<uint64_t>, dim3((unsigned)n_tiles), dim3(UNIQ_THREADS), 0, s,
                           (const uint64_t*)L, blocks, tile_prefix, n_blocks, out, count, cap);
    return hipGetLastError();
}

int unique_tile_y() { return TILE_Y; }

hipError_t launch_unique_tiles(const uint64_t* L, const int64_t* shape, const int64_t* b, const int64_t* e,
                               uint64_t* out, unsigned long long* count, int64_t cap, hipStream_t s) {
    dim3 grid((unsigned)((e[2] - b[2] + 63) / 64), (unsigned)((e[1] - b[1] + TILE_Y - 1) / TILE_Y),
              (unsigned)((e[0] - b[0] + 15) / 16));
    hipLaunchKernelGGL(k_unique_tiles, grid, dim3(UNIQ_THREADS), 0, s, L, shape[1], shape[2], b[0], b[1], b[2],
                       e[0], e[1], e[2], out, count, cap);
    return hipGetLastError();
}

}  // namespace ctg
