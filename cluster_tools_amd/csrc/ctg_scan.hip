// Face scan: the O(V) hot loop of the RAG + edge-feature path (gfx950).
//
// One workgroup (8 waves) owns a tile of 64 (x) x 32 (y) x tile_z (z) voxels.
// Each wave holds 4 rows (+ the y-halo row) of one z-plane in registers
// (lane = x) and walks z with the next plane's loads in flight while it works
// on the current one, so every label/value is read from HBM once.  Every
// boundary face (p, p+e_a) with differing labels is folded into an LDS
// open-addressing edge table keyed by (u<<32)|v that holds, per edge, the
// sample count, f64 sum and sum of squares, order-preserving min/max and the
// 42-slot vigra histogram (u16 slots packed in u32 words).  The table is
// flushed to HBM as one record per (tile, edge) when it is half full, when a
// u16 slot could wrap within the next plane, and at the end of the tile.
//
// Per-face work is kept off the LDS critical path:
//  * per-lane caches hold the last key of each face axis (x and z faces repeat
//    along y, y faces along z), with x/z statistics pending in registers;
//  * the keys of a row batch are resolved together: every cache miss reads its
//    2-slot home bucket with one 16-byte LDS load, all issued back to back, and
//    only keys missing from their home bucket walk the probe/insert loop.
// Replaces the per-face std::set / findEdge loop of nifty.distributed (called
// at graph/initial_sub_graphs.py:124-129 and features/block_edge_features.py:127-145).
#include "ctg_internal.h"

namespace ctg {

enum { MODE_GRAPH = 0, MODE_BOUNDARY = 1, MODE_AFFINITY = 2 };

struct __align__(16) Table {
    uint64_t key[TABLE_CAP];
    double sum[TABLE_CAP];
    double sq[TABLE_CAP];
    // hist words 0..20, 21 cnt|ADJ, 22 min, 23 max; odd row stride (25 words)
    // so atomics to different entries spread over the 32 LDS banks
    uint32_t w[TABLE_CAP][NREC_WORDS + 1];
    uint16_t compact[TABLE_CAP];
    uint32_t wave_cnt[SCAN_THREADS / WAVE];
    uint32_t used;
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
}

// home bucket of a key: two slots (even, odd) read by one ds_read_b128
// home bucket of a key: four slots, read by two ds_read_b128
__device__ __forceinline__ uint32_t home_bucket(uint64_t key) { return hash_key(key) & (TABLE_CAP - 4); }

// linear probing from the home bucket; returns the slot or -1 when full
__device__ __forceinline__ int table_insert(Table& T, uint64_t key) {
    uint32_t h = home_bucket(key);
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
        uint64_t cur = __hip_atomic_load(&T.key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == key) return (int)h;
        if (cur == EMPTY_KEY) {
            uint64_t old = atomicCAS((unsigned long long*)&T.key[h], (unsigned long long)EMPTY_KEY,
                                     (unsigned long long)key);
            if (old == EMPTY_KEY) {
                atomicAdd(&T.used, 1u);
                return (int)h;
            }
            if (old == key) return (int)h;
        }
        h = (h + 1) & (TABLE_CAP - 1);
    }
    return -1;
}

template <int MODE>
__device__ void table_flush(Table& T, RecordBuf R, Counters* C) {
    static_assert(TABLE_CAP == SCAN_THREADS, "one table entry per thread in the flush");
    __syncthreads();
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1), wv = tid >> 6;
    // ballot compaction: entry tid goes to wave offset + rank among its wave
    const uint64_t k = T.key[tid];
    const bool live = k != EMPTY_KEY;
    const uint64_t m = __ballot(live);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    uint64_t mv = live ? (k & 0xFFFFFFFFull) : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t other = ((uint64_t)__shfl_xor((uint32_t)(mv >> 32), o, WAVE) << 32) |
                               __shfl_xor((uint32_t)mv, o, WAVE);
        mv = max(mv, other);
    }
    if (lane == 0) {
        T.wave_cnt[wv] = (uint32_t)__popcll(m);
        if (mv) atomicMax(&T.maxv, (unsigned long long)mv);
    }
    __syncthreads();
    uint32_t off = 0, n = 0;
#pragma unroll
    for (int w = 0; w < SCAN_THREADS / WAVE; ++w) {
        off += w < wv ? T.wave_cnt[w] : 0u;
        n += T.wave_cnt[w];
    }
    if (live) T.compact[off + rank] = (uint16_t)tid;
    if (tid == 0) T.ncompact = n;
    __syncthreads();
    if (tid == 0 && n) {
        T.base = atomicAdd(&C->n_records, (unsigned long long)n);
        atomicMax(&C->max_v, T.maxv);
    }
    __syncthreads();
    if (n) {
        const unsigned long long base = T.base;
        for (uint32_t r = tid; r < n; r += SCAN_THREADS) {
            const int e = T.compact[r];
            if (base + r < (unsigned long long)R.cap) {
                R.key[base + r] = T.key[e];
                if (MODE != MODE_GRAPH) R.sums[base + r] = make_double2(T.sum[e], T.sq[e]);
            }
        }
        if (MODE != MODE_GRAPH) {
            // coalesced copy of the 24-word rows
            for (uint32_t f = tid; f < n * NREC_WORDS; f += SCAN_THREADS) {
                const uint32_t r = f / NREC_WORDS, j = f - r * NREC_WORDS;
                if (base + r < (unsigned long long)R.cap)
                    R.hist[(base + r) * NREC_WORDS + j] = T.w[T.compact[r]][j];
            }
        }
        __syncthreads();
        for (uint32_t r = tid; r < n; r += SCAN_THREADS) entry_reset(T, T.compact[r]);
    }
    __syncthreads();
    if (tid == 0) {
        T.used = 0;
        T.ncompact = 0;
        T.maxv = 0;
    }
    __syncthreads();
}

// a face or affinity sample that found no room in the LDS table goes straight
// to HBM as a one-sample (or two-sample) record
__device__ __noinline__ void emit_direct(RecordBuf R, Counters* C, uint64_t key, int nsamp, float a, float b,
                                         double scale, double offset, uint32_t flag, bool with_stats) {
    unsigned long long i = atomicAdd(&C->n_records, 1ull);
    atomicAdd(&C->n_direct, 1ull);
    atomicMax(&C->max_v, (unsigned long long)(key & 0xFFFFFFFFull));
    if (i >= (unsigned long long)R.cap) return;
    R.key[i] = key;
    if (!with_stats) return;
    uint32_t w21 = 0;
    uint32_t mn = ORD_POS_INF, mx = ORD_NEG_INF;
    double s = 0.0, q = 0.0;
    int sa = -1, sb = -1;
    if (nsamp >= 1) {
        sa = hist_slot((double)a, scale, offset);
        s += (double)a;
        q += (double)a * (double)a;
        mn = min(mn, f2ord(a));
        mx = max(mx, f2ord(a));
    }
    if (nsamp >= 2) {
        sb = hist_slot((double)b, scale, offset);
        s += (double)b;
        q += (double)b * (double)b;
        mn = min(mn, f2ord(b));
        mx = max(mx, f2ord(b));
    }
    w21 = (uint32_t)nsamp | flag;
    R.sums[i] = make_double2(s, q);
    for (int j = 0; j < HWORDS; ++j) {
        uint32_t v = 0;
        if (sa >= 0 && (sa >> 1) == j) v += 1u << ((sa & 1) * 16);
        if (sb >= 0 && (sb >> 1) == j) v += 1u << ((sb & 1) * 16);
        R.hist[i * NREC_WORDS + j] = v;
    }
    R.hist[i * NREC_WORDS + 21] = w21;
    R.hist[i * NREC_WORDS + 22] = mn;
    R.hist[i * NREC_WORDS + 23] = mx;
}

template <typename DataT>
__device__ __forceinline__ float load_val(const DataT* p, int64_t i) {
    if constexpr (sizeof(DataT) == 1) {
        return __fdiv_rn((float)p[i], 255.0f);
    } else {
        return p[i];
    }
}

template <typename LabelT>
__device__ __forceinline__ LabelT shfl_lane(LabelT v, int src) {
    if constexpr (sizeof(LabelT) == 8) {
        uint32_t lo = __shfl((uint32_t)v, src, WAVE), hi = __shfl((uint32_t)(v >> 32), src, WAVE);
        return ((LabelT)hi << 32) | lo;
    } else {
        return (LabelT)__shfl((uint32_t)v, src, WAVE);
    }
}

template <typename LabelT>
__device__ __forceinline__ LabelT shfl_down1(LabelT v) {
    if constexpr (sizeof(LabelT) == 8) {
        uint32_t lo = __shfl_down((uint32_t)v, 1, WAVE), hi = __shfl_down((uint32_t)(v >> 32), 1, WAVE);
        return ((LabelT)hi << 32) | lo;
    } else {
        return (LabelT)__shfl_down((uint32_t)v, 1, WAVE);
    }
}

// vigra binning of one sample.  fast40: range [0,1) with 40 bins, where
// m = 40*x is computed exactly as p + e (two-product with an f32 FMA): the
// slot equals the double-precision rule of hist_slot for every float x >= 0.
__device__ __forceinline__ int sample_slot(float x, bool fast40, double scale, double offset) {
    if (fast40 && x >= 0.f) {
        const float p = x * 40.0f;
        const float e = __builtin_fmaf(x, 40.0f, -p);
        // m == 40 -> bin 39 (slot 40); m in (39,40) -> slot 40; m > 40 -> right outlier
        if (p >= 40.0f) return (p == 40.0f && e <= 0.0f) ? NBINS : NBINS + 1;
        float fl = floorf(p);
        if (fl == p && e < 0.0f) fl -= 1.0f;
        return (int)fl + 1;
    }
    return hist_slot((double)x, scale, offset);
}

__device__ __forceinline__ void hist_add(Table& T, int s, int k) {
    atomicAdd(&T.w[s][k >> 1], 1u << ((k & 1) * 16));
}

constexpr int ROWS = 4;                                   // y rows per wave, held in registers
constexpr int WAVES = SCAN_THREADS / WAVE;                // 8
constexpr int WG_ROWS = ROWS * WAVES;                     // 32 = tile y extent
constexpr uint32_t MARK_ADJ = 0xFFFFFFFFu;                // stage entry: nearest-neighbour face, no sample
constexpr uint32_t MARK_ONE = 0xFFFFFFFEu;                // stage entry: one affinity sample in .z

// canonical (min, max) key, branch free; with 64-bit labels a label >= 2^32
// deactivates the face and raises the lane's overflow flag
template <typename LabelT>
__device__ __forceinline__ bool make_key(bool act, LabelT a, LabelT b, uint64_t& key, bool& ovf) {
    const LabelT u = a < b ? a : b;
    const LabelT v = a < b ? b : a;
    bool bad = false;
    if constexpr (sizeof(LabelT) == 8) bad = (v >> 32) != 0;
    ovf = ovf | (act & bad);
    key = ((uint64_t)u << 32) | (uint64_t)(uint32_t)v;
    return act & !bad;
}

// Compacted face stream.  Each site (one row of one face axis) contributes
// only its active lanes: they append (key, sample a, sample b) to the wave's
// LDS stage at ballot/mbcnt positions; once the next site would overflow the
// 64 entries, the wave takes the staged faces one per lane and folds them into
// the edge table (home-bucket probe, statistics atomics, histogram).  Every
// lane of a batch carries a face, instead of ~1 in 10 lanes of a site.
#ifdef CTG_FOLD_NOINLINE
#define CTG_FOLD_INLINE __noinline__
#else
#define CTG_FOLD_INLINE __forceinline__
#endif
template <int MODE>
__device__ CTG_FOLD_INLINE void fold_batch(Table& T, const uint4* __restrict__ stage, int nb, int lane, RecordBuf R,
                                           Counters* C, bool fast40, double scale, double offset, int ablate) {
    constexpr bool BND = MODE == MODE_BOUNDARY;
    constexpr bool AFF = MODE == MODE_AFFINITY;
    constexpr bool STATS = MODE != MODE_GRAPH;
    if (lane >= nb) return;
    const uint4 e = stage[lane];
    if (ablate & 32) {   // diagnostic: no fold
        if (e.x == 0x12345u && e.y == 0x6789u) atomicAdd(&C->pad[1], 1ull);
        return;
    }
    const uint64_t key = ((uint64_t)e.y << 32) | e.x;
    const uint32_t h = home_bucket(key);
    const uint4 b01 = *reinterpret_cast<const uint4*>(&T.key[h]);
    const uint4 b23 = *reinterpret_cast<const uint4*>(&T.key[h + 2]);
    const uint64_t kk[4] = {((uint64_t)b01.y << 32) | b01.x, ((uint64_t)b01.w << 32) | b01.z,
                            ((uint64_t)b23.y << 32) | b23.x, ((uint64_t)b23.w << 32) | b23.z};
    int s = -1, empty = -1;
#pragma unroll
    for (int j = 3; j >= 0; --j) {
        s = kk[j] == key ? (int)h + j : s;
        empty = kk[j] == EMPTY_KEY ? j : empty;
    }
    if (s < 0) {
        // not in the home bucket: claim its first empty slot with one CAS
        // (the probe order is linear from the bucket start, so the key cannot
        // sit beyond an empty slot); a lost race or a full bucket probes on
        bool done = false;
        if (empty >= 0) {
            const uint64_t old = atomicCAS((unsigned long long*)&T.key[h + empty], (unsigned long long)EMPTY_KEY,
                                           (unsigned long long)key);
            if (old == EMPTY_KEY) atomicAdd(&T.used, 1u);
            if (old == EMPTY_KEY || old == key) {
                s = (int)h + empty;
                done = true;
            }
        }
        if (!done) s = table_insert(T, key);
    }
    const float a = __uint_as_float(e.z), b = __uint_as_float(e.w);
    if (s < 0) {
        if constexpr (BND) emit_direct(R, C, key, 2, a, b, scale, offset, 0u, true);
        if constexpr (AFF) {
            if (e.w == MARK_ADJ) emit_direct(R, C, key, 0, 0.f, 0.f, scale, offset, ADJ_FLAG, true);
            else emit_direct(R, C, key, 1, a, 0.f, scale, offset, 0u, true);
        }
        if constexpr (!STATS) emit_direct(R, C, key, 0, 0.f, 0.f, scale, offset, 0u, false);
        return;
    }
    if (ablate & 64) {   // diagnostic: probe only
        if (s == 0x7FFFFFFF) atomicAdd(&C->pad[1], 1ull);
        return;
    }
    if constexpr (BND) {
        atomicAdd(&T.w[s][21], 2u);
        atomicAdd(&T.sum[s], (double)a + (double)b);
        atomicAdd(&T.sq[s], (double)a * (double)a + (double)b * (double)b);
        atomicMin(&T.w[s][22], f2ord(fminf(a, b)));
        atomicMax(&T.w[s][23], f2ord(fmaxf(a, b)));
        if (ablate & 128) return;   // diagnostic: no histogram
        hist_add(T, s, sample_slot(a, fast40, scale, offset));
        hist_add(T, s, sample_slot(b, fast40, scale, offset));
    }
    if constexpr (AFF) {
        if (e.w == MARK_ADJ) {
            atomicOr(&T.w[s][21], ADJ_FLAG);
        } else {
            atomicAdd(&T.w[s][21], 1u);
            atomicAdd(&T.sum[s], (double)a);
            atomicAdd(&T.sq[s], (double)a * (double)a);
            atomicMin(&T.w[s][22], f2ord(a));
            atomicMax(&T.w[s][23], f2ord(a));
            hist_add(T, s, sample_slot(a, fast40, scale, offset));
        }
    }
}

template <typename LabelT, typename DataT, int MODE>
__global__ __launch_bounds__(SCAN_THREADS, 4) void k_face_scan(ScanParams P, RecordBuf R, Counters* C) {
    __shared__ Table T;
    // per-wave stage: 64 live entries + 64 slots where inactive lanes park
    // their (unconditional, branch-free) store
    __shared__ uint4 stage_all[SCAN_THREADS / WAVE][2 * WAVE];
    constexpr bool STATS = MODE != MODE_GRAPH;
    constexpr bool BND = MODE == MODE_BOUNDARY;
    constexpr bool AFF = MODE == MODE_AFFINITY;
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    // wave index through readfirstlane: row/plane coordinates become scalar
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint4* stage = stage_all[wave];
    for (int e = tid; e < TABLE_CAP; e += SCAN_THREADS) entry_reset(T, e);
    if (tid == 0) {
        T.used = 0;
        T.ncompact = 0;
        T.maxv = 0;
    }
    __syncthreads();

    const int64_t Z = P.shape[0], Y = P.shape[1], X = P.shape[2];
    const int64_t sz = Y * X;
    const int64_t x0 = (int64_t)blockIdx.x * TILE_X;
    const int64_t x = x0 + lane;
    const int64_t yw = (int64_t)blockIdx.y * WG_ROWS + wave * ROWS;   // first row of this wave
    const int64_t z0 = (int64_t)blockIdx.z * P.tile_z;
    const int64_t z1 = min(z0 + (int64_t)P.tile_z, Z);
    const bool inx = x < X;
    const bool hx = x + 1 < X;
    const LabelT* L = (const LabelT*)P.labels;
    const DataT* D = (const DataT*)P.data;
    const double scale = P.scale, offset = P.offset;
    const bool fast40 = P.fast40 != 0;
    const int64_t obz = P.own_begin[0], oby = P.own_begin[1], obx = P.own_begin[2];
    const int64_t oez = P.own_end[0], oey = P.own_end[1], oex = P.own_end[2];
    const bool own_x_lo = x >= obx && x < oex;
    const bool own_x_up = x + 1 >= obx && x + 1 < oex;
    const int64_t xh = x0 + TILE_X;          // x of the lane-63 neighbour
    const bool has_xh = xh < X;

    // plane buffers: rows 0..ROWS-1 of this wave + the y-halo row; the x-halo
    // voxel of row r lives in lane r of XL/XD
    LabelT Lc[ROWS + 1], Ln[ROWS + 1];
    float Dc[ROWS + 1], Dn[ROWS + 1];
    LabelT XLc = 0, XLn = 0;
    float XDc = 0.f, XDn = 0.f;

    auto load_plane = [&](int64_t z, LabelT (&Lb)[ROWS + 1], float (&Db)[ROWS + 1], LabelT& XL, float& XD) {
        const LabelT* Lz = L + z * sz + yw * X;
        const DataT* Dz = BND ? D + z * sz + yw * X : nullptr;
#pragma unroll
        for (int r = 0; r <= ROWS; ++r) {
            Lb[r] = 0;
            Db[r] = 0.f;
            if (inx && yw + r < Y) {
                Lb[r] = Lz[r * X + x];
                if constexpr (BND) Db[r] = load_val<DataT>(Dz, r * X + x);
            }
        }
        XL = 0;
        XD = 0.f;
        if (lane < ROWS && has_xh && yw + lane < Y) {
            XL = Lz[lane * X + xh];
            if constexpr (BND) XD = load_val<DataT>(Dz, lane * X + xh);
        }
    };

    const int ablate = P.ablate;
    // diagnostic (ablate & 256): shader-clock stamps per phase, summed per wave
    const bool stamps = (ablate & 256) != 0;
    uint64_t t_fold = 0, t_flush = 0, t_check = 0, t_start = stamps ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t chk = 0;
    bool ovf = false;
    int nbuf = 0;   // staged faces (wave-uniform)

    auto flush_stage = [&]() {
        if (nbuf) {
            const uint64_t t0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
            fold_batch<MODE>(T, stage, nbuf, lane, R, C, fast40, scale, offset, ablate);
            if (stamps) {
                __builtin_amdgcn_s_waitcnt(0);
                t_fold += __builtin_amdgcn_s_memtime() - t0;
            }
            nbuf = 0;
        }
    };
    // append the active lanes of one site to the stage
    auto push = [&](bool act, uint64_t key, float a, uint32_t bbits) {
        const uint64_t m = __ballot(act);
        const int k = __popcll(m);
        if (nbuf + k > WAVE) flush_stage();
        // active lanes append at nbuf + rank; inactive lanes park behind them
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        const int pos = act ? nbuf + rank : nbuf + k + (lane - rank);
        stage[pos] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), __float_as_uint(a), bbits);
        nbuf += k;
    };
    auto face_bits = [&](float b) -> uint32_t { return AFF ? MARK_ADJ : __float_as_uint(b); };

    if (z0 < z1) load_plane(z0, Lc, Dc, XLc, XDc);
    for (int64_t z = z0; z < z1; ++z) {
        const bool hz = z + 1 < Z;
        if (hz) load_plane(z + 1, Ln, Dn, XLn, XDn);        // prefetch: in flight during x/y faces
        const bool own_z_lo = z >= obz && z < oez;
        const bool own_z_up = z + 1 >= obz && z + 1 < oez;
        if (ablate & 8) {   // diagnostic: loads only
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
                chk ^= (uint64_t)(Lc[r] ^ Lc[r + 1] ^ Ln[r]) + (uint64_t)__float_as_uint(Dc[r] + Dn[r]);
        } else {
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const int64_t y = yw + r;
                const bool own_y_lo = y >= oby && y < oey;
                const bool own_y_up = y + 1 >= oby && y + 1 < oey;
                const LabelT lc = Lc[r];
                // x face (x, x+1): lane 63 takes its neighbour from the x-halo
                LabelT lx = shfl_down1<LabelT>(lc);
                float dx = __shfl_down(Dc[r], 1, WAVE);
                const LabelT xl63 = shfl_lane<LabelT>(XLc, r);
                const float xd63 = __shfl(XDc, r, WAVE);
                if (lane == WAVE - 1) {
                    lx = xl63;
                    dx = xd63;
                }
                uint64_t key = 0;
                bool act = y < Y && inx && hx && own_z_lo && own_y_lo && own_x_up && lc != lx;
                act = make_key<LabelT>(act, lc, lx, key, ovf);
                push(act, key, Dc[r], face_bits(dx));
                // y face (y, y+1)
                act = y + 1 < Y && inx && own_z_lo && own_y_up && own_x_lo && lc != Lc[r + 1];
                act = make_key<LabelT>(act, lc, Lc[r + 1], key, ovf);
                push(act, key, Dc[r], face_bits(Dc[r + 1]));
                // affinity samples aff[c, p] for q = p + o_c, p in the owned box
                if constexpr (AFF) {
                    const bool own_p = y < Y && inx && own_z_lo && own_y_lo && own_x_lo;
                    const int64_t i = z * sz + y * X + x;
                    for (int c = 0; c < P.n_channels; ++c) {
                        const int64_t qz = z + P.offsets[c][0];
                        const int64_t qy = y + P.offsets[c][1];
                        const int64_t qx = x + P.offsets[c][2];
                        const bool inq = own_p && qz >= 0 && qz < Z && qy >= 0 && qy < Y && qx >= 0 && qx < X;
                        LabelT lq = lc;
                        float av = 0.f;
                        if (inq) {
                            lq = L[qz * sz + qy * X + qx];
                            av = load_val<DataT>(D, (int64_t)c * Z * sz + i);
                        }
                        bool sact = inq && lq != lc;
                        sact = make_key<LabelT>(sact, lc, lq, key, ovf);
                        push(sact, key, av, MARK_ONE);
                    }
                }
            }
            // z faces: plane z against the prefetched plane z+1
            if (hz) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    const int64_t y = yw + r;
                    const bool own_y_lo = y >= oby && y < oey;
                    uint64_t key = 0;
                    bool act = y < Y && inx && own_z_up && own_y_lo && own_x_lo && Lc[r] != Ln[r];
                    act = make_key<LabelT>(act, Lc[r], Ln[r], key, ovf);
                    push(act, key, Dc[r], face_bits(Dn[r]));
                }
            }
        }
        // every CHECK_PLANES planes: decide on a flush.  Staged faces stay
        // staged (raw faces are valid for whatever table they are folded into
        // later); hist_guard leaves room for them and for CHECK_PLANES planes
        // in the u16 slot bound, the fill threshold leaves room for the new
        // keys of CHECK_PLANES planes (a full table still falls back to
        // direct records).
        if (!(ablate & 16) && ((z - z0) % P.check_planes == P.check_planes - 1 || z + 1 == z1)) {
            const uint64_t t2 = stamps ? __builtin_amdgcn_s_memtime() : 0;
            __syncthreads();
            if (stamps) t_check += __builtin_amdgcn_s_memtime() - t2;
            bool need = tid == 0 && T.used > TABLE_CAP * 3 / 8;
            if constexpr (STATS) {
                for (int e = tid; e < TABLE_CAP; e += SCAN_THREADS) need |= (T.w[e][21] & ~ADJ_FLAG) > P.hist_guard;
            }
            const bool do_flush = __syncthreads_or(need);
            const uint64_t t1 = stamps ? __builtin_amdgcn_s_memtime() : 0;
            if (do_flush) table_flush<MODE>(T, R, C);
            if (stamps) t_flush += __builtin_amdgcn_s_memtime() - t1;
        }
#pragma unroll
        for (int r = 0; r <= ROWS; ++r) {
            Lc[r] = Ln[r];
            Dc[r] = Dn[r];
        }
        XLc = XLn;
        XDc = XDn;
    }
    if (ablate & 8) {
        if (chk == 0x9E3779B97F4A7C15ull) atomicAdd(&C->pad[0], 1ull);
    }
    if (__ballot(ovf) && lane == 0) atomicAdd(&C->label_overflow, 1ull);
    if (stamps && lane == 0) {
        atomicAdd(&C->pad[2], (unsigned long long)t_fold);
        atomicAdd(&C->pad[3], (unsigned long long)t_flush);
        atomicAdd((unsigned long long*)&C->pad[1], (unsigned long long)t_check);
        atomicAdd(&C->pad[0], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
    }
    flush_stage();
    table_flush<MODE>(T, R, C);
}

// ---------------------------------------------------------------------------
// launcher
// ---------------------------------------------------------------------------
template <typename LabelT, typename DataT, int MODE>
static hipError_t launch_scan_t(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    dim3 grid((unsigned)((P.shape[2] + TILE_X - 1) / TILE_X), (unsigned)((P.shape[1] + WG_ROWS - 1) / WG_ROWS),
              (unsigned)((P.shape[0] + P.tile_z - 1) / P.tile_z));
    hipLaunchKernelGGL((k_face_scan<LabelT, DataT, MODE>), grid, dim3(SCAN_THREADS), 0, s, P, R, C);
    return hipGetLastError();
}

template <typename LabelT>
static hipError_t launch_scan_l(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    if (P.data_kind == CTG_DATA_NONE || P.data == nullptr)
        return launch_scan_t<LabelT, float, MODE_GRAPH>(P, R, C, s);
    const bool aff = P.n_channels > 0;
    if (P.data_kind == CTG_DATA_U8)
        return aff ? launch_scan_t<LabelT, uint8_t, MODE_AFFINITY>(P, R, C, s)
                   : launch_scan_t<LabelT, uint8_t, MODE_BOUNDARY>(P, R, C, s);
    return aff ? launch_scan_t<LabelT, float, MODE_AFFINITY>(P, R, C, s)
               : launch_scan_t<LabelT, float, MODE_BOUNDARY>(P, R, C, s);
}

hipError_t launch_face_scan(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    if (P.label_bits == 32) return launch_scan_l<uint32_t>(P, R, C, s);
    return launch_scan_l<uint64_t>(P, R, C, s);
}

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

hipError_t launch_unique_tiles(const uint64_t* L, const int64_t* shape, const int64_t* b, const int64_t* e,
                               uint64_t* out, unsigned long long* count, int64_t cap, hipStream_t s) {
    dim3 grid((unsigned)((e[2] - b[2] + 63) / 64), (unsigned)((e[1] - b[1] + TILE_Y - 1) / TILE_Y),
              (unsigned)((e[0] - b[0] + 15) / 16));
    hipLaunchKernelGGL(k_unique_tiles, grid, dim3(UNIQ_THREADS), 0, s, L, shape[1], shape[2], b[0], b[1], b[2],
                       e[0], e[1], e[2], out, count, cap);
    return hipGetLastError();
}

}  // namespace ctg
