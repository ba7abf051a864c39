// Face scan: the O(V) hot loop of the RAG + edge-feature path (gfx950).
//
// One workgroup (4 waves) owns a tile of 64 (x) x 8 (y) x tile_z (z) voxels.
// A wave walks one z-plane of the tile row by row (lane = x), carrying the
// y-neighbour row in registers, so every label/value is read from HBM once;
// the z-neighbour row and the lane-63 x-neighbour come from L2.  Every
// boundary face (p, p+e_a) with differing labels is folded into an LDS
// open-addressing edge table keyed by (u<<32)|v that holds, per edge, the
// sample count, f64 sum and sum of squares, order-preserving min/max and the
// 42-slot vigra histogram (u16 slots packed in u32 words).  The table is
// flushed to HBM as one record per (tile, edge) when it is half full and at the
// end of the tile, so HBM sees ~E*(tile surface factor) records instead of one
// entry per face.  Replaces the per-face std::set / findEdge loop of
// nifty.distributed (called at graph/initial_sub_graphs.py:124-129 and
// features/block_edge_features.py:127-145).
#include "ctg_internal.h"

namespace ctg {

enum { MODE_GRAPH = 0, MODE_BOUNDARY = 1, MODE_AFFINITY = 2 };

struct __align__(16) Table {
    uint64_t key[TABLE_CAP];
    double sum[TABLE_CAP];
    double sq[TABLE_CAP];
    uint32_t w[TABLE_CAP][NREC_WORDS];   // hist words 0..20, 21 cnt|ADJ, 22 min, 23 max
    uint16_t compact[TABLE_CAP];
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

__device__ __forceinline__ int table_insert(Table& T, uint64_t key) {
    uint32_t h = hash_key(key) & (TABLE_CAP - 1);
#pragma unroll 1
    for (int i = 0; i < 48; ++i) {
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
    __syncthreads();
    const int tid = threadIdx.x;
    uint64_t mv = 0;
    for (int e = tid; e < TABLE_CAP; e += SCAN_THREADS) {
        uint64_t k = T.key[e];
        if (k != EMPTY_KEY) {
            uint32_t r = atomicAdd(&T.ncompact, 1u);
            T.compact[r] = (uint16_t)e;
            mv = max(mv, k & 0xFFFFFFFFull);
        }
    }
    if (mv) atomicMax(&T.maxv, (unsigned long long)mv);
    __syncthreads();
    const uint32_t n = T.ncompact;
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
__device__ void emit_direct(RecordBuf R, Counters* C, uint64_t key, int nsamp, float a, float b,
                            double scale, double offset, uint32_t flag, bool with_stats) {
    unsigned long long i = atomicAdd(&C->n_records, 1ull);
    atomicAdd(&C->n_direct, 1ull);
    atomicMax(&C->max_v, (unsigned long long)(key & 0xFFFFFFFFull));
    if (i >= (unsigned long long)R.cap) return;
    R.key[i] = key;
    if (!with_stats) return;
    uint32_t row[NREC_WORDS];
#pragma unroll
    for (int j = 0; j < NREC_WORDS; ++j) row[j] = 0;
    double s = 0.0, q = 0.0;
    uint32_t mn = ORD_POS_INF, mx = ORD_NEG_INF;
    if (nsamp >= 1) {
        int sa = hist_slot((double)a, scale, offset);
        row[sa >> 1] += 1u << ((sa & 1) * 16);
        s += (double)a; q += (double)a * (double)a;
        mn = min(mn, f2ord(a)); mx = max(mx, f2ord(a));
    }
    if (nsamp >= 2) {
        int sb = hist_slot((double)b, scale, offset);
        row[sb >> 1] += 1u << ((sb & 1) * 16);
        s += (double)b; q += (double)b * (double)b;
        mn = min(mn, f2ord(b)); mx = max(mx, f2ord(b));
    }
    row[21] = (uint32_t)nsamp | flag;
    row[22] = mn;
    row[23] = mx;
    R.sums[i] = make_double2(s, q);
#pragma unroll
    for (int j = 0; j < NREC_WORDS; ++j) R.hist[i * NREC_WORDS + j] = row[j];
}

template <typename DataT>
__device__ __forceinline__ float load_val(const DataT* p, int64_t i) {
    if constexpr (sizeof(DataT) == 1) {
        return __fdiv_rn((float)p[i], 255.0f);
    } else {
        return p[i];
    }
}

template <int MODE>
__device__ __forceinline__ void add_samples(Table& T, int s, int nsamp, float a, float b,
                                            double scale, double offset) {
    double sum = (double)a, sq = (double)a * (double)a;
    float mn = a, mx = a;
    if (nsamp == 2) {
        sum += (double)b;
        sq += (double)b * (double)b;
        mn = fminf(a, b);
        mx = fmaxf(a, b);
    }
    atomicAdd(&T.w[s][21], (uint32_t)nsamp);
    atomicAdd(&T.sum[s], sum);
    atomicAdd(&T.sq[s], sq);
    atomicMin(&T.w[s][22], f2ord(mn));
    atomicMax(&T.w[s][23], f2ord(mx));
    int sa = hist_slot((double)a, scale, offset);
    atomicAdd(&T.w[s][sa >> 1], 1u << ((sa & 1) * 16));
    if (nsamp == 2) {
        int sb = hist_slot((double)b, scale, offset);
        atomicAdd(&T.w[s][sb >> 1], 1u << ((sb & 1) * 16));
    }
}

template <typename LabelT>
__device__ __forceinline__ LabelT shfl_down1(LabelT v) {
    if constexpr (sizeof(LabelT) == 8) {
        uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
        lo = __shfl_down(lo, 1, WAVE);
        hi = __shfl_down(hi, 1, WAVE);
        return ((LabelT)hi << 32) | lo;
    } else {
        return (LabelT)__shfl_down((uint32_t)v, 1, WAVE);
    }
}

template <typename LabelT, typename DataT, int MODE>
__global__ __launch_bounds__(SCAN_THREADS) void k_face_scan(ScanParams P, RecordBuf R, Counters* C) {
    __shared__ Table T;
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wave = tid >> 6;
    for (int e = tid; e < TABLE_CAP; e += SCAN_THREADS) entry_reset(T, e);
    if (tid == 0) {
        T.used = 0;
        T.ncompact = 0;
        T.maxv = 0;
    }
    __syncthreads();

    const int64_t Z = P.shape[0], Y = P.shape[1], X = P.shape[2];
    const int64_t sz = Y * X;
    const int64_t x = (int64_t)blockIdx.x * TILE_X + lane;
    const int64_t y0 = (int64_t)blockIdx.y * TILE_Y;
    const int64_t z0 = (int64_t)blockIdx.z * P.tile_z;
    const bool inx = x < X;
    const LabelT* L = (const LabelT*)P.labels;
    const DataT* D = (const DataT*)P.data;
    const double scale = P.scale, offset = P.offset;
    const int64_t obz = P.own_begin[0], oby = P.own_begin[1], obx = P.own_begin[2];
    constexpr bool STATS = MODE != MODE_GRAPH;
    constexpr bool BND = MODE == MODE_BOUNDARY;
    const uint32_t adj_flag = (MODE == MODE_AFFINITY) ? ADJ_FLAG : 0u;

    // RAG face: key + (boundary) both voxel values as samples
    auto face = [&](LabelT lp, LabelT lq, float dp, float dq, bool valid) {
        if (!(valid && lp != lq)) return;
        LabelT u = lp < lq ? lp : lq;
        LabelT v = lp < lq ? lq : lp;
        if constexpr (sizeof(LabelT) == 8) {
            if (v >> 32) {
                atomicAdd(&C->label_overflow, 1ull);
                return;
            }
        }
        const uint64_t key = ((uint64_t)u << 32) | (uint64_t)v;
        const int s = table_insert(T, key);
        if (s < 0) {
            emit_direct(R, C, key, BND ? 2 : 0, dp, dq, scale, offset, adj_flag, STATS);
            return;
        }
        if constexpr (BND) add_samples<MODE>(T, s, 2, dp, dq, scale, offset);
        if constexpr (MODE == MODE_AFFINITY) atomicOr(&T.w[s][21], ADJ_FLAG);
    };

    for (int zs = 0; zs < P.tile_z; zs += 4) {
        const int dz = zs + wave;
        const int64_t z = z0 + dz;
        if (dz < P.tile_z && z < Z) {
            const bool hz = z + 1 < Z;
            const bool own_z_lo = z >= obz;          // p_z >= own (faces along y, x)
            const bool own_z_up = z + 1 >= obz;      // q_z >= own (face along z)
            const bool own_x_lo = x >= obx;
            const bool own_x_up = x + 1 >= obx;
            int64_t i = z * sz + y0 * X + x;
            LabelT cl = 0;
            float cd = 0.f;
            if (inx && y0 < Y) {
                cl = L[i];
                if constexpr (BND) cd = load_val<DataT>(D, i);
            }
            for (int dy = 0; dy < TILE_Y; ++dy) {
                const int64_t y = y0 + dy;
                if (y >= Y) break;
                const bool hy = y + 1 < Y;
                LabelT yl = 0, zl = 0, xl;
                float yd = 0.f, zd = 0.f, xd;
                if (inx) {
                    if (hy) {
                        yl = L[i + X];
                        if constexpr (BND) yd = load_val<DataT>(D, i + X);
                    }
                    if (hz) {
                        zl = L[i + sz];
                        if constexpr (BND) zd = load_val<DataT>(D, i + sz);
                    }
                }
                xl = shfl_down1<LabelT>(cl);
                xd = __shfl_down(cd, 1, WAVE);
                const bool hx = x + 1 < X;
                if (lane == WAVE - 1 && hx) {
                    xl = L[i + 1];
                    if constexpr (BND) xd = load_val<DataT>(D, i + 1);
                }
                const bool own_y_lo = y >= oby;
                const bool own_y_up = y + 1 >= oby;
                if (inx) {
                    face(cl, xl, cd, xd, hx && own_z_lo && own_y_lo && own_x_up);
                    face(cl, yl, cd, yd, hy && own_z_lo && own_y_up && own_x_lo);
                    face(cl, zl, cd, zd, hz && own_z_up && own_y_lo && own_x_lo);
                    if constexpr (MODE == MODE_AFFINITY) {
                        // samples aff[c, p] for q = p + o_c, p in the owned box
                        if (own_z_lo && own_y_lo && own_x_lo) {
                            for (int c = 0; c < P.n_channels; ++c) {
                                const int64_t qz = z + P.offsets[c][0];
                                const int64_t qy = y + P.offsets[c][1];
                                const int64_t qx = x + P.offsets[c][2];
                                if (qz < 0 || qz >= Z || qy < 0 || qy >= Y || qx < 0 || qx >= X) continue;
                                const LabelT lq = L[qz * sz + qy * X + qx];
                                if (lq == cl) continue;
                                LabelT u = cl < lq ? cl : lq;
                                LabelT v = cl < lq ? lq : cl;
                                if constexpr (sizeof(LabelT) == 8) {
                                    if (v >> 32) {
                                        atomicAdd(&C->label_overflow, 1ull);
                                        continue;
                                    }
                                }
                                const float a = load_val<DataT>(D, (int64_t)c * Z * sz + i);
                                const uint64_t key = ((uint64_t)u << 32) | (uint64_t)v;
                                const int s = table_insert(T, key);
                                if (s < 0) {
                                    emit_direct(R, C, key, 1, a, 0.f, scale, offset, 0u, true);
                                    continue;
                                }
                                add_samples<MODE>(T, s, 1, a, 0.f, scale, offset);
                            }
                        }
                    }
                }
                cl = yl;
                cd = yd;
                i += X;
            }
        }
        __syncthreads();
        if (T.used > TABLE_CAP / 2) table_flush<MODE>(T, R, C);
    }
    table_flush<MODE>(T, R, C);
}

// ---------------------------------------------------------------------------
// launcher
// ---------------------------------------------------------------------------
template <typename LabelT, typename DataT, int MODE>
static hipError_t launch_scan_t(const ScanParams& P, const RecordBuf& R, Counters* C, hipStream_t s) {
    dim3 grid((unsigned)((P.shape[2] + TILE_X - 1) / TILE_X), (unsigned)((P.shape[1] + TILE_Y - 1) / TILE_Y),
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
constexpr int USET_CAP = 2048;

__global__ __launch_bounds__(SCAN_THREADS) void k_unique_tiles(const uint64_t* L, int64_t Y, int64_t X,
                                                                int64_t bz, int64_t by, int64_t bx,
                                                                int64_t ez, int64_t ey, int64_t ex,
                                                                uint64_t* out, unsigned long long* count,
                                                                int64_t cap) {
    __shared__ uint64_t set[USET_CAP];
    __shared__ uint32_t used;
    __shared__ uint32_t n;
    __shared__ unsigned long long base;
    __shared__ uint32_t w;
    const int tid = threadIdx.x;
    for (int e = tid; e < USET_CAP; e += SCAN_THREADS) set[e] = EMPTY_KEY;
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
                            if (old == EMPTY_KEY) { atomicAdd(&used, 1u); break; }
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
                n = used;
                base = atomicAdd(count, (unsigned long long)used);
            }
            __syncthreads();
            // compaction order is irrelevant (sorted afterwards)
            if (tid == 0) w = 0;
            __syncthreads();
            for (int e = tid; e < USET_CAP; e += SCAN_THREADS) {
                uint64_t k = set[e];
                if (k != EMPTY_KEY) {
                    uint32_t r = atomicAdd(&w, 1u);
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
    hipLaunchKernelGGL(k_unique_tiles, grid, dim3(SCAN_THREADS), 0, s, L, shape[1], shape[2], b[0], b[1], b[2],
                       e[0], e[1], e[2], out, count, cap);
    return hipGetLastError();
}

}  // namespace ctg
