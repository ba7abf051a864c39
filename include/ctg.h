/*
 * ctg.h -- C ABI of the MI355X-native RAG + edge-feature library (libctg.so).
 *
 * This is the drop-in boundary for the hot path of cluster_tools' multicut
 * feature stage.  In the reference, the job bodies call the pybind11 module
 * ``nifty.distributed`` (C++, third party, pinned nifty >=v1.0.7 in
 * conda-recipe/meta.yaml:30).  Each entry point below replaces the array-level
 * work of one of those calls; the N5 I/O those calls do stays in the Python
 * host layer (cluster_tools_amd/ndist.py), which mirrors the reference's
 * function names and arguments:
 *
 *   ctg_rag_features(... data=NULL)   <- ndist.computeMergeableRegionGraph
 *                                        graph/initial_sub_graphs.py:124-129
 *   ctg_rag_features(... boundary)    <- ndist.extractBlockFeaturesFromBoundaryMaps_{float32,uint8}
 *                                        features/block_edge_features.py:127-134
 *   ctg_rag_features(... affinities)  <- ndist.extractBlockFeaturesFromAffinityMaps_{float32,uint8}
 *                                        features/block_edge_features.py:138-145
 *   ctg_merge_stats                   <- ndist.mergeSubgraphs / ndist.mergeFeatureBlocks
 *                                        graph/merge_sub_graphs.py:130-135,
 *                                        features/merge_edge_features.py:141-147
 *   ctg_map_edge_ids                  <- ndist.mapEdgeIds / Graph.findEdges
 *                                        graph/map_edge_ids.py:116-119, test/graph/test_graph.py:92
 *   ctg_unique_labels                 <- the per-block ``nodes`` of computeMergeableRegionGraph
 *                                        test/graph/test_graph.py:53-60
 *   ctg_merge_feature_rows            <- ndist.mergeFeatureBlocks on reference-layout
 *                                        (10-column) sub_features rows,
 *                                        features/merge_edge_features.py:141-147
 *
 * Conventions: plain pointers and sizes; ``mem`` says whether array
 * arguments live in host memory (CTG_MEM_HOST) or in device memory of the
 * current HIP device (CTG_MEM_DEVICE); ``stream`` is a hipStream_t (NULL =
 * default stream).  Every function returns CTG_OK (0) or a negative status;
 * ctg_last_error() returns a thread-local message (the Python shim raises
 * RuntimeError with it, as pybind11 does for nifty's C++ exceptions).
 * Results are library-owned handles released with ctg_free().
 */
#ifndef CTG_H_
#define CTG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CTG_OK 0
#define CTG_ERR_ARG -1
#define CTG_ERR_HIP -2
#define CTG_ERR_NOMEM -3
#define CTG_ERR_UNSUPPORTED -4
#define CTG_ERR_STALE -5   /* a CTG_DEFER_STATS handle whose records were overwritten by a later call */

#define CTG_MEM_HOST 0
#define CTG_MEM_DEVICE 1

#define CTG_DATA_NONE 0   /* graph only */
#define CTG_DATA_F32 1
#define CTG_DATA_U8 2     /* mapped to [0,1] by /255 before binning (SURVEY OPEN-7) */

/* ctg_rag_features flags */
#define CTG_KEEP_STATS 1      /* keep mergeable per-edge statistics (ctg_result_copy_stats) */
#define CTG_NO_NODES 4        /* ctg_rag_blocks: skip the per-block node lists */
#define CTG_NO_ADJ_FILTER 2   /* affinities: keep sample pairs that are not nearest-neighbour
                                 edges of this array (their records carry no ADJ bit); the
                                 caller filters after a merge or by an edge list */
#define CTG_DEFER_STATS 8     /* with CTG_KEEP_STATS, for the ctg_mgpu_* exchange: no statistics
                                 rows are written; ctg_mgpu_pack / ctg_mgpu_merge rebuild a row's
                                 statistics from the call's records where the exchange needs them
                                 (rows sent to another rank, own rows that meet a received key).
                                 The records stay in the device's workspace, so the handle serves
                                 ctg_mgpu_pack / ctg_mgpu_merge only until the next ctg_rag_* or
                                 ctg_merge_stats call on that device (then CTG_ERR_STALE), and
                                 ctg_result_copy_stats has no rows to copy.  Boundary maps without
                                 ignore_label; any other call writes the CTG_KEEP_STATS rows. */

#define CTG_MAX_CHANNELS 24
#define CTG_N_FEATURES 10
#define CTG_NBINS 40
#define CTG_WIDE_RECORD_WORDS 48  /* u32 words of one wide statistics record */

typedef struct ctg_result ctg_result;

/* version / device */
int ctg_version(void);
int ctg_init(int device);
const char* ctg_last_error(void);
int ctg_device_count(int* count);

/*
 * RAG (+ edge features) of one 3-D label array.
 *   labels     uint64 (label_bits=64) or uint32 (label_bits=32), C-order (Z,Y,X)
 *   data       NULL, boundary map (Z,Y,X) or channel-first affinities (C,Z,Y,X)
 *   offsets    NULL for a boundary map, else n_channels x 3 int32 (z,y,x) offsets
 *   own_begin, own_end  faces / samples are counted only when their owning
 *              voxel lies in [own_begin, own_end): the upper voxel of a face, the
 *              voxel p of an affinity sample.  NULL = 0 / shape.  A 1-voxel
 *              own_begin is the lower-halo geometry of increaseRoi=True.
 *   ignore_label  drop edges that contain label 0 (nodes still contain 0)
 *   hist_lo/hi    histogram range (nifty: [0,1])
 *   flags         CTG_KEEP_STATS | CTG_NO_ADJ_FILTER
 * Result: sorted unique edges (u<v, lexicographic), sorted unique nodes and,
 * if data != NULL, an (E,10) float64 feature table
 * [mean, var, min, q10, q25, q50, q75, q90, max, count].
 */
int ctg_rag_features(const void* labels, int label_bits,
                     const void* data, int data_kind,
                     int n_channels, const int32_t* offsets,
                     const int64_t* shape, const int64_t* own_begin, const int64_t* own_end,
                     int ignore_label, double hist_lo, double hist_hi,
                     int flags, int mem, void* stream, ctg_result** out);

/*
 * Batched per-block sub-graphs and features (the ndist per-block calls in
 * one launch): block b is a C-order array of shape[b] starting at element
 * label_offset[b] of `labels` (and data_offset[b] of `data`; affinities
 * channel-first, C x shape).  For every block:
 *   nodes    sorted unique labels of the own box (inner block,
 *            test/graph/test_graph.py:53-60)
 *   edges    sorted unique (u<v) keys of the faces with both voxels in the
 *            graph box (increaseRoi: [begin-1, end), test_graph.py:42-84)
 *   features (data != NULL) per edge, the 10 features of the samples owned by
 *            the block -- boundary faces / affinity voxels whose upper voxel /
 *            voxel p lies in the own box; edges of the graph box without owned
 *            samples get count 0 (block_edge_features.py:127-145).  With
 *            affinities a sample counts only if its pair is an edge of the
 *            block's sub-graph.
 * Rows [edge_off[b], edge_off[b+1]) of the edge / feature / stats tables and
 * [node_off[b], node_off[b+1]) of the node table belong to block b
 * (ctg_result_block_offsets).  Replaces the per-block loops of
 * ndist.computeMergeableRegionGraph (graph/initial_sub_graphs.py:124-129) and
 * ndist.extractBlockFeaturesFrom*Maps_* (features/block_edge_features.py:127-145).
 */
typedef struct ctg_block_desc {
    int64_t label_offset;
    int64_t data_offset;
    int64_t shape[3];
    int64_t own_begin[3], own_end[3];
    int64_t graph_begin[3], graph_end[3];
} ctg_block_desc;

int ctg_rag_blocks(const void* labels, int label_bits, const void* data, int data_kind, int n_channels,
                   const int32_t* offsets, const ctg_block_desc* blocks, int n_blocks, int64_t labels_len,
                   int64_t data_len, int ignore_label, double hist_lo, double hist_hi, int flags, int mem,
                   void* stream, ctg_result** out);
int ctg_result_num_blocks(const ctg_result* r);
/* page-locked host buffers for staging batched inputs (H2D at full PCIe rate) */
void* ctg_host_alloc(int64_t bytes);
void ctg_host_free(void* p);
int ctg_result_block_offsets(const ctg_result* r, int64_t* edge_off, int64_t* node_off);

/* sorted unique labels of labels[begin:end] (box in array coordinates) */
int ctg_unique_labels(const uint64_t* labels, const int64_t* shape,
                      const int64_t* begin, const int64_t* end,
                      int mem, void* stream, ctg_result** out);

/* sorted unique values of an (n,) uint64 list -> result nodes (union of the
 * per-slab node lists of the multi-GPU path; ndist.mergeSubgraphs node union,
 * graph/merge_sub_graphs.py:130-135) */
int ctg_unique_values(const uint64_t* values, int64_t n, int mem, void* stream, ctg_result** out);

/* Combine partial statistics tables (wide records, one per (part, edge)) into
 * one table: counts add, moments combine exactly (re-pivoted shifted sums,
 * i.e. Chan's pairwise rule), min/max elementwise, histograms add.
 *   keys     n x 2 uint64 (u,v) per record;
 *   sums     n x 2 float64 (S1, S2) = (sum(x - p), sum((x - p)^2)) about the
 *            record's pivot p = the float32 in record word 45 (0: power sums);
 *   records  n x CTG_WIDE_RECORD_WORDS uint32: 42 histogram slots, count|ADJ,
 *            ordered min, ordered max, pivot bits, 2 zero words. */
int ctg_merge_stats(const uint64_t* keys, const double* sums, const uint32_t* records,
                    int64_t n, double hist_lo, double hist_hi, int keep_stats,
                    int mem, void* stream, ctg_result** out);

/* Multi-GPU z-slab plan (SURVEY §8(b) ctg_mgpu_*; replaces the reference's
 * block-grid job split, graph/initial_sub_graphs.py:110-129 with
 * utils/volume_utils.py blocks_in_volume, for one rank per GPU): rank `rank` of
 * `world_size` owns planes [out[1], out[2]) = [Z*rank/W, Z*(rank+1)/W) of a
 * volume of Z planes and reads [out[0], out[2]): below its owned range as many
 * halo planes as the face / offsets reach down (1 for boundary maps and
 * nearest-neighbour affinities, max(-o_z) for long-range offsets), none for
 * rank 0.  ctg_rag_features' own_begin[0] is out[1] - out[0].  Positive z
 * offsets (a partner above the slab) with world_size > 1 are
 * CTG_ERR_UNSUPPORTED: the z-slab layout has no upper halo.  Host-only: needs
 * no device. */
int ctg_mgpu_slab(int64_t Z, int world_size, int rank, const int64_t* offsets, int n_channels, int64_t* out);

/* Multi-GPU combine of the ranks' partial tables (replaces the
 * block -> merge step of ndist.mergeSubgraphs, graph/merge_sub_graphs.py:130-135,
 * and ndist.mergeFeatureBlocks, features/merge_edge_features.py:141-147, at the
 * scale of whole GPUs).  `local` is a rank's CTG_KEEP_STATS result of its slab
 * (affinities: also CTG_NO_ADJ_FILTER).  The global sorted edge table is
 * range-partitioned by u; the host runs the collectives (RCCL over xGMI via
 * torch.distributed in cluster_tools_amd/dist.py) between these steps, all
 * arrays in device memory of the current device:
 *   1. ctg_mgpu_sample -> meta (CTG_MGPU_SAMPLES + 1 int64): evenly spaced u
 *      values (unsigned order as int64: u xor 2^63) and the edge count;
 *      all_gather of meta -> meta_all (world x (CTG_MGPU_SAMPLES + 1));
 *   2. ctg_mgpu_split -> counts (world x 2 int64): rows and node ids this rank
 *      sends to each rank (its own entry: what it keeps); all_gather ->
 *      counts_all (world x world x 2, [src][dst][rows, nodes]), read to host;
 *   3. ctg_mgpu_pack -> send (int64 words): for every dst != rank with data, in
 *      rank order, rows x CTG_MGPU_ROW_WORDS words ((u, v), (S1, S2) bits, the
 *      48-word wide record) then the node ids; all_to_all with those sizes ->
 *      recv (segments of every src != rank in rank order);
 *   4. ctg_mgpu_merge -> *out: this rank's shard of the global table (sorted
 *      edges, features, nodes); equal keys combine exactly (counts and
 *      histograms add, moments by Chan's rule), affinity partials keep keys
 *      whose ADJ bit some record carries.  `local`'s arrays move into the shard
 *      (a range of them when nothing was received: no copy); ctg_free(local)
 *      is still required.  counts_all is host memory.
 * world_size <= CTG_MGPU_MAX_WORLD. */
#define CTG_MGPU_SAMPLES 1024
#define CTG_MGPU_ROW_WORDS 28
#define CTG_MGPU_MAX_WORLD 32
int ctg_mgpu_sample(const ctg_result* local, int64_t* meta, void* stream);
int ctg_mgpu_split(const ctg_result* local, const int64_t* meta_all, int world_size, int64_t* counts, void* stream);
int ctg_mgpu_pack(const ctg_result* local, const int64_t* counts_all, int world_size, int rank, int64_t* send,
                  void* stream);
int ctg_mgpu_merge(ctg_result* local, const int64_t* recv, const int64_t* counts_all, int world_size, int rank,
                   double hist_lo, double hist_hi, void* stream, ctg_result** out);

/* Merge reference-layout feature rows (n x 10 float64, [mean, var, min,
 * q10..q90, max, count]) of global edges ids[i] in [id_begin, id_end) into
 * out ((id_end - id_begin) x 10): count sum, count-weighted mean, exact pooled
 * variance, min / max over rows with count > 0, count-weighted quantiles.
 * Edges without rows get zero rows.  An id outside the range is CTG_ERR_ARG. */
int ctg_merge_feature_rows(const uint64_t* ids, const double* rows, int64_t n, int64_t id_begin, int64_t id_end,
                           double* out, int mem, void* stream);

/* sorted unique (u,v) pairs of an (n,2) uint64 list (union of block sub-graph
 * edge lists, ndist.mergeSubgraphs); result nodes = unique endpoints */
int ctg_unique_pairs(const uint64_t* pairs, int64_t n, int mem, void* stream, ctg_result** out);

/* position of each query (u,v) in the sorted global edge table, -1 if absent */
int ctg_map_edge_ids(const uint64_t* global_edges, int64_t n_global,
                     const uint64_t* query, int64_t n_query, int64_t* out_ids,
                     int mem, void* stream);

/* result accessors; dst lives in host (CTG_MEM_HOST) or device memory */
int64_t ctg_result_num_edges(const ctg_result* r);
int64_t ctg_result_num_nodes(const ctg_result* r);
int ctg_result_copy_edges(const ctg_result* r, uint64_t* dst, int mem);
int ctg_result_copy_nodes(const ctg_result* r, uint64_t* dst, int mem);
int ctg_result_copy_features(const ctg_result* r, double* dst, int mem);
int ctg_result_copy_stats(const ctg_result* r, double* sums_dst, uint32_t* records_dst, int mem);
/* device pointers for zero-copy consumers (valid until ctg_free) */
const uint64_t* ctg_result_device_edges(const ctg_result* r);
const double* ctg_result_device_features(const ctg_result* r);
int ctg_result_info(const ctg_result* r, int64_t* n_records, int64_t* n_direct);
void ctg_free(ctg_result* r);

/* deterministic synthetic volumes (Voronoi supervoxels + boundary map), device */
int ctg_synth_volume(uint64_t* labels, float* boundary, const int64_t* shape,
                     int64_t z_offset, const int64_t* global_shape, int cell,
                     uint64_t seed, uint64_t label_offset, double noise_amp, void* stream);
/* Filter-feature branch (features/block_edge_features.py:151-238): the
 * fastfilters / vigra filters vu.apply_filter runs (utils/volume_utils.py:80-94),
 * on device float32 arrays (cluster_tools_amd/fastfilters.py).
 * ctg_filter_conv_axis: out[p] = sum_k taps[k] in[reflect(p + (k - n_taps/2) e_axis)],
 *   C-order shape[ndim] (ndim <= 3), odd n_taps <= 257, mirror borders. */
int ctg_filter_conv_axis(const float* in, float* out, const int64_t* shape, int ndim, int axis, const float* taps,
                         int n_taps, void* stream);
/* op 0: sqrt(a^2+b^2+c^2), 1: a+b+c (b, c may be NULL), 2: a*b, 3: a-b; n elements */
int ctg_filter_combine(int op, const float* a, const float* b, const float* c, float* out, int64_t n, void* stream);
/* eigenvalues (descending) of n symmetric dim x dim matrices (dim 2 or 3), upper-triangle
 * components as planes comps[k*n + i]; out (n, dim) */
int ctg_sym_eigenvalues(const float* comps, int dim, int64_t n, float* out, void* stream);

int ctg_synth_affinities(const float* boundary, float* affs, const int64_t* shape,
                         int n_channels, const int32_t* offsets, void* stream);

/*
 * Native N5 / zarr chunk I/O (host memory; zlib + a thread pool).  The ndist
 * mirror reads the ROIs and writes the varlength chunks of the per-block path
 * through these (z5's role in the reference: graph/initial_sub_graphs.py:72-75,
 * features/block_edge_features.py:63-64, 236).
 *   format       CTG_IO_N5 | CTG_IO_ZARR_DOT (i.j.k keys) | CTG_IO_ZARR_SLASH
 *   big_endian   1: stored elements are big-endian (N5; zarr '>' dtypes)
 *   compression  CTG_IO_RAW | CTG_IO_GZIP (writes gzip streams: N5 {"type":"gzip"},
 *                zarr "gzip") | CTG_IO_ZLIB (writes zlib streams: N5 "useZlib":
 *                true, zarr "zlib"); reads auto-detect gzip and zlib for both
 */
#define CTG_IO_N5 0
#define CTG_IO_ZARR_DOT 1
#define CTG_IO_ZARR_SLASH 2
#define CTG_IO_RAW 0
#define CTG_IO_GZIP 1
#define CTG_IO_ZLIB 2
/* C-order box [begin, end) of a chunked dataset into `out`; missing chunks are
 * filled with the dtype_size-byte pattern fill_value (native byte order), or
 * zeros when fill_value is NULL */
int ctg_io_read_box(const char* ds_path, int format, int dtype_size, int big_endian, int ndim, const int64_t* shape,
                    const int64_t* chunks, int compression, const int64_t* begin, const int64_t* end, void* out,
                    int n_threads, const void* fill_value);
/* varlength N5 chunks at n_chunks grid positions: out[i] = malloc'ed native-
 * endian elements (free with ctg_io_free), n_out[i] = count, or NULL / -1 if
 * the chunk does not exist */
int ctg_io_read_varlen(const char* ds_path, int dtype_size, int ndim, int64_t n_chunks, const int64_t* positions,
                       int compression, void** out, int64_t* n_out, int n_threads);
void ctg_io_free(void* p);
/* drop the decoded-chunk cache of ctg_io_read_box (budget: env CTG_IO_CACHE_MB,
 * default 4096; an entry is reused only while its file keeps its inode, size,
 * mtime and ctime -- every writer here replaces chunk files by rename) */
void ctg_io_cache_clear(void);
/* cache counters since process start: out[0] chunk reads the cache served
 * (decoded, or in flight on the readahead pool), out[1] decodes on the
 * caller's threads, out[2] decodes by the readahead pool */
void ctg_io_cache_stats(int64_t* out);
/* drop the cached decodes of one chunk file (writers outside ctg_io call it) */
void ctg_io_cache_drop(const char* chunk_path);
/* write n_chunks chunks (default mode with chunk_shapes, or N5 varlength) */
int ctg_io_write_chunks(const char* ds_path, int format, int dtype_size, int big_endian, int ndim, int64_t n_chunks,
                        const int64_t* positions, const int64_t* chunk_shapes, const void* const* data,
                        const int64_t* n_elements, int varlen, int compression, int level, int n_threads);

/* release every device block the library caches on the current device
 * (workspace and allocator pool); result handles stay valid */
int ctg_trim(void);

/* profiling: per-phase device milliseconds of the last ctg_rag_features call
 * (HIP events on the call's stream): [0] face scan, [1] key pack, [2] sort,
 * [3] segment, [4] reduce+finalize, [5] nodes, [6] total */
int ctg_set_profiling(int on);
int ctg_last_timings(double* ms, int n);

#ifdef __cplusplus
}
#endif
#endif /* CTG_H_ */
