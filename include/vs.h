/*
 * vs.h -- C ABI of the MI355X-native exact flat k-NN backend (libvs.so).
 *
 * Drop-in boundary for the vector arithmetic behind the reference's VectorStore
 * (/root/reference/utils/vector_store.py).  The reference reaches faiss through SWIG at these
 * call sites; each entry point below replaces one of them:
 *
 *   faiss.IndexFlatIP(d) / faiss.IndexFlatL2(d)   utils/vector_store.py:79-81   -> vs_create
 *   index.add(vector)                             utils/vector_store.py:163-164 -> vs_add
 *   index.search(vector, k)                       utils/vector_store.py:190-191 -> vs_search
 *   index.reconstruct(i)                          utils/vector_store.py:207     -> vs_reconstruct
 *   index.ntotal / index.d                        utils/vector_store.py:183,188,255-258,271 -> vs_ntotal, vs_dim
 *   _create_index() on clear()                    utils/vector_store.py:277     -> vs_reset
 *   faiss.write_index (storage payload)           utils/vector_store.py:234     -> vs_reconstruct_n
 *
 * Plain pointers and sizes only; no torch types.  Rows are row-major n x d fp32, already
 * normalised by the Python layer exactly as the reference does it (utils/vector_store.py:83-90).
 *
 * Semantics of vs_search (faiss IndexFlat semantics, made exact):
 *   - IP: D descending, L2: D ascending (squared L2), ties -> lower id.
 *   - The returned ids are the exact top-k under the canonical fp64 score (oracle/vs_oracle.c);
 *     D is that score rounded to fp32 (|D - faiss fp32 D| <= 1e-5 for unit vectors).
 *   - Unfilled slots (k > ntotal): I = -1, D = -FLT_MAX (IP) / +FLT_MAX (L2).
 *
 * Errors: every int-returning function returns 0 on success, < 0 on failure; the message is
 * in vs_last_error() (thread-local).  No C++ exception crosses the ABI.
 *
 * Threading: concurrent vs_search* calls on one handle are safe (shared corpus, one stream +
 * workspace per call from a pool).  vs_add, vs_add_device, vs_add_synthetic and vs_reset take an exclusive lock.
 */
#ifndef VS_H_
#define VS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vs_index vs_index;

enum { VS_METRIC_IP = 0, VS_METRIC_L2 = 1 };
enum { VS_DTYPE_F32 = 0, VS_DTYPE_BF16 = 1, VS_DTYPE_F16 = 2 };
enum { VS_SCREEN_NATIVE = 0, VS_SCREEN_I8 = 1 };

enum {
    VS_OK = 0,
    VS_ERR_ARG = -1,          /* bad argument (dims, k, null pointer) */
    VS_ERR_DEVICE = -2,       /* no HIP device / HIP runtime failure */
    VS_ERR_OOM = -3,          /* device allocation failed */
    VS_ERR_UNCERTIFIED = -4,  /* exactness certificate could not be established (IVF list search
                               * only: every flat search ends in the exact full scan instead) */
    VS_ERR_INTERNAL = -5
};

/* ---- lifecycle (faiss.IndexFlatIP / IndexFlatL2 constructors, utils/vector_store.py:79-81) */
int vs_create(int d, int metric, int dtype, int device, vs_index** out);
void vs_destroy(vs_index* index);
int vs_reset(vs_index* index);                    /* clear(): utils/vector_store.py:273-280 */

/* ---- add (index.add, utils/vector_store.py:164) */
int vs_add(vs_index* index, const float* x, int64_t n);                 /* host fp32 n x d */
int vs_add_device(vs_index* index, const float* x_dev, int64_t n, void* stream); /* device fp32, packed on
                                                                                  * `stream` (NULL: legacy default) */
/* Fill rows [ntotal, ntotal+n) with synthetic rows global_row0.. of the counter-hash generator
 * (bench / tests; bit-identical to oracle/vs_oracle.c orc_synth_rows). */
int vs_add_synthetic(vs_index* index, uint64_t seed, int64_t global_row0, int64_t n, int normalize);
/* Size the row storage (and the int8 screen copy) for n more rows in one allocation: later adds up
 * to that size never regrow (a regrow copies the rows into a 1.5x larger buffer, so the old and
 * the new storage coexist for the copy).  vs_capacity: rows the storage holds without regrowing. */
int vs_reserve(vs_index* index, int64_t n);
int64_t vs_capacity(const vs_index* index);
/* Same generator, written as row-major fp32 (values rounded to `dtype`) into device memory on
 * `device`: synthetic query batches for bench.py / tests. */
int vs_synthesize(int device, uint64_t seed, int64_t global_row0, int64_t n, int d, int normalize, int dtype,
                  float* out_dev, void* stream);

/* ---- search (index.search, utils/vector_store.py:191).  Exact for every query: a failed
 * certificate re-screens the query 4x deeper, and past the deepest screen (KP_MAX) the exact full
 * scan answers it (faiss's k lowest ids among any number of tied rows). */
int vs_search(vs_index* index, const float* q, int64_t nq, int32_t k, float* D, int64_t* I);
/* All pointers device-resident; enqueued on `stream` (NULL = the legacy default stream, which is
 * torch's default stream: device calls are always ordered with the caller's stream), no host
 * sync.  S64 (optional, may be NULL) receives the exact fp64 scores; id_offset is added to every
 * returned id (row-sharded corpora).  Certification failures are counted on the device
 * (vs_uncertified_count) and are NOT retried on this path. */
int vs_search_device(vs_index* index, const float* q_dev, int64_t nq, int32_t k, float* D_dev,
                     int64_t* I_dev, double* S64_dev, int64_t id_offset, void* stream);

/* Same outputs, but exact for every query (every dtype): each query block's first pass is
 * followed on the stream by a fallback round at the deepest screen (KP_MAX, proven seed; the MFMA
 * screen of the stored dtype, fp32 included) whose kernels do nothing unless a certificate of that
 * block failed, and which rewrites only the failed queries; a query even that round cannot certify
 * (more near-tied rows than KP_MAX, e.g. thousands of identical embeddings) is answered by a gated
 * exact full scan of the shard (every row scored, a running top-k: faiss's lowest ids among any
 * number of ties; counted in vs_full_scan_count) -- no host sync: the call returns with the work
 * queued.  The product's multi-GPU layers (photo_search_engine_amd/distributed.py,
 * vs_multi_search) use this one. */
int vs_search_device_exact(vs_index* index, const float* q_dev, int64_t nq, int32_t k, float* D_dev,
                           int64_t* I_dev, double* S64_dev, int64_t id_offset, void* stream);

/* ---- two-phase exact device search: the sharded step (one shard per rank) with a global T'
 * exchange (no faiss counterpart; replaces vs_search_device_exact inside
 * photo_search_engine_amd/distributed.py when vs_two_phase_ok says so).
 *  phase A: screen the shard and score each query's best keys exactly; S_a / I_a (nq x k, device,
 *           best-first, ids + id_offset, padded with -1 / worst score) are this shard's best so far;
 *           returns a pending search in *out that holds the index's read lock and workspace;
 *  (the caller all-gathers every shard's (S_a, I_a) and merges them: vs_merge_shards_device)
 *  phase B: floor_S = that merged nq x k list (device): its k-th score per query is a lower bound
 *           of the global k-th best, so the shard scores only rows whose bound reaches it and
 *           certifies against it; writes the shard's exact top-k as vs_search_device_exact does
 *           (its gated device fallback round included) and frees the pending search.
 * Results after the final all-gather + merge are identical to vs_search_device_exact's.  Every rank
 * must take the same path: vs_two_phase_ok depends only on the index configuration (int8 screen,
 * bf16/f16 rows) and on (nq, k) -- one int8 MFMA block, 8 < nq <= 256, k <= 1024.  world = the
 * number of shards (sets phase A's depth).  stride: the element stride of the (S, I) outputs (2 =
 * interleaved (score bits, id) pairs, ready for the all-gather; D_dev stays nq x k).
 * vs_search_pending_free drops a pending search whose phase B will not run. */
typedef struct vs_pending vs_pending;
int vs_two_phase_ok(vs_index* index, int64_t nq, int32_t k);
int vs_search_device_phase_a(vs_index* index, const float* q_dev, int64_t nq, int32_t k, int32_t world,
                             int64_t id_offset, double* S_a, int64_t* I_a, int32_t stride, void* stream,
                             vs_pending** out);
int vs_search_device_phase_b(vs_pending* pending, const double* floor_S, float* D_dev, int64_t* I_dev,
                             double* S64_dev, int32_t stride, void* stream);
void vs_search_pending_free(vs_pending* pending);

/* ---- merge of per-shard results (all-gather + K3 merge).
 * S_in/I_in: G x nq x k (device), each list sorted best-first, element (g, q, j) at index
 * ((g * nq + q) * k + j) * in_stride (1 = separate arrays; 2 = one interleaved array of (score bits,
 * id) pairs, S_in = its base, I_in = base + 8 bytes: what one all-gather of packed pairs yields);
 * output nq x k best-first under (score desc | asc for L2, id asc).  D_out is S_out rounded to
 * fp32 (may be NULL). */
int vs_merge_shards_device(int metric, const double* S_in, const int64_t* I_in, int32_t in_stride, int G,
                           int64_t nq, int32_t k, double* S_out, int64_t* I_out, float* D_out, void* stream);

/* ---- the int8 / native MFMA screens' threshold seed, exposed for verification: for each of nq
 * queries, the rank-th largest of its M sampled maxima (device fp32 [nq][M]) as a starting key
 * (ordered fp32 << 32) in thr_dev[q] (device u64 [nq]); 0 when M < rank.  M <= 8192, rank >= 1. */
int vs_seed_select_device(int device, const float* maxima_dev, int32_t M, int64_t nq, int32_t rank,
                          uint64_t* thr_dev, void* stream);

/* ---- reconstruct (index.reconstruct, utils/vector_store.py:207) */
int vs_reconstruct(vs_index* index, int64_t id, float* out);
int vs_reconstruct_n(vs_index* index, int64_t i0, int64_t n, float* out); /* host n x d */

/* ---- persistence (faiss.read_index / faiss.write_index payloads, utils/vector_store.py:249, :234;
 * SURVEY.md §8 f3).  The host layer parses / writes the 45-byte IxFI/IxF2 header; these move the
 * row-major fp32 payload between the file and HBM through pinned double buffers (file reads and
 * writes overlap the PCIe copies and the pack / unpack kernels).
 * vs_add_from_file appends rows [0, n) of the payload at byte_offset (== index.add of them).
 * vs_write_rows_to_file writes stored rows [i0, i0+n) at byte_offset of `path` (created if absent,
 * never truncated): a full rewrite, or an append of the rows added since the last save. */
int vs_add_from_file(vs_index* index, const char* path, int64_t byte_offset, int64_t n);
int vs_write_rows_to_file(vs_index* index, const char* path, int64_t byte_offset, int64_t i0, int64_t n);

/* ---- screen selection (no reference counterpart: faiss IndexFlat has one exact scan).
 * VS_SCREEN_NATIVE (default): batches screen the stored rows (bf16/f16 MFMA, or the fp32 GEMV).
 * VS_SCREEN_I8: the index keeps an int8 copy of its rows (per-row scale, +1 byte per element,
 * built from the stored values now and on every add) and batches of > 8 queries with k <= 1024
 * screen it with int8 MFMAs under a proven per-row error bound; an adaptive exact refine then
 * scores every candidate the bound cannot exclude.  Results are identical to the native path
 * (same exact ids and scores); queries the certificate rejects are re-searched natively.
 * Both metrics: L2 keys bound the transformed score 2 <x, q> - ||x||^2 from above (the fp32 row
 * norm and its rounding inside the margin), and the refine compares canonical distances. */
int vs_set_screen(vs_index* index, int screen);
int vs_screen(const vs_index* index);

/* ---- introspection */
int64_t vs_ntotal(const vs_index* index);
int vs_dim(const vs_index* index);
int vs_metric(const vs_index* index);
int vs_dtype(const vs_index* index);
int vs_device(const vs_index* index);
const char* vs_last_error(void);
const char* vs_version(void);

/* ---- measurement hooks (bench.py): HIP events around the dominant screen kernel, recorded on
 * the stream it is launched on.  vs_timing_fetch synchronises those events and returns up to
 * `cap` per-launch durations (ms), oldest first, then clears them. */
int vs_set_timing(vs_index* index, int enable);
/* Calls of 1-2 queries with k <= 64 over an index of at most 65536 rows and at most `bytes` stored
 * bytes (rows x padded d x element size; default 192 MiB) skip the screen: one launch scores every
 * row exactly and selects the top-k (the full scan of vs_search_device_exact's last tier, run
 * first) -- the product's single-query call on a photo library, BASELINE cfg1.  0 = always screen
 * (tests of the screen kernels).  Results are the same bits either way. */
int vs_set_scan_limit(vs_index* index, int64_t bytes);
/* One launch of the main screen kernel (screen = VS_SCREEN_I8: the int8 direct screen; NATIVE: the
 * bf16 / f16 direct screen) over the whole index for 9..256 device queries, every query's threshold
 * at +inf (the bound test passes nothing: the K loop + epilogue test, no survivors); zero_queries
 * zeroes the packed query tile first, so one MFMA operand is all zeros.  Five launches back to
 * back; *ms = the fastest one's duration (HIP events on `stream`, synchronised).  bench.py runs both forms in the same process as the timed
 * steps: the box's own zero / real operand pair behind the power note of its roofline. */
int vs_screen_probe(vs_index* index, const float* q_dev, int64_t nq, int32_t screen, int32_t zero_queries,
                    void* stream, float* ms);
/* Diagnostic forms of the direct screen's loop (csrc/vs_k1probe.hip; DESIGN §5 "Where K1 int8's time
 * goes"), over the whole index like vs_screen_probe (thresholds at +inf, 9..256 device queries,
 * zero_queries as there).  screen = VS_SCREEN_I8 (inner-product int8 direct screen; variants
 * LOADS, LDS, MFMA, FULL, FULL_MS, FULL_PRIO, FULL_MS_PRIO) or VS_SCREEN_NATIVE (bf16 direct
 * screen; LOADS, MFMA, FULL).  `reps` launches back to back, each between its own HIP events:
 * ms[r] = launch r's duration; stamps[(r * G + b) * 4 + {0,1,2,3}] = workgroup b's s_memtime at the
 * loop's start and end, and its s_memrealtime (100 MHz) at the same points (host array of
 * reps * 256 * 4); *G_out = the launch's workgroups.  Synchronises. */
/* The K-step schedule of the int8 inner-product direct screen (K1), process-wide: 0 = one barrier at
 * the head of every K-step; 1 (default) = the mid-step barrier.  The same keys,
 * survivors and results under either schedule. */
int vs_set_k1_schedule(int32_t schedule);
int vs_k1_schedule(void);
enum {
    VS_K1P_LOADS = 0,        /* corpus loads + query LDS-DMAs + the per-K-step barriers */
    VS_K1P_LDS = 1,          /* + the query-fragment LDS reads */
    VS_K1P_MFMA = 2,         /* + the MFMAs (no tile epilogue) */
    VS_K1P_FULL = 3,         /* the whole loop with the epilogue's bound test (the product's schedule) */
    VS_K1P_FULL_MS = 4,      /* the same under the mid-step-barrier schedule */
    VS_K1P_FULL_PRIO = 5,    /* FULL with static priority 1 for waves 4-7 */
    VS_K1P_FULL_MS_PRIO = 6  /* FULL_MS with static priority 1 for waves 4-7 */
};
int vs_k1_probe(vs_index* index, const float* q_dev, int64_t nq, int32_t screen, int32_t variant,
                int32_t zero_queries, int32_t reps, void* stream, float* ms, unsigned long long* stamps,
                int32_t* G_out);
int vs_timing_fetch(vs_index* index, float* ms, int cap, int* kernel_kind);
int64_t vs_uncertified_count(vs_index* index);   /* first-pass certificate failures; synchronises */
/* queries answered by the exact full scan (no bounded screen could certify them; see
 * vs_search_device_exact); synchronises */
int64_t vs_full_scan_count(vs_index* index);
/* pinned host bytes the index holds for vs_search's query / result staging (all contexts); each
 * context stages at most 8 MiB and loops over query chunks beyond that */
int64_t vs_host_staging_bytes(vs_index* index);
/* HBM bytes the screen copies hold beyond the stored rows (VS_SCREEN_I8: int8 codes, per-row scale |
 * error norm); 0 for native screens */
int64_t vs_screen_copy_bytes(vs_index* index);
/* the screen's state, up to `cap` doubles: [0] screen, [1] group residuals in use, [2] groups coded
 * against a mean, [3] max ||mu_g||, [4] max ||x_hat|| of the int8 codes, [5] max row error norm,
 * [6] int8 union log2 depth, [7] searches still routed to the native screen, [8] native seed log2
 * depth (the screen-health feedback described at vs_search_device_exact); synchronises */
#define VS_SCREEN_STATE_N 9
int vs_screen_state(vs_index* index, double* out, int cap);

/* ==== multi-device flat index (one process, several GPUs; SURVEY.md §8 b/e) =================
 * The reference holds ONE index in ONE process (main.py:59-68 -> utils/vector_store.py:72-81); this
 * handle keeps that contract over G devices.  Rows are dealt in chunks of 2^16 consecutive ids
 * (chunk j on dev_ids[j mod G]), so ids stay insertion order 0..ntotal-1 under incremental and bulk
 * adds.  vs_multi_search runs every shard's exact search concurrently (one host worker + stream per
 * device), maps local ids to global ids on each device, copies the per-shard (fp64 score, id) lists
 * to dev_ids[0] over xGMI peer copies and merges them there (vs_merge_shards_device's kernel):
 * results equal a single index over all rows.  Devices may repeat (several shards on one GPU).
 * Calls on one handle are serialised. */
typedef struct vs_multi vs_multi;

int vs_multi_create(int d, int metric, int dtype, int n_dev, const int* dev_ids, vs_multi** out);
void vs_multi_destroy(vs_multi* m);
int vs_multi_add(vs_multi* m, const float* x, int64_t n);                           /* host rows */
int vs_multi_add_from_file(vs_multi* m, const char* path, int64_t byte_offset, int64_t n);
int vs_multi_write_rows_to_file(vs_multi* m, const char* path, int64_t byte_offset, int64_t i0, int64_t n);
int vs_multi_search(vs_multi* m, const float* q, int64_t nq, int32_t k, float* D, int64_t* I);
int vs_multi_reconstruct_n(vs_multi* m, int64_t i0, int64_t n, float* out);
int vs_multi_reset(vs_multi* m);
int vs_multi_set_screen(vs_multi* m, int screen);
int64_t vs_multi_ntotal(const vs_multi* m);
int vs_multi_ndev(const vs_multi* m);
int64_t vs_multi_shard_rows(const vs_multi* m, int shard);

/* ==== IVF-Flat (BASELINE cfg5) ===========================================
 * Not a reference call site: the reference's VectorStore offers flat and HNSW only
 * (utils/vector_store.py:51-53, 72-81).  This is the faiss IndexIVFFlat surface (faiss-cpu,
 * requirements.txt:5): IndexIVFFlat(quantizer, d, nlist, metric) -> vs_ivf_create,
 * .train -> vs_ivf_set_centroids (k-means runs in the Python layer over vs_ivf_assign),
 * .add -> vs_ivf_add, .search with .nprobe -> vs_ivf_search, .reconstruct -> vs_ivf_reconstruct.
 * Semantics (made exact, oracle/ivf_oracle.py): rows go to their exact best centroid (ties ->
 * lower list id) by its stored (dtype-rounded) values; a query probes its exact top-nprobe centroids and gets the exact top-k of the
 * rows of those lists (canonical fp64 score, ties -> lower id; -1 / worst-score padding).
 * Ids are insertion order 0..ntotal-1, as for the flat index.  Searches on one handle are
 * serialised; add/reset take an exclusive lock. */
typedef struct vs_ivf vs_ivf;

int vs_ivf_create(int d, int nlist, int metric, int dtype, int device, vs_ivf** out);
void vs_ivf_destroy(vs_ivf* ivf);
int vs_ivf_set_centroids(vs_ivf* ivf, const float* c);        /* host nlist x d; only while empty */
int vs_ivf_get_centroids(vs_ivf* ivf, float* out);            /* host nlist x d, values as stored */
int vs_ivf_is_trained(const vs_ivf* ivf);
int vs_ivf_assign(vs_ivf* ivf, const float* x, int64_t n, int64_t* lists); /* host; by the rows' dtype-rounded values */
int vs_ivf_add(vs_ivf* ivf, const float* x, int64_t n);       /* host fp32 n x d */
int vs_ivf_add_device(vs_ivf* ivf, const float* x_dev, int64_t n, void* stream); /* device fp32 n x d */
int vs_ivf_add_synthetic(vs_ivf* ivf, uint64_t seed, int64_t global_row0, int64_t n, int normalize);
/* size the HBM page pool for n more rows at once (chunked adds otherwise grow it by device copy,
 * which needs the old and the new pool side by side) */
int vs_ivf_reserve(vs_ivf* ivf, int64_t n);
int vs_ivf_search(vs_ivf* ivf, const float* q, int64_t nq, int32_t k, int32_t nprobe, float* D, int64_t* I);
/* device q/D/I/S64 (D, S64 may be NULL); host-synchronising (the probe -> work-item step). */
int vs_ivf_search_device(vs_ivf* ivf, const float* q_dev, int64_t nq, int32_t k, int32_t nprobe, float* D_dev,
                         int64_t* I_dev, double* S64_dev, void* stream);
int vs_ivf_reconstruct(vs_ivf* ivf, int64_t id, float* out);
int vs_ivf_list_sizes(vs_ivf* ivf, int64_t* out);             /* nlist entries */
int vs_ivf_reset(vs_ivf* ivf);                                /* drop rows, keep centroids */
int64_t vs_ivf_ntotal(const vs_ivf* ivf);
int vs_ivf_nlist(const vs_ivf* ivf);
/* bench: HIP events around the list-scan kernels of each search (same contract as vs_timing_fetch);
 * bytes_scanned (may be NULL) receives the algorithmic bytes those scans read, per search. */
int vs_ivf_set_timing(vs_ivf* ivf, int enable);
int vs_ivf_timing_fetch(vs_ivf* ivf, float* ms, double* bytes_scanned, int cap);
/* List-scan kernels (results are identical either way): VS_IVF_SCAN_AUTO (default) scans a list
 * probed by many queries with the MFMA screen over its pages (bf16/f16, once per 256 queries) when
 * a cost model says it beats re-reading it per 8 queries with the GEMV scan; _GEMV never does;
 * _MFMA does for every list probed by > 1 query (tests).  vs_ivf_last_search_stats reports the
 * first pass of the last search: its MFMA list scans, the queries its certificate rejected
 * (re-searched together, deeper) and the page bytes the MFMA and the GEMV scans read, re-reads
 * included (bytes_read[0], [1]); any pointer may be NULL. */
#define VS_IVF_SCAN_AUTO 0
#define VS_IVF_SCAN_GEMV 1
#define VS_IVF_SCAN_MFMA 2
int vs_ivf_set_scan(vs_ivf* ivf, int mode);
/* Query tiles of the MFMA list scans' first pass (results are identical either way):
 * VS_IVF_QTILE_SPLIT (default) packs (hi, lo) parts of each query (128 queries a tile, two MFMA
 * columns per query); VS_IVF_QTILE_PLAIN packs each query once, rounded to the list dtype (256
 * queries a tile; lists probed by <= 64 queries take the narrow 64-column form), its ~2^8 x wider
 * rounding margin taken by the certificate, so more queries may need a re-search.  Re-search
 * rounds always pack split tiles; plain tiles need the direct form (padded dim a multiple of 128),
 * otherwise split tiles are used. */
#define VS_IVF_QTILE_PLAIN 0
#define VS_IVF_QTILE_SPLIT 1
int vs_ivf_set_query_tiles(vs_ivf* ivf, int mode);
int vs_ivf_last_search_stats(const vs_ivf* ivf, int* mfma_lists, int* uncertified, double* bytes_read);

/* ==== HNSW graph search ===================================================
 * Replaces the search of faiss.IndexHNSWFlat, which the reference builds for
 * index_type="hnsw" (utils/vector_store.py:73-78: IndexHNSWFlat(d, M, metric), hnsw.efSearch) and
 * searches at utils/vector_store.py:191.  A vs_hnsw is a graph in faiss's HNSW layout (the arrays
 * of an IHNf file: node levels, per-node offsets into the neighbour array, cumulative neighbour
 * counts per level, entry point, max level) over the rows of a flat vs_index (graph node i = row
 * i); the graph is copied to the index's device and validated (ids in range, neighbours present
 * on their level, offsets matching the levels); a later duplicate in a neighbour list is dropped,
 * which changes no search.  vs_hnsw_search runs faiss HNSW::search (greedy descent on the upper
 * levels, then efSearch-bounded best-first search on level 0; oracle/hnsw_oracle.py) on the GPU,
 * one workgroup per query, with the flat path's exact canonical scores as distances: D = scores
 * (IP) / squared distances (L2) best first, I = row ids, -1 padded.  The graph covers the first
 * n rows of the index: rows added behind it are not reachable (the caller searches them exactly
 * and merges); an index holding fewer than n rows is VS_ERR_ARG; max(ef_search, k) <= 2048. */
typedef struct vs_hnsw vs_hnsw;

int vs_hnsw_create(vs_index* index, int64_t n, const int32_t* levels, const uint64_t* offsets,
                   const int32_t* neighbors, const int32_t* cum_nneighbor_per_level, int32_t n_cum,
                   int32_t entry_point, int32_t max_level, vs_hnsw** out);
void vs_hnsw_destroy(vs_hnsw* graph);
int vs_hnsw_search(vs_hnsw* graph, const float* q, int64_t nq, int32_t k, int32_t ef_search, float* D,
                   int64_t* I);
int64_t vs_hnsw_ntotal(const vs_hnsw* graph);
/* Rewrite m neighbour slots (positions into the create call's neighbour array) and set the entry
 * point / top level: the batched insertion of faiss IndexHNSWFlat.add (utils/vector_store.py:164)
 * keeps ONE device graph laid out for the final node count -- nodes not inserted yet have empty
 * lists and no links to them, so they are unreachable -- and patches in each batch's new lists
 * and reverse links (photo_search_engine_amd/hnsw.py insert_rows).  Slots and ids are validated
 * as in vs_hnsw_create, and a patch must rewrite whole (node, level) lists -- every slot of each list
 * it touches -- each as distinct ids followed by -1s (VS_ERR_ARG otherwise, the graph unchanged). */
int vs_hnsw_patch(vs_hnsw* graph, int64_t m, const uint64_t* pos, const int32_t* val, int32_t entry_point,
                  int32_t max_level);

/* HNSW graph build: faiss HNSW::shrink_neighbor_list (the neighbour-selection heuristic
 * IndexHNSWFlat.add applies to a new node's candidates and to a full list receiving a reverse link,
 * utils/vector_store.py:164) for m nodes at once on the GPU.  nodes[i] = row id of node i;
 * cand[i * C ..] = its distinct candidate row ids, -1 padded at the end; with fewer than W
 * candidates all are kept (faiss returns early below max_size), else candidates are taken in
 * ascending (distance, id) order and one is kept unless an already kept neighbour is strictly closer
 * to it than the node is, up to W.  Distances are the flat path's canonical fp64 scores (IP: -score).
 * out[i * W ..] = kept ids best first, -1 padded.  C <= 2048, W <= 1024; ids are validated. */
int vs_hnsw_prune(vs_index* index, int64_t m, const int64_t* nodes, const int32_t* cand, int32_t C, int32_t W,
                  int32_t* out);

#ifdef __cplusplus
}
#endif

#endif /* VS_H_ */
