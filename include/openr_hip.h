/*
 * libopenr_hip — C ABI of the MI355X SPF / route-computation engine for the
 * OpenR Decision module.
 *
 * This is the device boundary that sits under the reference's C++ class API
 * (there is no C ABI or plugin in the reference):
 *
 *   LinkState::getSpfResult(node, useLinkMetric)   openr/decision/LinkState.h:271-272
 *   LinkState::runSpf(src, useLinkMetric, ignore)  openr/decision/LinkState.cpp:808-882
 *   LinkState::getKthPaths(src, dst, k) (k = 2 re-runs SPF with links ignored)
 *                                                  openr/decision/LinkState.cpp:762-791
 *   SpfSolver::SpfSolverImpl::getMinCostNodes / getNextHopsWithMetric
 *                                                  openr/decision/Decision.cpp:1152-1228
 *   LinkState::updateAdjacencyDatabase / deleteAdjacencyDatabase /
 *   decrementHolds (sources of the CSR-mirror deltas)
 *                                                  openr/decision/LinkState.h:327-337
 *
 * The host library (openr_amd/csrc/host, C++) keeps the reference's graph
 * store semantics and mirrors each area's LinkState into an orh_graph; every
 * SPF the Decision path runs is an orh_spf_* call.
 *
 * Conventions
 *  - Plain pointers and sizes only; no exceptions cross the ABI.
 *  - Every function returns ORH_OK (0) or a negative ORH_E_* code; the
 *    message of the last failure on a context is orh_last_error(ctx).
 *  - A context is bound to one HIP device and one HIP stream and is
 *    single-thread-affine (the reference runs Decision on one thread,
 *    Decision.cpp:1453-1495). Use one context per GPU.
 *  - "d_" pointers are device pointers (from orh_device_alloc or
 *    hipMalloc on the context's device); "h_" pointers are host pointers.
 *
 * SPF result layout (per source s of a batch, N = graph node count):
 *   dist[s*N + v]  uint32  shortest-path metric src->v, ORH_UNREACHABLE if
 *                          v is not reachable (absent from the reference's
 *                          SpfResult)
 *   nh[(s*N + v)*W + k]    ECMP first-hop set of v as a bitmask over the
 *                          source's distinct neighbour nodes in ascending
 *                          node-id order (orh_graph_neighbors); W words of
 *                          32 bits (orh_spf_words). Equals the reference's
 *                          NodeSpfResult::nextHops() (LinkState.h:256).
 */
#ifndef OPENR_HIP_H_
#define OPENR_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORH_OK 0
#define ORH_E_INVALID (-1)     /* bad argument / shape */
#define ORH_E_DEVICE (-2)      /* HIP runtime error */
#define ORH_E_UNSUPPORTED (-3) /* input outside what the kernels implement */
#define ORH_E_NOMEM (-4)       /* device allocation failed */
#define ORH_E_STATE (-5)       /* call out of order (e.g. no graph loaded) */

#define ORH_UNREACHABLE 0xFFFFFFFFu

/* bits of orh_csr.meta[e] */
#define ORH_META_LINK_MASK 0x3FFFFFFFu /* link id of the CSR entry */
#define ORH_META_COL_OVERLOADED 0x40000000u /* neighbour node is overloaded */
#define ORH_META_DOWN 0x80000000u      /* !Link::isUp() (LinkState.cpp:233-236) */
/* a free CSR slot (row capacity not in use): down, link id all ones; its
 * col is ignored (the library keeps it at the row's own node) */
#define ORH_META_EMPTY (ORH_META_DOWN | ORH_META_LINK_MASK)

typedef struct orh_ctx orh_ctx;
typedef struct orh_graph orh_graph;

/* One area's adjacency database as a directed CSR (2 entries per
 * bidirectional Link). Metrics are the effective HoldableValue values. */
typedef struct orh_csr {
  uint32_t n_nodes;
  uint32_t n_edges;
  uint32_t n_links;
  const uint32_t* row_ptr;        /* [n_nodes+1] */
  const uint32_t* col;            /* [n_edges] neighbour node id */
  const uint32_t* w_out;          /* [n_edges] Link::getMetricFromNode(row) */
  const uint32_t* w_in;           /* [n_edges] Link::getMetricFromNode(col) */
  const uint32_t* meta;           /* [n_edges] ORH_META_* bits | link id */
  const uint8_t* node_overloaded; /* [n_nodes] LinkState::isNodeOverloaded */
  /* [n_nodes] rank of each node's name in byte order (the reference's
   * DijkstraQ tie order, LinkState.h:488-498); NULL: node id order */
  const uint32_t* name_rank;
} orh_csr;

typedef struct orh_spf_request {
  const uint32_t* h_srcs; /* [n_src] source node ids */
  uint32_t n_src;
  /* optional per-source ignored links (runSpf's linksToIgnore), CSR over
   * sources: links of source i are h_ignore_links[h_ignore_ptr[i] ..
   * h_ignore_ptr[i+1]); both NULL for none */
  const uint32_t* h_ignore_ptr;
  const uint32_t* h_ignore_links;
  int32_t use_link_metric; /* 0: hop count (useLinkMetric = false) */
  /* ORH_SPF_* flags; zero-initialise the request (0 = the default run) */
  uint32_t flags;
} orh_spf_request;

/* orh_spf_request.flags: a multi-source sweep's second phase (level rows ->
 * distance rows, first hops) runs on the context's second stream, so the
 * context stream takes the next sweep's search at once. The rows are complete
 * for work issued on the context after the next orh_sync / orh_memcpy_* /
 * orh_row_digest / SPF, KSP2, what-if or route call (each joins the deferred
 * work first); other readers wait for orh_sync. */
#define ORH_SPF_DEFER_HOPS 1u

typedef struct orh_counters {
  uint64_t spf_runs;      /* fb303 decision.spf_runs equivalent */
  uint64_t spf_launches;  /* kernel launches */
  double last_kernel_ms;  /* device time of the last SPF launch (HIP events) */
  double total_kernel_ms; /* accumulated device time of SPF launches */
} orh_counters;

/* ---- context --------------------------------------------------------- */
int orh_device_count(int* out_count);
int orh_create(int device, uint32_t flags, orh_ctx** out_ctx);
int orh_destroy(orh_ctx* ctx);
const char* orh_last_error(const orh_ctx* ctx);
int orh_sync(orh_ctx* ctx);
int orh_get_counters(const orh_ctx* ctx, orh_counters* out);
int orh_reset_counters(orh_ctx* ctx);
/* distance-kernel selection for later orh_spf_run calls on this context:
 *   ORH_SPF_AUTO (default)  multi-source BFS when every live link has one
 *                           metric and the batch has no ignore sets, else the
 *                           LDS-resident per-source kernels, else the HBM
 *                           frontier kernel (graphs beyond LDS, e.g. 50k nodes)
 *   ORH_SPF_PER_SOURCE      per-source kernels only (LDS, HBM when too large)
 *   ORH_SPF_GLOBAL          the HBM frontier kernel for every graph, with the
 *                           first hops fused into the search when every
 *                           source has <= 32 distinct neighbours (AUTO fuses
 *                           too when the two-phase scheme would need extra
 *                           neighbour rows: what-if and KSP2 batches)
 *   ORH_SPF_GLOBAL_TWO_PHASE the HBM frontier kernel, never fused
 * All modes produce identical results; the choice is performance only. */
#define ORH_SPF_AUTO 0
#define ORH_SPF_PER_SOURCE 1
#define ORH_SPF_GLOBAL 2
#define ORH_SPF_GLOBAL_TWO_PHASE 3
/* the exact kernel (reference extraction order) for every graph; it runs
 * anyway for graphs with a zero-metric live link */
#define ORH_SPF_EXACT 4
int orh_set_spf_mode(orh_ctx* ctx, int mode);
/* what-if repair for ignore-set batches (runSpf(src, m, linksToIgnore)):
 * the batch's distinct sources get plain SPFs and every request's row is
 * derived from its source's row (only nodes below a tight ignored link are
 * recomputed; results are identical). ORH_REPAIR_AUTO (default) uses it when
 * sources repeat (distinct <= half the requests) and every ignore set has at
 * most 8 links; ORH_REPAIR_ALWAYS for every batch it can take; env
 * ORH_WHATIF_REPAIR sets the initial mode */
#define ORH_REPAIR_OFF 0
#define ORH_REPAIR_AUTO 1
#define ORH_REPAIR_ALWAYS 2
int orh_set_repair_mode(orh_ctx* ctx, int mode);
/* kernel plan of the last orh_spf_run on this context (tests and profiling
 * assert which variant ran; results never depend on it) */
#define ORH_VARIANT_MSBFS 1     /* bit-parallel multi-source BFS */
#define ORH_VARIANT_BFS8 2      /* per-source BFS, u8 / u16 / u32 levels in LDS */
#define ORH_VARIANT_BFS16 3
#define ORH_VARIANT_BFS32 4
#define ORH_VARIANT_DIST16 5    /* per-source level-synchronous Dijkstra in LDS */
#define ORH_VARIANT_DIST32 6
#define ORH_VARIANT_GLOBAL 7    /* HBM frontier kernel, two-phase */
#define ORH_VARIANT_GLOBAL_NH 8 /* HBM frontier kernel with fused first hops */
#define ORH_VARIANT_EXACT 9     /* exact Dijkstra in the reference's extraction order */
#define ORH_VARIANT_BFS_NH 10   /* BFS with fused first hops, one workgroup per source */
#define ORH_VARIANT_REPAIR 11   /* ignore-set batch repaired from its sources' plain rows
                                   (batch_sources = distinct sources searched) */
#define ORH_VARIANT_LDS_NH 12   /* general metrics, {dist, first hops} labels in LDS,
                                   first hops fused, one workgroup per source */
#define ORH_VARIANT_WMS 13      /* general metrics, many sources: 4-source Bellman-Ford
                                   batches in LDS, then the first-hop phase */
typedef struct orh_spf_info {
  int32_t variant;     /* ORH_VARIANT_* of the distance phase */
  uint32_t rows;       /* distance rows searched (sources + neighbour rows) */
  uint32_t mask_bits;  /* MS-BFS: source-mask width (64, 32 or 16), else 0 */
  uint32_t hop_nodes;  /* first-hop phase: nodes per thread over u8 level rows
                          (16 or 4), 1 for the u32-row kernel, 0 when fused */
  uint32_t hop_split;  /* first-hop phase: workgroups per source */
  uint32_t batch_sources; /* MS-BFS: sources per workgroup (<= mask_bits), else 0 */
  uint32_t ms_threads;    /* MS-BFS: threads per workgroup (1024: the latency plan), else 0 */
  uint32_t ms_skip;       /* MS-BFS: interval skip on (latency plan or ORH_MS_SKIP=1) */
  uint32_t ms_direct;     /* MS-BFS / WMS: the node layout kept the host order (MS-BFS: rows
                             written by the search kernel, no finalize pass) */
} orh_spf_info;
int orh_last_spf_info(const orh_ctx* ctx, orh_spf_info* out);
/* device time (HIP events on the context stream) of the last orh_spf_run;
 * waits for that launch to finish */
int orh_last_spf_ms(orh_ctx* ctx, double* ms_out);
/* the same split by phase: distance rows, then first-hop masks */
int orh_last_spf_phase_ms(orh_ctx* ctx, double* dist_ms_out, double* hop_ms_out);
/* device memory helpers for callers without their own allocator */
int orh_device_alloc(orh_ctx* ctx, size_t bytes, void** d_out);
int orh_device_free(orh_ctx* ctx, void* d_ptr);
int orh_memcpy_d2h(orh_ctx* ctx, void* h_dst, const void* d_src, size_t bytes);
int orh_memcpy_h2d(orh_ctx* ctx, void* d_dst, const void* h_src, size_t bytes);
/* device-to-device copy on the context stream, completed before return (hands
 * rows to a caller-owned buffer, e.g. the RCCL all-gather of a central RIB) */
int orh_memcpy_d2d(orh_ctx* ctx, void* d_dst, const void* d_src, size_t bytes);

/* verification utility (no reference counterpart): per row r < n_rows of
 * dist [n_rows*n] / nh [n_rows*n*words], the 64-bit digest
 *   sum over v < n of mix(v, dist[r][v], nh[r][v][0..words))  (mod 2^64)
 * into d_out[r], asynchronously on the context stream. Equal rows give equal
 * digests whatever produced them, so a batch too large to copy out (the C4
 * what-if job: 262,144 rows x 50,000 nodes) is compared row by row with
 * another run or an independent checker (mix: tests/helpers.py row_digest). */
int orh_row_digest(orh_ctx* ctx, const uint32_t* d_dist, const uint32_t* d_nh, uint32_t words, uint32_t n,
                   uint32_t n_rows, uint64_t* d_out);

/* ---- graph mirror (one per area LinkState) ---------------------------- */
int orh_graph_create(orh_ctx* ctx, orh_graph** out_graph);
int orh_graph_destroy(orh_graph* g);
/* full upload of the CSR mirror (host arrays are copied) */
int orh_graph_load(orh_graph* g, const orh_csr* csr);
/* in-place attribute deltas: metric / up-down / overload changes that keep
 * the CSR structure (LinkState.cpp:640-710, :480-493, :500-514).
 * ORH_META_COL_OVERLOADED is maintained by the library from node_overloaded
 * (on load and on orh_graph_patch_nodes); callers' values of that bit are
 * ignored. */
int orh_graph_patch_edges(orh_graph* g, uint32_t n, const uint32_t* h_edge_idx,
                          const uint32_t* h_w_out, const uint32_t* h_w_in,
                          const uint32_t* h_meta);
int orh_graph_patch_nodes(orh_graph* g, uint32_t n, const uint32_t* h_node_idx,
                          const uint8_t* h_overloaded);
/* structural delta (links added / removed: LinkState::addLink / removeLink /
 * removeNode, LinkState.cpp:421-455, as updateAdjacencyDatabase and
 * deleteAdjacencyDatabase drive them, :564-738): row h_rows[i] becomes the
 * entries [h_ptr[i], h_ptr[i+1]) of h_col / h_w_out / h_w_in / h_meta, in
 * the caller's LinkSet order, and the rest of the row's capacity (its slot
 * count at load) turns into free slots. CSR entry indices stay stable, so
 * orh_graph_patch_edges keeps addressing entries by them. n_links is the new
 * link-id bound. Node ids and n_nodes are unchanged (a new node needs
 * orh_graph_load). ORH_E_UNSUPPORTED when a row outgrows its capacity:
 * reload. Only the changed rows' device records are re-uploaded. */
int orh_graph_apply_delta(orh_graph* g, uint32_t n_rows, const uint32_t* h_rows,
                          const uint32_t* h_ptr, const uint32_t* h_col, const uint32_t* h_w_out,
                          const uint32_t* h_w_in, const uint32_t* h_meta, uint32_t n_links);
int orh_graph_info(const orh_graph* g, uint32_t* n_nodes, uint32_t* n_edges);
/* device array of the graph's node overload flags (u8 [n_nodes]), valid
 * until the next orh_graph_load (route selection's drained-node filter) */
int orh_graph_device_flags(const orh_graph* g, const uint8_t** d_overloaded);
/* distinct neighbour node ids of src in ascending order (bit k of an nh
 * mask is h_out[k]); *n_out receives the count even if it exceeds cap */
int orh_graph_neighbors(const orh_graph* g, uint32_t src, uint32_t* h_out, uint32_t cap,
                        uint32_t* n_out);

/* ---- SPF -------------------------------------------------------------- */
/* nh words per node needed for a batch (max distinct-neighbour count / 32) */
int orh_spf_words(const orh_graph* g, const uint32_t* h_srcs, uint32_t n_src,
                  uint32_t* out_words);
/* asynchronous batched SPF on the context stream; d_dist [n_src*N] and
 * d_nh [n_src*N*words] are device buffers; words >= orh_spf_words(). */
int orh_spf_run(orh_graph* g, const orh_spf_request* req, uint32_t words, uint32_t* d_dist,
                uint32_t* d_nh);
/* synchronous convenience form: results copied into host buffers */
int orh_spf_batch(orh_graph* g, const orh_spf_request* req, uint32_t words, uint32_t* h_dist,
                  uint32_t* h_nh);
/* orh_spf_batch into context-owned pinned host memory: *h_dist / *h_nh point
 * at n_src rows of dist / n_src * N * words masks, valid until the next call
 * on this context (no pageable bounce copy, no caller allocation) */
int orh_spf_batch_pinned(orh_graph* g, const orh_spf_request* req, uint32_t words,
                         const uint32_t** h_dist, const uint32_t** h_nh);

/* Exact SPF: LinkState::runSpf (LinkState.cpp:808-882) in the reference's own
 * extraction order, with 64-bit path metrics (LinkStateMetric = uint64_t,
 * LinkState.h:22). With a zero-metric live link the first hops of a node
 * depend on which equal-metric neighbour is extracted first; orh_spf_run then
 * runs this kernel itself (u32 distances). When path metrics can reach
 * 2^32 - 1, orh_spf_run returns ORH_E_UNSUPPORTED and this entry point is the
 * one to use. d_dist [n_src*N] u64 (~0 = unreachable), d_nh as in
 * orh_spf_run, d_rank [n_src*N] (nullable): extraction order of every node
 * (the order of NodeSpfResult::pathLinks' predecessors; ~0 = unreachable). */
int orh_spf_run_exact(orh_graph* g, const orh_spf_request* req, uint32_t words, uint64_t* d_dist,
                      uint32_t* d_nh, uint32_t* d_rank);
int orh_spf_batch_exact(orh_graph* g, const orh_spf_request* req, uint32_t words,
                        uint64_t* h_dist, uint32_t* h_nh, uint32_t* h_rank);
/* ORH_GRAPH_* properties of the loaded graph */
#define ORH_GRAPH_ZERO_METRIC 1u /* a live link has metric 0 */
#define ORH_GRAPH_WIDE_METRIC 2u /* link-metric path sums can reach 2^32 - 1 */
int orh_graph_flags(const orh_graph* g, uint32_t* flags);

/* ---- what-if jobs (batched link-failure SPFs) ---------------------------
 * runSpf(src, useLinkMetric, linksToIgnore) (LinkState.cpp:808-882) for many
 * (source, ignore set) requests over a fixed source set - the C4 shape,
 * "4,096 links x 64 sources" (SURVEY.md §8d). orh_whatif_create searches the
 * plain rows of its sources once; every orh_whatif_run derives its requests'
 * rows from them: a request's row is its source's row except below a tight
 * ignored link, where it is re-derived (results are bit-identical to a fresh
 * runSpf). A job is bound to the graph structure it was created on
 * (ORH_E_STATE after a delta or reload). Everything is asynchronous on the
 * context stream; one mask word per node (every source has <= 32 distinct
 * neighbours), no zero-metric links (ORH_E_UNSUPPORTED otherwise). */
typedef struct orh_whatif orh_whatif;
int orh_whatif_create(orh_graph* g, const uint32_t* h_srcs, uint32_t n_srcs, int32_t use_link_metric,
                      orh_whatif** out_job);
/* requests i < n_req: source h_srcs[h_src_idx[i]] of the job, ignored links
 * h_ignore_links[h_ignore_ptr[i] .. h_ignore_ptr[i+1]) (orh_csr link ids);
 * rows into d_dist [n_req*N] and d_nh [n_req*N] (one word per node). d_info
 * (nullable, [n_req]): ORH_WHATIF_TIER(x) = how the row was made, and
 * ORH_WHATIF_AFFECTED(x) = nodes re-derived (0: the source's row stands, or a full search).
 * Host arrays may be reused once the call returns. */
int orh_whatif_run(orh_whatif* job, uint32_t n_req, const uint32_t* h_src_idx, const uint32_t* h_ignore_ptr,
                   const uint32_t* h_ignore_links, uint32_t* d_dist, uint32_t* d_nh, uint32_t* d_info);
#define ORH_WHATIF_TIER(x) ((x) & 7u) /* 0 source row, 1/2 LDS repair, 3 global-slot repair, 4 full search
                                         (subtrees too large for LDS, up to ORH_WHATIF_FULL per run; every
                                         such request without slots) */
#define ORH_WHATIF_AFFECTED(x) ((x) >> 3)
/* job flags (orh_whatif_set_flags, before a run):
 * ORH_WHATIF_SHARE_BASE  a request whose source row stands (tier 0) is not
 *   copied into d_dist / d_nh: its row IS the job's base row of its source
 *   (orh_whatif_base_rows). A C4-shaped run then writes the repaired rows
 *   only (half the 105 GB). */
#define ORH_WHATIF_SHARE_BASE 1u
/* ORH_WHATIF_SEARCH_LARGE  requests whose re-derived set outgrows the small
 *   LDS tier (256 nodes) are searched in full (delta-stepping, one workgroup
 *   each, up to 256 per run; the rest take the global slots) instead of
 *   repaired in the large LDS tier and global slots after it: for a short
 *   job - one device's block of a split job - whose largest repairs are its
 *   critical path (C4 at 8 / 4 blocks: the slowest block 7.1 -> 4.7 / 9.3 ->
 *   6.8 ms); a long job overlaps its slot repairs with its later chunks and
 *   is faster without it (one C4 job 21.0 vs 27.2 ms) */
#define ORH_WHATIF_SEARCH_LARGE 2u
int orh_whatif_set_flags(orh_whatif* job, uint32_t flags);
/* the job's base rows: dist [m][N] and first-hop masks [m][N] (one word per
 * node) of its m sources, valid until the next orh_whatif_refresh / destroy */
int orh_whatif_base_rows(orh_whatif* job, const uint32_t** d_dist, const uint32_t** d_nh);
/* search the job's sources again on the graph as it is now (after topology
 * deltas; allocations are kept) - the next runs derive from these rows */
int orh_whatif_refresh(orh_whatif* job);
/* A run's few large repairs may still be in flight on the job's internal
 * second stream when later work is queued on the context stream; after
 * orh_whatif_flush every row of every run so far is complete in stream order
 * (a later run waits by itself before it overwrites rows of an earlier one). */
int orh_whatif_flush(orh_whatif* job);
/* device time from the job's creation (base searches) to the end of its last
 * run (flushes; HIP events; waits for that run) */
int orh_whatif_elapsed_ms(orh_whatif* job, double* ms_out);
int orh_whatif_destroy(orh_whatif* job);

/* ---- KSP2 (LinkState::getKthPaths, LinkState.cpp:762-791) --------------
 * For each dsts[i]: the k = 1 paths, traced (traceOnePath, :398-419) over
 * src's SPF with link metrics, then the k = 2 paths over a fresh SPF that
 * ignores every k = 1 link - all fresh SPFs of the call in batched launches.
 * pathLinks follow runSpf's insertion order: predecessors in extraction
 * order (metric, then name rank; the exact kernel's order with zero
 * metrics), parallel links in CSR row order (= the caller's LinkSet
 * iteration order, which orh_csr rows must follow for KSP2 parity).
 * Output words, per dst and k = 1, 2: n_paths, then per path its length
 * and its link ids (orh_csr link ids, src -> dst order). *n_words receives
 * the total; when it exceeds cap, nothing is written and ORH_E_INVALID is
 * returned (query with cap = 0 first). Replaces the reference's memoized
 * getKthPaths(src, dst, 1 / 2) pair for a batch of destinations. */
int orh_ksp2(orh_graph* g, uint32_t src, const uint32_t* dsts, uint32_t n_dst, uint32_t* out,
             size_t cap, size_t* n_words);

/* Device form for a batch of (src, dst) pairs (the C4 shape: 1,024 pairs):
 * the sources' SPFs, the k = 1 traces, the k = 2 searches (each pair's k = 1
 * links ignored) and the k = 2 traces all run on the device; only the paths
 * are copied back. *out_blocks points at n_pairs blocks of *block_words words
 * in context-owned pinned memory, valid until the next call on the context:
 *   [0] status: 0, or 1 = the pair outgrew the device trace's bounds (trace
 *       it with orh_ksp2 / on the host)
 *   [1] offset of the k = 2 section within the block
 *   [2..] k = 1 section, then the k = 2 section, each as in orh_ksp2
 * Graphs with zero-metric links or 64-bit path metrics: ORH_E_UNSUPPORTED
 * (orh_ksp2 follows the exact kernel's extraction order there). */
int orh_ksp2_batch(orh_graph* g, uint32_t n_pairs, const uint32_t* h_src, const uint32_t* h_dst,
                   const uint32_t** out_blocks, uint32_t* block_words);

/* ---- device prefix mirror (PrefixState) ------------------------------- */
/* Replaces the per-prefix PrefixEntries map PrefixState::prefixes() hands to
 * the route build (openr/decision/PrefixState.h:22-70, updatePrefix /
 * deletePrefix PrefixState.cpp:17-56). Prefix p is a dense id chosen by the
 * caller; its advertisements are an ordered list of orh_adv records (the
 * order only numbers them: route selection reports the best one by its
 * position). Node names and areas are caller-side ids. */
typedef struct orh_prefix_set orh_prefix_set;

typedef struct orh_adv {
  uint32_t name;        /* advertiser node name id */
  uint32_t meta;        /* area id (bits 0-7) | ORH_ADV_* flags */
  int32_t path_pref;    /* PrefixMetrics.path_preference */
  int32_t source_pref;  /* PrefixMetrics.source_preference */
  int32_t distance;     /* PrefixMetrics.distance */
} orh_adv;
#define ORH_ADV_AREA_MASK 0xFFu
#define ORH_ADV_SR_MPLS (1u << 8)     /* forwardingType == SR_MPLS */
#define ORH_ADV_KSP2 (1u << 9)        /* forwardingAlgorithm == KSP2_ED_ECMP */
#define ORH_ADV_BGP (1u << 10)        /* type == BGP */
#define ORH_ADV_MIN_NEXTHOP (1u << 11) /* minNexthop is set */
#define ORH_ADV_PREPEND (1u << 12)    /* prependLabel is set */
/* bits 13-31 of meta: the caller's id of the advertisement's PrefixEntry.tags
 * set (0: no tags; ORH_ADV_TAGSET_OVF: more distinct sets than ids, which
 * sends a policy-matched route to the host, orh_route_policy) */
#define ORH_ADV_TAGSET_SHIFT 13u
#define ORH_ADV_TAGSET_OVF 0x7FFFFu
#define ORH_PFX_V4 1u                 /* prefix_flags: an IPv4 prefix */

int orh_prefix_create(orh_ctx* ctx, orh_prefix_set** out);
int orh_prefix_destroy(orh_prefix_set* ps);
/* full upload: prefix p owns advs[adv_ptr[p] .. adv_ptr[p+1]) */
int orh_prefix_load(orh_prefix_set* ps, uint32_t n_prefix, const uint32_t* h_adv_ptr,
                    const orh_adv* h_advs, const uint8_t* h_prefix_flags);
/* incremental: prefix ids[i] gets advs[adv_ptr[i] .. adv_ptr[i+1]) (an empty
 * list withdraws it; ids beyond the current count grow the set) */
int orh_prefix_apply_delta(orh_prefix_set* ps, uint32_t n, const uint32_t* h_ids,
                           const uint32_t* h_adv_ptr, const orh_adv* h_advs,
                           const uint8_t* h_prefix_flags);
/* string order of the name and area ids (std::set<NodeAndArea> order, which
 * picks bestNodeArea, Decision.cpp:817 / Util.cpp:902-913) */
int orh_prefix_set_order(orh_prefix_set* ps, uint32_t n_names, const uint32_t* h_name_rank,
                         uint32_t n_areas, const uint32_t* h_area_rank);
int orh_prefix_info(const orh_prefix_set* ps, uint32_t* n_prefix, uint32_t* n_adv_live,
                    uint32_t* n_adv_pool);

/* ---- route selection (createRouteForPrefix -> getNextHopsWithMetric) --- */
/* One thread per prefix, for the solver's node `me`:
 *   drop advertisers unreachable in their own area   Decision.cpp:468-480
 *   best-route (max PrefixMetrics) or all-advertiser
 *   selection, bestNodeArea, drained-node filter     :794-862, Util.h:491-526
 *   forwarding type / algorithm                      Util.cpp:452-480
 *   getMinCostNodes per area (area ignored) and the
 *   cross-area min + first-hop mask OR               :1152-1228
 * status[p]: ORH_SEL_NONE (no route), ORH_SEL_ROUTE (metric[p] = shortest,
 * best[p] = position of bestNodeArea in p's list, mask[p] = per area the OR of
 * the argmin advertisers' first-hop masks, zero for areas above the minimum),
 * or ORH_SEL_HOST (a case the host path keeps: BGP metric vectors, SR_MPLS /
 * KSP2 forwarding, minNexthop, self-advertised, unknown area, > 255
 * advertisers). */
#define ORH_SEL_NONE 0
#define ORH_SEL_ROUTE 1
#define ORH_SEL_HOST 2
#define ORH_NO_NODE 0xFFFFFFFFu
#define ORH_SELECT_BEST_ROUTE 1u /* enable_best_route_selection */
#define ORH_SELECT_V4 2u         /* enable_v4 */

typedef struct orh_select_area {
  uint32_t present;            /* 0: the solver has no LinkState of this area id */
  const uint32_t* d_dist;      /* me's distance row (device), NULL: me not in this area */
  const uint32_t* d_nh;        /* me's first-hop rows [N][words] (device) */
  const uint8_t* d_overloaded; /* [N] node overload flags (device) */
  const uint32_t* d_name_node; /* [n_names] node id of each name id, ORH_NO_NODE if absent */
  uint32_t words;              /* mask words of this area */
  uint32_t word_off;           /* this area's first word in a prefix's mask */
} orh_select_area;

typedef struct orh_select_out {
  uint8_t* d_status;  /* [n_prefix] ORH_SEL_* */
  uint32_t* d_metric; /* [n_prefix] shortest metric */
  uint32_t* d_best;   /* [n_prefix] position of the best advertisement */
  uint32_t* d_mask;   /* [n_prefix][total_words] */
  uint32_t total_words;
} orh_select_out;

/* asynchronous on the context stream; the area table is copied */
int orh_route_select(orh_prefix_set* ps, uint32_t me_name, uint32_t flags, uint32_t n_areas,
                     const orh_select_area* h_areas, const orh_select_out* out);
/* the same for the prefix ids [pid_lo, pid_hi) only (a prefix shard of a
 * route build): out arrays are still indexed by prefix id
 * (sized for pid_hi), entries outside the range are not written */
int orh_route_select_range(orh_prefix_set* ps, uint32_t me_name, uint32_t flags, uint32_t n_areas,
                           const orh_select_area* h_areas, uint32_t pid_lo, uint32_t pid_hi,
                           const orh_select_out* out);
/* Keyed compare of two selection outputs of the same prefix set (the device
 * half of DecisionRouteDb::calculateUpdate, Decision.cpp:108-143): prefix p
 * < n_prefix whose record (status, metric, best, mask words) differs from
 * prev's, or with p >= prev_n, is appended to d_changed as one packed record
 * of 4 + total_words u32 {p, status, metric, best, mask...}; *d_count
 * receives how many (d_changed must hold n_prefix records). Asynchronous on
 * the context stream. */
int orh_route_diff(orh_prefix_set* ps, uint32_t n_prefix, uint32_t prev_n, const orh_select_out* cur,
                   const orh_select_out* prev, uint32_t* d_changed, uint32_t* d_count);
/* device time of the last orh_route_select kernel (HIP events; waits for it) */
int orh_last_select_ms(orh_prefix_set* ps, double* ms_out);

/* ---- RibPolicy over a route selection (RibPolicy::applyPolicy) --------- */
/* Replaces the per-route loop of RibPolicy::applyPolicy (RibPolicy.cpp
 * :229-247) with RibPolicyStatement::match / applyAction (:73-158) for the
 * routes a selection made (status ORH_SEL_ROUTE). A route's nexthops are the
 * tight links behind the set bits of its first-hop mask, and a set_weight
 * action gives every nexthop of one bit (one neighbour, one area) the same
 * weight, so statement s is a bitmask keep[s] of the mask bits whose weight
 * is > 0 (neighbour weight, else area weight, else default weight). Per
 * route, the statements in order: s matches when every non-empty matcher
 * matches (tags: the best advertisement's tag set meets s's tag set; prefixes:
 * the route's prefix id is in s's list) and at least one is non-empty; a
 * matching s whose keep[s] misses the route's mask drops every nexthop, so the
 * route stays as it was and counts as invalidated (:146-152), and the next
 * statement is tried; the first matching s that keeps a nexthop applies.
 * out[p] = that s, ORH_POL_NONE, or ORH_POL_HOST (tag set id overflow: the
 * host applies the policy). *d_invalidated receives the invalidated count.
 * Asynchronous on the context stream; the tables are copied. */
#define ORH_POL_NONE 0xFFu
#define ORH_POL_HOST 0xFEu
#define ORH_POL_MAX_STMTS 32u
typedef struct orh_policy {
  uint32_t n_stmts;                /* <= ORH_POL_MAX_STMTS */
  uint32_t stmt_tags;              /* bit s: statement s has a non-empty tag matcher */
  uint32_t stmt_prefixes;          /* bit s: statement s has a non-empty prefix matcher */
  uint32_t n_tagsets;              /* tag set ids 0 .. n_tagsets - 1 */
  const uint32_t* h_tagset_stmts;  /* [n_tagsets] bit s: the set meets statement s's tags */
  uint32_t n_pfx;                  /* prefixes named by any prefix matcher */
  const uint32_t* h_pfx_id;        /* [n_pfx] prefix ids, ascending */
  const uint32_t* h_pfx_stmts;     /* [n_pfx] bit s: statement s names the prefix */
  const uint32_t* h_keep;          /* [n_stmts][total_words] */
  uint32_t total_words;            /* the selection's mask words */
} orh_policy;
int orh_route_policy(orh_prefix_set* ps, uint32_t n_prefix, const orh_select_out* sel,
                     const orh_policy* pol, uint8_t* d_out, uint32_t* d_invalidated);
/* the same for the prefix ids [pid_lo, pid_hi) only (a prefix shard): d_out
 * indexed by prefix id, *d_invalidated counts the range's routes */
int orh_route_policy_range(orh_prefix_set* ps, uint32_t pid_lo, uint32_t pid_hi, const orh_select_out* sel,
                           const orh_policy* pol, uint8_t* d_out, uint32_t* d_invalidated);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_HIP_H_ */
