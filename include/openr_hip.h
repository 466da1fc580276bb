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
} orh_spf_request;

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
int orh_set_spf_mode(orh_ctx* ctx, int mode);
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
typedef struct orh_spf_info {
  int32_t variant;     /* ORH_VARIANT_* of the distance phase */
  uint32_t rows;       /* distance rows searched (sources + neighbour rows) */
  uint32_t mask_bits;  /* MS-BFS: sources per workgroup (32 or 16), else 0 */
  uint32_t hop_nodes;  /* first-hop phase: nodes per thread over u8 level rows
                          (16 or 4), 1 for the u32-row kernel, 0 when fused */
  uint32_t hop_split;  /* first-hop phase: workgroups per source */
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
/* device-to-device copy on the context stream, completed before return (hands
 * rows to a caller-owned buffer, e.g. the RCCL all-gather of a central RIB) */
int orh_memcpy_d2d(orh_ctx* ctx, void* d_dst, const void* d_src, size_t bytes);

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
int orh_graph_info(const orh_graph* g, uint32_t* n_nodes, uint32_t* n_edges);
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

/* ---- route selection (getMinCostNodes + getNextHopsWithMetric) --------- */
/* For each prefix p with candidate advertisers h/d_adv[adv_ptr[p]..adv_ptr[p+1])
 * (node ids, already best-route-selected, Decision.cpp:794-822), over the
 * SPF row of `me` (d_dist/d_nh as produced by orh_spf_run for one source):
 *   d_min[p]            = min over advertisers of dist (ORH_UNREACHABLE if none)
 *   d_nh_out[p*W + k]   = OR of nh masks of the argmin advertisers
 * Asynchronous on the context stream; all pointers are device pointers. */
int orh_route_select(orh_ctx* ctx, uint32_t n_prefix, const uint32_t* d_adv_ptr,
                     const uint32_t* d_adv, const uint32_t* d_dist, const uint32_t* d_nh,
                     uint32_t words, uint32_t* d_min, uint32_t* d_nh_out);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_HIP_H_ */
