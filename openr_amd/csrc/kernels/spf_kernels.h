// Internal interface between the C ABI (orh_api.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// Device edge record (uint2): x = col | flags, y = w_out.
// A continuation record is {overflow start | CONT, count}.
#define ORH_REC_COL_MASK 0x07FFFFFFu
#define ORH_REC_CONT 0x08000000u     // continuation into the overflow area
#define ORH_REC_ROW_OVL 0x10000000u  // the record's row node is overloaded
#define ORH_REC_SKIP 0x80000000u     // link down, or an empty ELL slot

namespace orh {

// phase 1: distance rows. Rows [0, n_out) are written to out_dist, rows
// [n_out, n_rows) (neighbour rows the first-hop phase needs) to scratch.
struct SpfArgs {
  uint32_t n_nodes;
  uint32_t n_out;
  uint32_t n_rows;
  const uint32_t* dev_of;     // multi-source BFS: [N] host id -> Cuthill-McKee id
  const uint32_t* host_of;    // multi-source BFS: [N] Cuthill-McKee id -> host id
  const uint32_t* order;      // [n_rows] multi-source batch order of the rows
  uint8_t* ms_lvl;            // multi-source BFS: node-major level bytes [batches][N][S]
  uint64_t* ms_log;           // multi-source BFS (u16 / u32 masks): arrival logs [batches][waves][J * 64 * S]
  // u16 LDS search (nullable): row r may stop once the nodes stop_nodes
  // [stop_ptr[r], stop_ptr[r + 1]) are final - rows that feed path traces to
  // those targets (KSP2) need no node beyond them
  const uint32_t* stop_ptr;
  const uint32_t* stop_nodes;
  uint32_t ms_pitch;          // multi-source BFS: frontier-array entries (> N)
  uint32_t ms_zero;           // multi-source BFS: index of the always-zero entry
  uint32_t ms_bw;             // multi-source BFS: layout bandwidth for the interval skip (0: no skip)
  uint32_t ms_width;          // multi-source BFS: sources per batch (<= mask bits)
  uint32_t ms_direct;         // multi-source BFS (u16 / u32 masks, host-order layout): the
                              // level assembly writes the rows itself (no ms_lvl, no finalize)
  const uint2* recs;       // ELL slots [N * K] then overflow records
  const uint32_t* link;    // per record: link id (ignore sets)
  const uint32_t* srcs;    // [n_rows]
  const uint32_t* ignore_ptr;  // [n_rows + 1], nullable
  const uint32_t* ignore_links;
  int32_t use_link_metric;
  uint32_t w0;  // the uniform metric (BFS variant)
  uint32_t lds_pend_off;
  uint32_t delta;  // HBM frontier kernel: near/far bucket width
  uint32_t* out_dist;
  uint32_t* scratch;
  uint64_t* diag;  // ORH_DIAG_STAMPS builds only
  // HBM kernel with fused first hops (kGlobalNh): per-row {dist, nh} labels,
  // the first-hop output rows, and the record -> neighbour-rank table
  unsigned long long* labels;  // [n_rows][N]
  uint32_t* out_nh;            // [n_out][N][words]
  uint32_t words;
  const uint16_t* rank_out;
  uint8_t* lvl_rows;  // multi-source BFS: u8 level row per row [n_rows][lvl_pitch]
  uint32_t lvl_pitch;  // N rounded up to 16
  // HBM kernel with fused first hops: rows whose flag is 0 are skipped (the
  // what-if repair's fallback searches only the rows it could not repair)
  const uint32_t* row_mask;  // [n_rows], nullable
  // HBM kernel with fused first hops: workgroup b searches row row_list[b]
  // while b < *row_count (else exits), with its labels in slot b (nullable:
  // workgroup b searches row b)
  const uint32_t* row_list;
  const uint32_t* row_count;
  // u16 LDS search (spf_lds16_kernel): workgroup b searches row row_order[b]
  // (nullable: row b), e.g. the longest searches first
  const uint32_t* row_order;
  // HBM kernel (kGlobalNh plan): distances only, u32 labels, out_nh unused
  int32_t dist_only;
  // u16 LDS search (launch_spf_lds16): [0] count, then the rows it left to
  // the HBM kernel (a distance that needs 17 bits)
  uint32_t* ovf_rows;
  // multi-source Bellman-Ford (kWms): per Cuthill-McKee node K in-link slots
  // {u | w(u -> v) << 16 | overloaded(u) << 31} (u = N: no link), and the
  // largest u16 label that proves its row fits 16 bits (0xFFFE - max metric)
  const uint32_t* wms_slots;
  uint32_t wms_limit;
  // 1: a wave owns a contiguous band of J 64-node chunks and a round sweeps it
  // forward then backward (else chunk j of wave w is j * waves + w, one pass)
  uint32_t wms_band;
  uint32_t recs_k;  // ELL width of `recs` (kernels launched from plans that do not know it)
};

// phase 2: first-hop masks of the requested rows from the distance rows of
// each source and of its neighbours
struct HopArgs {
  uint32_t n_nodes;
  uint32_t n_out;  // requested rows (= sources of this phase)
  uint32_t words;
  uint32_t ell_k;
  uint32_t tiles;  // node tiles per source
  uint32_t tile_split;  // level-row kernel: workgroups per source (tile phases)
  const uint2* recs;
  const uint32_t* link;
  const uint16_t* rank_out;  // per record: col's rank among the row node's distinct neighbours
  const uint8_t* overloaded;
  const uint32_t* srcs;
  const uint32_t* ignore_ptr;
  const uint32_t* ignore_links;
  int32_t use_link_metric;
  const uint32_t* nbr_ptr;  // [n_out + 1] into nbr_row
  const uint32_t* nbr_row;  // per (source, neighbour rank): row of that neighbour's distances
  const uint32_t* dist;
  const uint32_t* scratch;
  uint32_t* out_nh;
  // multi-source BFS plans: u8 level rows (255 unreached, 254 = read the u32
  // row) replace the u32 distance rows as the input; w0 = the uniform metric
  const uint8_t* lvl_rows;
  uint32_t lvl_pitch;
  uint32_t w0;
  // level-row kernel block order: 0 = one contiguous source range per XCD,
  // G > 0 = runs of G consecutive blocks dealt round-robin over the XCDs
  uint32_t xcd_group;
  uint32_t xcd_hop;  // first_hop_kernel: XCD-aware source order (set by launch_first_hop)
  // logical blocks (sources x tile phases); a grid smaller than this runs
  // persistent workgroups, each striding through its XCD's logical range
  uint32_t n_logical;
};

enum class SpfVariant {
  kUnsupported = 0, kMsBfs, kBfs8, kBfs16, kBfs32, kDist16, kDist32, kGlobal,
  kGlobalNh,  // HBM frontier kernel that also derives the first hops (no phase 2)
  kExact,     // the reference's Dijkstra order (zero metrics, 64-bit path metrics)
  kBfsNh,     // uniform metric, few sources: BFS with the first hops fused (no phase 2)
  kRepair,    // ignore-set batch derived from its sources' plain SPFs (whatif_kernels.hip)
  kLdsNh,     // general metrics, labels {dist, first hops} in LDS, first hops fused (no phase 2)
  kWms        // general metrics, many sources: 4-source Bellman-Ford in LDS, then phase 2
};
// spf_wms_kernel: LDS bytes of one batch of `sources` (4 or 8) sources
// (u16 x sources per node + 1), and the batch width launch_spf_wms takes
size_t wms_lds_bytes(uint32_t n_nodes, uint32_t sources = 4);
uint32_t wms_sources(uint32_t n_nodes, size_t lds_limit);
// batches of 4 or 8 rows (a.order; wms_sources), 1024 threads each; rows whose labels come too
// close to 16 bits are listed in a.ovf_rows (n_rows + 1 words) and redone by
// the u64 spf_lds_nh_kernel (its LDS must fit). Writes dist rows only.
// wms_k: in-link slots per node of a.wms_slots (4 or 8); a.recs_k: the ELL
// width of a.recs (for the u64 LDS search of the flagged rows)
hipError_t launch_spf_wms(SpfArgs a, uint32_t n_rows, uint32_t wms_k, size_t lds_limit, hipStream_t s);
// spf_lds_nh_kernel: LDS bytes per search (packed: u32 labels, <= 16
// distinct neighbours per source; else u64 labels)
size_t lds_nh_bytes(uint32_t n_nodes, bool packed);
// one workgroup of `block` threads per row; packed: rows whose distances
// outgrow 16 bits are listed in a.ovf_rows (n_rows + 1 words) and redone
// with u64 labels. Writes out_dist / out_nh rows [0, n_rows)
hipError_t launch_spf_lds_nh(SpfArgs a, uint32_t n_rows, uint32_t ell_k, bool packed, uint32_t block,
                             hipStream_t s);
// fused BFS + first hops (spf_bfs_nh_kernel): workgroup size, nodes per
// thread and LDS bytes for N nodes and `words` first-hop words per node;
// false when the graph does not fit (N > 32768 or LDS)
bool bfs_nh_shape(uint32_t n_nodes, uint32_t words, size_t lds_limit, uint32_t* block,
                  uint32_t* j, size_t* lds);

// exact Dijkstra (spf_exact_kernel): one wave per source row; heap, 64-bit
// metrics and first-hop masks in LDS (or per-row global scratch when the
// graph is too large); outputs u32 or u64 distances, masks and the
// extraction rank of every node (the reference's pathLinks order)
struct ExactArgs {
  uint32_t n_nodes;
  uint32_t n_rows;
  uint32_t words;
  int32_t use_link_metric;
  uint32_t ell_k;
  const uint2* recs;
  const uint32_t* link;
  const uint16_t* rank_out;
  const uint32_t* name_rank;  // [N] byte order of the node names (heap ties)
  const uint32_t* srcs;
  const uint32_t* ignore_ptr;
  const uint32_t* ignore_links;
  uint32_t* out_dist32;  // nullable: [rows][N], ORH_UNREACHABLE
  uint64_t* out_dist64;  // nullable: [rows][N], ~0 unreachable
  uint32_t* out_nh;      // [rows][N][words]
  uint32_t* out_rank;    // nullable: [rows][N], extraction order (~0 unreached)
  uint8_t* scratch;      // global per-row state when not in LDS
  size_t scratch_stride;
};
size_t exact_state_bytes(uint32_t n_nodes, uint32_t words);
hipError_t launch_exact(const ExactArgs& a, size_t lds_limit, hipStream_t s);

// distance-kernel selection (orh_set_spf_mode): automatic (multi-source BFS
// when eligible, else the LDS-resident per-source kernels, else the HBM
// frontier kernel), per-source LDS kernels only, the HBM kernel always (with
// fused first hops when every source has <= 32 distinct neighbours), or the
// two-phase HBM kernel always
enum class SpfMode { kAuto = 0, kPerSource = 1, kGlobal = 2, kGlobalTwoPhase = 3, kExact = 4 };
constexpr int kSpfModes = 5;

struct SpfPlan {
  SpfVariant variant;
  uint32_t ell_k;
  uint32_t block;
  uint32_t mask_bytes;  // multi-source BFS: source-mask width (up to 8 * mask_bytes sources)
  uint32_t ms_width;    // multi-source BFS: sources per batch (ms_set_width)
  uint32_t ms_j;        // multi-source BFS: nodes owned per thread (template)
  uint32_t ms_pitch;    // multi-source BFS: frontier-array entries
  uint32_t ms_skip;     // multi-source BFS: interval skip (latency plan)
  size_t pend_off;
  size_t lds_bytes;
};

// uniform: every live link carries the same metric (BFS levels suffice);
// path_bound: upper bound on any tentative distance
// multi_source: the batch has no ignore sets, so rows may share one search
SpfPlan plan_spf(uint32_t n_nodes, bool uniform, uint64_t path_bound, uint32_t ell_k,
                 size_t lds_limit, bool multi_source, SpfMode mode);
hipError_t launch_spf(const SpfPlan& plan, SpfArgs a, uint32_t n_rows, hipStream_t s);
// distances only, one search per CU with u16 distances in LDS
// (spf_lds16_kernel), rows it cannot finish re-run by `fallback` (a kGlobalNh
// plan) over the list a.ovf_rows (n_rows + 1 words); needs a.dist_only
size_t lds16_bytes(uint32_t n_nodes);
hipError_t launch_spf_lds16(const SpfPlan& fallback, SpfArgs a, uint32_t n_rows, uint32_t ell_k,
                            hipStream_t s);
// multi-source plans, once the row count is known: sources per batch, and
// u64 masks when u32 ones would put more than one batch on a CU
// alone: no other sweep in flight on the device (lone-sweep plan)
void ms_set_width(SpfPlan& plan, uint32_t n_nodes, uint32_t n_rows, uint32_t n_cu, size_t lds_limit,
                  bool alone = false);
// bytes of node-major level scratch a multi-source plan needs for n_rows rows
size_t ms_scratch_bytes(const SpfPlan& plan, uint32_t n_nodes, uint32_t n_rows);
// bytes of the multi-source arrival logs (u16 / u32 masks; 0 otherwise), after
// ms_set_width: per batch J * block * mask bits events of 8 bytes
size_t ms_log_bytes(const SpfPlan& plan, uint32_t n_rows);

// LDS bytes the first-hop kernel needs for max_nbr distinct neighbours
size_t hop_lds_bytes(uint32_t max_nbr);
// *nodes_per_thread / *split receive the chosen kernel shape (16 or 4 nodes
// per thread over level rows, 1 for u32 rows)
hipError_t launch_first_hop(HopArgs a, uint32_t max_nbr, hipStream_t s,
                            uint32_t* nodes_per_thread = nullptr, uint32_t* split = nullptr);
// multi-source BFS plans, phase 2a: node-major level bytes -> requested dist
// rows (host order) and u8 level rows of every row (a.lvl_rows), which the
// first-hop phase reads instead of u32 distance rows
hipError_t launch_ms_finalize(const SpfPlan& plan, SpfArgs a, uint32_t n_rows, hipStream_t s);

// recs[pos[i]] = vals[i] for i < n (device pointers)
// recs[pos[i]] = vals[i], link[pos[i]] = links[i], rank[pos[i]] = ranks[i]
hipError_t launch_scatter_rows(uint2* recs, uint32_t* link, uint16_t* rank, const uint32_t* pos,
                               const uint2* vals, const uint32_t* links, const uint16_t* ranks,
                               uint32_t n, hipStream_t s);
hipError_t launch_scatter_recs(uint2* recs, const uint32_t* pos, const uint2* vals, uint32_t n,
                               hipStream_t s);

}  // namespace orh
