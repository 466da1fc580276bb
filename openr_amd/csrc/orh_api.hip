// libopenr_hip: C ABI (include/openr_hip.h) over the gfx950 SPF kernels.
//
// Owns per-device contexts (stream, events, counters, request staging,
// scratch distance rows) and per-area graph mirrors (ELL edge records, link
// ids, node flags and the neighbour-rank table that numbers first-hop bits).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/openr_hip.h"
#include "kernels/ksp_kernels.h"
#include "kernels/route_kernels.h"
#include "kernels/spf_kernels.h"
#include "kernels/whatif_kernels.h"

struct orh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, evm = nullptr, ev1 = nullptr;  // around phase 1 | phase 2
  size_t lds_limit = 160 * 1024;
  uint32_t n_cu = 256;  // compute units (multi-source batch sizing)
  orh::SpfMode spf_mode = orh::SpfMode::kAuto;  // orh_set_spf_mode
  // ORH_DELTA_PCT: HBM-kernel near/far width in % of the mean live metric;
  // 50 measured best on the C4 WAN what-if batch (25: 12.4, 50: 11.9,
  // 100: 13.1, 200: 17.0, 400: 23.6 ms; log-normal metrics, mean ~3x median)
  uint32_t delta_pct = 50;
  orh_spf_info last_info{};    // orh_last_spf_info
  std::string err;
  orh_counters counters{};
  // reusable device staging for the exact kernel's request arrays
  uint32_t* d_req = nullptr;
  size_t d_req_cap = 0;
  std::vector<uint32_t> req_key;
  // distance rows of neighbours that are not themselves requested sources
  uint32_t* d_scratch = nullptr;
  size_t d_scratch_cap = 0;  // in u32
  // HBM kernel with fused first hops: {dist, nh} labels per row
  unsigned long long* d_labels = nullptr;
  size_t d_labels_cap = 0;  // in labels
  // multi-source BFS: u8 level row per row (first-hop input)
  uint8_t* d_lvl_rows = nullptr;
  size_t d_lvl_rows_cap = 0;  // in bytes
  // multi-source BFS: node-major level bytes
  uint8_t* d_ms_lvl = nullptr;
  size_t d_ms_lvl_cap = 0;
  // deferred second phase (ORH_SPF_DEFER_HOPS): finalize + first hops of a
  // sweep on stream2 while the context stream takes the next sweep's search.
  // The level bytes alternate between two halves of d_ms_lvl; a search into
  // half b first waits for the phase 2 still reading it (ev_p2[b])
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_ms2 = nullptr;                // end of the search phase 2 follows
  hipEvent_t ev_p2[2] = {nullptr, nullptr};   // end of the phase 2 reading half b
  bool p2_pending[2] = {false, false};        // ev_p2[b] not yet joined
  uint32_t p2_half = 0;                       // half of the next deferred sweep
  // orh_spf_batch's device rows (reused: a hipMalloc/hipFree pair per call
  // costs more than a single-source SPF)
  uint32_t* d_batch = nullptr;
  size_t d_batch_cap = 0;  // in u32
  // mirror-patch staging (positions + records of one delta batch)
  uint32_t* d_patch = nullptr;
  size_t d_patch_cap = 0;  // in u32
  // exact kernel: per-row heap state when it does not fit in LDS, and
  // orh_spf_batch_exact's device rows
  uint8_t* d_exact = nullptr;
  size_t d_exact_cap = 0;  // in bytes
  uint8_t* d_batch_x = nullptr;
  size_t d_batch_x_cap = 0;  // in bytes
  uint8_t* d_ksp = nullptr;  // orh_ksp2_batch: rows, traces' scratch and output
  size_t d_ksp_cap = 0;
  uint32_t* h_ksp = nullptr;  // orh_ksp2_batch's pinned output blocks
  size_t h_ksp_cap = 0;       // in u32
  uint8_t* d_rep_slots = nullptr;  // global repair slots (requests that outgrow LDS)
  size_t d_rep_slots_cap = 0;
  const orh_whatif* slots_owner = nullptr;  // the what-if job using them (one at a time)
  uint32_t* h_pinned = nullptr;  // orh_spf_batch_pinned's host rows (hipHostMalloc)
  size_t h_pinned_cap = 0;       // in u32
  // ORH_WHATIF_REPAIR: 0 off, 1 automatic (sources repeat, small ignore
  // sets), 2 every ignore-set batch the repair can take
  int repair_mode = 1;
  uint32_t rep_cap_a = 0, rep_cap_e = 0;  // LDS repair caps; 0 = by graph size (ORH_REPAIR_CAPS=A,E)
};

struct orh_graph {
  orh_ctx* ctx = nullptr;
  // process-wide unique id of the uploaded structure (new on every load), so
  // a context's staged request can never match a different or reloaded graph
  // even when a new orh_graph reuses a freed one's address
  uint64_t gen = 0;
  uint32_t n_nodes = 0, n_edges = 0, n_links = 0;
  // host CSR (ABI semantics) kept for deltas, neighbour tables and bounds
  std::vector<uint32_t> row_ptr, col, w_out, w_in, meta;
  std::vector<uint32_t> ent_row;  // entry -> row (entry_rows), valid for ent_row_gen
  uint64_t ent_row_gen = ~0ull;
  std::vector<uint8_t> overloaded;
  std::vector<uint32_t> dn_ptr, dn;  // distinct neighbours per node, ascending id
  std::vector<uint16_t> rank_out;    // per CSR entry: col's rank among row's distinct neighbours
  uint64_t sum_max_metric = 0;       // sum over up CSR entries of max(w_out, w_in)
  uint32_t max_metric = 0;
  uint32_t min_out = 0, max_out = 0;  // w_out range over up CSR entries
  uint32_t mean_out = 1;               // mean w_out over up CSR entries
  bool has_zero = false;               // an up CSR entry has w_out == 0
  std::vector<uint32_t> name_rank;     // orh_csr::name_rank (identity when not given)
  uint32_t* d_name_rank = nullptr;
  // device layout: ELL slots v*K .. v*K+K-1, the last one a continuation
  // record into the overflow area when deg(v) > K
  uint32_t ell_k = 4;
  uint32_t n_recs = 0;
  std::vector<uint32_t> pos;  // CSR entry -> device record index
  uint2* d_recs = nullptr;
  uint32_t* d_link = nullptr;
  uint16_t* d_rank_out = nullptr;
  uint8_t* d_ovl = nullptr;
  // multi-source BFS layout: the same ELL records in a Cuthill-McKee node
  // order (neighbours get nearby ids, so a batch of consecutive sources is a
  // compact region and a wave's 64 nodes progress together). Rebuilt lazily
  // after attribute patches. Rows in HBM are always indexed by host id.
  std::vector<uint32_t> ms_dev_of, ms_host_of;  // host -> CM id, CM id -> host
  bool ms_identity = false;  // the layout kept the host order (order_nodes)
  bool ms_dirty = true;
  uint32_t ms_bw = 0;  // CM bandwidth over live records when the interval skip is on, else 0
  uint32_t ms_bw_layout = 1;  // the same bandwidth whatever the opt-in (latency-plan skip)
  uint2* d_ms_recs = nullptr;
  uint32_t* d_ms_dev_of = nullptr;
  uint32_t* d_ms_host_of = nullptr;
  // multi-source Bellman-Ford (kWms): in-link slots per Cuthill-McKee node,
  // rebuilt with the multi-source layout; wms_ok: the graph qualifies (every
  // degree <= 8, metrics < 2^15, N < 20,481); wms_k slots per node (4 or 8)
  uint32_t* d_wms = nullptr;
  bool wms_dirty = true, wms_ok = false;
  uint32_t wms_maxw = 0, wms_k = 4;
  std::vector<int32_t> row_of;  // scratch for orh_spf_run (all -1 between calls)
  // orh_spf_run's staged request on this graph (sources, ignore sets,
  // neighbour rows, batch order), keyed by the request: a repeated sweep
  // neither rebuilds nor uploads it, even when several graphs share a context
  uint32_t* d_req = nullptr;
  size_t d_req_cap = 0;
  std::vector<uint32_t> req_key;
  uint32_t req_xcd_group = 0;  // HopArgs::xcd_group of the staged request
  // what-if repair: per record, the record of the same link from the other
  // end; per link, its two CSR entries (~0 when absent); valid for rev_gen
  uint32_t* d_rev = nullptr;
  uint64_t rev_gen = 0;
  std::vector<uint32_t> link_ent;  // [2 * n_links]
};

namespace {

int fail(orh_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(orh_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, ORH_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define ORH_HIP(ctx, call)                                 \
  do {                                                     \
    hipError_t e_ = (call);                                \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
  } while (0)

void free_graph_device(orh_graph* g) {
  (void)hipFree(g->d_recs);
  (void)hipFree(g->d_link);
  (void)hipFree(g->d_rank_out);
  (void)hipFree(g->d_ovl);
  (void)hipFree(g->d_ms_recs);
  (void)hipFree(g->d_ms_dev_of);
  (void)hipFree(g->d_ms_host_of);
  (void)hipFree(g->d_name_rank);
  (void)hipFree(g->d_rev);
  g->d_rev = nullptr;
  (void)hipFree(g->d_req);
  g->d_req = nullptr;
  g->d_req_cap = 0;
  g->req_key.clear();
  g->rev_gen = 0;
  g->d_name_rank = nullptr;
  g->d_ms_recs = nullptr;
  g->d_ms_dev_of = nullptr;
  g->d_ms_host_of = nullptr;
  g->ms_dirty = true;
  (void)hipFree(g->d_wms);
  g->d_wms = nullptr;
  g->wms_dirty = true;
  g->d_recs = nullptr;
  g->d_link = nullptr;
  g->d_rank_out = nullptr;
  g->d_ovl = nullptr;
}

// distinct neighbour lists and, per CSR entry, the neighbour's rank in its
// row's list (= the first-hop bit of that neighbour)
void build_neighbours(orh_graph* g) {
  const uint32_t N = g->n_nodes;
  g->dn_ptr.assign(N + 1, 0);
  g->dn.clear();
  g->rank_out.assign(g->n_edges, 0);
  std::vector<uint32_t> l;
  for (uint32_t v = 0; v < N; ++v) {
    l.clear();
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e)
      if (g->meta[e] != ORH_META_EMPTY) l.push_back(g->col[e]);
    std::sort(l.begin(), l.end());
    l.erase(std::unique(l.begin(), l.end()), l.end());
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e)
      g->rank_out[e] = g->meta[e] == ORH_META_EMPTY
          ? 0
          : static_cast<uint16_t>(std::lower_bound(l.begin(), l.end(), g->col[e]) - l.begin());
    g->dn.insert(g->dn.end(), l.begin(), l.end());
    g->dn_ptr[v + 1] = static_cast<uint32_t>(g->dn.size());
  }
}

uint32_t n_distinct(const orh_graph* g, uint32_t v) { return g->dn_ptr[v + 1] - g->dn_ptr[v]; }

// ELL width: smallest power of two covering 90% of the node degrees, in [4, 8]
uint32_t choose_ell_k(const orh_graph* g) {
  std::vector<uint32_t> deg(g->n_nodes);
  for (uint32_t v = 0; v < g->n_nodes; ++v) deg[v] = g->row_ptr[v + 1] - g->row_ptr[v];
  if (deg.empty()) return 4;
  std::nth_element(deg.begin(), deg.begin() + deg.size() * 9 / 10, deg.end());
  return deg[deg.size() * 9 / 10] > 4 ? 8 : 4;
}

// Cuthill-McKee: BFS from a low-degree node of each component, neighbours
// visited in ascending degree (then host id) order
void order_nodes(orh_graph* g) {
  const uint32_t N = g->n_nodes;
  auto& host_of = g->ms_host_of;
  auto& dev_of = g->ms_dev_of;
  host_of.clear();
  host_of.reserve(N);
  dev_of.assign(N, 0xFFFFFFFFu);
  std::vector<uint32_t> deg(N), by_deg(N), nb;
  for (uint32_t v = 0; v < N; ++v) {
    deg[v] = g->dn_ptr[v + 1] - g->dn_ptr[v];
    by_deg[v] = v;
  }
  std::stable_sort(by_deg.begin(), by_deg.end(),
                   [&](uint32_t a, uint32_t b) { return deg[a] < deg[b]; });
  for (uint32_t root : by_deg) {
    if (dev_of[root] != 0xFFFFFFFFu) continue;
    size_t head = host_of.size();
    dev_of[root] = static_cast<uint32_t>(host_of.size());
    host_of.push_back(root);
    while (head < host_of.size()) {
      const uint32_t v = host_of[head++];
      nb.clear();
      for (uint32_t k = g->dn_ptr[v]; k < g->dn_ptr[v + 1]; ++k)
        if (dev_of[g->dn[k]] == 0xFFFFFFFFu) nb.push_back(g->dn[k]);
      std::stable_sort(nb.begin(), nb.end(), [&](uint32_t a, uint32_t b) { return deg[a] < deg[b]; });
      for (uint32_t u : nb) {
        dev_of[u] = static_cast<uint32_t>(host_of.size());
        host_of.push_back(u);
      }
    }
  }
  // ORH_MS_ORDER=host (A/B): the host order itself. Its slices are runs of
  // host ids, so the multi-source BFS writes the u32 distance rows straight
  // from its level assembly (no ms_finalize pass) and a wave's gathers read
  // neighbours at the same offsets (v +- 1, v +- n on a grid numbered row by
  // row) instead of across anti-diagonal boundaries. Measured slower on the
  // C2 grid, so Cuthill-McKee stays the default: the 32-sweep step 24.2-24.6
  // ms against 22.9, one sweep 1.10 against 0.93 ms (the host-order BFS 0.75
  // against 0.64 ms, the direct rows another 0.13 ms in it for 0.06 ms of
  // phase 2; profiles/r06/j_ms_ab.txt). ORH_MS_ORDER=cm forces the default
  const char* fe = getenv("ORH_MS_ORDER");  // read per layout (tests set it per graph)
  g->ms_identity = fe && strcmp(fe, "host") == 0;
  if (g->ms_identity)
    for (uint32_t v = 0; v < N; ++v) dev_of[v] = host_of[v] = v;
}

uint2 device_record(const orh_graph* g, uint32_t v, uint32_t e, const uint32_t* dev_of = nullptr) {
  uint32_t x = dev_of ? dev_of[g->col[e]] : g->col[e];
  if (g->meta[e] & ORH_META_DOWN) x |= ORH_REC_SKIP;
  if (g->overloaded[v]) x |= ORH_REC_ROW_OVL;
  return make_uint2(x, g->w_out[e]);
}

void build_layout(orh_graph* g, std::vector<uint2>& recs, std::vector<uint32_t>& link,
                  std::vector<uint16_t>& rank) {
  const uint32_t K = g->ell_k, N = g->n_nodes;
  size_t n = static_cast<size_t>(N) * K;
  for (uint32_t v = 0; v < N; ++v) {
    const uint32_t d = g->row_ptr[v + 1] - g->row_ptr[v];
    if (d > K) n += d - (K - 1);
  }
  recs.assign(std::max<size_t>(n, 1), make_uint2(ORH_REC_SKIP, 1));
  link.assign(recs.size(), 0);
  rank.assign(recs.size(), 0);
  g->pos.assign(g->n_edges, 0);
  uint32_t ovf = N * K;
  for (uint32_t v = 0; v < N; ++v) {
    const uint32_t e0 = g->row_ptr[v], d = g->row_ptr[v + 1] - e0, base = v * K;
    const uint32_t inl = d <= K ? d : K - 1;
    for (uint32_t j = 0; j < inl; ++j) g->pos[e0 + j] = base + j;
    if (d > K) {
      recs[base + K - 1] = make_uint2(ovf | ORH_REC_CONT, d - inl);
      for (uint32_t j = inl; j < d; ++j) g->pos[e0 + j] = ovf++;
    }
    for (uint32_t j = 0; j < d; ++j) {
      const uint32_t q = g->pos[e0 + j];
      recs[q] = device_record(g, v, e0 + j);
      link[q] = g->meta[e0 + j] & ORH_META_LINK_MASK;
      rank[q] = g->rank_out[e0 + j];
    }
  }
  g->n_recs = static_cast<uint32_t>(recs.size());
}

// the ELL records again, rows and columns in Cuthill-McKee ids
void build_ms_layout(orh_graph* g, std::vector<uint2>& recs) {
  const uint32_t K = g->ell_k, N = g->n_nodes;
  recs.assign(g->n_recs, make_uint2(ORH_REC_SKIP, 1));
  uint32_t ovf = N * K, bw = 0;
  auto put = [&](uint32_t q, uint32_t dv, uint32_t v, uint32_t e) {
    recs[q] = device_record(g, v, e, g->ms_dev_of.data());
    if (!(recs[q].x & ORH_REC_SKIP)) {
      const uint32_t u = recs[q].x & ORH_REC_COL_MASK;
      bw = std::max(bw, u > dv ? u - dv : dv - u);
    }
  };
  for (uint32_t dv = 0; dv < N; ++dv) {
    const uint32_t v = g->ms_host_of[dv];
    const uint32_t e0 = g->row_ptr[v], d = g->row_ptr[v + 1] - e0, base = dv * K;
    const uint32_t inl = d <= K ? d : K - 1;
    for (uint32_t j = 0; j < inl; ++j) put(base + j, dv, v, e0 + j);
    if (d > K) {
      recs[base + K - 1] = make_uint2(ovf | ORH_REC_CONT, d - inl);
      for (uint32_t j = inl; j < d; ++j) put(ovf++, dv, v, e0 + j);
    }
  }
  // the pull OR is order-free, so each node's inline slots are sorted by
  // neighbour id: a slot then reads the same relative neighbour (e.g. "lower
  // anti-diagonal, left") across a wave's consecutive Cuthill-McKee nodes,
  // consecutive frontier words instead of a mix of directions at the border
  // rows (bank conflicts of the ds_read_b32 gathers). ORH_MS_SORT=0: CSR order.
  const char* es = getenv("ORH_MS_SORT");
  if (!(es && atoi(es) == 0)) {
    for (uint32_t dv = 0; dv < N; ++dv) {
      uint2* r = recs.data() + static_cast<size_t>(dv) * K;
      const uint32_t n_inl = (r[K - 1].x & ORH_REC_CONT) ? K - 1 : K;
      std::stable_sort(r, r + n_inl, [](const uint2& a, const uint2& b) {
        const uint32_t ka = (a.x & ORH_REC_SKIP) ? ~0u : (a.x & ORH_REC_COL_MASK);
        const uint32_t kb = (b.x & ORH_REC_SKIP) ? ~0u : (b.x & ORH_REC_COL_MASK);
        return ka < kb;
      });
    }
  }
  // interval skip (spf_msbfs_kernel<..., true>), opt-in with ORH_MS_SKIP=1:
  // it cuts a lone corner batch of the C2 grid from 0.48 to 0.32 ms, but the
  // all-sources sweep stays at 0.75-0.77 ms either way (profiles/r02/
  // msbfs_ab.md: with every CU busy the level-byte stores, not the skipped
  // slices, set the time)
  const char* e = getenv("ORH_MS_SKIP");
  const bool on = e && atoi(e) == 1;
  g->ms_bw = on ? std::max(bw, 1u) : 0u;
  g->ms_bw_layout = std::max(bw, 1u);
}

int sync_ms_layout(orh_graph* g) {
  if (!g->ms_dirty) return ORH_OK;
  orh_ctx* ctx = g->ctx;
  std::vector<uint2> recs;
  build_ms_layout(g, recs);
  if (!g->d_ms_recs) {
    const size_t nn = std::max<uint32_t>(g->n_nodes, 1);
    if (hipMalloc(&g->d_ms_recs, recs.size() * sizeof(uint2)) != hipSuccess ||
        hipMalloc(&g->d_ms_dev_of, nn * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&g->d_ms_host_of, nn * sizeof(uint32_t)) != hipSuccess)
      return fail(ctx, ORH_E_NOMEM, "multi-source layout: device allocation failed");
    ORH_HIP(ctx, hipMemcpyAsync(g->d_ms_dev_of, g->ms_dev_of.data(), g->n_nodes * sizeof(uint32_t),
                                hipMemcpyHostToDevice, ctx->stream));
    ORH_HIP(ctx, hipMemcpyAsync(g->d_ms_host_of, g->ms_host_of.data(), g->n_nodes * sizeof(uint32_t),
                                hipMemcpyHostToDevice, ctx->stream));
  }
  ORH_HIP(ctx, hipMemcpyAsync(g->d_ms_recs, recs.data(), recs.size() * sizeof(uint2),
                              hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // recs is a local
  g->ms_dirty = false;
  return ORH_OK;
}

// kWms in-link slots: per Cuthill-McKee node dv, ell_k slots {u | w(u -> v)
// << 16 | overloaded(u) << 31}, u the Cuthill-McKee id of the neighbour and
// w the metric of the link from u's side (LinkState.cpp:851-852: the search
// relaxes getMetricFromNode(u)); a down link or an unused slot is u = N
int sync_wms_layout(orh_graph* g) {
  if (!g->wms_dirty) return ORH_OK;
  int rc = sync_ms_layout(g);
  if (rc) return rc;
  const uint32_t N = g->n_nodes;
  uint32_t maxdeg = 0;
  for (uint32_t v = 0; v < N; ++v) maxdeg = std::max(maxdeg, g->row_ptr[v + 1] - g->row_ptr[v]);
  const uint32_t K = maxdeg <= 4 ? 4u : 8u;  // slots per node (its own width, not the ELL's)
  g->wms_k = K;
  g->wms_ok = N > 0 && N <= 20480 && maxdeg <= 8;
  g->wms_maxw = 0;
  std::vector<uint32_t> slots;
  if (g->wms_ok) {
    slots.assign(static_cast<size_t>(N) * K, N);
    for (uint32_t dv = 0; dv < N && g->wms_ok; ++dv) {
      const uint32_t v = g->ms_host_of[dv];
      uint32_t k = 0;
      for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e, ++k) {
        if (g->meta[e] & ORH_META_DOWN) continue;
        const uint32_t w = g->w_in[e], u = g->col[e];
        if (w == 0 || w > 0x7FFFu) {
          g->wms_ok = false;
          break;
        }
        g->wms_maxw = std::max(g->wms_maxw, w);
        slots[static_cast<size_t>(dv) * K + k] = g->ms_dev_of[u] | (w << 16) | (g->overloaded[u] ? 0x80000000u : 0u);
      }
    }
  }
  if (g->wms_ok) {
    orh_ctx* ctx = g->ctx;
    if (!g->d_wms) ORH_HIP(ctx, hipMalloc(&g->d_wms, static_cast<size_t>(N) * 8 * sizeof(uint32_t)));
    ORH_HIP(ctx, hipMemcpyAsync(g->d_wms, slots.data(), slots.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                ctx->stream));
    ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // slots is a local
  }
  g->wms_dirty = false;
  return ORH_OK;
}

uint64_t next_graph_gen() {
  static std::atomic<uint64_t> gen{0};
  return ++gen;
}

// re-upload the device records of CSR entries `edges` (row node, entry) with
// one staging copy and one scatter launch
int upload_records(orh_graph* g, const std::vector<std::pair<uint32_t, uint32_t>>& edges) {
  if (edges.empty()) return ORH_OK;
  orh_ctx* ctx = g->ctx;
  const uint32_t n = static_cast<uint32_t>(edges.size());
  // staging: pos[n] (u32, padded to 8 bytes) | vals[n] (uint2)
  const size_t pos_words = (n + 1) & ~1u;
  std::vector<uint32_t> staging(pos_words + 2 * static_cast<size_t>(n));
  uint2* vals = reinterpret_cast<uint2*>(staging.data() + pos_words);
  for (uint32_t i = 0; i < n; ++i) {
    staging[i] = g->pos[edges[i].second];
    vals[i] = device_record(g, edges[i].first, edges[i].second);
  }
  if (staging.size() > ctx->d_patch_cap) {
    (void)hipFree(ctx->d_patch);
    ctx->d_patch = nullptr;
    ctx->d_patch_cap = 0;
    ORH_HIP(ctx, hipMalloc(&ctx->d_patch, staging.size() * sizeof(uint32_t)));
    ctx->d_patch_cap = staging.size();
  }
  ORH_HIP(ctx, hipMemcpyAsync(ctx->d_patch, staging.data(), staging.size() * sizeof(uint32_t),
                              hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, orh::launch_scatter_recs(g->d_recs, ctx->d_patch,
                                        reinterpret_cast<const uint2*>(ctx->d_patch + pos_words), n,
                                        ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // staging is a local
  g->ms_dirty = true;
  g->wms_dirty = true;
  return ORH_OK;
}

uint32_t row_of(const orh_graph* g, uint32_t e) {
  return static_cast<uint32_t>(std::upper_bound(g->row_ptr.begin(), g->row_ptr.end(), e) -
                               g->row_ptr.begin()) - 1;
}

// row of every CSR entry, rebuilt when the structure generation moves (a
// what-if run stages two cuts per ignored link: 131k binary searches over
// row_ptr per 65,536-request C4 chunk otherwise)
const std::vector<uint32_t>& entry_rows(orh_graph* g) {
  if (g->ent_row_gen != g->gen || g->ent_row.size() != g->n_edges) {
    g->ent_row.assign(g->n_edges, 0u);
    for (uint32_t v = 0; v < g->n_nodes; ++v)
      for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) g->ent_row[e] = v;
    g->ent_row_gen = g->gen;
  }
  return g->ent_row;
}

void recompute_bounds(orh_graph* g) {
  g->sum_max_metric = 0;
  g->max_metric = 0;
  g->min_out = 0xFFFFFFFFu;
  g->max_out = 0;
  g->has_zero = false;
  for (uint32_t e = 0; e < g->n_edges; ++e) {
    if (g->meta[e] & ORH_META_DOWN) continue;
    g->has_zero |= g->w_out[e] == 0;
    const uint32_t m = std::max(g->w_out[e], g->w_in[e]);
    g->max_metric = std::max(g->max_metric, m);
    g->sum_max_metric += m;  // each link is counted twice (both CSR entries)
    g->min_out = std::min(g->min_out, g->w_out[e]);
    g->max_out = std::max(g->max_out, g->w_out[e]);
  }
  if (g->max_out == 0) g->min_out = g->max_out = 1;  // no up link
  uint64_t sum_out = 0, n_up = 0;
  for (uint32_t e = 0; e < g->n_edges; ++e)
    if (!(g->meta[e] & ORH_META_DOWN)) {
      sum_out += g->w_out[e];
      ++n_up;
    }
  g->mean_out = n_up ? static_cast<uint32_t>(sum_out / n_up) : 1u;
}

int ensure_req(orh_ctx* ctx, size_t words) {
  if (words <= ctx->d_req_cap) return ORH_OK;
  hipFree(ctx->d_req);
  ctx->d_req = nullptr;
  ctx->req_key.clear();
  const size_t cap = std::max<size_t>(words, 4096);
  ORH_HIP(ctx, hipMalloc(&ctx->d_req, cap * sizeof(uint32_t)));
  ctx->d_req_cap = cap;
  return ORH_OK;
}

int ensure_graph_req(orh_graph* g, size_t words) {
  if (words <= g->d_req_cap) return ORH_OK;
  hipFree(g->d_req);
  g->d_req = nullptr;
  g->d_req_cap = 0;
  g->req_key.clear();
  const size_t cap = std::max<size_t>(words, 4096);
  ORH_HIP(g->ctx, hipMalloc(&g->d_req, cap * sizeof(uint32_t)));
  g->d_req_cap = cap;
  return ORH_OK;
}

// deferred second phases: the context stream waits for them (device side)
void join_deferred(orh_ctx* ctx) {
  for (int b = 0; b < 2; ++b)
    if (ctx->p2_pending[b]) {
      hipStreamWaitEvent(ctx->stream, ctx->ev_p2[b], 0);
      ctx->p2_pending[b] = false;
    }
}

// ... or the host waits for them (before a buffer they read is freed or
// rewritten outside the context stream's order)
void drain_deferred(orh_ctx* ctx) {
  if (!ctx->stream2) return;
  hipStreamSynchronize(ctx->stream2);
  ctx->p2_pending[0] = ctx->p2_pending[1] = false;
}

int ensure_lvl_rows(orh_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->d_lvl_rows_cap) return ORH_OK;
  drain_deferred(ctx);
  hipFree(ctx->d_lvl_rows);
  ctx->d_lvl_rows = nullptr;
  ctx->d_lvl_rows_cap = 0;
  ORH_HIP(ctx, hipMalloc(&ctx->d_lvl_rows, bytes));
  ctx->d_lvl_rows_cap = bytes;
  return ORH_OK;
}

int ensure_labels(orh_ctx* ctx, size_t n) {
  if (n <= ctx->d_labels_cap) return ORH_OK;
  hipFree(ctx->d_labels);
  ctx->d_labels = nullptr;
  ctx->d_labels_cap = 0;
  ORH_HIP(ctx, hipMalloc(&ctx->d_labels, n * sizeof(unsigned long long)));
  ctx->d_labels_cap = n;
  return ORH_OK;
}

int ensure_scratch(orh_ctx* ctx, size_t words) {
  if (words <= ctx->d_scratch_cap) return ORH_OK;
  drain_deferred(ctx);
  hipFree(ctx->d_scratch);
  ctx->d_scratch = nullptr;
  ctx->d_scratch_cap = 0;
  ORH_HIP(ctx, hipMalloc(&ctx->d_scratch, words * sizeof(uint32_t)));
  ctx->d_scratch_cap = words;
  return ORH_OK;
}

int ensure_bytes(orh_ctx* ctx, uint8_t** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return ORH_OK;
  hipFree(*p);
  *p = nullptr;
  *cap = 0;
  ORH_HIP(ctx, hipMalloc(p, bytes));
  *cap = bytes;
  return ORH_OK;
}

// path metrics of the graph can reach the 32-bit sentinel (link metrics are
// summed in 64 bits by the reference, LinkState.h:22)
bool wide_metrics(const orh_graph* g) {
  return g->sum_max_metric / 2 + g->max_metric >= 0xFFFFFFFFull;
}

// a staged request is reused when the stored key is this request's key
// followed by `extra` words of staging offsets
bool staged_key_matches(const std::vector<uint32_t>& stored, const std::vector<uint32_t>& key, size_t extra) {
  return stored.size() == key.size() + extra && std::equal(key.begin(), key.end(), stored.begin());
}

int ensure_ms_lvl(orh_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->d_ms_lvl_cap) return ORH_OK;
  drain_deferred(ctx);
  hipFree(ctx->d_ms_lvl);
  ctx->d_ms_lvl = nullptr;
  ctx->d_ms_lvl_cap = 0;
  ORH_HIP(ctx, hipMalloc(&ctx->d_ms_lvl, bytes));
  ctx->d_ms_lvl_cap = bytes;
  return ORH_OK;
}

}  // namespace

extern "C" {

int orh_device_count(int* out) {
  if (!out) return ORH_E_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return ORH_OK;
}

// every live context, by device: a sweep planned while no other context of
// its device has a sweep in flight (its end event not reached) takes the
// lone-sweep plan (orh::ms_set_width)
static std::mutex g_ctx_mu;
static std::vector<orh_ctx*> g_ctxs;

static bool device_busy_elsewhere(const orh_ctx* ctx) {
  std::lock_guard<std::mutex> lock(g_ctx_mu);
  for (const orh_ctx* o : g_ctxs)
    if (o != ctx && o->device == ctx->device && hipEventQuery(o->ev1) == hipErrorNotReady) return true;
  return false;
}

int orh_create(int device, uint32_t flags, orh_ctx** out) {
  (void)flags;
  if (!out) return ORH_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORH_E_DEVICE;
  if (device < 0 || device >= n) return ORH_E_INVALID;
  auto* ctx = new (std::nothrow) orh_ctx();
  if (!ctx) return ORH_E_NOMEM;
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->evm) != hipSuccess ||
      hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return ORH_E_DEVICE;
  }
  if (const char* e = getenv("ORH_SPF_MODE")) ctx->spf_mode = static_cast<orh::SpfMode>(atoi(e) % orh::kSpfModes);
  if (const char* e = getenv("ORH_DELTA_PCT")) ctx->delta_pct = std::max(1, atoi(e));
  if (const char* e = getenv("ORH_WHATIF_REPAIR")) ctx->repair_mode = atoi(e);
  if (const char* e = getenv("ORH_REPAIR_CAPS")) {
    unsigned ca = 0, ce = 0;
    if (sscanf(e, "%u,%u", &ca, &ce) == 2 && ca >= 64 && ce >= 256) {
      ctx->rep_cap_a = ca;
      ctx->rep_cap_e = ce;
    }
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.sharedMemPerBlock > 0) {
    ctx->lds_limit = std::max<size_t>(prop.sharedMemPerBlock, 64 * 1024);
    if (prop.multiProcessorCount > 0) ctx->n_cu = static_cast<uint32_t>(prop.multiProcessorCount);
  }
  {
    std::lock_guard<std::mutex> lock(g_ctx_mu);
    g_ctxs.push_back(ctx);
  }
  *out = ctx;
  return ORH_OK;
}

int orh_set_spf_mode(orh_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode >= orh::kSpfModes) return ORH_E_INVALID;
  ctx->spf_mode = static_cast<orh::SpfMode>(mode);
  return ORH_OK;
}

int orh_set_repair_mode(orh_ctx* ctx, int mode) {
  if (!ctx || mode < ORH_REPAIR_OFF || mode > ORH_REPAIR_ALWAYS) return ORH_E_INVALID;
  ctx->repair_mode = mode;
  return ORH_OK;
}

int orh_destroy(orh_ctx* ctx) {
  if (!ctx) return ORH_E_INVALID;
  {
    std::lock_guard<std::mutex> lock(g_ctx_mu);
    g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), ctx), g_ctxs.end());
  }
  hipSetDevice(ctx->device);
  drain_deferred(ctx);
  hipStreamSynchronize(ctx->stream);
  hipFree(ctx->d_req);
  hipFree(ctx->d_scratch);
  hipFree(ctx->d_labels);
  hipFree(ctx->d_lvl_rows);
  hipFree(ctx->d_ms_lvl);
  hipFree(ctx->d_batch);
  hipFree(ctx->d_patch);
  hipFree(ctx->d_exact);
  hipFree(ctx->d_batch_x);
  hipFree(ctx->d_rep_slots);
  hipFree(ctx->d_ksp);
  if (ctx->h_ksp) hipHostFree(ctx->h_ksp);
  if (ctx->h_pinned) hipHostFree(ctx->h_pinned);
  hipEventDestroy(ctx->ev0);
  hipEventDestroy(ctx->evm);
  hipEventDestroy(ctx->ev1);
  if (ctx->stream2) {
    hipEventDestroy(ctx->ev_ms2);
    hipEventDestroy(ctx->ev_p2[0]);
    hipEventDestroy(ctx->ev_p2[1]);
    hipStreamDestroy(ctx->stream2);
  }
  hipStreamDestroy(ctx->stream);
  delete ctx;
  return ORH_OK;
}

const char* orh_last_error(const orh_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int orh_sync(orh_ctx* ctx) {
  if (!ctx) return ORH_E_INVALID;
  join_deferred(ctx);
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_get_counters(const orh_ctx* ctx, orh_counters* out) {
  if (!ctx || !out) return ORH_E_INVALID;
  *out = ctx->counters;
  return ORH_OK;
}

int orh_reset_counters(orh_ctx* ctx) {
  if (!ctx) return ORH_E_INVALID;
  ctx->counters = orh_counters{};
  return ORH_OK;
}

int orh_device_alloc(orh_ctx* ctx, size_t bytes, void** d_out) {
  if (!ctx || !d_out) return ORH_E_INVALID;
  hipSetDevice(ctx->device);
  if (hipMalloc(d_out, std::max<size_t>(bytes, 16)) != hipSuccess)
    return fail(ctx, ORH_E_NOMEM, "device allocation failed");
  return ORH_OK;
}

int orh_device_free(orh_ctx* ctx, void* d_ptr) {
  if (!ctx) return ORH_E_INVALID;
  hipFree(d_ptr);
  return ORH_OK;
}

int orh_memcpy_d2h(orh_ctx* ctx, void* h_dst, const void* d_src, size_t bytes) {
  if (!ctx || (!h_dst && bytes) || (!d_src && bytes)) return ORH_E_INVALID;
  if (!bytes) return ORH_OK;
  join_deferred(ctx);
  ORH_HIP(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_memcpy_h2d(orh_ctx* ctx, void* d_dst, const void* h_src, size_t bytes) {
  if (!ctx || (!d_dst && bytes) || (!h_src && bytes)) return ORH_E_INVALID;
  if (!bytes) return ORH_OK;
  join_deferred(ctx);
  ORH_HIP(ctx, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_memcpy_d2d(orh_ctx* ctx, void* d_dst, const void* d_src, size_t bytes) {
  if (!ctx || (!d_dst && bytes) || (!d_src && bytes)) return ORH_E_INVALID;
  join_deferred(ctx);
  ORH_HIP(ctx, hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_row_digest(orh_ctx* ctx, const uint32_t* d_dist, const uint32_t* d_nh, uint32_t words, uint32_t n,
                   uint32_t n_rows, uint64_t* d_out) {
  if (!ctx || words == 0 || (n_rows && (!d_dist || !d_nh || !d_out))) return ORH_E_INVALID;
  if (n_rows == 0) return ORH_OK;
  join_deferred(ctx);
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  ORH_HIP(ctx, orh::launch_row_digest(d_dist, d_nh, words, n, n_rows, d_out, ctx->stream));
  return ORH_OK;
}

int orh_graph_create(orh_ctx* ctx, orh_graph** out) {
  if (!ctx || !out) return ORH_E_INVALID;
  auto* g = new (std::nothrow) orh_graph();
  if (!g) return ORH_E_NOMEM;
  g->ctx = ctx;
  *out = g;
  return ORH_OK;
}

int orh_graph_destroy(orh_graph* g) {
  if (!g) return ORH_E_INVALID;
  hipSetDevice(g->ctx->device);
  drain_deferred(g->ctx);
  hipStreamSynchronize(g->ctx->stream);
  free_graph_device(g);
  g->ctx->req_key.clear();  // the staged request may describe this graph
  delete g;
  return ORH_OK;
}

int orh_graph_load(orh_graph* g, const orh_csr* c) {
  if (!g || !c) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  drain_deferred(ctx);  // the deferred phase 2 reads the graph
  if (!c->row_ptr || (c->n_edges && (!c->col || !c->w_out || !c->w_in || !c->meta)) ||
      (c->n_nodes && !c->node_overloaded))
    return fail(ctx, ORH_E_INVALID, "orh_graph_load: null array");
  if (c->row_ptr[0] != 0 || c->row_ptr[c->n_nodes] != c->n_edges)
    return fail(ctx, ORH_E_INVALID, "orh_graph_load: row_ptr does not span n_edges");
  if (c->n_nodes > ORH_REC_COL_MASK)
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_graph_load: more than 2^27 nodes");
  for (uint32_t v = 0; v < c->n_nodes; ++v)
    if (c->row_ptr[v] > c->row_ptr[v + 1])
      return fail(ctx, ORH_E_INVALID, "orh_graph_load: row_ptr not monotone");
  for (uint32_t e = 0; e < c->n_edges; ++e)
    if (c->meta[e] != ORH_META_EMPTY && c->col[e] >= c->n_nodes)
      return fail(ctx, ORH_E_INVALID, "orh_graph_load: col out of range");
  if (c->name_rank)
    for (uint32_t v = 0; v < c->n_nodes; ++v)
      if (c->name_rank[v] >= c->n_nodes)
        return fail(ctx, ORH_E_INVALID, "orh_graph_load: name_rank out of range");
  // ORH_LOAD_PROF=1: phase times on stderr
  static const bool prof_on = getenv("ORH_LOAD_PROF") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!prof_on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "load-prof %-14s %8.3f ms\n", what,
            std::chrono::duration<double, std::milli>(now - t_prev).count());
    t_prev = now;
  };
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  free_graph_device(g);
  mark("free");
  g->n_nodes = c->n_nodes;
  g->n_edges = c->n_edges;
  g->n_links = c->n_links;
  g->row_ptr.assign(c->row_ptr, c->row_ptr + c->n_nodes + 1);
  g->col.assign(c->col, c->col + c->n_edges);
  g->w_out.assign(c->w_out, c->w_out + c->n_edges);
  g->w_in.assign(c->w_in, c->w_in + c->n_edges);
  g->meta.assign(c->meta, c->meta + c->n_edges);
  for (uint32_t v = 0; v < c->n_nodes; ++v)  // free slots point at their own row
    for (uint32_t e = c->row_ptr[v]; e < c->row_ptr[v + 1]; ++e)
      if (g->meta[e] == ORH_META_EMPTY) g->col[e] = v;
  g->overloaded.assign(c->node_overloaded, c->node_overloaded + c->n_nodes);
  for (auto& o : g->overloaded) o = o ? 1 : 0;
  g->name_rank.resize(c->n_nodes);
  for (uint32_t v = 0; v < c->n_nodes; ++v) g->name_rank[v] = c->name_rank ? c->name_rank[v] : v;
  g->gen = next_graph_gen();
  g->row_of.assign(g->n_nodes, -1);
  mark("copy-in");
  recompute_bounds(g);
  mark("bounds");
  build_neighbours(g);
  mark("neighbours");
  for (uint32_t v = 0; v < g->n_nodes; ++v)
    if (n_distinct(g, v) > 0xFFFFu)
      return fail(ctx, ORH_E_UNSUPPORTED, "orh_graph_load: more than 65535 neighbours");
  g->ell_k = choose_ell_k(g);
  order_nodes(g);
  mark("order");
  std::vector<uint2> recs;
  std::vector<uint32_t> link;
  std::vector<uint16_t> rank;
  build_layout(g, recs, link, rank);
  mark("layout");
  const size_t nn = std::max<uint32_t>(g->n_nodes, 1);
  if (hipMalloc(&g->d_recs, recs.size() * sizeof(uint2)) != hipSuccess ||
      hipMalloc(&g->d_link, link.size() * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&g->d_rank_out, rank.size() * sizeof(uint16_t)) != hipSuccess ||
      hipMalloc(&g->d_ovl, nn) != hipSuccess ||
      hipMalloc(&g->d_name_rank, nn * sizeof(uint32_t)) != hipSuccess) {
    free_graph_device(g);
    return fail(ctx, ORH_E_NOMEM, "orh_graph_load: device allocation failed");
  }
  ORH_HIP(ctx, hipMemcpyAsync(g->d_recs, recs.data(), recs.size() * sizeof(uint2),
                              hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipMemcpyAsync(g->d_link, link.data(), link.size() * sizeof(uint32_t),
                              hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipMemcpyAsync(g->d_rank_out, rank.data(), rank.size() * sizeof(uint16_t),
                              hipMemcpyHostToDevice, ctx->stream));
  if (g->n_nodes) {
    ORH_HIP(ctx, hipMemcpyAsync(g->d_ovl, g->overloaded.data(), g->n_nodes, hipMemcpyHostToDevice,
                                ctx->stream));
    ORH_HIP(ctx, hipMemcpyAsync(g->d_name_rank, g->name_rank.data(), g->n_nodes * sizeof(uint32_t),
                                hipMemcpyHostToDevice, ctx->stream));
  }
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  mark("upload");
  return ORH_OK;
}

int orh_graph_patch_edges(orh_graph* g, uint32_t n, const uint32_t* idx, const uint32_t* w_out,
                          const uint32_t* w_in, const uint32_t* meta) {
  if (!g || (n && (!idx || !w_out || !w_in || !meta))) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  drain_deferred(ctx);  // the deferred phase 2 reads the graph
  if (!g->d_recs && n) return fail(ctx, ORH_E_STATE, "orh_graph_patch_edges: no graph loaded");
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = idx[i];
    if (e >= g->n_edges) return fail(ctx, ORH_E_INVALID, "orh_graph_patch_edges: bad edge index");
    if ((meta[i] & ORH_META_LINK_MASK) != (g->meta[e] & ORH_META_LINK_MASK))
      return fail(ctx, ORH_E_INVALID, "orh_graph_patch_edges: link id changed (use orh_graph_apply_delta)");
    if (g->meta[e] == ORH_META_EMPTY && meta[i] != ORH_META_EMPTY)
      return fail(ctx, ORH_E_INVALID, "orh_graph_patch_edges: free slot (use orh_graph_apply_delta)");
  }
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<std::pair<uint32_t, uint32_t>> edges;
  edges.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = idx[i];
    g->w_out[e] = w_out[i];
    g->w_in[e] = w_in[i];
    g->meta[e] = meta[i] & ~ORH_META_COL_OVERLOADED;
    edges.emplace_back(row_of(g, e), e);
  }
  std::sort(edges.begin(), edges.end());
  edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
  int rc = upload_records(g, edges);
  if (rc) return rc;
  recompute_bounds(g);
  return ORH_OK;
}

int orh_graph_apply_delta(orh_graph* g, uint32_t n_rows, const uint32_t* rows, const uint32_t* ptr,
                          const uint32_t* col, const uint32_t* w_out, const uint32_t* w_in,
                          const uint32_t* meta, uint32_t n_links) {
  if (!g || (n_rows && (!rows || !ptr))) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  drain_deferred(ctx);  // the deferred phase 2 reads the graph
  if (!g->d_recs) return fail(ctx, ORH_E_STATE, "orh_graph_apply_delta: no graph loaded");
  const uint32_t N = g->n_nodes;
  if (n_rows && ptr[0] != 0) return fail(ctx, ORH_E_INVALID, "orh_graph_apply_delta: ptr[0] != 0");
  std::vector<uint8_t> seen(N, 0);
  for (uint32_t i = 0; i < n_rows; ++i) {
    const uint32_t v = rows[i];
    if (v >= N || seen[v]) return fail(ctx, ORH_E_INVALID, "orh_graph_apply_delta: bad or repeated row");
    seen[v] = 1;
    if (ptr[i + 1] < ptr[i]) return fail(ctx, ORH_E_INVALID, "orh_graph_apply_delta: ptr not monotone");
    if (ptr[i + 1] - ptr[i] > g->row_ptr[v + 1] - g->row_ptr[v])
      return fail(ctx, ORH_E_UNSUPPORTED, "orh_graph_apply_delta: row " + std::to_string(v) +
                                              " outgrows its capacity (reload)");
  }
  const uint32_t n_ent = n_rows ? ptr[n_rows] : 0u;
  if (n_ent && (!col || !w_out || !w_in || !meta)) return fail(ctx, ORH_E_INVALID, "orh_graph_apply_delta: null array");
  for (uint32_t k = 0; k < n_ent; ++k) {
    if (col[k] >= N) return fail(ctx, ORH_E_INVALID, "orh_graph_apply_delta: col out of range");
    if (meta[k] != ORH_META_EMPTY && (meta[k] & ORH_META_LINK_MASK) >= std::max<uint32_t>(n_links, 1))
      return fail(ctx, ORH_E_INVALID, "orh_graph_apply_delta: link id >= n_links");
  }
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  for (uint32_t i = 0; i < n_rows; ++i) {
    const uint32_t v = rows[i], e0 = g->row_ptr[v], cap = g->row_ptr[v + 1] - e0;
    const uint32_t d = ptr[i + 1] - ptr[i];
    for (uint32_t j = 0; j < cap; ++j) {
      const uint32_t e = e0 + j;
      if (j < d) {
        const uint32_t k = ptr[i] + j;
        g->col[e] = meta[k] == ORH_META_EMPTY ? v : col[k];
        g->w_out[e] = w_out[k];
        g->w_in[e] = w_in[k];
        g->meta[e] = meta[k] == ORH_META_EMPTY ? meta[k] : meta[k] & ~ORH_META_COL_OVERLOADED;
      } else {
        g->col[e] = v;
        g->w_out[e] = g->w_in[e] = 1;
        g->meta[e] = ORH_META_EMPTY;
      }
    }
  }
  g->n_links = n_links;
  build_neighbours(g);
  for (uint32_t i = 0; i < n_rows; ++i)
    if (n_distinct(g, rows[i]) > 0xFFFFu)
      return fail(ctx, ORH_E_UNSUPPORTED, "orh_graph_apply_delta: more than 65535 neighbours (reload)");
  recompute_bounds(g);
  // the changed rows' device records, link ids and neighbour ranks
  std::vector<uint32_t> pos;
  std::vector<uint2> vals;
  std::vector<uint32_t> links;
  std::vector<uint16_t> ranks;
  for (uint32_t i = 0; i < n_rows; ++i) {
    const uint32_t v = rows[i];
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) {
      pos.push_back(g->pos[e]);
      vals.push_back(device_record(g, v, e));
      links.push_back(g->meta[e] & ORH_META_LINK_MASK);
      ranks.push_back(g->rank_out[e]);
    }
  }
  const uint32_t n = static_cast<uint32_t>(pos.size());
  if (n) {
    // staging: pos u32[n] | links u32[n] | vals uint2[n] | ranks u16[n]
    const size_t words = 2 * size_t{n} + 2 * size_t{n} + (size_t{n} + 1) / 2;
    std::vector<uint32_t> st(words, 0);
    std::memcpy(st.data(), pos.data(), 4 * size_t{n});
    std::memcpy(st.data() + n, links.data(), 4 * size_t{n});
    std::memcpy(st.data() + 2 * size_t{n}, vals.data(), 8 * size_t{n});
    std::memcpy(st.data() + 4 * size_t{n}, ranks.data(), 2 * size_t{n});
    if (st.size() > ctx->d_patch_cap) {
      (void)hipFree(ctx->d_patch);
      ctx->d_patch = nullptr;
      ctx->d_patch_cap = 0;
      ORH_HIP(ctx, hipMalloc(&ctx->d_patch, st.size() * sizeof(uint32_t)));
      ctx->d_patch_cap = st.size();
    }
    ORH_HIP(ctx, hipMemcpyAsync(ctx->d_patch, st.data(), st.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    ORH_HIP(ctx, orh::launch_scatter_rows(
                     g->d_recs, g->d_link, g->d_rank_out, ctx->d_patch,
                     reinterpret_cast<const uint2*>(ctx->d_patch + 2 * size_t{n}), ctx->d_patch + n,
                     reinterpret_cast<const uint16_t*>(ctx->d_patch + 4 * size_t{n}), n, ctx->stream));
    ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // staging is a local
  }
  g->ms_dirty = true;
  g->wms_dirty = true;
  g->gen = next_graph_gen();  // staged requests hold neighbour lists of the old rows
  return ORH_OK;
}

int orh_graph_patch_nodes(orh_graph* g, uint32_t n, const uint32_t* idx, const uint8_t* ovl) {
  if (!g || (n && (!idx || !ovl))) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  drain_deferred(ctx);  // the deferred phase 2 reads the graph
  if (!g->d_recs && n) return fail(ctx, ORH_E_STATE, "orh_graph_patch_nodes: no graph loaded");
  for (uint32_t i = 0; i < n; ++i)
    if (idx[i] >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_graph_patch_nodes: bad node");
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<std::pair<uint32_t, uint32_t>> edges;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t v = idx[i];
    g->overloaded[v] = ovl[i] ? 1 : 0;
    // v's own records carry its row bit
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) edges.emplace_back(v, e);
  }
  std::sort(edges.begin(), edges.end());
  edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
  if (n && g->n_nodes)  // the whole flag array: one copy instead of one per node
    ORH_HIP(ctx, hipMemcpyAsync(g->d_ovl, g->overloaded.data(), g->n_nodes, hipMemcpyHostToDevice,
                                ctx->stream));
  int rc = upload_records(g, edges);  // synchronizes the stream
  if (rc) return rc;
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_graph_device_flags(const orh_graph* g, const uint8_t** d_overloaded) {
  if (!g || !d_overloaded) return ORH_E_INVALID;
  if (!g->d_ovl) return fail(g->ctx, ORH_E_STATE, "orh_graph_device_flags: no graph loaded");
  *d_overloaded = g->d_ovl;
  return ORH_OK;
}

int orh_graph_flags(const orh_graph* g, uint32_t* flags) {
  if (!g || !flags) return ORH_E_INVALID;
  *flags = (g->has_zero ? ORH_GRAPH_ZERO_METRIC : 0u) | (wide_metrics(g) ? ORH_GRAPH_WIDE_METRIC : 0u);
  return ORH_OK;
}

int orh_graph_info(const orh_graph* g, uint32_t* n_nodes, uint32_t* n_edges) {
  if (!g) return ORH_E_INVALID;
  if (n_nodes) *n_nodes = g->n_nodes;
  if (n_edges) *n_edges = g->n_edges;
  return ORH_OK;
}

int orh_graph_neighbors(const orh_graph* g, uint32_t src, uint32_t* out, uint32_t cap,
                        uint32_t* n_out) {
  if (!g || !n_out) return ORH_E_INVALID;
  if (src >= g->n_nodes) return ORH_E_INVALID;
  const uint32_t n = n_distinct(g, src);
  *n_out = n;
  for (uint32_t i = 0; i < n && i < cap; ++i) out[i] = g->dn[g->dn_ptr[src] + i];
  return ORH_OK;
}

int orh_spf_words(const orh_graph* g, const uint32_t* srcs, uint32_t n, uint32_t* out) {
  if (!g || !out || (n && !srcs)) return ORH_E_INVALID;
  uint32_t mx = 1;
  for (uint32_t i = 0; i < n; ++i) {
    if (srcs[i] >= g->n_nodes) return ORH_E_INVALID;
    mx = std::max(mx, n_distinct(g, srcs[i]));
  }
  *out = (mx + 31) / 32;
  return ORH_OK;
}

// The exact kernel (LinkState::runSpf's own extraction order): one wave per
// requested row, nothing shared between rows. Rows run in chunks whose heap
// state fits a bounded scratch when it is too large for LDS.
static int run_exact(orh_graph* g, const orh_spf_request* req, uint32_t words, uint32_t* d_dist32,
                     uint64_t* d_dist64, uint32_t* d_nh, uint32_t* d_rank) {
  orh_ctx* ctx = g->ctx;
  const uint32_t n_src = req->n_src, N = g->n_nodes;
  uint32_t max_nbr = 1;
  for (uint32_t i = 0; i < n_src; ++i) {
    if (req->h_srcs[i] >= N) return fail(ctx, ORH_E_INVALID, "exact SPF: source out of range");
    max_nbr = std::max(max_nbr, n_distinct(g, req->h_srcs[i]));
  }
  if (words < (max_nbr + 31) / 32) return fail(ctx, ORH_E_INVALID, "exact SPF: words too small");
  hipSetDevice(ctx->device);
  // staging: srcs[n_src] | ign_ptr[n_src + 1] ign[..] (ignore sets sorted for
  // the device binary search)
  const bool has_ign = req->h_ignore_ptr != nullptr;
  std::vector<uint32_t> staging(req->h_srcs, req->h_srcs + n_src);
  const size_t off_ign_ptr = staging.size();
  if (has_ign) {
    const size_t off_ign = off_ign_ptr + n_src + 1;
    staging.resize(off_ign);
    staging[off_ign_ptr] = 0;
    for (uint32_t i = 0; i < n_src; ++i) {
      std::vector<uint32_t> set(req->h_ignore_links + req->h_ignore_ptr[i],
                                req->h_ignore_links + req->h_ignore_ptr[i + 1]);
      std::sort(set.begin(), set.end());
      staging.insert(staging.end(), set.begin(), set.end());
      staging[off_ign_ptr + i + 1] = static_cast<uint32_t>(staging.size() - off_ign);
    }
  }
  int rc = ensure_req(ctx, staging.size());
  if (rc) return rc;
  ctx->req_key.clear();  // the staged request of orh_spf_run is overwritten
  ORH_HIP(ctx, hipMemcpyAsync(ctx->d_req, staging.data(), staging.size() * 4, hipMemcpyHostToDevice,
                              ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // staging is a local
  orh::ExactArgs a{};
  a.n_nodes = N;
  a.words = words;
  a.use_link_metric = req->use_link_metric;
  a.ell_k = g->ell_k;
  a.recs = g->d_recs;
  a.link = g->d_link;
  a.rank_out = g->d_rank_out;
  a.name_rank = g->d_name_rank;
  a.ignore_links = has_ign ? ctx->d_req + off_ign_ptr + n_src + 1 : nullptr;
  const size_t state = orh::exact_state_bytes(N, words);
  uint32_t chunk = n_src;
  if (state > ctx->lds_limit) {  // per-row global heap state, at most 1 GiB at a time
    chunk = static_cast<uint32_t>(std::max<size_t>(1, std::min<size_t>(n_src, (size_t{1} << 30) / state)));
    rc = ensure_bytes(ctx, &ctx->d_exact, &ctx->d_exact_cap, state * chunk);
    if (rc) return rc;
    a.scratch = ctx->d_exact;
    a.scratch_stride = state;
  }
  ORH_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  for (uint32_t r0 = 0; r0 < n_src; r0 += chunk) {
    const size_t base = static_cast<size_t>(r0) * N;
    a.n_rows = std::min(chunk, n_src - r0);
    a.srcs = ctx->d_req + r0;
    a.ignore_ptr = has_ign ? ctx->d_req + off_ign_ptr + r0 : nullptr;
    a.out_dist32 = d_dist32 ? d_dist32 + base : nullptr;
    a.out_dist64 = d_dist64 ? d_dist64 + base : nullptr;
    a.out_nh = d_nh + base * words;
    a.out_rank = d_rank ? d_rank + base : nullptr;
    hipError_t e = orh::launch_exact(a, ctx->lds_limit, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "exact SPF kernel launch");
  }
  ORH_HIP(ctx, hipEventRecord(ctx->evm, ctx->stream));
  ORH_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  orh_spf_info info{};
  info.variant = static_cast<int32_t>(orh::SpfVariant::kExact);
  info.rows = n_src;
  ctx->last_info = info;
  ctx->counters.spf_runs += n_src;
  ctx->counters.spf_launches += 1;
  ctx->counters.last_kernel_ms = -1.0;
  return ORH_OK;
}

// ---- what-if repair (whatif_kernels.hip) ----------------------------------
// per-record reverse records and per-link CSR entries of the current structure
static int ensure_rev(orh_graph* g) {
  if (g->d_rev && g->rev_gen == g->gen) return ORH_OK;
  orh_ctx* ctx = g->ctx;
  const uint32_t L = g->n_links;
  g->link_ent.assign(2 * static_cast<size_t>(L), ~0u);
  for (uint32_t e = 0; e < g->n_edges; ++e) {
    if (g->meta[e] == ORH_META_EMPTY) continue;
    const uint32_t l = g->meta[e] & ORH_META_LINK_MASK;
    if (l >= L) continue;
    uint32_t* ent = &g->link_ent[2 * static_cast<size_t>(l)];
    (ent[0] == ~0u ? ent[0] : ent[1]) = e;
  }
  std::vector<uint32_t> rev(std::max<uint32_t>(g->n_recs, 1), 0u);
  for (uint32_t e = 0; e < g->n_recs && e < rev.size(); ++e) rev[e] = e;
  for (uint32_t l = 0; l < L; ++l) {
    const uint32_t a = g->link_ent[2 * l], b = g->link_ent[2 * l + 1];
    if (a == ~0u || b == ~0u) continue;
    rev[g->pos[a]] = g->pos[b];
    rev[g->pos[b]] = g->pos[a];
  }
  if (!g->d_rev) ORH_HIP(ctx, hipMalloc(&g->d_rev, rev.size() * sizeof(uint32_t)));
  ORH_HIP(ctx, hipMemcpyAsync(g->d_rev, rev.data(), rev.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                              ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // rev is a local
  g->rev_gen = g->gen;
  return ORH_OK;
}

// LDS caps of the repair pass: 2,048 nodes / 8,192 edges when that state fits
// the LDS (C4 what-if 2.05 -> 1.93 ms against 1,024 / 4,096: fewer requests
// fall through to the global-slot pass), else 1,024 / 4,096
static void repair_caps(const orh_ctx* ctx, uint32_t n_nodes, uint32_t* cap_a, uint32_t* cap_e) {
  if (ctx->rep_cap_a) {
    *cap_a = ctx->rep_cap_a;
    *cap_e = ctx->rep_cap_e;
  } else if (orh::repair_lds_bytes(n_nodes, 2048, 8192) <= ctx->lds_limit) {
    *cap_a = 2048;
    *cap_e = 8192;
  } else {
    *cap_a = 1024;
    *cap_e = 4096;
  }
}

constexpr uint32_t kRepairSlots = 64;       // tier 3: whole-graph state in global memory
constexpr size_t kRepairSlotBudget = 1ull << 30;  // bytes for all slots
constexpr uint32_t kRepairMaxIgnore = 8;  // link-failure sets; KSP2 k = 2 sets are whole paths

// What-if search plan for the graph: the repair needs one mask word per
// source, no zero metrics (the exact kernel's extraction order decides those
// first hops) and a full-search plan for the no-slot fallback
static int whatif_plan(orh_graph* g, bool use_link_metric, uint64_t* bound, bool* uniform) {
  orh_ctx* ctx = g->ctx;
  if (!g->d_recs || g->n_nodes == 0) return fail(ctx, ORH_E_STATE, "what-if: no graph loaded");
  if (use_link_metric && g->has_zero)
    return fail(ctx, ORH_E_UNSUPPORTED, "what-if: zero link metrics need the exact kernel");
  const uint32_t N = g->n_nodes;
  *uniform = !use_link_metric || g->min_out == g->max_out;
  const uint32_t w0 = use_link_metric ? g->max_out : 1u;
  *bound = *uniform ? static_cast<uint64_t>(N) * w0
           : use_link_metric ? g->sum_max_metric / 2 + g->max_metric
                             : static_cast<uint64_t>(g->n_links) + 1;
  uint32_t cap_a = 0, cap_e = 0;
  repair_caps(ctx, N, &cap_a, &cap_e);
  if (orh::repair_lds_bytes(N, cap_a, cap_e) > ctx->lds_limit)
    return fail(ctx, ORH_E_UNSUPPORTED, "what-if: repair state exceeds LDS");
  const orh::SpfPlan fp = orh::plan_spf(N, *uniform, *bound, g->ell_k, ctx->lds_limit, false, orh::SpfMode::kGlobal);
  if (fp.variant == orh::SpfVariant::kUnsupported)
    return fail(ctx, ORH_E_UNSUPPORTED, "what-if: no search plan for this graph");
  return ORH_OK;
}

// Can run_repair take this ignore-set batch? (sources repeat, small sets,
// one mask word, the LDS state fits, and the fallback search has a plan)
static bool repair_eligible(orh_graph* g, const orh_spf_request* req, uint32_t words) {
  const orh_ctx* ctx = g->ctx;
  if (ctx->repair_mode == 0 || words != 1 || !req->h_ignore_ptr) return false;
  uint64_t bound = 0;
  bool uniform = false;
  const std::string err = g->ctx->err;
  const int rc = whatif_plan(g, req->use_link_metric != 0, &bound, &uniform);
  g->ctx->err = err;  // not eligible is not an error of this call
  if (rc) return false;
  if (ctx->repair_mode >= 2) return true;
  for (uint32_t i = 0; i < req->n_src; ++i)
    if (req->h_ignore_ptr[i + 1] - req->h_ignore_ptr[i] > kRepairMaxIgnore) return false;
  std::vector<uint32_t> s(req->h_srcs, req->h_srcs + req->n_src);
  std::sort(s.begin(), s.end());
  const size_t m = static_cast<size_t>(std::unique(s.begin(), s.end()) - s.begin());
  return 2 * m <= req->n_src;
}

}  // extern "C"

// A what-if job (include/openr_hip.h): the plain rows of its sources, then
// any number of request batches repaired from them
// run slots a job cycles through: run r + kRunSlots reuses run r's queues,
// staging and slot memory (and waits for its side part)
constexpr int kRunSlots = 3;

struct orh_whatif {
  orh_graph* g = nullptr;
  uint64_t gen = 0;  // graph structure the base rows belong to
  int32_t use_link_metric = 1;
  bool uniform = false;
  uint64_t bound = 0;
  std::vector<uint32_t> srcs;
  uint32_t* d_base = nullptr;  // dist rows [m][N], then mask rows [m][N]
  size_t base_cap = 0;         // bytes
  // runs cycle through kRunSlots slots, each with its request staging (pinned
  // host + device), its work queues / counters / fallback flags, and the
  // side-stream part of its last run: the repair tiers of run r run on
  // `side` (and t3[slot]) while run r + 1's seed / copy run on the context
  // stream
  hipStream_t side = nullptr;
  uint32_t* h_stage[kRunSlots] = {};
  uint32_t* d_stage[kRunSlots] = {};
  size_t stage_cap[kRunSlots] = {};  // u32, both sides
  hipEvent_t stage_ev[kRunSlots] = {};  // upload done
  uint32_t* d_work[kRunSlots] = {};     // queues [3][n] | counters | fallback flags [n]
  size_t work_cap[kRunSlots] = {};
  hipEvent_t front_ev[kRunSlots] = {};  // context-stream part done
  hipEvent_t side_ev[kRunSlots] = {};   // side-stream part done
  bool pending[kRunSlots] = {};             // side part not yet joined into the context stream
  uintptr_t out_lo[kRunSlots] = {}, out_hi[kRunSlots] = {};  // output span of that run (hazard checks)
  int cur = 0;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;  // create .. last flush
  uint64_t requests = 0;
  // tier-3 slots: the context's (when no other job holds them) or the job's own
  uint8_t* own_slots = nullptr;
  size_t own_slots_cap = 0;
  // labels of the full searches that take the slot tier's largest repairs
  // (side stream only, so one buffer serves both run slots)
  void* d_full_lab = nullptr;
  size_t full_lab_cap = 0;
  uint32_t flags = 0;  // ORH_WHATIF_* job flags
  // the slot tier of a run on a stream of its own (t3[run % kT3]), with its
  // slot's memory, after event mid_ev[slot] (tiers 1 and 2 done on `side`):
  // the next run's small tiers start without waiting for its largest repairs
  // two streams, by run parity: with the context stream and `side` that is
  // HIP's 4 hardware queues (GPU_MAX_HW_QUEUES); a fifth stream would share
  // a queue with `side` and hold its next tiers behind a slot tier
  static constexpr int kT3 = 2;
  hipStream_t t3[kT3] = {};
  uint64_t runs = 0;
  hipEvent_t mid_ev[kRunSlots] = {};
  uint8_t* t3_slots[kRunSlots] = {};
  size_t t3_slots_cap[kRunSlots] = {};
};

namespace {

int whatif_stage(orh_whatif* job, size_t words, uint32_t** h, uint32_t** d) {
  orh_ctx* ctx = job->g->ctx;
  const int c = job->cur;
  if (job->stage_ev[c]) ORH_HIP(ctx, hipEventSynchronize(job->stage_ev[c]));  // its last upload is done
  if (words > job->stage_cap[c]) {
    if (job->h_stage[c]) hipHostFree(job->h_stage[c]);
    hipFree(job->d_stage[c]);
    job->h_stage[c] = nullptr;
    job->d_stage[c] = nullptr;
    job->stage_cap[c] = 0;
    const size_t cap = std::max<size_t>(words + words / 4, 4096);
    ORH_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&job->h_stage[c]), cap * 4, hipHostMallocDefault));
    ORH_HIP(ctx, hipMalloc(&job->d_stage[c], cap * 4));
    job->stage_cap[c] = cap;
  }
  if (!job->stage_ev[c]) ORH_HIP(ctx, hipEventCreateWithFlags(&job->stage_ev[c], hipEventDisableTiming));
  *h = job->h_stage[c];
  *d = job->d_stage[c];
  return ORH_OK;
}

// one batch of requests of a job: seed and copy and the small repair tiers
// on the context stream; the large tiers, the slot tier (t3 streams) and,
// without slots, the full search for what outgrew tier 2 on the job's side
// streams, over job-owned memory (slots, labels), joined back into the
// context stream through side_ev
int whatif_run(orh_whatif* job, uint32_t n_req, const uint32_t* src_idx, const uint32_t* ign_ptr,
               const uint32_t* ign_links, uint32_t* d_dist, uint32_t* d_nh, uint32_t* d_info) {
  orh_graph* g = job->g;
  orh_ctx* ctx = g->ctx;
  const uint32_t N = g->n_nodes, m = static_cast<uint32_t>(job->srcs.size());
  for (uint32_t i = 0; i < n_req; ++i)
    if (src_idx[i] >= m) return fail(ctx, ORH_E_INVALID, "orh_whatif_run: source index out of range");
  // staging: base_row[n] | srcs[n] | ign_ptr[n+1] | ign[..] | cut_ptr[n+1] | (pad to 16 B) cuts uint4[..]
  const uint32_t n_ign = ign_ptr[n_req];
  size_t n_cuts = 0;
  for (uint32_t k = 0; k < n_ign; ++k) {
    const uint32_t l = ign_links[k];
    if (l < g->n_links) n_cuts += (g->link_ent[2 * static_cast<size_t>(l)] != ~0u) + (g->link_ent[2 * static_cast<size_t>(l) + 1] != ~0u);
  }
  const size_t off_src = n_req, off_ip = 2 * size_t{n_req}, off_ign = off_ip + n_req + 1;
  const size_t off_cp = off_ign + n_ign;
  const size_t off_cuts = (off_cp + n_req + 1 + 3) & ~size_t{3};
  const size_t words = off_cuts + 4 * n_cuts + 4;
  {
    // slot `cur` is reused: its previous run's side part must be done (the
    // context stream waits); so must the other slot's when it writes rows
    // this run overwrites
    const int c = job->cur;
    const uintptr_t lo = std::min(reinterpret_cast<uintptr_t>(d_dist), reinterpret_cast<uintptr_t>(d_nh));
    const uintptr_t hi = std::max(reinterpret_cast<uintptr_t>(d_dist), reinterpret_cast<uintptr_t>(d_nh)) +
                         size_t{n_req} * N * 4;
    for (int k = 0; k < kRunSlots; ++k)
      if (job->pending[k] && (k == c || (lo < job->out_hi[k] && job->out_lo[k] < hi))) {
        ORH_HIP(ctx, hipStreamWaitEvent(ctx->stream, job->side_ev[k], 0));
        job->pending[k] = false;
      }
  }
  uint32_t *h = nullptr, *d = nullptr;
  int rc = whatif_stage(job, words, &h, &d);
  if (rc) return rc;
  std::memcpy(h, src_idx, n_req * 4ull);
  for (uint32_t i = 0; i < n_req; ++i) h[off_src + i] = job->srcs[src_idx[i]];
  uint32_t* hp = h + off_ip;
  uint32_t* hi = h + off_ign;
  uint32_t* hc = h + off_cp;
  uint4* cuts = reinterpret_cast<uint4*>(h + off_cuts);
  const std::vector<uint32_t>& erow = entry_rows(g);
  size_t ni = 0, nc = 0;
  hp[0] = 0;
  hc[0] = 0;
  for (uint32_t i = 0; i < n_req; ++i) {
    uint32_t* set = hi + ni;
    size_t len = 0;
    for (uint32_t k = ign_ptr[i]; k < ign_ptr[i + 1]; ++k) set[len++] = ign_links[k];
    std::sort(set, set + len);  // bsearch on device
    len = static_cast<size_t>(std::unique(set, set + len) - set);
    for (size_t k = 0; k < len; ++k) {
      const uint32_t l = set[k];
      if (l >= g->n_links) continue;
      for (int e2 = 0; e2 < 2; ++e2) {
        const uint32_t e = g->link_ent[2 * static_cast<size_t>(l) + e2];
        if (e == ~0u) continue;
        cuts[nc++] = make_uint4(erow[e], g->col[e], g->pos[e], 0u);
      }
    }
    ni += len;
    hp[i + 1] = static_cast<uint32_t>(ni);
    hc[i + 1] = static_cast<uint32_t>(nc);
  }
  const int c = job->cur;
  job->cur = (job->cur + 1) % kRunSlots;
  ORH_HIP(ctx, hipMemcpyAsync(d, h, words * 4, hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipEventRecord(job->stage_ev[c], ctx->stream));

  const size_t work = 3 * size_t{n_req} + orh::kWhatifCounters + n_req;
  if (work > job->work_cap[c]) {
    if (job->pending[c]) ORH_HIP(ctx, hipStreamSynchronize(job->side));  // its old buffer may be in use
    hipFree(job->d_work[c]);
    job->d_work[c] = nullptr;
    job->work_cap[c] = 0;
    ORH_HIP(ctx, hipMalloc(&job->d_work[c], work * 4));
    job->work_cap[c] = work;
  }
  uint32_t* counters = job->d_work[c] + 3 * size_t{n_req};
  uint32_t* flags = counters + orh::kWhatifCounters;
  ORH_HIP(ctx, hipMemsetAsync(counters, 0, (orh::kWhatifCounters + n_req) * 4ull, ctx->stream));
  const size_t slot_bytes = orh::repair_slot_bytes(N, g->n_recs);
  const uint32_t n_slots = static_cast<uint32_t>(std::min<size_t>(
      std::min<size_t>(kRepairSlots, n_req), kRepairSlotBudget / std::max<size_t>(slot_bytes, 1)));
  uint8_t* slot_mem = nullptr;
  static const uint32_t full_env = [] {
    const char* e = getenv("ORH_WHATIF_FULL");
    return e ? static_cast<uint32_t>(atoi(e)) : 0u;
  }();
  static const bool t3_split = [] {  // ORH_WHATIF_T3_SPLIT=0: the slot tier stays on `side` (A/B)
    const char* e = getenv("ORH_WHATIF_T3_SPLIT");
    return !(e && atoi(e) == 0);
  }();
  // full searches for the slot tier's queue: ORH_WHATIF_FULL=n (A/B), or the
  // job's ORH_WHATIF_SEARCH_LARGE (16 per run)
  static const uint32_t large_cap = [] {  // ORH_WHATIF_SEARCH_CAP (A/B): the flag's searches per run
    const char* e = getenv("ORH_WHATIF_SEARCH_CAP");
    // 256: tier 1's whole overflow of a C4 block (profiles/r06/an_skip_t2_ab/);
    // 8 / 16 / 32 behind tier 2: profiles/r06/ab_search_cap.txt
    return e && atoi(e) > 0 ? static_cast<uint32_t>(atoi(e)) : 256u;
  }();
  const uint32_t full_n = full_env ? full_env : (job->flags & ORH_WHATIF_SEARCH_LARGE) ? large_cap : 0u;
  const bool split = n_slots && full_n == 0 && t3_split;
  if (split) {
    // run slot c's own slot memory, grown only with its stream idle
    if (n_slots * slot_bytes > job->t3_slots_cap[c]) {
      for (hipStream_t t : job->t3) ORH_HIP(ctx, hipStreamSynchronize(t));
      hipFree(job->t3_slots[c]);
      job->t3_slots[c] = nullptr;
      job->t3_slots_cap[c] = 0;
      ORH_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&job->t3_slots[c]), n_slots * slot_bytes));
      job->t3_slots_cap[c] = n_slots * slot_bytes;
    }
    slot_mem = job->t3_slots[c];
  } else if (n_slots) {
    // the context's slots while no other job's side stream may use them,
    // else the job's own; grown only with the side stream idle
    if (!ctx->slots_owner) ctx->slots_owner = job;
    const bool borrowed = ctx->slots_owner == job;
    uint8_t** p = borrowed ? &ctx->d_rep_slots : &job->own_slots;
    size_t* cap = borrowed ? &ctx->d_rep_slots_cap : &job->own_slots_cap;
    if (n_slots * slot_bytes > *cap) ORH_HIP(ctx, hipStreamSynchronize(job->side));
    rc = ensure_bytes(ctx, p, cap, n_slots * slot_bytes);
    if (rc) return rc;
    slot_mem = *p;
  }
  const size_t nd = static_cast<size_t>(m) * N;
  orh::RepairArgs ra{};
  ra.n_nodes = N;
  ra.n_req = n_req;
  ra.use_link_metric = job->use_link_metric;
  repair_caps(ctx, N, &ra.cap_a, &ra.cap_e);
  ra.recs = g->d_recs;
  ra.link = g->d_link;
  ra.rank_out = g->d_rank_out;
  ra.rev = g->d_rev;
  ra.ovl = g->d_ovl;
  ra.base_dist = job->d_base;
  ra.base_nh = job->d_base + nd;
  ra.base_row = d;
  ra.srcs = d + off_src;
  ra.ign_ptr = d + off_ip;
  ra.ign = d + off_ign;
  ra.cut_ptr = d + off_cp;
  ra.cuts = reinterpret_cast<const uint4*>(d + off_cuts);
  ra.out_dist = d_dist;
  ra.out_nh = d_nh;
  ra.fallback = flags;
  ra.info = d_info;
  ra.queues = job->d_work[c];
  ra.counters = counters;
  ra.slot_mem = slot_mem;
  ra.slot_bytes = slot_bytes;
  ra.n_slots = n_slots;
  ra.n_recs = g->n_recs;
  ra.n_cu = ctx->n_cu;
  ra.share_base = (job->flags & ORH_WHATIF_SHARE_BASE) ? 1u : 0u;
  // ORH_WHATIF_FULL=n (A/B, default 0): the slot tier's queue goes to full
  // searches first, up to n rows (labels within 1 GB). C4: 79 requests per
  // job searched in full 30.7-31.2 ms against 29.6 ms in slots
  // (profiles/r03/r_c4_full_search_ab.txt): the slots stay the default
  if (n_slots) {
    const size_t by_mem = (size_t{1} << 30) / (static_cast<size_t>(N) * 8);
    ra.full_cap = static_cast<uint32_t>(std::min<size_t>({full_n, by_mem, n_req}));
    // with full searches, tier 1's overflow goes to them directly: tier 2
    // between them put its 0.4 ms on a short job's critical path (C4 block of
    // 8: 5.34 -> 4.73 ms, profiles/r06/an_skip_t2_ab/); ORH_WHATIF_SKIP_T2=0
    // keeps tier 2 (A/B)
    static const bool skip_t2 = [] {
      const char* e = getenv("ORH_WHATIF_SKIP_T2");
      return !(e && atoi(e) == 0);
    }();
    ra.skip_large = (skip_t2 && ra.full_cap) ? 1u : 0u;
    if (ra.full_cap) {
      const size_t need = static_cast<size_t>(ra.full_cap) * N * 8;
      if (need > job->full_lab_cap) {
        ORH_HIP(ctx, hipStreamSynchronize(job->side));  // the old buffer may be in use
        hipFree(job->d_full_lab);
        job->d_full_lab = nullptr;
        job->full_lab_cap = 0;
        ORH_HIP(ctx, hipMalloc(&job->d_full_lab, need));
        job->full_lab_cap = need;
      }
    }
  }
  hipError_t e = orh::launch_repair_front(ra, g->ell_k, ctx->lds_limit, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "what-if repair launch");
  ORH_HIP(ctx, hipEventRecord(job->front_ev[c], ctx->stream));
  // the large repairs on the side stream, after this run's front part; the
  // previous side part is ordered before them on that stream
  ORH_HIP(ctx, hipStreamWaitEvent(job->side, job->front_ev[c], 0));
  hipStream_t t3s = job->t3[job->runs % orh_whatif::kT3];
  ++job->runs;
  e = split ? orh::launch_repair_back_split(ra, g->ell_k, ctx->lds_limit, job->side, t3s, job->mid_ev[c])
            : orh::launch_repair_back(ra, g->ell_k, ctx->lds_limit, job->side);
  if (e != hipSuccess) return hip_fail(ctx, e, "what-if repair launch (large tiers)");
  if (n_slots && ra.full_cap) {
    // workgroup b searches request queue[b] while b < the queue's length
    const uint32_t q = orh::repair_slot_queue(ra);
    orh::SpfPlan fp = orh::plan_spf(N, job->uniform, job->bound, g->ell_k, ctx->lds_limit, false,
                                    orh::SpfMode::kGlobal);
    if (fp.variant == orh::SpfVariant::kUnsupported)
      return fail(ctx, ORH_E_UNSUPPORTED, "what-if: no search plan for this graph");
    fp.variant = orh::SpfVariant::kGlobalNh;
    fp.block = 1024;
    orh::SpfArgs a{};
    a.n_nodes = N;
    a.n_out = n_req;
    a.recs = g->d_recs;
    a.link = g->d_link;
    a.srcs = ra.srcs;
    a.ignore_ptr = ra.ign_ptr;
    a.ignore_links = ra.ign;
    a.use_link_metric = job->use_link_metric;
    a.w0 = job->use_link_metric ? g->max_out : 1u;
    a.delta = job->uniform ? a.w0
                           : std::max<uint32_t>(1u, static_cast<uint32_t>(
                                                        static_cast<uint64_t>(g->mean_out) * ctx->delta_pct / 100u));
    a.out_dist = d_dist;
    a.scratch = ctx->d_scratch;
    a.labels = static_cast<unsigned long long*>(job->d_full_lab);
    a.out_nh = d_nh;
    a.words = 1;
    a.rank_out = g->d_rank_out;
    a.row_list = ra.queues + static_cast<size_t>(q) * n_req;
    a.row_count = ra.counters + 2 * q;
    e = orh::launch_spf(fp, a, ra.full_cap, job->side);
    if (e != hipSuccess) return hip_fail(ctx, e, "what-if full-search launch");
  }
  if (n_slots == 0) {
    // no slot fits the budget: the requests that outgrew tier 2 are searched
    // in full (spf_global_nh_kernel with the flags as its row mask)
    orh::SpfPlan fp = orh::plan_spf(N, job->uniform, job->bound, g->ell_k, ctx->lds_limit, false,
                                    orh::SpfMode::kGlobal);
    fp.variant = orh::SpfVariant::kGlobalNh;
    fp.block = 1024;  // only the flagged rows search; the rest exit at once
    // job-owned labels: this search runs on the job's side stream, which
    // later work on the context stream (searches over ctx->d_labels) does
    // not wait for
    const size_t need = static_cast<size_t>(n_req) * N * 8;
    if (need > job->full_lab_cap) {
      ORH_HIP(ctx, hipStreamSynchronize(job->side));  // the old buffer may be in use
      hipFree(job->d_full_lab);
      job->d_full_lab = nullptr;
      job->full_lab_cap = 0;
      ORH_HIP(ctx, hipMalloc(&job->d_full_lab, need));
      job->full_lab_cap = need;
    }
    orh::SpfArgs a{};
    a.n_nodes = N;
    a.n_out = n_req;
    a.recs = g->d_recs;
    a.link = g->d_link;
    a.srcs = ra.srcs;
    a.ignore_ptr = ra.ign_ptr;
    a.ignore_links = ra.ign;
    a.use_link_metric = job->use_link_metric;
    a.w0 = job->use_link_metric ? g->max_out : 1u;
    a.delta = job->uniform ? a.w0
                           : std::max<uint32_t>(1u, static_cast<uint32_t>(
                                                        static_cast<uint64_t>(g->mean_out) * ctx->delta_pct / 100u));
    a.out_dist = d_dist;
    a.scratch = ctx->d_scratch;  // unused: every row is < n_out
    a.labels = static_cast<unsigned long long*>(job->d_full_lab);
    a.out_nh = d_nh;
    a.words = 1;
    a.rank_out = g->d_rank_out;
    a.row_mask = flags;
    e = orh::launch_spf(fp, a, n_req, job->side);
    if (e != hipSuccess) return hip_fail(ctx, e, "what-if fallback launch");
  }
  // the run's side part ends with its slot tier (t3[c], ordered after tiers
  // 1 and 2 through mid_ev[c]) or on `side`
  ORH_HIP(ctx, hipEventRecord(job->side_ev[c], split ? t3s : job->side));
  job->pending[c] = true;
  job->out_lo[c] = std::min(reinterpret_cast<uintptr_t>(d_dist), reinterpret_cast<uintptr_t>(d_nh));
  job->out_hi[c] = std::max(reinterpret_cast<uintptr_t>(d_dist), reinterpret_cast<uintptr_t>(d_nh)) +
                   size_t{n_req} * N * 4;
  job->requests += n_req;
  ctx->counters.spf_runs += n_req;  // one runSpf per request (LinkState.cpp:815)
  ctx->counters.spf_launches += 1;
  ctx->counters.last_kernel_ms = -1.0;
  return ORH_OK;
}

// the side-stream parts of every run so far join the context stream: work
// queued on it afterwards sees all of the job's rows
int whatif_flush(orh_whatif* job) {
  orh_ctx* ctx = job->g->ctx;
  for (int c = 0; c < kRunSlots; ++c)
    if (job->pending[c]) {
      ORH_HIP(ctx, hipStreamWaitEvent(ctx->stream, job->side_ev[c], 0));
      job->pending[c] = false;
    }
  ORH_HIP(ctx, hipEventRecord(job->ev_end, ctx->stream));
  return ORH_OK;
}

// the plain SPFs of the job's sources into its base rows, on the graph as it
// is now (create, and orh_whatif_refresh after topology changes); the side
// parts of earlier runs, which read the old rows, are joined first
int whatif_base(orh_whatif* job) {
  orh_graph* g = job->g;
  orh_ctx* ctx = g->ctx;
  uint64_t bound = 0;
  bool uniform = false;
  int rc = whatif_plan(g, job->use_link_metric != 0, &bound, &uniform);
  if (rc) return rc;
  for (uint32_t s : job->srcs) {
    if (s >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "what-if: source out of range");
    if (n_distinct(g, s) > 32) return fail(ctx, ORH_E_UNSUPPORTED, "what-if: a source has more than 32 neighbours");
  }
  job->uniform = uniform;
  job->bound = bound;
  rc = ensure_rev(g);
  if (rc) return rc;
  for (int c = 0; c < kRunSlots; ++c)
    if (job->pending[c]) {
      ORH_HIP(ctx, hipStreamWaitEvent(ctx->stream, job->side_ev[c], 0));
      job->pending[c] = false;
    }
  const uint32_t m = static_cast<uint32_t>(job->srcs.size());
  const size_t nd = static_cast<size_t>(std::max<uint32_t>(m, 1)) * g->n_nodes;
  if (nd * 8 > job->base_cap) {
    ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    hipFree(job->d_base);
    job->d_base = nullptr;
    job->base_cap = 0;
    if (hipMalloc(&job->d_base, nd * 8) != hipSuccess) return fail(ctx, ORH_E_NOMEM, "what-if: base rows");
    job->base_cap = nd * 8;
  }
  ORH_HIP(ctx, hipEventRecord(job->ev_begin, ctx->stream));
  if (m) {
    // internal searches: spf_runs counts the requests
    orh_spf_request br{};
    br.h_srcs = job->srcs.data();
    br.n_src = m;
    br.use_link_metric = job->use_link_metric;
    const orh_counters c0 = ctx->counters;
    rc = orh_spf_run(g, &br, 1, job->d_base, job->d_base + static_cast<size_t>(m) * g->n_nodes);
    ctx->counters = c0;
    if (rc) return rc;
  }
  ORH_HIP(ctx, hipEventRecord(job->ev_end, ctx->stream));
  job->gen = g->gen;
  return ORH_OK;
}

int whatif_create(orh_graph* g, const uint32_t* h_srcs, uint32_t n_srcs, int32_t use_link_metric,
                  orh_whatif** out) {
  orh_ctx* ctx = g->ctx;
  uint64_t bound = 0;
  bool uniform = false;
  int rc = whatif_plan(g, use_link_metric != 0, &bound, &uniform);
  if (rc) return rc;
  for (uint32_t i = 0; i < n_srcs; ++i) {
    if (h_srcs[i] >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_whatif_create: source out of range");
    if (n_distinct(g, h_srcs[i]) > 32)
      return fail(ctx, ORH_E_UNSUPPORTED, "orh_whatif_create: a source has more than 32 neighbours");
  }
  hipSetDevice(ctx->device);
  auto* job = new (std::nothrow) orh_whatif();
  if (!job) return fail(ctx, ORH_E_NOMEM, "orh_whatif_create");
  job->g = g;
  job->gen = g->gen;
  job->use_link_metric = use_link_metric ? 1 : 0;
  job->uniform = uniform;
  job->bound = bound;
  job->srcs.assign(h_srcs, h_srcs + n_srcs);
  auto bail = [&](int code) {
    orh_whatif_destroy(job);
    return code;
  };
  if (hipEventCreate(&job->ev_begin) != hipSuccess || hipEventCreate(&job->ev_end) != hipSuccess ||
      hipStreamCreateWithFlags(&job->side, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(ctx, ORH_E_DEVICE, "orh_whatif_create: events / stream"));
  for (int c = 0; c < kRunSlots; ++c)
    if (hipEventCreateWithFlags(&job->front_ev[c], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&job->side_ev[c], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&job->mid_ev[c], hipEventDisableTiming) != hipSuccess)
      return bail(fail(ctx, ORH_E_DEVICE, "orh_whatif_create: events"));
  for (hipStream_t& t : job->t3)
    if (hipStreamCreateWithFlags(&t, hipStreamNonBlocking) != hipSuccess)
      return bail(fail(ctx, ORH_E_DEVICE, "orh_whatif_create: streams"));
  rc = whatif_base(job);
  if (rc) return bail(rc);
  *out = job;
  return ORH_OK;
}

// runSpf(src, useLinkMetric, ignore) for every request of an ignore-set batch
// from the plain rows of its distinct sources: a what-if job over those
// sources, one run, destroyed after its kernels are queued (stream order)
int run_repair(orh_graph* g, const orh_spf_request* req, uint32_t* d_dist, uint32_t* d_nh) {
  orh_ctx* ctx = g->ctx;
  const uint32_t n_src = req->n_src;
  std::vector<uint32_t> base_srcs, base_row(n_src);
  auto& ro = g->row_of;
  for (uint32_t i = 0; i < n_src; ++i) {
    const uint32_t s = req->h_srcs[i];
    if (ro[s] < 0) {
      ro[s] = static_cast<int32_t>(base_srcs.size());
      base_srcs.push_back(s);
    }
    base_row[i] = static_cast<uint32_t>(ro[s]);
  }
  for (uint32_t s : base_srcs) ro[s] = -1;
  orh_whatif* job = nullptr;
  ORH_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  int rc = whatif_create(g, base_srcs.data(), static_cast<uint32_t>(base_srcs.size()), req->use_link_metric, &job);
  if (rc) return rc;
  ORH_HIP(ctx, hipEventRecord(ctx->evm, ctx->stream));
  rc = whatif_run(job, n_src, base_row.data(), req->h_ignore_ptr, req->h_ignore_links, d_dist, d_nh, nullptr);
  if (!rc) rc = whatif_flush(job);
  if (rc) {
    orh_whatif_destroy(job);
    return rc;
  }
  ORH_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  orh_whatif_destroy(job);
  orh_spf_info info{};
  info.variant = static_cast<int32_t>(orh::SpfVariant::kRepair);
  info.rows = n_src;
  info.batch_sources = static_cast<uint32_t>(base_srcs.size());
  ctx->last_info = info;
  return ORH_OK;
}

}  // namespace

extern "C" {

int orh_whatif_create(orh_graph* g, const uint32_t* h_srcs, uint32_t n_srcs, int32_t use_link_metric,
                      orh_whatif** out) {
  if (!g || !out || (n_srcs && !h_srcs)) return g ? fail(g->ctx, ORH_E_INVALID, "orh_whatif_create: null argument")
                                                  : ORH_E_INVALID;
  *out = nullptr;
  join_deferred(g->ctx);
  return whatif_create(g, h_srcs, n_srcs, use_link_metric, out);
}

int orh_whatif_run(orh_whatif* job, uint32_t n_req, const uint32_t* h_src_idx, const uint32_t* h_ignore_ptr,
                   const uint32_t* h_ignore_links, uint32_t* d_dist, uint32_t* d_nh, uint32_t* d_info) {
  if (!job) return ORH_E_INVALID;
  orh_ctx* ctx = job->g->ctx;
  join_deferred(ctx);
  if (n_req == 0) return ORH_OK;
  if (!h_src_idx || !h_ignore_ptr || (h_ignore_ptr[n_req] && !h_ignore_links) || !d_dist || !d_nh)
    return fail(ctx, ORH_E_INVALID, "orh_whatif_run: null argument");
  if (job->gen != job->g->gen)
    return fail(ctx, ORH_E_STATE, "orh_whatif_run: the graph changed since the job was created");
  hipSetDevice(ctx->device);
  return whatif_run(job, n_req, h_src_idx, h_ignore_ptr, h_ignore_links, d_dist, d_nh, d_info);
}

int orh_whatif_refresh(orh_whatif* job) {
  if (!job) return ORH_E_INVALID;
  hipSetDevice(job->g->ctx->device);
  return whatif_base(job);
}

int orh_whatif_flush(orh_whatif* job) {
  if (!job) return ORH_E_INVALID;
  hipSetDevice(job->g->ctx->device);
  return whatif_flush(job);
}

int orh_whatif_elapsed_ms(orh_whatif* job, double* ms_out) {
  if (!job || !ms_out) return ORH_E_INVALID;
  orh_ctx* ctx = job->g->ctx;
  int rc = whatif_flush(job);
  if (rc) return rc;
  ORH_HIP(ctx, hipEventSynchronize(job->ev_end));
  float ms = 0.f;
  ORH_HIP(ctx, hipEventElapsedTime(&ms, job->ev_begin, job->ev_end));
  *ms_out = ms;
  return ORH_OK;
}

int orh_whatif_set_flags(orh_whatif* job, uint32_t flags) {
  if (!job) return ORH_E_INVALID;
  if (flags & ~(ORH_WHATIF_SHARE_BASE | ORH_WHATIF_SEARCH_LARGE))
    return fail(job->g->ctx, ORH_E_INVALID, "orh_whatif_set_flags: unknown flag");
  job->flags = flags;
  return ORH_OK;
}

int orh_whatif_base_rows(orh_whatif* job, const uint32_t** d_dist, const uint32_t** d_nh) {
  if (!job || !d_dist || !d_nh) return ORH_E_INVALID;
  const size_t nd = job->srcs.size() * static_cast<size_t>(job->g->n_nodes);
  *d_dist = job->d_base;
  *d_nh = job->d_base + nd;
  return ORH_OK;
}

int orh_whatif_destroy(orh_whatif* job) {
  if (!job) return ORH_E_INVALID;
  // queued kernels may still read the job's buffers: drain both streams
  if (job->side) {
    whatif_flush(job);
    hipStreamSynchronize(job->side);
  }
  for (hipStream_t t : job->t3)
    if (t) hipStreamSynchronize(t);
  hipStreamSynchronize(job->g->ctx->stream);
  for (hipStream_t t : job->t3)
    if (t) hipStreamDestroy(t);
  for (int c = 0; c < kRunSlots; ++c) {
    hipFree(job->t3_slots[c]);
    if (job->mid_ev[c]) hipEventDestroy(job->mid_ev[c]);
    hipFree(job->d_work[c]);
    if (job->front_ev[c]) hipEventDestroy(job->front_ev[c]);
    if (job->side_ev[c]) hipEventDestroy(job->side_ev[c]);
    if (job->stage_ev[c]) {
      hipEventSynchronize(job->stage_ev[c]);
      hipEventDestroy(job->stage_ev[c]);
    }
    if (job->h_stage[c]) hipHostFree(job->h_stage[c]);
    hipFree(job->d_stage[c]);
  }
  hipFree(job->d_base);
  hipFree(job->own_slots);
  hipFree(job->d_full_lab);
  if (job->g->ctx->slots_owner == job) job->g->ctx->slots_owner = nullptr;
  if (job->side) hipStreamDestroy(job->side);
  if (job->ev_begin) hipEventDestroy(job->ev_begin);
  if (job->ev_end) hipEventDestroy(job->ev_end);
  delete job;
  return ORH_OK;
}

}  // extern "C"

extern "C" {

// Phase 1 computes a distance row for every requested source and for every
// distinct neighbour of one (the first-hop phase reads them). Without ignore
// sets rows are shared by node: a neighbour that is itself requested reuses
// its output row, the others get scratch rows. With per-source ignore sets a
// source's neighbour rows are its own (same ignore set).
int orh_spf_run(orh_graph* g, const orh_spf_request* req, uint32_t words, uint32_t* d_dist,
                uint32_t* d_nh) {
  if (!g || !req || (req->n_src && (!req->h_srcs || !d_dist || !d_nh)))
    return g ? fail(g->ctx, ORH_E_INVALID, "orh_spf_run: null argument") : ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  if (req->n_src == 0) return ORH_OK;
  if (!g->d_recs || g->n_nodes == 0) return fail(ctx, ORH_E_STATE, "orh_spf_run: no graph loaded");
  const uint32_t n_src = req->n_src, N = g->n_nodes;
  uint32_t max_nbr = 1;
  for (uint32_t i = 0; i < n_src; ++i) {
    if (req->h_srcs[i] >= N) return fail(ctx, ORH_E_INVALID, "orh_spf_run: source out of range");
    max_nbr = std::max(max_nbr, n_distinct(g, req->h_srcs[i]));
  }
  if (words < (max_nbr + 31) / 32) return fail(ctx, ORH_E_INVALID, "orh_spf_run: words too small");
  // zero link metrics: the first hops depend on the extraction order among
  // equal-metric nodes, which only the exact kernel follows
  if (ctx->spf_mode == orh::SpfMode::kExact || (req->use_link_metric && g->has_zero)) {
    if (req->use_link_metric && wide_metrics(g))
      return fail(ctx, ORH_E_UNSUPPORTED,
                  "orh_spf_run: path metrics may reach 2^32 - 1 (use orh_spf_run_exact)");
    return run_exact(g, req, words, d_dist, nullptr, d_nh, nullptr);
  }
  const bool uniform = !req->use_link_metric || g->min_out == g->max_out;
  const uint32_t w0 = req->use_link_metric ? g->max_out : 1u;
  // any tentative value is at most (sum of link metrics) + max metric; BFS
  // levels at most (N - 1) * w0
  const uint64_t bound = uniform ? static_cast<uint64_t>(N) * w0
      : req->use_link_metric ? g->sum_max_metric / 2 + g->max_metric
                             : static_cast<uint64_t>(g->n_links) + 1;
  const bool has_ign = req->h_ignore_ptr != nullptr;
  if (has_ign && ctx->spf_mode == orh::SpfMode::kAuto && max_nbr <= 32 && repair_eligible(g, req, words)) {
    hipSetDevice(ctx->device);
    return run_repair(g, req, d_dist, d_nh);
  }
  const orh::SpfPlan plan =
      orh::plan_spf(N, uniform, bound, g->ell_k, ctx->lds_limit, !has_ign, ctx->spf_mode);
  if (plan.variant == orh::SpfVariant::kUnsupported)
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_spf_run: no distance kernel for this graph (N=" +
                                            std::to_string(N) + ", path bound " +
                                            std::to_string(bound) + "; orh_spf_run_exact covers it)");
  if (orh::hop_lds_bytes(max_nbr) > ctx->lds_limit)
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_spf_run: too many neighbours for the first-hop phase");
  hipSetDevice(ctx->device);

  const uint32_t n_ign = has_ign ? req->h_ignore_ptr[n_src] : 0u;
  // request key: graph generation + sources + ignore sets
  std::vector<uint32_t> key;
  key.reserve(6 + n_src + (has_ign ? n_src + 1 + n_ign : 0));
  const uint64_t gp = reinterpret_cast<uintptr_t>(g);
  key.insert(key.end(), {static_cast<uint32_t>(gp), static_cast<uint32_t>(gp >> 32),
                         static_cast<uint32_t>(g->gen), static_cast<uint32_t>(g->gen >> 32),
                         n_src, has_ign ? 1u : 0u});
  key.insert(key.end(), req->h_srcs, req->h_srcs + n_src);
  if (has_ign) {
    key.insert(key.end(), req->h_ignore_ptr, req->h_ignore_ptr + n_src + 1);
    key.insert(key.end(), req->h_ignore_links, req->h_ignore_links + n_ign);
  }
  // staged layout: srcs[n_rows] | ign_ptr[n_rows+1] ign[..] | nbr_ptr[n_src+1] nbr_row[..]
  uint32_t n_rows = n_src;
  size_t off_ign_ptr = 0, off_ign = 0, off_nbr_ptr = 0, off_nbr_row = 0, off_order = 0;
  // the stored key carries six staging offsets after the request key
  if (!staged_key_matches(g->req_key, key, 6)) {
    std::vector<uint32_t> srcs(req->h_srcs, req->h_srcs + n_src), nbr_ptr(n_src + 1, 0), nbr_row;
    std::vector<uint32_t> ign_ptr, ign;
    std::vector<uint32_t> row_owner;  // source index whose ignore set a row uses
    if (!has_ign) {
      auto& ro = g->row_of;
      for (uint32_t i = 0; i < n_src; ++i)
        if (ro[req->h_srcs[i]] < 0) ro[req->h_srcs[i]] = static_cast<int32_t>(i);
      for (uint32_t i = 0; i < n_src; ++i) {
        const uint32_t s = req->h_srcs[i];
        for (uint32_t k = g->dn_ptr[s]; k < g->dn_ptr[s + 1]; ++k) {
          const uint32_t u = g->dn[k];
          if (ro[u] < 0) {
            ro[u] = static_cast<int32_t>(srcs.size());
            srcs.push_back(u);
          }
          nbr_row.push_back(static_cast<uint32_t>(ro[u]));
        }
        nbr_ptr[i + 1] = static_cast<uint32_t>(nbr_row.size());
      }
      for (uint32_t u : srcs) ro[u] = -1;
    } else {
      ign_ptr.assign(1, 0);
      auto add_set = [&](uint32_t i) {
        std::vector<uint32_t> s(req->h_ignore_links + req->h_ignore_ptr[i],
                                req->h_ignore_links + req->h_ignore_ptr[i + 1]);
        std::sort(s.begin(), s.end());  // bsearch on device
        ign.insert(ign.end(), s.begin(), s.end());
        ign_ptr.push_back(static_cast<uint32_t>(ign.size()));
      };
      for (uint32_t i = 0; i < n_src; ++i) add_set(i);
      for (uint32_t i = 0; i < n_src; ++i) {
        const uint32_t s = req->h_srcs[i];
        for (uint32_t k = g->dn_ptr[s]; k < g->dn_ptr[s + 1]; ++k) {
          nbr_row.push_back(static_cast<uint32_t>(srcs.size()));
          srcs.push_back(g->dn[k]);
          add_set(i);
        }
        nbr_ptr[i + 1] = static_cast<uint32_t>(nbr_row.size());
      }
    }
    n_rows = static_cast<uint32_t>(srcs.size());
    {  // first-hop block order: one contiguous source range per XCD when the
       // per-source work (neighbour rows) is even, else runs of 16 so heavy
       // sources (Clos spines) still spread over the XCDs (A/B: C2 0.342 vs
       // 0.350 ms, C3 0.231 vs 0.107 ms for contiguous vs runs of 16/64)
      uint64_t sum = 0;
      uint32_t mx = 0;
      for (uint32_t i = 0; i < n_src; ++i) {
        const uint32_t d = nbr_ptr[i + 1] - nbr_ptr[i];
        sum += d;
        mx = std::max(mx, d);
      }
      g->req_xcd_group = static_cast<uint64_t>(mx) * n_src <= 2 * sum ? 0u : 16u;
    }
    std::vector<uint32_t> staging;
    staging.reserve(srcs.size() + ign_ptr.size() + ign.size() + nbr_ptr.size() + nbr_row.size() + 1);
    staging.push_back(n_rows);
    staging.insert(staging.end(), srcs.begin(), srcs.end());
    off_ign_ptr = staging.size();
    staging.insert(staging.end(), ign_ptr.begin(), ign_ptr.end());
    off_ign = staging.size();
    staging.insert(staging.end(), ign.begin(), ign.end());
    off_nbr_ptr = staging.size();
    staging.insert(staging.end(), nbr_ptr.begin(), nbr_ptr.end());
    off_nbr_row = staging.size();
    staging.insert(staging.end(), nbr_row.begin(), nbr_row.end());
    // multi-source batches (consecutive runs of ms_width rows): rows in
    // ascending Cuthill-McKee id of their source, so a batch's sources are
    // neighbours. (Measured alternatives on C2: BFS balls of 32 rows - 10.6
    // arrival levels per node and batch against 16.4 - swept in 0.92 ms
    // against 0.77; dispatching the batches middle-out changed nothing.)
    off_order = staging.size();
    {
      std::vector<uint32_t> order(n_rows);
      for (uint32_t r = 0; r < n_rows; ++r) order[r] = r;
      std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
        return g->ms_dev_of[srcs[x]] < g->ms_dev_of[srcs[y]];
      });
      staging.insert(staging.end(), order.begin(), order.end());
    }
    drain_deferred(ctx);  // a deferred phase 2 may still read the staged request
    int rc = ensure_graph_req(g, staging.size());
    if (rc) return rc;
    ORH_HIP(ctx, hipMemcpyAsync(g->d_req, staging.data(), staging.size() * 4,
                                hipMemcpyHostToDevice, ctx->stream));
    ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // staging is a local
    key.push_back(static_cast<uint32_t>(off_ign_ptr));
    key.push_back(static_cast<uint32_t>(off_ign));
    key.push_back(static_cast<uint32_t>(off_nbr_ptr));
    key.push_back(static_cast<uint32_t>(off_nbr_row));
    key.push_back(static_cast<uint32_t>(off_order));
    key.push_back(n_rows);
    g->req_key = std::move(key);
  }
  {
    const auto& k = g->req_key;
    const size_t t = k.size();
    off_order = k[t - 2];
    off_ign_ptr = k[t - 6];
    off_ign = k[t - 5];
    off_nbr_ptr = k[t - 4];
    off_nbr_row = k[t - 3];
    n_rows = k[t - 1];
  }
  // HBM kernel: fuse the first hops into the search (one row per source)
  // when one mask word covers every source and the two-phase scheme would
  // need extra neighbour rows (or the HBM kernel is forced)
  orh::SpfPlan run_plan = plan;
  orh::ms_set_width(run_plan, N, n_rows, ctx->n_cu, ctx->lds_limit,
                    run_plan.variant == orh::SpfVariant::kMsBfs && !device_busy_elsewhere(ctx));
  // uniform metric, at most ORH_BFS_NH_MAX sources (default: one per CU):
  // one fused BFS + first-hop workgroup per source instead of searching
  // every neighbour row too (ORH_BFS_NH_MAX=0 turns it off)
  {
    const bool bfs_plan = plan.variant == orh::SpfVariant::kMsBfs || plan.variant == orh::SpfVariant::kBfs8 ||
                          plan.variant == orh::SpfVariant::kBfs16 || plan.variant == orh::SpfVariant::kBfs32;
    uint32_t fused_max = ctx->n_cu;
    if (const char* e = getenv("ORH_BFS_NH_MAX")) fused_max = static_cast<uint32_t>(atoi(e));
    uint32_t blk = 0, jj = 0;
    size_t lds = 0;
    if (bfs_plan && ctx->spf_mode == orh::SpfMode::kAuto && n_src <= fused_max &&
        orh::bfs_nh_shape(N, words, ctx->lds_limit, &blk, &jj, &lds)) {
      run_plan.variant = orh::SpfVariant::kBfsNh;
      run_plan.block = blk;
      run_plan.lds_bytes = lds;
      n_rows = n_src;
    }
  }
  // general metrics whose labels fit LDS: one search per source with the
  // first hops fused (spf_lds_nh_kernel) instead of the two-phase LDS kernels,
  // which also search every neighbour row and then stream 1 + deg rows per
  // source. ORH_LDS_NH=0: the two-phase plan (A/B); orh_set_spf_mode(1)
  // (per-source) keeps it too
  // many sources, general metrics, a graph whose in-links fit the ELL rows:
  // 4-source Bellman-Ford batches in LDS (spf_wms_kernel), then the first
  // hops over the u32 rows (phase 2). ORH_WMS=0 off (A/B); ORH_WMS_MIN: the
  // fewest requested sources that take it (default 256: below, the fused
  // per-source search, which needs no neighbour rows, is the better plan)
  bool wms = false;
  {
    static const bool on = [] {
      const char* e = getenv("ORH_WMS");
      return !(e && e[0] == '0');
    }();
    static const uint32_t wms_min = [] {
      const char* e = getenv("ORH_WMS_MIN");
      return e ? static_cast<uint32_t>(atoi(e)) : 256u;
    }();
    if (on && ctx->spf_mode == orh::SpfMode::kAuto && !uniform && !has_ign && n_src >= wms_min &&
        (plan.variant == orh::SpfVariant::kDist16 || plan.variant == orh::SpfVariant::kDist32) &&
        orh::wms_lds_bytes(N) <= ctx->lds_limit && orh::lds_nh_bytes(N, false) <= ctx->lds_limit) {
      int rc = sync_wms_layout(g);
      if (rc) return rc;
      if (g->wms_ok) {
        wms = true;
        run_plan.variant = orh::SpfVariant::kWms;
        rc = ensure_labels(ctx, (static_cast<size_t>(n_rows) + 2) / 2 + 1);  // the overflow row list
        if (rc) return rc;
      }
    }
  }
  // A few sources without ignore sets keep the two-phase LDS plan: a lone
  // search pays the fused kernel's per-bucket barriers with nothing beside it
  // (C2's buildRouteDb after a metric change: spf(me) 1.15 ms fused against
  // ~0.6 two-phase, profiles/r06/e_bench_phases.json); ORH_LDS_NH_MIN (32)
  bool lds_nh_packed = false;
  {
    static const bool on = [] {
      const char* e = getenv("ORH_LDS_NH");
      return !(e && e[0] == '0');
    }();
    static const uint32_t lds_nh_min = [] {
      const char* e = getenv("ORH_LDS_NH_MIN");
      return e ? static_cast<uint32_t>(atoi(e)) : 32u;
    }();
    if (on && !wms && (has_ign || n_src >= lds_nh_min) && ctx->spf_mode == orh::SpfMode::kAuto && !uniform &&
        max_nbr <= 32 &&
        (plan.variant == orh::SpfVariant::kDist16 || plan.variant == orh::SpfVariant::kDist32) &&
        orh::lds_nh_bytes(N, false) <= ctx->lds_limit) {
      run_plan.variant = orh::SpfVariant::kLdsNh;
      lds_nh_packed = max_nbr <= 16;
      n_rows = n_src;
      // few rows: wide workgroups (latency); many: narrow ones, several per CU
      static const uint32_t blk_env = [] {
        const char* e = getenv("ORH_LDS_NH_BLOCK");
        const int b = e ? atoi(e) : 0;
        return (b >= 64 && b <= 1024 && b % 64 == 0) ? static_cast<uint32_t>(b) : 0u;
      }();
      run_plan.block = blk_env ? blk_env
                     : n_src <= ctx->n_cu ? 1024u : n_src <= 2 * ctx->n_cu ? 512u : 256u;
      int rc = ensure_labels(ctx, (static_cast<size_t>(n_src) + 2) / 2 + 1);  // the overflow row list
      if (rc) return rc;
    }
  }
  if (plan.variant == orh::SpfVariant::kGlobal && max_nbr <= 32 &&
      ctx->spf_mode != orh::SpfMode::kGlobalTwoPhase &&
      (ctx->spf_mode == orh::SpfMode::kGlobal || n_rows > n_src)) {
    run_plan.variant = orh::SpfVariant::kGlobalNh;
    n_rows = n_src;
    // few rows: wider workgroups (a big frontier phase is split over more
    // threads; the rows do not fill the CUs anyway)
    run_plan.block = n_src <= ctx->n_cu ? 1024u : n_src <= 2 * ctx->n_cu ? 512u : 256u;
    int rc = ensure_labels(ctx, static_cast<size_t>(n_src) * N);
    if (rc) return rc;
  }
  const bool fused = run_plan.variant == orh::SpfVariant::kGlobalNh ||
                     run_plan.variant == orh::SpfVariant::kBfsNh ||
                     run_plan.variant == orh::SpfVariant::kLdsNh;
  const size_t n_extra = n_rows - n_src;
  if (n_extra) {
    int rc = ensure_scratch(ctx, n_extra * N);
    if (rc) return rc;
  }

  orh::SpfArgs a{};
  a.n_nodes = N;
  a.n_out = n_src;
  a.recs = g->d_recs;
  a.link = g->d_link;
  bool defer = false;  // this sweep's phase 2 goes to stream2
  if (run_plan.variant == orh::SpfVariant::kMsBfs) {
    int rc = sync_ms_layout(g);
    if (rc) return rc;
    // the interval skip: opt-in for every sweep (ORH_MS_SKIP=1) or for the
    // latency plan alone (ORH_MS_LATENCY=2)
    a.ms_bw = g->ms_bw ? g->ms_bw : run_plan.ms_skip ? g->ms_bw_layout : 0u;
    a.ms_width = run_plan.ms_width;
    // host-order layout, u16 / u32 masks: the rows come out of the search
    // kernel itself (ORH_MS_DIRECT=0: through ms_lvl and ms_finalize, A/B)
    const char* de = getenv("ORH_MS_DIRECT");  // read per run (tests flip it)
    const bool direct_on = !(de && de[0] == '0');
    a.ms_direct = direct_on && g->ms_identity && run_plan.mask_bytes <= 4 ? 1u : 0u;
    const size_t scratch =
        a.ms_direct ? 0 : (orh::ms_scratch_bytes(run_plan, N, n_rows) + 255) & ~size_t{255};
    const size_t log_bytes = orh::ms_log_bytes(run_plan, n_rows);
    // ORH_SPF_DEFER_HOPS: the level bytes in half p2_half of two. Off unless
    // ORH_MS_DEFER=1: the 32-sweep C2 step measured 23.1-23.2 ms deferred
    // against 23.05 (2 lanes; 36.2 ms at 1 lane), i.e. the GPU is already
    // busy while a sweep's phase 2 runs - the searches and the phase-2
    // streams share the CUs, so starting the next search earlier only
    // reorders the same work (profiles/r06/n_defer_ab.txt)
    static const bool defer_on = [] {
      const char* e = getenv("ORH_MS_DEFER");
      return e && e[0] == '1';
    }();
    defer = defer_on && (req->flags & ORH_SPF_DEFER_HOPS) && !a.ms_direct && n_extra == 0;
    const size_t halves = defer ? 2 : 1;
    rc = ensure_ms_lvl(ctx, halves * scratch + log_bytes);
    if (rc) return rc;
    a.ms_log = log_bytes ? reinterpret_cast<uint64_t*>(ctx->d_ms_lvl + halves * scratch) : nullptr;
    a.recs = g->d_ms_recs;
    a.dev_of = g->d_ms_dev_of;
    a.host_of = g->d_ms_host_of;
    a.ms_lvl = ctx->d_ms_lvl + (defer ? ctx->p2_half * scratch : 0);
    a.lvl_pitch = (N + 15u) & ~15u;
    rc = ensure_lvl_rows(ctx, static_cast<size_t>(n_rows) * a.lvl_pitch);
    if (rc) return rc;
    a.lvl_rows = ctx->d_lvl_rows;
  }
  a.order = g->d_req + off_order;
  a.srcs = g->d_req + 1;
  a.ignore_ptr = has_ign ? g->d_req + off_ign_ptr : nullptr;
  a.ignore_links = has_ign ? g->d_req + off_ign : nullptr;
  a.use_link_metric = req->use_link_metric;
  a.w0 = w0;
  // near/far width of the HBM kernel: the mean live metric (one BFS level
  // when metrics are uniform)
  a.delta = uniform ? w0
                    : std::max<uint32_t>(1u, static_cast<uint32_t>(
                                                 static_cast<uint64_t>(g->mean_out) * ctx->delta_pct / 100u));
  if (run_plan.variant == orh::SpfVariant::kLdsNh || run_plan.variant == orh::SpfVariant::kWms) {
    // ORH_LDS_NH_DELTA_PCT: bucket width of the LDS search in % of the mean
    // live metric. Its relaxations cost LDS latency, not a global atomic, so
    // wider buckets (fewer bucket barriers) pay: C2w sweep 45.5 / 30.8 / 28.9 /
    // 29.0 / 31.4 ms at 25 / 100 / 200 / 400 / 800 (profiles/r06/b_c2w_delta_block.txt)
    static const uint32_t pct = [] {
      const char* e = getenv("ORH_LDS_NH_DELTA_PCT");
      const int v = e ? atoi(e) : 200;
      return v > 0 ? static_cast<uint32_t>(v) : 200u;
    }();
    a.delta = std::max<uint32_t>(1u, static_cast<uint32_t>(static_cast<uint64_t>(g->mean_out) * pct / 100u));
  }
  a.out_dist = d_dist;
  a.scratch = ctx->d_scratch;
  a.labels = ctx->d_labels;
  a.out_nh = d_nh;
  a.words = words;
  a.rank_out = g->d_rank_out;

  orh::HopArgs h{};
  h.n_nodes = N;
  h.n_out = n_src;
  h.words = words;
  h.ell_k = g->ell_k;
  h.recs = g->d_recs;
  h.link = g->d_link;
  h.rank_out = g->d_rank_out;
  h.overloaded = g->d_ovl;
  h.srcs = a.srcs;
  h.ignore_ptr = a.ignore_ptr;
  h.ignore_links = a.ignore_links;
  h.use_link_metric = req->use_link_metric;
  h.nbr_ptr = g->d_req + off_nbr_ptr;
  h.xcd_group = g->req_xcd_group;
  h.nbr_row = g->d_req + off_nbr_row;
  h.dist = d_dist;
  h.scratch = ctx->d_scratch;
  h.out_nh = d_nh;
  h.lvl_rows = run_plan.variant == orh::SpfVariant::kMsBfs ? a.lvl_rows : nullptr;
  h.lvl_pitch = a.lvl_pitch;
  h.w0 = w0;

  if (!defer) {
    join_deferred(ctx);  // earlier deferred sweeps share the scratch
  } else if (ctx->p2_pending[ctx->p2_half]) {
    // the search rewrites the half the phase 2 two sweeps back reads
    ORH_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_p2[ctx->p2_half], 0));
    ctx->p2_pending[ctx->p2_half] = false;
  }
  ORH_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
#ifdef ORH_DIAG_STAMPS
  static uint64_t* d_diag = nullptr;
  constexpr size_t kDiagWords = 16 + 4 * 4096;
  if (!d_diag) hipMalloc(&d_diag, kDiagWords * 8);
  hipMemsetAsync(d_diag, 0, kDiagWords * 8, ctx->stream);
  a.diag = d_diag;
#endif
  {
    hipError_t pre = hipGetLastError();
    if (pre != hipSuccess) { std::string m = "pending HIP error before spf launch (variant " + std::to_string(int(run_plan.variant)) + " rows " + std::to_string(n_rows) + ")"; return hip_fail(ctx, pre, m.c_str()); }
  }
  if (run_plan.variant == orh::SpfVariant::kLdsNh || run_plan.variant == orh::SpfVariant::kWms)
    a.ovf_rows = reinterpret_cast<uint32_t*>(ctx->d_labels);
  if (run_plan.variant == orh::SpfVariant::kWms) {
    a.dev_of = g->d_ms_dev_of;
    a.wms_slots = g->d_wms;
    a.wms_limit = 0xFFFEu - g->wms_maxw;
    // the in-links' reach in layout ids: the activity skip, opt-in
    // (ORH_WMS_SKIP=1). Its per-slice bitmap test costs more than the slices
    // it skips once a round sweeps each band both ways: C2w distances 5.07 ms
    // with it, 3.58 ms without (profiles/r06/v_wms_skip_ab.txt)
    const char* skip_e = getenv("ORH_WMS_SKIP");  // read per run (tests flip it)
    const bool skip = skip_e && skip_e[0] == '1';
    a.ms_bw = skip ? g->ms_bw_layout : 0u;
    a.recs_k = g->ell_k;
    // the band schedule (ORH_WMS_BAND=0: interleaved chunks, one sweep per
    // round, A/B)
    const char* band_e = getenv("ORH_WMS_BAND");  // read per run (tests flip it)
    a.wms_band = (band_e && band_e[0] == '0') ? 0u : 1u;
  }
  hipError_t e = run_plan.variant == orh::SpfVariant::kLdsNh
      ? orh::launch_spf_lds_nh(a, n_rows, g->ell_k, lds_nh_packed, run_plan.block, ctx->stream)
      : run_plan.variant == orh::SpfVariant::kWms ? orh::launch_spf_wms(a, n_rows, g->wms_k, ctx->lds_limit, ctx->stream)
      : orh::launch_spf(run_plan, a, n_rows, ctx->stream);
  if (e != hipSuccess) { std::string m = "spf kernel launch variant " + std::to_string(int(run_plan.variant)) + " rows " + std::to_string(n_rows) + " lds " + std::to_string(run_plan.lds_bytes) + " block " + std::to_string(run_plan.block) + " j " + std::to_string(run_plan.ms_j); return hip_fail(ctx, e, m.c_str()); }
#ifdef ORH_DIAG_STAMPS
  {
    std::vector<uint64_t> h(kDiagWords);
    hipMemcpyAsync(h.data(), d_diag, kDiagWords * 8, hipMemcpyDeviceToHost, ctx->stream);
    hipStreamSynchronize(ctx->stream);
    if (h[4])
      fprintf(stderr, "diag: waves %llu avg cycles %.0f barrier %.0f groups/wave %.1f levels %.1f max cycles %llu max levels %llu read %.0f proc %.0f\n",
              (unsigned long long)h[4], double(h[0]) / h[4], double(h[1]) / h[4],
              double(h[2]) / h[4], double(h[3]) / h[4], (unsigned long long)h[5], (unsigned long long)h[6], double(h[7]) / h[4], double(h[8]) / h[4]);
    // per workgroup: duration, and how many workgroups shared its CU at any time
    struct Wg { uint64_t t0, t1, cu; uint32_t lv, b; };
    std::vector<Wg> wg;
    for (uint32_t b = 0; b < 4096; ++b) {
      const uint64_t* w = &h[16 + 4 * b];
      if (!w[1]) continue;
      const uint64_t hw = w[2];
      // HW_ID: CU_ID [11:8], SH_ID [12], SE_ID [15:13]; XCC_ID in the high word
      const uint64_t cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | ((hw >> 32) & 0xF) << 8;
      wg.push_back({w[0], w[1], cu, static_cast<uint32_t>(w[3]), b});
    }
    if (!wg.empty()) {
      uint64_t t_min = ~0ull, t_max = 0;
      for (auto& x : wg) { t_min = std::min(t_min, x.t0); t_max = std::max(t_max, x.t1); }
      std::vector<uint64_t> dur_solo, dur_shared;
      uint64_t worst = 0; uint32_t worst_b = 0, worst_lv = 0; int worst_share = 0;
      for (auto& x : wg) {
        int share = 0;
        for (auto& y : wg) if (&y != &x && y.cu == x.cu && y.t0 < x.t1 && x.t0 < y.t1) ++share;
        (share ? dur_shared : dur_solo).push_back(x.t1 - x.t0);
        if (x.t1 - x.t0 > worst) { worst = x.t1 - x.t0; worst_b = x.b; worst_lv = x.lv; worst_share = share; }
      }
      auto med = [](std::vector<uint64_t> v) { if (v.empty()) return 0.0; std::sort(v.begin(), v.end()); return double(v[v.size() / 2]); };
      auto mx = [](const std::vector<uint64_t>& v) { uint64_t m = 0; for (auto x : v) m = std::max(m, x); return double(m); };
      uint64_t last_start = 0;
      for (auto& x : wg) last_start = std::max(last_start, x.t0 - t_min);
      fprintf(stderr, "diag-wg: %zu wgs span %llu; solo %zu med %.0f max %.0f; shared %zu med %.0f max %.0f; worst wg %u (%u levels, %d partners) %llu; last start %llu\n",
              wg.size(), (unsigned long long)(t_max - t_min), dur_solo.size(), med(dur_solo), mx(dur_solo),
              dur_shared.size(), med(dur_shared), mx(dur_shared), worst_b, worst_lv, worst_share,
              (unsigned long long)worst, (unsigned long long)last_start);
    }
  }
#endif
  ORH_HIP(ctx, hipEventRecord(ctx->evm, ctx->stream));
  orh_spf_info info{};
  info.variant = static_cast<int32_t>(run_plan.variant);
  info.rows = n_rows;
  info.mask_bits = run_plan.variant == orh::SpfVariant::kMsBfs ? run_plan.mask_bytes * 8 : 0;
  info.batch_sources = run_plan.variant == orh::SpfVariant::kMsBfs ? run_plan.ms_width : 0;
  info.ms_threads = run_plan.variant == orh::SpfVariant::kMsBfs ? run_plan.block : 0;
  info.ms_skip = run_plan.variant == orh::SpfVariant::kMsBfs && a.ms_bw ? 1u : 0u;
  info.ms_direct = run_plan.variant == orh::SpfVariant::kMsBfs ? a.ms_direct
                 : run_plan.variant == orh::SpfVariant::kWms && g->ms_identity ? 1u : 0u;
  if (run_plan.variant == orh::SpfVariant::kMsBfs) {
#ifdef ORH_EXP_MSBFS_ONLY  // timing experiment only (tools/diag_build.sh): no phase 2
    ctx->last_info = info;
    ORH_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    return ORH_OK;
#endif
    hipStream_t s2 = ctx->stream;
    if (defer) {
      // phase 2 on stream2 after this search; the context stream is free for
      // the next sweep's search
      if (!ctx->stream2) {
        // ORH_MS_DEFER_PRIO (A/B): stream2's priority, -1 high / 1 low / 0 (default) normal
        int lo = 0, hi = 0;
        const char* pe = getenv("ORH_MS_DEFER_PRIO");
        const int want = pe ? atoi(pe) : 0;
        if (want != 0 && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
          ORH_HIP(ctx, hipStreamCreateWithPriority(&ctx->stream2, hipStreamNonBlocking, want < 0 ? hi : lo));
        } else {
          ORH_HIP(ctx, hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
        }
        ORH_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_ms2, hipEventDisableTiming));
        ORH_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_p2[0], hipEventDisableTiming));
        ORH_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_p2[1], hipEventDisableTiming));
      }
      ORH_HIP(ctx, hipEventRecord(ctx->ev_ms2, ctx->stream));
      ORH_HIP(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_ms2, 0));
      s2 = ctx->stream2;
    }
    if (!a.ms_direct) {
      e = orh::launch_ms_finalize(run_plan, a, n_rows, s2);
      if (e != hipSuccess) return hip_fail(ctx, e, "multi-source finalize launch");
    }
    e = orh::launch_first_hop(h, max_nbr, s2, &info.hop_nodes, &info.hop_split);
    if (e != hipSuccess) return hip_fail(ctx, e, "first-hop kernel launch");
    if (defer) {
      ORH_HIP(ctx, hipEventRecord(ctx->ev_p2[ctx->p2_half], s2));
      ctx->p2_pending[ctx->p2_half] = true;
      ctx->p2_half ^= 1u;
      ctx->last_info = info;
      ORH_HIP(ctx, hipEventRecord(ctx->ev1, s2));
      ctx->counters.spf_runs += n_src;
      ctx->counters.spf_launches += 1;
      ctx->counters.last_kernel_ms = -1.0;
      return ORH_OK;
    }
  } else if (!fused) {
    e = orh::launch_first_hop(h, max_nbr, ctx->stream, &info.hop_nodes, &info.hop_split);
    if (e != hipSuccess) return hip_fail(ctx, e, "first-hop kernel launch");
  }
  ctx->last_info = info;
  ORH_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  ctx->counters.spf_runs += n_src;
  ctx->counters.spf_launches += 1;
  ctx->counters.last_kernel_ms = -1.0;  // resolved lazily by orh_spf_batch / orh_sync users
  return ORH_OK;
}

int orh_spf_batch(orh_graph* g, const orh_spf_request* req, uint32_t words, uint32_t* h_dist,
                  uint32_t* h_nh) {
  if (!g || !req) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  if (req->n_src == 0) return ORH_OK;
  if (!h_dist || !h_nh) return fail(ctx, ORH_E_INVALID, "orh_spf_batch: null output");
  const size_t nd = static_cast<size_t>(req->n_src) * g->n_nodes;
  hipSetDevice(ctx->device);
  if (nd * (1 + words) > ctx->d_batch_cap) {
    hipFree(ctx->d_batch);
    ctx->d_batch = nullptr;
    ctx->d_batch_cap = 0;
    if (hipMalloc(&ctx->d_batch, nd * (1 + words) * 4) != hipSuccess)
      return fail(ctx, ORH_E_NOMEM, "orh_spf_batch: device allocation failed");
    ctx->d_batch_cap = nd * (1 + words);
  }
  uint32_t* d_dist = ctx->d_batch;
  uint32_t* d_nh = ctx->d_batch + nd;
  int rc = orh_spf_run(g, req, words, d_dist, d_nh);
  if (rc == ORH_OK) {
    join_deferred(ctx);
    hipError_t e = hipMemcpyAsync(h_dist, d_dist, nd * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(h_nh, d_nh, nd * words * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = hip_fail(ctx, e, "orh_spf_batch: copy-out");
    float ms = 0.f;
    if (rc == ORH_OK && hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess) {
      ctx->counters.last_kernel_ms = ms;
      ctx->counters.total_kernel_ms += ms;
    }
  }
  return rc;
}

int orh_spf_batch_pinned(orh_graph* g, const orh_spf_request* req, uint32_t words,
                         const uint32_t** h_dist, const uint32_t** h_nh) {
  if (!g || !req || !h_dist || !h_nh) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  *h_dist = *h_nh = nullptr;
  if (req->n_src == 0) return ORH_OK;
  const size_t nd = static_cast<size_t>(req->n_src) * g->n_nodes;
  hipSetDevice(ctx->device);
  if (nd * (1 + words) > ctx->d_batch_cap) {
    hipFree(ctx->d_batch);
    ctx->d_batch = nullptr;
    ctx->d_batch_cap = 0;
    if (hipMalloc(&ctx->d_batch, nd * (1 + words) * 4) != hipSuccess)
      return fail(ctx, ORH_E_NOMEM, "orh_spf_batch_pinned: device allocation failed");
    ctx->d_batch_cap = nd * (1 + words);
  }
  if (nd * (1 + words) > ctx->h_pinned_cap) {
    if (ctx->h_pinned) hipHostFree(ctx->h_pinned);
    ctx->h_pinned = nullptr;
    ctx->h_pinned_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_pinned), nd * (1 + words) * 4, hipHostMallocDefault) !=
        hipSuccess)
      return fail(ctx, ORH_E_NOMEM, "orh_spf_batch_pinned: pinned host allocation failed");
    ctx->h_pinned_cap = nd * (1 + words);
  }
  int rc = orh_spf_run(g, req, words, ctx->d_batch, ctx->d_batch + nd);
  if (rc != ORH_OK) return rc;
  join_deferred(ctx);
  hipError_t e = hipMemcpyAsync(ctx->h_pinned, ctx->d_batch, nd * (1 + words) * 4, hipMemcpyDeviceToHost,
                                ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "orh_spf_batch_pinned: copy-out");
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess) {
    ctx->counters.last_kernel_ms = ms;
    ctx->counters.total_kernel_ms += ms;
  }
  *h_dist = ctx->h_pinned;
  *h_nh = ctx->h_pinned + nd;
  return ORH_OK;
}

int orh_spf_run_exact(orh_graph* g, const orh_spf_request* req, uint32_t words, uint64_t* d_dist,
                      uint32_t* d_nh, uint32_t* d_rank) {
  if (!g || !req || (req->n_src && (!req->h_srcs || !d_dist || !d_nh)))
    return g ? fail(g->ctx, ORH_E_INVALID, "orh_spf_run_exact: null argument") : ORH_E_INVALID;
  if (req->n_src == 0) return ORH_OK;
  join_deferred(g->ctx);
  if (!g->d_recs || g->n_nodes == 0)
    return fail(g->ctx, ORH_E_STATE, "orh_spf_run_exact: no graph loaded");
  return run_exact(g, req, words, nullptr, d_dist, d_nh, d_rank);
}

int orh_spf_batch_exact(orh_graph* g, const orh_spf_request* req, uint32_t words, uint64_t* h_dist,
                        uint32_t* h_nh, uint32_t* h_rank) {
  if (!g || !req) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  join_deferred(ctx);
  if (req->n_src == 0) return ORH_OK;
  if (!h_dist || !h_nh) return fail(ctx, ORH_E_INVALID, "orh_spf_batch_exact: null output");
  const size_t nd = static_cast<size_t>(req->n_src) * g->n_nodes;
  const size_t bytes = nd * 8 + nd * words * 4 + nd * 4;
  hipSetDevice(ctx->device);
  int rc = ensure_bytes(ctx, &ctx->d_batch_x, &ctx->d_batch_x_cap, bytes);
  if (rc) return fail(ctx, ORH_E_NOMEM, "orh_spf_batch_exact: device allocation failed");
  uint64_t* d_dist = reinterpret_cast<uint64_t*>(ctx->d_batch_x);
  uint32_t* d_nh = reinterpret_cast<uint32_t*>(d_dist + nd);
  uint32_t* d_rank = d_nh + nd * words;
  rc = orh_spf_run_exact(g, req, words, d_dist, d_nh, h_rank ? d_rank : nullptr);
  if (rc == ORH_OK) {
    hipError_t e = hipMemcpyAsync(h_dist, d_dist, nd * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(h_nh, d_nh, nd * words * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && h_rank)
      e = hipMemcpyAsync(h_rank, d_rank, nd * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = hip_fail(ctx, e, "orh_spf_batch_exact: copy-out");
    float ms = 0.f;
    if (rc == ORH_OK && hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess) {
      ctx->counters.last_kernel_ms = ms;
      ctx->counters.total_kernel_ms += ms;
    }
  }
  return rc;
}

}  // extern "C"

namespace {

// one source's SPF row as the KSP2 traces read it: u64 distances (~0 =
// unreachable) and, from the exact kernel, the extraction rank (else empty:
// extraction order is (distance, name rank))
struct KspRow {
  std::vector<uint64_t> dist;
  std::vector<uint32_t> rank;
};

// rows for `n` searches from src (ignore sets ign_ptr / ign, or none), in
// chunks that bound the device and host buffers
int ksp_rows(orh_graph* g, uint32_t src, uint32_t n, const uint32_t* ign_ptr, const uint32_t* ign,
             std::vector<KspRow>& rows) {
  orh_ctx* ctx = g->ctx;
  const uint32_t N = g->n_nodes;
  uint32_t words = 1;
  int rc = orh_spf_words(g, &src, 1, &words);
  if (rc) return rc;
  const bool exact = g->has_zero || wide_metrics(g);
  const uint32_t chunk = static_cast<uint32_t>(std::max<size_t>(1, (size_t{256} << 20) / (size_t{N} * (12 + 4 * words))));
  rows.resize(n);
  std::vector<uint32_t> srcs, ptr;
  std::vector<uint32_t> d32;
  for (uint32_t r0 = 0; r0 < n; r0 += chunk) {
    const uint32_t m = std::min(chunk, n - r0);
    srcs.assign(m, src);
    orh_spf_request req{};
    req.h_srcs = srcs.data();
    req.n_src = m;
    req.use_link_metric = 1;
    if (ign_ptr) {
      ptr.assign(m + 1, 0);
      for (uint32_t i = 0; i <= m; ++i) ptr[i] = ign_ptr[r0 + i] - ign_ptr[r0];
      req.h_ignore_ptr = ptr.data();
      req.h_ignore_links = ign + ign_ptr[r0];
      if (ptr[m] == 0) req.h_ignore_links = ptr.data();  // non-null, nothing read
    }
    const size_t nd = static_cast<size_t>(m) * N;
    const size_t bytes = nd * 8 + nd * 4 + nd * 4 * words;
    rc = ensure_bytes(ctx, &ctx->d_batch_x, &ctx->d_batch_x_cap, bytes);
    if (rc) return rc;
    uint64_t* dd64 = reinterpret_cast<uint64_t*>(ctx->d_batch_x);
    uint32_t* drank = reinterpret_cast<uint32_t*>(dd64 + nd);
    uint32_t* dnh = drank + nd;
    if (exact) {
      rc = run_exact(g, &req, words, nullptr, dd64, dnh, drank);
    } else {
      rc = orh_spf_run(g, &req, words, reinterpret_cast<uint32_t*>(dd64), dnh);
    }
    if (rc) return rc;
    if (exact) {
      std::vector<uint64_t> h(nd);
      std::vector<uint32_t> hr(nd);
      ORH_HIP(ctx, hipMemcpyAsync(h.data(), dd64, nd * 8, hipMemcpyDeviceToHost, ctx->stream));
      ORH_HIP(ctx, hipMemcpyAsync(hr.data(), drank, nd * 4, hipMemcpyDeviceToHost, ctx->stream));
      ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
      for (uint32_t i = 0; i < m; ++i) {
        rows[r0 + i].dist.assign(h.begin() + size_t{i} * N, h.begin() + size_t{i + 1} * N);
        rows[r0 + i].rank.assign(hr.begin() + size_t{i} * N, hr.begin() + size_t{i + 1} * N);
      }
    } else {
      d32.resize(nd);
      ORH_HIP(ctx, hipMemcpyAsync(d32.data(), dd64, nd * 4, hipMemcpyDeviceToHost, ctx->stream));
      ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
      for (uint32_t i = 0; i < m; ++i) {
        auto& d = rows[r0 + i].dist;
        d.resize(N);
        for (uint32_t v = 0; v < N; ++v) {
          const uint32_t x = d32[size_t{i} * N + v];
          d[v] = x == ORH_UNREACHABLE ? ~0ull : x;
        }
        rows[r0 + i].rank.clear();
      }
    }
  }
  return ORH_OK;
}

// NodeSpfResult::pathLinks of v (LinkState.cpp:857-873 insertion order):
// (link id, prev) over live, non-ignored CSR entries v <- u with
// dist[u] + metric(u -> v) == dist[v], u extracted before v and transit
// (u == src or not overloaded); by u's extraction order, then the link's
// position in u's row
void ksp_path_links(const orh_graph* g, uint32_t src, const KspRow& row, uint32_t v,
                    const std::vector<uint32_t>& ign, std::vector<std::pair<uint32_t, uint32_t>>& out) {
  out.clear();
  const uint64_t dv = row.dist[v];
  if (dv == ~0ull || v == src) return;
  struct Cand {
    uint64_t k1;
    uint32_t k2, pos, link, prev;
  };
  std::vector<Cand> c;
  for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) {
    if (g->meta[e] & ORH_META_DOWN) continue;
    const uint32_t link = g->meta[e] & ORH_META_LINK_MASK;
    if (!ign.empty() && std::binary_search(ign.begin(), ign.end(), link)) continue;
    const uint32_t u = g->col[e];
    const uint64_t du = row.dist[u];
    if (du == ~0ull) continue;
    if (u != src && g->overloaded[u]) continue;
    if (du + g->w_in[e] != dv) continue;
    if (!row.rank.empty() && row.rank[u] > row.rank[v]) continue;
    uint32_t pos = 0;
    for (uint32_t f = g->row_ptr[u]; f < g->row_ptr[u + 1]; ++f, ++pos)
      if ((g->meta[f] & ORH_META_LINK_MASK) == link && g->col[f] == v) break;
    if (row.rank.empty()) c.push_back({du, g->name_rank[u], pos, link, u});
    else c.push_back({row.rank[u], 0u, pos, link, u});
  }
  std::sort(c.begin(), c.end(), [](const Cand& a, const Cand& b) {
    if (a.k1 != b.k1) return a.k1 < b.k1;
    if (a.k2 != b.k2) return a.k2 < b.k2;
    return a.pos < b.pos;
  });
  for (const auto& x : c) out.emplace_back(x.link, x.prev);
}

// traceOnePath (LinkState.cpp:398-419): greedy DFS dst -> src; a link is
// consumed on first touch even when its branch fails. false = no path.
bool ksp_trace(const orh_graph* g, uint32_t src, uint32_t dst, const KspRow& row,
               const std::vector<uint32_t>& ign, std::vector<uint8_t>& visited,
               std::vector<uint32_t>& path) {
  if (src == dst) return true;
  std::vector<std::pair<uint32_t, uint32_t>> links;
  ksp_path_links(g, src, row, dst, ign, links);
  for (const auto& [link, prev] : links) {
    if (visited[link]) continue;
    visited[link] = 1;
    if (ksp_trace(g, src, prev, row, ign, visited, path)) {
      path.push_back(link);
      return true;
    }
  }
  return false;
}

// successive traces sharing one visited-link set (LinkState.cpp:778-787)
std::vector<std::vector<uint32_t>> ksp_paths(const orh_graph* g, uint32_t src, uint32_t dst,
                                             const KspRow& row, const std::vector<uint32_t>& ign) {
  std::vector<std::vector<uint32_t>> paths;
  if (src != dst && row.dist[dst] == ~0ull) return paths;
  std::vector<uint8_t> visited(std::max<uint32_t>(g->n_links, 1), 0);
  for (;;) {
    std::vector<uint32_t> p;
    if (!ksp_trace(g, src, dst, row, ign, visited, p) || p.empty()) break;
    paths.push_back(std::move(p));
  }
  return paths;
}

}  // namespace

extern "C" {

int orh_ksp2(orh_graph* g, uint32_t src, const uint32_t* dsts, uint32_t n_dst, uint32_t* out,
             size_t cap, size_t* n_words) {
  if (!g || !n_words || (n_dst && !dsts) || (cap && !out)) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  join_deferred(ctx);
  if (!g->d_recs || g->n_nodes == 0) return fail(ctx, ORH_E_STATE, "orh_ksp2: no graph loaded");
  if (src >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_ksp2: source out of range");
  for (uint32_t i = 0; i < n_dst; ++i)
    if (dsts[i] >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_ksp2: destination out of range");
  for (uint32_t e = 0; e < g->n_edges; ++e)
    if (g->meta[e] != ORH_META_EMPTY && (g->meta[e] & ORH_META_LINK_MASK) >= std::max<uint32_t>(g->n_links, 1))
      return fail(ctx, ORH_E_INVALID, "orh_ksp2: link id >= n_links");
  // k = 1: src's own SPF
  std::vector<KspRow> base;
  int rc = ksp_rows(g, src, 1, nullptr, nullptr, base);
  if (rc) return rc;
  const std::vector<uint32_t> none;
  std::vector<std::vector<std::vector<uint32_t>>> k1(n_dst), k2(n_dst);
  std::vector<uint32_t> ptr(1, 0), ign;
  std::vector<std::vector<uint32_t>> sets(n_dst);
  for (uint32_t i = 0; i < n_dst; ++i) {
    k1[i] = ksp_paths(g, src, dsts[i], base[0], none);
    for (const auto& p : k1[i]) sets[i].insert(sets[i].end(), p.begin(), p.end());
    std::sort(sets[i].begin(), sets[i].end());
    sets[i].erase(std::unique(sets[i].begin(), sets[i].end()), sets[i].end());
  }
  // k = 2: one fresh SPF per destination whose k = 1 paths exist; without
  // k = 1 links the memoized row serves (LinkState.cpp:775-776)
  std::vector<uint32_t> fresh;
  for (uint32_t i = 0; i < n_dst; ++i) {
    if (sets[i].empty()) continue;
    fresh.push_back(i);
    ign.insert(ign.end(), sets[i].begin(), sets[i].end());
    ptr.push_back(static_cast<uint32_t>(ign.size()));
  }
  std::vector<KspRow> rows;
  if (!fresh.empty()) {
    rc = ksp_rows(g, src, static_cast<uint32_t>(fresh.size()), ptr.data(), ign.data(), rows);
    if (rc) return rc;
  }
  for (uint32_t i = 0, f = 0; i < n_dst; ++i) {
    if (sets[i].empty()) {
      k2[i] = ksp_paths(g, src, dsts[i], base[0], none);
    } else {
      k2[i] = ksp_paths(g, src, dsts[i], rows[f++], sets[i]);
    }
  }
  size_t need = 0;
  for (uint32_t i = 0; i < n_dst; ++i)
    for (const auto* ks : {&k1[i], &k2[i]}) {
      need += 1;
      for (const auto& p : *ks) need += 1 + p.size();
    }
  *n_words = need;
  if (need > cap) return cap ? fail(ctx, ORH_E_INVALID, "orh_ksp2: output buffer too small") : ORH_OK;
  size_t w = 0;
  for (uint32_t i = 0; i < n_dst; ++i)
    for (const auto* ks : {&k1[i], &k2[i]}) {
      out[w++] = static_cast<uint32_t>(ks->size());
      for (const auto& p : *ks) {
        out[w++] = static_cast<uint32_t>(p.size());
        for (uint32_t l : p) out[w++] = l;
      }
    }
  return ORH_OK;
}

// KSP2 for a batch of (src, dst) pairs on the device: the sources' plain
// rows, the k = 1 traces (ksp_trace_kernel), the k = 2 searches with each
// pair's k = 1 links ignored (spf_global_nh kernel over the pairs that have
// k = 1 paths), the k = 2 traces; only the paths leave the device
constexpr uint32_t kKspOutCap = 1024, kKspIgnCap = 512, kKspHashCap = 2048, kKspStackCap = 1024;
constexpr uint32_t kKspChunk = 2048;

int orh_ksp2_batch(orh_graph* g, uint32_t n_pairs, const uint32_t* h_src, const uint32_t* h_dst,
                   const uint32_t** out_blocks, uint32_t* block_words) {
  if (!g || !out_blocks || !block_words || (n_pairs && (!h_src || !h_dst))) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  join_deferred(ctx);
  if (!g->d_recs || g->n_nodes == 0) return fail(ctx, ORH_E_STATE, "orh_ksp2_batch: no graph loaded");
  if (g->has_zero || wide_metrics(g))
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_ksp2_batch: zero / 64-bit path metrics need the exact kernel's order");
  const uint32_t N = g->n_nodes;
  for (uint32_t i = 0; i < n_pairs; ++i)
    if (h_src[i] >= N || h_dst[i] >= N) return fail(ctx, ORH_E_INVALID, "orh_ksp2_batch: node out of range");
  *block_words = kKspOutCap;
  const size_t out_words = static_cast<size_t>(n_pairs) * kKspOutCap;
  if (out_words > ctx->h_ksp_cap) {
    if (ctx->h_ksp) hipHostFree(ctx->h_ksp);
    ctx->h_ksp = nullptr;
    ctx->h_ksp_cap = 0;
    ORH_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_ksp), std::max<size_t>(out_words, 1) * 4,
                               hipHostMallocDefault));
    ctx->h_ksp_cap = std::max<size_t>(out_words, 1);
  }
  *out_blocks = ctx->h_ksp;
  if (n_pairs == 0) return ORH_OK;
  hipSetDevice(ctx->device);
  int rc = ensure_rev(g);
  if (rc) return rc;
  const uint64_t bound = g->sum_max_metric / 2 + g->max_metric;
  const bool uniform = g->min_out == g->max_out;
  uint32_t chunk = kKspChunk;  // ORH_KSP_CHUNK: pairs per device pass (A/B)
  if (const char* e = getenv("ORH_KSP_CHUNK")) chunk = std::max(1, atoi(e));
  // ORH_KSP_PROF=1: host and device (events) time of each stage on stderr
  const bool prof = getenv("ORH_KSP_PROF") != nullptr;
  constexpr int kStages = 7;
  static const char* const kStageName[kStages] = {"stage", "k1 search", "k1 trace", "k2 search", "k2 trace",
                                                  "copy-out", ""};
  hipEvent_t ev[kStages] = {};
  double host_ms[kStages] = {};
  auto h_now = [] { return std::chrono::steady_clock::now(); };
  auto t_host = h_now();
  auto mark = [&](int k) {
    if (!prof) return;
    if (!ev[k]) hipEventCreate(&ev[k]);
    hipEventRecord(ev[k], ctx->stream);
    const auto t = h_now();
    host_ms[k] += std::chrono::duration<double, std::milli>(t - t_host).count();
    t_host = t;
  };
  for (uint32_t c0 = 0; c0 < n_pairs; c0 += chunk) {
    mark(0);
    const uint32_t P = std::min(chunk, n_pairs - c0);
    // distinct sources of the chunk, and each pair's row among them
    std::vector<uint32_t> srcs, row1(P), rowp(P);
    auto& ro = g->row_of;
    for (uint32_t i = 0; i < P; ++i) {
      const uint32_t x = h_src[c0 + i];
      if (ro[x] < 0) {
        ro[x] = static_cast<int32_t>(srcs.size());
        srcs.push_back(x);
      }
      row1[i] = static_cast<uint32_t>(ro[x]);
      rowp[i] = i;
    }
    for (uint32_t x : srcs) ro[x] = -1;
    const uint32_t S = static_cast<uint32_t>(srcs.size());
    // device layout (u32 words): the staged request first - src | dst | row1 |
    // rowp | ign_ptr [P+1] | sources [S] | stop targets - then dist1 [S][N] |
    // dist2 [P][N] | ign [P][cap] | need2 | out | visited | stack
    // (the traces read distances only: both searches run dist-only)
    const size_t nd1 = static_cast<size_t>(S) * N, nd2 = static_cast<size_t>(P) * N;
    size_t off = 0;
    auto take = [&](size_t words_) {
      const size_t o = off;
      off += (words_ + 63) & ~size_t{63};  // 256-byte aligned pieces
      return o;
    };
    const size_t o_src = take(P), o_dst = take(P), o_r1 = take(P), o_rp = take(P), o_ip = take(P + 1);
    const size_t o_s1 = take(S);
    // early-stop targets of the searches: the k = 1 row of a source stops once
    // all its pairs' destinations are final, a k = 2 row once its pair's is
    const size_t o_sp1 = take(S + 1), o_sn1 = take(P), o_sp2 = take(P + 1);
    const size_t staged = off;  // words uploaded in one copy
    const size_t o_d1 = take(nd1), o_d2 = take(nd2);
    const size_t o_ign = take(size_t{P} * kKspIgnCap), o_need = take(P), o_out = take(size_t{P} * kKspOutCap);
    const size_t o_vis = take(size_t{P} * kKspHashCap);
    const size_t o_st = take(size_t{P} * kKspStackCap * (sizeof(orh::KspFrame) / 4));
    const size_t o_ovf = take(size_t{std::max(S, P)} + 1);
    const size_t o_ord = take(P);  // k = 2 search order (longest first)
    rc = ensure_bytes(ctx, &ctx->d_ksp, &ctx->d_ksp_cap, off * 4);
    if (rc) return rc;
    uint32_t* D = reinterpret_cast<uint32_t*>(ctx->d_ksp);
    // the staged request is assembled in this chunk's pinned output block
    // (its copy-out comes later on the same stream) and goes up in one copy
    uint32_t* H = ctx->h_ksp + size_t{c0} * kKspOutCap;
    if (staged > size_t{P} * kKspOutCap) return fail(ctx, ORH_E_INVALID, "orh_ksp2_batch: staging block too small");
    std::memcpy(H + o_src, h_src + c0, P * 4ull);
    std::memcpy(H + o_dst, h_dst + c0, P * 4ull);
    std::memcpy(H + o_r1, row1.data(), P * 4ull);
    std::memcpy(H + o_rp, rowp.data(), P * 4ull);
    for (uint32_t i = 0; i <= P; ++i) H[o_ip + i] = i * kKspIgnCap;  // fixed-stride ignore lists
    std::memcpy(H + o_s1, srcs.data(), S * 4ull);
    const char* stop_e = getenv("ORH_KSP_STOP");  // 0: full searches (A/B)
    const bool stop = !(stop_e && stop_e[0] == '0');
    if (stop) {
      uint32_t* sp1 = H + o_sp1;
      std::fill(sp1, sp1 + S + 1, 0u);
      for (uint32_t i = 0; i < P; ++i) ++sp1[row1[i] + 1];
      for (uint32_t r = 0; r < S; ++r) sp1[r + 1] += sp1[r];
      std::vector<uint32_t> fill(sp1, sp1 + S);
      for (uint32_t i = 0; i < P; ++i) H[o_sn1 + fill[row1[i]]++] = h_dst[c0 + i];
      for (uint32_t i = 0; i <= P; ++i) H[o_sp2 + i] = i;
    }
    ORH_HIP(ctx, hipMemcpyAsync(D, H, staged * 4ull, hipMemcpyHostToDevice, ctx->stream));
    ORH_HIP(ctx, hipMemsetAsync(D + o_vis, 0, size_t{P} * kKspHashCap * 4, ctx->stream));
    // both searches: the HBM frontier kernel, distances only (u32 labels)
    orh::SpfPlan fp = orh::plan_spf(N, uniform, bound, g->ell_k, ctx->lds_limit, false, orh::SpfMode::kGlobal);
    if (fp.variant == orh::SpfVariant::kUnsupported)
      return fail(ctx, ORH_E_UNSUPPORTED, "orh_ksp2_batch: no search plan for this graph");
    fp.variant = orh::SpfVariant::kGlobalNh;
    auto block_for = [&](uint32_t rows) { return rows <= ctx->n_cu ? 1024u : rows <= 2 * ctx->n_cu ? 512u : 256u; };
    // one search per CU with u16 distances in LDS when they fit (the HBM
    // kernel finishes any row that needs wider distances); ORH_KSP_LDS=0: the
    // HBM kernel for every row (A/B)
    const char* lds_e = getenv("ORH_KSP_LDS");
    const bool lds_env = !(lds_e && lds_e[0] == '0');
    const bool use_lds16 = lds_env && orh::lds16_bytes(N) <= ctx->lds_limit;
    auto search = [&](const orh::SpfArgs& sa, uint32_t rows) {
      return use_lds16 ? orh::launch_spf_lds16(fp, sa, rows, g->ell_k, ctx->stream)
                       : orh::launch_spf(fp, sa, rows, ctx->stream);
    };
    rc = ensure_labels(ctx, (std::max(nd1, nd2) + 1) / 2);  // u64 units, u32 labels
    if (rc) return rc;
    orh::SpfArgs a{};
    a.n_nodes = N;
    a.recs = g->d_recs;
    a.link = g->d_link;
    a.use_link_metric = 1;
    a.w0 = g->max_out;
    a.delta = uniform ? a.w0
                      : std::max<uint32_t>(1u, static_cast<uint32_t>(
                                                   static_cast<uint64_t>(g->mean_out) * ctx->delta_pct / 100u));
    a.scratch = ctx->d_scratch;
    a.labels = ctx->d_labels;
    a.words = 1;
    a.rank_out = g->d_rank_out;
    a.dist_only = 1;
    a.ovf_rows = D + o_ovf;
    // k = 1 rows: the sources' plain SPFs (LinkState::getSpfResult), as far
    // as their pairs' destinations (the rows feed the k = 1 traces only)
    a.n_out = S;
    a.srcs = D + o_s1;
    a.out_dist = D + o_d1;
    a.stop_ptr = stop ? D + o_sp1 : nullptr;
    a.stop_nodes = stop ? D + o_sn1 : nullptr;
    fp.block = block_for(S);
    const orh_counters c_before = ctx->counters;
    mark(1);
    hipError_t e = search(a, S);
    if (e != hipSuccess) return hip_fail(ctx, e, "ksp2 k=1 search launch");
    mark(2);
    orh::KspArgs ka{};
    ka.n_nodes = N;
    ka.n_pairs = P;
    ka.recs = g->d_recs;
    ka.link = g->d_link;
    ka.rev = g->d_rev;
    ka.name_rank = g->d_name_rank;
    ka.src = D + o_src;
    ka.dst = D + o_dst;
    ka.ign = D + o_ign;
    ka.ign_cap = kKspIgnCap;
    ka.need2 = D + o_need;
    ka.out = D + o_out;
    ka.out_cap = kKspOutCap;
    ka.visited = D + o_vis;
    ka.hash_cap = kKspHashCap;
    ka.stack = reinterpret_cast<orh::KspFrame*>(D + o_st);
    ka.stack_cap = kKspStackCap;
    ka.k = 1;
    ka.row = D + o_r1;
    ka.dist = D + o_d1;
    e = orh::launch_ksp_trace(ka, g->ell_k, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "ksp2 k=1 trace launch");
    mark(3);
    // k = 2 searches: every pair with k = 1 paths, its k = 1 links ignored
    // (row mask = need2)
    a.n_out = P;
    a.srcs = D + o_src;
    a.ignore_ptr = D + o_ip;
    a.ignore_links = D + o_ign;
    a.out_dist = D + o_d2;
    a.row_mask = D + o_need;
    a.stop_ptr = stop ? D + o_sp2 : nullptr;
    a.stop_nodes = stop ? D + o_dst : nullptr;
    // the LDS searches start with the pairs whose k = 1 destination is
    // farthest (ORH_KSP_ORDER=0: pair order, A/B)
    static const bool by_dist = [] {
      const char* oe = getenv("ORH_KSP_ORDER");
      return !(oe && oe[0] == '0');
    }();
    if (use_lds16 && by_dist && P <= 4096) {
      e = orh::launch_ksp_order(D + o_d1, D + o_r1, D + o_dst, D + o_need, N, P, D + o_ord, ctx->stream);
      if (e != hipSuccess) return hip_fail(ctx, e, "ksp2 order launch");
      a.row_order = D + o_ord;
    }
    fp.block = block_for(P);
    e = search(a, P);
    a.row_order = nullptr;
    if (e != hipSuccess) return hip_fail(ctx, e, "ksp2 k=2 search launch");
    mark(4);
    ORH_HIP(ctx, hipMemsetAsync(D + o_vis, 0, size_t{P} * kKspHashCap * 4, ctx->stream));
    ka.k = 2;
    ka.row = D + o_rp;
    ka.dist = D + o_d2;
    e = orh::launch_ksp_trace(ka, g->ell_k, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "ksp2 k=2 trace launch");
    mark(5);
    ORH_HIP(ctx, hipMemcpyAsync(ctx->h_ksp + size_t{c0} * kKspOutCap, D + o_out, size_t{P} * kKspOutCap * 4,
                                hipMemcpyDeviceToHost, ctx->stream));
    mark(6);
    ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->counters = c_before;  // the caller counts runs the reference's way (memo)
    ctx->counters.spf_launches += 3;
    if (prof) {  // stage k: host time to issue it, device time between its events
      for (int k = 0; k + 1 < kStages; ++k) {
        float d = 0.f;
        hipEventElapsedTime(&d, ev[k], ev[k + 1]);
        std::fprintf(stderr, "ksp-batch %-10s host %8.3f ms  device %8.3f ms\n", kStageName[k], host_ms[k + 1], d);
      }
      std::fprintf(stderr, "ksp-batch after copy-out sync host %8.3f ms\n",
                   std::chrono::duration<double, std::milli>(h_now() - t_host).count());
      if (use_lds16) {
        uint32_t n_ovf = 0;
        ORH_HIP(ctx, hipMemcpy(&n_ovf, D + o_ovf, 4, hipMemcpyDeviceToHost));
        std::fprintf(stderr, "ksp-batch lds16: %u of %u k=2 rows re-run by the HBM kernel\n", n_ovf, P);
      }
      for (double& h : host_ms) h = 0;
    }
  }
  if (prof)
    for (auto& e : ev)
      if (e) hipEventDestroy(e);
  return ORH_OK;
}

// ---- device prefix mirror + route selection ---------------------------------
}  // extern "C"

struct orh_prefix_set {
  orh_ctx* ctx = nullptr;
  // host mirror of the device arrays (compaction and growth)
  std::vector<uint2> hdr;     // {pool offset, count | prefix flags << 16}
  std::vector<orh_adv> pool;  // advertisement runs, appended on update
  uint32_t live = 0;          // records referenced by a header
  uint2* d_hdr = nullptr;
  size_t hdr_cap = 0;
  orh_adv* d_pool = nullptr;
  size_t pool_cap = 0;
  uint32_t* d_rank = nullptr;  // name ranks then area ranks
  size_t rank_cap = 0;
  uint32_t n_names = 0, n_areas = 0;
  orh::SelArea* d_areas = nullptr;
  std::vector<orh::SelArea> h_areas;
  uint32_t* d_stage = nullptr;
  size_t stage_cap = 0;  // in u32
  uint32_t* d_pol = nullptr;  // policy tables (orh_route_policy)
  size_t pol_cap = 0;         // in u32
  std::vector<uint32_t> h_pol;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the last route_select launch
};

namespace {

int grow(orh_ctx* ctx, void** d, size_t* cap, size_t need, size_t elem, size_t keep) {
  if (need <= *cap) return ORH_OK;
  const size_t ncap = std::max(need, *cap * 2);
  void* nd = nullptr;
  ORH_HIP(ctx, hipMalloc(&nd, ncap * elem));
  if (*d && keep)
    ORH_HIP(ctx, hipMemcpyAsync(nd, *d, keep * elem, hipMemcpyDeviceToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  (void)hipFree(*d);
  *d = nd;
  *cap = ncap;
  return ORH_OK;
}

int stage(orh_prefix_set* ps, size_t words) {
  return grow(ps->ctx, reinterpret_cast<void**>(&ps->d_stage), &ps->stage_cap, words, 4, 0);
}

// room for a quarter more: the deltas that follow a full load append
// without reallocating (C5: 10k changed prefixes after a 1M-prefix load took
// 30 ms in the host and device pool growth alone)
size_t with_headroom(size_t n) { return n + n / 4 + 1024; }

int upload_all(orh_prefix_set* ps) {
  orh_ctx* ctx = ps->ctx;
  int rc = grow(ctx, reinterpret_cast<void**>(&ps->d_hdr), &ps->hdr_cap, with_headroom(ps->hdr.size()),
                sizeof(uint2), 0);
  if (rc) return rc;
  rc = grow(ctx, reinterpret_cast<void**>(&ps->d_pool), &ps->pool_cap, with_headroom(ps->pool.size()),
            sizeof(orh_adv), 0);
  if (rc) return rc;
  if (!ps->hdr.empty())
    ORH_HIP(ctx, hipMemcpyAsync(ps->d_hdr, ps->hdr.data(), ps->hdr.size() * sizeof(uint2),
                                hipMemcpyHostToDevice, ctx->stream));
  if (!ps->pool.empty())
    ORH_HIP(ctx, hipMemcpyAsync(ps->d_pool, ps->pool.data(), ps->pool.size() * sizeof(orh_adv),
                                hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

}  // namespace

extern "C" {

int orh_prefix_create(orh_ctx* ctx, orh_prefix_set** out) {
  if (!ctx || !out) return ORH_E_INVALID;
  auto* ps = new (std::nothrow) orh_prefix_set();
  if (!ps) return ORH_E_NOMEM;
  ps->ctx = ctx;
  *out = ps;
  return ORH_OK;
}

int orh_prefix_destroy(orh_prefix_set* ps) {
  if (!ps) return ORH_E_INVALID;
  hipSetDevice(ps->ctx->device);
  hipStreamSynchronize(ps->ctx->stream);
  hipFree(ps->d_hdr);
  hipFree(ps->d_pool);
  hipFree(ps->d_rank);
  hipFree(ps->d_areas);
  hipFree(ps->d_stage);
  hipFree(ps->d_pol);
  if (ps->ev0) hipEventDestroy(ps->ev0);
  if (ps->ev1) hipEventDestroy(ps->ev1);
  delete ps;
  return ORH_OK;
}

int orh_prefix_load(orh_prefix_set* ps, uint32_t n_prefix, const uint32_t* adv_ptr,
                    const orh_adv* advs, const uint8_t* pflags) {
  if (!ps || (n_prefix && (!adv_ptr || !pflags))) return ORH_E_INVALID;
  orh_ctx* ctx = ps->ctx;
  const uint32_t n_adv = n_prefix ? adv_ptr[n_prefix] : 0;
  if (n_adv && !advs) return fail(ctx, ORH_E_INVALID, "orh_prefix_load: null advertisements");
  for (uint32_t p = 0; p < n_prefix; ++p)
    if (adv_ptr[p + 1] < adv_ptr[p] || adv_ptr[p + 1] - adv_ptr[p] > 0xFFFFu)
      return fail(ctx, ORH_E_INVALID, "orh_prefix_load: bad adv_ptr / > 65535 advertisements");
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  ps->hdr.reserve(with_headroom(n_prefix));
  ps->hdr.resize(n_prefix);
  for (uint32_t p = 0; p < n_prefix; ++p)
    ps->hdr[p] = make_uint2(adv_ptr[p], (adv_ptr[p + 1] - adv_ptr[p]) | (uint32_t(pflags[p]) << 16));
  ps->pool.reserve(with_headroom(n_adv));
  ps->pool.assign(advs, advs + n_adv);
  ps->live = n_adv;
  return upload_all(ps);
}

int orh_prefix_apply_delta(orh_prefix_set* ps, uint32_t n, const uint32_t* ids,
                           const uint32_t* adv_ptr, const orh_adv* advs, const uint8_t* pflags) {
  if (!ps || (n && (!ids || !adv_ptr || !pflags))) return ORH_E_INVALID;
  if (n == 0) return ORH_OK;
  orh_ctx* ctx = ps->ctx;
  const uint32_t n_adv = adv_ptr[n];
  if (n_adv && !advs) return fail(ctx, ORH_E_INVALID, "orh_prefix_apply_delta: null advertisements");
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  uint32_t max_id = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (adv_ptr[i + 1] < adv_ptr[i] || adv_ptr[i + 1] - adv_ptr[i] > 0xFFFFu)
      return fail(ctx, ORH_E_INVALID, "orh_prefix_apply_delta: bad adv_ptr");
    max_id = std::max(max_id, ids[i]);
  }
  const size_t old_n = ps->hdr.size();
  if (max_id >= old_n) ps->hdr.resize(static_cast<size_t>(max_id) + 1, make_uint2(0u, 0u));
  const uint32_t base = static_cast<uint32_t>(ps->pool.size());
  std::vector<uint2> vals(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint2& h = ps->hdr[ids[i]];
    ps->live -= h.y & 0xFFFFu;
    const uint32_t c = adv_ptr[i + 1] - adv_ptr[i];
    h = make_uint2(base + adv_ptr[i], c | (uint32_t(pflags[i]) << 16));
    ps->live += c;
    vals[i] = h;
  }
  ps->pool.insert(ps->pool.end(), advs, advs + n_adv);
  // mostly garbage: rebuild the pool from the live runs and re-upload
  if (ps->pool.size() > 4096 && ps->pool.size() > 2 * static_cast<size_t>(ps->live)) {
    std::vector<orh_adv> packed;
    packed.reserve(with_headroom(ps->live));
    for (auto& h : ps->hdr) {
      const uint32_t c = h.y & 0xFFFFu;
      const uint32_t off = static_cast<uint32_t>(packed.size());
      packed.insert(packed.end(), ps->pool.begin() + h.x, ps->pool.begin() + h.x + c);
      h.x = off;
    }
    ps->pool.swap(packed);
    return upload_all(ps);
  }
  int rc = grow(ctx, reinterpret_cast<void**>(&ps->d_hdr), &ps->hdr_cap, ps->hdr.size(),
                sizeof(uint2), old_n);
  if (rc) return rc;
  if (ps->hdr.size() > old_n)  // new ids start withdrawn
    ORH_HIP(ctx, hipMemsetAsync(ps->d_hdr + old_n, 0, (ps->hdr.size() - old_n) * sizeof(uint2),
                                ctx->stream));
  rc = grow(ctx, reinterpret_cast<void**>(&ps->d_pool), &ps->pool_cap, std::max<size_t>(ps->pool.size(), 1),
            sizeof(orh_adv), base);
  if (rc) return rc;
  if (n_adv)
    ORH_HIP(ctx, hipMemcpyAsync(ps->d_pool + base, advs, static_cast<size_t>(n_adv) * sizeof(orh_adv),
                                hipMemcpyHostToDevice, ctx->stream));
  // staging: ids[n] (padded to 8 bytes) | headers[n]
  const size_t id_words = (n + 1) & ~1u;
  std::vector<uint32_t> st(id_words + 2 * static_cast<size_t>(n));
  std::copy(ids, ids + n, st.begin());
  std::memcpy(st.data() + id_words, vals.data(), n * sizeof(uint2));
  rc = stage(ps, st.size());
  if (rc) return rc;
  ORH_HIP(ctx, hipMemcpyAsync(ps->d_stage, st.data(), st.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, orh::launch_scatter_hdr(ps->d_hdr, ps->d_stage,
                                       reinterpret_cast<const uint2*>(ps->d_stage + id_words), n,
                                       ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // st is a local
  return ORH_OK;
}

int orh_prefix_set_order(orh_prefix_set* ps, uint32_t n_names, const uint32_t* name_rank,
                         uint32_t n_areas, const uint32_t* area_rank) {
  if (!ps || (n_names && !name_rank) || (n_areas && !area_rank)) return ORH_E_INVALID;
  orh_ctx* ctx = ps->ctx;
  if (n_areas > 256) return fail(ctx, ORH_E_UNSUPPORTED, "orh_prefix_set_order: more than 256 areas");
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  const size_t words = static_cast<size_t>(n_names) + 256;
  int rc = grow(ctx, reinterpret_cast<void**>(&ps->d_rank), &ps->rank_cap, words, 4, 0);
  if (rc) return rc;
  std::vector<uint32_t> r(words, 0xFFFFFFFFu);
  std::copy(name_rank, name_rank + n_names, r.begin());
  std::copy(area_rank, area_rank + n_areas, r.begin() + n_names);
  ORH_HIP(ctx, hipMemcpyAsync(ps->d_rank, r.data(), words * 4, hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ps->n_names = n_names;
  ps->n_areas = n_areas;
  return ORH_OK;
}

int orh_prefix_info(const orh_prefix_set* ps, uint32_t* n_prefix, uint32_t* n_live, uint32_t* n_pool) {
  if (!ps) return ORH_E_INVALID;
  if (n_prefix) *n_prefix = static_cast<uint32_t>(ps->hdr.size());
  if (n_live) *n_live = ps->live;
  if (n_pool) *n_pool = static_cast<uint32_t>(ps->pool.size());
  return ORH_OK;
}

int orh_route_select(orh_prefix_set* ps, uint32_t me_name, uint32_t flags, uint32_t n_areas,
                     const orh_select_area* areas, const orh_select_out* out) {
  if (!ps) return ORH_E_INVALID;
  return orh_route_select_range(ps, me_name, flags, n_areas, areas, 0, static_cast<uint32_t>(ps->hdr.size()), out);
}

int orh_route_select_range(orh_prefix_set* ps, uint32_t me_name, uint32_t flags, uint32_t n_areas,
                           const orh_select_area* areas, uint32_t pid_lo, uint32_t pid_hi,
                           const orh_select_out* out) {
  if (!ps || !out || (n_areas && !areas)) return ORH_E_INVALID;
  orh_ctx* ctx = ps->ctx;
  join_deferred(ctx);
  if (pid_lo > pid_hi || pid_hi > ps->hdr.size())
    return fail(ctx, ORH_E_INVALID, "orh_route_select_range: range beyond the prefix set");
  const uint32_t n_prefix = pid_hi;
  if (pid_lo == pid_hi) return ORH_OK;
  if (n_areas > orh::kMaxSelectAreas)
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_route_select: more than 32 areas");
  if (!out->d_status || !out->d_metric || !out->d_best || (out->total_words && !out->d_mask))
    return fail(ctx, ORH_E_INVALID, "orh_route_select: null output");
  if (!ps->d_rank) return fail(ctx, ORH_E_STATE, "orh_route_select: orh_prefix_set_order not called");
  uint32_t words = 0;
  for (uint32_t b = 0; b < n_areas; ++b) {
    const orh_select_area& A = areas[b];
    if (A.d_dist && (!A.d_nh || !A.d_overloaded || !A.d_name_node || A.words == 0))
      return fail(ctx, ORH_E_INVALID, "orh_route_select: incomplete area");
    if (A.word_off + A.words > out->total_words)
      return fail(ctx, ORH_E_INVALID, "orh_route_select: area words exceed total_words");
    words += A.words;
  }
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  if (!ps->d_areas) ORH_HIP(ctx, hipMalloc(&ps->d_areas, orh::kMaxSelectAreas * sizeof(orh::SelArea)));
  ps->h_areas.assign(orh::kMaxSelectAreas, orh::SelArea{});
  for (uint32_t b = 0; b < n_areas; ++b)
    ps->h_areas[b] = orh::SelArea{areas[b].present, areas[b].d_dist, areas[b].d_nh, areas[b].d_overloaded,
                                  areas[b].d_name_node, areas[b].words, areas[b].word_off};
  ORH_HIP(ctx, hipMemcpyAsync(ps->d_areas, ps->h_areas.data(), n_areas * sizeof(orh::SelArea),
                              hipMemcpyHostToDevice, ctx->stream));
  orh::RouteSelectArgs a{};
  a.pid_lo = pid_lo;
  a.n_prefix = n_prefix;
  a.hdr = ps->d_hdr;
  a.adv = ps->d_pool;
  a.name_rank = ps->d_rank;
  a.area_rank = ps->d_rank + ps->n_names;
  a.n_names = ps->n_names;
  a.me_name = me_name;
  a.flags = flags;
  a.n_areas = n_areas;
  a.areas = ps->d_areas;
  a.status = out->d_status;
  a.metric = out->d_metric;
  a.best = out->d_best;
  a.mask = out->d_mask;
  a.total_words = out->total_words;
  if (!ps->ev0) {
    ORH_HIP(ctx, hipEventCreate(&ps->ev0));
    ORH_HIP(ctx, hipEventCreate(&ps->ev1));
  }
  ORH_HIP(ctx, hipEventRecord(ps->ev0, ctx->stream));
  hipError_t e = orh::launch_route_select(a, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "route_select launch");
  ORH_HIP(ctx, hipEventRecord(ps->ev1, ctx->stream));
  (void)words;
  return ORH_OK;
}

int orh_route_diff(orh_prefix_set* ps, uint32_t n_prefix, uint32_t prev_n, const orh_select_out* cur,
                   const orh_select_out* prev, uint32_t* d_changed, uint32_t* d_count) {
  if (!ps || !cur || !prev || !d_changed || !d_count) return ORH_E_INVALID;
  orh_ctx* ctx = ps->ctx;
  if (cur->total_words != prev->total_words)
    return fail(ctx, ORH_E_INVALID, "orh_route_diff: different mask widths");
  if (!cur->d_status || !cur->d_metric || !cur->d_best || !prev->d_status || !prev->d_metric || !prev->d_best ||
      (cur->total_words && (!cur->d_mask || !prev->d_mask)))
    return fail(ctx, ORH_E_INVALID, "orh_route_diff: null selection output");
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  ORH_HIP(ctx, hipMemsetAsync(d_count, 0, sizeof(uint32_t), ctx->stream));
  orh::RouteDiffArgs a{};
  a.n_prefix = n_prefix;
  a.prev_n = std::min(prev_n, n_prefix);
  a.words = cur->total_words;
  a.status = cur->d_status;
  a.metric = cur->d_metric;
  a.best = cur->d_best;
  a.mask = cur->d_mask;
  a.p_status = prev->d_status;
  a.p_metric = prev->d_metric;
  a.p_best = prev->d_best;
  a.p_mask = prev->d_mask;
  a.out = d_changed;
  a.count = d_count;
  hipError_t e = orh::launch_route_diff(a, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "route_diff launch");
  return ORH_OK;
}

int orh_route_policy(orh_prefix_set* ps, uint32_t n_prefix, const orh_select_out* sel,
                     const orh_policy* pol, uint8_t* d_out, uint32_t* d_invalidated) {
  return orh_route_policy_range(ps, 0, n_prefix, sel, pol, d_out, d_invalidated);
}

int orh_route_policy_range(orh_prefix_set* ps, uint32_t pid_lo, uint32_t n_prefix, const orh_select_out* sel,
                           const orh_policy* pol, uint8_t* d_out, uint32_t* d_invalidated) {
  if (!ps || !sel || !pol || !d_out || !d_invalidated) return ORH_E_INVALID;
  orh_ctx* ctx = ps->ctx;
  if (pol->n_stmts > ORH_POL_MAX_STMTS)
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_route_policy: more than 32 statements");
  if (n_prefix > ps->hdr.size() || pid_lo > n_prefix)
    return fail(ctx, ORH_E_INVALID, "orh_route_policy: prefix range beyond the set");
  if (pol->total_words != sel->total_words)
    return fail(ctx, ORH_E_INVALID, "orh_route_policy: mask widths differ");
  if (!sel->d_status || !sel->d_best || (sel->total_words && !sel->d_mask) ||
      (pol->n_tagsets && !pol->h_tagset_stmts) || (pol->n_pfx && (!pol->h_pfx_id || !pol->h_pfx_stmts)) ||
      (pol->n_stmts && pol->total_words && !pol->h_keep))
    return fail(ctx, ORH_E_INVALID, "orh_route_policy: null table");
  for (uint32_t i = 1; i < pol->n_pfx; ++i)
    if (pol->h_pfx_id[i] <= pol->h_pfx_id[i - 1])
      return fail(ctx, ORH_E_INVALID, "orh_route_policy: prefix ids not ascending");
  ORH_HIP(ctx, hipSetDevice(ctx->device));
  // a previous launch may still read the device tables, and its upload the
  // host staging: the context stream drains before either is reused
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // one upload: tag-set table | prefix ids | prefix statements | keep masks
  const size_t nk = static_cast<size_t>(pol->n_stmts) * pol->total_words;
  auto& h = ps->h_pol;
  h.clear();
  h.reserve(pol->n_tagsets + 2ull * pol->n_pfx + nk + 1);
  h.insert(h.end(), pol->h_tagset_stmts, pol->h_tagset_stmts + pol->n_tagsets);
  h.insert(h.end(), pol->h_pfx_id, pol->h_pfx_id + pol->n_pfx);
  h.insert(h.end(), pol->h_pfx_stmts, pol->h_pfx_stmts + pol->n_pfx);
  if (nk) h.insert(h.end(), pol->h_keep, pol->h_keep + nk);
  h.push_back(0u);
  int rc = grow(ctx, reinterpret_cast<void**>(&ps->d_pol), &ps->pol_cap, h.size(), 4, 0);
  if (rc) return rc;
  ORH_HIP(ctx, hipMemcpyAsync(ps->d_pol, h.data(), h.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipMemsetAsync(d_invalidated, 0, sizeof(uint32_t), ctx->stream));
  orh::RoutePolicyArgs a{};
  a.pid_lo = pid_lo;
  a.n_prefix = n_prefix;
  a.words = sel->total_words;
  a.hdr = ps->d_hdr;
  a.adv = ps->d_pool;
  a.status = sel->d_status;
  a.best = sel->d_best;
  a.mask = sel->d_mask;
  a.n_stmts = pol->n_stmts;
  a.stmt_tags = pol->stmt_tags;
  a.stmt_pfx = pol->stmt_prefixes;
  a.n_tagsets = pol->n_tagsets;
  a.tagset_stmts = ps->d_pol;
  a.n_pfx = pol->n_pfx;
  a.pfx_id = ps->d_pol + pol->n_tagsets;
  a.pfx_stmts = a.pfx_id + pol->n_pfx;
  a.keep = a.pfx_stmts + pol->n_pfx;
  a.out = d_out;
  a.invalidated = d_invalidated;
  hipError_t e = orh::launch_route_policy(a, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "route_policy launch");
  return ORH_OK;
}

int orh_last_select_ms(orh_prefix_set* ps, double* ms_out) {
  if (!ps || !ms_out) return ORH_E_INVALID;
  if (!ps->ev1) return fail(ps->ctx, ORH_E_STATE, "orh_last_select_ms: no route_select yet");
  ORH_HIP(ps->ctx, hipEventSynchronize(ps->ev1));
  float ms = 0.f;
  ORH_HIP(ps->ctx, hipEventElapsedTime(&ms, ps->ev0, ps->ev1));
  *ms_out = ms;
  return ORH_OK;
}

}  // extern "C"

// timing helper used by bench/tests through the ABI: elapsed ms of the last
// SPF launch (waits for it)
extern "C" int orh_last_spf_ms(orh_ctx* ctx, double* ms_out) {
  if (!ctx || !ms_out) return ORH_E_INVALID;
  ORH_HIP(ctx, hipEventSynchronize(ctx->ev1));
  float ms = 0.f;
  ORH_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  *ms_out = ms;
  ctx->counters.last_kernel_ms = ms;
  ctx->counters.total_kernel_ms += ms;
  return ORH_OK;
}

extern "C" int orh_last_spf_info(const orh_ctx* ctx, orh_spf_info* out) {
  if (!ctx || !out) return ORH_E_INVALID;
  *out = ctx->last_info;
  return ORH_OK;
}

extern "C" int orh_last_spf_phase_ms(orh_ctx* ctx, double* dist_ms, double* hop_ms) {
  if (!ctx || !dist_ms || !hop_ms) return ORH_E_INVALID;
  ORH_HIP(ctx, hipEventSynchronize(ctx->ev1));
  float a = 0.f, b = 0.f;
  ORH_HIP(ctx, hipEventElapsedTime(&a, ctx->ev0, ctx->evm));
  ORH_HIP(ctx, hipEventElapsedTime(&b, ctx->evm, ctx->ev1));
  *dist_ms = a;
  *hop_ms = b;
  return ORH_OK;
}
