// libopenr_hip: C ABI (include/openr_hip.h) over the gfx950 SPF kernels.
//
// Owns per-device contexts (stream, events, counters) and per-area graph
// mirrors (device CSR of 16-byte edge records, row offsets, node flags and
// the neighbour-rank table used to number first-hop bits).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/openr_hip.h"
#include "kernels/spf_kernels.h"

struct orh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  size_t lds_limit = 160 * 1024;
  std::string err;
  orh_counters counters{};
  // reusable device staging for request arrays
  uint32_t* d_req = nullptr;
  size_t d_req_cap = 0;
};

struct orh_graph {
  orh_ctx* ctx = nullptr;
  uint32_t n_nodes = 0, n_edges = 0, n_links = 0;
  // host copies (needed for deltas, neighbour tables and bounds)
  std::vector<uint32_t> row_ptr, col, w_out, w_in, meta;
  std::vector<uint8_t> overloaded;
  std::vector<uint32_t> n_distinct;  // distinct neighbour count per node
  uint64_t sum_max_metric = 0;       // sum over links of max(w_out, w_in)
  uint32_t max_metric = 0;
  // device mirror
  uint32_t* d_row_ptr = nullptr;
  uint4* d_edges = nullptr;
  uint16_t* d_rank = nullptr;
  uint8_t* d_overloaded = nullptr;
};

namespace {

int fail(orh_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(orh_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, ORH_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define ORH_HIP(ctx, call)                              \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
  } while (0)

void free_graph_device(orh_graph* g) {
  hipFree(g->d_row_ptr);
  hipFree(g->d_edges);
  hipFree(g->d_rank);
  hipFree(g->d_overloaded);
  g->d_row_ptr = nullptr;
  g->d_edges = nullptr;
  g->d_rank = nullptr;
  g->d_overloaded = nullptr;
}

// rank of the row node among col's distinct neighbours (ascending id)
std::vector<uint16_t> build_ranks(const orh_graph* g, std::vector<uint32_t>& n_distinct) {
  const uint32_t N = g->n_nodes;
  std::vector<std::vector<uint32_t>> nbrs(N);
  n_distinct.assign(N, 0);
  for (uint32_t v = 0; v < N; ++v) {
    auto& l = nbrs[v];
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) l.push_back(g->col[e]);
    std::sort(l.begin(), l.end());
    l.erase(std::unique(l.begin(), l.end()), l.end());
    n_distinct[v] = static_cast<uint32_t>(l.size());
  }
  std::vector<uint16_t> rank(g->n_edges, 0);
  for (uint32_t v = 0; v < N; ++v) {
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) {
      const auto& l = nbrs[g->col[e]];
      const auto it = std::lower_bound(l.begin(), l.end(), v);
      const size_t r = static_cast<size_t>(it - l.begin());
      rank[e] = static_cast<uint16_t>(std::min<size_t>(r, 0xFFFF));
    }
  }
  return rank;
}

int upload_edges(orh_graph* g, uint32_t first, uint32_t count) {
  std::vector<uint4> rec(count);
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t e = first + i;
    rec[i] = make_uint4(g->col[e], g->w_out[e], g->w_in[e], g->meta[e]);
  }
  ORH_HIP(g->ctx, hipMemcpyAsync(g->d_edges + first, rec.data(), count * sizeof(uint4),
                                 hipMemcpyHostToDevice, g->ctx->stream));
  return ORH_OK;
}

void recompute_bounds(orh_graph* g) {
  g->sum_max_metric = 0;
  g->max_metric = 0;
  for (uint32_t e = 0; e < g->n_edges; ++e) {
    const uint32_t m = std::max(g->w_out[e], g->w_in[e]);
    g->max_metric = std::max(g->max_metric, m);
    g->sum_max_metric += m;  // each link is counted twice (both CSR entries)
  }
}

int ensure_req(orh_ctx* ctx, size_t words) {
  if (words <= ctx->d_req_cap) return ORH_OK;
  hipFree(ctx->d_req);
  ctx->d_req = nullptr;
  const size_t cap = std::max<size_t>(words, 4096);
  ORH_HIP(ctx, hipMalloc(&ctx->d_req, cap * sizeof(uint32_t)));
  ctx->d_req_cap = cap;
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
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return ORH_E_DEVICE;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.sharedMemPerBlock > 0) {
    ctx->lds_limit = std::max<size_t>(prop.sharedMemPerBlock, 64 * 1024);
  }
  *out = ctx;
  return ORH_OK;
}

int orh_destroy(orh_ctx* ctx) {
  if (!ctx) return ORH_E_INVALID;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  hipFree(ctx->d_req);
  hipEventDestroy(ctx->ev0);
  hipEventDestroy(ctx->ev1);
  hipStreamDestroy(ctx->stream);
  delete ctx;
  return ORH_OK;
}

const char* orh_last_error(const orh_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int orh_sync(orh_ctx* ctx) {
  if (!ctx) return ORH_E_INVALID;
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
  ORH_HIP(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
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
  hipStreamSynchronize(g->ctx->stream);
  free_graph_device(g);
  delete g;
  return ORH_OK;
}

int orh_graph_load(orh_graph* g, const orh_csr* c) {
  if (!g || !c) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  if (!c->row_ptr || (c->n_edges && (!c->col || !c->w_out || !c->w_in || !c->meta)) ||
      (c->n_nodes && !c->node_overloaded))
    return fail(ctx, ORH_E_INVALID, "orh_graph_load: null array");
  if (c->row_ptr[0] != 0 || c->row_ptr[c->n_nodes] != c->n_edges)
    return fail(ctx, ORH_E_INVALID, "orh_graph_load: row_ptr does not span n_edges");
  for (uint32_t v = 0; v < c->n_nodes; ++v)
    if (c->row_ptr[v] > c->row_ptr[v + 1])
      return fail(ctx, ORH_E_INVALID, "orh_graph_load: row_ptr not monotone");
  for (uint32_t e = 0; e < c->n_edges; ++e) {
    if (c->col[e] >= c->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_graph_load: col out of range");
    if (!(c->meta[e] & ORH_META_DOWN) && (c->w_out[e] == 0 || c->w_in[e] == 0))
      return fail(ctx, ORH_E_UNSUPPORTED,
                  "orh_graph_load: metric 0 on an up link (closed-form SPF needs metrics >= 1)");
  }
  hipSetDevice(ctx->device);
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  free_graph_device(g);
  g->n_nodes = c->n_nodes;
  g->n_edges = c->n_edges;
  g->n_links = c->n_links;
  g->row_ptr.assign(c->row_ptr, c->row_ptr + c->n_nodes + 1);
  g->col.assign(c->col, c->col + c->n_edges);
  g->w_out.assign(c->w_out, c->w_out + c->n_edges);
  g->w_in.assign(c->w_in, c->w_in + c->n_edges);
  g->meta.assign(c->meta, c->meta + c->n_edges);
  g->overloaded.assign(c->node_overloaded, c->node_overloaded + c->n_nodes);
  for (uint32_t e = 0; e < g->n_edges; ++e) {
    g->meta[e] = (g->meta[e] & ~ORH_META_COL_OVERLOADED) |
        (g->overloaded[g->col[e]] ? ORH_META_COL_OVERLOADED : 0u);
  }
  recompute_bounds(g);
  const auto rank = build_ranks(g, g->n_distinct);

  const size_t ne = std::max<uint32_t>(g->n_edges, 1), nn = std::max<uint32_t>(g->n_nodes, 1);
  if (hipMalloc(&g->d_row_ptr, (nn + 1) * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&g->d_edges, ne * sizeof(uint4)) != hipSuccess ||
      hipMalloc(&g->d_rank, ne * sizeof(uint16_t)) != hipSuccess ||
      hipMalloc(&g->d_overloaded, nn) != hipSuccess) {
    free_graph_device(g);
    return fail(ctx, ORH_E_NOMEM, "orh_graph_load: device allocation failed");
  }
  ORH_HIP(ctx, hipMemcpyAsync(g->d_row_ptr, g->row_ptr.data(), g->row_ptr.size() * 4,
                              hipMemcpyHostToDevice, ctx->stream));
  if (g->n_edges) {
    int rc = upload_edges(g, 0, g->n_edges);
    if (rc) return rc;
    ORH_HIP(ctx, hipMemcpyAsync(g->d_rank, rank.data(), rank.size() * 2, hipMemcpyHostToDevice,
                                ctx->stream));
  }
  if (g->n_nodes)
    ORH_HIP(ctx, hipMemcpyAsync(g->d_overloaded, g->overloaded.data(), g->n_nodes,
                                hipMemcpyHostToDevice, ctx->stream));
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_graph_patch_edges(orh_graph* g, uint32_t n, const uint32_t* idx, const uint32_t* w_out,
                          const uint32_t* w_in, const uint32_t* meta) {
  if (!g || (n && (!idx || !w_out || !w_in || !meta))) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  if (!g->d_edges && n) return fail(ctx, ORH_E_STATE, "orh_graph_patch_edges: no graph loaded");
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = idx[i];
    if (e >= g->n_edges) return fail(ctx, ORH_E_INVALID, "orh_graph_patch_edges: bad edge index");
    if ((meta[i] & ORH_META_LINK_MASK) != (g->meta[e] & ORH_META_LINK_MASK))
      return fail(ctx, ORH_E_INVALID, "orh_graph_patch_edges: link id changed (use load)");
    if (!(meta[i] & ORH_META_DOWN) && (w_out[i] == 0 || w_in[i] == 0))
      return fail(ctx, ORH_E_UNSUPPORTED, "orh_graph_patch_edges: metric 0 on an up link");
  }
  hipSetDevice(ctx->device);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = idx[i];
    g->w_out[e] = w_out[i];
    g->w_in[e] = w_in[i];
    g->meta[e] = (meta[i] & ~ORH_META_COL_OVERLOADED) | (g->meta[e] & ORH_META_COL_OVERLOADED);
    int rc = upload_edges(g, e, 1);
    if (rc) return rc;
  }
  recompute_bounds(g);
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ORH_OK;
}

int orh_graph_patch_nodes(orh_graph* g, uint32_t n, const uint32_t* idx, const uint8_t* ovl) {
  if (!g || (n && (!idx || !ovl))) return ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  hipSetDevice(ctx->device);
  for (uint32_t i = 0; i < n; ++i) {
    if (idx[i] >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_graph_patch_nodes: bad node");
    const uint32_t v = idx[i];
    g->overloaded[v] = ovl[i] ? 1 : 0;
    ORH_HIP(ctx, hipMemcpyAsync(g->d_overloaded + v, &g->overloaded[v], 1,
                                hipMemcpyHostToDevice, ctx->stream));
    // CSR entries that point at v carry v's overload bit
    for (uint32_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; ++e) {
      const uint32_t u = g->col[e];
      for (uint32_t e2 = g->row_ptr[u]; e2 < g->row_ptr[u + 1]; ++e2) {
        if (g->col[e2] != v) continue;
        const uint32_t m = (g->meta[e2] & ~ORH_META_COL_OVERLOADED) |
            (g->overloaded[v] ? ORH_META_COL_OVERLOADED : 0u);
        if (m != g->meta[e2]) {
          g->meta[e2] = m;
          int rc = upload_edges(g, e2, 1);
          if (rc) return rc;
        }
      }
    }
  }
  ORH_HIP(ctx, hipStreamSynchronize(ctx->stream));
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
  std::vector<uint32_t> l(g->col.begin() + g->row_ptr[src], g->col.begin() + g->row_ptr[src + 1]);
  std::sort(l.begin(), l.end());
  l.erase(std::unique(l.begin(), l.end()), l.end());
  *n_out = static_cast<uint32_t>(l.size());
  for (uint32_t i = 0; i < l.size() && i < cap; ++i) out[i] = l[i];
  return ORH_OK;
}

int orh_spf_words(const orh_graph* g, const uint32_t* srcs, uint32_t n, uint32_t* out) {
  if (!g || !out || (n && !srcs)) return ORH_E_INVALID;
  uint32_t mx = 1;
  for (uint32_t i = 0; i < n; ++i) {
    if (srcs[i] >= g->n_nodes) return ORH_E_INVALID;
    mx = std::max(mx, g->n_distinct[srcs[i]]);
  }
  *out = (mx + 31) / 32;
  return ORH_OK;
}

int orh_spf_run(orh_graph* g, const orh_spf_request* req, uint32_t words, uint32_t* d_dist,
                uint32_t* d_nh) {
  if (!g || !req || (req->n_src && (!req->h_srcs || !d_dist || !d_nh)))
    return g ? fail(g->ctx, ORH_E_INVALID, "orh_spf_run: null argument") : ORH_E_INVALID;
  orh_ctx* ctx = g->ctx;
  if (req->n_src == 0) return ORH_OK;
  if (!g->d_row_ptr || g->n_nodes == 0) return fail(ctx, ORH_E_STATE, "orh_spf_run: no graph loaded");
  uint32_t max_nbr = 1;
  for (uint32_t i = 0; i < req->n_src; ++i) {
    if (req->h_srcs[i] >= g->n_nodes) return fail(ctx, ORH_E_INVALID, "orh_spf_run: source out of range");
    max_nbr = std::max(max_nbr, g->n_distinct[req->h_srcs[i]]);
  }
  if (words < (max_nbr + 31) / 32) return fail(ctx, ORH_E_INVALID, "orh_spf_run: words too small");
  // any tentative value D + w is at most (sum of link metrics) + max metric
  const uint64_t bound = req->use_link_metric
      ? g->sum_max_metric / 2 + g->max_metric
      : static_cast<uint64_t>(g->n_links) + 1;
  const orh::SpfPlan plan = orh::plan_spf(g->n_nodes, words, max_nbr, bound, ctx->lds_limit);
  if (plan.variant == orh::SpfVariant::kUnsupported)
    return fail(ctx, ORH_E_UNSUPPORTED, "orh_spf_run: graph exceeds the LDS-resident kernels (N=" +
                                            std::to_string(g->n_nodes) + ")");

  // stage sources and ignore sets in one device buffer
  const bool has_ign = req->h_ignore_ptr != nullptr;
  const uint32_t n_ign = has_ign ? req->h_ignore_ptr[req->n_src] : 0u;
  const size_t total = req->n_src + (has_ign ? (req->n_src + 1 + n_ign) : 0);
  hipSetDevice(ctx->device);
  int rc = ensure_req(ctx, total);
  if (rc) return rc;
  std::vector<uint32_t> staging;
  staging.reserve(total);
  staging.insert(staging.end(), req->h_srcs, req->h_srcs + req->n_src);
  if (has_ign) {
    staging.insert(staging.end(), req->h_ignore_ptr, req->h_ignore_ptr + req->n_src + 1);
    for (uint32_t i = 0; i < req->n_src; ++i) {  // each source's set sorted for bsearch
      std::vector<uint32_t> s(req->h_ignore_links + req->h_ignore_ptr[i],
                              req->h_ignore_links + req->h_ignore_ptr[i + 1]);
      std::sort(s.begin(), s.end());
      staging.insert(staging.end(), s.begin(), s.end());
    }
  }
  ORH_HIP(ctx, hipMemcpyAsync(ctx->d_req, staging.data(), staging.size() * 4,
                              hipMemcpyHostToDevice, ctx->stream));

  orh::SpfArgs a{};
  a.n_nodes = g->n_nodes;
  a.words = words;
  a.row_ptr = g->d_row_ptr;
  a.edges = g->d_edges;
  a.rank_in_col = g->d_rank;
  a.node_overloaded = g->d_overloaded;
  a.srcs = ctx->d_req;
  a.ignore_ptr = has_ign ? ctx->d_req + req->n_src : nullptr;
  a.ignore_links = has_ign ? ctx->d_req + 2 * req->n_src + 1 : nullptr;
  a.use_link_metric = req->use_link_metric;
  a.out_dist = d_dist;
  a.out_nh = d_nh;
  ORH_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  hipError_t e = orh::launch_spf(plan, a, req->n_src, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "spf kernel launch");
  ORH_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  ctx->counters.spf_runs += req->n_src;
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
  uint32_t *d_dist = nullptr, *d_nh = nullptr;
  if (hipMalloc(&d_dist, nd * 4) != hipSuccess || hipMalloc(&d_nh, nd * words * 4) != hipSuccess) {
    hipFree(d_dist);
    return fail(ctx, ORH_E_NOMEM, "orh_spf_batch: device allocation failed");
  }
  int rc = orh_spf_run(g, req, words, d_dist, d_nh);
  if (rc == ORH_OK) {
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
  hipFree(d_dist);
  hipFree(d_nh);
  return rc;
}

int orh_route_select(orh_ctx* ctx, uint32_t n_prefix, const uint32_t* d_adv_ptr,
                     const uint32_t* d_adv, const uint32_t* d_dist, const uint32_t* d_nh,
                     uint32_t words, uint32_t* d_min, uint32_t* d_nh_out) {
  if (!ctx) return ORH_E_INVALID;
  if (n_prefix == 0) return ORH_OK;
  if (!d_adv_ptr || !d_adv || !d_dist || !d_nh || !d_min || !d_nh_out || words == 0)
    return fail(ctx, ORH_E_INVALID, "orh_route_select: null argument");
  hipSetDevice(ctx->device);
  orh::RouteSelectArgs a{n_prefix, words, d_adv_ptr, d_adv, d_dist, d_nh, d_min, d_nh_out};
  hipError_t e = orh::launch_route_select(a, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "route_select launch");
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
