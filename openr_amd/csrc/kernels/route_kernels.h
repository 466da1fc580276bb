// Internal interface of the route-selection kernels (route_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/openr_hip.h"

namespace orh {

constexpr uint32_t kMaxSelectAreas = 32;

// one area of a route-selection launch (device pointers; see orh_select_area)
struct SelArea {
  uint32_t present;
  const uint32_t* dist;
  const uint32_t* nh;
  const uint8_t* ovl;
  const uint32_t* name_node;
  uint32_t words;
  uint32_t word_off;
};

struct RouteSelectArgs {
  uint32_t pid_lo;    // prefixes [pid_lo, n_prefix)
  uint32_t n_prefix;
  const uint2* hdr;  // per prefix {pool offset, count | prefix flags << 16}
  const orh_adv* adv;
  const uint32_t* name_rank;
  const uint32_t* area_rank;
  uint32_t n_names;
  uint32_t me_name;
  uint32_t flags;  // ORH_SELECT_*
  uint32_t n_areas;
  const SelArea* areas;  // [n_areas], device
  uint8_t* status;
  uint32_t* metric;
  uint32_t* best;
  uint32_t* mask;
  uint32_t total_words;
};

hipError_t launch_route_select(const RouteSelectArgs& a, hipStream_t s);

// keyed compare of two selection outputs (route_diff_kernel)
struct RouteDiffArgs {
  uint32_t n_prefix, prev_n, words;
  const uint8_t* status;
  const uint32_t* metric;
  const uint32_t* best;
  const uint32_t* mask;
  const uint8_t* p_status;
  const uint32_t* p_metric;
  const uint32_t* p_best;
  const uint32_t* p_mask;
  uint32_t* out;    // packed records {p, status, metric, best, mask[words]}
  uint32_t* count;  // zeroed before the launch
};
hipError_t launch_route_diff(const RouteDiffArgs& a, hipStream_t s);

// RibPolicy over a selection (route_policy_kernel; see orh_route_policy)
struct RoutePolicyArgs {
  uint32_t pid_lo;  // prefixes [pid_lo, n_prefix)
  uint32_t n_prefix, words;
  const uint2* hdr;
  const orh_adv* adv;
  const uint8_t* status;
  const uint32_t* best;
  const uint32_t* mask;
  uint32_t n_stmts, stmt_tags, stmt_pfx;
  uint32_t n_tagsets;
  const uint32_t* tagset_stmts;
  uint32_t n_pfx;
  const uint32_t* pfx_id;
  const uint32_t* pfx_stmts;
  const uint32_t* keep;  // [n_stmts][words]
  uint8_t* out;
  uint32_t* invalidated;  // zeroed before the launch
};
hipError_t launch_route_policy(const RoutePolicyArgs& a, hipStream_t s);

// hdr[ids[i]] = vals[i]
hipError_t launch_scatter_hdr(uint2* hdr, const uint32_t* ids, const uint2* vals, uint32_t n,
                              hipStream_t s);

}  // namespace orh
