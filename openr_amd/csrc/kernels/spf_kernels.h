// Internal interface between the C ABI (orh_api.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// mirrors of the ORH_META_* bits in include/openr_hip.h
#define ORH_META_LINK_MASK_ 0x3FFFFFFFu
#define ORH_META_COL_OVERLOADED_ 0x40000000u
#define ORH_META_DOWN_ 0x80000000u

namespace orh {

struct SpfArgs {
  uint32_t n_nodes;
  uint32_t words;  // nh words per node in the output
  const uint32_t* row_ptr;
  const uint4* edges;  // {col, w_out, w_in, meta}
  const uint16_t* rank_in_col;  // rank of the row node among col's distinct neighbours
  const uint8_t* node_overloaded;
  const uint32_t* srcs;
  const uint32_t* ignore_ptr;  // nullable
  const uint32_t* ignore_links;
  int32_t use_link_metric;
  uint32_t lds_list_off;
  uint32_t lds_mask_off;
  uint32_t* out_dist;
  uint32_t* out_nh;
};

enum class SpfVariant { kUnsupported = 0, kK16, kK32, kWide };

struct SpfPlan {
  SpfVariant variant;
  bool id16;
  size_t list_off;
  size_t mask_off;
  size_t lds_bytes;
};

// max_nbr: largest distinct-neighbour count over the batch's sources;
// path_bound: upper bound on any D + w computed by the kernel
SpfPlan plan_spf(uint32_t n_nodes, uint32_t words, uint32_t max_nbr, uint64_t path_bound,
                 size_t lds_limit);
hipError_t launch_spf(const SpfPlan& plan, SpfArgs a, uint32_t n_src, hipStream_t s);

struct RouteSelectArgs {
  uint32_t n_prefix;
  uint32_t words;
  const uint32_t* adv_ptr;
  const uint32_t* adv;
  const uint32_t* dist;
  const uint32_t* nh;
  uint32_t* min_out;
  uint32_t* nh_out;
};
hipError_t launch_route_select(const RouteSelectArgs& a, hipStream_t s);

}  // namespace orh
