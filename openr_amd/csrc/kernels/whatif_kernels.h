// Internal interface of the what-if repair kernels (whatif_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace orh {

// ---- what-if repair (whatif_kernels.hip) ----------------------------------
// runSpf(src, useLinkMetric, ignore) for many (src, ignore set) requests from
// the plain SPF rows of their sources: a request's row is the base row except
// on the nodes downstream of a tight ignored link, which are re-derived.
struct RepairArgs {
  uint32_t n_nodes;
  uint32_t n_req;
  int32_t use_link_metric;
  uint32_t cap_a;  // affected nodes a workgroup repairs in LDS
  uint32_t cap_e;  // predecessor edges among them
  const uint2* recs;
  const uint32_t* link;
  const uint16_t* rank_out;
  const uint32_t* rev;  // per record: the record of the same link from the other end
  const uint8_t* ovl;   // [N] node overloaded
  const uint32_t* base_dist;  // [m][N]
  const uint32_t* base_nh;    // [m][N], one mask word
  const uint32_t* base_row;   // [n_req] base row of the request's source
  const uint32_t* srcs;       // [n_req]
  const uint32_t* ign_ptr;    // [n_req + 1]
  const uint32_t* ign;        // sorted per request
  const uint32_t* cut_ptr;    // [n_req + 1]
  const uint4* cuts;          // (tail, head, record tail -> head, 0) per ignored link end
  uint32_t* out_dist;         // [n_req][N]
  uint32_t* out_nh;           // [n_req][N], one mask word
  uint32_t* fallback;         // [n_req] set when a request needs the full search
  // second pass for the requests that outgrew LDS: n_slots global slots of
  // slot_bytes each, claimed through *slot_next (zeroed beforehand)
  uint8_t* slot_mem;
  size_t slot_bytes;
  uint32_t n_slots;
  uint32_t* slot_next;
  uint32_t n_recs;  // device records (slot edge capacity)
};
// LDS bytes of the repair kernel for the given caps
size_t repair_lds_bytes(uint32_t n_nodes, uint32_t cap_a, uint32_t cap_e);
// bytes of one global repair slot (whole-graph caps)
size_t repair_slot_bytes(uint32_t n_nodes, uint32_t n_recs);
// copy each request's base rows, then repair; rows the repair cannot hold
// get fallback[r] = 1 (fallback must be zeroed beforehand)
hipError_t launch_repair(const RepairArgs& a, uint32_t ell_k, hipStream_t s);

}  // namespace orh
