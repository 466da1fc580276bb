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
//
// Requests move through tiers; each tier is a work queue drained by a fixed
// grid of workgroups (every workgroup exits once the queue is empty):
//   seed   one thread per request: no tight ignored link -> the base row
//          stands (tier 0); else the request joins queue 1
//   tier 1 small LDS state (kSmallA nodes / kSmallE edges): most repairs
//   tier 2 large LDS state (cap_a / cap_e)
//   tier 3 global slots sized for the whole graph (cannot overflow)
//   tier 4 only without slots: the full HBM search (fallback flags)
constexpr uint32_t kWhatifTierBase = 0, kWhatifTierSmall = 1, kWhatifTierLarge = 2, kWhatifTierSlot = 3,
                   kWhatifTierSearch = 4;
constexpr uint32_t kSmallA = 256, kSmallE = 1024;
// counters (u32, zeroed before a run): per queue q = 0..2 its length and the
// next index to claim
constexpr uint32_t kWhatifCounters = 8;

struct RepairArgs {
  uint32_t n_nodes;
  uint32_t n_req;
  int32_t use_link_metric;
  uint32_t cap_a;  // tier 2: affected nodes a workgroup repairs in LDS
  uint32_t cap_e;  // tier 2: predecessor edges among them
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
  uint32_t* fallback;         // [n_req] set when a request needs the full search (no slots)
  uint32_t* info;             // [n_req] tier | affected nodes << 3 (nullable)
  uint32_t* queues;           // [3][n_req] request ids of queues 0..2 (tiers 1..3)
  uint32_t* counters;         // [kWhatifCounters]
  // tier 3: n_slots global slots of slot_bytes each, one per workgroup
  uint8_t* slot_mem;
  size_t slot_bytes;
  uint32_t n_slots;
  uint32_t n_recs;  // device records (slot edge capacity)
  uint32_t n_cu;    // grid sizing of the queue-draining tiers
  // the first full_cap entries of the slot tier's queue are searched in full
  // instead (a separate launch over that list, repair_slot_queue): a large
  // subtree repairs slower in a slot than the whole search runs; the slot
  // tier takes the rest and marks those requests kWhatifTierSearch
  uint32_t full_cap;
  // copy only the requests the seed queued for repair (queue 0): the others'
  // rows are their sources' base rows, which the caller reads from the job
  uint32_t share_base;
  // no tier 2 (host-side launch plan only): the requests that outgrow tier 1
  // go straight to the full searches / slot tier, which then start as soon
  // as tier 1 ends (a short job's largest repairs are its critical path)
  uint32_t skip_large;
};
// queue index the slot tier drains (the full search's list)
uint32_t repair_slot_queue(const RepairArgs& a);
// LDS bytes of the repair kernel for the given caps
size_t repair_lds_bytes(uint32_t n_nodes, uint32_t cap_a, uint32_t cap_e);
// bytes of one global repair slot (whole-graph caps)
size_t repair_slot_bytes(uint32_t n_nodes, uint32_t n_recs);
// seed, copy each request's base rows, then the repair tiers; with no slots
// the requests that outgrow tier 2 get fallback[r] = 1 (zeroed beforehand)
hipError_t launch_repair(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s);
// the same in two parts: seed and copy (HBM-bound, the whole GPU), then the
// repair tiers (latency-bound, a few thousand workgroups), which may run on a
// second stream, overlapping the next batch's copy
hipError_t launch_repair_front(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s);
hipError_t launch_repair_back(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s);
// the same with the slot tier on its own stream s3, after event `mid`
// (recorded on s behind tiers 1 and 2): the next run's small tiers on s do
// not wait for this run's largest repairs
hipError_t launch_repair_back_split(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s,
                                    hipStream_t s3, hipEvent_t mid);

// per row r < rows: the digest of (dist[r][v], nh[r][v][0..words)) over v < n
// (row_digest_kernel), into out[r]
hipError_t launch_row_digest(const uint32_t* dist, const uint32_t* nh, uint32_t words, uint32_t n,
                             uint32_t rows, uint64_t* out, hipStream_t s);

}  // namespace orh
