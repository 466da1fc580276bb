// Internal interface of the KSP2 trace kernel (ksp_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace orh {

// LinkState::getKthPaths k = 1 / k = 2 traces (traceOnePath,
// LinkState.cpp:398-419, :762-791) over device-resident SPF rows, one thread
// per (src, dst) pair. A pair's output block (out_cap words):
//   [0] status (0 ok, else kKspOverflow: the host traces the pair)
//   [1] end of the k = 1 section
//   k = 1 section: n_paths, then per path its length and link ids (src -> dst)
//   k = 2 section: the same
constexpr uint32_t kKspOverflow = 1;

struct KspFrame {
  uint32_t v;     // node of this frame
  uint32_t has;   // a candidate of v was tried (dp, rank, q2 below)
  uint32_t dp, rank, q2;  // key of the last candidate tried: (dist, name rank, record)
  uint32_t link;  // link taken to the next frame
};

struct KspArgs {
  uint32_t n_nodes;
  uint32_t n_pairs;
  uint32_t k;  // 1 or 2
  const uint2* recs;
  const uint32_t* link;
  const uint32_t* rev;        // per record: the record of the same link from the other end
  const uint32_t* name_rank;  // [N] (metric, name) tie order of the extraction
  const uint32_t* src;        // [n_pairs]
  const uint32_t* dst;        // [n_pairs]
  const uint32_t* row;        // [n_pairs] row of the pair in dist
  const uint32_t* dist;       // [rows][N] (k = 1: the sources' rows, k = 2: one per pair)
  // k = 2: the pair's k = 1 links, sorted, padded with ~0u to ign_cap (and
  // written by the k = 1 pass); need2[i] = 1 when they exist
  uint32_t* ign;
  uint32_t ign_cap;
  uint32_t* need2;
  uint32_t* out;
  uint32_t out_cap;
  uint32_t* visited;  // [n_pairs][hash_cap] open-addressing set of link id + 1 (zeroed)
  uint32_t hash_cap;  // power of two
  KspFrame* stack;    // [n_pairs][stack_cap]
  uint32_t stack_cap;
};

hipError_t launch_ksp_trace(const KspArgs& a, uint32_t ell_k, hipStream_t s);

// order[0 .. P) = the pairs by descending k = 1 distance of their destination
// (dist1[row1[i] * N + dst[i]]; pairs with need2[i] == 0 last): the k = 2
// searches that reach farthest start first, so the batch's last wave of
// searches is its shortest (P <= 4096, one workgroup)
hipError_t launch_ksp_order(const uint32_t* dist1, const uint32_t* row1, const uint32_t* dst,
                            const uint32_t* need2, uint32_t n_nodes, uint32_t n_pairs, uint32_t* order,
                            hipStream_t s);

}  // namespace orh
