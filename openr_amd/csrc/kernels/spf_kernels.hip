// Batched SPF and route-selection kernels for gfx950 (MI355X).
//
// Semantics: LinkState::runSpf (openr/decision/LinkState.cpp:808-882) in its
// closed form, valid for link metrics >= 1:
//   d(u)   shortest metric over up, non-ignored links, no transit through an
//          overloaded node other than the source (:831-838)
//   NH(u)  = OR over predecessors (l, v) with d(v) + w_v(l) == d(u) and v a
//          transit node of   (v == src ? {u} : NH(v))          (:857-873)
//
// Two phases, both batched over many sources:
//
// 1. Distance rows (one workgroup per source row). The first-hop masks are
//    NOT carried through the search, so the per-source LDS state is only what
//    the distances need:
//      BFS    (every live link has the same metric w0): a u8/u16/u32 level
//             per node plus two frontier bitmaps; the row (level * w0) is
//             written to HBM once, coalesced, when the search ends. No
//             atomics return, no min-reduction: the next level is the next
//             frontier.
//      Dist16 / Dist32 (general metrics): a u16 or u32 distance per node plus
//             a pending-set bitmap; level-synchronous Dijkstra that expands
//             every node at the minimum pending distance D at once (exact for
//             positive integer metrics), the next D from a DPP wave minimum.
//    Small state buys occupancy: BFS on N = 10,000 needs 22.5 KB, so seven
//    sources are resident per CU.
// 2. First hops (one workgroup per (source, 1024-node tile)). With metrics
//    >= 1 the closed form unrolls to: bit i (the source's i-th distinct
//    neighbour n_i) is in NH(v) iff some up link s->n_i is tight
//    (w == d_s(n_i)) and either v == n_i, or n_i is not overloaded and
//    d_s(n_i) + d_{n_i}(v) == d_s(v), where d_{n_i} is n_i's own SPF with the
//    same ignore set (a tight path leaves s through n_i and continues along
//    a shortest path of n_i whose intermediates are transit nodes; paths of
//    n_i back through s are never tight). Phase 1 therefore also computes
//    the rows of the sources' neighbours (free for an all-sources sweep: they
//    are sources themselves), and phase 2 is a streaming, coalesced pass over
//    1 + deg(s) distance rows per source.
//
// Graph records are 8 bytes (col|flags, w_out), ELL-style K per node with a
// continuation into an overflow area, so expanding a node is ONE dependent
// global round trip (K records issued together, served from L2 where the
// graph stays resident for every workgroup on the XCD).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "spf_kernels.h"

namespace orh {

constexpr int kBlock = 256;     // route selection, first hops
constexpr int kMaxBlock = 1024;  // SPF
constexpr int kOvfBatch = 8;     // overflow records in flight per expanded node
constexpr int kHopPer = 4;       // nodes per thread in the first-hop kernel
constexpr uint32_t kInf = 0xFFFFFFFFu;

__device__ inline bool ignored(const uint32_t* ign, uint32_t n, uint32_t link) {
  uint32_t lo = 0, hi = n;  // sorted ascending; tiny (KSP2 / what-if sets)
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t x = ign[mid];
    if (x == link) return true;
    if (x < link) lo = mid + 1; else hi = mid;
  }
  return false;
}

__device__ inline uint32_t* dist_row(uint32_t* out, uint32_t* scratch, uint32_t n_out, uint32_t N,
                                     uint32_t row) {
  return row < n_out ? out + static_cast<size_t>(row) * N
                     : scratch + static_cast<size_t>(row - n_out) * N;
}

// wave-wide minimum through DPP row shifts and row broadcasts (no LDS)
__device__ inline uint32_t wave_min(uint32_t v) {
#define ORH_DPP_MIN(ctrl, rmask)                                                         \
  v = min(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(                           \
                 static_cast<int>(kInf), static_cast<int>(v), ctrl, rmask, 0xF, false)))
  ORH_DPP_MIN(0x111, 0xF);  // row_shr:1
  ORH_DPP_MIN(0x112, 0xF);  // row_shr:2
  ORH_DPP_MIN(0x114, 0xF);  // row_shr:4
  ORH_DPP_MIN(0x118, 0xF);  // row_shr:8  -> lane 15 of each row holds the row minimum
  ORH_DPP_MIN(0x142, 0xA);  // row_bcast:15 into rows 1, 3
  ORH_DPP_MIN(0x143, 0xC);  // row_bcast:31 into rows 2, 3 -> lane 63 holds the minimum
#undef ORH_DPP_MIN
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// wave-wide sum (every lane active), the DPP pattern of wave_min
__device__ inline uint32_t wave_sum(uint32_t v) {
#define ORH_DPP_ADD(ctrl, rmask) \
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), ctrl, rmask, 0xF, false))
  ORH_DPP_ADD(0x111, 0xF);  // row_shr:1
  ORH_DPP_ADD(0x112, 0xF);  // row_shr:2
  ORH_DPP_ADD(0x114, 0xF);  // row_shr:4
  ORH_DPP_ADD(0x118, 0xF);  // row_shr:8  -> lane 15 of each row holds the row sum
  ORH_DPP_ADD(0x142, 0xA);  // row_bcast:15 into rows 1, 3
  ORH_DPP_ADD(0x143, 0xC);  // row_bcast:31 into rows 2, 3 -> lane 63 holds the sum
#undef ORH_DPP_ADD
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

struct Src {
  uint32_t node;
  const uint32_t* ign;
  uint32_t n_ign;
  // optional LDS filter of the ignore set (a bit per hashed link id, no
  // false negatives): a clear bit skips the binary search in global memory
  const uint32_t* filt;
  uint32_t fshift;
  __device__ Src(const SpfArgs& a, uint32_t row)
      : node(a.srcs[row]), ign(nullptr), n_ign(0), filt(nullptr), fshift(0) {
    if (a.ignore_ptr) {
      const uint32_t b = a.ignore_ptr[row];
      ign = a.ignore_links + b;
      n_ign = a.ignore_ptr[row + 1] - b;
    }
  }
};

__device__ inline uint32_t ign_hash(uint32_t link, uint32_t shift) { return (link * 0x9E3779B1u) >> shift; }

// a record the search may relax: up, not a continuation, not ignored
__device__ inline bool live(const SpfArgs& a, const Src& s, const uint2& r, uint32_t q) {
  if (r.x & (ORH_REC_SKIP | ORH_REC_CONT)) return false;
  if (!s.n_ign) return true;
  const uint32_t l = a.link[q];
  if (s.filt) {
    const uint32_t h = ign_hash(l, s.fshift);
    if (!((s.filt[h >> 5] >> (h & 31u)) & 1u)) return true;
  }
  return !ignored(s.ign, s.n_ign, l);
}

// live() with the record's link id already loaded (searches with ignore sets
// fetch the ids together with the records: one round trip, not two)
__device__ inline bool live_link(const Src& s, const uint2& r, uint32_t l) {
  if (r.x & (ORH_REC_SKIP | ORH_REC_CONT)) return false;
  if (!s.n_ign) return true;
  if (s.filt) {
    const uint32_t h = ign_hash(l, s.fshift);
    if (!((s.filt[h >> 5] >> (h & 31u)) & 1u)) return true;
  }
  return !ignored(s.ign, s.n_ign, l);
}

template <int K>
__device__ inline void load_recs(const SpfArgs& a, uint32_t v, uint2 (&rec)[K]) {
  const uint2* slots = a.recs + static_cast<size_t>(v) * K;
#pragma unroll
  for (int j = 0; j < K; ++j) rec[j] = slots[j];
}

// ---------------------------------------------------------------------------
// phase 1a: BFS levels (uniform metric)
// ---------------------------------------------------------------------------
// Per-source LDS state: the BFS level of every node (L = u8 / u16 / u32, all
// ones = unvisited) plus two frontier bitmaps. Levels stay in LDS until the
// search ends and the row is written to HBM once, coalesced (writing each
// node's distance when it is reached scatters 4-byte stores over the row and
// costs ~7x the row's bytes in partial-line writes).
template <class L>
struct Level {
  static constexpr uint32_t kInfL = static_cast<L>(~static_cast<L>(0));
};

template <int K, class L>
struct Bfs {
  const SpfArgs& a;
  const Src& s;
  L* lvl;
  uint32_t* nxt;
  L next_level;

  __device__ bool edge(const uint2& r, uint32_t lu) const {
    if (lu != Level<L>::kInfL) return false;
    const uint32_t u = r.x & ORH_REC_COL_MASK;
    lvl[u] = next_level;  // racing writers store the same value
    atomicOr(&nxt[u >> 5], 1u << (u & 31u));
    return true;
  }

  // expand v (its K records in rec): mark unvisited neighbours for the next level
  __device__ bool expand(uint32_t v, const uint2 (&rec)[K]) const {
    if (v != s.node && (rec[0].x & ORH_REC_ROW_OVL)) return false;  // no transit
    bool pushed = false;
    uint32_t lu[K];
    bool lv[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      lv[j] = live(a, s, rec[j], v * K + j);
      lu[j] = lv[j] ? static_cast<uint32_t>(lvl[rec[j].x & ORH_REC_COL_MASK]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (lv[j]) pushed |= edge(rec[j], lu[j]);
    const uint2 last = rec[K - 1];
    if (last.x & ORH_REC_CONT) {
      const uint32_t start = last.x & ORH_REC_COL_MASK;
      for (uint32_t base = 0; base < last.y; base += kOvfBatch) {
        const uint32_t cnt = min(last.y - base, static_cast<uint32_t>(kOvfBatch));
        uint2 ov[kOvfBatch];
#pragma unroll
        for (int j = 0; j < kOvfBatch; ++j)
          if (j < static_cast<int>(cnt)) ov[j] = a.recs[start + base + j];
        uint32_t ol_[kOvfBatch];
        bool ol[kOvfBatch];
#pragma unroll
        for (int j = 0; j < kOvfBatch; ++j) {
          ol[j] = j < static_cast<int>(cnt) && live(a, s, ov[j], start + base + j);
          ol_[j] = ol[j] ? static_cast<uint32_t>(lvl[ov[j].x & ORH_REC_COL_MASK]) : 0u;
        }
#pragma unroll
        for (int j = 0; j < kOvfBatch; ++j)
          if (ol[j]) pushed |= edge(ov[j], ol_[j]);
      }
    }
    return pushed;
  }
};

template <int K, class L>
__global__ __launch_bounds__(kMaxBlock) void spf_bfs_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_any[3];
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x, row = blockIdx.x;
  L* lvl = reinterpret_cast<L*>(lds);
  uint32_t* f0 = lds + a.lds_pend_off / 4;
  uint32_t* f1 = f0 + NB;
  const Src s(a, row);

  const uint32_t lwords = a.lds_pend_off / 4;
  for (uint32_t i = tid; i < lwords; i += nthr) lds[i] = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < 2 * NB; i += nthr) f0[i] = 0u;
  if (tid < 3) s_any[tid] = 0u;
  __syncthreads();
  if (tid == 0) {
    lvl[s.node] = 0;
    f0[s.node >> 5] = 1u << (s.node & 31u);
  }
  __syncthreads();

  constexpr int kBatch = 16 / K;  // nodes whose records are in flight together
  for (uint32_t level = 0;; ++level) {
    const uint32_t par = level & 1u;
    uint32_t* cur = par ? f1 : f0;
    const Bfs<K, L> b{a, s, lvl, par ? f0 : f1, static_cast<L>(level + 1)};
    bool pushed = false;
    // a thread owns frontier words w and w + nthr: their nodes' records go
    // out in one batch
    for (uint32_t w = tid; w < NB; w += 2 * nthr) {
      const uint32_t w2 = w + nthr;
      const uint32_t t0 = cur[w];
      const uint32_t t1 = w2 < NB ? cur[w2] : 0u;
      if (t0) cur[w] = 0u;  // becomes the level-after-next frontier
      if (t1) cur[w2] = 0u;
      uint64_t todo = t0 | (static_cast<uint64_t>(t1) << 32);
      while (todo) {
        uint32_t vs[kBatch];
        uint2 r[kBatch][K];
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < kBatch; ++i) {
          if (todo) {
            const uint32_t bit = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            vs[i] = bit < 32 ? w * 32 + bit : w2 * 32 + (bit - 32);
            load_recs<K>(a, vs[i], r[i]);
            cnt = i + 1;
          }
        }
#pragma unroll
        for (int i = 0; i < kBatch; ++i)
          if (i < cnt) pushed |= b.expand(vs[i], r[i]);
      }
    }
    // exit flags rotate over three slots: level L writes and reads slot L%3
    // around its barrier; the reset of slot (L+2)%3 = (L-1)%3 happens after
    // barrier L, when every wave has read that slot (right after barrier
    // L-1), and before barrier L+1, which every writer of level L+2 passes
    const uint32_t slot = level % 3u;
    if (pushed) s_any[slot] = 1u;
    __syncthreads();
    // every level expands >= 1 node and levels stay below the type's
    // all-ones (the planner picks L with N - 1 < kInfL), so the loop ends
    // and every wave reaches the exit
    if (!s_any[slot] || level >= N) break;
    if (tid == 0) s_any[(level + 2u) % 3u] = 0u;
  }
  uint32_t* out = dist_row(a.out_dist, a.scratch, a.n_out, N, row);
  const uint32_t w0 = a.w0;
  for (uint32_t i = tid; i < N; i += nthr) {
    const uint32_t l = lvl[i];
    __builtin_nontemporal_store(l == Level<L>::kInfL ? kInf : l * w0, &out[i]);
  }
}

// ---------------------------------------------------------------------------
// phase 1a': bit-parallel multi-source BFS (uniform metric, no ignore sets)
// ---------------------------------------------------------------------------
// One workgroup runs S = 32 (u32 masks) or 16 (u16) source rows at once, one
// bit per source (multi-source BFS, Then et al., VLDB 2015), as a pull over
// the nodes:
//   nx(v) = (OR over live records v -> u of F(u)) & ~visited(v)
// Thread t owns the Cuthill-McKee nodes t, t + B, ..., t + (J-1)B and keeps
// their ELL columns (packed 16-bit; a dead or down slot points at an
// always-zero LDS entry) and their visited masks in registers, so LDS holds
// only the two frontier arrays (this level's and the next): 8 bytes per node
// at S = 32, two workgroups per CU at N = 10,000. Groups of owned nodes whose
// masks are full on every lane are skipped (a full node's stale frontier
// entry only repeats bits every neighbour already holds). A node's bits
// reach its neighbours only if it is a transit node (not overloaded; a
// source always transits its own bit at level 0).
//
// Levels leave the CU as they are found, as bytes in a node-major scratch
// lvl[(batch * N + v) * S + b] (one S-byte block per node, written only by
// the node's owner thread, so a store instruction's 64 lanes land in one
// 2 KB span), and ms_finalize_kernel turns the scratch into host-order u32
// rows with coalesced stores. (Measured alternatives: a row-major scratch
// written per source bit issues ~5x more store instructions on the grid, where
// a node's bits arrive a few at a time but different lanes get different bits;
// dword stores for whole nibbles cost more than the stores they save.) Levels
// >= 254 are written to the output row directly (marker 254), so any depth is
// exact; 255 = unreached.
//
// Interval skip (kSkip): nodes are numbered in Cuthill-McKee order, so every
// live record v -> u has |u - v| <= bw (the layout's bandwidth). If the nodes
// that gained a bit at level L-1 span the ids [lo, hi], only nodes in
// [lo - bw, hi + bw] can gain one at level L; a 64-node slice (one wave's
// nodes of one j) outside it is skipped without reading its neighbours'
// frontier entries. The interval is two LDS words per level (wave min / max
// reductions); the per-slice test is scalar, so the variant costs no VGPRs
// beyond the two running bounds (a slice-bitmap form of the same skip needed
// 117 VGPRs, one workgroup per CU, and ran 1.4x slower). A skipped node keeps
// a stale f_nxt entry from two levels back: its bits reached every neighbour
// by the previous level, so it only repeats visited bits (see below).
//
// The search is latency-bound, not LDS-bound: on the 10k grid one workgroup
// takes ~0.7 ms whether 32 or 313 of them run (two fit per CU), ~165 levels
// of ~9k cycles, of which ~25 % are the level-byte stores and ~23 % the
// barrier. A top-down form (a node reads only its own word, new frontier
// nodes OR their bits into their neighbours' words with ds_or) issues ~4x
// fewer LDS operations and measured slower: 0.79 vs 0.74 ms (grid), 0.21 vs
// 0.18 ms (C3 Clos).
constexpr uint32_t kLvlDirect = 254u, kLvlNone = 255u;

template <class M>
struct MsMask;
// V: the register type of a node's visited / new bits
template <>
struct MsMask<uint64_t> {
  static constexpr uint32_t kS = 64;
  typedef uint64_t V;
  __device__ static uint32_t ctz(uint64_t x) { return static_cast<uint32_t>(__builtin_ctzll(x)); }
};
template <>
struct MsMask<uint32_t> {
  static constexpr uint32_t kS = 32;
  typedef uint32_t V;
  __device__ static uint32_t ctz(uint32_t x) { return static_cast<uint32_t>(__builtin_ctz(x)); }
};
template <>
struct MsMask<uint16_t> {
  static constexpr uint32_t kS = 16;
  typedef uint32_t V;
  __device__ static uint32_t ctz(uint32_t x) { return static_cast<uint32_t>(__builtin_ctz(x)); }
};

__device__ inline uint32_t ms_col(const uint2& r, uint32_t zero) {
  return (r.x & (ORH_REC_SKIP | ORH_REC_CONT)) ? zero : (r.x & ORH_REC_COL_MASK);
}

// workgroup barrier that orders LDS only (s_waitcnt lgkmcnt(0) + s_barrier);
// the "memory" clobber keeps the compiler from moving LDS accesses across it
__device__ inline void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// wave-wide OR (same DPP pattern as wave_min)
__device__ inline uint32_t wave_or(uint32_t v) {
#define ORH_DPP_OR(ctrl, rmask)                                                     \
  v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), ctrl, rmask, 0xF, false))
  ORH_DPP_OR(0x111, 0xF);
  ORH_DPP_OR(0x112, 0xF);
  ORH_DPP_OR(0x114, 0xF);
  ORH_DPP_OR(0x118, 0xF);
  ORH_DPP_OR(0x142, 0xA);
  ORH_DPP_OR(0x143, 0xC);
#undef ORH_DPP_OR
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

template <int K, class M, int J, bool kSkip>
__global__ __launch_bounds__(1024) void spf_msbfs_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr uint32_t kS = MsMask<M>::kS;
  typedef typename MsMask<M>::V V;
  constexpr int KH = (K + 1) / 2;
  const uint32_t N = a.n_nodes;
  const uint32_t NZ = a.ms_zero;  // index of the always-zero frontier entry
  const uint32_t tid = threadIdx.x, B = blockDim.x;
  const uint32_t b0 = blockIdx.x * a.ms_width;  // a batch: ms_width <= kS sources
  const uint32_t S = min(a.ms_width, a.n_rows - b0);
  const V full = S >= 8 * sizeof(V) ? ~V(0) : (V(1) << S) - V(1);
  __shared__ uint32_t s_prog[3];
  __shared__ uint32_t s_lo[3], s_hin[3];  // per level: min / ~max id with a new frontier bit
  M* f_cur = reinterpret_cast<M*>(lds);
  M* f_nxt = f_cur + a.ms_pitch;
  // the ELL columns hold byte offsets into a frontier array (16 bits each:
  // the planner keeps pitch * sizeof(M) <= 64 KiB), so a gather address is
  // one add of the array's offset that also picks the half-word (3 VALU ->
  // 1 per gather, ~3 % of the step: profiles/r05/l_msbfs_offsets_ab.txt); u64
  // masks (opt-in) store dword offsets, doubled at the read
  constexpr uint32_t kE = sizeof(M);
  constexpr uint32_t kC = kE <= 4 ? kE : 4;  // bytes per stored column unit
  const char* const lbase = reinterpret_cast<const char*>(lds);
  uint32_t cur_off = 0u, nxt_off = a.ms_pitch * kE;  // f_cur / f_nxt in bytes
  uint8_t* lvl = a.ms_direct ? nullptr : a.ms_lvl + static_cast<size_t>(blockIdx.x) * N * kS;  // [N][kS]
  // arrival log (u16 / u32 masks, kLog): each wave appends its nodes' level
  // events {new bits (hi), slice j << 14 | lane << 8 | level (lo)} to a log
  // of its own - one scalar count, one coalesced store per (j, level) with
  // arrivals - and the node-major level blocks are assembled from the logs
  // once the search ends. Capacity: a node gains >= 1 bit per event, so
  // J * 64 * kS events per wave
  constexpr bool kLog = sizeof(M) <= 4;
  const uint32_t lane = tid & 63u, wave = tid >> 6, waves = B >> 6;
  uint64_t* wlog = kLog ? a.ms_log + (static_cast<size_t>(blockIdx.x) * waves + wave) * J * 64u * kS : nullptr;
  uint32_t wcnt = 0;  // events in this wave's log (wave-uniform)
  __shared__ uint32_t s_wcnt[16];
  auto log_events = [&](int j, V nx, uint32_t lv) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(nx != 0u);
    if (!m) return;
    if (nx) {
      const uint32_t pos = wcnt + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
      wlog[pos] = (static_cast<uint64_t>(nx) << 32) | (static_cast<uint32_t>(j) << 14) | (lane << 8) |
                  min(lv, kLvlDirect);
    }
    wcnt += static_cast<uint32_t>(__builtin_popcountll(m));
  };
#ifdef ORH_DIAG_STAMPS
  const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif

  for (uint32_t i = tid; i < 2 * a.ms_pitch; i += B) f_cur[i] = 0;
  if (tid < 3) {
    s_prog[tid] = 0u;
    s_lo[tid] = ~0u;
    s_hin[tid] = ~0u;
  }
  if (!kLog) {  // every level byte starts as "unreached"
    uint4* l4 = reinterpret_cast<uint4*>(lvl);
    for (uint32_t i = tid; i < N * kS / 16; i += B) l4[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
  }
  __syncthreads();
  if (tid < S) {  // sources may repeat: OR the bits in
    const uint32_t src = a.dev_of[a.srcs[a.order[b0 + tid]]];
    const uintptr_t byte = reinterpret_cast<uintptr_t>(f_cur + src) + tid / 8u;
    atomicOr(reinterpret_cast<uint32_t*>(byte & ~uintptr_t(3)), 1u << ((byte & 3u) * 8u + (tid & 7u)));
    if (!kLog) lvl[static_cast<size_t>(src) * kS + tid] = 0;
  }
  if (kSkip && tid < S) {  // level 0's frontier: the sources
    const uint32_t src = a.dev_of[a.srcs[a.order[b0 + tid]]];
    atomicMin(&s_lo[0], src);
    atomicMin(&s_hin[0], ~src);
  }

  uint32_t col[J][KH];
  V vis[J];
  uint32_t ovlm = 0u, ovfm = 0u;  // bit j: owned node j overloaded / has an overflow list
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t v = j * B + tid;
#pragma unroll
    for (int h = 0; h < KH; ++h) col[j][h] = (NZ * kC) | ((NZ * kC) << 16);
    vis[j] = full;
    if (v < N) {
      const uint2* slots = a.recs + static_cast<size_t>(v) * K;
      uint2 r[K];
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] = slots[k];
#ifdef ORH_X_SORT
      uint32_t c[2 * KH];
#pragma unroll
      for (int k = 0; k < 2 * KH; ++k) c[k] = k < K ? ms_col(r[k], NZ) : NZ;
#pragma unroll
      for (int x = 0; x < 2 * KH; ++x)
#pragma unroll
        for (int y = 0; y + 1 < 2 * KH - x; ++y) {
          const uint32_t lo = min(c[y], c[y + 1]), hi = max(c[y], c[y + 1]);
          c[y] = lo;
          c[y + 1] = hi;
        }
#pragma unroll
      for (int h = 0; h < KH; ++h) col[j][h] = c[2 * h] * kC | (c[2 * h + 1] * kC << 16);
#else
#pragma unroll
      for (int h = 0; h < KH; ++h)
        col[j][h] = ms_col(r[2 * h], NZ) * kC | ((2 * h + 1 < K ? ms_col(r[2 * h + 1], NZ) : NZ) * kC << 16);
#endif
      if (r[0].x & ORH_REC_ROW_OVL) ovlm |= 1u << j;
      if (r[K - 1].x & ORH_REC_CONT) ovfm |= 1u << j;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t v = j * B + tid;
    if (v < N) vis[j] = f_cur[v];  // level 0: the sources
    if (kLog) log_events(j, v < N ? vis[j] : V(0), 0u);
  }
  // ORH_MS_WAVE_UNIFORM (A/B builds): wave-uniform bit j, some lane of this
  // wave owns, in slice j, a node with an overflow list / an overloaded node,
  // tested before the per-lane tests. Measured slower: the kernel grew from 89
  // to 107 VGPRs and the 2-lane step from 23.0 to 26.5 ms
  // (profiles/r06/g_ms_ab.txt), so the per-lane tests stay alone
#ifdef ORH_MS_WAVE_UNIFORM
  uint32_t wovf = 0u, wovl = 0u;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    wovf |= (__builtin_amdgcn_ballot_w64((ovfm >> j) & 1u) != 0u ? 1u : 0u) << j;
    wovl |= (__builtin_amdgcn_ballot_w64((ovlm >> j) & 1u) != 0u ? 1u : 0u) << j;
  }
  wovf = __builtin_amdgcn_readfirstlane(wovf);
  wovl = __builtin_amdgcn_readfirstlane(wovl);
#else
  const uint32_t wovf = ~0u, wovl = ~0u;
#endif

  const uint32_t w0 = a.w0;
#ifdef ORH_DIAG_STAMPS
  const uint64_t t_begin = __builtin_amdgcn_s_memtime();
  uint64_t t_bar = 0, t_store = 0;
  uint32_t n_levels = 0;
#endif
  const uint32_t bw = a.ms_bw;
  const uint32_t wave_base = __builtin_amdgcn_readfirstlane(tid & ~63u);
  for (uint32_t level = 1;; ++level) {
    int prog = 0;
    // opaque per level: keeps the compiler from hoisting J * K unpacked LDS
    // addresses and J per-node pointers out of the level loop (VGPR budget:
    // a 768-thread workgroup per CU at J = 16 uses ~74)
    uint32_t me = tid;
    asm volatile("" : "+v"(me));
    // ids that can gain a bit at this level: within bw of the previous
    // level's new frontier (scalar; empty when the frontier was)
    uint32_t reach_lo = 0u, reach_hi = ~0u, jm = 0u;  // jm: this wave's slices with a new frontier bit
    // first id of this wave's slice j0 (advanced by B per slice; opaque per
    // level so the 16 slice bases are not hoisted into SGPRs that spill)
    uint32_t slice = wave_base;
    if constexpr (kSkip) asm volatile("" : "+s"(slice));
    if constexpr (kSkip) {
      const uint32_t lo = __builtin_amdgcn_readfirstlane(s_lo[(level + 2u) % 3u]);
      const uint32_t hi = ~__builtin_amdgcn_readfirstlane(s_hin[(level + 2u) % 3u]);
      reach_lo = lo > bw ? lo - bw : 0u;
      reach_hi = hi + bw;
      if (tid < 1) {  // read at level - 1, written at level + 1
        s_lo[(level + 1u) % 3u] = ~0u;
        s_hin[(level + 1u) % 3u] = ~0u;
      }
    }
    // groups of G owned nodes: a group is skipped when every lane holds all
    // bits for all G nodes (wave-uniform branch); otherwise all G * K
    // frontier reads go out back to back before any is consumed. The skip
    // variant tests single slices (G = 1): its active band is a slice or two
    // per wave, and a group of 4 would do 2-4x the reads the band needs
// owned nodes whose frontier reads go out together: 2 (round 4: one C2 sweep
// 0.859 -> 0.823 ms and the 4-lane step 25.6 -> 25.0 ms against 4; 5: no
// change; 10: slower - profiles/r04/v_ms_group_ab.txt). A/B builds: -DORH_MS_GROUP
#ifndef ORH_MS_GROUP
#define ORH_MS_GROUP 2
#endif
    constexpr int G = kSkip ? 1 : (J % ORH_MS_GROUP == 0 ? ORH_MS_GROUP : 2);
#pragma unroll
    for (int j0 = 0; j0 < J; j0 += G) {
      const uint32_t sl = slice;
      if constexpr (kSkip) slice += B;
      bool open = false;
#pragma unroll
      for (int g = 0; g < G; ++g) open |= vis[j0 + g] != full;
      if (!__builtin_amdgcn_ballot_w64(open)) continue;
      // no new frontier within reach of the slice: nothing can arrive, and
      // its f_nxt entries stay stale (harmless, see above)
      if (kSkip && (sl > reach_hi || sl + 63u < reach_lo)) continue;
      V acc[G];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int h = 0; h < KH; ++h) asm volatile("" : "+v"(col[j0 + g][h]));
#pragma unroll
      for (int g = 0; g < G; ++g) {
        acc[g] = 0u;
#pragma unroll
        for (int h = 0; h < KH; ++h) {
          acc[g] |= *reinterpret_cast<const M*>(lbase + cur_off + (col[j0 + g][h] & 0xFFFFu) * (kE / kC));
          if (2 * h + 1 < K)
            acc[g] |= *reinterpret_cast<const M*>(lbase + cur_off + (col[j0 + g][h] >> 16) * (kE / kC));
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int j = j0 + g;
        const uint32_t v = j * B + me;
        V nx = 0u;
        if (vis[j] != full) {  // also every v >= N
          if (((wovf >> j) & 1u) && ((ovfm >> j) & 1u)) {
            const uint2 last = a.recs[static_cast<size_t>(v) * K + K - 1];
            const uint2* ov = a.recs + (last.x & ORH_REC_COL_MASK);
            for (uint32_t q = 0; q < last.y; ++q) {
              const uint32_t r = ov[q].x;
              if (!(r & ORH_REC_SKIP)) acc[g] |= f_cur[r & ORH_REC_COL_MASK];
            }
          }
          nx = acc[g] & ~vis[j];
          vis[j] |= nx;
        }
#ifdef ORH_DIAG_STAMPS
        const uint64_t t_s0 = __builtin_amdgcn_s_memtime();
#endif
#ifndef ORH_EXP_NO_LVL_STORE  // timing experiment only: drops the level bytes
        if (kLog) log_events(j, nx, level);
#endif
        if (nx) {
          prog = 1;
#ifndef ORH_EXP_NO_LVL_STORE
          {
          uint8_t* lb = lvl + static_cast<size_t>(v) * kS;
          if (level < kLvlDirect) {
            if (!kLog)
              for (V q = nx; q; q &= q - 1) lb[MsMask<M>::ctz(q)] = static_cast<uint8_t>(level);
          } else {  // deep levels: the distance row directly (the level byte says so)
            const uint32_t vh = a.host_of[v];
            for (V q = nx; q; q &= q - 1) {
              const uint32_t b = MsMask<M>::ctz(q);
              if (!kLog) lb[b] = kLvlDirect;
              dist_row(a.out_dist, a.scratch, a.n_out, N, a.order[b0 + b])[vh] = level * w0;
            }
          }
          }
#endif
        }
#ifdef ORH_DIAG_STAMPS
        t_store += __builtin_amdgcn_s_memtime() - t_s0;
#endif
        if (((wovl >> j) & 1u) && ((ovlm >> j) & 1u)) nx = 0u;  // reached, but no transit through an overloaded node
#ifndef ORH_MS_WRITE_ZEROS
        // only a node with new bits writes its entry: whatever an entry still
        // holds from an older level (bits that reached it at level L - 2k)
        // reached every neighbour by level L - 2k + 1, so the pull masks it
        // with the neighbour's visited bits. Writing the zeros (every open
        // node, every level) was ~1/3 of the loop's LDS cycles
        // (ORH_MS_WRITE_ZEROS, A/B builds: the former stores)
        if (nx) f_nxt[v] = static_cast<M>(nx);
#else
        if (vis[j] != full || nx) f_nxt[v] = static_cast<M>(nx);
#endif
        if constexpr (kSkip) jm |= (__builtin_amdgcn_ballot_w64(nx != 0u) != 0u ? 1u : 0u) << j;
      }
    }
    if constexpr (kSkip) {  // this wave's new-frontier slices into the level's interval
      if (jm && (tid & 63u) == 0) {
        const uint32_t jl = static_cast<uint32_t>(__builtin_ctz(jm));
        const uint32_t jh = 31u - static_cast<uint32_t>(__builtin_clz(jm));
        atomicMin(&s_lo[level % 3u], jl * B + wave_base);
        atomicMin(&s_hin[level % 3u], ~(jh * B + wave_base + 63u));
      }
    }
    // every level that makes progress adds >= 1 visited bit: at most S * N
    // levels. The barrier waits for LDS traffic only: the level bytes on
    // their way to memory are read by the next kernel, and waiting for their
    // write acknowledgements every level (what __syncthreads does) is wasted.
    if (prog) s_prog[level % 3u] = 1u;
#ifdef ORH_DIAG_STAMPS
    const uint64_t t_b0 = __builtin_amdgcn_s_memtime();
#endif
    lds_barrier();
#ifdef ORH_DIAG_STAMPS
    t_bar += __builtin_amdgcn_s_memtime() - t_b0;
    ++n_levels;
#endif
    if (!s_prog[level % 3u]) break;
    if (tid == 0) s_prog[(level + 2u) % 3u] = 0u;  // the previous level's flag, read before this barrier
    M* t = f_cur;
    f_cur = f_nxt;
    f_nxt = t;
    const uint32_t to = cur_off;
    cur_off = nxt_off;
    nxt_off = to;
  }
  if constexpr (kLog) {
    // the logs -> node-major level blocks, one wave's nodes at a time: the
    // workgroup zeroes their J * 64 blocks in LDS (the frontier arrays are
    // free once every wave has left the level loop), scatters the wave's
    // events into them (loads in flight eight at a time) and writes the
    // blocks out whole, 16 bytes a thread
    if (lane == 0) s_wcnt[wave] = wcnt;
    __shared__ uint32_t s_row[kS];
    if (tid < S) s_row[tid] = a.order[b0 + tid];
    __syncthreads();
    // node blocks padded to kS + 4 bytes: consecutive blocks start 9 (kS =
    // 32) or 5 (kS = 16) banks apart, so the scattered byte writes of a wave
    // spread over the banks instead of 8 blocks sharing one
    constexpr uint32_t kP = kS + 4, kQ = kS / 16;
    uint8_t* blk = reinterpret_cast<uint8_t*>(lds);
    const uint32_t nw32 = J * 64u * kP / 4u;
    for (uint32_t w = 0; w < waves; ++w) {
      for (uint32_t i = tid; i < nw32; i += B) lds[i] = ~0u;
      __syncthreads();
      const uint32_t n_ev = s_wcnt[w];
      const uint64_t* wl = a.ms_log + (static_cast<size_t>(blockIdx.x) * waves + w) * J * 64u * kS;
      for (uint32_t e0 = tid; e0 < n_ev; e0 += 8u * B) {
        uint64_t x[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) x[u] = e0 + u * B < n_ev ? wl[e0 + u * B] : 0ull;
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          uint8_t* nb = blk + ((static_cast<uint32_t>(x[u]) >> 8) & 0x7FFu) * kP;  // (j * 64 + lane) * kP
          const uint8_t lv = static_cast<uint8_t>(x[u] & 0xFFu);
          for (V q = static_cast<V>(x[u] >> 32); q; q &= q - 1) nb[MsMask<M>::ctz(q)] = lv;
        }
      }
      __syncthreads();
      if (a.ms_direct) {
        // host-order layout: the wave's slice j is the host ids j * B + w * 64
        // + [0, 64), so each source's row gets 64 consecutive levels - the
        // u8 level row and the u32 distance row written here, coalesced (a
        // thread: 4 nodes of one source; 16 threads: one 64-node run). The
        // padding [N, lvl_pitch) of the level rows is "unreached" (no event
        // lands there). Deep levels (marker 254) were written during the search
        const uint32_t P = a.lvl_pitch, w0 = a.w0, nq = J * 16u;
        for (uint32_t i = tid; i < S * nq; i += B) {
          const uint32_t b = i / nq, jq = i % nq;
          const uint32_t j = jq >> 4, n0 = j * 64u + (jq & 15u) * 4u;
          const uint32_t v0 = j * B + w * 64u + (jq & 15u) * 4u;
          if (v0 >= P) continue;
          const uint8_t* nb = blk + n0 * kP + b;
          const uint32_t l[4] = {nb[0], nb[kP], nb[2 * kP], nb[3 * kP]};
          const uint32_t r = s_row[b];
          *reinterpret_cast<uint32_t*>(a.lvl_rows + static_cast<size_t>(r) * P + v0) =
              l[0] | (l[1] << 8) | (l[2] << 16) | (l[3] << 24);
          if (r >= a.n_out || v0 >= N) continue;  // a neighbour row is read through its level row
          uint32_t d[4];
          bool deep = false;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            d[k] = l[k] == kLvlNone ? kInf : l[k] * w0;
            deep |= l[k] == kLvlDirect;
          }
          uint32_t* od = a.out_dist + static_cast<size_t>(r) * N + v0;
          if (!deep && v0 + 4u <= N && (reinterpret_cast<uintptr_t>(od) & 15u) == 0u) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 q = {d[0], d[1], d[2], d[3]};
            __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(od));
          } else {
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
              if (v0 + k < N && l[k] != kLvlDirect) __builtin_nontemporal_store(d[k], od + k);
          }
        }
      } else {
        for (uint32_t i = tid; i < J * 64u * kQ; i += B) {
          const uint32_t node = i / kQ, q = i % kQ;  // node = j * 64 + lane
          const uint32_t v = (node >> 6) * B + w * 64u + (node & 63u);
          const uint32_t* src = lds + node * (kP / 4u) + q * 4u;
          if (v < N)
            reinterpret_cast<uint4*>(lvl + static_cast<size_t>(v) * kS)[q] = make_uint4(src[0], src[1], src[2], src[3]);
        }
      }
      __syncthreads();
    }
  }
#ifdef ORH_DIAG_STAMPS
  if (tid == 0 && blockIdx.x < 4096) {  // per workgroup: entry, exit, hardware id, levels
    uint64_t* w = a.diag + 16 + 4 * static_cast<size_t>(blockIdx.x);
    w[0] = t_entry;
    w[1] = __builtin_amdgcn_s_memtime();
    w[2] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF804)) |
           (static_cast<uint64_t>(__builtin_amdgcn_s_getreg(0xF814)) << 32);
    w[3] = n_levels;
  }
  if ((tid & 63u) == 0) {  // per wave: total, barrier and store-block cycles, levels
    const uint64_t tot = __builtin_amdgcn_s_memtime() - t_begin;
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.diag[0]), tot);
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.diag[1]), t_bar);
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.diag[3]), static_cast<unsigned long long>(n_levels));
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.diag[4]), 1ull);
    atomicMax(reinterpret_cast<unsigned long long*>(&a.diag[5]), tot);
    atomicMax(reinterpret_cast<unsigned long long*>(&a.diag[6]), static_cast<unsigned long long>(n_levels));
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.diag[8]), t_store);
  }
#endif
}

// node-major level bytes -> host-order u32 distance rows, one workgroup per
// (batch, 256-node host tile); per source bit b the 256 stores of a row are
// contiguous
template <class M>
__global__ __launch_bounds__(256) void ms_finalize_kernel(SpfArgs a, uint32_t tiles) {
  constexpr uint32_t kS = MsMask<M>::kS;
  __shared__ uint32_t* s_out[kS];
  __shared__ uint32_t s_row[kS];
  const uint32_t N = a.n_nodes;
  const uint32_t batch = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const uint32_t i = tile * 256 + threadIdx.x;
  const uint32_t b0 = batch * a.ms_width;
  const uint32_t S = min(a.ms_width, a.n_rows - b0);
  if (threadIdx.x < S) {
    s_row[threadIdx.x] = a.order[b0 + threadIdx.x];
    s_out[threadIdx.x] = dist_row(a.out_dist, a.scratch, a.n_out, N, s_row[threadIdx.x]);
  }
  __syncthreads();
  if (i >= N) {  // level-row padding [N, pitch): "unreached" for the 16-byte reads
    if (i < a.lvl_pitch)
      for (uint32_t b = 0; b < S; ++b)
        a.lvl_rows[static_cast<size_t>(s_row[b]) * a.lvl_pitch + i] = static_cast<uint8_t>(kLvlNone);
    return;
  }
  const uint32_t v = a.dev_of[i];
  const uint4* blk = reinterpret_cast<const uint4*>(a.ms_lvl + (static_cast<size_t>(batch) * N + v) * kS);
  uint32_t w[kS / 4];
#pragma unroll
  for (int q = 0; q < static_cast<int>(kS / 16); ++q) {
    const uint4 x = blk[q];
    w[4 * q] = x.x;
    w[4 * q + 1] = x.y;
    w[4 * q + 2] = x.z;
    w[4 * q + 3] = x.w;
  }
  const uint32_t w0 = a.w0;
#pragma unroll
  for (uint32_t b = 0; b < kS; ++b) {
    if (b >= S) break;
    const uint32_t l = (w[b / 4] >> ((b & 3u) * 8u)) & 0xFFu;
    const uint32_t r = s_row[b];
    a.lvl_rows[static_cast<size_t>(r) * a.lvl_pitch + i] = static_cast<uint8_t>(l);
    // neighbour-only rows are read through their level row
    if (l == kLvlDirect || r >= a.n_out) continue;
    __builtin_nontemporal_store(l == kLvlNone ? kInf : l * w0, &s_out[b][i]);
  }
}

// ---------------------------------------------------------------------------
// fused BFS + first hops, one workgroup per source (kBfsNh)
// ---------------------------------------------------------------------------
// For a few sources (a route build's own SPF, small what-if batches) the
// two-phase plans search the source AND each of its neighbours (the
// closed-form first hops read the neighbours' rows), 5x the rows on a grid,
// then launch the first-hop phase. Here the first hops ride along the
// search, as in runSpf itself (LinkState.cpp:857-873): a level-L node pushes
// to its neighbours, claims the unvisited ones for level L+1 (LDS CAS) and
// ORs its first-hop mask into every neighbour at level L+1 - all of them
// tight, the metric being uniform. The source's neighbours start with their
// own bit. Overloaded nodes are reached but do not push (no transit).
// Thread t owns nodes t, t + B, ...: their ELL columns (dead, down and
// ignored records folded to a never-claimable dummy slot) sit in registers,
// so a level is one batch of LDS reads (the owned unsettled nodes' levels),
// then per frontier node one batch of neighbour-level reads and
// fire-and-forget claims / ORs (no return-value round trips); no global
// memory is touched until the rows are written out, coalesced.
// LDS: level u32 [N + 1] | first hops u32 [N * words].
template <int K, int J>
__global__ __launch_bounds__(kMaxBlock) void spf_bfs_nh_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr int KH = (K + 1) / 2;
  const uint32_t N = a.n_nodes, W = a.words, B = blockDim.x, tid = threadIdx.x;
  const uint32_t row = blockIdx.x;
  const uint32_t NZ = N;  // dummy slot: level 0, never claimed, never expanded
  uint32_t* lvl = lds;
  uint32_t* nh = lds + ((N + 4u) & ~3u);
  __shared__ uint32_t s_prog[3];
  const uint32_t src = a.srcs[row];
  const uint32_t* ign = nullptr;
  uint32_t n_ign = 0;
  if (a.ignore_ptr) {
    ign = a.ignore_links + a.ignore_ptr[row];
    n_ign = a.ignore_ptr[row + 1] - a.ignore_ptr[row];
  }
  for (uint32_t i = tid; i < N; i += B) lvl[i] = kInf;
  if (tid == 0) lvl[NZ] = 0u;
  for (uint32_t i = tid; i < N * W; i += B) nh[i] = 0u;
  if (tid < 3) s_prog[tid] = 0u;
  auto live = [&](const uint2& r, size_t q) {
    return !(r.x & (ORH_REC_SKIP | ORH_REC_CONT)) && !(n_ign && ignored(ign, n_ign, a.link[q]));
  };
  uint32_t col[J][KH];
  uint32_t ovlm = 0u, ovfm = 0u, open = 0u;  // bit j: overloaded / overflow list / not yet expanded
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t v = j * B + tid;
#pragma unroll
    for (int h = 0; h < KH; ++h) col[j][h] = NZ | (NZ << 16);
    if (v < N) {
      open |= 1u << j;
      const size_t q0 = static_cast<size_t>(v) * K;
      uint32_t c[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint2 r = a.recs[q0 + k];
        c[k] = live(r, q0 + k) ? (r.x & ORH_REC_COL_MASK) : NZ;
        if (k == 0 && (r.x & ORH_REC_ROW_OVL)) ovlm |= 1u << j;
        if (k == K - 1 && (r.x & ORH_REC_CONT)) ovfm |= 1u << j;
      }
#pragma unroll
      for (int h = 0; h < KH; ++h) col[j][h] = c[2 * h] | ((2 * h + 1 < K ? c[2 * h + 1] : NZ) << 16);
    }
  }
  __syncthreads();
  // level 1: the source's live neighbours, each with its own first-hop bit
  // (its rank among the source's distinct neighbours, LinkState.cpp:869-872)
  if (tid == 0) lvl[src] = 0u;
  {
    const size_t q0 = static_cast<size_t>(src) * K;
    const uint2 last = a.recs[q0 + K - 1];
    const uint32_t n_ovf = (last.x & ORH_REC_CONT) ? last.y : 0u;
    const size_t ovf0 = last.x & ORH_REC_COL_MASK;
    for (uint32_t k = tid; k < K + n_ovf; k += B) {
      const size_t q = k < K ? q0 + k : ovf0 + (k - K);
      const uint2 r = a.recs[q];
      if (!live(r, q)) continue;
      const uint32_t u = r.x & ORH_REC_COL_MASK;
      if (u == src) continue;
      atomicCAS(&lvl[u], kInf, 1u);
      const uint32_t b = a.rank_out[q];
      atomicOr(&nh[static_cast<size_t>(u) * W + (b >> 5)], 1u << (b & 31u));
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j)  // the source itself is settled: it pushed above
    if (j * B + tid == src) open &= ~(1u << j);
  for (uint32_t level = 1;; ++level) {
    int prog = 0;
    uint32_t me = tid;
    asm volatile("" : "+v"(me));
    // the packed columns are opaque per level: otherwise the compiler hoists
    // their unpacked halves and the neighbour addresses out of the level loop
    // (4 x the registers of col per owned node, spilling at J >= 8)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int h = 0; h < KH; ++h) asm volatile("" : "+v"(col[j][h]));
    // every owned unsettled node's level in one batch of independent reads
    uint32_t lv[J];
#pragma unroll
    for (int j = 0; j < J; ++j) lv[j] = ((open >> j) & 1u) ? lvl[j * B + me] : 0u;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if (lv[j] != level) continue;  // settled, unreached, or claimed for the next level
      open &= ~(1u << j);
      if ((ovlm >> j) & 1u) continue;  // reached, no transit
      const uint32_t v = j * B + me;
      // the neighbours' levels, then fire-and-forget claims and ORs: only
      // level + 1 claims happen during this level, so a neighbour read as
      // unreached or level + 1 ends the level at level + 1
      uint32_t u[2 * KH], lu[2 * KH];
#pragma unroll
      for (int h = 0; h < KH; ++h) {
        u[2 * h] = col[j][h] & 0xFFFFu;
        u[2 * h + 1] = col[j][h] >> 16;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) lu[k] = lvl[u[k]];
      uint32_t m0 = nh[static_cast<size_t>(v) * W];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (lu[k] != kInf && lu[k] != level + 1u) continue;
        if (lu[k] == kInf) {
          prog = 1;
          atomicMin(&lvl[u[k]], level + 1u);
        }
        if (m0) atomicOr(&nh[static_cast<size_t>(u[k]) * W], m0);
        for (uint32_t w = 1; w < W; ++w) {
          const uint32_t m = nh[static_cast<size_t>(v) * W + w];
          if (m) atomicOr(&nh[static_cast<size_t>(u[k]) * W + w], m);
        }
      }
      if ((ovfm >> j) & 1u) {
        const uint2 last = a.recs[static_cast<size_t>(v) * K + K - 1];
        const size_t ovf0 = last.x & ORH_REC_COL_MASK;
        for (uint32_t q = 0; q < last.y; ++q) {
          const uint2 r = a.recs[ovf0 + q];
          if (!live(r, ovf0 + q)) continue;
          const uint32_t x = r.x & ORH_REC_COL_MASK;
          const uint32_t lx = lvl[x];
          if (lx != kInf && lx != level + 1u) continue;
          if (lx == kInf) {
            prog = 1;
            atomicMin(&lvl[x], level + 1u);
          }
          for (uint32_t w = 0; w < W; ++w) {
            const uint32_t m = nh[static_cast<size_t>(v) * W + w];
            if (m) atomicOr(&nh[static_cast<size_t>(x) * W + w], m);
          }
        }
      }
    }
    // levels are < N, so the loop ends; a level that claims nothing is the last
    if (prog) s_prog[level % 3u] = 1u;
    __syncthreads();
    if (!s_prog[level % 3u]) break;
    if (tid == 0) s_prog[(level + 2u) % 3u] = 0u;
  }
  uint32_t* od = a.out_dist + static_cast<size_t>(row) * N;
  uint32_t* on = a.out_nh + static_cast<size_t>(row) * N * W;
  const uint32_t w0 = a.w0;
  for (uint32_t i = tid; i < N; i += B) {
    const uint32_t l = lvl[i];
    __builtin_nontemporal_store(l == kInf ? kInf : l * w0, &od[i]);
  }
  for (uint32_t i = tid; i < N * W; i += B) __builtin_nontemporal_store(nh[i], &on[i]);
}

// ---------------------------------------------------------------------------
// phase 1b: level-synchronous Dijkstra on a u16 / u32 distance per node
// ---------------------------------------------------------------------------
template <class T>
struct DistWord;

template <>
struct DistWord<uint32_t> {
  static constexpr uint32_t kInfT = 0xFFFFFFFFu;
  __device__ static uint32_t get(const uint32_t* d, uint32_t u) { return d[u]; }
  // lower d[u] to nd (> D); returns the previous value if it was lowered, else nd
  __device__ static bool lower(uint32_t* d, uint32_t u, uint32_t du, uint32_t nd, bool& first) {
    if (nd >= du) return false;
    atomicMin(&d[u], nd);
    first = du == kInfT;
    return true;
  }
};

template <>
struct DistWord<uint16_t> {  // two nodes per u32 word; updated by compare-and-swap
  static constexpr uint32_t kInfT = 0xFFFFu;
  __device__ static uint32_t get(const uint32_t* d, uint32_t u) {
    return (d[u >> 1] >> ((u & 1u) * 16u)) & 0xFFFFu;
  }
  __device__ static bool lower(uint32_t* d, uint32_t u, uint32_t du, uint32_t nd, bool& first) {
    if (nd >= du) return false;
    const uint32_t sh = (u & 1u) * 16u;
    uint32_t old = d[u >> 1];
    for (;;) {
      const uint32_t cur = (old >> sh) & 0xFFFFu;
      if (nd >= cur) return false;  // lowered further by another lane
      const uint32_t nw = (old & ~(0xFFFFu << sh)) | (nd << sh);
      const uint32_t prev = atomicCAS(&d[u >> 1], old, nw);
      if (prev == old) {
        first = cur == 0xFFFFu;
        return true;
      }
      old = prev;
    }
  }
};

template <class T, int K>
struct Dij {
  using DW = DistWord<T>;
  const SpfArgs& a;
  const Src& s;
  uint32_t* dist;  // LDS, T per node
  uint32_t* pend;

  __device__ void edge(const uint2& r, uint32_t du, uint32_t D, uint32_t& lowered) const {
    const uint32_t u = r.x & ORH_REC_COL_MASK;
    const uint32_t nd = D + (a.use_link_metric ? r.y : 1u);
    bool first = false;
    if (DW::lower(dist, u, du, nd, first)) {
      lowered = min(lowered, nd);
      if (first) atomicOr(&pend[u >> 5], 1u << (u & 31u));
    }
  }

  // relax v's out-links at distance D; returns the smallest distance it lowered
  __device__ uint32_t expand(uint32_t v, const uint2 (&rec)[K], uint32_t D) const {
    uint32_t lowered = kInf;
    if (v != s.node && (rec[0].x & ORH_REC_ROW_OVL)) return lowered;
    uint32_t du[K];
    bool lv[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      lv[j] = live(a, s, rec[j], v * K + j);
      du[j] = lv[j] ? DW::get(dist, rec[j].x & ORH_REC_COL_MASK) : 0u;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (lv[j]) edge(rec[j], du[j], D, lowered);
    const uint2 last = rec[K - 1];
    if (last.x & ORH_REC_CONT) {
      const uint32_t start = last.x & ORH_REC_COL_MASK;
      for (uint32_t base = 0; base < last.y; base += kOvfBatch) {
        const uint32_t cnt = min(last.y - base, static_cast<uint32_t>(kOvfBatch));
        uint2 ov[kOvfBatch];
#pragma unroll
        for (int j = 0; j < kOvfBatch; ++j)
          if (j < static_cast<int>(cnt)) ov[j] = a.recs[start + base + j];
        uint32_t od[kOvfBatch];
        bool ol[kOvfBatch];
#pragma unroll
        for (int j = 0; j < kOvfBatch; ++j) {
          ol[j] = j < static_cast<int>(cnt) && live(a, s, ov[j], start + base + j);
          od[j] = ol[j] ? DW::get(dist, ov[j].x & ORH_REC_COL_MASK) : 0u;
        }
#pragma unroll
        for (int j = 0; j < kOvfBatch; ++j)
          if (ol[j]) edge(ov[j], od[j], D, lowered);
      }
    }
    return lowered;
  }
};

template <class T, int K>
__global__ __launch_bounds__(kMaxBlock) void spf_dist_kernel(SpfArgs a) {
  using DW = DistWord<T>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_min[3];
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x, row = blockIdx.x;
  uint32_t* dist = lds;
  uint32_t* pend = lds + a.lds_pend_off / 4;
  const Src s(a, row);
  const Dij<T, K> d{a, s, dist, pend};

  const uint32_t dwords = a.lds_pend_off / 4;
  for (uint32_t i = tid; i < dwords; i += nthr) dist[i] = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < NB; i += nthr) pend[i] = 0u;
  if (tid < 3) s_min[tid] = kInf;
  __syncthreads();
  if (tid == 0) {
    bool first;
    DW::lower(dist, s.node, DW::kInfT, 0u, first);
    pend[s.node >> 5] = 1u << (s.node & 31u);
  }
  __syncthreads();

  constexpr int kBatch = 16 / K;
  constexpr int kScan = 8;  // pending distances read together
  uint32_t D = 0;
  for (uint32_t level = 0;; ++level) {
    const uint32_t slot = level % 3u;  // rotation as in spf_bfs_kernel
    uint32_t local_min = kInf;
    for (uint32_t w = tid; w < NB; w += 2 * nthr) {
      const uint32_t w2 = w + nthr;
      uint64_t bits = pend[w] | (static_cast<uint64_t>(w2 < NB ? pend[w2] : 0u) << 32);
      // split the pending nodes into those at D (expand now) and the rest
      // (candidates for the next D)
      uint64_t todo = 0;
      while (bits) {
        uint32_t bs[kScan], dv[kScan];
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < kScan; ++i) {
          if (bits) {
            bs[i] = static_cast<uint32_t>(__builtin_ctzll(bits));
            bits &= bits - 1;
            const uint32_t v = bs[i] < 32 ? w * 32 + bs[i] : w2 * 32 + (bs[i] - 32);
            dv[i] = DW::get(dist, v);
            cnt = i + 1;
          }
        }
#pragma unroll
        for (int i = 0; i < kScan; ++i) {
          if (i < cnt) {
            if (dv[i] == D) todo |= 1ull << bs[i];
            else local_min = min(local_min, dv[i]);
          }
        }
      }
      if (!todo) continue;
      if (static_cast<uint32_t>(todo)) atomicAnd(&pend[w], ~static_cast<uint32_t>(todo));
      if (todo >> 32) atomicAnd(&pend[w2], ~static_cast<uint32_t>(todo >> 32));
      while (todo) {
        uint32_t vs[kBatch];
        uint2 r[kBatch][K];
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < kBatch; ++i) {
          if (todo) {
            const uint32_t bit = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            vs[i] = bit < 32 ? w * 32 + bit : w2 * 32 + (bit - 32);
            load_recs<K>(a, vs[i], r[i]);
            cnt = i + 1;
          }
        }
#pragma unroll
        for (int i = 0; i < kBatch; ++i)
          if (i < cnt) local_min = min(local_min, d.expand(vs[i], r[i], D));
      }
    }
    const uint32_t wm = wave_min(local_min);
    if ((tid & 63u) == 0 && wm != kInf) atomicMin(&s_min[slot], wm);
    __syncthreads();
    const uint32_t next = s_min[slot];
    if (next == kInf || level >= N) break;
    if (tid == 0) s_min[(level + 2u) % 3u] = kInf;  // read before this barrier by every wave
    D = next;
  }

  uint32_t* out = dist_row(a.out_dist, a.scratch, a.n_out, N, row);
  for (uint32_t i = tid; i < N; i += nthr) {
    const uint32_t dv = DW::get(dist, i);
    __builtin_nontemporal_store(dv == DW::kInfT ? kInf : dv, &out[i]);
  }
}

// ---------------------------------------------------------------------------
// phase 1c: frontier relaxation with the distances in HBM (graphs whose
// per-source state does not fit LDS, e.g. the 50k-node WAN of C4)
// ---------------------------------------------------------------------------
// One workgroup per source row. The row itself (u32, in the output or the
// scratch) holds the tentative distances; LDS holds only frontier bitmaps,
// so any N up to ~400k fits. Label-correcting with a near/far split
// (delta-stepping): a node lowered to d < T joins the next near frontier,
// one lowered to d >= T the far set; when the near frontier empties, T
// advances to (smallest far distance) + delta and the far nodes below it
// become the frontier. Exact for positive integer metrics: every lowering is
// re-expanded, so the fixpoint is the shortest-path distance. Relaxation is
// an atomicMin on the row (L2 atomics); the row is L2-resident while its
// source is searched.
template <int K>
__global__ __launch_bounds__(256) void spf_global_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_flag[3];
  __shared__ uint32_t s_min;
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x, row = blockIdx.x;
  uint32_t* near0 = lds;
  uint32_t* near1 = lds + NB;
  uint32_t* far = lds + 2 * NB;
  const Src s(a, row);
  uint32_t* dist = dist_row(a.out_dist, a.scratch, a.n_out, N, row);

  for (uint32_t i = tid; i < 3 * NB; i += nthr) lds[i] = 0u;
  for (uint32_t i = tid; i < N; i += nthr) dist[i] = kInf;
  if (tid < 3) s_flag[tid] = 0u;
  __syncthreads();  // also orders the row initialisation before the search
  if (tid == 0) {
    dist[s.node] = 0u;
    near0[s.node >> 5] = 1u << (s.node & 31u);
  }
  __syncthreads();

  const uint32_t delta = a.delta;
  uint32_t T = delta;  // near/far threshold
  uint32_t* cur = near0;
  uint32_t* nxt = near1;
  for (uint32_t it = 0;; ++it) {
    // expand the near frontier
    bool pushed_near = false;
    for (uint32_t w = tid; w < NB; w += nthr) {
      uint32_t bits = cur[w];
      if (!bits) continue;
      cur[w] = 0u;
      while (bits) {
        const uint32_t v = w * 32 + __builtin_ctz(bits);
        bits &= bits - 1;
        uint2 rec[K];
        load_recs<K>(a, v, rec);
        if (v != s.node && (rec[0].x & ORH_REC_ROW_OVL)) continue;  // no transit
        const uint32_t dv = __hip_atomic_load(&dist[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        auto relax = [&](const uint2& r, uint32_t q) {
          if (!live(a, s, r, q)) return;
          const uint32_t u = r.x & ORH_REC_COL_MASK;
          const uint32_t nd = dv + (a.use_link_metric ? r.y : 1u);
          if (nd >= __hip_atomic_load(&dist[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
          const uint32_t old = atomicMin(&dist[u], nd);
          if (nd >= old) return;
          if (nd < T) {
            atomicOr(&nxt[u >> 5], 1u << (u & 31u));
            pushed_near = true;
          } else {
            atomicOr(&far[u >> 5], 1u << (u & 31u));
          }
        };
#pragma unroll
        for (int j = 0; j < K; ++j) relax(rec[j], v * K + j);
        const uint2 last = rec[K - 1];
        if (last.x & ORH_REC_CONT) {
          const uint32_t start = last.x & ORH_REC_COL_MASK;
          for (uint32_t q = 0; q < last.y; ++q) relax(a.recs[start + q], start + q);
        }
      }
    }
    const uint32_t par = it % 3u;
    if (pushed_near) s_flag[par] = 1u;
    if (tid == 0) s_min = kInf;
    __syncthreads();  // relaxations (global atomics) and bitmaps settled
    const bool more_near = s_flag[par] != 0u;
    if (tid == 0) s_flag[(par + 2u) % 3u] = 0u;  // the previous iteration's flag
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
    if (more_near) continue;
    // near frontier empty: smallest far distance, then promote far nodes below
    // the new threshold
    uint32_t local_min = kInf;
    for (uint32_t w = tid; w < NB; w += nthr) {
      for (uint32_t bits = far[w]; bits; bits &= bits - 1) {
        const uint32_t v = w * 32 + __builtin_ctz(bits);
        local_min = min(local_min, __hip_atomic_load(&dist[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
    }
    const uint32_t wm = wave_min(local_min);
    if ((tid & 63u) == 0 && wm != kInf) atomicMin(&s_min, wm);
    __syncthreads();
    const uint32_t m = s_min;
    if (m == kInf) break;  // far set empty: done (every wave sees the same value)
    T = m + delta;
    for (uint32_t w = tid; w < NB; w += nthr) {
      uint32_t bits = far[w], promote = 0u;
      for (uint32_t q = bits; q; q &= q - 1) {
        const uint32_t b = __builtin_ctz(q);
        if (__hip_atomic_load(&dist[w * 32 + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < T)
          promote |= 1u << b;
      }
      if (promote) {
        far[w] = bits & ~promote;
        cur[w] |= promote;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// phase 1c': HBM frontier relaxation with fused first hops
// ---------------------------------------------------------------------------
// The two-phase scheme derives NH(v) from the rows of the source's
// neighbours; for a batch whose neighbour rows are not sources themselves
// (what-if SPFs, KSP2 k=2 re-runs, a subset of sources) that multiplies the
// searches by 1 + deg(s). Here the search carries the closed form directly:
// each node has a 64-bit label {dist (hi), first-hop mask (lo)} in HBM, and a
// relaxation from v offers u the candidate {d(v) + w, v == src ? bit(u) :
// nh(v)}. Labels merge in a lattice: a smaller distance replaces, an equal
// one ORs the masks; any change re-queues u (near if below the threshold,
// else far). A candidate whose distance equals d*(u) comes from a predecessor
// whose distance is already final, so stale bits never survive: the fixpoint
// is exactly (d*, NH) of SURVEY.md Appendix A.1. Used when every source has
// at most 32 distinct neighbours (one mask word).
//
// The far set also tracks a lower bound of its distances (LDS atomicMin on
// every far push, recomputed exactly while promoting), so advancing the
// threshold costs one pass over the far nodes instead of two.

// Expand frontier nodes vs[0..c) of one row: the group's record, label and
// neighbour-label loads are in flight together (one round trip per stage for
// the group instead of per node), then merge(u, nd, cnh, cl) runs per live
// out-edge with u's label cl as loaded.
// label access: {dist (hi), first-hop mask (lo)} in a u64, or the distance
// alone in a u32 (dist-only searches: KSP2 rows feed traces, not first hops)
__device__ inline uint32_t lab_dist(unsigned long long l) { return static_cast<uint32_t>(l >> 32); }
__device__ inline uint32_t lab_dist(uint32_t l) { return l; }
__device__ inline uint32_t lab_nh(unsigned long long l) { return static_cast<uint32_t>(l); }
__device__ inline uint32_t lab_nh(uint32_t) { return 0u; }

struct NoPre {
  __device__ void operator()(uint32_t) const {}
};
// pre(bound): called once the group's records are in, before any merge, with
// the most pushes the group can make (its records, continuation lists
// included); a caller that passes one calls expand_group from every lane
// (c = 0 included), so pre runs with the whole wave active
template <int K, int G, typename L, typename Merge, typename Pre = NoPre>
__device__ __forceinline__ void expand_group(const SpfArgs& a, const Src& s, L* lab,
                                             const uint32_t (&vs)[G], int c, Merge& merge,
                                             Pre&& pre = Pre{}) {
  constexpr bool kNh = sizeof(L) == 8;
  uint2 rec[G][K];
  L lv[G];
  uint32_t lk[G][K];  // link ids (ignore sets), loaded with the records
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (g >= c) break;
    load_recs<K>(a, vs[g], rec[g]);
#pragma unroll
    for (int j = 0; j < K; ++j) lk[g][j] = s.n_ign ? a.link[vs[g] * K + j] : 0u;
    lv[g] = __hip_atomic_load(&lab[vs[g]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  {
    uint32_t bound = 0;
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (g < c) bound += K + ((rec[g][K - 1].x & ORH_REC_CONT) ? rec[g][K - 1].y : 0u);
    pre(bound);
  }
  L cl[G][K];
  bool ok[G][K];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bool transit = g < c && (vs[g] == s.node || !(rec[g][0].x & ORH_REC_ROW_OVL));
#pragma unroll
    for (int j = 0; j < K; ++j) {
      ok[g][j] = transit && live_link(s, rec[g][j], lk[g][j]);
      if (ok[g][j])
        cl[g][j] = __hip_atomic_load(&lab[rec[g][j].x & ORH_REC_COL_MASK], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (g >= c) break;
    const uint32_t v = vs[g];
    if (v != s.node && (rec[g][0].x & ORH_REC_ROW_OVL)) continue;  // no transit
    const uint32_t dv = lab_dist(lv[g]);
    const uint32_t nhv = lab_nh(lv[g]);
    const bool from_src = kNh && v == s.node;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (!ok[g][j]) continue;
      const uint2 r = rec[g][j];
      merge(r.x & ORH_REC_COL_MASK, dv + (a.use_link_metric ? r.y : 1u),
            from_src ? (1u << a.rank_out[v * K + j]) : nhv, cl[g][j]);
    }
    const uint2 last = rec[g][K - 1];
    if (last.x & ORH_REC_CONT) {
      const uint32_t start = last.x & ORH_REC_COL_MASK;
      for (uint32_t q = 0; q < last.y; ++q) {
        const uint2 r = a.recs[start + q];
        if (!live(a, s, r, start + q)) continue;
        const uint32_t u = r.x & ORH_REC_COL_MASK;
        merge(u, dv + (a.use_link_metric ? r.y : 1u), from_src ? (1u << a.rank_out[start + q]) : nhv,
              __hip_atomic_load(&lab[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
    }
  }
}

// Asynchronous twin of spf_global_nh_kernel (below): within a bucket no
// barrier separates relaxation rounds. A thread claims the near nodes of its
// own words (atomicExch of the word; others only set bits) as soon as they
// appear and expands them; the bucket ends when s_work, the count of queued
// plus claimed-but-unexpanded near nodes, reaches zero. A push counts itself
// before its bit becomes visible and an expansion uncounts its nodes after
// its pushes, so the count never undercounts: zero means no near work exists
// or can appear, and every wave leaves the loop on the same condition. The
// lattice fixpoint does not depend on the order relaxations run in, so the
// result is the synchronous kernel's bit for bit; what goes away is the
// per-round barrier that held every wave to the slowest one (the C4 WAN runs
// about a hundred near rounds per search).
// ORH_ASYNC_WAVE_COUNT=0 (A/B builds): per-lane updates of the work count
#ifndef ORH_ASYNC_WAVE_COUNT
#define ORH_ASYNC_WAVE_COUNT 1
#endif
template <int K, bool kNh>
__global__ __launch_bounds__(1024) void spf_global_nh_async_kernel(SpfArgs a) {
  typedef typename std::conditional<kNh, unsigned long long, uint32_t>::type L;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_work;
  __shared__ uint32_t s_min[2];
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  if (a.row_list && blockIdx.x >= *a.row_count) return;
  const uint32_t row = a.row_list ? a.row_list[blockIdx.x] : blockIdx.x;
  constexpr L kInfLabel = kNh ? static_cast<L>(0xFFFFFFFF00000000ull) : static_cast<L>(kInf);
  constexpr int G = K <= 4 ? 4 : 2;
  __shared__ uint32_t s_nign;
  uint32_t* near = lds;
  uint32_t* far = lds + NB;
  if (a.row_mask && !a.row_mask[row]) return;  // repaired elsewhere (whole workgroup)
  Src s(a, row);
  L* lab = reinterpret_cast<L*>(a.labels) + static_cast<size_t>(a.row_list ? blockIdx.x : row) * N;
  // the plan's third bitmap (the synchronous kernel's second near set) holds
  // the ignore filter: FW words, a power of two <= 256, and the set's real
  // length (fixed-stride lists end in ~0u padding, e.g. KSP2's k = 2 rows)
  uint32_t* filt = lds + 2 * NB;
  uint32_t FW = 1;
  while (2 * FW <= min(NB, 256u)) FW *= 2;
  const uint32_t fshift = 32u - (5u + static_cast<uint32_t>(__builtin_ctz(FW)));

  for (uint32_t i = tid; i < 2 * NB; i += nthr) lds[i] = 0u;
  if (s.n_ign)
    for (uint32_t i = tid; i < FW; i += nthr) filt[i] = 0u;
  for (uint32_t i = tid; i < N; i += nthr) lab[i] = kInfLabel;
  if (tid < 2) s_min[tid] = kInf;
  if (tid == 0) s_nign = 0u;
  __syncthreads();
  if (s.n_ign) {
    for (uint32_t i = tid; i < s.n_ign; i += nthr) {
      const uint32_t l = s.ign[i];
      if (l == 0xFFFFFFFFu) continue;
      atomicAdd(&s_nign, 1u);
      const uint32_t h = ign_hash(l, fshift);
      atomicOr(&filt[h >> 5], 1u << (h & 31u));
    }
    __syncthreads();
    s.n_ign = s_nign;  // sorted: the real entries come first
    s.filt = filt;
    s.fshift = fshift;
  }
  if (tid == 0) {
    lab[s.node] = static_cast<L>(0);
    near[s.node >> 5] = 1u << (s.node & 31u);
    s_work = 1u;
  }
  __syncthreads();

  const uint32_t delta = a.delta;
  uint32_t T = delta;
  uint32_t mpar = 0;
  for (;;) {
    uint32_t far_min = kInf;
    uint32_t newq = 0;  // pushes of the current group that queued a node
    auto merge = [&](uint32_t u, uint32_t nd, uint32_t cnh, L cl) {
      if constexpr (kNh) {
        for (;;) {
          const uint32_t cd = static_cast<uint32_t>(cl >> 32);
          if (nd > cd) return;
          const unsigned long long nl = nd < cd
              ? ((static_cast<unsigned long long>(nd) << 32) | cnh)
              : (cl | cnh);
          if (nl == cl) return;
          const unsigned long long old = atomicCAS(&lab[u], cl, nl);
          if (old == cl) break;
          cl = old;
        }
      } else {  // distance alone: a strict decrease re-queues
        (void)cnh;
        if (nd >= cl) return;
        if (nd >= atomicMin(&lab[u], nd)) return;
      }
      const uint32_t bit = 1u << (u & 31u);
      if (nd < T) {
        if (!ORH_ASYNC_WAVE_COUNT) atomicAdd(&s_work, 1u);  // counted before the bit is visible
        const uint32_t old = atomicOr(&near[u >> 5], bit);
        atomicAnd(&far[u >> 5], ~bit);
        if (ORH_ASYNC_WAVE_COUNT) newq += (old & bit) ? 0u : 1u;  // reserved by the wave
        else if (old & bit) atomicSub(&s_work, 1u);  // already queued
      } else {
        atomicOr(&far[u >> 5], bit);
        far_min = min(far_min, nd);
      }
    };
    uint32_t w = tid, bits = 0, wbase = 0;
    for (;;) {
      uint32_t vs[G];
      int c = 0;
      while (c < G) {
        while (!bits && w < NB) {
          bits = __hip_atomic_load(&near[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (bits) bits = atomicExch(&near[w], 0u);  // at least the bits seen: only we clear
          wbase = w * 32;
          w += nthr;
        }
        if (!bits) break;
        vs[c++] = wbase + __builtin_ctz(bits);
        bits &= bits - 1;
      }
      if (!bits && w >= NB) w = tid;  // words exhausted: rescan them next time
      if (__builtin_amdgcn_ballot_w64(c > 0) == 0ull) {
        // the whole wave found nothing: done once nothing is queued or claimed
        const uint32_t pending = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&s_work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (pending == 0u) break;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      if (ORH_ASYNC_WAVE_COUNT) {
        // the work count per wave, as in spf_lds16_kernel: the group's
        // possible pushes reserved before its merges, the unused ones and
        // the expanded nodes returned after them
        uint32_t bound = 0;
        newq = 0;
        expand_group<K, G, L>(a, s, lab, vs, c, merge, [&](uint32_t b) {
          bound = b;
          const uint32_t r = wave_sum(b);
          if ((tid & 63u) == 0u && r) atomicAdd(&s_work, r);
        });
        const uint32_t back = wave_sum(c > 0 ? bound - newq + static_cast<uint32_t>(c) : 0u);
        if ((tid & 63u) == 0u && back) atomicSub(&s_work, back);
      } else if (c > 0) {
        expand_group<K, G, L>(a, s, lab, vs, c, merge);
        atomicSub(&s_work, static_cast<uint32_t>(c));
      }
    }
    {
      const uint32_t fm = wave_min(far_min);
      if ((tid & 63u) == 0 && fm != kInf) atomicMin(&s_min[mpar], fm);
    }
    __syncthreads();  // bucket drained everywhere; far bound folded
    const uint32_t m = s_min[mpar];
    if (m == kInf) break;  // far set empty: done (every thread read the same value)
    T = m + delta;
    const uint32_t npar = mpar ^ 1u;
    if (tid == 0) s_min[npar] = kInf;
    __syncthreads();
    uint32_t local_min = kInf, promoted = 0;
    for (uint32_t w2 = tid; w2 < NB; w2 += nthr) {
      uint32_t fb = far[w2], promote = 0u;
      for (uint32_t q = fb; q; q &= q - 1) {
        const uint32_t b = __builtin_ctz(q);
        const uint32_t d = lab_dist(__hip_atomic_load(&lab[w2 * 32 + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (d < T) promote |= 1u << b;
        else local_min = min(local_min, d);
      }
      if (promote) {
        far[w2] = fb & ~promote;
        near[w2] = promote;  // the near set is empty between buckets
        promoted += __builtin_popcount(promote);
      }
    }
    if (ORH_ASYNC_WAVE_COUNT) {
      const uint32_t pr = wave_sum(promoted);
      if ((tid & 63u) == 0u && pr) atomicAdd(&s_work, pr);
    } else if (promoted) {
      atomicAdd(&s_work, promoted);
    }
    const uint32_t wm = wave_min(local_min);
    if ((tid & 63u) == 0 && wm != kInf) atomicMin(&s_min[npar], wm);
    mpar = npar;
    __syncthreads();
  }
  __syncthreads();
  uint32_t* od = a.out_dist + static_cast<size_t>(row) * N;
  uint32_t* on = kNh ? a.out_nh + static_cast<size_t>(row) * N * a.words : nullptr;
  for (uint32_t i = tid; i < N; i += nthr) {
    const L l = __hip_atomic_load(&lab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_nontemporal_store(lab_dist(l), &od[i]);
    if constexpr (kNh) {
      if (a.words == 1) {
        __builtin_nontemporal_store(lab_nh(l), &on[i]);
      } else {
        on[static_cast<size_t>(i) * a.words] = lab_nh(l);
        for (uint32_t k = 1; k < a.words; ++k) on[static_cast<size_t>(i) * a.words + k] = 0u;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// phase 1c'': the asynchronous delta-stepping search with u16 distances in LDS
// ---------------------------------------------------------------------------
// Distances only (KSP2 searches): the async kernel above with its labels moved
// from HBM into LDS as u16 pairs (two nodes per word, lowered by
// compare-and-swap), so the 50k-node WAN of C4 (100 KB of distances + 12.5 KB
// of near / far bitmaps + a 16 KB spill table) keeps a whole search on one
// CU. Relaxation chains then pay LDS latency instead of a global atomic per
// hop; only the edge records (read-only, shared by every search,
// L2-resident) come from memory.
// A u16 entry holds distances 0..0xFFFD inline; 0xFFFF is unreached and
// 0xFFFE "spilled": the node's distance (>= 0xFFFE, the heavy-tailed metrics
// of C4 leave a few such nodes per row) sits in an LDS hash table keyed by
// node id. A spilled node that later gets an inline distance simply drops its
// table entry from use (inline < any spilled value). Only when the table is
// full is a candidate dropped; the row is then exact unless a node ends
// unreached (a dropped candidate exceeds every finite distance its node ends
// with, and a node whose distance needed the table stays unreached), so such
// a row is queued in ovf_rows for the HBM kernel (launch_spf_lds16).
constexpr uint32_t kSpillSlots = 2048, kSpillProbe = 64;
constexpr uint32_t kIgnLds = 1024;  // ignore sets up to this size are searched in LDS
constexpr uint32_t kD16Spill = 0xFFFEu, kD16None = 0xFFFFu;

// The bucket's work count s_work is one LDS word every thread updates: per
// lane, an add per push and a subtract per duplicate and per expanded group
// serialise on that one address. Here a wave reserves, before its group's
// merges, every push the group could make (its nodes' records) with one
// atomic, counts locally the pushes that queued a new node, and returns the
// rest together with its expanded nodes with one more (wave sums over DPP).
// The count still never undercounts: the reservation precedes the wave's
// near-bit updates in its LDS order, and the release follows them.
// A/B of the round-6 search knobs on the C4 batch (profiles/r06/j_ksp2_ab.txt,
// k_ksp2_ab.txt): a thread expanding the nodes it lowered itself instead of
// publishing them (3.0 -> 3.8 ms), a longer s_sleep (no change), 512 threads
// (3.0 -> 4.2 ms), 2 or 8 nodes per group instead of 4 (no change).
#ifndef ORH_LDS16_SLEEP
#define ORH_LDS16_SLEEP 1
#endif
#ifndef ORH_LDS16_G
#define ORH_LDS16_G 4
#endif
#ifndef ORH_LDS16_WAVE_COUNT
#define ORH_LDS16_WAVE_COUNT 1
#endif
template <int K>
__global__ __launch_bounds__(1024) void spf_lds16_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_work, s_min[2], s_nign, s_ovf, s_inf, s_stop;
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  const uint32_t row = a.row_order ? a.row_order[blockIdx.x] : blockIdx.x;
  if (a.row_mask && !a.row_mask[row]) return;
  constexpr int G = K <= 4 ? ORH_LDS16_G : 2;  // nodes a thread expands together
  const uint32_t DWp = ((N + 1) / 2 + 3) & ~3u;
  uint32_t stop_lo = 0, stop_hi = 0;  // this row's target nodes (early stop)
  if (a.stop_ptr) {
    stop_lo = a.stop_ptr[row];
    stop_hi = a.stop_ptr[row + 1];
  }
  uint32_t* dist = lds;  // node u: bits 16 (u & 1) .. of word u / 2
  uint32_t* near = lds + DWp;
  uint32_t* far = near + NB;
  uint32_t* filt = far + NB;
  uint32_t FW = 1;
  while (2 * FW <= min(NB, 256u)) FW *= 2;
  uint32_t* sp_key = filt + FW;  // spill table: node id (~0u empty) | distance
  uint32_t* sp_val = sp_key + kSpillSlots;
  const uint32_t fshift = 32u - (5u + static_cast<uint32_t>(__builtin_ctz(FW)));
  Src s(a, row);
  for (uint32_t i = tid; i < DWp; i += nthr) dist[i] = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < 2 * NB; i += nthr) near[i] = 0u;
  for (uint32_t i = tid; i < 2 * kSpillSlots; i += nthr) sp_key[i] = ~0u;
  if (s.n_ign)
    for (uint32_t i = tid; i < FW; i += nthr) filt[i] = 0u;
  if (tid < 2) s_min[tid] = kInf;
  if (tid == 0) {
    s_nign = 0u;
    s_ovf = 0u;
    s_inf = 0u;
    s_stop = 0u;
  }
  __syncthreads();
  if (s.n_ign) {
    for (uint32_t i = tid; i < s.n_ign; i += nthr) {
      const uint32_t l = s.ign[i];
      if (l == 0xFFFFFFFFu) continue;
      atomicAdd(&s_nign, 1u);
      const uint32_t h = ign_hash(l, fshift);
      atomicOr(&filt[h >> 5], 1u << (h & 31u));
    }
    __syncthreads();
    s.n_ign = s_nign;  // sorted: the real entries come first
    s.filt = filt;
    s.fshift = fshift;
    // the set itself into LDS too: a filter hit (every relaxation of an
    // ignored link - KSP2's k = 2 searches start on the k = 1 path) then
    // binary-searches LDS instead of a chain of dependent global loads
#ifndef ORH_LDS16_IGN_GLOBAL  // (A/B builds: the set stays in global memory)
    if (s.n_ign <= kIgnLds) {
#else
    if (false) {
#endif
      uint32_t* ign_lds = sp_key + 2 * kSpillSlots;
      for (uint32_t i = tid; i < s.n_ign; i += nthr) ign_lds[i] = s.ign[i];
      __syncthreads();
      s.ign = ign_lds;
    }
  }
  if (tid == 0) {
    dist[s.node >> 1] &= ~(0xFFFFu << ((s.node & 1u) * 16u));
    near[s.node >> 5] = 1u << (s.node & 31u);
    s_work = 1u;
  }
  __syncthreads();
  // spill slot of u (inserted when `insert`), or -1: absent / table full
  auto sp_slot = [&](uint32_t u, bool insert) -> int {
    uint32_t h = (u * 0x9E3779B1u) >> (32u - 11u);  // 2048 slots
    for (uint32_t p = 0; p < kSpillProbe; ++p, h = (h + 1u) & (kSpillSlots - 1u)) {
      const uint32_t k = sp_key[h];
      if (k == u) return static_cast<int>(h);
      if (k != ~0u) continue;
      if (!insert) return -1;
      const uint32_t prev = atomicCAS(&sp_key[h], ~0u, u);
      if (prev == ~0u || prev == u) return static_cast<int>(h);
    }
    return -1;
  };
  // distance of u from its u16 entry e (kInf: unreached)
  auto eff = [&](uint32_t u, uint32_t e) -> uint32_t {
    if (e < kD16Spill) return e;
    if (e == kD16None) return kInf;
    const int sl = sp_slot(u, false);
    return sl < 0 ? kInf : sp_val[sl];
  };
  auto get = [&](uint32_t u) { return eff(u, (dist[u >> 1] >> ((u & 1u) * 16u)) & 0xFFFFu); };

  const uint32_t delta = a.delta;
  uint32_t T = delta;
  uint32_t mpar = 0;
  uint32_t stop_m = 0;  // > 0: stopped with every node at distance <= stop_m final
  bool ovf = false;
  const bool lane0 = (tid & 63u) == 0u;
  for (;;) {
    uint32_t far_min = kInf;
    uint32_t newq = 0;  // pushes of the current group that queued a node
    // lower u to nd, starting from the word w as read; queue it if lowered
    auto merge = [&](uint32_t u, uint32_t nd, uint32_t w) {
      const uint32_t sh = (u & 1u) * 16u;
      uint32_t e = (w >> sh) & 0xFFFFu;
      if (nd < kD16Spill) {  // inline: below any spilled distance
        for (;;) {
          if (e < kD16Spill && nd >= e) return;
          const uint32_t nw = (w & ~(0xFFFFu << sh)) | (nd << sh);
          const uint32_t prev = atomicCAS(&dist[u >> 1], w, nw);
          if (prev == w) break;
          w = prev;
          e = (w >> sh) & 0xFFFFu;
        }
      } else {
        if (e < kD16Spill) return;  // an inline distance is smaller
        const int sl = sp_slot(u, true);
        if (sl < 0) {  // table full: dropped
          ovf = true;
          return;
        }
        if (nd >= atomicMin(&sp_val[sl], nd)) return;
        while (e == kD16None) {  // mark the entry spilled (unless it went inline meanwhile)
          const uint32_t nw = w & ~(0x1u << sh);  // 0xFFFF -> 0xFFFE
          const uint32_t prev = atomicCAS(&dist[u >> 1], w, nw);
          if (prev == w) break;
          w = prev;
          e = (w >> sh) & 0xFFFFu;
        }
        if (e < kD16Spill) return;
      }
      const uint32_t bit = 1u << (u & 31u);
      if (nd < T) {
        if (!ORH_LDS16_WAVE_COUNT) atomicAdd(&s_work, 1u);  // counted before the bit is visible
        const uint32_t old = atomicOr(&near[u >> 5], bit);
        atomicAnd(&far[u >> 5], ~bit);
        if (ORH_LDS16_WAVE_COUNT) newq += (old & bit) ? 0u : 1u;  // reserved by the wave
        else if (old & bit) atomicSub(&s_work, 1u);  // already queued
      } else {
        atomicOr(&far[u >> 5], bit);
        far_min = min(far_min, nd);
      }
    };
    uint32_t wi = tid, bits = 0, wbase = 0;
    for (;;) {
      uint32_t vs[G];
      int c = 0;
      while (c < G) {
        while (!bits && wi < NB) {
          bits = __hip_atomic_load(&near[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (bits) bits = atomicExch(&near[wi], 0u);  // at least the bits seen: only we clear
          wbase = wi * 32;
          wi += nthr;
        }
        if (!bits) break;
        vs[c++] = wbase + __builtin_ctz(bits);
        bits &= bits - 1;
      }
      if (!bits && wi >= NB) wi = tid;  // words exhausted: rescan them next time
      if (__builtin_amdgcn_ballot_w64(c > 0) == 0ull) {
        const uint32_t pending = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&s_work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (pending == 0u) break;
        __builtin_amdgcn_s_sleep(ORH_LDS16_SLEEP);
        continue;
      }
      // the group's records in flight together, then the neighbours' words
      uint2 rec[G][K];
      uint32_t lk[G][K];  // link ids (ignore sets), loaded with the records
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (g < c) load_recs<K>(a, vs[g], rec[g]);
#pragma unroll
        for (int j = 0; j < K; ++j) lk[g][j] = (g < c && s.n_ign) ? a.link[vs[g] * K + j] : 0u;
      }
      // every push the group can make (its records, continuation lists
      // included), reserved in s_work by the wave before any of its merges
      uint32_t bound = 0;
      if (ORH_LDS16_WAVE_COUNT) {
#pragma unroll
        for (int g = 0; g < G; ++g)
          if (g < c) bound += K + ((rec[g][K - 1].x & ORH_REC_CONT) ? rec[g][K - 1].y : 0u);
        const uint32_t r = wave_sum(bound);
        if (lane0 && r) atomicAdd(&s_work, r);
      }
      newq = 0;
      if (c > 0) {
        uint32_t dv[G], nw[G][K];
        bool ok[G][K];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          dv[g] = g < c ? get(vs[g]) : 0u;
          const bool transit = g < c && (vs[g] == s.node || !(rec[g][0].x & ORH_REC_ROW_OVL));
#pragma unroll
          for (int j = 0; j < K; ++j) {
            ok[g][j] = transit && live_link(s, rec[g][j], lk[g][j]);
            nw[g][j] = ok[g][j] ? dist[(rec[g][j].x & ORH_REC_COL_MASK) >> 1] : 0u;
          }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if (g >= c) break;
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (ok[g][j])
              merge(rec[g][j].x & ORH_REC_COL_MASK, dv[g] + (a.use_link_metric ? rec[g][j].y : 1u), nw[g][j]);
          const uint2 last = rec[g][K - 1];
          const bool transit = vs[g] == s.node || !(rec[g][0].x & ORH_REC_ROW_OVL);
          if (transit && (last.x & ORH_REC_CONT)) {
            const uint32_t start = last.x & ORH_REC_COL_MASK;
            for (uint32_t q = 0; q < last.y; ++q) {
              const uint2 r = a.recs[start + q];
              if (!live(a, s, r, start + q)) continue;
              const uint32_t u = r.x & ORH_REC_COL_MASK;
              merge(u, dv[g] + (a.use_link_metric ? r.y : 1u), dist[u >> 1]);
            }
          }
        }
        if (!ORH_LDS16_WAVE_COUNT) atomicSub(&s_work, static_cast<uint32_t>(c));
      }
      if (ORH_LDS16_WAVE_COUNT) {
        // the unused reservation and the expanded nodes, after the merges
        const uint32_t back = wave_sum(c > 0 ? bound - newq + static_cast<uint32_t>(c) : 0u);
        if (lane0 && back) atomicSub(&s_work, back);
      }
    }
    {
      const uint32_t fm = wave_min(far_min);
      if ((tid & 63u) == 0 && fm != kInf) atomicMin(&s_min[mpar], fm);
    }
    __syncthreads();  // bucket drained everywhere; far bound folded
    const uint32_t m = s_min[mpar];
    if (m == kInf) break;  // far set empty: done
    T = m + delta;
    const uint32_t npar = mpar ^ 1u;
    if (tid == 0) {
      s_min[npar] = kInf;
      // every node at distance <= m is final (m: the least unsettled one);
      // once the targets are among them, no trace to them reads further
      if (stop_hi > stop_lo) {
        bool done = true;
        for (uint32_t q = stop_lo; q < stop_hi && done; ++q) done = get(a.stop_nodes[q]) <= m;
        if (done) s_stop = m;
      }
    }
    __syncthreads();
    if (s_stop) {
      stop_m = s_stop;
      break;
    }
    uint32_t local_min = kInf, promoted = 0;
    for (uint32_t w2 = tid; w2 < NB; w2 += nthr) {
      const uint32_t fb = far[w2];
      uint32_t promote = 0u;
      for (uint32_t q = fb; q; q &= q - 1) {
        const uint32_t b = __builtin_ctz(q);
        const uint32_t d = get(w2 * 32 + b);
        if (d < T) promote |= 1u << b;
        else local_min = min(local_min, d);
      }
      if (promote) {
        far[w2] = fb & ~promote;
        near[w2] = promote;  // the near set is empty between buckets
        promoted += __builtin_popcount(promote);
      }
    }
    if (ORH_LDS16_WAVE_COUNT) {
      const uint32_t pr = wave_sum(promoted);
      if (lane0 && pr) atomicAdd(&s_work, pr);
    } else if (promoted) {
      atomicAdd(&s_work, promoted);
    }
    const uint32_t wm = wave_min(local_min);
    if ((tid & 63u) == 0 && wm != kInf) atomicMin(&s_min[npar], wm);
    mpar = npar;
    __syncthreads();
  }
  if (ovf) s_ovf = 1u;
  __syncthreads();
  uint32_t* od = dist_row(a.out_dist, a.scratch, a.n_out, N, row);
  bool inf = false;
  for (uint32_t i = tid; i < N; i += nthr) {
    const uint32_t d = get(i);
    inf |= d == kInf;
    __builtin_nontemporal_store(d, &od[i]);
  }
  // exact unless a node ended unreached; stopped early, exact up to stop_m
  // unless the spill table overflowed below it (dropped candidates are all
  // >= 0xFFFE): otherwise the HBM kernel redoes the row
  if (s_ovf && !(stop_m && stop_m < kD16Spill)) {
    if (inf || stop_m) s_inf = 1u;
    __syncthreads();
    if (tid == 0 && s_inf) {
      const uint32_t k = atomicAdd(&a.ovf_rows[0], 1u);
      a.ovf_rows[1 + k] = row;
    }
  }
}

// ---------------------------------------------------------------------------
// phase 1c''': general metrics, first hops fused, labels in LDS (kLdsNh)
// ---------------------------------------------------------------------------
// The asynchronous delta-stepping of spf_global_nh_async_kernel with its
// {dist, first-hop mask} labels in LDS instead of HBM: a weighted graph that
// fits (N = 10,000: 40 KB packed) is searched by one workgroup per source
// with no global atomics and no second phase - the first hops ride along the
// search as in runSpf itself (LinkState.cpp:857-873): a smaller candidate
// replaces a label, an equal one ORs its mask in (and re-queues the node so
// the new bits reach its successors). The fixpoint is order-independent, so
// the rows are the HBM kernel's bit for bit.
// kPacked: a u32 label {dist (16 bits, hi) | mask (16 bits, lo)}, for sources
// with <= 16 distinct neighbours; a candidate distance >= 0xFFFF cannot be
// held, so the row is appended to a.ovf_rows and written by the u64 form
// (launch_spf_lds_nh runs it over that list). Else a u64 label {dist (32) |
// mask (32)} as in the HBM kernel.
template <int K, bool kPacked>
__global__ __launch_bounds__(1024) void spf_lds_nh_kernel(SpfArgs a) {
  typedef typename std::conditional<kPacked, uint32_t, unsigned long long>::type L;
  constexpr uint32_t kSh = kPacked ? 16u : 32u;
  constexpr uint32_t kDInf = kPacked ? 0xFFFFu : 0xFFFFFFFFu;  // the unreached distance
  constexpr L kInfLabel = static_cast<L>(static_cast<L>(kDInf) << kSh);
  constexpr L kMaskBits = static_cast<L>((static_cast<L>(1) << kSh) - 1u);
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_work, s_min[2], s_nign, s_ovf;
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  if (a.row_list && blockIdx.x >= *a.row_count) return;
  const uint32_t row = a.row_list ? a.row_list[blockIdx.x] : blockIdx.x;
  constexpr int G = K <= 4 ? 4 : 2;
  L* lab = reinterpret_cast<L*>(lds);
  const uint32_t lab_words = kPacked ? ((N + 1u) & ~1u) : 2u * N;  // keeps near 8-byte aligned
  uint32_t* near = lds + lab_words;
  uint32_t* far = near + NB;
  uint32_t* filt = far + NB;
  uint32_t FW = 1;
  while (2 * FW <= min(NB, 256u)) FW *= 2;
  const uint32_t fshift = 32u - (5u + static_cast<uint32_t>(__builtin_ctz(FW)));
  Src s(a, row);
  for (uint32_t i = tid; i < N; i += nthr) lab[i] = kInfLabel;
  for (uint32_t i = tid; i < 2 * NB; i += nthr) near[i] = 0u;
  if (s.n_ign)
    for (uint32_t i = tid; i < FW; i += nthr) filt[i] = 0u;
  if (tid < 2) s_min[tid] = kInf;
  if (tid == 0) {
    s_nign = 0u;
    s_ovf = 0u;
  }
  __syncthreads();
  if (s.n_ign) {
    for (uint32_t i = tid; i < s.n_ign; i += nthr) {
      const uint32_t l = s.ign[i];
      if (l == 0xFFFFFFFFu) continue;
      atomicAdd(&s_nign, 1u);
      const uint32_t h = ign_hash(l, fshift);
      atomicOr(&filt[h >> 5], 1u << (h & 31u));
    }
    __syncthreads();
    s.n_ign = s_nign;  // sorted: the real entries come first
    s.filt = filt;
    s.fshift = fshift;
  }
  if (tid == 0) {
    lab[s.node] = static_cast<L>(0);
    near[s.node >> 5] = 1u << (s.node & 31u);
    s_work = 1u;
  }
  __syncthreads();

  const uint32_t delta = a.delta;
  uint32_t T = delta;
  uint32_t mpar = 0;
  bool ovf = false;
  for (;;) {
    uint32_t far_min = kInf;
    // merge the candidate {nd, cnh} into u's label (cl: as loaded); re-queue
    // u if the label changed
    auto merge = [&](uint32_t u, uint32_t nd, uint32_t cnh, L cl) {
      if (kPacked && nd >= kDInf) {  // not representable: the u64 form redoes the row
        ovf = true;
        return;
      }
      for (;;) {
        const uint32_t cd = static_cast<uint32_t>(cl >> kSh);
        if (nd > cd) return;
        const L nl = nd < cd ? static_cast<L>((static_cast<L>(nd) << kSh) | cnh) : static_cast<L>(cl | cnh);
        if (nl == cl) return;
        const L old = atomicCAS(&lab[u], cl, nl);
        if (old == cl) break;
        cl = old;
      }
      const uint32_t bit = 1u << (u & 31u);
      if (nd < T) {
        atomicAdd(&s_work, 1u);  // counted before the bit is visible
        const uint32_t old = atomicOr(&near[u >> 5], bit);
        atomicAnd(&far[u >> 5], ~bit);
        if (old & bit) atomicSub(&s_work, 1u);  // already queued
      } else {
        atomicOr(&far[u >> 5], bit);
        far_min = min(far_min, nd);
      }
    };
    uint32_t wi = tid, bits = 0, wbase = 0;
    for (;;) {
      uint32_t vs[G];
      int c = 0;
      while (c < G) {
        while (!bits && wi < NB) {
          bits = __hip_atomic_load(&near[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (bits) bits = atomicExch(&near[wi], 0u);  // at least the bits seen: only we clear
          wbase = wi * 32;
          wi += nthr;
        }
        if (!bits) break;
        vs[c++] = wbase + __builtin_ctz(bits);
        bits &= bits - 1;
      }
      if (!bits && wi >= NB) wi = tid;  // words exhausted: rescan them next time
      if (__builtin_amdgcn_ballot_w64(c > 0) == 0ull) {
        const uint32_t pending = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&s_work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (pending == 0u) break;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      if (c > 0) {
        // the group's records in flight together, then the labels
        uint2 rec[G][K];
        uint32_t lk[G][K];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if (g < c) load_recs<K>(a, vs[g], rec[g]);
#pragma unroll
          for (int j = 0; j < K; ++j) lk[g][j] = (g < c && s.n_ign) ? a.link[vs[g] * K + j] : 0u;
        }
        L lv[G], cl[G][K];
        bool ok[G][K];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          lv[g] = g < c ? lab[vs[g]] : static_cast<L>(0);
          const bool transit = g < c && (vs[g] == s.node || !(rec[g][0].x & ORH_REC_ROW_OVL));
#pragma unroll
          for (int j = 0; j < K; ++j) {
            ok[g][j] = transit && live_link(s, rec[g][j], lk[g][j]);
            cl[g][j] = ok[g][j] ? lab[rec[g][j].x & ORH_REC_COL_MASK] : static_cast<L>(0);
          }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if (g >= c) break;
          const uint32_t v = vs[g];
          const uint32_t dv = static_cast<uint32_t>(lv[g] >> kSh);
          const uint32_t nhv = static_cast<uint32_t>(lv[g] & kMaskBits);
          const bool from_src = v == s.node;
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (ok[g][j])
              merge(rec[g][j].x & ORH_REC_COL_MASK, dv + (a.use_link_metric ? rec[g][j].y : 1u),
                    from_src ? (1u << a.rank_out[v * K + j]) : nhv, cl[g][j]);
          const uint2 last = rec[g][K - 1];
          const bool transit = from_src || !(rec[g][0].x & ORH_REC_ROW_OVL);
          if (transit && (last.x & ORH_REC_CONT)) {
            const uint32_t start = last.x & ORH_REC_COL_MASK;
            for (uint32_t q = 0; q < last.y; ++q) {
              const uint2 r = a.recs[start + q];
              if (!live(a, s, r, start + q)) continue;
              const uint32_t u = r.x & ORH_REC_COL_MASK;
              merge(u, dv + (a.use_link_metric ? r.y : 1u), from_src ? (1u << a.rank_out[start + q]) : nhv,
                    lab[u]);
            }
          }
        }
        atomicSub(&s_work, static_cast<uint32_t>(c));
      }
    }
    {
      const uint32_t fm = wave_min(far_min);
      if ((tid & 63u) == 0 && fm != kInf) atomicMin(&s_min[mpar], fm);
    }
    __syncthreads();  // bucket drained everywhere; far bound folded
    const uint32_t m = s_min[mpar];
    if (m == kInf) break;  // far set empty: done
    T = m + delta;
    const uint32_t npar = mpar ^ 1u;
    if (tid == 0) s_min[npar] = kInf;
    __syncthreads();
    uint32_t local_min = kInf, promoted = 0;
    for (uint32_t w2 = tid; w2 < NB; w2 += nthr) {
      const uint32_t fb = far[w2];
      uint32_t promote = 0u;
      for (uint32_t q = fb; q; q &= q - 1) {
        const uint32_t b = __builtin_ctz(q);
        const uint32_t d = static_cast<uint32_t>(lab[w2 * 32 + b] >> kSh);
        if (d < T) promote |= 1u << b;
        else local_min = min(local_min, d);
      }
      if (promote) {
        far[w2] = fb & ~promote;
        near[w2] = promote;  // the near set is empty between buckets
        promoted += __builtin_popcount(promote);
      }
    }
    if (promoted) atomicAdd(&s_work, promoted);
    const uint32_t wm = wave_min(local_min);
    if ((tid & 63u) == 0 && wm != kInf) atomicMin(&s_min[npar], wm);
    mpar = npar;
    __syncthreads();
  }
  if (kPacked && ovf) s_ovf = 1u;
  __syncthreads();
  if (kPacked && s_ovf) {  // the u64 form writes this row
    if (tid == 0) {
      const uint32_t k = atomicAdd(&a.ovf_rows[0], 1u);
      a.ovf_rows[1 + k] = row;
    }
    return;
  }
  // labels -> dist row (kInf = unreachable) and first-hop row, coalesced (a
  // neighbour row of a two-phase plan, row >= n_out: the distances alone)
  uint32_t* od = dist_row(a.out_dist, a.scratch, a.n_out, N, row);
  uint32_t* on = row < a.n_out ? a.out_nh + static_cast<size_t>(row) * N * a.words : nullptr;
  for (uint32_t i = tid; i < N; i += nthr) {
    const L l = lab[i];
    const uint32_t d = static_cast<uint32_t>(l >> kSh);
    __builtin_nontemporal_store(d == kDInf ? kInf : d, &od[i]);
    const uint32_t m = static_cast<uint32_t>(l & kMaskBits);
    if (!on) continue;
    if (a.words == 1) {
      __builtin_nontemporal_store(m, &on[i]);
    } else {
      on[static_cast<size_t>(i) * a.words] = m;
      for (uint32_t k = 1; k < a.words; ++k) on[static_cast<size_t>(i) * a.words + k] = 0u;
    }
  }
}

// ---------------------------------------------------------------------------
// phase 1d: general metrics, many sources: multi-source Bellman-Ford in LDS
// ---------------------------------------------------------------------------
// The weighted counterpart of spf_msbfs_kernel. A workgroup holds the u16
// distances of 4 sources for every node in LDS (8 bytes per node, two packed
// u16 pairs) and relaxes them in pull form: per round each thread recomputes
// its own nodes, d(v) = min(d(v), min over in-links (u, w) of d(u) + w), for
// the 4 sources at once with packed 16-bit adds (saturating: 0xFFFF stays
// "unreached") and packed minima. The in-links of a thread's nodes sit in
// its registers ({u, w(u -> v)} per slot, a_wms layout, Cuthill-McKee ids),
// so a round touches no global memory. Writes go in place (any value read
// is a path length, so the fixpoint is the same in any order) and a round
// without a change anywhere ends the search: the labels are then the
// shortest distances of runSpf (LinkState.cpp:808-882) for positive metrics.
// No transit through an overloaded node: a slot whose u is overloaded is dead,
// except that an overloaded source still reaches its own neighbours (applied
// once before the rounds). First hops: phase 2 over the u32 rows.
// A label past 0xFFFF - 1 - max metric could hide a distance that does not fit
// 16 bits: such a batch lists its rows in a.ovf_rows and the caller redoes
// them (spf_lds_nh_kernel, u64 labels, fused first hops - phase 2 then
// recomputes the same first hops).
template <int J, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < J) {
    f(std::integral_constant<int, I>{});
    static_for<J, I + 1>(f);
  }
}
constexpr uint32_t kWmsOvl = 0x80000000u;  // slot flag: u is overloaded

// packed u16 pairs: saturating add (v_pk_add_u16 clamp: 0xFFFF stays
// "unreached") and minimum (v_pk_min_u16)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ inline uint32_t pk_add_sat_u16(uint32_t a, uint32_t b) {
  const u16x2 r = __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
  return __builtin_bit_cast(uint32_t, r);
}
__device__ inline uint32_t pk_min_u16(uint32_t a, uint32_t b) {
  const u16x2 r = __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
  return __builtin_bit_cast(uint32_t, r);
}

// ORH_WMS_OCC2 (A/B builds): J <= 10 capped at 64 VGPRs so two 1,024-thread
// batches share a CU (their LDS, 2 x 80 KB, fits). Measured slower on C2w
// (profiles/r06/g_c2w_*), so one batch per CU
#ifdef ORH_WMS_OCC2
#define ORH_WMS_ATTR __attribute__((amdgpu_waves_per_eu(J <= 10 ? 8 : 1)))
#else
#define ORH_WMS_ATTR
#endif
// S = 4 or 8 sources per batch: a node's labels are S u16 in S / 2 dwords
// (8: 16 B per node, so N <= ~10,200 fits one batch per CU)
template <int K, int J, int S>
__global__ __launch_bounds__(1024) ORH_WMS_ATTR void spf_wms_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr uint32_t W = S / 2;  // dwords per node
  typedef uint32_t DV __attribute__((ext_vector_type(W)));
  const uint32_t N = a.n_nodes;
  const uint32_t tid = threadIdx.x, B = blockDim.x;
  const uint32_t b0 = blockIdx.x * S;
  const uint32_t nsrc = min(static_cast<uint32_t>(S), a.n_rows - b0);
  __shared__ uint32_t s_prog[3], s_ovf;
  DV* D = reinterpret_cast<DV*>(lds);  // [N + 1]; D[N] stays unreached
  // kSplit (ORH_WMS_SPLIT builds, S = 8): sources 0-3 and 4-7 in two arrays
  // of 8-byte entries, read by two ds_read_b64 instead of one ds_read_b128
  // (whose 16-lane groups take a conflict at every shift of the neighbour
  // offset inside a wave)
#ifdef ORH_WMS_SPLIT
  constexpr bool kSplit = S == 8;
#else
  constexpr bool kSplit = false;
#endif
  uint2* H0 = reinterpret_cast<uint2*>(lds);
  uint2* H1 = H0 + (N + 1);
  auto ld = [&](uint32_t u) -> DV {
    if constexpr (kSplit) {
      const uint2 x = H0[u], y = H1[u];
      DV r;
      r[0] = x.x; r[1] = x.y; r[2 % W] = y.x; r[3 % W] = y.y;
      return r;
    } else {
      return D[u];
    }
  };
  auto st = [&](uint32_t u, const DV& v) {
    if constexpr (kSplit) {
      H0[u] = make_uint2(v[0], v[1]);
      H1[u] = make_uint2(v[2 % W], v[3 % W]);
    } else {
      D[u] = v;
    }
  };
  {
    DV none;
#pragma unroll
    for (uint32_t q = 0; q < W; ++q) none[q] = ~0u;
    for (uint32_t i = tid; i <= N; i += B) st(i, none);
  }
  if (tid < 3) s_prog[tid] = 0u;
  if (tid == 0) s_ovf = 0u;
  __syncthreads();
  if (tid < nsrc) {  // sources may repeat: clear each lane's half alone
    const uint32_t src = a.dev_of[a.srcs[a.order[b0 + tid]]];
    uint32_t* w = kSplit ? reinterpret_cast<uint32_t*>((tid >> 2) ? H1 + src : H0 + src) + ((tid >> 1) & 1u)
                         : reinterpret_cast<uint32_t*>(D + src) + (tid >> 1);
    atomicAnd(w, (tid & 1u) ? 0x0000FFFFu : 0xFFFF0000u);
  }
  __syncthreads();
  // the in-link slots of the owned nodes: {u (16 bits) | w (15 bits) << 16 |
  // kWmsOvl}; an unused slot (no link, link down) reads u = N, the entry that
  // stays unreached
  // node of (this thread, j): band schedule - wave w owns chunks [w J, (w +
  // 1) J) - or interleaved - chunk j * waves + w
  const bool band = a.wms_band != 0u;
  const uint32_t wave = tid >> 6;
  const uint32_t lane = tid & 63u;
  auto node_of = [&](uint32_t j) { return band ? (wave * J + j) * 64u + lane : j * B + tid; };
  uint32_t slot[J][K];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t v = node_of(j);
#pragma unroll
    for (int k = 0; k < K; ++k) slot[j][k] = v < N ? a.wms_slots[static_cast<size_t>(v) * K + k] : N;
  }
  // an overloaded source reaches its neighbours and no further: a slot whose
  // u is overloaded contributes w to the lanes where u is the source (label
  // 0: only a source holds it, and this pass writes nothing below 1), once,
  // and is dead from then on like every other slot of an overloaded node
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t v = node_of(j);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!(slot[j][k] & kWmsOvl)) continue;
      const uint32_t u = slot[j][k] & 0xFFFFu, w = (slot[j][k] >> 16) & 0x7FFFu;
      slot[j][k] = N;
      const DV du = ld(u);
      DV d = ld(v);  // v < N: a slot of a padding node is never flagged
#pragma unroll
      for (uint32_t q = 0; q < W; ++q) {
        const uint32_t lo = (du[q] & 0xFFFFu) == 0u ? w : 0xFFFFu, hi = (du[q] >> 16) == 0u ? w : 0xFFFFu;
        d[q] = pk_min_u16(d[q], lo | (hi << 16));
      }
      st(v, d);
    }
  }
  __syncthreads();
  // activity: a wave's slice j is the 64-node chunk c = v / 64 (Cuthill-McKee
  // ids). A chunk whose nodes changed in round r sets its bit in chg[r % 3];
  // in round r + 1 a slice is recomputed only if a chunk within the layout
  // bandwidth of it (where all its in-links come from) changed in round r -
  // a node whose in-neighbours all kept their labels since it was last
  // recomputed cannot change. (A change later in the same round is seen in
  // the next one.) Three rotating bitmaps: one read, one written, one cleared.
  // a.ms_bw = 0: every slice every round (ORH_WMS_SKIP, orh_spf_run)
  const uint32_t nchunk = (N + 63) / 64, cw = (nchunk + 31) / 32;
  uint32_t* chg = reinterpret_cast<uint32_t*>(D + N + 1);  // [3][cw] (kSplit: H1 + N + 1, the same bytes)
  for (uint32_t i = tid; i < 3 * cw; i += B) chg[i] = 0u;
  const uint32_t bw = a.ms_bw;
  __syncthreads();
  // (the owner keeping its J labels in registers instead of reading its own
  // back from LDS measured slower: C2w distances 3.65 vs 3.55 ms,
  // profiles/r06/x_wms_ab.txt; two forward/backward passes per round 3.72)
  for (uint32_t round = 1;; ++round) {
    int prog = 0;
    const uint32_t* prev = chg + ((round + 2u) % 3u) * cw;
    uint32_t* cur = chg + (round % 3u) * cw;
    if (tid < cw) chg[((round + 1u) % 3u) * cw + tid] = 0u;  // read in round - 1, written in round + 1
    // back: the band schedule's backward sweep, which also sees the chunks
    // this round's forward sweep changed
    auto relax = [&](auto jc, bool back) {
      constexpr int j = decltype(jc)::value;
      const uint32_t v = node_of(j);
      const uint32_t c = __builtin_amdgcn_readfirstlane(band ? wave * J + j : j * (B >> 6) + wave);  // this slice's chunk
      if ((round > 1 || back) && bw) {
        const uint32_t lo = c * 64u > bw ? (c * 64u - bw) >> 6 : 0u;
        const uint32_t hi = min(nchunk - 1u, (c * 64u + 63u + bw) >> 6);
        bool act = false;
        for (uint32_t w = lo >> 5; w <= (hi >> 5) && !act; ++w) {
          uint32_t m = (round > 1 ? prev[w] : 0u) | (back ? cur[w] : 0u);
          if (w == (lo >> 5)) m &= ~0u << (lo & 31u);
          if (w == (hi >> 5) && (hi & 31u) != 31u) m &= (2u << (hi & 31u)) - 1u;
          act = m != 0u;
        }
        if (!act) return;
      }
      if (v >= N) return;
      // opaque per round: the addresses and replicated weights are derived
      // again each time instead of held in J * K more registers
#pragma unroll
      for (int k = 0; k < K; ++k) asm volatile("" : "+v"(slot[j][k]));
      DV du[K];
#pragma unroll
      for (int k = 0; k < K; ++k) du[k] = ld(slot[j][k] & 0xFFFFu);
      const DV own = ld(v);
      DV acc = own;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        // {w, w}: the high half twice (an unused slot: w = 0 on the unreached entry)
        const uint32_t wr = __builtin_amdgcn_perm(slot[j][k], slot[j][k], 0x03020302u);
#pragma unroll
        for (uint32_t q = 0; q < W; ++q) acc[q] = pk_min_u16(acc[q], pk_add_sat_u16(du[k][q], wr));
      }
      bool changed = false;
#pragma unroll
      for (uint32_t q = 0; q < W; ++q) changed |= acc[q] != own[q];
      if (changed) {
        st(v, acc);
        prog = 1;
      }
      if (__builtin_amdgcn_ballot_w64(changed) && (tid & 63u) == 0u) atomicOr(&cur[c >> 5], 1u << (c & 31u));
    };
    // (walking the slices backwards in odd rounds, for paths against the
    // slice order, measured no faster: profiles/r06/h_c2w_variants.txt)
#ifndef ORH_WMS_PASSES
#define ORH_WMS_PASSES 1  // forward + backward sweeps of a band per round (A/B builds)
#endif
    for (int pass = 0; pass < (band ? ORH_WMS_PASSES : 1); ++pass) {
      static_for<J>([&](auto jc) { relax(jc, pass > 0); });
      if (band)  // and back: a band passes its changes both ways in one round
        static_for<J>([&](auto jc) { relax(std::integral_constant<int, J - 1 - decltype(jc)::value>{}, true); });
    }
    if (prog) s_prog[round % 3u] = 1u;
    lds_barrier();
    if (!s_prog[round % 3u]) break;
    if (tid == 0) s_prog[(round + 2u) % 3u] = 0u;
  }
  // rows out in host order (coalesced), a u16 label widened to u32; a label
  // within max metric of 0xFFFF may stand for a distance that did not fit
  const uint32_t lim = a.wms_limit;
  uint32_t* out[S];
#pragma unroll
  for (uint32_t k = 0; k < S; ++k)
    out[k] = k < nsrc ? dist_row(a.out_dist, a.scratch, a.n_out, N, a.order[b0 + k]) : nullptr;
  bool ovf = false;
  for (uint32_t i = tid; i < N; i += B) {
    const DV d = ld(a.dev_of[i]);
#pragma unroll
    for (uint32_t k = 0; k < S; ++k) {
      if (k >= nsrc) break;
      const uint32_t l = (d[k / 2] >> ((k & 1u) * 16u)) & 0xFFFFu;
      ovf |= l != 0xFFFFu && l > lim;
      __builtin_nontemporal_store(l == 0xFFFFu ? kInf : l, &out[k][i]);
    }
  }
  if (ovf) s_ovf = 1u;
  __syncthreads();
  if (s_ovf && tid < nsrc) {
    const uint32_t k = atomicAdd(&a.ovf_rows[0], 1u);
    a.ovf_rows[1 + k] = a.order[b0 + tid];
  }
}

size_t wms_lds_bytes(uint32_t n_nodes, uint32_t sources) {
  const size_t cw = (static_cast<size_t>(n_nodes) + 63) / 64 / 32 + 1;
  return (static_cast<size_t>(n_nodes) + 1) * 2 * sources + 3 * cw * 4;  // labels, then the chunk-change bitmaps
}

size_t lds_nh_bytes(uint32_t n_nodes, bool packed) {
  const size_t nb = (n_nodes + 31) / 32;
  size_t fw = 1;
  while (2 * fw <= std::min<size_t>(nb, 256)) fw *= 2;
  const size_t lab = packed ? ((n_nodes + 1) & ~size_t{1}) : 2 * static_cast<size_t>(n_nodes);
  return 4 * (lab + 2 * nb + fw);
}

template <int K>
__global__ __launch_bounds__(1024) void spf_global_nh_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_flag[3];
  __shared__ uint32_t s_min[2];
  const uint32_t N = a.n_nodes;
  const uint32_t NB = (N + 31) >> 5;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  if (a.row_list && blockIdx.x >= *a.row_count) return;
  const uint32_t row = a.row_list ? a.row_list[blockIdx.x] : blockIdx.x;
  constexpr unsigned long long kInfLabel = 0xFFFFFFFF00000000ull;
  // frontier nodes a thread expands together: their record, label and
  // neighbour-label loads are in flight at once (one round trip per stage
  // for the group instead of per node)
  constexpr int G = K <= 4 ? 4 : 2;
  uint32_t* near0 = lds;
  uint32_t* near1 = lds + NB;
  uint32_t* far = lds + 2 * NB;
  if (a.row_mask && !a.row_mask[row]) return;  // repaired elsewhere (whole workgroup)
  const Src s(a, row);
  unsigned long long* lab = a.labels + static_cast<size_t>(a.row_list ? blockIdx.x : row) * N;

  for (uint32_t i = tid; i < 3 * NB; i += nthr) lds[i] = 0u;
  for (uint32_t i = tid; i < N; i += nthr) lab[i] = kInfLabel;
  if (tid < 3) s_flag[tid] = 0u;
  if (tid < 2) s_min[tid] = kInf;
  __syncthreads();
  if (tid == 0) {
    lab[s.node] = 0ull;
    near0[s.node >> 5] = 1u << (s.node & 31u);
  }
  __syncthreads();

  const uint32_t delta = a.delta;
  uint32_t T = delta;  // near/far threshold
  uint32_t* cur = near0;
  uint32_t* nxt = near1;
  uint32_t mpar = 0;  // s_min[mpar] bounds the far set from below
  for (uint32_t it = 0;; ++it) {
    bool pushed_near = false;
    uint32_t far_min = kInf;  // this thread's smallest far push (one LDS atomic per wave below)
    // merge the candidate {nd, cnh} into u's label: smaller replaces, equal
    // ORs (cl: u's label as loaded); re-queue u if the label changed
    auto merge = [&](uint32_t u, uint32_t nd, uint32_t cnh, unsigned long long cl) {
      for (;;) {
        const uint32_t cd = static_cast<uint32_t>(cl >> 32);
        if (nd > cd) return;
        const unsigned long long nl = nd < cd
            ? ((static_cast<unsigned long long>(nd) << 32) | cnh)
            : (cl | cnh);
        if (nl == cl) return;
        const unsigned long long old = atomicCAS(&lab[u], cl, nl);
        if (old == cl) break;
        cl = old;
      }
      const uint32_t bit = 1u << (u & 31u);
      if (nd < T) {
        atomicOr(&nxt[u >> 5], bit);
        atomicAnd(&far[u >> 5], ~bit);  // expanded from the near set instead
        pushed_near = true;
      } else {
        atomicOr(&far[u >> 5], bit);
        far_min = min(far_min, nd);
      }
    };
    uint32_t w = tid, bits = 0, wbase = 0;
    for (;;) {
      // up to G frontier nodes of this thread's words
      uint32_t vs[G];
      int c = 0;
      while (c < G) {
        while (!bits && w < NB) {
          bits = cur[w];
          if (bits) {
            cur[w] = 0u;
            wbase = w * 32;
          }
          w += nthr;
        }
        if (!bits) break;
        vs[c++] = wbase + __builtin_ctz(bits);
        bits &= bits - 1;
      }
      if (c == 0) break;
      expand_group<K, G>(a, s, lab, vs, c, merge);
    }
    {  // the far set's lower bound: every far push folded per wave, not per push
      const uint32_t fm = wave_min(far_min);
      if ((tid & 63u) == 0 && fm != kInf) atomicMin(&s_min[mpar], fm);
    }
    const uint32_t par = it % 3u;
    if (pushed_near) s_flag[par] = 1u;
    __syncthreads();  // relaxations (global atomics) and bitmaps settled
    const bool more_near = s_flag[par] != 0u;
    if (tid == 0) s_flag[(par + 2u) % 3u] = 0u;  // the previous iteration's flag
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
    if (more_near) continue;
    // near frontier empty: advance the threshold past the far set's lower
    // bound and promote the far nodes below it; the rest give the exact bound
    const uint32_t m = s_min[mpar];
    if (m == kInf) break;  // far set empty: done (every thread read the same value)
    T = m + delta;
    const uint32_t npar = mpar ^ 1u;
    if (tid == 0) s_min[npar] = kInf;
    __syncthreads();
    uint32_t local_min = kInf;
    for (uint32_t w = tid; w < NB; w += nthr) {
      uint32_t bits = far[w], promote = 0u;
      for (uint32_t q = bits; q; q &= q - 1) {
        const uint32_t b = __builtin_ctz(q);
        const uint32_t d = static_cast<uint32_t>(
            __hip_atomic_load(&lab[w * 32 + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32);
        if (d < T) promote |= 1u << b;
        else local_min = min(local_min, d);
      }
      if (promote) {
        far[w] = bits & ~promote;
        cur[w] |= promote;
      }
    }
    const uint32_t wm = wave_min(local_min);
    if ((tid & 63u) == 0 && wm != kInf) atomicMin(&s_min[npar], wm);
    mpar = npar;
    __syncthreads();
  }
  __syncthreads();
  // labels -> dist row (kInf = unreachable) and first-hop row, coalesced
  uint32_t* od = a.out_dist + static_cast<size_t>(row) * N;
  uint32_t* on = a.out_nh + static_cast<size_t>(row) * N * a.words;
  for (uint32_t i = tid; i < N; i += nthr) {
    const unsigned long long l =
        __hip_atomic_load(&lab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_nontemporal_store(static_cast<uint32_t>(l >> 32), &od[i]);
    if (a.words == 1) {
      __builtin_nontemporal_store(static_cast<uint32_t>(l), &on[i]);
    } else {
      on[static_cast<size_t>(i) * a.words] = static_cast<uint32_t>(l);
      for (uint32_t k = 1; k < a.words; ++k) on[static_cast<size_t>(i) * a.words + k] = 0u;
    }
  }
}

// ---------------------------------------------------------------------------
// exact Dijkstra in the reference's extraction order
// ---------------------------------------------------------------------------
// LinkState::runSpf (LinkState.cpp:808-882) step for step: a binary heap on
// (metric, name), `>=` relaxations that union the first-hop sets, reset on a
// strictly better metric, no transit through overloaded nodes. With a
// zero-metric link the closed form of the other kernels does not hold (a node
// at the same metric contributes its first hops only if it is extracted
// first), and path metrics may exceed 32 bits; this kernel covers both. Lane 0
// of one wave per source runs the search (its state is one source's heap),
// the other lanes initialise and copy out.
size_t exact_state_bytes(uint32_t n, uint32_t words) {
  // metric u64 | pos u32 | heap u32 | nh u32 * words, 16-byte aligned
  return ((static_cast<size_t>(n) * (16 + 4 * words)) + 15) & ~static_cast<size_t>(15);
}

template <bool kLds>
__global__ __launch_bounds__(64) void spf_exact_kernel(ExactArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t N = a.n_nodes, W = a.words, row = blockIdx.x, lane = threadIdx.x;
  uint8_t* base = kLds ? reinterpret_cast<uint8_t*>(lds) : a.scratch + row * a.scratch_stride;
  uint64_t* metric = reinterpret_cast<uint64_t*>(base);
  uint32_t* pos = reinterpret_cast<uint32_t*>(metric + N);  // heap index + 1, kRec when extracted
  uint32_t* heap = pos + N;
  uint32_t* nh = heap + N;
  constexpr uint64_t kInf64 = ~0ull;
  constexpr uint32_t kRec = 0xFFFFFFFFu;
  for (uint32_t v = lane; v < N; v += 64) {
    metric[v] = kInf64;
    pos[v] = 0u;
  }
  for (uint32_t i = lane; i < N * W; i += 64) nh[i] = 0u;
  __syncthreads();
  const uint32_t src = a.srcs[row];
  const uint32_t* ign = nullptr;
  uint32_t n_ign = 0;
  if (a.ignore_ptr) {
    ign = a.ignore_links + a.ignore_ptr[row];
    n_ign = a.ignore_ptr[row + 1] - a.ignore_ptr[row];
  }
  uint32_t* rank_out = a.out_rank ? a.out_rank + static_cast<size_t>(row) * N : nullptr;
  if (lane == 0) {
    auto less = [&](uint32_t x, uint32_t y) {
      const uint64_t mx = metric[x], my = metric[y];
      return mx < my || (mx == my && a.name_rank[x] < a.name_rank[y]);
    };
    auto sift_up = [&](uint32_t i) {
      const uint32_t x = heap[i];
      while (i > 0) {
        const uint32_t p = (i - 1) >> 1, y = heap[p];
        if (!less(x, y)) break;
        heap[i] = y;
        pos[y] = i + 1;
        i = p;
      }
      heap[i] = x;
      pos[x] = i + 1;
    };
    auto sift_down = [&](uint32_t i, uint32_t n) {
      const uint32_t x = heap[i];
      for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= n) break;
        if (c + 1 < n && less(heap[c + 1], heap[c])) ++c;
        const uint32_t y = heap[c];
        if (!less(y, x)) break;
        heap[i] = y;
        pos[y] = i + 1;
        i = c;
      }
      heap[i] = x;
      pos[x] = i + 1;
    };
    uint32_t n_heap = 0, order = 0;
    metric[src] = 0;
    heap[n_heap++] = src;
    pos[src] = 1;
    const uint32_t K = a.ell_k;
    while (n_heap) {
      const uint32_t v = heap[0];
      if (--n_heap) {
        heap[0] = heap[n_heap];
        sift_down(0, n_heap);
      }
      pos[v] = kRec;  // recorded: final (LinkState.cpp:824)
      if (rank_out) rank_out[v] = order;
      ++order;
      const uint2 r0 = a.recs[static_cast<size_t>(v) * K];
      if (v != src && (r0.x & ORH_REC_ROW_OVL)) continue;  // no transit (:831-838)
      const uint64_t dv = metric[v];
      auto relax = [&](uint32_t q) {
        const uint2 r = a.recs[q];
        if (r.x & (ORH_REC_SKIP | ORH_REC_CONT)) return;
        if (n_ign && ignored(ign, n_ign, a.link[q])) return;
        const uint32_t u = r.x & ORH_REC_COL_MASK;
        if (pos[u] == kRec) return;
        const uint64_t nd = dv + (a.use_link_metric ? static_cast<uint64_t>(r.y) : 1ull);
        if (pos[u] == 0u) {  // first seen: queued at nd (:853-856)
          metric[u] = nd;
          heap[n_heap] = u;
          sift_up(n_heap++);
        } else if (metric[u] > nd) {  // strictly better: reset and re-heap (:862-866)
          metric[u] = nd;
          for (uint32_t k = 0; k < W; ++k) nh[static_cast<size_t>(u) * W + k] = 0u;
          sift_up(pos[u] - 1);
        }
        if (metric[u] != nd) return;
        if (v == src) {  // a direct neighbour's own bit (:869-872)
          const uint32_t b = a.rank_out[q];
          nh[static_cast<size_t>(u) * W + (b >> 5)] |= 1u << (b & 31u);
        } else {
          for (uint32_t k = 0; k < W; ++k)
            nh[static_cast<size_t>(u) * W + k] |= nh[static_cast<size_t>(v) * W + k];
        }
      };
      for (uint32_t j = 0; j < K; ++j) relax(v * K + j);
      const uint2 last = a.recs[static_cast<size_t>(v) * K + K - 1];
      if (last.x & ORH_REC_CONT) {
        const uint32_t start = last.x & ORH_REC_COL_MASK;
        for (uint32_t q = 0; q < last.y; ++q) relax(start + q);
      }
    }
  }
  __syncthreads();
  for (uint32_t v = lane; v < N; v += 64) {
    const uint64_t m = metric[v];
    const bool reached = pos[v] == kRec;
    if (a.out_dist64) a.out_dist64[static_cast<size_t>(row) * N + v] = reached ? m : kInf64;
    if (a.out_dist32) a.out_dist32[static_cast<size_t>(row) * N + v] = reached ? static_cast<uint32_t>(m) : kInf;
    if (rank_out && !reached) rank_out[v] = kInf;
  }
  for (uint32_t i = lane; i < N * W; i += 64) {
    const uint32_t v = i / W;
    a.out_nh[static_cast<size_t>(row) * N * W + i] = (pos[v] == kRec && v != src) ? nh[i] : 0u;
  }
}

// ---------------------------------------------------------------------------
// phase 2: first-hop masks
// ---------------------------------------------------------------------------
// distance of node x in row `row`: the u32 distance row, or (multi-source
// plans) the u8 level row scaled by w0
template <bool kLvl>
__device__ inline uint32_t hop_dist(const HopArgs& a, uint32_t row, uint32_t x) {
  const uint32_t* dr = dist_row(const_cast<uint32_t*>(a.dist), const_cast<uint32_t*>(a.scratch),
                                a.n_out, a.n_nodes, row);
  if (!kLvl) return dr[x];
  const uint32_t l = a.lvl_rows[static_cast<size_t>(row) * a.lvl_pitch + x];
  return l == kLvlNone ? kInf : l == kLvlDirect ? dr[x] : l * a.w0;
}

// the source's tight first links into LDS: ent[k] = {n, d_s(n), n's row,
// rank | 0x80000000 if n is overloaded}; returns the count. LDS layout:
// minw[nb] | node[nb] | ent[nb] (hop_lds_bytes)
template <bool kLvl>
__device__ inline uint32_t hop_entries(const HopArgs& a, uint32_t i, uint32_t* lds, uint32_t* s_cnt) {
  const uint32_t tid = threadIdx.x;
  const uint32_t src = a.srcs[i];
  const uint32_t nb0 = a.nbr_ptr[i], nb = a.nbr_ptr[i + 1] - nb0;
  uint32_t* minw = lds;
  uint32_t* node = lds + nb;
  uint4* ent = reinterpret_cast<uint4*>(lds + ((2 * nb + 3) & ~3u));
  const uint32_t* ign = nullptr;
  uint32_t n_ign = 0;
  if (a.ignore_ptr) {
    ign = a.ignore_links + a.ignore_ptr[i];
    n_ign = a.ignore_ptr[i + 1] - a.ignore_ptr[i];
  }

  for (uint32_t r = tid; r < nb; r += kBlock) minw[r] = kInf;
  if (tid == 0) *s_cnt = 0;
  __syncthreads();
  // the source's links: smallest live metric per distinct neighbour
  const uint32_t K = a.ell_k;
  auto consider = [&](uint32_t q) {
    const uint2 r = a.recs[q];
    if (r.x & (ORH_REC_SKIP | ORH_REC_CONT)) return;
    if (n_ign && ignored(ign, n_ign, a.link[q])) return;
    const uint32_t rk = a.rank_out[q];
    atomicMin(&minw[rk], a.use_link_metric ? r.y : 1u);
    node[rk] = r.x & ORH_REC_COL_MASK;
  };
  for (uint32_t j = tid; j < K; j += kBlock) consider(src * K + j);
  const uint2 last = a.recs[static_cast<size_t>(src) * K + K - 1];
  if (last.x & ORH_REC_CONT)
    for (uint32_t j = tid; j < last.y; j += kBlock) consider((last.x & ORH_REC_COL_MASK) + j);
  __syncthreads();
  // tight first links: d_s(n) equals the cheapest live link to n
  for (uint32_t r = tid; r < nb; r += kBlock) {
    if (minw[r] == kInf) continue;
    const uint32_t u = node[r];
    const uint32_t du = hop_dist<kLvl>(a, i, u);
    if (du != minw[r]) continue;
    const uint32_t k = atomicAdd(s_cnt, 1u);
    ent[k] = make_uint4(u, du, a.nbr_row[nb0 + r], r | (a.overloaded[u] ? 0x80000000u : 0u));
  }
  __syncthreads();
  return *s_cnt;
}

__device__ inline uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t group);

__global__ __launch_bounds__(kBlock) void first_hop_kernel(HopArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_cnt;
  const uint32_t N = a.n_nodes;
  const uint32_t tid = threadIdx.x;
  // XCD-aware order (opt-in, ORH_HOP_XCD=1): an XCD runs a contiguous range
  // of sources, so the neighbour rows its sources share would be read
  // through its own L2; measured slower on the C2w sweep (0.395 vs 0.372 ms,
  // profiles/r06/ah_hop_xcd_ab.txt): a source's tiles spread over the XCDs
  // balance better than the L2 reuse pays
  const uint32_t lb = a.xcd_hop ? xcd_block(blockIdx.x, gridDim.x, a.xcd_group) : blockIdx.x;
  const uint32_t i = lb / a.tiles, tile = lb % a.tiles;
  const uint32_t src = a.srcs[i];
  const uint32_t nb = a.nbr_ptr[i + 1] - a.nbr_ptr[i];
  const uint4* ent = reinterpret_cast<const uint4*>(lds + ((2 * nb + 3) & ~3u));
  const uint32_t ne = hop_entries<false>(a, i, lds, &s_cnt);
  const uint32_t* ds = dist_row(const_cast<uint32_t*>(a.dist), const_cast<uint32_t*>(a.scratch),
                                a.n_out, N, i);


  uint32_t v[kHopPer], dv[kHopPer];
#pragma unroll
  for (int k = 0; k < kHopPer; ++k) {
    v[k] = tile * (kBlock * kHopPer) + k * kBlock + tid;
    dv[k] = v[k] < N ? ds[v[k]] : kInf;
    if (v[k] == src) dv[k] = kInf;  // the source has no next hops
  }
  const uint32_t W = a.words;
  uint32_t* nh = a.out_nh + static_cast<size_t>(i) * N * W;
  for (uint32_t word = 0; word < W; ++word) {
    uint32_t acc[kHopPer] = {};
    for (uint32_t e = 0; e < ne; ++e) {
      const uint4 en = ent[e];
      const uint32_t r = en.w & 0x7FFFFFFFu;
      if ((r >> 5) != word) continue;
      const uint32_t bit = 1u << (r & 31u);
      const bool transit = !(en.w & 0x80000000u);
      const uint32_t* dr = dist_row(const_cast<uint32_t*>(a.dist),
                                    const_cast<uint32_t*>(a.scratch), a.n_out, N, en.z);
      uint32_t x[kHopPer];
#pragma unroll
      for (int k = 0; k < kHopPer; ++k) x[k] = (transit && dv[k] != kInf) ? dr[v[k]] : kInf;
#pragma unroll
      for (int k = 0; k < kHopPer; ++k) {
        if (dv[k] == kInf) continue;
        if (v[k] == en.x ||
            (x[k] != kInf && static_cast<uint64_t>(en.y) + x[k] == dv[k]))
          acc[k] |= bit;
      }
    }
#pragma unroll
    for (int k = 0; k < kHopPer; ++k)
      if (v[k] < N) __builtin_nontemporal_store(acc[k], &nh[static_cast<size_t>(v[k]) * W + word]);
  }
}

// first hops of multi-source BFS rows: the same closed form over u8 level
// rows (pitch a multiple of 16), P consecutive nodes per thread so every row
// access is one P-byte load (P = 16 for large batches; 4 keeps small ones
// spread over more workgroups)
template <uint32_t P>
struct LvlVec;
template <>
struct LvlVec<16> {
  typedef uint4 T;
  __device__ static uint32_t byte(const uint4& x, uint32_t k) {
    const uint32_t w = k < 4 ? x.x : k < 8 ? x.y : k < 12 ? x.z : x.w;
    return (w >> ((k & 3u) * 8u)) & 0xFFu;
  }
};
template <>
struct LvlVec<8> {
  typedef uint2 T;
  __device__ static uint32_t byte(const uint2& x, uint32_t k) { return ((k < 4 ? x.x : x.y) >> ((k & 3u) * 8u)) & 0xFFu; }
};
template <>
struct LvlVec<4> {
  typedef uint32_t T;
  __device__ static uint32_t byte(const uint32_t& x, uint32_t k) { return (x >> (k * 8u)) & 0xFFu; }
};

__device__ inline bool has_byte_fe(uint32_t x) {  // some byte == kLvlDirect
  const uint32_t z = x ^ 0xFEFEFEFEu;
  return ((z - 0x01010101u) & ~z & 0x80808080u) != 0u;
}

// XCD-aware block order: the dispatcher deals workgroups round-robin over the
// 8 XCDs (block b -> XCD b % 8), each with its own L2. Remapped, XCD x runs a
// contiguous range of logical blocks, so the sources resident on one XCD at a
// time are neighbours in row order and share their neighbours' level rows in
// that XCD's L2 instead of each XCD fetching them from HBM. Bijective for any
// grid size.
__device__ inline uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t group) {
  constexpr uint32_t kXcd = 8;
  if (group == 0) {  // one contiguous range per XCD
    const uint32_t x = b % kXcd, k = b / kXcd, q = nb / kXcd, r = nb % kXcd;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  // runs of `group` consecutive blocks per XCD, dealt round-robin; the tail
  // that does not fill a whole round keeps its order
  const uint32_t full = nb / (kXcd * group) * (kXcd * group);
  if (b >= full) return b;
  const uint32_t x = b % kXcd, k = b / kXcd;
  return ((k / group) * kXcd + x) * group + k % group;
}

// One workgroup per (source, tile phase): the source's tight first links are
// gathered once, then the workgroup walks tiles phase, phase + split, ...
// ORH_HOP_WAVES (A/B builds): waves per SIMD the register allocation must
// allow (4: <= 128 VGPRs, room beside the MS-BFS workgroups of other streams)
#ifdef ORH_HOP_WAVES
#define ORH_HOP_ATTR __attribute__((amdgpu_waves_per_eu(ORH_HOP_WAVES)))
#else
#define ORH_HOP_ATTR
#endif
template <uint32_t kLvlPer>
__global__ __launch_bounds__(kBlock) ORH_HOP_ATTR void first_hop_lvl_kernel(HopArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_cnt;
  typedef typename LvlVec<kLvlPer>::T Vec;
  constexpr uint32_t kWords = kLvlPer / 4;
  const uint32_t N = a.n_nodes, P = a.lvl_pitch, w0 = a.w0;
  const uint32_t tid = threadIdx.x;
  const uint32_t split = a.tile_split;
  // one logical block per workgroup, or (persistent grid, a multiple of the
  // 8 XCDs; ORH_HOP_WG_PER_CU) XCD x = b % 8 owns a contiguous logical range
  // its workgroups stride through
  uint32_t lb, lb_end, lb_step;
  if (gridDim.x >= a.n_logical) {
    lb = xcd_block(blockIdx.x, gridDim.x, a.xcd_group);
    lb_end = lb + 1;
    lb_step = 1;
  } else {
    constexpr uint32_t kXcd = 8;
    const uint32_t x = blockIdx.x % kXcd, k = blockIdx.x / kXcd;
    const uint32_t q = a.n_logical / kXcd, r = a.n_logical % kXcd;
    const uint32_t lo = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    lb = lo + k;
    lb_end = lo + q + (x < r ? 1u : 0u);
    lb_step = gridDim.x / kXcd;
  }
  for (; lb < lb_end; lb += lb_step) {
  const uint32_t i = lb / split, phase = lb % split;
  const uint32_t src = a.srcs[i];
  const uint32_t nb = a.nbr_ptr[i + 1] - a.nbr_ptr[i];
  const uint4* ent = reinterpret_cast<const uint4*>(lds + ((2 * nb + 3) & ~3u));
  const uint32_t ne = hop_entries<true>(a, i, lds, &s_cnt);
  const uint32_t W = a.words;
  uint32_t* nh = a.out_nh + static_cast<size_t>(i) * N * W;
  for (uint32_t tile = phase; tile < a.tiles; tile += split) {
    const uint32_t v0 = (tile * kBlock + tid) * kLvlPer;
    if (v0 >= N) break;
    auto dist_at = [&](uint32_t row, const Vec& x, uint32_t k) -> uint32_t {
      const uint32_t l = LvlVec<kLvlPer>::byte(x, k);
      if (l == kLvlNone) return kInf;
      if (l == kLvlDirect)
        return dist_row(const_cast<uint32_t*>(a.dist), const_cast<uint32_t*>(a.scratch), a.n_out,
                        N, row)[v0 + k];
      return l * w0;
    };
    auto words_of = [](const Vec& x, uint32_t (&w)[kWords]) {
      if constexpr (kLvlPer == 16) {
        w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
      } else if constexpr (kLvlPer == 8) {
        w[0] = x.x; w[1] = x.y;
      } else {
        w[0] = x;
      }
    };
    const Vec own = *reinterpret_cast<const Vec*>(a.lvl_rows + static_cast<size_t>(i) * P + v0);
    uint32_t ow[kWords];
    words_of(own, ow);
    bool own_direct = false;
#pragma unroll
    for (uint32_t q = 0; q < kWords; ++q) own_direct |= has_byte_fe(ow[q]);
    // d_s(v0 + k) where needed (the direct path; kInf: the source, which has
    // no next hops, and the padding past N) - not held for all k (VGPRs)
    auto own_dist = [&](uint32_t k) -> uint32_t {
      return (v0 + k == src || v0 + k >= N) ? kInf : dist_at(i, own, k);
    };
    // own level bytes with the source's byte forced to "unreached" (no next
    // hops; bytes past N are the row padding, unreached already)
    uint32_t ot[kWords];
#pragma unroll
    for (uint32_t q = 0; q < kWords; ++q) ot[q] = ow[q];
    if (src >= v0 && src < v0 + kLvlPer) {
#pragma unroll
      for (uint32_t q = 0; q < kWords; ++q)
        if ((src - v0) / 4u == q) ot[q] |= 0xFFu << (((src - v0) & 3u) * 8u);
    }
    for (uint32_t word = 0; word < W; ++word) {
      uint32_t acc[kLvlPer] = {};
      uint32_t pk[kWords] = {};  // byte k of word q: mask bits 0..7 of node 4q + k (packed path)
      // the neighbour rows of kGroup entries are loaded back to back before
      // any is used: one memory round trip per group, not per entry (the
      // loads of a dynamic-length loop are otherwise issued one at a time)
#ifndef ORH_HOP_GROUP
#define ORH_HOP_GROUP 4  // (1: one entry per round trip, the round-3 loop; A/B builds)
#endif
      constexpr uint32_t kGroup = ORH_HOP_GROUP;
      for (uint32_t e0 = 0; e0 < ne; e0 += kGroup) {
      uint4 ens[kGroup];
      Vec nxs[kGroup];
      uint32_t use = 0;  // bit g: entry e0 + g belongs to this word
#pragma unroll
      for (uint32_t g = 0; g < kGroup; ++g) {
        if (e0 + g >= ne) break;
        ens[g] = ent[e0 + g];
        if (((ens[g].w & 0x7FFFFFFFu) >> 5) != word) continue;
        use |= 1u << g;
        if (!(ens[g].w & 0x80000000u))
          nxs[g] = *reinterpret_cast<const Vec*>(a.lvl_rows + static_cast<size_t>(ens[g].z) * P + v0);
      }
#pragma unroll
      for (uint32_t g = 0; g < kGroup; ++g) {
        if (!((use >> g) & 1u)) continue;
        const uint4 en = ens[g];
        const uint32_t r = en.w & 0x7FFFFFFFu;
        const uint32_t bit = 1u << (r & 31u);
        if (en.x >= v0 && en.x < v0 + kLvlPer) {
#pragma unroll
          for (uint32_t k = 0; k < kLvlPer; ++k)
            if (v0 + k == en.x && ((ot[k / 4] >> ((k & 3u) * 8u)) & 0xFFu) != kLvlNone) acc[k] |= bit;
        }
        if (en.w & 0x80000000u) continue;  // overloaded neighbour: no transit
        const Vec nx = nxs[g];
        uint32_t nw[kWords];
        words_of(nx, nw);
        bool direct = own_direct || en.y != w0;
#pragma unroll
        for (uint32_t q = 0; q < kWords; ++q) direct |= has_byte_fe(nw[q]);
        if (!direct && bit < 256u) {
          // plain levels, four nodes per word op: tight iff L_n(v) + 1 ==
          // L_s(v), bytewise mod 256 (an unreached 255 wraps to 0, a level
          // only the source holds, forced to 255 in ot)
#pragma unroll
          for (uint32_t q = 0; q < kWords; ++q) {
            const uint32_t inc = ((nw[q] & 0x7F7F7F7Fu) + 0x01010101u) ^ (nw[q] & 0x80808080u);
            const uint32_t z = inc ^ ot[q];
            const uint32_t eq = ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z | 0x7F7F7F7Fu);  // 0x80 per zero byte
            pk[q] |= (eq >> 7) * bit;
          }
        } else if (!direct) {  // plain levels, a rank past 7
#pragma unroll
          for (uint32_t k = 0; k < kLvlPer; ++k)
            if (((nw[k / 4] >> ((k & 3u) * 8u)) & 0xFFu) + 1u == ((ot[k / 4] >> ((k & 3u) * 8u)) & 0xFFu))
              acc[k] |= bit;
        } else {
#pragma unroll
          for (uint32_t k = 0; k < kLvlPer; ++k) {
            const uint32_t dk = own_dist(k);
            if (dk == kInf) continue;
            const uint32_t x = dist_at(en.z, nx, k);
            if (x != kInf && static_cast<uint64_t>(en.y) + x == dk) acc[k] |= bit;
          }
        }
      }
      }  // entry group
#pragma unroll
      for (uint32_t k = 0; k < kLvlPer; ++k) acc[k] |= (pk[k / 4] >> ((k & 3u) * 8u)) & 0xFFu;
      if (kLvlPer >= 8 && W == 1 && v0 + kLvlPer <= N && (N & 3u) == 0) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4* o = reinterpret_cast<u32x4*>(nh + v0);
#pragma unroll
        for (uint32_t q = 0; q < kLvlPer / 4; ++q) {
          const u32x4 x = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
          __builtin_nontemporal_store(x, &o[q]);
        }
      } else {
#pragma unroll
        for (uint32_t k = 0; k < kLvlPer; ++k)
          if (v0 + k < N) nh[static_cast<size_t>(v0 + k) * W + word] = acc[k];
      }
    }
  }
  __syncthreads();  // every thread is done with this source's entries
  }
}

// ---------------------------------------------------------------------------
// planning and launch
// ---------------------------------------------------------------------------
// dynamic-LDS opt-in, raised once per kernel to the largest size launched
// (hipFuncSetAttribute is a runtime call worth avoiding on every sweep)
template <typename Kern>
static hipError_t lds_opt_in(Kern kernel, size_t lds) {
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> granted;
  const void* f = reinterpret_cast<const void*>(kernel);
  std::lock_guard<std::mutex> lock(mu);
  auto it = granted.find(f);
  if (it != granted.end() && lds <= it->second) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(lds));
  if (e == hipSuccess) granted[f] = lds;
  return e;
}

template <typename Kern, typename Args>
static hipError_t launch(Kern kernel, const Args& a, uint32_t grid, uint32_t block, size_t lds,
                         hipStream_t s) {
  hipError_t e = lds_opt_in(kernel, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), lds, s, a);
  return hipGetLastError();
}

static size_t align16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

static SpfPlan plan_global(SpfPlan p, uint32_t n_nodes, uint64_t path_bound, size_t lds_limit) {
  const size_t bytes = 3 * static_cast<size_t>((n_nodes + 31) / 32) * 4;
  if (path_bound >= 0xFFFFFFFFull || bytes > lds_limit) {
    p.variant = SpfVariant::kUnsupported;
    return p;
  }
  p.variant = SpfVariant::kGlobal;
  p.lds_bytes = std::max<size_t>(bytes, 16);
  p.block = 256;
  return p;
}

SpfPlan plan_spf(uint32_t n_nodes, bool uniform, uint64_t path_bound, uint32_t ell_k,
                 size_t lds_limit, bool multi_source, SpfMode mode) {
  SpfPlan p{};
  p.ell_k = ell_k;
  if (ell_k != 4 && ell_k != 8) return p;
  if (mode == SpfMode::kGlobal || mode == SpfMode::kGlobalTwoPhase)
    return plan_global(p, n_nodes, path_bound, lds_limit);
  const size_t nb = (n_nodes + 31) / 32;
  if (mode == SpfMode::kAuto && multi_source && uniform && path_bound < 0xFFFFFFFFull) {
    // a thread owns J <= 32 nodes (registers); the frontier arrays hold
    // N + 1 entries (the last is the always-zero target of dead slots).
    // 8 waves per workgroup (J = 20 on the 10k grid): one sweep alone takes
    // 0.82 ms against 0.73 at 12 waves (J = 16), but sweeps running side by
    // side on 4 streams - the bench step, any batch of what-if topologies -
    // finish 7 % sooner (26.8 vs 28.7 ms per 32 sweeps): two 8-wave
    // workgroups per CU leave wave slots and VGPRs for the other streams'
    // first-hop and finalize kernels (profiles/r03/o_ms_block_ab.txt)
    // (past 16,384 nodes 512 threads would need J > 32: 12 waves)
    uint32_t block = n_nodes <= 4096 ? 256 : n_nodes <= 16384 ? 512 : 768;
    // ORH_MS_BLOCK (A/B): threads per multi-source workgroup (multiple of 64)
    if (const char* e = getenv("ORH_MS_BLOCK")) {
      const int b = atoi(e);
      if (b >= 64 && b <= 1024 && b % 64 == 0) block = static_cast<uint32_t>(b);
    }
    const uint32_t j = (n_nodes + block - 1) / block;
    const uint32_t pitch = (n_nodes + 1 + 15) & ~15u;
    if (j <= 32) {
      for (uint32_t mb = 4; mb >= 2; mb /= 2) {
        const size_t bytes = 2 * static_cast<size_t>(mb) * pitch;
        // (16-bit byte offsets in the kernel's ELL columns)
        if (bytes <= lds_limit && static_cast<size_t>(mb) * pitch <= 65536) {
          p.variant = SpfVariant::kMsBfs;
          p.mask_bytes = mb;
          p.ms_j = (j + 3) & ~3u;
          p.ms_pitch = pitch;
          p.lds_bytes = bytes;
          p.block = block;
          return p;
        }
      }
    }
  }
  if (uniform && path_bound < 0xFFFFFFFFull) {
    // levels are < N; the level type's all-ones marks "unvisited"
    p.variant = n_nodes < 0xFFu ? SpfVariant::kBfs8
        : n_nodes < 0xFFFFu     ? SpfVariant::kBfs16
                                : SpfVariant::kBfs32;
    const size_t lb = n_nodes < 0xFFu ? 1 : n_nodes < 0xFFFFu ? 2 : 4;
    p.pend_off = align16(static_cast<size_t>(n_nodes) * lb);
    p.lds_bytes = p.pend_off + 2 * nb * 4;
  } else if (path_bound < 0xFFFFull) {
    p.variant = SpfVariant::kDist16;
    p.pend_off = align16(static_cast<size_t>(n_nodes) * 2);
    p.lds_bytes = p.pend_off + align16(nb * 4);
  } else if (path_bound < 0xFFFFFFFFull) {
    p.variant = SpfVariant::kDist32;
    p.pend_off = align16(static_cast<size_t>(n_nodes) * 4);
    p.lds_bytes = p.pend_off + align16(nb * 4);
  } else {
    return p;
  }
  // a thread owns two bitmap words per pass; 256 threads cover N <= 16,384
  // in one pass and leave room for 8 workgroups per CU
  const uint32_t half = static_cast<uint32_t>((nb + 1) / 2);
  p.block = std::min<uint32_t>(kMaxBlock, std::max<uint32_t>(256, (half + 63) / 64 * 64));
  if (p.lds_bytes > lds_limit) return plan_global(p, n_nodes, path_bound, lds_limit);
  return p;
}

template <int K, class M, int J>
static hipError_t launch_ms_j(const SpfPlan& plan, const SpfArgs& a, uint32_t n_rows, hipStream_t s) {
  if (a.ms_width == 0 || a.ms_width > MsMask<M>::kS) return hipErrorInvalidValue;
  const uint32_t batches = (n_rows + a.ms_width - 1) / a.ms_width;
  // the arrival log's block assembly reuses the frontier arrays' LDS: 64 x kS
  // bytes per wave
  // the log's block assembly reuses the frontier arrays' LDS: one wave's
  // J * 64 node blocks at a time
  size_t lds = plan.lds_bytes;
  if (sizeof(M) <= 4) {
    if (!a.ms_log) return hipErrorInvalidValue;
    lds = std::max<size_t>(lds, size_t{J} * 64 * (MsMask<M>::kS + 4));
  }
  const SpfArgs& b = a;
  if (a.ms_bw)
    return launch(spf_msbfs_kernel<K, M, J, true>, b, batches, plan.block, lds, s);
  return launch(spf_msbfs_kernel<K, M, J, false>, b, batches, plan.block, lds, s);
}

template <int K, class M>
static hipError_t launch_ms_m(const SpfPlan& plan, const SpfArgs& a, uint32_t n_rows, hipStream_t s) {
  switch (plan.ms_j) {
    case 4: return launch_ms_j<K, M, 4>(plan, a, n_rows, s);
    case 8: return launch_ms_j<K, M, 8>(plan, a, n_rows, s);
    case 12: return launch_ms_j<K, M, 12>(plan, a, n_rows, s);
    case 16: return launch_ms_j<K, M, 16>(plan, a, n_rows, s);
    case 20: return launch_ms_j<K, M, 20>(plan, a, n_rows, s);
    case 24: return launch_ms_j<K, M, 24>(plan, a, n_rows, s);
    case 28: return launch_ms_j<K, M, 28>(plan, a, n_rows, s);
    case 32: return launch_ms_j<K, M, 32>(plan, a, n_rows, s);
    default: return hipErrorInvalidValue;
  }
}

template <int K>
static hipError_t launch_ms(const SpfPlan& plan, const SpfArgs& a, uint32_t n_rows, hipStream_t s) {
  switch (plan.mask_bytes) {
    case 2: return launch_ms_m<K, uint16_t>(plan, a, n_rows, s);
    case 4: return launch_ms_m<K, uint32_t>(plan, a, n_rows, s);
    case 8: return launch_ms_m<K, uint64_t>(plan, a, n_rows, s);
    default: return hipErrorInvalidValue;
  }
}

size_t ms_log_bytes(const SpfPlan& plan, uint32_t n_rows) {
  if (plan.variant != SpfVariant::kMsBfs || plan.ms_width == 0 || plan.mask_bytes > 4) return 0;
  const size_t batches = (n_rows + plan.ms_width - 1) / plan.ms_width;
  return batches * plan.ms_j * plan.block * (plan.mask_bytes * 8) * sizeof(uint64_t);
}

size_t ms_scratch_bytes(const SpfPlan& plan, uint32_t n_nodes, uint32_t n_rows) {
  if (plan.variant != SpfVariant::kMsBfs || plan.ms_width == 0) return 0;
  const uint32_t w = plan.ms_width;
  return static_cast<size_t>((n_rows + w - 1) / w) * n_nodes * (plan.mask_bytes * 8);
}

void ms_set_width(SpfPlan& plan, uint32_t n_nodes, uint32_t n_rows, uint32_t n_cu, size_t lds_limit,
                  bool alone) {
  if (plan.variant != SpfVariant::kMsBfs) return;
  plan.ms_width = plan.mask_bytes * 8;
  // ORH_MS_WIDE=1 (opt-in): when u32 masks need more than one batch per CU
  // and u64 frontier arrays fit in LDS, widen the masks and spread the rows
  // over at most n_cu batches of ceil(n_rows / n_cu) sources. On C2 (250
  // batches of 40) this swept in 0.86-0.92 ms against 0.75 for 313 u32
  // batches: the batches that share a CU are not the slow ones
  // (per-workgroup stamps, profiles/r02/msbfs_ab.md), and u64 masks cost more
  // per level than they save
  // latency plan: when every batch has a CU to itself (a sweep over a shard
  // of the sources, N GPUs sharing one topology), the per-level time of one
  // workgroup is the sweep time, so the batch gets 1024 threads (fewer nodes
  // per thread: J = 12 instead of 20 on the 10k grid). ORH_MS_LATENCY=0: off;
  // ORH_MS_LATENCY=2: with the interval skip as well (it cuts a lone C2
  // corner batch 0.48 -> 0.32 ms, profiles/r02/msbfs_ab.md, but a C2 shard of
  // 1,254 sources measured 0.785 vs 0.748 ms with it, profiles/r04/
  // f_strong_rehearsal_skip.txt vs e_strong_rehearsal.txt)
  plan.ms_skip = 0;
  {
    const char* lat = getenv("ORH_MS_LATENCY");
    const uint32_t batches = (n_rows + plan.mask_bytes * 8 - 1) / (plan.mask_bytes * 8);
    const uint32_t j = (n_nodes + 1023) / 1024;
    if (!(lat && atoi(lat) == 0) && !getenv("ORH_MS_BLOCK") && n_cu && batches <= n_cu &&
        plan.block < 1024 && j <= 32) {
      plan.block = 1024;
      plan.ms_j = (j + 3) & ~3u;
      plan.ms_skip = lat && atoi(lat) == 2;
    } else if (!(lat && atoi(lat) == 0) && !getenv("ORH_MS_BLOCK") && alone && plan.block == 512) {
      // lone-sweep plan: no other sweep in flight on the device, so the
      // batches do not share CUs with other streams' kernels and 12 waves
      // per batch cut the per-level time (one C2 sweep 0.82 -> 0.68 ms of
      // MS-BFS); under concurrent sweeps 8 waves stay (the 4-lane step
      // 24.8 vs 26.3 ms at 12, profiles/r04/ai_ms_block_ab.txt)
      const uint32_t j12 = (n_nodes + 767) / 768;
      if (j12 <= 32) {
        plan.block = 768;
        plan.ms_j = (j12 + 3) & ~3u;
      }
    }
  }
  const size_t bytes64 = 2 * 8 * static_cast<size_t>(plan.ms_pitch);
  const char* e = getenv("ORH_MS_WIDE");
  const bool allow = e && atoi(e) == 1;
  if (allow && plan.mask_bytes == 4 && n_cu && n_rows > 32ull * n_cu && bytes64 <= lds_limit &&
      4ull * plan.ms_pitch <= 65536) {
    plan.mask_bytes = 8;
    plan.lds_bytes = bytes64;
    plan.ms_width = std::min<uint32_t>(64, (n_rows + n_cu - 1) / n_cu);
  }
  (void)n_nodes;
}

// ORH_HBM_ASYNC=0 selects the round-synchronous HBM frontier kernel (A/B)
static bool nh_async() {
  static const bool on = [] {
    const char* e = getenv("ORH_HBM_ASYNC");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

template <int K>
static hipError_t launch_k(const SpfPlan& plan, const SpfArgs& a, uint32_t n_rows, hipStream_t s) {
  switch (plan.variant) {
    case SpfVariant::kMsBfs:
      return launch_ms<K>(plan, a, n_rows, s);
    case SpfVariant::kBfs8:
      return launch(spf_bfs_kernel<K, uint8_t>, a, n_rows, plan.block, plan.lds_bytes, s);
    case SpfVariant::kBfs16:
      return launch(spf_bfs_kernel<K, uint16_t>, a, n_rows, plan.block, plan.lds_bytes, s);
    case SpfVariant::kBfs32:
      return launch(spf_bfs_kernel<K, uint32_t>, a, n_rows, plan.block, plan.lds_bytes, s);
    case SpfVariant::kDist16:
      return launch(spf_dist_kernel<uint16_t, K>, a, n_rows, plan.block, plan.lds_bytes, s);
    case SpfVariant::kDist32:
      return launch(spf_dist_kernel<uint32_t, K>, a, n_rows, plan.block, plan.lds_bytes, s);
    case SpfVariant::kGlobal:
      return launch(spf_global_kernel<K>, a, n_rows, plan.block, plan.lds_bytes, s);
    case SpfVariant::kGlobalNh:
      if (a.dist_only)  // distances alone (u32 labels), no first-hop rows
        return launch(spf_global_nh_async_kernel<K, false>, a, n_rows, plan.block, plan.lds_bytes, s);
      if (nh_async())
        return launch(spf_global_nh_async_kernel<K, true>, a, n_rows, plan.block, plan.lds_bytes, s);
      return launch(spf_global_nh_kernel<K>, a, n_rows, plan.block, plan.lds_bytes, s);
    default:
      return hipErrorInvalidValue;
  }
}

bool bfs_nh_shape(uint32_t n_nodes, uint32_t words, size_t lds_limit, uint32_t* block,
                  uint32_t* j, size_t* lds) {
  if (n_nodes == 0 || n_nodes > 32768u) return false;  // 16-bit packed columns, J <= 32
  const uint32_t b = std::min<uint32_t>(kMaxBlock, std::max<uint32_t>(64, ((n_nodes + 3) / 4 + 63) / 64 * 64));
  const uint32_t jj = ((n_nodes + b - 1) / b + 3) & ~3u;
  const size_t bytes = 4 * static_cast<size_t>((n_nodes + 4u) & ~3u) + 4 * static_cast<size_t>(n_nodes) * words;
  if (jj > 32 || bytes > lds_limit) return false;
  *block = b;
  *j = jj;
  *lds = bytes;
  return true;
}

template <int K>
static hipError_t launch_bfs_nh(const SpfArgs& a, uint32_t n_rows, uint32_t block, uint32_t j,
                                size_t lds, hipStream_t s) {
  switch (j) {
    case 4: return launch(spf_bfs_nh_kernel<K, 4>, a, n_rows, block, lds, s);
    case 8: return launch(spf_bfs_nh_kernel<K, 8>, a, n_rows, block, lds, s);
    case 12: return launch(spf_bfs_nh_kernel<K, 12>, a, n_rows, block, lds, s);
    case 16: return launch(spf_bfs_nh_kernel<K, 16>, a, n_rows, block, lds, s);
    case 20: return launch(spf_bfs_nh_kernel<K, 20>, a, n_rows, block, lds, s);
    case 24: return launch(spf_bfs_nh_kernel<K, 24>, a, n_rows, block, lds, s);
    case 28: return launch(spf_bfs_nh_kernel<K, 28>, a, n_rows, block, lds, s);
    case 32: return launch(spf_bfs_nh_kernel<K, 32>, a, n_rows, block, lds, s);
    default: return hipErrorInvalidValue;
  }
}

size_t lds16_bytes(uint32_t n_nodes) {
  const size_t nb = (n_nodes + 31) / 32;
  size_t fw = 1;
  while (2 * fw <= std::min<size_t>(nb, 256)) fw *= 2;
  return 4 * ((((n_nodes + 1) / 2 + 3) & ~size_t{3}) + 2 * nb + fw + 2 * kSpillSlots + kIgnLds);
}

hipError_t launch_spf_lds16(const SpfPlan& fallback, SpfArgs a, uint32_t n_rows, uint32_t ell_k,
                            hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  if (!a.ovf_rows || !a.dist_only || fallback.variant != SpfVariant::kGlobalNh) return hipErrorInvalidValue;
  a.n_rows = n_rows;
  const size_t lds = lds16_bytes(a.n_nodes);
  hipError_t e = hipMemsetAsync(a.ovf_rows, 0, 4, s);
  if (e != hipSuccess) return e;
  // ORH_LDS16_BLOCK (A/B): threads per search (one search per CU either way)
  static const uint32_t block = [] {
    const char* v = getenv("ORH_LDS16_BLOCK");
    const int b = v ? atoi(v) : 1024;
    return (b >= 64 && b <= 1024 && b % 64 == 0) ? static_cast<uint32_t>(b) : 1024u;
  }();
  e = ell_k == 8 ? launch(spf_lds16_kernel<8>, a, n_rows, block, lds, s)
                 : launch(spf_lds16_kernel<4>, a, n_rows, block, lds, s);
  if (e != hipSuccess) return e;
  // rows the u16 search could not finish: the HBM kernel over that list
  // (workgroups past the list's length exit at once)
  SpfArgs b = a;
  b.row_list = a.ovf_rows + 1;
  b.row_count = a.ovf_rows;
  b.row_order = nullptr;
  return launch_spf(fallback, b, n_rows, s);
}

hipError_t launch_spf_lds_nh(SpfArgs a, uint32_t n_rows, uint32_t ell_k, bool packed, uint32_t block,
                             hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  if (packed && !a.ovf_rows) return hipErrorInvalidValue;
  a.n_rows = n_rows;
  a.row_list = nullptr;
  a.row_count = nullptr;
  hipError_t e = hipSuccess;
  if (packed) {
    e = hipMemsetAsync(a.ovf_rows, 0, 4, s);
    if (e != hipSuccess) return e;
    const size_t lds = lds_nh_bytes(a.n_nodes, true);
    e = ell_k == 8 ? launch(spf_lds_nh_kernel<8, true>, a, n_rows, block, lds, s)
                   : launch(spf_lds_nh_kernel<4, true>, a, n_rows, block, lds, s);
    if (e != hipSuccess) return e;
    // rows with a distance past 16 bits: the u64 form over that list
    // (workgroups past the list's length exit at once)
    a.row_list = a.ovf_rows + 1;
    a.row_count = a.ovf_rows;
  }
  const size_t lds = lds_nh_bytes(a.n_nodes, false);
  return ell_k == 8 ? launch(spf_lds_nh_kernel<8, false>, a, n_rows, block, lds, s)
                    : launch(spf_lds_nh_kernel<4, false>, a, n_rows, block, lds, s);
}

template <int K, int S>
static hipError_t launch_wms_k(const SpfArgs& a, uint32_t batches, size_t lds, hipStream_t s) {
  const uint32_t j = (a.n_nodes + 1023) / 1024;
  if constexpr (S == 8) {  // 16 B a node: N <= ~10,200, J <= 10
    switch (j <= 2 ? 2 : j <= 4 ? 4 : j <= 6 ? 6 : j <= 8 ? 8 : 10) {
      case 2: return launch(spf_wms_kernel<K, 2, 8>, a, batches, 1024, lds, s);
      case 4: return launch(spf_wms_kernel<K, 4, 8>, a, batches, 1024, lds, s);
      case 6: return launch(spf_wms_kernel<K, 6, 8>, a, batches, 1024, lds, s);
      case 8: return launch(spf_wms_kernel<K, 8, 8>, a, batches, 1024, lds, s);
      default: return launch(spf_wms_kernel<K, 10, 8>, a, batches, 1024, lds, s);
    }
  } else {
    switch (j <= 2 ? 2 : j <= 4 ? 4 : j <= 6 ? 6 : j <= 8 ? 8 : j <= 10 ? 10 : j <= 12 ? 12 : j <= 16 ? 16 : 20) {
      case 2: return launch(spf_wms_kernel<K, 2, 4>, a, batches, 1024, lds, s);
      case 4: return launch(spf_wms_kernel<K, 4, 4>, a, batches, 1024, lds, s);
      case 6: return launch(spf_wms_kernel<K, 6, 4>, a, batches, 1024, lds, s);
      case 8: return launch(spf_wms_kernel<K, 8, 4>, a, batches, 1024, lds, s);
      case 10: return launch(spf_wms_kernel<K, 10, 4>, a, batches, 1024, lds, s);
      case 12: return launch(spf_wms_kernel<K, 12, 4>, a, batches, 1024, lds, s);
      case 16: return launch(spf_wms_kernel<K, 16, 4>, a, batches, 1024, lds, s);
      default: return launch(spf_wms_kernel<K, 20, 4>, a, batches, 1024, lds, s);
    }
  }
}

uint32_t wms_sources(uint32_t n_nodes, size_t lds_limit) {
  // ORH_WMS_SOURCES=4 (A/B): 4-source batches even where 8 fit
  const char* e = getenv("ORH_WMS_SOURCES");  // read per launch (tests flip it)
  const bool four = e && atoi(e) == 4;
  return !four && n_nodes <= 10240 && wms_lds_bytes(n_nodes, 8) <= lds_limit ? 8u : 4u;
}

hipError_t launch_spf_wms(SpfArgs a, uint32_t n_rows, uint32_t wms_k, size_t lds_limit, hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  if (!a.ovf_rows || !a.wms_slots || a.n_nodes > 20480 || a.n_nodes >= 0xFFFFu) return hipErrorInvalidValue;
  a.n_rows = n_rows;
  a.row_list = nullptr;
  a.row_count = nullptr;
  hipError_t e = hipMemsetAsync(a.ovf_rows, 0, 4, s);
  if (e != hipSuccess) return e;
  // 8 sources per batch where their labels fit one CU's LDS (the rounds, the
  // barriers and the slot registers then serve twice the sources)
  const uint32_t S = wms_sources(a.n_nodes, lds_limit);
  const uint32_t batches = (n_rows + S - 1) / S;
  const size_t lds = wms_lds_bytes(a.n_nodes, S);
  if (S == 8)
    e = wms_k == 8 ? launch_wms_k<8, 8>(a, batches, lds, s) : launch_wms_k<4, 8>(a, batches, lds, s);
  else
    e = wms_k == 8 ? launch_wms_k<8, 4>(a, batches, lds, s) : launch_wms_k<4, 4>(a, batches, lds, s);
  if (e != hipSuccess) return e;
  // rows whose distances may not fit 16 bits: the u64 LDS search over the
  // list (workgroups past its length exit at once); its first-hop rows are
  // rewritten, identically, by phase 2
  a.row_list = a.ovf_rows + 1;
  a.row_count = a.ovf_rows;
  const size_t lds64 = lds_nh_bytes(a.n_nodes, false);
  return a.recs_k == 8 ? launch(spf_lds_nh_kernel<8, false>, a, n_rows, 256, lds64, s)
                       : launch(spf_lds_nh_kernel<4, false>, a, n_rows, 256, lds64, s);
}

hipError_t launch_spf(const SpfPlan& plan, SpfArgs a, uint32_t n_rows, hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  a.lds_pend_off = static_cast<uint32_t>(plan.pend_off);
  a.n_rows = n_rows;
  a.ms_pitch = plan.ms_pitch;
  a.ms_zero = a.n_nodes;
  if (plan.variant == SpfVariant::kBfsNh) {
    uint32_t block = 0, j = 0;
    size_t lds = 0;
    if (!bfs_nh_shape(a.n_nodes, a.words, SIZE_MAX, &block, &j, &lds)) return hipErrorInvalidValue;
    return plan.ell_k == 8 ? launch_bfs_nh<8>(a, n_rows, block, j, lds, s)
                           : launch_bfs_nh<4>(a, n_rows, block, j, lds, s);
  }
  return plan.ell_k == 8 ? launch_k<8>(plan, a, n_rows, s) : launch_k<4>(plan, a, n_rows, s);
}

size_t hop_lds_bytes(uint32_t max_nbr) {
  return static_cast<size_t>((2 * max_nbr + 3) & ~3u) * 4 + static_cast<size_t>(max_nbr) * 16;
}

hipError_t launch_first_hop(HopArgs a, uint32_t max_nbr, hipStream_t s, uint32_t* nodes_per_thread,
                            uint32_t* split) {
  if (a.n_out == 0) return hipSuccess;
  a.tiles = (a.n_nodes + kBlock * kHopPer - 1) / (kBlock * kHopPer);
  const uint64_t grid = static_cast<uint64_t>(a.tiles) * a.n_out;
  if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
  size_t lds = std::max<size_t>(hop_lds_bytes(max_nbr), 16);
  // ORH_HOP_LDS_MIN (experiment): reserve at least this much LDS per
  // first-hop workgroup, capping how many share a CU with the level searches
  // of other streams
  static const size_t lds_min = [] {
    const char* e = getenv("ORH_HOP_LDS_MIN");
    return e ? static_cast<size_t>(atol(e)) : size_t{0};
  }();
  lds = std::max(lds, lds_min);
  if (a.lvl_rows) {
    // 16 nodes per thread unless that leaves fewer than ~32 workgroups per CU
    // a workgroup per source walks the tiles (one gather of the source's
    // first links), split over phases while that leaves < 8192 workgroups
    const uint32_t t16 = (a.n_nodes + kBlock * 16 - 1) / (kBlock * 16);
    // ORH_HOP_NARROW=1 (A/B): 4 nodes per thread even for large batches
    // (65 instead of 158 VGPRs: waves that fit beside the MS-BFS workgroups
    // of other streams)
    static const bool narrow = [] {
      const char* e = getenv("ORH_HOP_NARROW");
      return e && atoi(e) == 1;
    }();
    const bool wide = !narrow && static_cast<uint64_t>(t16) * a.n_out >= 8192;
    // 8 nodes per thread for large batches (104 VGPRs, 8-byte row loads):
    // one C2 sweep's first hops 0.323 -> 0.292 ms against 16 per thread (158
    // VGPRs), the 4-lane step the same (profiles/r04/r_hop_nodes_ab.txt);
    // ORH_HOP_NODES=16 (A/B): the 16-node form
    static const uint32_t wide_nodes = [] {
      const char* e = getenv("ORH_HOP_NODES");
      return (e && atoi(e) == 16) ? 16u : 8u;
    }();
    const uint32_t per = wide ? wide_nodes : 4u;
    a.tiles = (a.n_nodes + kBlock * per - 1) / (kBlock * per);
    a.tile_split = 1;
    while (a.tile_split < a.tiles && static_cast<uint64_t>(a.tile_split) * a.n_out < 8192) ++a.tile_split;
    // ORH_HOP_SPLIT=n (A/B): at least n workgroups per source (tile phases)
    static const uint32_t split_min = [] {
      const char* e = getenv("ORH_HOP_SPLIT");
      return e ? static_cast<uint32_t>(std::max(1, atoi(e))) : 1u;
    }();
    a.tile_split = std::max(a.tile_split, std::min(split_min, a.tiles));
    uint64_t g2 = static_cast<uint64_t>(a.tile_split) * a.n_out;
    if (g2 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    a.n_logical = static_cast<uint32_t>(g2);
    // ORH_HOP_WG_PER_CU (A/B, default 0 = one workgroup per logical block):
    // persistent workgroups, that many per CU, for even per-source work. C2
    // sweep, first hops: 0.362 ms one per block, 0.389 ms at 8 per CU, 0.439
    // at 4 (profiles/r03/n_ms_variants_ab.txt): more workgroups in flight beat
    // fewer, longer-lived ones
    static const uint32_t per_cu = [] {
      const char* e = getenv("ORH_HOP_WG_PER_CU");
      return e ? static_cast<uint32_t>(atoi(e)) : 0u;
    }();
    static const uint32_t n_cu = [] {
      int d = 0, c = 0;
      if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
        return 0u;
      return static_cast<uint32_t>(c);
    }();
    if (a.xcd_group == 0 && per_cu && n_cu) {
      const uint64_t cap = (static_cast<uint64_t>(n_cu) * per_cu) & ~uint64_t{7};
      if (cap >= 8 && cap < g2) g2 = cap;
    }
    if (nodes_per_thread) *nodes_per_thread = per;
    if (split) *split = a.tile_split;
    return per == 16 ? launch(first_hop_lvl_kernel<16>, a, static_cast<uint32_t>(g2), kBlock, lds, s)
         : per == 8  ? launch(first_hop_lvl_kernel<8>, a, static_cast<uint32_t>(g2), kBlock, lds, s)
                     : launch(first_hop_lvl_kernel<4>, a, static_cast<uint32_t>(g2), kBlock, lds, s);
  }
  if (nodes_per_thread) *nodes_per_thread = 1;
  if (split) *split = a.tiles;
  const char* xe = getenv("ORH_HOP_XCD");  // read per launch (A/B)
  a.xcd_hop = (xe && xe[0] == '1') ? 1u : 0u;
  return launch(first_hop_kernel, a, static_cast<uint32_t>(grid), kBlock, lds, s);
}

hipError_t launch_ms_finalize(const SpfPlan& plan, SpfArgs a, uint32_t n_rows, hipStream_t s) {
  if (plan.variant != SpfVariant::kMsBfs || n_rows == 0) return hipErrorInvalidValue;
  a.n_rows = n_rows;
  if (a.ms_width == 0 || a.ms_width > plan.mask_bytes * 8) return hipErrorInvalidValue;
  const uint32_t batches = (n_rows + a.ms_width - 1) / a.ms_width;
  const uint32_t tiles = (a.n_nodes + 255) / 256;
  if (plan.mask_bytes == 2)
    hipLaunchKernelGGL(ms_finalize_kernel<uint16_t>, dim3(batches * tiles), dim3(256), 0, s, a, tiles);
  else if (plan.mask_bytes == 4)
    hipLaunchKernelGGL(ms_finalize_kernel<uint32_t>, dim3(batches * tiles), dim3(256), 0, s, a, tiles);
  else
    hipLaunchKernelGGL(ms_finalize_kernel<uint64_t>, dim3(batches * tiles), dim3(256), 0, s, a, tiles);
  return hipGetLastError();
}

// in-place mirror patch: recs[pos[i]] = vals[i] (one launch per delta batch)
__global__ __launch_bounds__(kBlock) void scatter_recs_kernel(uint2* recs, const uint32_t* pos,
                                                             const uint2* vals, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) recs[pos[i]] = vals[i];
}

__global__ __launch_bounds__(kBlock) void scatter_rows_kernel(uint2* recs, uint32_t* link, uint16_t* rank,
                                                               const uint32_t* pos, const uint2* vals,
                                                               const uint32_t* links,
                                                               const uint16_t* ranks, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t q = pos[i];
  recs[q] = vals[i];
  link[q] = links[i];
  rank[q] = ranks[i];
}

hipError_t launch_scatter_rows(uint2* recs, uint32_t* link, uint16_t* rank, const uint32_t* pos,
                               const uint2* vals, const uint32_t* links, const uint16_t* ranks,
                               uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, recs,
                     link, rank, pos, vals, links, ranks, n);
  return hipGetLastError();
}

hipError_t launch_scatter_recs(uint2* recs, const uint32_t* pos, const uint2* vals, uint32_t n,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_recs_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, recs,
                     pos, vals, n);
  return hipGetLastError();
}

hipError_t launch_exact(const ExactArgs& a, size_t lds_limit, hipStream_t s) {
  if (a.n_rows == 0) return hipSuccess;
  const size_t bytes = exact_state_bytes(a.n_nodes, a.words);
  if (bytes <= lds_limit) return launch(spf_exact_kernel<true>, a, a.n_rows, 64, bytes, s);
  if (!a.scratch) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spf_exact_kernel<false>, dim3(a.n_rows), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace orh
