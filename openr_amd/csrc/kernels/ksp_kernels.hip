// KSP2 edge-disjoint path traces over device-resident SPF rows (gfx950).
//
// LinkState::getKthPaths (LinkState.cpp:762-791): k = 1 traces over the
// source's SPF, k = 2 over a fresh SPF that ignores every k = 1 link; each is
// a run of traceOnePath (:398-419) calls sharing one visited-link set until a
// trace fails. traceOnePath is a greedy DFS from dst back to src over
// NodeSpfResult::pathLinks in insertion order; a link is consumed on first
// touch, even when its branch fails.
//
// pathLinks(v) in insertion order (runSpf, :857-873):
// the predecessors (link, p) with p transit (p == src or not overloaded), the
// link up and not ignored, and dist(p) + metric_p(link) == dist(v), ordered
// by p's extraction order - (dist(p), name rank(p)) for metrics >= 1 - and
// then by the link's position in p's LinkSet iteration. The device records of
// p's row follow that iteration order and the overflow area lies above every
// ELL slot, so the record index of the p -> v record (rev of v's record)
// orders parallel links. The DFS keeps, per frame, the key of the last
// candidate it tried; the next candidate is the smallest key above it (a
// frame's candidates are re-scanned, never stored: a WAN node has ~4).
//
// The trace is a chain of dependent loads (records, then the neighbours'
// distances, reverse records and name ranks), so a pair is latency-bound and
// the batch's pairs run side by side. Default: one wave per pair
// (ksp_trace_wave_kernel: lanes split each step's candidates, the DFS stack
// and the visited set in LDS); ORH_KSP_WAVE=0: one thread per pair
// (ksp_trace_kernel: the visited set an open-addressing table per pair and
// the stack in global memory). A pair that outgrows either, or its output
// block, is flagged and traced by the host instead.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "ksp_kernels.h"
#include "spf_kernels.h"  // edge record flags

namespace orh {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;

__device__ inline bool ign_has(const uint32_t* ign, uint32_t n, uint32_t link) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t x = ign[mid];
    if (x == link) return true;
    if (x < link) lo = mid + 1; else hi = mid;
  }
  return false;
}

// inserts link; 0 = already present, 1 = inserted, 2 = table too full
__device__ inline uint32_t visit(uint32_t* tab, uint32_t cap, uint32_t* count, uint32_t link) {
  if (2 * (*count + 1) > cap) return 2u;
  uint32_t h = (link * 0x9E3779B1u) & (cap - 1);
  for (;;) {
    const uint32_t x = tab[h];
    if (x == link + 1) return 0u;
    if (x == 0u) {
      tab[h] = link + 1;
      ++*count;
      return 1u;
    }
    h = (h + 1) & (cap - 1);
  }
}

struct Cand {
  uint32_t dp, rank, q2, link, prev;
  bool valid;
};

__device__ inline bool key_less(uint32_t ad, uint32_t ar, uint32_t aq, uint32_t bd, uint32_t br, uint32_t bq) {
  if (ad != bd) return ad < bd;
  if (ar != br) return ar < br;
  return aq < bq;
}

// the smallest pathLinks candidate of v above the frame's last key
template <int K>
__device__ inline Cand next_cand(const KspArgs& a, const uint32_t* d, uint32_t s, uint32_t v, const KspFrame& f,
                                 const uint32_t* ign, uint32_t n_ign) {
  Cand best{0, 0, 0, 0, 0, false};
  const uint32_t dv = d[v];
  auto consider = [&](const uint2& rec, uint32_t q) {
    const uint32_t p = rec.x & ORH_REC_COL_MASK;
    const uint32_t dp = d[p];
    if (dp == kInf) return;
    const uint32_t l = a.link[q];
    if (n_ign && ign_has(ign, n_ign, l)) return;
    const uint32_t q2 = a.rev[q];
    const uint2 back = a.recs[q2];  // p -> v: p's metric, p's overload bit
    if (p != s && (back.x & ORH_REC_ROW_OVL)) return;
    if (static_cast<uint64_t>(dp) + back.y != dv) return;
    const uint32_t rk = a.name_rank[p];
    if (f.has && !key_less(f.dp, f.rank, f.q2, dp, rk, q2)) return;
    if (!best.valid || key_less(dp, rk, q2, best.dp, best.rank, best.q2)) best = Cand{dp, rk, q2, l, p, true};
  };
  const uint2* slots = a.recs + static_cast<size_t>(v) * K;
  uint2 r[K];
#pragma unroll
  for (int j = 0; j < K; ++j) r[j] = slots[j];
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (!(r[j].x & (ORH_REC_SKIP | ORH_REC_CONT))) consider(r[j], static_cast<uint32_t>(v * K + j));
  if (r[K - 1].x & ORH_REC_CONT) {
    const uint32_t start = r[K - 1].x & ORH_REC_COL_MASK;
    for (uint32_t q = 0; q < r[K - 1].y; ++q) {
      const uint2 o = a.recs[start + q];
      if (!(o.x & ORH_REC_SKIP)) consider(o, start + q);
    }
  }
  return best;
}

template <int K>
__global__ __launch_bounds__(64) void ksp_trace_kernel(KspArgs a) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= a.n_pairs) return;
  const uint32_t N = a.n_nodes;
  uint32_t* blk = a.out + static_cast<size_t>(i) * a.out_cap;
  uint32_t w;
  if (a.k == 1) {
    blk[0] = 0u;
    w = 2;
  } else {
    if (blk[0] != 0u) return;  // the host traces this pair
    w = blk[1];
  }
  const uint32_t s = a.src[i], t = a.dst[i];
  const uint32_t* d = a.dist + static_cast<size_t>(a.row[i]) * N;
  uint32_t* ign = a.ign + static_cast<size_t>(i) * a.ign_cap;
  const uint32_t n_ign = a.k == 2 ? a.ign_cap : 0u;
  const uint32_t n_pos = w;
  blk[w++] = 0u;
  uint32_t n_paths = 0, n_links = 0, status = 0;
  // k = 2 without k = 1 paths: the memoized row serves and dst is unreachable
  // or the source itself, so there are none (LinkState.cpp:775-777)
  const bool run = (a.k == 1 || a.need2[i]) && s != t && d[t] != kInf;
  if (run) {
    uint32_t* tab = a.visited + static_cast<size_t>(i) * a.hash_cap;
    KspFrame* st = a.stack + static_cast<size_t>(i) * a.stack_cap;
    uint32_t count = 0;
    for (;;) {  // successive traces sharing the visited set (:778-787)
      int top = 0;
      st[0] = KspFrame{t, 0u, 0u, 0u, 0u, 0u};
      bool found = false;
      while (top >= 0) {
        KspFrame f = st[top];
        if (f.v == s) {
          found = true;
          break;
        }
        const Cand c = next_cand<K>(a, d, s, f.v, f, ign, n_ign);
        if (!c.valid) {  // every candidate tried: this branch fails
          --top;
          continue;
        }
        f.has = 1u;
        f.dp = c.dp;
        f.rank = c.rank;
        f.q2 = c.q2;
        const uint32_t ins = visit(tab, a.hash_cap, &count, c.link);
        if (ins == 2u || (ins == 1u && static_cast<uint32_t>(top) + 1 >= a.stack_cap)) {
          status = kKspOverflow;
          break;
        }
        if (ins == 1u) {  // consumed on first touch; descend
          f.link = c.link;
          st[top] = f;
          st[++top] = KspFrame{c.prev, 0u, 0u, 0u, 0u, 0u};
        } else {
          st[top] = f;  // already consumed: the next candidate
        }
      }
      if (status || !found) break;
      const uint32_t len = static_cast<uint32_t>(top);  // links from src (frame top) to dst (frame 0)
      if (w + 1 + len + 1 > a.out_cap || (a.k == 1 && n_links + len > a.ign_cap)) {
        status = kKspOverflow;
        break;
      }
      blk[w++] = len;
      for (int j = top - 1; j >= 0; --j) {
        const uint32_t l = st[j].link;
        blk[w++] = l;
        if (a.k == 1) ign[n_links++] = l;
      }
      ++n_paths;
    }
  }
  if (status) {
    blk[0] = status;
    if (a.k == 1) a.need2[i] = 0u;
    return;
  }
  blk[n_pos] = n_paths;
  if (a.k == 1) {
    blk[1] = w;
    a.need2[i] = n_paths ? 1u : 0u;
    // the k = 2 ignore set: the k = 1 paths' links (edge-disjoint, so no
    // duplicates), sorted for the searches' binary search, padded with ~0u
    for (uint32_t x = 1; x < n_links; ++x) {
      const uint32_t v = ign[x];
      uint32_t y = x;
      for (; y > 0 && ign[y - 1] > v; --y) ign[y] = ign[y - 1];
      ign[y] = v;
    }
    for (uint32_t x = n_links; x < a.ign_cap; ++x) ign[x] = ~0u;
  }
}

// ---------------------------------------------------------------------------
// one wave per pair (default)
// ---------------------------------------------------------------------------
// The same traces with the pair's DFS state in LDS and the wave's 64 lanes
// working each step together: lane j evaluates the j-th candidate record of
// the frame's node (ELL slot j, then the overflow records), a wave argmin
// picks the smallest key above the frame's last one, the visited-link set is
// probed 64 slots per LDS read, and a found path's links are written by all
// lanes. Control flow is uniform per wave (one pair), so a pair never waits
// for the divergent branches of other pairs as in one thread per pair, and
// the stack and the visited set cost LDS round trips, not global ones.
constexpr uint32_t kWaveWaves = 4;     // pairs per workgroup
constexpr uint32_t kWaveStack = 512;   // DFS frames per pair (deeper: the host traces it)
constexpr uint32_t kWaveHash = 1024;   // visited-set slots per pair (power of two)

__device__ inline uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(x), off));
    const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(x >> 32), off));
    const uint64_t y = (static_cast<uint64_t>(hi) << 32) | lo;
    x = y < x ? y : x;
  }
  return x;
}

template <int K>
__global__ __launch_bounds__(kWaveWaves * 64) void ksp_trace_wave_kernel(KspArgs a) {
  __shared__ KspFrame s_stack[kWaveWaves][kWaveStack];
  __shared__ uint32_t s_tab[kWaveWaves][kWaveHash];
  const uint32_t wv = threadIdx.x / 64u, lane = threadIdx.x % 64u;
  const uint32_t i = blockIdx.x * kWaveWaves + wv;
  if (i >= a.n_pairs) return;  // the whole wave: nothing below syncs the workgroup
  const uint32_t N = a.n_nodes;
  uint32_t* blk = a.out + static_cast<size_t>(i) * a.out_cap;
  uint32_t w;
  if (a.k == 1) {
    w = 2;
  } else {
    if (blk[0] != 0u) return;  // the host traces this pair
    w = blk[1];
  }
  const uint32_t s = a.src[i], t = a.dst[i];
  const uint32_t* d = a.dist + static_cast<size_t>(a.row[i]) * N;
  uint32_t* ign = a.ign + static_cast<size_t>(i) * a.ign_cap;
  const uint32_t n_ign = a.k == 2 ? a.ign_cap : 0u;
  const uint32_t n_pos = w++;
  uint32_t n_paths = 0, n_links = 0, status = 0;
  KspFrame* st = s_stack[wv];
  uint32_t* tab = s_tab[wv];
  const bool run = (a.k == 1 || a.need2[i]) && s != t && d[t] != kInf;
  if (run) {
    for (uint32_t x = lane; x < kWaveHash; x += 64) tab[x] = 0u;
    uint32_t count = 0;
    for (;;) {  // successive traces sharing the visited set (:778-787)
      int top = 0;
      KspFrame f{t, 0u, 0u, 0u, 0u, 0u};  // the top frame, kept in registers
      bool found = false;
      while (top >= 0) {
        if (f.v == s) {
          found = true;
          break;
        }
        // candidates of f.v: lane j takes virtual slot j (ELL slots, then the
        // overflow records), in passes of 64
        const uint32_t dv = d[f.v];
        const uint2* slots = a.recs + static_cast<size_t>(f.v) * K;
        const uint2 lastr = slots[K - 1];
        const bool cont = (lastr.x & ORH_REC_CONT) != 0u;
        const uint32_t n_virt = cont ? (K - 1) + lastr.y : K;
        uint64_t best1 = ~0ull;
        uint32_t best_q2 = ~0u, best_link = 0, best_prev = 0;
        for (uint32_t base = 0; base < n_virt; base += 64) {
          const uint32_t j = base + lane;
          uint64_t key1 = ~0ull;
          uint32_t q2 = ~0u, l = 0, p = 0;
          if (j < n_virt) {
            const uint32_t q = j < K - (cont ? 1u : 0u) ? f.v * K + j
                                                        : (lastr.x & ORH_REC_COL_MASK) + (j - (K - 1));
            const uint2 rec = a.recs[q];
            if (!(rec.x & (ORH_REC_SKIP | ORH_REC_CONT))) {
              p = rec.x & ORH_REC_COL_MASK;
              const uint32_t dp = d[p];
              l = a.link[q];
              if (dp != kInf && !(n_ign && ign_has(ign, n_ign, l))) {
                const uint32_t qq = a.rev[q];
                const uint2 back = a.recs[qq];  // p -> v: p's metric and overload bit
                if ((p == s || !(back.x & ORH_REC_ROW_OVL)) && static_cast<uint64_t>(dp) + back.y == dv) {
                  const uint32_t rk = a.name_rank[p];
                  if (!f.has || key_less(f.dp, f.rank, f.q2, dp, rk, qq)) {
                    key1 = (static_cast<uint64_t>(dp) << 32) | rk;
                    q2 = qq;
                  }
                }
              }
            }
          }
          // wave argmin of (dp, rank, q2): q2 (a record index) is unique
          const uint64_t m1 = wave_min_u64(key1);
          if (m1 == ~0ull) continue;
          const uint32_t m2 = static_cast<uint32_t>(wave_min_u64(key1 == m1 ? q2 : ~0u));
          const uint64_t win = __ballot(key1 == m1 && q2 == m2);
          const int wl = static_cast<int>(__builtin_ctzll(win));
          if (m1 < best1 || (m1 == best1 && m2 < best_q2)) {
            best1 = m1;
            best_q2 = m2;
            best_link = static_cast<uint32_t>(__shfl(static_cast<int>(l), wl));
            best_prev = static_cast<uint32_t>(__shfl(static_cast<int>(p), wl));
          }
        }
        if (best1 == ~0ull) {  // every candidate tried: this branch fails
          if (--top >= 0) f = st[top];
          continue;
        }
        f.has = 1u;
        f.dp = static_cast<uint32_t>(best1 >> 32);
        f.rank = static_cast<uint32_t>(best1);
        f.q2 = best_q2;
        // visit(link): probe 64 slots per LDS read; a present link lies
        // before the first empty slot of its probe sequence
        uint32_t ins = 2u;  // 0 present, 1 inserted, 2 set too full
        if (2 * (count + 1) <= kWaveHash) {
          uint32_t h = (best_link * 0x9E3779B1u) & (kWaveHash - 1);
          for (uint32_t probed = 0; probed < kWaveHash; probed += 64) {
            const uint32_t x = tab[(h + lane) & (kWaveHash - 1)];
            const uint64_t hit = __ballot(x == best_link + 1);
            const uint64_t empty = __ballot(x == 0u);
            const uint64_t before = empty ? (empty & (~empty + 1)) - 1 : ~0ull;  // lanes before the first empty
            if (hit & before) {
              ins = 0u;
              break;
            }
            if (empty) {
              const uint32_t at = (h + static_cast<uint32_t>(__builtin_ctzll(empty))) & (kWaveHash - 1);
              if (lane == 0) tab[at] = best_link + 1;
              ++count;
              ins = 1u;
              break;
            }
            h = (h + 64) & (kWaveHash - 1);
          }
        }
        if (ins == 2u || (ins == 1u && static_cast<uint32_t>(top) + 1 >= kWaveStack)) {
          status = kKspOverflow;
          break;
        }
        if (ins == 1u) {  // consumed on first touch; descend
          f.link = best_link;
          if (lane == 0) st[top] = f;
          ++top;
          f = KspFrame{best_prev, 0u, 0u, 0u, 0u, 0u};
        }
        // already consumed: the next candidate of the same frame
      }
      if (status || !found) break;
      const uint32_t len = static_cast<uint32_t>(top);  // links from src (frame top) to dst (frame 0)
      if (w + 1 + len + 1 > a.out_cap || (a.k == 1 && n_links + len > a.ign_cap)) {
        status = kKspOverflow;
        break;
      }
      if (lane == 0) blk[w] = len;
      for (uint32_t j = lane; j < len; j += 64) {
        const uint32_t l = st[top - 1 - static_cast<int>(j)].link;
        blk[w + 1 + j] = l;
        if (a.k == 1) ign[n_links + j] = l;
      }
      w += 1 + len;
      if (a.k == 1) n_links += len;
      ++n_paths;
    }
  }
  if (status) {
    if (lane == 0) {
      blk[0] = status;
      if (a.k == 1) a.need2[i] = 0u;
    }
    return;
  }
  if (lane == 0) {
    blk[n_pos] = n_paths;
    if (a.k == 1) {
      blk[0] = 0u;
      blk[1] = w;
      a.need2[i] = n_paths ? 1u : 0u;
    }
  }
  if (a.k == 1) {
    // the k = 2 ignore set sorted (rank sort: the k = 1 links are distinct,
    // the paths being edge-disjoint), padded with ~0u
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t x = lane; x < n_links; x += 64) tab[x] = ign[x];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t x = lane; x < n_links; x += 64) {
      const uint32_t v = tab[x];
      uint32_t r = 0;
      for (uint32_t y = 0; y < n_links; ++y) r += tab[y] < v ? 1u : 0u;
      ign[r] = v;
    }
    for (uint32_t x = n_links + lane; x < a.ign_cap; x += 64) ign[x] = ~0u;
  }
}

}  // namespace

namespace {
constexpr uint32_t kOrderMax = 4096;

// rank of pair i = pairs with a larger key, or an equal key and a smaller
// index (a stable descending order); keys in LDS, P^2 / 1024 compares a thread
__global__ __launch_bounds__(1024) void ksp_order_kernel(const uint32_t* dist1, const uint32_t* row1,
                                                         const uint32_t* dst, const uint32_t* need2, uint32_t N,
                                                         uint32_t P, uint32_t* order) {
  __shared__ uint32_t key[kOrderMax];
  for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
    const uint32_t d = need2[i] ? dist1[static_cast<size_t>(row1[i]) * N + dst[i]] : 0u;
    key[i] = need2[i] ? (d == 0xFFFFFFFFu ? 0xFFFFFFFEu : d) + 1u : 0u;  // searching pairs above the rest
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
    const uint32_t k = key[i];
    uint32_t r = 0;
    for (uint32_t j = 0; j < P; ++j) {
      const uint32_t x = key[j];  // the same j for the whole wave: an LDS broadcast
      r += (x > k || (x == k && j < i)) ? 1u : 0u;
    }
    order[r] = i;
  }
}
}  // namespace

hipError_t launch_ksp_order(const uint32_t* dist1, const uint32_t* row1, const uint32_t* dst,
                            const uint32_t* need2, uint32_t n_nodes, uint32_t n_pairs, uint32_t* order,
                            hipStream_t s) {
  if (n_pairs == 0) return hipSuccess;
  if (n_pairs > kOrderMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ksp_order_kernel, dim3(1), dim3(1024), 0, s, dist1, row1, dst, need2, n_nodes, n_pairs, order);
  return hipGetLastError();
}

hipError_t launch_ksp_trace(const KspArgs& a, uint32_t ell_k, hipStream_t s) {
  if (a.n_pairs == 0) return hipSuccess;
  if ((a.hash_cap & (a.hash_cap - 1)) != 0 || a.out_cap < 4 || a.stack_cap < 2) return hipErrorInvalidValue;
  if (ell_k != 4 && ell_k != 8) return hipErrorInvalidValue;
  // ORH_KSP_WAVE=0: one thread per pair (A/B)
  static const bool wave = !getenv("ORH_KSP_WAVE") || atoi(getenv("ORH_KSP_WAVE")) != 0;
  if (wave && a.ign_cap <= kWaveHash) {
    const dim3 grid((a.n_pairs + kWaveWaves - 1) / kWaveWaves);
    if (ell_k == 8) hipLaunchKernelGGL(ksp_trace_wave_kernel<8>, grid, dim3(kWaveWaves * 64), 0, s, a);
    else hipLaunchKernelGGL(ksp_trace_wave_kernel<4>, grid, dim3(kWaveWaves * 64), 0, s, a);
    return hipGetLastError();
  }
  const dim3 grid((a.n_pairs + 63) / 64);
  if (ell_k == 8) hipLaunchKernelGGL(ksp_trace_kernel<8>, grid, dim3(64), 0, s, a);
  else hipLaunchKernelGGL(ksp_trace_kernel<4>, grid, dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace orh
