// ============================================================================
//  whatif.hip -- what-if batches: the SPF of one source re-run for every
//  single-link failure of a list, reduced to a
//  per-failure digest.
//
//  Reference semantics per failure l: runSpf(src, true, {l})
//  (openr/decision/LinkState.cpp:808-882 with linksToIgnore = {l}, the
//  primitive getKthPaths uses at :776-779), compared with runSpf(src).
//
//  Exact incremental evaluation instead of one full Dijkstra per failure:
//    * l is "cold" when neither direction is a tight edge of the unfailed
//      shortest-path DAG (tail expanded, d(tail) + w = d(head)).  Removing a
//      link that no shortest path uses changes no distance, no pathLinks and
//      so no next hop: the digest is the unfailed one.
//    * l is "hot" when a -> b is tight (one direction at most: metrics are
//      positive).  Only D = the DAG descendants of b (b included) can change:
//      a node outside D has no tight path through a -> b, keeps its distance
//      and its tight predecessors, none of which is in D.  On D:
//        - distances: seeds from in-edges leaving nodes outside D (exact,
//          unchanged) and a label-correcting sweep inside D;
//        - next hops: nh(v) = union over tight expanded predecessors u of
//          ({v} if u = src else nh(u)) -- the reference's addNextHops rule
//          (:867-872) -- iterated to its fixed point (monotone union over a
//          DAG, so the least fixed point is the Dijkstra result);
//        - the digest delta is summed over D.
//  Teams: a wave per hot failure while |D| fits its scratch (4096 nodes),
//  the rest re-done by whole 1024-thread workgroups with room for all nodes.
//
//  Digest of a result (same definition in oracle/spf_oracle.cpp):
//    n_dist_changed, n_nh_changed (a node becoming unreachable counts in both)
//    hash = sum over reachable v of mix(mix(v + 1) + d(v)) ^ fnv(nh(v) words)
//  with nh(v) a bitset over the distinct up neighbours of src in the unfailed
//  graph (ascending id).
// ============================================================================
#include "engine_internal.h"
#include "wave_ops.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

using namespace spfi;

namespace {

constexpr uint32_t kBusy = 0xFFFFFFFEu;
constexpr uint32_t kWaveCap = 1024;            // |D| a wave team can hold
constexpr size_t kBigScratch = 8ull << 30;     // HBM budget of the workgroup teams (both sets)
constexpr size_t kWaveScratch = 8ull << 30;    // HBM budget of the wave teams
constexpr uint32_t kDialLevels = 1024;         // distinct distances settled bucket by bucket

__device__ __forceinline__ uint32_t ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-wide minimum with DPP moves (row shifts, then row broadcasts; lanes
// with no source keep ~0u) -- __shfl compiles to ds_bpermute, an LDS round
// trip per step.  Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return __builtin_amdgcn_readlane(x, 63);
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct WiGraph {
  const uint32_t* row_ptr;
  const uint32_t* col;
  const uint32_t* wt;
  const uint32_t* rev;
  const uint32_t* link;
  const uint8_t* ovl;
  const uint32_t* nbr_bit;  // [N] j if v is the src's j-th distinct neighbour, else kInf
  uint32_t N, src, W;
  uint32_t hop = 0;  // hop counts: every up link weighs 1 (useLinkMetric = false)
  uint32_t* fault = nullptr;  // the context's barrier-timeout word (spf_device_check)
  // per CSR edge, interleaved: {col, wt, link, wt of the reverse edge} -- one
  // 16-byte load where the wave teams' repairs read four arrays (and the
  // rev -> wt chain) at random nodes (what-if plans)
  const uint4* ed = nullptr;
};

// directed weight of the edge reverse to e (tail -> head of the in-edge)
__device__ __forceinline__ uint32_t in_w(const WiGraph& g, uint32_t e) {
  return g.hop ? 1u : g.wt[g.rev[e]];
}

struct WiBase {
  const uint32_t* dist;  // [N] unfailed distances
  const uint32_t* nhb;   // [N][W] unfailed next-hop bitsets
  const unsigned long long* H;  // unfailed hash
};

// ---------------------------------------------------------------------------
//  grid-synchronised (XGrid) single-source SSSP and unfailed result
// ---------------------------------------------------------------------------
constexpr int kCoopThreads = 512;  // one block per CU: always co-resident
constexpr uint32_t kCoopHubDeg = 32;  // nodes above this degree get a whole wave

// Grid barrier of the grid-resident kernels, XCD-hierarchical (MI355X_MICROARCH
// barrier-xcd: 4.1 us at 256 workgroups against 26.3 us for the software
// cooperative_groups grid sync, which the what-if base pass crossed ~70
// times).  Blocks are grouped by blockIdx % 8 (the XCD round-robin of the
// dispatcher); each arrival bumps its group's counter, the group's last
// arrival bumps the top counter, waits for every group and publishes the
// generation its group polls.  Counters only grow within a launch (the k-th
// barrier completes at k arrivals per block) and are zeroed before each
// launch (kGridBarWords words, one 128-byte line per counter).
constexpr uint32_t kBarPad = 32;
constexpr uint32_t kGridBarWords = 17 * kBarPad;  // cnt[8], top, gen[8]
constexpr uint32_t kBarSpin = 1u << 26;            // ~seconds: never a silent hang

// A barrier spin that ran out (a member never arrived: not co-resident, or
// a fault) sets the launching context's fault word and falls through; the
// host reads and clears it (spf_device_check) and reports SPF_E_HIP instead
// of the launch's output.  One word per context (spf_ctx::d_fault), so a
// check on one context neither reports nor clears another's timeout.
__device__ __forceinline__ void barrier_timed_out(uint32_t* fault) {
  if (fault) __hip_atomic_fetch_or(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A repair loop that reached its iteration bound (it cannot, for a correct
// kernel: every bound is the loop's worst case + 2) reports where instead of
// spinning on: bit 3 of the fault word, the phase in bits 8-15
// (spf_device_check names it).  1 D discovery, 2 label-correcting sweeps,
// 3 next-hop fixed point.
__device__ __forceinline__ void loop_bound_hit(uint32_t* fault, uint32_t phase) {
  if (fault)
    __hip_atomic_fetch_or(fault, 8u | (phase << 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// After one barrier timed out the launch's results are void; later barriers
// must not each wait out their own spin (a desynchronised team would cross
// thousands of them): a spin polls the fault word every 1024 polls and gives
// up once it is set.
__device__ __forceinline__ bool fault_set(const uint32_t* fault) {
  return fault && __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

struct XGrid {
  uint32_t* bar;
  uint32_t* fault;
  __device__ void sync() const {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores drained
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t nb = gridDim.x, x = blockIdx.x & 7u;
      const uint32_t nx = (nb - x + 7u) / 8u;  // blocks of this group (>= 1)
      const uint32_t ngroups = nb < 8u ? nb : 8u;
      uint32_t* top = bar + 8 * kBarPad;
      uint32_t* gen = bar + (9 + x) * kBarPad;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t t =
          __hip_atomic_fetch_add(bar + x * kBarPad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t g = t / nx + 1;  // the generation this arrival completes
      uint32_t k = 0;
      if (t % nx == nx - 1) {         // last of its group: the group's leader
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (; k < kBarSpin &&
               __hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g * ngroups;
             ++k) {
          if ((k & 1023u) == 1023u && fault_set(fault)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(gen, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (; k < kBarSpin &&
               __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g;
             ++k) {
          if ((k & 1023u) == 1023u && fault_set(fault)) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (k == kBarSpin) barrier_timed_out(fault);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
};

// inclusive prefix sum over the wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// ---------------------------------------------------------------------------
//  wave helpers of the repairs: lanes over flattened edges
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_pull(uint32_t x, uint32_t k) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)x);
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The edges of up to 64 nodes (lane k holds node v, `valid`), flattened:
// chunks of 64 (node slot, edge) pairs.  f(k, e, act) runs on every lane of
// the wave (so it may ballot / pull); `act` marks the lanes holding an edge,
// k is the node slot (lane) that edge belongs to.  All 64 lanes must be
// active.
template <class F>
__device__ __forceinline__ void wave_edges(const uint32_t* __restrict__ row_ptr, uint32_t v,
                                           bool valid, F&& f) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t b0 = 0, deg = 0;
  if (valid) {
    b0 = row_ptr[v];
    deg = row_ptr[v + 1] - b0;
  }
  const uint32_t incl = wave_incl_scan32(deg);
  const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
  const uint32_t excl = incl - deg;
  for (uint32_t base = 0; base < total; base += 64) {
    const uint32_t s = base + lane;
    // owner: the last slot whose first edge is <= s (slots with no edges
    // share their successor's offset and lose to it)
    uint32_t k = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1)
      if (lane_pull(excl, k + step) <= s) k += step;
    const uint32_t e = lane_pull(b0, k) + s - lane_pull(excl, k);
    f(k, e, s < total);
  }
}

struct CoopSssp {
  const uint32_t* row_ptr;
  const uint32_t* col;
  const uint32_t* wt;
  const uint8_t* ovl;
  const uint32_t* link;
  const uint32_t* ign;  // optional link bitmap
  uint32_t N, src, hop;
  uint32_t* dist;
  uint32_t* qa;
  uint32_t* qb;
  uint32_t* bm;   // [ceil(N/32)] next-frontier bitmap
  uint32_t* ctr;  // [4] rotating queue lengths + spare
  uint32_t* bar = nullptr;  // [kGridBarWords] XGrid counters, zero at launch
  uint32_t* fault = nullptr;  // the context's barrier-timeout word
};

// Frontier Bellman-Ford over the whole grid: expansion, grid barrier,
// bitmap compaction into the other queue, grid barrier.  Data written by
// other workgroups is read with agent-scope atomics (ld) or atomicExch.
__device__ void coop_sssp(const XGrid& grid, const CoopSssp& a) {
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t gsz = gridDim.x * blockDim.x;  // a multiple of 64
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t bm_words = (a.N + 31) / 32;
  for (uint32_t v = gtid; v < a.N; v += gsz) st(&a.dist[v], v == a.src ? 0u : kInf);
  for (uint32_t i = gtid; i < bm_words; i += gsz) st(&a.bm[i], 0u);
  if (gtid == 0) {
    st(&a.qa[0], a.src);
    st(&a.ctr[0], 1u);
    st(&a.ctr[1], 0u);
    st(&a.ctr[2], 0u);
  }
  grid.sync();
  for (uint32_t it = 0;; ++it) {
    const uint32_t len = ld(&a.ctr[it % 3]);
    if (len == 0) break;
    const uint32_t* cur = (it & 1) ? a.qb : a.qa;
    uint32_t* nxt = (it & 1) ? a.qa : a.qb;
    uint32_t* nctr = &a.ctr[(it + 1) % 3];
    if (gtid == 0) st(&a.ctr[(it + 2) % 3], 0u);  // read last at iteration it - 1
    // wave-uniform sweep over the frontier: a lane expands its own node
    // unless the node is a hub (degree > kCoopHubDeg), whose edges the whole
    // wave then relaxes together -- one thread walking a scale-free hub's
    // thousands of returning atomics serially was the critical path
    auto relax = [&](uint32_t e, uint32_t du) {
      if (a.ign && ((a.ign[a.link[e] >> 5] >> (a.link[e] & 31)) & 1u)) return;
      const uint32_t v = a.col[e];
      const uint32_t nd = du + (a.hop ? 1u : a.wt[e]);
      if (nd < atomicMin(&a.dist[v], nd)) atomicOr(&a.bm[v >> 5], 1u << (v & 31));
    };
    // a wave takes 64 frontier nodes at a time, lanes over their flattened
    // out-edges (wave_edges): a node's relaxations go out 64 at a time
    // instead of one returning atomic after another per lane (a degree-30
    // node was 30 dependent round trips of the iteration's critical path)
    for (uint32_t b = gtid - lane; b < len; b += gsz) {
      const uint32_t i = b + lane;
      uint32_t u = 0, du = 0;
      bool x = false;
      if (i < len) {
        u = ld(&cur[i]);
        x = !a.ovl[u] || u == a.src;  // drained: recorded, not expanded
        if (x) du = ld(&a.dist[u]);
      }
      wave_edges(a.row_ptr, u, x, [&](uint32_t k, uint32_t e, bool act) {
        const uint32_t dk = lane_pull(du, k);
        if (act) relax(e, dk);
      });
    }
    grid.sync();
    for (uint32_t wb = gtid - lane; wb < bm_words; wb += gsz) {  // wave-uniform
      const uint32_t w = wb + lane;
      uint32_t word = w < bm_words ? atomicExch(&a.bm[w], 0u) : 0u;
      // one queue-counter atomic per wave (a returning atomic per word on one
      // counter serialises at ~88 per us)
      const uint32_t cnt = (uint32_t)__popc(word);
      const uint32_t incl = wave_incl_scan32(cnt);
      const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
      if (!total) continue;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(nctr, total);
      base = __builtin_amdgcn_readlane(base, 0);
      uint32_t at = base + incl - cnt;
      while (word) {
        const uint32_t b = __ffs(word) - 1;
        word &= word - 1;
        st(&nxt[at++], w * 32 + b);
      }
    }
    grid.sync();
  }
}

__global__ __launch_bounds__(kCoopThreads) void gsssp_coop_kernel(CoopSssp a) {
  const XGrid grid{a.bar, a.fault};
  coop_sssp(grid, a);
}

// The unfailed result of a what-if batch in one grid-resident launch:
// SPF, next-hop bitsets in distance order (bucketed by distance value when
// at most kMaxLevels distinct values occur, fixed-point sweeps otherwise),
// result hash.
constexpr uint32_t kLevelCap = 1u << 16;  // distance values bucketed directly
constexpr uint32_t kMaxLevels = 1024;     // non-empty levels worth a barrier each
constexpr uint32_t kLdsHist = 4096;       // distance values a block histograms in LDS

struct BaseArgs {
  CoopSssp sp;
  WiGraph g;
  uint32_t* nhb;        // [N][W]
  uint32_t* lvl;        // [kLevelCap + 1] bucket counts / offsets
  uint32_t* order;      // [N] nodes by distance
  uint32_t* misc;       // [8]: 0 max dist, 1 nonempty levels, 2..4 flags
  unsigned long long* H;
  unsigned long long* prof;  // SPF_WHATIF_PROF: [16] phase clocks of block 0
  uint32_t* parent;     // [N] one tight expanded predecessor (levels path)
  uint32_t* sub;        // [N] subtree sizes of the parent tree, 0 without levels
  unsigned long long* lprof = nullptr;  // SPF_WHATIF_PROF: [2 x 64] per-level clock, size
};

// word j of nh(v) from v's in-edges first, first + stride, ... (a wave
// splits a hub's edges over its lanes and ORs the parts)
__device__ __forceinline__ uint32_t nh_word(const WiGraph& g, const uint32_t* dist,
                                            const uint32_t* nhb, uint32_t v, uint32_t j,
                                            uint32_t first = 0, uint32_t stride = 1) {
  // edges in groups of 4, each stage's loads issued together: the column and
  // reverse-edge ids, then the tails' distances / drain bytes / metrics, then
  // the tight tails' words -- three memory round trips per group where an
  // edge-at-a-time loop made three per edge
  const uint32_t dv = dist[v];
  uint32_t acc = 0;
  const uint32_t e1 = g.row_ptr[v + 1];
  for (uint32_t e = g.row_ptr[v] + first; e < e1; e += 4 * stride) {
    uint32_t u[4], r[4], du[4], w[4], x[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t ek = e + k * stride;
      ok[k] = ek < e1;
      u[k] = ok[k] ? g.col[ek] : 0u;
      r[k] = ok[k] && !g.hop ? g.rev[ek] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      du[k] = ok[k] ? ld(&dist[u[k]]) : kInf;
      w[k] = ok[k] ? (g.hop ? 1u : g.wt[r[k]]) : 0u;
      if (ok[k] && g.ovl[u[k]] && u[k] != g.src) du[k] = kInf;  // drained: not expanded
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[k] = 0;
      if (du[k] != kInf && du[k] + w[k] == dv) {
        if (u[k] == g.src) {
          const uint32_t jb = g.nbr_bit[v];
          if ((jb >> 5) == j) x[k] = 1u << (jb & 31);
        } else {
          x[k] = ld(&nhb[(size_t)u[k] * g.W + j]);
        }
      }
    }
    acc |= x[0] | x[1] | x[2] | x[3];
  }
  return acc;
}

// nh(v) of a hub by one wave: lanes test v's in-edges 64 at a time, then
// every tight predecessor's W words are ORed in with lane = word (a (v, j)
// item per thread would rescan the hub's edges W times)
__device__ void hub_nh(const WiGraph& g, const uint32_t* dist, uint32_t* nhb, uint32_t* parent,
                       uint32_t v, uint32_t lane) {
  const uint32_t dv = dist[v], W = g.W;
  const uint32_t e0 = g.row_ptr[v], e1 = g.row_ptr[v + 1];
  bool have_parent = false;
  for (uint32_t j0 = 0; j0 < W; j0 += 64) {
    const uint32_t j = j0 + lane;
    uint32_t acc = 0;
    // 4 chunks of 64 in-edges per pass, each stage's loads issued together
    // (ids, then the tails' distances / drains / metrics): a hub's scan was
    // one dependent round trip chain per 64 edges and set its level's time
    for (uint32_t eb4 = e0; eb4 < e1; eb4 += 256) {
    uint32_t cu4[4], r4[4], u4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t e = eb4 + q * 64 + lane;
      cu4[q] = e < e1 ? g.col[e] : kInf;
      r4[q] = e < e1 && !g.hop ? g.rev[e] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u4[q] = kInf;
      if (cu4[q] != kInf) {
        const uint32_t cu = cu4[q];
        const uint32_t du = ld(&dist[cu]);
        const uint32_t w = g.hop ? 1u : g.wt[r4[q]];
        if ((!g.ovl[cu] || cu == g.src) && du != kInf && du + w == dv) u4[q] = cu;
      }
    }
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {  // chunks in CSR order: the first tight tail is the parent
      const uint32_t u = u4[c4];
      const uint64_t tight = __ballot(u != kInf);
      if (tight && !have_parent) {  // wave-uniform
        have_parent = true;
        const uint32_t first = __builtin_amdgcn_readlane(u, __builtin_ctzll(tight));
        if (lane == 0) st(&parent[v], first);
      }
      // the tight tails' words 8 at a time, their loads issued together
      for (uint64_t t = tight; t;) {
        uint32_t tu[8], x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          tu[q] = kInf;
          if (t) {  // wave-uniform
            tu[q] = __builtin_amdgcn_readlane(u, __builtin_ctzll(t));
            t &= t - 1;
          }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
          x[q] = tu[q] != kInf && tu[q] != g.src && j < W ? ld(&nhb[(size_t)tu[q] * W + j]) : 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          acc |= x[q];
          if (tu[q] == g.src) {
            const uint32_t jb = g.nbr_bit[v];
            if (j == (jb >> 5)) acc |= 1u << (jb & 31);
          }
        }
      }
    }
    }
    if (j < W) st(&nhb[(size_t)v * W + j], acc);
  }
}

// nh(v) and parent[v] of a non-hub node (degree <= kCoopHubDeg) by a
// segment of S lanes (S = a power of two >= min(W, 64), 64 / S nodes per
// wave, segment-uniform call): lane l of the segment tests in-edges l, l + S,
// ... once, then every tight tail's words are ORed in with lane = word.  An
// item per (v, word) instead rescans v's in-edges W times (what-if base:
// W = 31, next hops 4.3 ms of the 5.7 ms pass, r02_v61).
__device__ void seg_nh(const WiGraph& g, const uint32_t* dist, uint32_t* nhb, uint32_t* parent,
                       uint32_t v, uint32_t S, uint32_t lane) {
  const uint32_t sl = lane & (S - 1), base = lane - sl;
  const uint64_t segmask = (S == 64 ? ~0ull : ((1ull << S) - 1ull)) << base;
  const uint32_t dv = ld(&dist[v]), W = g.W;
  const uint32_t e0 = g.row_ptr[v], e1 = g.row_ptr[v + 1];
  bool have_parent = false;
  for (uint32_t j0 = 0; j0 < W; j0 += S) {
    const uint32_t j = j0 + sl;
    uint32_t acc = 0;
    for (uint32_t eb = e0; eb < e1; eb += S) {  // segment-uniform
      const uint32_t e = eb + sl;
      uint32_t u = kInf;
      if (e < e1) {
        const uint32_t cu = g.col[e];
        const uint32_t du = ld(&dist[cu]);
        const uint32_t w = g.hop ? 1u : g.wt[g.rev[e]];
        if ((!g.ovl[cu] || cu == g.src) && du != kInf && du + w == dv) u = cu;
      }
      uint64_t tight = __ballot(u != kInf) & segmask;
      if (tight && !have_parent) {  // segment-uniform: CSR order, first tight tail
        have_parent = true;
        const uint32_t first = __shfl(u, __builtin_ctzll(tight), 64);
        if (sl == 0) st(&parent[v], first);
      }
      while (tight) {  // the tight tails' words, 4 loads in flight
        uint32_t tu[4], x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          tu[q] = kInf;
          if (tight) {
            tu[q] = __shfl(u, __builtin_ctzll(tight), 64);
            tight &= tight - 1;
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          x[q] = tu[q] != kInf && tu[q] != g.src && j < W ? ld(&nhb[(size_t)tu[q] * W + j]) : 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc |= x[q];
          if (tu[q] == g.src) {
            const uint32_t jb = g.nbr_bit[v];
            if (j == (jb >> 5)) acc |= 1u << (jb & 31);
          }
        }
      }
    }
    if (j < W) st(&nhb[(size_t)v * W + j], acc);
  }
  if (!have_parent && sl == 0) st(&parent[v], kInf);
}

// Next-hop bitsets nhb[v][W] of the SPF in `dist` (every distance final,
// after coop_sssp): nodes bucketed by distance value and settled level by
// level (every tight predecessor of a level-d node sits at a lower level)
// when at most kMaxLevels distinct values occur, fixed-point sweeps of the
// monotone union otherwise.  nhb must be zero and lvl[0..kLevelCap],
// misc[0..7] zero on entry.  Returns whether the level path ran (then
// lvl[d] = end of bucket d in `order`).  Starts and ends with a grid barrier.
__device__ bool level_nh(const XGrid& grid, const WiGraph& g, const uint32_t* dist,
                         uint32_t* nhb, uint32_t* lvl, uint32_t* order, uint32_t* misc,
                         uint32_t* parent, unsigned long long* lstamp = nullptr) {
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t gsz = gridDim.x * blockDim.x;  // a multiple of 64
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t N = g.N, W = g.W;
  const uint64_t NW = (uint64_t)N * W;
  // per-block histogram of the distance values and the block's write
  // cursors into `order` (LDS, when maxd < kLdsHist): one global atomic per
  // (block, value) instead of one per node -- 250k node atomics on ~30
  // counters (and on one for the maximum) were 1.6 ms of the what-if base
  // pass's 2.4 ms next-hop phase (per-level clocks, r05_wb)
  __shared__ uint32_t bh[kLdsHist], bc[kLdsHist];
  grid.sync();
  // ---- distance range (one atomic per wave) and per-value counts ----
  {
    uint32_t m = 0;
    for (uint32_t v = gtid; v < N; v += gsz) {
      const uint32_t d = ld(&dist[v]);
      if (d != kInf) m = max(m, d);
    }
    m = wave_max32(m);
    if (lane == 0 && m) atomicMax(&misc[0], m);
  }
  grid.sync();
  const uint32_t maxd = ld(&misc[0]);
  bool levels = maxd < kLevelCap;
  const bool hist = maxd < kLdsHist;  // block-uniform
  if (levels) {
    if (hist) {
      for (uint32_t i = threadIdx.x; i <= maxd; i += blockDim.x) bh[i] = 0u;
      __syncthreads();
      for (uint32_t v = gtid; v < N; v += gsz) {
        const uint32_t d = ld(&dist[v]);
        if (d != kInf) atomicAdd(&bh[d], 1u);
      }
      __syncthreads();
      for (uint32_t i = threadIdx.x; i <= maxd; i += blockDim.x)
        if (bh[i] && atomicAdd(&lvl[i], bh[i]) == 0) atomicAdd(&misc[1], 1u);
    } else {
      for (uint32_t v = gtid; v < N; v += gsz) {
        const uint32_t d = ld(&dist[v]);
        if (d != kInf && atomicAdd(&lvl[d], 1u) == 0) atomicAdd(&misc[1], 1u);
      }
    }
    grid.sync();
    levels = ld(&misc[1]) <= kMaxLevels;
  }
  if (levels) {
    // exclusive scan of the counts by block 0 (maxd + 1 <= kLevelCap entries)
    if (blockIdx.x == 0) {
      __shared__ uint32_t carry;
      if (threadIdx.x == 0) carry = 0;
      __syncthreads();
      for (uint32_t base = 0; base <= maxd; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t x = i <= maxd ? ld(&lvl[i]) : 0u;
        // block scan through LDS
        __shared__ uint32_t buf[kCoopThreads];
        buf[threadIdx.x] = x;
        __syncthreads();
        for (uint32_t d = 1; d < blockDim.x; d <<= 1) {
          const uint32_t y = threadIdx.x >= d ? buf[threadIdx.x - d] : 0u;
          __syncthreads();
          buf[threadIdx.x] += y;
          __syncthreads();
        }
        const uint32_t incl = buf[threadIdx.x] + carry;
        if (i <= maxd) st(&lvl[i], incl - x);
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) carry = incl;
        __syncthreads();
      }
      if (threadIdx.x == 0) st(&lvl[maxd + 1], carry);
    }
    grid.sync();
    // scatter nodes into distance order (lvl[d] advances to the bucket end):
    // with the block histogram, one global atomic per (block, value)
    // reserves the block's range, LDS cursors place its nodes
    if (hist) {
      for (uint32_t i = threadIdx.x; i <= maxd; i += blockDim.x)
        if (bh[i]) bc[i] = atomicAdd(&lvl[i], bh[i]);
      __syncthreads();
      for (uint32_t v = gtid; v < N; v += gsz) {
        const uint32_t d = ld(&dist[v]);
        if (d != kInf) st(&order[atomicAdd(&bc[d], 1u)], v);
      }
    } else {
      for (uint32_t v = gtid; v < N; v += gsz) {
        const uint32_t d = ld(&dist[v]);
        if (d != kInf) st(&order[atomicAdd(&lvl[d], 1u)], v);
      }
    }
    grid.sync();
    // level by level: every predecessor of a level-d node sits at a lower level
    uint32_t begin = ld(&lvl[0]);  // bucket 0 (the source) ends here
    for (uint32_t d = 1; d <= maxd; ++d) {
      const uint32_t end = ld(&lvl[d]);
      if (end == begin) continue;  // empty level: uniform skip
      const uint32_t n_lvl = end - begin;
      // 64 / S nodes per wave, a segment of S lanes each (seg_nh)
      const uint32_t S = W <= 16 ? 16u : (W <= 32 ? 32u : 64u);
      const uint32_t per_wave = 64 / S, seg = lane / S;
      const uint32_t waves = gsz / 64, wave = gtid / 64;
      for (uint32_t wb = wave * per_wave; wb < n_lvl; wb += waves * per_wave) {  // wave-uniform
        const uint32_t i = wb + seg;
        uint32_t v = 0;
        bool hub = false;
        if (i < n_lvl) {
          v = ld(&order[begin + i]);
          hub = g.row_ptr[v + 1] - g.row_ptr[v] > kCoopHubDeg;
          if (!hub) seg_nh(g, dist, nhb, parent, v, S, lane);  // segment-uniform
        }
        // a hub's W words are made once, by the whole wave
        for (uint64_t hubs = __ballot(hub && (lane & (S - 1)) == 0); hubs; hubs &= hubs - 1)
          hub_nh(g, dist, nhb, parent, __builtin_amdgcn_readlane(v, __builtin_ctzll(hubs)), lane);
      }
      begin = end;
      grid.sync();
      // diagnostics (SPF_WHATIF_PROF): the clock after level d, its size
      if (lstamp && gtid == 0 && d < 64) {
        lstamp[2 * d] = wall_clock64();
        lstamp[2 * d + 1] = n_lvl;
      }
    }
  } else {
    // fixed-point sweeps (monotone union over the DAG), flags rotate by 3
    for (uint32_t it = 0;; ++it) {
      bool any = false;
      for (uint64_t x = gtid; x < NW; x += gsz) {
        const uint32_t v = (uint32_t)(x / W), j = (uint32_t)(x % W);
        if (v == g.src || ld(&dist[v]) == kInf) continue;
        const uint32_t acc = nh_word(g, dist, nhb, v, j);
        if (acc != ld(&nhb[x])) {
          st(&nhb[x], acc);
          any = true;
        }
      }
      if (any) st(&misc[2 + it % 3], 1u);
      if (gtid == 0) st(&misc[2 + (it + 1) % 3], 0u);
      grid.sync();
      if (!ld(&misc[2 + it % 3])) break;
    }
  }
  grid.sync();
  return levels;
}

__global__ __launch_bounds__(kCoopThreads) void whatif_base_kernel(BaseArgs a) {
  const XGrid grid{a.sp.bar, a.sp.fault};
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t gsz = gridDim.x * blockDim.x;  // a multiple of 64
  const WiGraph& g = a.g;
  const uint32_t N = g.N, W = g.W;
  const uint64_t NW = (uint64_t)N * W;
  for (uint64_t x = gtid; x < NW; x += gsz) st(&a.nhb[x], 0u);
  for (uint32_t i = gtid; i <= kLevelCap; i += gsz) st(&a.lvl[i], 0u);
  for (uint32_t v = gtid; v < N; v += gsz) st(&a.sub[v], 0u);
  if (gtid == 0) {
    for (int i = 0; i < 8; ++i) st(&a.misc[i], 0u);
    *a.H = 0;
  }
  const bool stamp = a.prof && gtid == 0;
  if (stamp) a.prof[0] = wall_clock64();
  coop_sssp(grid, a.sp);  // starts and ends with a grid barrier
  if (stamp) a.prof[1] = wall_clock64();
  const uint32_t* dist = a.sp.dist;
  const bool levels = level_nh(grid, g, dist, a.nhb, a.lvl, a.order, a.misc, a.parent, a.lprof);
  if (stamp) a.prof[6] = wall_clock64();
  if (levels) {
    const uint32_t maxd = ld(&a.misc[0]);
    // subtree sizes of the parent tree, deepest level first: a lower bound
    // on the DAG descendants a failure of the tree edge into v can change,
    // used to hand big repairs to workgroup teams up front
    for (uint32_t v = gtid; v < N; v += gsz)
      if (ld(&dist[v]) != kInf) atomicAdd(&a.sub[v], 1u);
    grid.sync();
    for (uint32_t d = maxd; d >= 1; --d) {
      const uint32_t lo = ld(&a.lvl[d - 1]), hi = ld(&a.lvl[d]);
      if (lo == hi) continue;  // empty level: uniform skip
      for (uint32_t x = lo + gtid; x < hi; x += gsz) {
        const uint32_t v = ld(&a.order[x]);
        const uint32_t pu = ld(&a.parent[v]);
        if (pu != kInf) atomicAdd(&a.sub[pu], ld(&a.sub[v]));
      }
      grid.sync();
    }
  }
  if (stamp) {
    a.prof[2] = wall_clock64();
    a.prof[4] = ld(&a.misc[0]);
    a.prof[5] = ld(&a.misc[1]);
  }
  // ---- result hash ----
  uint64_t h = 0;
  for (uint32_t v = gtid; v < N; v += gsz) {
    const uint32_t d = ld(&dist[v]);
    if (d == kInf) continue;
    uint64_t f = 0xcbf29ce484222325ull;
    for (uint32_t w = 0; w < W; ++w) {
      f ^= ld(&a.nhb[(size_t)v * W + w]);
      f *= 0x100000001b3ull;
    }
    h += mix64(mix64((uint64_t)v + 1) + d) ^ f;
  }
  uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
  for (int d = 32; d >= 1; d >>= 1) {  // wave sum, one atomic per wave
    const uint32_t l2 = __shfl_down(lo, d, 64), h2 = __shfl_down(hi, d, 64);
    const uint64_t t = ((uint64_t)hi << 32 | lo) + ((uint64_t)h2 << 32 | l2);
    lo = (uint32_t)t;
    hi = (uint32_t)(t >> 32);
  }
  if ((threadIdx.x & 63) == 0 && (lo | hi)) atomicAdd(a.H, ((unsigned long long)hi << 32) | lo);
  if (stamp) a.prof[3] = wall_clock64();
}

// ---------------------------------------------------------------------------
//  batched SPF + next hops beyond the LDS-resident kernels (plans on graphs
//  too large for them, positive metrics or hop counts)
// ---------------------------------------------------------------------------
// One grid-resident launch walks the plan's sources one after another, the
// whole chip on each: frontier SSSP straight into the source's output row
// (coop_sssp), next hops per node in distance order (level_nh, node-major
// scratch nhb[v][W]), then a transpose into the plan's bitmap layout (bit v
// of word v/32 of neighbour j's bitmap): a wave holds the scratch word w of
// 64 consecutive nodes, one ballot per bit j of it is the 64-node slice of
// bitmap 32w + j, and lanes 0..31 store the 32 slices as 8-byte words.
struct BigArgs {
  CoopSssp sp;  // src and dist set per source
  WiGraph g;    // src, W set per source; g.nbr_bit = nbr_bit below
  const uint32_t* srcs;
  uint32_t n_src;
  const uint32_t* nb_ptr;  // distinct up neighbours (ascending id)
  const uint32_t* nb_id;
  uint32_t* D;  // [n_src][pitch] output rows
  uint32_t pitch;
  uint32_t* nh;  // output bitmaps
  const uint64_t* nh_off;
  uint32_t* nbr_bit;  // [N] scratch, kInf between sources
  uint32_t* nhb;      // [N][W] scratch
  uint32_t* lvl;      // [kLevelCap + 1]
  uint32_t* order;    // [N]
  uint32_t* misc;     // [8]
  uint32_t* parent;   // [N]
};

__global__ __launch_bounds__(kCoopThreads) void spf_big_kernel(BigArgs a) {
  const XGrid grid{a.sp.bar, a.sp.fault};
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t gsz = gridDim.x * blockDim.x;  // a multiple of 64
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t N = a.g.N, wpm = a.pitch / 32;
  for (uint32_t i = 0; i < a.n_src; ++i) {
    const uint32_t s = a.srcs[i];
    const uint32_t nb0 = a.nb_ptr[s], k = a.nb_ptr[s + 1] - nb0;
    const uint32_t W = k ? (k + 31) / 32 : 1u;
    WiGraph g = a.g;
    g.src = s;
    g.W = W;
    CoopSssp sp = a.sp;
    sp.src = s;
    sp.dist = a.D + (size_t)i * a.pitch;
    // per-source state (the previous source's readers finished at its last barrier)
    for (uint32_t j = gtid; j < k; j += gsz) st(&a.nbr_bit[a.nb_id[nb0 + j]], j);
    const uint64_t NW = (uint64_t)N * W;
    for (uint64_t x = gtid; x < NW; x += gsz) st(&a.nhb[x], 0u);
    for (uint32_t d = gtid; d <= kLevelCap; d += gsz) st(&a.lvl[d], 0u);
    if (gtid < 8) st(&a.misc[gtid], 0u);
    for (uint32_t v = N + gtid; v < a.pitch; v += gsz) st(&sp.dist[v], kInf);  // row padding
    coop_sssp(grid, sp);  // starts and ends with a grid barrier
    level_nh(grid, g, sp.dist, a.nhb, a.lvl, a.order, a.misc, a.parent);
    // transpose into the plan's bitmaps: items (64-node group, scratch word)
    if (k) {
      uint32_t* out = a.nh + a.nh_off[i];
      const uint32_t groups = a.pitch / 64;
      const uint64_t items = (uint64_t)groups * W;
      for (uint64_t t = (gtid >> 6); t < items; t += gsz / 64) {  // a wave per item
        const uint32_t grp = (uint32_t)(t / W), w = (uint32_t)(t % W);
        const uint32_t v = grp * 64 + lane;
        const uint32_t x = v < N ? ld(&a.nhb[(size_t)v * W + w]) : 0u;
        uint64_t mine = 0;
#pragma unroll 4
        for (uint32_t jj = 0; jj < 32; ++jj) {
          const uint64_t m = __ballot((x >> jj) & 1u);
          if (lane == jj) mine = m;
        }
        const uint32_t j = w * 32 + lane;
        if (lane < 32 && j < k) {
          uint2* o = reinterpret_cast<uint2*>(out + (size_t)j * wpm + grp * 2);
          *o = make_uint2((uint32_t)mine, (uint32_t)(mine >> 32));
        }
      }
    }
    for (uint32_t j = gtid; j < k; j += gsz) st(&a.nbr_bit[a.nb_id[nb0 + j]], kInf);
    grid.sync();
  }
}

// ---------------------------------------------------------------------------
//  classify failures: cold -> digest now, hot -> work list (failure, edge)
// ---------------------------------------------------------------------------
__global__ void classify_kernel(WiGraph g, const uint32_t* __restrict__ dist,
                                const unsigned long long* __restrict__ H,
                                const uint32_t* __restrict__ fails, uint32_t n_fail,
                                const uint32_t* __restrict__ link_edge,
                                const uint32_t* __restrict__ sub, uint32_t wave_cap,
                                spf_whatif_digest* out, uint2* hot, uint32_t* n_hot,
                                uint2* big, uint32_t* n_big) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_fail) return;
  const uint32_t e0 = link_edge[fails[f]];
  uint32_t tight = kInf;
  if (e0 != kInf) {
    for (uint32_t k = 0; k < 2; ++k) {
      const uint32_t e = k ? g.rev[e0] : e0;
      const uint32_t a = g.col[g.rev[e]], b = g.col[e];  // a -> b
      if (g.ovl[a] && a != g.src) continue;
      if (dist[a] != kInf && dist[a] + g.wt[e] == dist[b]) tight = e;
    }
  }
  if (tight == kInf) {
    out[f] = spf_whatif_digest{0u, 0u, (uint64_t)*H};
  } else if (sub[g.col[tight]] > wave_cap) {  // |D| >= subtree: a workgroup's repair
    big[atomicAdd(n_big, 1u)] = make_uint2(f, tight);
  } else {
    hot[atomicAdd(n_hot, 1u)] = make_uint2(f, tight);
  }
}

// ---------------------------------------------------------------------------
//  repair of one hot failure by a team (a wave, or a whole workgroup)
// ---------------------------------------------------------------------------
struct TeamCtl {
  uint32_t n, ovf, flag[3], dmin, dmax, nxt[3], lc[3], hub;
  unsigned long long ndist, nnh, dh;
  uint32_t bar;   // group teams: arrivals at the team barrier (monotonic)
  uint32_t next;  // group teams: the failure the team takes next
};

// A team is a wave (64), a workgroup (1024) or a group of TEAM / 1024
// workgroups of one grid-resident launch on one XCD (team_sync = the agent-scope
// release -> arrival counter -> poll -> acquire hand-off of
// MI355X_MICROARCH.md §Workgroup dispatch; the counter only grows, so the
// barrier of the k-th call completes at k * G arrivals)
template <int TEAM, bool GROUP = false>
__device__ __forceinline__ void team_sync(TeamCtl* ctl, uint32_t* fault) {
  if constexpr (GROUP) {
    const uint32_t G = TEAM / blockDim.x;  // workgroups per team
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores drained
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t ticket =
          __hip_atomic_fetch_add(&ctl->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t target = (ticket / G + 1) * G;
      uint32_t k = 0;
      for (; k < kBarSpin &&
             __hip_atomic_load(&ctl->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;
           ++k) {
        if ((k & 1023u) == 1023u && fault_set(fault)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (k == kBarSpin) barrier_timed_out(fault);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  } else if constexpr (TEAM == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Returns false (nothing written, scratch clean) when |D| exceeds cap.
// a wave's or workgroup's scratch (mark, dlist, dnew, level lists) is private
// to one workgroup: workgroup-scope accesses may be served by the CU's L1; a
// group team's is shared by several CUs: agent scope (L1 bypassed)
template <bool GROUP>
__device__ __forceinline__ uint32_t ldw(const uint32_t* p) {
  if constexpr (GROUP) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool GROUP>
__device__ __forceinline__ void stw(uint32_t* p, uint32_t v) {
  if constexpr (GROUP) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool GROUP>
__device__ __forceinline__ unsigned long long ldq(const unsigned long long* p) {
  if constexpr (GROUP) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool GROUP>
__device__ __forceinline__ void stq(unsigned long long* p, unsigned long long v) {
  if constexpr (GROUP) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// FNV-1a of both next-hop rows of a D node and whether they differ: the
// words in batches of 8, loads of a batch in flight together.  A node's hash
// is mix64(mix64(v + 1) + d) ^ FNV-1a(row), as in the base pass's result hash.
template <bool GROUP>
__device__ __forceinline__ void row_pair_hash(const uint32_t* h0, const uint32_t* h1, uint32_t W,
                                              uint64_t& f0, uint64_t& f1, bool& diff) {
  f0 = f1 = 0xcbf29ce484222325ull;
  for (uint32_t w = 0; w < W; w += 8) {
    uint32_t a[8], c[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      a[q] = w + q < W ? h0[w + q] : 0u;
      c[q] = w + q < W ? ldw<GROUP>(&h1[w + q]) : 0u;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (w + q < W) {
        f0 = (f0 ^ a[q]) * 0x100000001b3ull;
        f1 = (f1 ^ c[q]) * 0x100000001b3ull;
        diff |= a[q] != c[q];
      }
    }
  }
}

// The next-hop row ORs of one flattened edge chunk's tight pairs (lanes in
// pm: a tight predecessor u / its D index mu; lanes in sm: the source itself,
// jk = the node's source-neighbour bit), in lane order.  A pair belongs to D
// node ik.  W <= 64: lane j keeps word j of the current node's row in `acc`
// (`cur` = that node's D index, kInf for none), the loads of 8 pairs in
// flight together, and the row is stored once, when the node changes (a
// node's pairs are contiguous in flattened order, its row is zero before its
// level, and one wave builds it): the caller flushes the last one.  W > 64:
// a read-modify-write of the row per pair.
__device__ __forceinline__ void row_pairs(uint64_t pm, uint64_t sm, uint32_t ik, uint32_t jk,
                                          uint32_t u, uint32_t mu, uint32_t W, uint32_t* nhn,
                                          const uint32_t* nhb, uint32_t lane, uint32_t& cur,
                                          uint32_t& acc) {
  pm |= sm;
  if (W <= 64) {
    while (pm) {  // wave-uniform
      uint32_t pi[8], pj[8], x[8];
      bool pv[8], ps[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        pv[q] = pm != 0;
        ps[q] = false;
        pi[q] = pj[q] = x[q] = 0;
        if (pv[q]) {
          const uint32_t bl = __ffsll((unsigned long long)pm) - 1;
          pm &= pm - 1;
          pi[q] = __builtin_amdgcn_readlane(ik, bl);
          ps[q] = (sm >> bl) & 1;
          if (ps[q]) {
            pj[q] = __builtin_amdgcn_readlane(jk, bl);
          } else {
            const uint32_t pu = __builtin_amdgcn_readlane(u, bl), pmu = __builtin_amdgcn_readlane(mu, bl);
            const uint32_t* from = pmu != kInf ? nhn + (size_t)pmu * W : nhb + (size_t)pu * W;
            if (lane < W) x[q] = from[lane];
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (!pv[q]) continue;
        if (pi[q] != cur) {
          if (cur != kInf && lane < W) nhn[(size_t)cur * W + lane] = acc;
          cur = pi[q];
          acc = 0;
        }
        acc |= ps[q] ? (lane == (pj[q] >> 5) ? 1u << (pj[q] & 31) : 0u) : x[q];
      }
    }
  } else {
    for (; pm; pm &= pm - 1) {
      const uint32_t bl = __ffsll((unsigned long long)pm) - 1;
      uint32_t* row = nhn + (size_t)__builtin_amdgcn_readlane(ik, bl) * W;
      if ((sm >> bl) & 1) {
        const uint32_t pj = __builtin_amdgcn_readlane(jk, bl);
        if (lane == ((pj >> 5) & 63) && (pj >> 5) < W) row[pj >> 5] |= 1u << (pj & 31);
      } else {
        const uint32_t pu = __builtin_amdgcn_readlane(u, bl), pmu = __builtin_amdgcn_readlane(mu, bl);
        const uint32_t* from = pmu != kInf ? nhn + (size_t)pmu * W : nhb + (size_t)pu * W;
        for (uint32_t j = lane; j < W; j += 64) row[j] |= from[j];
      }
    }
  }
}

// Nodes per wave chunk of a team's node loops: the count spread over the
// team's waves, 1..64 (team-uniform).
template <int TEAM>
__device__ __forceinline__ uint32_t team_chunk(uint32_t count) {
  constexpr uint32_t kW = TEAM / 64;
  return min(64u, max(1u, (count + kW - 1) / kW));
}

// Phase counters of a profiled repair (SPF_WHATIF_PROF).  Registers (GPH
// false): ph is the caller's array, stored once when the team exits.  Global
// (GPH true, SPF_WHATIF_PROF=global): ph is the team's 16-slot row of the
// prof buffer, updated by the team's first thread with device atomics at
// every event -- the round-5 variant that faulted; its row was
// range-checked by the kernel before it got here.
template <bool GPH>
__device__ __forceinline__ void ph_add(uint64_t* ph, int k, uint64_t v, bool leader) {
  if constexpr (GPH) {
    if (leader) atomicAdd(reinterpret_cast<unsigned long long*>(ph + k), (unsigned long long)v);
  } else {
    ph[k] += v;
  }
}
template <bool GPH>
__device__ __forceinline__ void ph_max(uint64_t* ph, int k, uint64_t v, bool leader) {
  if constexpr (GPH) {
    if (leader) atomicMax(reinterpret_cast<unsigned long long*>(ph + k), (unsigned long long)v);
  } else {
    ph[k] = ph[k] > v ? ph[k] : v;
  }
}

// CHK (the profiled instances, SPF_WHATIF_PROF): every scratch-derived
// index is range-checked before use; an out-of-range one sets bit 4 of the
// fault word with the site in bits 16-23 and is replaced by a safe value
// (results then invalid, reported by spf_device_check).
template <int TEAM, bool GROUP = false, bool CHK = false, bool GPH = false>
__device__ bool repair(const WiGraph& g, const WiBase& B, uint32_t* mark, uint32_t* dlist,
                       uint32_t* dnew, uint32_t* nhn, uint32_t* lvl, uint32_t* ord, uint32_t cap,
                       TeamCtl* ctl, uint32_t tt, uint32_t e_fail, spf_whatif_digest* out,
                       uint64_t* ph = nullptr) {
  // diagnostics (SPF_WHATIF_PROF): 12 counters, accumulated over the team's
  // failures (ph_add) -- [0] repairs, [1..5] 100 MHz ticks in D discovery,
  // seeds, Dial, fallback sweeps, digest; [8] sum |D|, [9] sum Dial levels,
  // [10] max |D|, [11] repairs given up
  uint64_t tprev = ph ? wall_clock64() : 0ull;
#define WI_STAMP(k)                              \
  do {                                           \
    if (ph) {                                    \
      const uint64_t now_ = wall_clock64();      \
      ph_add<GPH>(ph, k, now_ - tprev, tt == 0); \
      tprev = now_;                              \
    }                                            \
  } while (0)
  const uint32_t W = g.W;
  // range check (CHK): x < lim, or x == kInf when `inf_ok`
  auto chk = [&](uint32_t x, uint32_t lim, bool inf_ok, uint32_t site, uint32_t safe) -> uint32_t {
    if constexpr (CHK) {
      if (!(x < lim || (inf_ok && x == kInf))) {
        if (g.fault)
          __hip_atomic_fetch_or(g.fault, 16u | (site << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return safe;
      }
    }
    return x;
  };
  const uint32_t lane = tt & 63, wv = tt >> 6;
  const uint32_t l = g.link[e_fail];
  const uint32_t b = g.col[e_fail];
  if (tt == 0) {
    stw<GROUP>(&ctl->n, 1u);
    stw<GROUP>(&ctl->ovf, 0u);
    stw<GROUP>(&ctl->hub, 0u);
    for (int q = 0; q < 3; ++q) stw<GROUP>(&ctl->flag[q], 0u);
    stq<GROUP>(&ctl->ndist, 0ull);
    stq<GROUP>(&ctl->nnh, 0ull);
    stq<GROUP>(&ctl->dh, 0ull);
    dlist[0] = b;
    stw<GROUP>(&mark[b], 0);
  }
  team_sync<TEAM, GROUP>(ctl, g.fault);
  // ---- D = descendants of b in the unfailed DAG (level by level) ----
  // Control words (ctl->n / ovf / hub / flag / nxt / lc) are written by
  // atomics and plain stores of other lanes, waves or CUs: every read of one
  // is an atomic load at the team's scope (ldw), so the compiler can neither
  // keep a stale copy in a register nor move the read across the team
  // barrier.  Every loop is bounded by its worst case + 2 (an iteration adds
  // a node, or settles one more level); a bound hit reports its phase in the
  // fault word and leaves the repair (loop_bound_hit).
  uint32_t lo = 0;
  bool bound_hit = false;
  for (uint32_t iter = 0;; ++iter) {
    const uint32_t n = ldw<GROUP>(&ctl->n);
    team_sync<TEAM, GROUP>(ctl, g.fault);
    if (lo >= n || ldw<GROUP>(&ctl->ovf)) break;
    if (iter > cap + 2) {  // team-uniform
      bound_hit = true;
      if (tt == 0) loop_bound_hit(g.fault, 1);
      break;
    }
    // each wave takes cs frontier nodes at a time (cs = the frontier over
    // the team's waves, at most 64: a small frontier still spreads over every
    // wave), lanes over their flattened edges (wave_edges); new nodes are
    // appended by one counter atomic per wave
    const uint32_t cs = team_chunk<TEAM>(n - lo);
    for (uint32_t c0 = lo + wv * cs; c0 < n; c0 += (TEAM / 64) * cs) {
      const uint32_t i = c0 + lane;
      const bool in = lane < cs && i < n;
      const uint32_t v = in ? chk(dlist[i], g.N, false, 1, b) : 0u;
      const bool x = in && !g.ovl[v];  // drained (v != src): no DAG children
      const uint32_t dv = x ? B.dist[v] : 0u;
      wave_edges(g.row_ptr, v, x, [&](uint32_t k, uint32_t e, bool act) {
        const uint32_t dk = lane_pull(dv, k);
        uint32_t c = 0;
        bool won = false;
        if (act) {
          const uint4 q = g.ed[e];
          c = q.x;
          if (dk + q.y == B.dist[c]) won = atomicCAS(&mark[c], kInf, kBusy) == kInf;
        }
        const uint64_t wm = __ballot(won);
        if (wm) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(&ctl->n, (uint32_t)__popcll(wm));
          base = __builtin_amdgcn_readlane(base, 0);
          if (won) {
            const uint32_t idx = base + lanes_below(wm);
            if (idx < cap) {
              dlist[idx] = c;
              stw<GROUP>(&mark[c], idx);
            } else {
              stw<GROUP>(&mark[c], kInf);
              stw<GROUP>(&ctl->ovf, 1u);
            }
          }
        }
      });
    }
    lo = n;
    team_sync<TEAM, GROUP>(ctl, g.fault);
  }
  const uint32_t n = min(ldw<GROUP>(&ctl->n), cap);
  const bool ovf = ldw<GROUP>(&ctl->ovf) != 0 || bound_hit;
  WI_STAMP(1);
  if (ph) {
    ph_add<GPH>(ph, 0, 1, tt == 0);
    ph_add<GPH>(ph, 8, n, tt == 0);
    ph_max<GPH>(ph, 10, n, tt == 0);
    ph_add<GPH>(ph, 11, ovf, tt == 0);
  }
  team_sync<TEAM, GROUP>(ctl, g.fault);
  if (ovf) {
    for (uint32_t i = tt; i < n; i += TEAM) stw<GROUP>(&mark[dlist[i]], kInf);
    team_sync<TEAM, GROUP>(ctl, g.fault);
    return false;
  }
  // ---- seeds: best in-edge from outside D (unchanged distances) ----
  // waves over 64 D nodes at a time, lanes over their flattened in-edges,
  // the per-node minimum by atomics on dnew
  for (uint32_t i = tt; i < n; i += TEAM) stw<GROUP>(&dnew[i], kInf);
  team_sync<TEAM, GROUP>(ctl, g.fault);
  const uint32_t cs_seed = team_chunk<TEAM>(n);
  for (uint32_t c0 = wv * cs_seed; c0 < n; c0 += (TEAM / 64) * cs_seed) {
    const uint32_t i = c0 + lane;
    const bool in = lane < cs_seed && i < n;
    const uint32_t v = in ? dlist[i] : 0u;
    wave_edges(g.row_ptr, v, in, [&](uint32_t k, uint32_t e, bool act) {
      uint32_t s = kInf;
      const uint4 q = act ? g.ed[e] : make_uint4(0u, 0u, l, 0u);
      if (act && q.z != l) {
        const uint32_t u = q.x;
        if (ldw<GROUP>(&mark[u]) == kInf && !(g.ovl[u] && u != g.src)) {
          const uint32_t du = B.dist[u];
          if (du != kInf) s = du + q.w;
        }
      }
      if (s != kInf) {
        if constexpr (GROUP)
          __hip_atomic_fetch_min(&dnew[c0 + k], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          __hip_atomic_fetch_min(&dnew[c0 + k], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    });
  }
  team_sync<TEAM, GROUP>(ctl, g.fault);
  // nh word j of a D node from its tight expanded predecessors (D or not);
  // used by the fixed-point fallback
  auto nh_of = [&](uint32_t i, uint32_t j) -> uint32_t {
    const uint32_t v = dlist[i];
    const uint32_t dv = ldw<GROUP>(&dnew[i]);
    uint32_t acc = 0;
    for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
      if (g.link[e] == l) continue;
      const uint32_t u = g.col[e];
      if (g.ovl[u] && u != g.src) continue;
      const uint32_t mu = chk(ldw<GROUP>(&mark[u]), n, true, 5, kInf);
      const uint32_t du = mu != kInf ? ldw<GROUP>(&dnew[mu]) : B.dist[u];
      if (du == kInf || du + in_w(g, e) != dv) continue;
      if (u == g.src) {
        const uint32_t jb = g.nbr_bit[v];
        if ((jb >> 5) == j) acc |= 1u << (jb & 31);
      } else {
        acc |= mu != kInf ? nhn[(size_t)mu * W + j] : B.nhb[(size_t)u * W + j];
      }
    }
    return acc;
  };
  const size_t nw = (size_t)n * W;
  for (size_t x = tt; x < nw; x += TEAM) nhn[x] = 0;
  if (tt == 0) {
    stw<GROUP>(&ctl->dmin, kInf);
    stw<GROUP>(&ctl->nxt[0], kInf);
    stw<GROUP>(&ctl->lc[0], 0u);
  }
  team_sync<TEAM, GROUP>(ctl, g.fault);
  {
    uint32_t m = kInf;
    for (uint32_t i = tt; i < n; i += TEAM) m = min(m, ldw<GROUP>(&dnew[i]));
    if (m != kInf) atomicMin(&ctl->dmin, m);
  }
  team_sync<TEAM, GROUP>(ctl, g.fault);
  WI_STAMP(2);
  // ---- Dial: settle D one distance value at a time (metrics are positive:
  // a node holding the smallest pending value is final), next hops inline ----
  bool settled = true;
  uint32_t t = ldw<GROUP>(&ctl->dmin);
  for (uint32_t it = 0; t != kInf; ++it) {
    if (it >= kDialLevels) {  // too many distinct values: sweep instead
      settled = false;
      break;
    }
    uint32_t* next = &ctl->nxt[it % 3];
    uint32_t* cnt = &ctl->lc[it % 3];
    if (tt == 0) {  // the next level's slots, last read two levels ago
      stw<GROUP>(&ctl->nxt[(it + 1) % 3], kInf);
      stw<GROUP>(&ctl->lc[(it + 1) % 3], 0u);
    }
    // (a) the level's nodes (their distance is final) into ord, one counter
    // atomic per wave
    // (4 chunks per pass: their loads in flight together, one atomic)
    uint32_t m = kInf;
    for (uint32_t c0 = wv * 64; c0 < n; c0 += 4 * TEAM) {
      uint32_t d[4];
      uint64_t sm[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t i = c0 + q * TEAM + lane;
        d[q] = i < n ? ldw<GROUP>(&dnew[i]) : kInf;
      }
      uint32_t tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (d[q] != kInf && d[q] > t) m = min(m, d[q]);
        sm[q] = __ballot(d[q] == t);
        tot += (uint32_t)__popcll(sm[q]);
      }
      if (tot) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(cnt, tot);
        base = __builtin_amdgcn_readlane(base, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (d[q] == t) stw<GROUP>(&ord[base + lanes_below(sm[q])], c0 + q * TEAM + lane);
          base += (uint32_t)__popcll(sm[q]);
        }
      }
    }
    team_sync<TEAM, GROUP>(ctl, g.fault);
    // (b) level nodes, cs per wave at a time (a level of ~150 nodes in 64-
    // node chunks kept 3 of a group team's 64 waves busy, each walking ~8
    // flattened edge chunks in turn), lanes over their flattened edges:
    // tight predecessors give the next-hop rows (row_pairs), out-edges relax
    // the pending nodes
    const uint32_t K = ldw<GROUP>(cnt);
    const uint32_t cs = team_chunk<TEAM>(K);
    for (uint32_t q0 = wv * cs; q0 < K; q0 += (TEAM / 64) * cs) {
      const uint32_t q = q0 + lane;
      const bool valid = lane < cs && q < K;
      const uint32_t i = valid ? chk(ldw<GROUP>(&ord[q]), n, false, 9, 0) : 0u;
      const uint32_t v = valid ? chk(dlist[i], g.N, false, 10, b) : 0u;
      const uint32_t transit = valid && !g.ovl[v];  // drained: no transit
      const uint32_t jb = valid ? g.nbr_bit[v] : 0u;
      uint32_t cur = kInf, acc = 0;  // row_pairs' open row
      wave_edges(g.row_ptr, v, valid, [&](uint32_t k, uint32_t e, bool act) {
        const uint32_t ik = lane_pull(i, k), tk = lane_pull(transit, k), jk = lane_pull(jb, k);
        uint32_t u = 0, mu = kInf;
        bool tight = false, from_src = false;
        const uint4 q = act ? g.ed[e] : make_uint4(0u, 0u, l, 0u);
        if (act && q.z != l) {
          u = q.x;
          mu = chk(ldw<GROUP>(&mark[u]), n, true, 13, kInf);
          if (!(g.ovl[u] && u != g.src)) {
            const uint32_t du = mu != kInf ? ldw<GROUP>(&dnew[mu]) : B.dist[u];
            tight = du != kInf && du + (g.hop ? 1u : q.w) == t;
          }
          if (tk && mu != kInf) {  // relax v -> u (u pending: its value only drops)
            const uint32_t nd = t + q.y;
            if (nd < atomicMin(&dnew[mu], nd)) m = min(m, nd);
          }
          if (tight && u == g.src) {
            from_src = true;
            tight = false;
          }
        }
        row_pairs(__ballot(tight), __ballot(from_src), ik, jk, u, mu, W, nhn, B.nhb, lane, cur, acc);
      });
      if (cur != kInf && lane < W) nhn[(size_t)cur * W + lane] = acc;
    }
    if (m != kInf) atomicMin(next, m);
    team_sync<TEAM, GROUP>(ctl, g.fault);
    t = ldw<GROUP>(next);
    if (ph) ph_add<GPH>(ph, 9, 1, tt == 0);
  }
  WI_STAMP(3);
  if (!settled) {
    // ---- label-correcting sweeps inside D (Bellman-Ford: at most n + 1) ----
    for (uint32_t it = 0;; ++it) {
      if (it > n + 2) {  // team-uniform
        if (tt == 0) loop_bound_hit(g.fault, 2);
        break;
      }
      bool any = false;
      for (uint32_t i = tt; i < n; i += TEAM) {
        const uint32_t v = dlist[i];
        const uint32_t dv = ldw<GROUP>(&dnew[i]);
        if (dv == kInf || g.ovl[v]) continue;
        for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
          if (g.link[e] == l) continue;
          const uint32_t ic = chk(ldw<GROUP>(&mark[g.col[e]]), n, true, 14, kInf);
          if (ic == kInf) continue;
          const uint32_t nd = dv + g.wt[e];
          if (nd < atomicMin(&dnew[ic], nd)) any = true;
        }
      }
      if (any) stw<GROUP>(&ctl->flag[it % 3], 1u);
      if (tt == 0) stw<GROUP>(&ctl->flag[(it + 1) % 3], 0u);
      team_sync<TEAM, GROUP>(ctl, g.fault);
      if (!ldw<GROUP>(&ctl->flag[it % 3])) break;
    }

    const size_t nw = (size_t)n * W;
    for (size_t x = tt; x < nw; x += TEAM) nhn[x] = 0;
    if (tt == 0) {
      for (int q = 0; q < 3; ++q) stw<GROUP>(&ctl->flag[q], 0u);
      stw<GROUP>(&ctl->dmin, kInf);
      stw<GROUP>(&ctl->dmax, 0u);
    }
    team_sync<TEAM, GROUP>(ctl, g.fault);
    for (uint32_t i = tt; i < n; i += TEAM) {
      const uint32_t d = ldw<GROUP>(&dnew[i]);
      if (d != kInf) {
        atomicMin(&ctl->dmin, d);
        atomicMax(&ctl->dmax, d);
      }
    }
    team_sync<TEAM, GROUP>(ctl, g.fault);
    const uint32_t dmin = ldw<GROUP>(&ctl->dmin);
    const uint32_t nlev = dmin == kInf ? 0u : ldw<GROUP>(&ctl->dmax) - dmin + 1;
    if (nlev <= cap) {
      // counting sort of D by new distance; a predecessor always sits in a
      // lower level (positive metrics), so one pass per level is exact
      for (uint32_t b = tt; b < nlev; b += TEAM) stw<GROUP>(&lvl[b], 0u);
      team_sync<TEAM, GROUP>(ctl, g.fault);
      for (uint32_t i = tt; i < n; i += TEAM) {
        const uint32_t d = ldw<GROUP>(&dnew[i]);
        if (d != kInf) atomicAdd(&lvl[d - dmin], 1u);
      }
      team_sync<TEAM, GROUP>(ctl, g.fault);
      if (tt < 64) {  // exclusive scan by the team's first wave
        uint32_t carry = 0;
        for (uint32_t base = 0; base < nlev; base += 64) {
          const uint32_t b = base + tt;
          const uint32_t x = b < nlev ? ldw<GROUP>(&lvl[b]) : 0u;
          const uint32_t inc = wave_incl_scan32(x);
          if (b < nlev) stw<GROUP>(&lvl[b], carry + inc - x);
          carry += __builtin_amdgcn_readlane(inc, 63);
        }
      }
      team_sync<TEAM, GROUP>(ctl, g.fault);
      for (uint32_t i = tt; i < n; i += TEAM) {
        const uint32_t d = ldw<GROUP>(&dnew[i]);
        if (d != kInf) stw<GROUP>(&ord[atomicAdd(&lvl[d - dmin], 1u)], i);
      }
      team_sync<TEAM, GROUP>(ctl, g.fault);
      uint32_t begin = 0;
      for (uint32_t b = 0; b < nlev; ++b) {
        const uint32_t end = ldw<GROUP>(&lvl[b]);
        if (end == begin) continue;
        const size_t items = (size_t)(end - begin) * W;
        for (size_t x = tt; x < items; x += TEAM) {
          const uint32_t i = chk(ldw<GROUP>(&ord[begin + x / W]), n, false, 15, 0), j = (uint32_t)(x % W);
          nhn[(size_t)i * W + j] = nh_of(i, j);
        }
        begin = end;
        team_sync<TEAM, GROUP>(ctl, g.fault);
      }
    } else {
      // fixed-point sweeps (monotone union over the DAG: at most depth + 1)
      for (uint32_t it = 0;; ++it) {
        if (it > n + 2) {  // team-uniform
          if (tt == 0) loop_bound_hit(g.fault, 3);
          break;
        }
        bool any = false;
        for (uint32_t x = tt; x < nw; x += TEAM) {
          const uint32_t i = x / W, j = x % W;
          if (ldw<GROUP>(&dnew[i]) == kInf) continue;
          const uint32_t acc = nh_of(i, j);
          if (acc != nhn[x]) {
            nhn[x] = acc;
            any = true;
          }
        }
        if (any) stw<GROUP>(&ctl->flag[it % 3], 1u);
        if (tt == 0) stw<GROUP>(&ctl->flag[(it + 1) % 3], 0u);
        team_sync<TEAM, GROUP>(ctl, g.fault);
        if (!ldw<GROUP>(&ctl->flag[it % 3])) break;
      }
    }
  }
  WI_STAMP(4);
  // ---- digest delta over D, scratch reset ----
  uint32_t nd_ = 0, nn_ = 0;
  uint64_t dh = 0;
  for (uint32_t i = tt; i < n; i += TEAM) {
    const uint32_t v = dlist[i];
    const uint32_t d1 = ldw<GROUP>(&dnew[i]), d0 = B.dist[v];
    uint64_t f0, f1;
    bool diff = d1 == kInf;
    row_pair_hash<GROUP>(B.nhb + (size_t)v * W, nhn + (size_t)i * W, W, f0, f1, diff);
    const uint64_t base = mix64((uint64_t)v + 1);
    nd_ += d1 != d0;
    nn_ += diff;
    dh += (d1 == kInf ? 0ull : mix64(base + d1) ^ f1) - (mix64(base + d0) ^ f0);
    stw<GROUP>(&mark[v], kInf);
  }
  if (nd_) atomicAdd(&ctl->ndist, (unsigned long long)nd_);
  if (nn_) atomicAdd(&ctl->nnh, (unsigned long long)nn_);
  if (dh) atomicAdd(&ctl->dh, (unsigned long long)dh);
  team_sync<TEAM, GROUP>(ctl, g.fault);
  if (tt == 0)
    *out = spf_whatif_digest{(uint32_t)ldq<GROUP>(&ctl->ndist), (uint32_t)ldq<GROUP>(&ctl->nnh),
                             (uint64_t)(*B.H + ldq<GROUP>(&ctl->dh))};
  team_sync<TEAM, GROUP>(ctl, g.fault);
  WI_STAMP(5);
#undef WI_STAMP
  return true;
}

// A wave team's node -> D-index map: an open-addressed table of T = 4 * cap
// (a power of two) u64 slots, key (node) in the low word, value (D index, or
// kBusy while being claimed) in the high word, linear probing from a
// multiplicative hash.  It replaces an N-word `mark` array per wave team:
// 4,096 teams x 250k nodes x 4 B = 4 GB of scratch whose random lookups
// missed every cache -- the tables take 32 KB a team.
// Slots start (and are always left) empty (~0): a repair clears the slots it
// used, an aborted one the whole table.
struct WaveSet {
  unsigned long long* tab;
  uint32_t mask, shift;  // T - 1, 32 - log2(T)
};
constexpr unsigned long long kSlotEmpty = ~0ull;
__device__ __forceinline__ unsigned long long ws_ld(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ws_st(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// insert v (value kBusy): its slot, or ~0u when v is present already; `full`
// when no slot is left (the caller aborts the repair)
__device__ __forceinline__ uint32_t ws_claim(const WaveSet& s, uint32_t v, bool& full) {
  uint32_t h = (v * 0x9E3779B1u) >> s.shift;
  for (uint32_t k = 0; k <= s.mask; ++k, h = (h + 1) & s.mask) {
    const unsigned long long old = atomicCAS(&s.tab[h], kSlotEmpty, ((unsigned long long)kBusy << 32) | v);
    if (old == kSlotEmpty) return h;
    if ((uint32_t)old == v) return ~0u;
  }
  full = true;
  return ~0u;
}
// v's slot, or ~0u when absent
__device__ __forceinline__ uint32_t ws_slot(const WaveSet& s, uint32_t v) {
  uint32_t h = (v * 0x9E3779B1u) >> s.shift;
  for (uint32_t k = 0; k <= s.mask; ++k, h = (h + 1) & s.mask) {
    const unsigned long long x = ws_ld(&s.tab[h]);
    if ((uint32_t)x == v) return h;
    if (x == kSlotEmpty) return ~0u;
  }
  return ~0u;
}
// v's value (its D index), kInf when absent
__device__ __forceinline__ uint32_t ws_find(const WaveSet& s, uint32_t v) {
  uint32_t h = (v * 0x9E3779B1u) >> s.shift;
  for (uint32_t k = 0; k <= s.mask; ++k, h = (h + 1) & s.mask) {
    const unsigned long long x = ws_ld(&s.tab[h]);
    if ((uint32_t)x == v) return (uint32_t)(x >> 32);
    if (x == kSlotEmpty) return kInf;
  }
  return kInf;
}

// A wave team's repair (|D| <= cap): repair()'s three phases -- D discovery,
// seeds, Dial with next hops inline -- and its digest delta, bit for bit, but
// with the wave's lanes over the flattened edges of up to 64 nodes at a time
// (wave_edges) instead of a lane per node walking its edges one by one: a
// node's dependent chain (row_ptr -> col -> mark -> dnew / base row) is paid
// once per 64 edges instead of once per edge.  The team is one wave, so |D|,
// the level list length and the next Dial value live in registers
// (ballot + mbcnt compaction instead of counter atomics); the level list of
// a D of <= 64 nodes never leaves the registers (ds_permute).  |D| <= cap <=
// kDialLevels distinct values, so Dial always settles (no fallback sweeps).
template <bool CHK, bool GPH = false>
__device__ bool repair_wave(const WiGraph& g, const WiBase& B, const WaveSet& hs, uint32_t* dlist,
                            uint32_t* dnew, uint32_t* nhn, uint32_t* ord, uint32_t cap,
                            TeamCtl* ctl, uint32_t lane, uint32_t e_fail, spf_whatif_digest* out,
                            uint64_t* ph) {
  uint64_t tprev = ph ? wall_clock64() : 0ull;
#define WI_STAMP(k)                                \
  do {                                             \
    if (ph) {                                      \
      const uint64_t now_ = wall_clock64();        \
      ph_add<GPH>(ph, k, now_ - tprev, lane == 0); \
      tprev = now_;                                \
    }                                              \
  } while (0)
  auto chk = [&](uint32_t x, uint32_t lim, bool inf_ok, uint32_t site, uint32_t safe) -> uint32_t {
    if constexpr (CHK) {
      if (!(x < lim || (inf_ok && x == kInf))) {
        if (g.fault)
          __hip_atomic_fetch_or(g.fault, 16u | (site << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return safe;
      }
    }
    return x;
  };
  auto sync = [&]() { team_sync<64>(ctl, g.fault); };
  const uint32_t W = g.W;
  const uint32_t l = g.link[e_fail];
  const uint32_t b = g.col[e_fail];
  if (lane == 0) {
    dlist[0] = b;
    bool full = false;
    const uint32_t s0 = ws_claim(hs, b, full);  // (the table is empty)
    ws_st(&hs.tab[s0], b);                      // value 0: D index 0
    stq<false>(&ctl->ndist, 0ull);
    stq<false>(&ctl->nnh, 0ull);
    stq<false>(&ctl->dh, 0ull);
  }
  sync();
  // ---- D = descendants of b in the unfailed DAG, frontier by frontier ----
  uint32_t n = 1, lo = 0;
  bool bad = false;
  for (uint32_t iter = 0; lo < n && n <= cap; ++iter) {
    if (iter > cap + 2) {  // wave-uniform
      bad = true;
      if (lane == 0) loop_bound_hit(g.fault, 1);
      break;
    }
    const uint32_t hi = n;
    for (uint32_t c0 = lo; c0 < hi && n <= cap; c0 += 64) {
      const uint32_t i = c0 + lane;
      const uint32_t v = i < hi ? chk(ldw<false>(&dlist[i]), g.N, false, 1, b) : 0u;
      const bool x = i < hi && !g.ovl[v];  // drained (v != src): no DAG children
      const uint32_t dv = x ? B.dist[v] : 0u;
      bool full = false;
      wave_edges(g.row_ptr, v, x, [&](uint32_t k, uint32_t e, bool act) {
        const uint32_t dk = lane_pull(dv, k);
        uint32_t c = 0, slot = ~0u;
        if (act) {
          const uint4 q = g.ed[e];
          c = q.x;
          if (dk + q.y == B.dist[c]) slot = ws_claim(hs, c, full);
        }
        const bool won = slot != ~0u;
        const uint64_t wm = __ballot(won);
        if (won) {
          const uint32_t idx = n + lanes_below(wm);
          ws_st(&hs.tab[slot], ((unsigned long long)(idx < cap ? idx : kInf) << 32) | c);
          if (idx < cap) dlist[idx] = c;
        }
        n += (uint32_t)__popcll(wm);
      });
      if (__ballot(full)) {  // no slot left: abort as an overflow
        bad = true;
        break;
      }
    }
    lo = hi;
    sync();
    if (bad) break;
  }
  const bool ovf = n > cap || bad;
  n = min(n, cap);
  WI_STAMP(1);
  if (ph) {
    ph_add<GPH>(ph, 0, 1, lane == 0);
    ph_add<GPH>(ph, 8, n, lane == 0);
    ph_max<GPH>(ph, 10, n, lane == 0);
    ph_add<GPH>(ph, 11, ovf, lane == 0);
  }
  if (ovf) {  // slots past the cap hold kInf values: clear the whole table
    for (uint32_t q = lane; q <= hs.mask; q += 64) ws_st(&hs.tab[q], kSlotEmpty);
    sync();
    return false;
  }
  // ---- seeds: best in-edge from outside D (unchanged distances) ----
  for (uint32_t i = lane; i < n; i += 64) stw<false>(&dnew[i], kInf);
  for (size_t x = lane; x < (size_t)n * W; x += 64) nhn[x] = 0;
  sync();
  for (uint32_t c0 = 0; c0 < n; c0 += 64) {
    const uint32_t i = c0 + lane;
    const uint32_t v = i < n ? ldw<false>(&dlist[i]) : 0u;
    wave_edges(g.row_ptr, v, i < n, [&](uint32_t k, uint32_t e, bool act) {
      uint32_t s = kInf;
      const uint4 q = act ? g.ed[e] : make_uint4(0u, 0u, l, 0u);
      if (act && q.z != l) {
        const uint32_t u = q.x;
        if (ws_find(hs, u) == kInf && !(g.ovl[u] && u != g.src)) {
          const uint32_t du = B.dist[u];
          if (du != kInf) s = du + q.w;
        }
      }
      if (s != kInf)
        __hip_atomic_fetch_min(&dnew[c0 + k], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    });
  }
  sync();
  // the D of <= 64 nodes stays in registers through Dial: lane i holds D
  // node i (index, node, the source-neighbour bit)
  const bool small = n <= 64;
  const uint32_t sv = small && lane < n ? ldw<false>(&dlist[lane]) : 0u;
  uint32_t t = kInf;
  for (uint32_t c0 = 0; c0 < n; c0 += 64) {
    const uint32_t i = c0 + lane;
    t = min(t, i < n ? ldw<false>(&dnew[i]) : kInf);
  }
  t = wave_min32(t);
  WI_STAMP(2);
  // ---- Dial: settle D one distance value at a time (metrics are positive:
  // a node holding the smallest pending value is final), next hops inline ----
  for (uint32_t it = 0; t != kInf; ++it) {
    if (it > n + 2) {  // every level settles a node: cannot happen
      if (lane == 0) loop_bound_hit(g.fault, 4);
      break;
    }
    // (a) the level's nodes (their distance is final) and the next value
    uint32_t m = kInf, K = 0, li = 0, lv = 0;
    if (small) {
      const uint32_t d = lane < n ? ldw<false>(&dnew[lane]) : kInf;
      const bool sel = d == t;
      if (d != kInf && d > t) m = d;
      const uint64_t sm = __ballot(sel);
      K = (uint32_t)__popcll(sm);
      // compact: the r-th level node to lane r, the rest after them
      const uint32_t r = lanes_below(sm);
      const uint32_t dst = sel ? r : K + lane - r;
      li = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)lane);
      lv = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)sv);
    } else {
      for (uint32_t c0 = 0; c0 < n; c0 += 64) {
        const uint32_t i = c0 + lane;
        const uint32_t d = i < n ? ldw<false>(&dnew[i]) : kInf;
        const bool sel = d == t;
        if (d != kInf && d > t) m = min(m, d);
        const uint64_t sm = __ballot(sel);
        if (sel) stw<false>(&ord[K + lanes_below(sm)], i);
        K += (uint32_t)__popcll(sm);
      }
      sync();
    }
    // (b) level nodes, 64 at a time: tight predecessors give the next-hop
    // rows, out-edges relax the pending nodes
    for (uint32_t q0 = 0; q0 < K; q0 += 64) {
      const uint32_t q = q0 + lane;
      const bool valid = q < K;
      uint32_t i = li, v = lv;
      if (!small) {
        i = valid ? chk(ldw<false>(&ord[q]), n, false, 9, 0) : 0u;
        v = valid ? chk(ldw<false>(&dlist[i]), g.N, false, 10, b) : 0u;
      }
      const uint32_t transit = valid && !g.ovl[v];  // drained: no transit
      const uint32_t jb = valid ? g.nbr_bit[v] : 0u;
      uint32_t cur = kInf, acc = 0;  // row_pairs' open row
      wave_edges(g.row_ptr, v, valid, [&](uint32_t k, uint32_t e, bool act) {
        const uint32_t ik = lane_pull(i, k), tk = lane_pull(transit, k), jk = lane_pull(jb, k);
        uint32_t u = 0, mu = kInf;
        bool tight = false, from_src = false;
        const uint4 q = act ? g.ed[e] : make_uint4(0u, 0u, l, 0u);
        if (act && q.z != l) {
          u = q.x;
          mu = chk(ws_find(hs, u), n, true, 13, kInf);
          if (!(g.ovl[u] && u != g.src)) {
            const uint32_t du = mu != kInf ? ldw<false>(&dnew[mu]) : B.dist[u];
            tight = du != kInf && du + (g.hop ? 1u : q.w) == t;
          }
          if (tk && mu != kInf) {  // relax v -> u (u pending: its value only drops)
            const uint32_t nd = t + q.y;
            if (nd < atomicMin(&dnew[mu], nd)) m = min(m, nd);
          }
          if (tight && u == g.src) {
            from_src = true;
            tight = false;
          }
        }
        // the row ORs, one tight pair at a time in lane order
        row_pairs(__ballot(tight), __ballot(from_src), ik, jk, u, mu, W, nhn, B.nhb, lane, cur, acc);
      });
      if (cur != kInf && lane < W) nhn[(size_t)cur * W + lane] = acc;
    }
    sync();
    t = wave_min32(m);
    if (ph) ph_add<GPH>(ph, 9, 1, lane == 0);
  }
  WI_STAMP(3);
  // ---- digest delta over D, scratch reset ----
  uint32_t nd_ = 0, nn_ = 0;
  uint64_t dh = 0;
  for (uint32_t i = lane; i < n; i += 64) {
    const uint32_t v = ldw<false>(&dlist[i]);
    const uint32_t d1 = ldw<false>(&dnew[i]), d0 = B.dist[v];
    uint64_t f0, f1;
    bool diff = d1 == kInf;
    row_pair_hash<false>(B.nhb + (size_t)v * W, nhn + (size_t)i * W, W, f0, f1, diff);
    const uint64_t base = mix64((uint64_t)v + 1);
    nd_ += d1 != d0;
    nn_ += diff;
    dh += (d1 == kInf ? 0ull : mix64(base + d1) ^ f1) - (mix64(base + d0) ^ f0);
    stw<false>(&dnew[i], ws_slot(hs, v));  // (every lookup is done: find the slots, then clear)
  }
  sync();
  for (uint32_t i = lane; i < n; i += 64) {
    const uint32_t q = ldw<false>(&dnew[i]);
    if (q <= hs.mask) ws_st(&hs.tab[q], kSlotEmpty);
  }
  if (nd_) atomicAdd(&ctl->ndist, (unsigned long long)nd_);
  if (nn_) atomicAdd(&ctl->nnh, (unsigned long long)nn_);
  if (dh) atomicAdd(&ctl->dh, (unsigned long long)dh);
  sync();
  if (lane == 0)
    *out = spf_whatif_digest{(uint32_t)ldq<false>(&ctl->ndist), (uint32_t)ldq<false>(&ctl->nnh),
                             (uint64_t)(*B.H + ldq<false>(&ctl->dh))};
  sync();
  WI_STAMP(5);
#undef WI_STAMP
  return true;
}

// The profiled instances' phase-counter row of `team` (16 slots) in a
// region of `rows` rows: a team past the region sets bit 5 of the fault word
// (kernel in bits 24-31) and counts nothing -- the layout of the prof buffer
// ([block / group teams][base][wave teams] x 16, spf_whatif_plan_create) is
// checked, not assumed.
__device__ __forceinline__ uint64_t* prof_row(unsigned long long* prof, size_t team, uint32_t rows,
                                              uint32_t kernel, uint32_t* fault) {
  if (team < rows) return reinterpret_cast<uint64_t*>(prof + 16 * team);
  if (fault) __hip_atomic_fetch_or(fault, 32u | (kernel << 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return nullptr;
}

// wave teams over the hot list; failures whose D overflows kWaveCap are
// queued for the workgroup teams.  PROF (SPF_WHATIF_PROF): separate
// instances with the per-team phase counters (prof row `team`, prof_rows
// rows) -- 1: in registers, stored at team exit; 2: global read-modify-writes
// per event -- so the production instance's registers, which set its
// co-residency with the group teams (spf_whatif_plan_create), do not change
// with diagnostics.
template <int PROF>
__global__ __launch_bounds__(256) void repair_wave_kernel(
    WiGraph g, WiBase B, const uint2* __restrict__ hot, const uint32_t* __restrict__ n_hot,
    uint32_t* cursor, uint2* big, uint32_t* n_big, unsigned long long* tab, uint32_t* dlist,
    uint32_t* dnew, uint32_t* nhn, uint32_t* lvl, uint32_t* ord, spf_whatif_digest* out, uint32_t cap,
    uint32_t tab_log2, unsigned long long* prof, uint32_t prof_rows) {
  __shared__ TeamCtl ctl[4];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t team = (size_t)blockIdx.x * 4 + w;
  const WaveSet hs{tab + (team << tab_log2), (1u << tab_log2) - 1u, 32u - tab_log2};
  dlist += team * cap;
  dnew += team * cap;
  nhn += team * cap * g.W;
  lvl += team * (cap + 1);
  ord += team * 2 * cap;  // level list + its hubs
  const uint32_t total = *n_hot;
  uint64_t ph[12] = {};
  uint64_t* gph = PROF == 2 ? prof_row(prof, team, prof_rows, 1, lane == 0 ? g.fault : nullptr) : nullptr;
  for (;;) {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(cursor, 1u);
    k = __builtin_amdgcn_readlane(k, 0);
    if (k >= total) break;
    const uint2 h = hot[k];
    if (!repair_wave<PROF != 0, PROF == 2>(g, B, hs, dlist, dnew, nhn, ord, cap, &ctl[w], lane, h.y,
                                          out + h.x, PROF == 1 ? ph : gph)) {
      if (lane == 0) big[atomicAdd(n_big, 1u)] = h;
    }
  }
  if (PROF == 1 && lane == 0)
    if (uint64_t* r = prof_row(prof, team, prof_rows, 1, g.fault))
      for (int q = 0; q < 12; ++q) r[q] = ph[q];
}

template <int PROF>
__global__ __launch_bounds__(1024) void repair_block_kernel(
    WiGraph g, WiBase B, const uint2* __restrict__ big, const uint32_t* __restrict__ n_big,
    uint32_t* mark, uint32_t* dlist, uint32_t* dnew, uint32_t* nhn, uint32_t* lvl, uint32_t* ord,
    spf_whatif_digest* out, unsigned long long* prof, uint32_t prof_rows) {
  __shared__ TeamCtl ctl;
  // the largest repairs are the critical path of a batch and share their CU
  // with wave teams running concurrently: win the issue arbitration
  __builtin_amdgcn_s_setprio(3);
  const size_t team = blockIdx.x;
  mark += team * g.N;
  dlist += team * g.N;
  dnew += team * g.N;
  nhn += team * (size_t)g.N * g.W;
  lvl += team * ((size_t)g.N + 1);
  ord += team * 2 * (size_t)g.N;  // level list + its hubs
  const uint32_t total = *n_big;
  uint64_t ph[12] = {};
  uint64_t* gph =
      PROF == 2 ? prof_row(prof, team, prof_rows, 2, threadIdx.x == 0 ? g.fault : nullptr) : nullptr;
  for (uint32_t k = blockIdx.x; k < total; k += gridDim.x) {
    const uint2 h = big[k];
    repair<1024, false, false, PROF == 2>(g, B, mark, dlist, dnew, nhn, lvl, ord, g.N, &ctl,
                                          threadIdx.x, h.y, out + h.x, PROF == 1 ? ph : gph);
  }
  if (PROF == 1 && threadIdx.x == 0)
    if (uint64_t* r = prof_row(prof, team, prof_rows, 2, g.fault))
      for (int q = 0; q < 12; ++q) r[q] = ph[q];
}

// The classified big failures, largest subtree first (the order the group
// teams pull them in): a rank sort by one workgroup; lists longer than
// kSortCap keep their order.
constexpr uint32_t kSortCap = 8192;
__global__ __launch_bounds__(1024) void sort_big_kernel(const uint2* __restrict__ in,
                                                        const uint32_t* __restrict__ n_in,
                                                        const uint32_t* __restrict__ sub,
                                                        const uint32_t* __restrict__ col,
                                                        uint2* __restrict__ out) {
  const uint32_t n = *n_in;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (n > kSortCap) {
      out[i] = in[i];
      continue;
    }
    const uint32_t ki = sub[col[in[i].y]];
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j) {
      const uint32_t kj = sub[col[in[j].y]];
      r += kj > ki || (kj == ki && j < i);
    }
    out[r] = in[i];
  }
}

// Group teams of G workgroups of kGroupWg threads (one grid-resident launch, a
// workgroup per CU): the largest repairs get G CUs each.  Half-size
// workgroups (8 waves, 2 per SIMD) co-reside with the wave teams' blocks, so
// both progress from the start.  Members of a team sit on one XCD (blocks x
// and x + 8 share one); teams pull failures, largest first.
constexpr int kGroupWg = 512;
template <int G, int PROF>
__global__ __launch_bounds__(kGroupWg) void repair_group_kernel(
    WiGraph g, WiBase B, const uint2* __restrict__ big, const uint32_t* __restrict__ n_big,
    uint32_t* cursor, TeamCtl* ctls, uint32_t* mark, uint32_t* dlist, uint32_t* dnew,
    uint32_t* nhn, uint32_t* lvl, uint32_t* ord, spf_whatif_digest* out,
    unsigned long long* prof, uint32_t prof_rows) {
  constexpr int TEAM = kGroupWg * G;
  __builtin_amdgcn_s_setprio(3);
  const uint32_t idx = blockIdx.x >> 3;
  const uint32_t member = idx % G;
  const size_t team = (size_t)(idx / G) * 8 + (blockIdx.x & 7);
  TeamCtl* ctl = ctls + team;
  const uint32_t tt = member * kGroupWg + threadIdx.x;
  mark += team * g.N;
  dlist += team * g.N;
  dnew += team * g.N;
  nhn += team * (size_t)g.N * g.W;
  lvl += team * ((size_t)g.N + 1);
  ord += team * 2 * (size_t)g.N;
  const uint32_t total = *n_big;
  uint64_t ph[12] = {};
  uint64_t* gph = PROF == 2 ? prof_row(prof, team, prof_rows, 3, tt == 0 ? g.fault : nullptr) : nullptr;
  for (;;) {
    if (tt == 0) stw<true>(&ctl->next, atomicAdd(cursor, 1u));
    team_sync<TEAM, true>(ctl, g.fault);
    const uint32_t k = ldw<true>(&ctl->next);
    if (k >= total) break;  // team-uniform
    const uint2 h = big[k];
    repair<TEAM, true, false, PROF == 2>(g, B, mark, dlist, dnew, nhn, lvl, ord, g.N, ctl, tt, h.y,
                                         out + h.x, PROF == 1 ? ph : gph);
  }
  if (PROF == 1 && tt == 0)
    if (uint64_t* r = prof_row(prof, team, prof_rows, 3, g.fault))
      for (int q = 0; q < 12; ++q) r[q] = ph[q];
}

struct GroupArgs {
  WiGraph g;
  WiBase B;
  const uint2* big;
  const uint32_t* n_big;
  uint32_t* cursor;
  TeamCtl* ctls;
  uint32_t *mark, *dlist, *dnew, *nhn, *lvl, *ord;
  spf_whatif_digest* out;
  unsigned long long* prof;
  uint32_t prof_rows;  // rows of the prof region the group teams own
};

// A launch whose blocks meet at barriers (XGrid, the group teams'
// team_sync): a regular launch of at most `per_cu` blocks per CU, checked
// against the occupancy calculator so that every block of the grid fits on
// the chip at once -- the barriers' precondition, which the cooperative
// launch used to assert.  Blocks of other kernels running beside it (the
// wave teams) never wait on it, so its blocks all become resident.  (The
// cooperative launch is not used: under rocprofv3 a process that made one
// faulted in exit-time runtime teardown)
hipError_t launch_resident(const void* kernel, uint32_t blocks, uint32_t threads, void** args,
                           uint32_t n_cu, hipStream_t s) {
  int fit = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit, kernel, threads, 0);
  if (e != hipSuccess) return e;
  if (fit < 1 || (uint64_t)fit * n_cu < blocks) return hipErrorCooperativeLaunchTooLarge;
  return hipLaunchKernel(kernel, dim3(blocks), dim3(threads), args, 0, s);
}

// SPF_WHATIF_PROF: unset 0 (production instances), "global" 2 (per-event
// global read-modify-writes), anything else 1 (register counters)
int whatif_prof_mode() {
  const char* e = std::getenv("SPF_WHATIF_PROF");
  return !e ? 0 : (std::strcmp(e, "global") == 0 ? 2 : 1);
}

template <int G>
const void* group_kernel_g(int prof) {
  return prof == 2 ? (const void*)repair_group_kernel<G, 2>
                   : prof == 1 ? (const void*)repair_group_kernel<G, 1> : (const void*)repair_group_kernel<G, 0>;
}

const void* group_kernel(uint32_t G, int prof) {
  switch (G) {
    case 2: return group_kernel_g<2>(prof);
    case 4: return group_kernel_g<4>(prof);
    case 8: return group_kernel_g<8>(prof);
    case 16: return group_kernel_g<16>(prof);
    default: return nullptr;
  }
}

// one launch, a workgroup per CU (every member of every team resident at
// once: the team barrier's precondition)
hipError_t launch_group(uint32_t G, GroupArgs& a, uint32_t n_cu, int prof, hipStream_t s) {
  const void* k = group_kernel(G, a.prof ? prof : 0);
  if (!k) return hipErrorInvalidValue;
  void* args[] = {&a.g, &a.B, &a.big, &a.n_big, &a.cursor, &a.ctls, &a.mark, &a.dlist, &a.dnew,
                  &a.nhn, &a.lvl, &a.ord, &a.out, &a.prof, &a.prof_rows};
  return launch_resident(k, n_cu, kGroupWg, args, n_cu, s);
}

__global__ void base_digest_kernel(spf_whatif_digest* o, const unsigned long long* H) {
  *o = spf_whatif_digest{0u, 0u, (uint64_t)*H};
}

}  // namespace

struct spf_whatif_plan {
  spf_ctx* ctx = nullptr;
  uint32_t src = 0, n_fail = 0, W = 0, wave_teams = 0;
  uint64_t epoch = 0;  // graph state the plan was derived from
  DevBuf<uint32_t> d_fails, d_link_edge, d_nbr_bit, d_dist, d_q, d_q2, d_bm, d_nhb, d_ctr;
  DevBuf<uint32_t> d_bar;  // the base kernel's grid-barrier counters
  DevBuf<uint32_t> d_lvl, d_order, d_misc;
  DevBuf<unsigned long long> d_H;
  DevBuf<uint2> d_hot, d_big, d_big0, d_big1;  // d_big1: d_big0 largest first
  // [0] n_hot, [1] cursor, [2] n_big (overflow), [3] n_big0 (classified),
  // [4] group teams' cursor
  DevBuf<uint32_t> d_cnt;
  DevBuf<unsigned char> d_ctl;  // group teams' TeamCtl
  uint32_t group = 0, group_teams = 0;  // workgroups per group team (0: one-workgroup teams)
  int prof_mode = 0;                    // whatif_prof_mode() at plan creation
  DevBuf<uint32_t> d_parent, d_sub;
  uint32_t big_teams = 0;
  // |D| a wave team holds (its scratch) and the parent-subtree size past
  // which classify sends a failure to the workgroup teams (A/B:
  // SPF_WHATIF_WAVECAP, SPF_WHATIF_CLASSIFY)
  uint32_t wave_cap = kWaveCap, classify_cap = kWaveCap;
  DevBuf<unsigned long long> d_prof;  // SPF_WHATIF_PROF diagnostics
  DevBuf<uint32_t> w_dlist, w_dnew, w_nhn, w_lvl, w_ord;  // wave-team scratch
  DevBuf<unsigned long long> w_tab;  // wave-team node sets (WaveSet), 1 << tab_log2 slots each
  DevBuf<uint4> d_ed;                 // interleaved edges (WiGraph::ed)
  uint32_t tab_log2 = 0;
  DevBuf<uint32_t> b_mark, b_dlist, b_dnew, b_nhn, b_lvl, b_ord;  // workgroup-team scratch
  DevBuf<uint32_t> c_mark, c_dlist, c_dnew, c_nhn, c_lvl, c_ord;  // same, concurrent set
  std::vector<hipEvent_t> ev;
  uint32_t timing_cap = 0, timing_n = 0;
  hipStream_t last = nullptr;  // stream of the last execute (spf_whatif_stats waits on it)
  // zero / negative metrics or u64 labels: every failure on the exact kernel
  std::unique_ptr<spfi::ExactWhatIf> exact;
  ~spf_whatif_plan() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
};

namespace spfi {

// Blocks of a grid-barrier launch: `per_cu` 512-thread blocks per CU, clamped
// to what the occupancy calculator says stays co-resident (XGrid needs every
// block resident).  SPF_COOP_PER_CU overrides (A/B).
uint32_t coop_blocks(spf_ctx* c, const void* kernel, uint32_t per_cu) {
  if (const char* e = std::getenv("SPF_COOP_PER_CU")) per_cu = std::max(1, atoi(e));
  int fit = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit, kernel, kCoopThreads, 0) != hipSuccess ||
      fit < 1) {
    (void)hipGetLastError();
    fit = 1;
  }
  return c->n_cu * std::min<uint32_t>(per_cu, (uint32_t)fit);
}

spf_status launch_gsssp(spf_ctx* c, uint32_t src, bool hop, const uint32_t* ign, uint32_t* dist,
                        hipStream_t s) {
  const uint32_t N = c->N;
  HIP_TRY(c, c->d_gq.alloc(N));
  HIP_TRY(c, c->d_gq2.alloc(N));
  HIP_TRY(c, c->d_gbm.alloc((N + 31) / 32));
  HIP_TRY(c, c->d_gctr.alloc(4));
  HIP_TRY(c, c->d_gbar.alloc(kGridBarWords));
  HIP_TRY(c, hipMemsetAsync(c->d_gbar.p, 0, 4 * kGridBarWords, s));
  CoopSssp a{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_ovl.p, c->d_link.p, ign, N, src,
             hop ? 1u : 0u, dist, c->d_gq.p, c->d_gq2.p, c->d_gbm.p, c->d_gctr.p};
  a.bar = c->d_gbar.p;
  a.fault = c->d_fault.p;
  void* args[] = {&a};
  if (const spf_status st = resident_order(c, s); st != SPF_OK) return st;
  HIP_TRY(c, launch_resident((const void*)gsssp_coop_kernel,
                             coop_blocks(c, (const void*)gsssp_coop_kernel, 1), kCoopThreads, args,
                             c->n_cu, s));
  return resident_done(c, s);
}

spf_status launch_big(spf_ctx* c, spf_plan* p, uint32_t* d_dist, uint32_t* d_nh, bool hop,
                      hipStream_t s) {
  const uint32_t N = c->N;
  HIP_TRY(c, p->b_q.alloc(N));
  HIP_TRY(c, p->b_q2.alloc(N));
  HIP_TRY(c, p->b_bm.alloc((N + 31) / 32));
  HIP_TRY(c, p->b_ctr.alloc(4));
  HIP_TRY(c, p->b_bar.alloc(kGridBarWords));
  HIP_TRY(c, hipMemsetAsync(p->b_bar.p, 0, 4 * kGridBarWords, s));
  if (!p->b_nbr_bit.p) {
    HIP_TRY(c, p->b_nbr_bit.alloc(N));
    HIP_TRY(c, hipMemsetAsync(p->b_nbr_bit.p, 0xFF, 4ull * N, s));
  }
  HIP_TRY(c, p->b_nhb.alloc((size_t)N * p->wmax));
  HIP_TRY(c, p->b_lvl.alloc(kLevelCap + 1));
  HIP_TRY(c, p->b_order.alloc(N));
  HIP_TRY(c, p->b_misc.alloc(8));
  HIP_TRY(c, p->b_parent.alloc(N));
  WiGraph g{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_rev.p, c->d_link.p, c->d_ovl.p,
            p->b_nbr_bit.p, N, 0u, 1u, hop ? 1u : 0u, c->d_fault.p};
  BigArgs a{CoopSssp{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_ovl.p, c->d_link.p, nullptr, N,
                     0u, hop ? 1u : 0u, d_dist, p->b_q.p, p->b_q2.p, p->b_bm.p, p->b_ctr.p},
            g, p->d_srcs.p, p->n_src, c->d_nb_ptr.p, c->d_nb_id.p, d_dist, c->pitch, d_nh,
            p->d_nh_off.p, p->b_nbr_bit.p, p->b_nhb.p, p->b_lvl.p, p->b_order.p, p->b_misc.p,
            p->b_parent.p};
  a.sp.bar = p->b_bar.p;
  a.sp.fault = c->d_fault.p;
  void* args[] = {&a};
  if (const spf_status st = resident_order(c, s); st != SPF_OK) return st;
  HIP_TRY(c, launch_resident((const void*)spf_big_kernel,
                             coop_blocks(c, (const void*)spf_big_kernel, 1), kCoopThreads, args,
                             c->n_cu, s));
  return resident_done(c, s);
}

}  // namespace spfi

extern "C" {

spf_status spf_whatif_plan_create(spf_ctx* c, uint32_t src, const uint32_t* fail_links,
                                  uint32_t n_fail, spf_whatif_plan** out) {
  if (!c || !out) return fail(c, SPF_E_INVALID, "spf_whatif_plan_create: NULL argument");
  *out = nullptr;
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (src >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", src);
  auto p = std::make_unique<spf_whatif_plan>();
  p->ctx = c;
  p->src = src;
  const uint32_t N = c->N, E = c->E;
  // link -> one of its directed edges (up links only: a dead slot is a self-loop)
  std::vector<uint32_t> link_edge((size_t)c->max_link + 1, kInf);
  for (uint32_t u = 0; u < N; ++u)
    for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
      if (c->col[e] != u && link_edge[c->link[e]] == kInf) link_edge[c->link[e]] = e;
  std::vector<uint32_t> fails;
  if (fail_links) {
    fails.assign(fail_links, fail_links + n_fail);
    for (uint32_t l : fails)
      if (l > c->max_link || link_edge[l] == kInf)
        return fail(c, SPF_E_INVALID, "link %u is not an up link of the graph", l);
  } else {  // every up link, ascending id
    for (uint32_t l = 0; l <= c->max_link && E; ++l)
      if (link_edge[l] != kInf) fails.push_back(l);
  }
  p->n_fail = (uint32_t)fails.size();
  if (c->nonpos || c->needs64) {
    // zero / negative metrics, u64 labels: the exact kernel replays
    // runSpf(src, true, {l}) for every failure touching a pathLink
    HIP_TRY(c, hipSetDevice(c->device));
    p->exact = std::make_unique<spfi::ExactWhatIf>();
    const spf_status st = exact_whatif_prepare(c, p->exact.get(), src, fails, link_edge);
    if (st != SPF_OK) return st;
    if (!fails.empty()) HIP_TRY(c, p->d_fails.upload(fails.data(), fails.size(), c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    p->W = p->exact->W;
    p->epoch = c->epoch;
    *out = p.release();
    return SPF_OK;
  }
  // bit of each distinct up neighbour of src
  std::vector<uint32_t> nbr_bit(N, kInf);
  const uint32_t k = c->nb_ptr[src + 1] - c->nb_ptr[src];
  for (uint32_t j = 0; j < k; ++j) nbr_bit[c->nb_id[c->nb_ptr[src] + j]] = j;
  p->W = std::max<uint32_t>(1, (k + 31) / 32);
  {  // wave teams: 16 per CU within the scratch budget (failures on the
     // 1M-link graph, r02_v75 with 8 GB: 12: 17.9 ms, 16: 16.4, 20: 20.2,
     // 24: 19.6; r02_v30 before the lane-read / DPP repairs: 12 best)
     // (SPF_WHATIF_WAVES=<per CU>, a multiple of 4: A/B)
    const char* e = std::getenv("SPF_WHATIF_WAVES");
    const size_t per_cu = e ? std::max(4, atoi(e) & ~3) : 16;
    if (const char* ec = std::getenv("SPF_WHATIF_WAVECAP")) p->wave_cap = std::max(64, atoi(ec));
    p->classify_cap = p->wave_cap;
    if (const char* ec = std::getenv("SPF_WHATIF_CLASSIFY")) p->classify_cap = std::max(1, atoi(ec));
    const size_t cap = p->wave_cap;
    const size_t per_team = 4ull * (N + cap * (4ull + p->W) + cap + 1);
    const size_t fit = std::max<size_t>(4, kWaveScratch / per_team) & ~size_t(3);
    p->wave_teams = (uint32_t)std::min<size_t>(per_cu * c->n_cu, fit);
  }
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, p->d_fails.upload(fails.data(), fails.size(), c->stream));
  HIP_TRY(c, p->d_link_edge.upload(link_edge.data(), link_edge.size(), c->stream));
  HIP_TRY(c, p->d_nbr_bit.upload(nbr_bit.data(), N, c->stream));
  HIP_TRY(c, p->d_dist.alloc(N));
  HIP_TRY(c, p->d_q.alloc(N));
  HIP_TRY(c, p->d_q2.alloc(N));
  HIP_TRY(c, p->d_bm.alloc((N + 31) / 32));
  HIP_TRY(c, p->d_nhb.alloc((size_t)N * p->W));
  HIP_TRY(c, p->d_ctr.alloc(4));
  HIP_TRY(c, p->d_bar.alloc(kGridBarWords));
  HIP_TRY(c, p->d_lvl.alloc(kLevelCap + 1));
  HIP_TRY(c, p->d_order.alloc(N));
  HIP_TRY(c, p->d_misc.alloc(8));
  HIP_TRY(c, p->d_H.alloc(1));
  HIP_TRY(c, p->d_hot.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, p->d_big.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, p->d_big0.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, p->d_big1.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, p->d_parent.alloc(N));
  HIP_TRY(c, p->d_sub.alloc(N));
  if (!c->side) {  // the classified big failures' workgroup teams run here
    HIP_TRY(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    HIP_TRY(c, hipEventCreateWithFlags(&c->side_fork, hipEventDisableTiming));
    HIP_TRY(c, hipEventCreateWithFlags(&c->side_join, hipEventDisableTiming));
  }
  HIP_TRY(c, p->d_cnt.alloc(8));
  {  // workgroup teams: one per CU, two sets (b_*, c_*) within the scratch budget
    const size_t per_team = 4ull * ((size_t)N * (6 + p->W) + 1);
    p->big_teams = (uint32_t)std::max<size_t>(4, std::min<size_t>(c->n_cu, kBigScratch / 2 / per_team));
  }
  const size_t bt = p->big_teams;
  {  // group teams over the concurrent (c_*) scratch sets: G workgroups each,
     // n_cu / G teams (a multiple of 8: members share an XCD), no more teams
     // than scratch sets (SPF_WHATIF_GROUP=1: one-workgroup teams, A/B).
     // G = 8 by default: ba_whatif's failures took 9.3 ms at G = 8 against
     // 10.2 at 4 and 14.8 at 16 (profiles/r05_whatif/flat)
    const char* e = std::getenv("SPF_WHATIF_GROUP");
    uint32_t G = e ? (uint32_t)atoi(e) : 8u;
    if (G > 1) {
      while (G <= 16 && (c->n_cu / G > bt || (c->n_cu / G) % 8)) G *= 2;
      if (G <= 16 && c->n_cu % (8 * G) == 0 && c->n_cu / G >= 8) {
        p->group = G;
        p->group_teams = c->n_cu / G;
        HIP_TRY(c, p->d_ctl.alloc(sizeof(TeamCtl) * p->group_teams));
      }
    }
  }
  if (p->group) {
    // The group teams' members must all be resident while the wave teams'
    // blocks hold their CUs (launched beside them on the side stream; a
    // member that cannot be placed stalls its team at every barrier).  Per
    // SIMD: the wave teams' waves (one per 256-thread block) and the group
    // workgroup's 2 waves share 512 VGPRs (granule 8).  Fewer wave teams per
    // CU until both fit.  (Round 4's stamp pointer in the wave kernel --
    // 75 -> 80+ VGPRs at 4 waves per SIMD beside 2 x 88 -- broke this sum.)
    hipFuncAttributes fw{}, fg{};
    const int pm = whatif_prof_mode();
    const void* wk = pm == 2 ? (const void*)repair_wave_kernel<2>
                             : pm == 1 ? (const void*)repair_wave_kernel<1> : (const void*)repair_wave_kernel<0>;
    HIP_TRY(c, hipFuncGetAttributes(&fw, wk));
    HIP_TRY(c, hipFuncGetAttributes(&fg, group_kernel(p->group, pm)));
    const auto gran = [](int r) { return (uint32_t)((std::max(r, 1) + 7) & ~7); };
    const uint32_t per_simd_group = kGroupWg / 64 / 4;
    const uint32_t vw = gran(fw.numRegs), vg = gran(fg.numRegs);
    uint32_t per_simd_wave = (p->wave_teams + 4 * c->n_cu - 1) / (4 * c->n_cu);
    while (per_simd_wave > 1 && per_simd_wave * vw + per_simd_group * vg > 512) --per_simd_wave;
    p->wave_teams = std::min(p->wave_teams, per_simd_wave * 4 * c->n_cu);
    if (std::getenv("SPF_WHATIF_DEBUG"))
      std::fprintf(stderr, "whatif: wave kernel %d VGPRs, group<%u> %d VGPRs: %u wave teams (%u per SIMD)\n",
                   fw.numRegs, p->group, fg.numRegs, p->wave_teams, per_simd_wave);
  }
  const size_t wt = p->wave_teams;
  while ((1u << p->tab_log2) < 4 * p->wave_cap) ++p->tab_log2;
  {  // WiGraph::ed from the context's host CSR (the plan lives within one graph epoch)
    std::vector<uint4> ed(std::max<uint32_t>(c->E, 1));
    for (uint32_t e = 0; e < c->E; ++e) ed[e] = make_uint4(c->col[e], c->wt[e], c->link[e], c->wt[c->rev[e]]);
    HIP_TRY(c, p->d_ed.upload(ed.data(), ed.size(), c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // (ed is freed on return)
  }
  HIP_TRY(c, p->w_tab.alloc(wt << p->tab_log2));
  HIP_TRY(c, p->w_dlist.alloc(wt * p->wave_cap));
  HIP_TRY(c, p->w_dnew.alloc(wt * p->wave_cap));
  HIP_TRY(c, p->w_nhn.alloc(wt * p->wave_cap * p->W));
  HIP_TRY(c, p->w_lvl.alloc(wt * (p->wave_cap + 1)));
  HIP_TRY(c, p->w_ord.alloc(wt * 2 * p->wave_cap));
  HIP_TRY(c, p->b_mark.alloc(bt * N));
  HIP_TRY(c, p->b_dlist.alloc(bt * N));
  HIP_TRY(c, p->b_dnew.alloc(bt * N));
  HIP_TRY(c, p->b_nhn.alloc(bt * N * p->W));
  HIP_TRY(c, p->b_lvl.alloc(bt * (N + 1)));
  HIP_TRY(c, p->b_ord.alloc(bt * 2 * N));
  HIP_TRY(c, p->c_mark.alloc(bt * N));
  HIP_TRY(c, p->c_dlist.alloc(bt * N));
  HIP_TRY(c, p->c_dnew.alloc(bt * N));
  HIP_TRY(c, p->c_nhn.alloc(bt * N * p->W));
  HIP_TRY(c, p->c_lvl.alloc(bt * (N + 1)));
  HIP_TRY(c, p->c_ord.alloc(bt * 2 * N));
  HIP_TRY(c, hipMemsetAsync(p->c_mark.p, 0xFF, bt * N * 4, c->stream));
  // marks start (and are always left) at kInf
  HIP_TRY(c, hipMemsetAsync(p->w_tab.p, 0xFF, (wt << p->tab_log2) * 8, c->stream));
  HIP_TRY(c, hipMemsetAsync(p->b_mark.p, 0xFF, bt * N * 4, c->stream));
  p->prof_mode = whatif_prof_mode();
  if (p->prof_mode) {  // [bt teams][base][wave teams] x 16 (row bounds checked in the kernels)
    const size_t slots = 16 * (bt + 1 + p->wave_teams) + 128;  // + the base's per-level clocks
    HIP_TRY(c, p->d_prof.alloc(slots));
    HIP_TRY(c, hipMemsetAsync(p->d_prof.p, 0, slots * 8, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  p->epoch = c->epoch;
  *out = p.release();
  return SPF_OK;
}

void spf_whatif_plan_destroy(spf_whatif_plan* p) { delete p; }
uint32_t spf_whatif_plan_failures(const spf_whatif_plan* p) { return p ? p->n_fail : 0; }

spf_status spf_whatif_plan_links(const spf_whatif_plan* p, uint32_t* links) {
  if (!p || !links) return SPF_E_INVALID;
  spf_ctx* c = p->ctx;
  HIP_TRY(c, hipMemcpy(links, p->d_fails.p, 4ull * p->n_fail, hipMemcpyDeviceToHost));
  return SPF_OK;
}

spf_status spf_whatif_execute(spf_whatif_plan* p, spf_whatif_digest* d_out,
                              spf_whatif_digest* d_base, void* stream) {
  if (!p || !d_out) return fail(p ? p->ctx : nullptr, SPF_E_INVALID, "spf_whatif_execute: NULL");
  spf_ctx* c = p->ctx;
  if (!c->loaded) return fail(c, SPF_E_STATE, "graph no longer loaded");
  if (p->epoch != c->epoch)
    return fail(c, SPF_E_STATE, "graph changed since the plan was created: recreate it");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  p->last = s;
  const uint32_t N = c->N;
  hipEvent_t* ev = nullptr;
  if (p->timing_cap) {
    ev = &p->ev[3 * (p->timing_n % p->timing_cap)];
    ++p->timing_n;
    HIP_TRY(c, hipEventRecord(ev[0], s));
  }
  if (p->exact) {
    const spf_status st = exact_whatif_launch(c, p->exact.get(), d_out, d_base, s, ev ? ev[1] : nullptr);
    if (st != SPF_OK) return st;
    if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
    c->solves += 1ull + p->n_fail;
    return SPF_OK;
  }
  WiGraph g{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_rev.p, c->d_link.p, c->d_ovl.p,
            p->d_nbr_bit.p, N, p->src, p->W};
  g.fault = c->d_fault.p;
  g.ed = p->d_ed.p;
  // 1. unfailed SPF, next hops, hash: one grid-resident launch
  {
    BaseArgs a{CoopSssp{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_ovl.p, c->d_link.p, nullptr,
                        N, p->src, 0u, p->d_dist.p, p->d_q.p, p->d_q2.p, p->d_bm.p, p->d_ctr.p},
               g, p->d_nhb.p, p->d_lvl.p, p->d_order.p, p->d_misc.p, p->d_H.p,
               p->d_prof.p ? p->d_prof.p + 16ull * p->big_teams : nullptr, p->d_parent.p,
               p->d_sub.p};
    a.sp.bar = p->d_bar.p;
    a.sp.fault = c->d_fault.p;
    if (p->d_prof.p) a.lprof = p->d_prof.p + 16ull * (p->big_teams + 1 + p->wave_teams);
    HIP_TRY(c, hipMemsetAsync(p->d_bar.p, 0, 4 * kGridBarWords, s));
    void* args[] = {&a};
    if (const spf_status st = resident_order(c, s); st != SPF_OK) return st;
    HIP_TRY(c, launch_resident((const void*)whatif_base_kernel,
                               coop_blocks(c, (const void*)whatif_base_kernel, 1), kCoopThreads,
                               args, c->n_cu, s));
    if (const spf_status st = resident_done(c, s); st != SPF_OK) return st;
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[1], s));
  // 2. failures
  HIP_TRY(c, hipMemsetAsync(p->d_cnt.p, 0, 32, s));
  if (p->group) HIP_TRY(c, hipMemsetAsync(p->d_ctl.p, 0, sizeof(TeamCtl) * p->group_teams, s));
  if (p->n_fail) {
    hipLaunchKernelGGL(classify_kernel, dim3((p->n_fail + 255) / 256), dim3(256), 0, s, g,
                       p->d_dist.p, p->d_H.p, p->d_fails.p, p->n_fail, p->d_link_edge.p,
                       p->d_sub.p, p->classify_cap, d_out, p->d_hot.p, p->d_cnt.p, p->d_big0.p,
                       p->d_cnt.p + 3);
    HIP_TRY(c, hipGetLastError());
    WiBase B{p->d_dist.p, p->d_nhb.p, p->d_H.p};
    // failures classified big (parent subtree > kWaveCap) go to workgroup
    // teams on a second stream right away, beside the wave teams; separate
    // scratch, separate list, no dependence between the two grids
    hipStream_t side = c->side ? c->side : s;
    if (c->side) {
      HIP_TRY(c, hipEventRecord(c->side_fork, s));
      HIP_TRY(c, hipStreamWaitEvent(c->side, c->side_fork, 0));
    }
    bool grouped = false;
    if (p->group) {
      hipLaunchKernelGGL(sort_big_kernel, dim3(1), dim3(1024), 0, side, p->d_big0.p, p->d_cnt.p + 3,
                         p->d_sub.p, c->d_col.p, p->d_big1.p);
      HIP_TRY(c, hipGetLastError());
      GroupArgs ga{g, B, p->d_big1.p, p->d_cnt.p + 3, p->d_cnt.p + 4,
                   reinterpret_cast<TeamCtl*>(p->d_ctl.p), p->c_mark.p, p->c_dlist.p, p->c_dnew.p,
                   p->c_nhn.p, p->c_lvl.p, p->c_ord.p, d_out, p->d_prof.p, p->big_teams};
      if (const spf_status st = resident_order(c, side); st != SPF_OK) return st;
      grouped = launch_group(p->group, ga, c->n_cu, p->prof_mode, side) == hipSuccess;
      if (!grouped) (void)hipGetLastError();  // fall back to one-workgroup teams
      else if (const spf_status st = resident_done(c, side); st != SPF_OK) return st;
    }
    if (!grouped) {
      const uint32_t bt = p->big_teams;
      if (p->prof_mode == 2)
        hipLaunchKernelGGL(repair_block_kernel<2>, dim3(bt), dim3(1024), 0, side, g, B, p->d_big0.p,
                           p->d_cnt.p + 3, p->c_mark.p, p->c_dlist.p, p->c_dnew.p, p->c_nhn.p,
                           p->c_lvl.p, p->c_ord.p, d_out, p->d_prof.p, bt);
      else if (p->prof_mode == 1)
        hipLaunchKernelGGL(repair_block_kernel<1>, dim3(bt), dim3(1024), 0, side, g, B, p->d_big0.p,
                           p->d_cnt.p + 3, p->c_mark.p, p->c_dlist.p, p->c_dnew.p, p->c_nhn.p,
                           p->c_lvl.p, p->c_ord.p, d_out, p->d_prof.p, bt);
      else
        hipLaunchKernelGGL(repair_block_kernel<0>, dim3(bt), dim3(1024), 0, side, g, B, p->d_big0.p,
                           p->d_cnt.p + 3, p->c_mark.p, p->c_dlist.p, p->c_dnew.p, p->c_nhn.p,
                           p->c_lvl.p, p->c_ord.p, d_out, nullptr, 0u);
    }
    HIP_TRY(c, hipGetLastError());
    if (c->side) HIP_TRY(c, hipEventRecord(c->side_join, c->side));
    {
      unsigned long long* wp = p->d_prof.p ? p->d_prof.p + 16ull * (p->big_teams + 1) : nullptr;
      const uint32_t wr = p->wave_teams;
      if (p->prof_mode == 2)
        hipLaunchKernelGGL(repair_wave_kernel<2>, dim3(p->wave_teams / 4), dim3(256), 0, s, g, B,
                           p->d_hot.p, p->d_cnt.p, p->d_cnt.p + 1, p->d_big.p, p->d_cnt.p + 2,
                           p->w_tab.p, p->w_dlist.p, p->w_dnew.p, p->w_nhn.p, p->w_lvl.p,
                           p->w_ord.p, d_out, p->wave_cap, p->tab_log2, wp, wr);
      else if (p->prof_mode == 1)
        hipLaunchKernelGGL(repair_wave_kernel<1>, dim3(p->wave_teams / 4), dim3(256), 0, s, g, B,
                           p->d_hot.p, p->d_cnt.p, p->d_cnt.p + 1, p->d_big.p, p->d_cnt.p + 2,
                           p->w_tab.p, p->w_dlist.p, p->w_dnew.p, p->w_nhn.p, p->w_lvl.p,
                           p->w_ord.p, d_out, p->wave_cap, p->tab_log2, wp, wr);
      else
        hipLaunchKernelGGL(repair_wave_kernel<0>, dim3(p->wave_teams / 4), dim3(256), 0, s, g, B,
                           p->d_hot.p, p->d_cnt.p, p->d_cnt.p + 1, p->d_big.p, p->d_cnt.p + 2,
                           p->w_tab.p, p->w_dlist.p, p->w_dnew.p, p->w_nhn.p, p->w_lvl.p,
                           p->w_ord.p, d_out, p->wave_cap, p->tab_log2, nullptr, 0u);
    }
    HIP_TRY(c, hipGetLastError());
    hipLaunchKernelGGL(repair_block_kernel<0>, dim3(p->big_teams), dim3(1024), 0, s, g, B, p->d_big.p,
                       p->d_cnt.p + 2, p->b_mark.p, p->b_dlist.p, p->b_dnew.p, p->b_nhn.p,
                       p->b_lvl.p, p->b_ord.p, d_out, nullptr, 0u);
    HIP_TRY(c, hipGetLastError());
    if (c->side) HIP_TRY(c, hipStreamWaitEvent(s, c->side_join, 0));
  }
  if (p->d_prof.p) {  // diagnostics: phase ticks (100 MHz) per team, accumulated over repairs
    const size_t bt = p->big_teams, wt = p->wave_teams;
    std::vector<unsigned long long> h(16ull * (bt + 1 + wt) + 128);
    HIP_TRY(c, hipMemcpyAsync(h.data(), p->d_prof.p, h.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    auto line = [&](const char* who, const unsigned long long* r) {
      std::fprintf(stderr, "whatif %s repairs=%llu sum|D|=%llu max|D|=%llu dial_levels=%llu gave_up=%llu "
                   "bfs=%llu seeds=%llu dial=%llu fallback=%llu digest=%llu (x10ns)\n", who, r[0], r[8],
                   r[10], r[9], r[11], r[1], r[2], r[3], r[4], r[5]);
    };
    for (size_t t = 0; t < bt; ++t) {
      const unsigned long long* r = &h[16 * t];
      if (!r[0]) continue;
      char who[32];
      std::snprintf(who, sizeof who, "team %zu", t);
      line(who, r);
    }
    std::vector<unsigned long long> sum(16, 0);  // the wave teams, summed
    unsigned long long busiest = 0;
    for (size_t t = 0; t < wt; ++t) {
      const unsigned long long* r = &h[16 * (bt + 1 + t)];
      for (int k = 0; k < 16; ++k) sum[k] = k == 10 ? std::max(sum[k], r[k]) : sum[k] + r[k];
      busiest = std::max(busiest, r[1] + r[2] + r[3] + r[4] + r[5]);
    }
    line("wave-teams(sum)", sum.data());
    std::fprintf(stderr, "whatif wave teams %zu, busiest team %llu ticks (x10ns)\n", wt, busiest);
    const unsigned long long* r = &h[16 * bt];
    std::fprintf(stderr, "whatif base sssp=%llu nh=%llu (of which subtree sizes %llu) hash=%llu (x10ns) maxd=%llu levels=%llu W=%u\n",
                 r[1] - r[0], r[2] - r[1], r[6] ? r[2] - r[6] : 0ull, r[3] - r[2], r[4], r[5], p->W);
    const unsigned long long* lv = &h[16 * (bt + 1 + wt)];
    unsigned long long prev = 0;
    std::string line2 = "whatif base levels (distance:nodes:ticks)";
    for (int d = 1; d < 64; ++d) {
      if (!lv[2 * d]) continue;
      const unsigned long long t0 = prev ? prev : lv[2 * d];
      line2 += " " + std::to_string(d) + ":" + std::to_string(lv[2 * d + 1]) + ":" +
               std::to_string(prev ? lv[2 * d] - t0 : 0ull);
      prev = lv[2 * d];
    }
    std::fprintf(stderr, "%s\n", line2.c_str());
  }
  if (d_base) {
    // the unfailed digest: nothing changed, hash = H
    hipLaunchKernelGGL(base_digest_kernel, dim3(1), dim3(1), 0, s, d_base, p->d_H.p);
    HIP_TRY(c, hipGetLastError());
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
  c->solves += 1ull + p->n_fail;
  return SPF_OK;
}

spf_status spf_whatif_stats(spf_whatif_plan* p, uint32_t* n_hot, uint32_t* n_big) {
  if (!p) return SPF_E_INVALID;
  spf_ctx* c = p->ctx;
  uint32_t cnt[4] = {0, 0, 0, 0};
  if (!p->last) return fail(c, SPF_E_STATE, "spf_whatif_stats: no execute yet");
  if (p->exact) {  // every failure is a re-run on the exact kernel (cold ones skipped inside)
    HIP_TRY(c, hipStreamSynchronize(p->last));
    if (n_hot) *n_hot = p->n_fail;
    if (n_big) *n_big = 0;
    return SPF_OK;
  }
  // the counters are written on the execute stream (non-blocking, so the
  // null stream does not order after it): copy on that stream and wait
  HIP_TRY(c, hipMemcpyAsync(cnt, p->d_cnt.p, sizeof cnt, hipMemcpyDeviceToHost, p->last));
  HIP_TRY(c, hipStreamSynchronize(p->last));
  if (const spf_status st = spf_device_check(c); st != SPF_OK) return st;
  if (n_hot) *n_hot = cnt[0] + cnt[3];  // wave list + classified big
  if (n_big) *n_big = cnt[2] + cnt[3];  // wave overflow + classified big
  return SPF_OK;
}

spf_status spf_whatif_enable_timing(spf_whatif_plan* p, uint32_t max_executes) {
  if (!p) return SPF_E_INVALID;
  spf_ctx* c = p->ctx;
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  p->ev.assign(3ull * max_executes, nullptr);
  // timing only: no system-scope fence (its L2 writeback + invalidate cost
  // ~5 us per event and left the next kernel a cold L2)
  for (auto& e : p->ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  p->timing_cap = max_executes;
  p->timing_n = 0;
  return SPF_OK;
}

spf_status spf_whatif_timing(spf_whatif_plan* p, double* base_ms, double* fail_ms, uint32_t* n) {
  if (!p || !p->timing_cap) return SPF_E_STATE;
  spf_ctx* c = p->ctx;
  const uint32_t cnt = std::min(p->timing_n, p->timing_cap);
  double a = 0, b = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    float t0 = 0, t1 = 0;
    HIP_TRY(c, hipEventSynchronize(p->ev[3 * i + 2]));
    HIP_TRY(c, hipEventElapsedTime(&t0, p->ev[3 * i], p->ev[3 * i + 1]));
    HIP_TRY(c, hipEventElapsedTime(&t1, p->ev[3 * i + 1], p->ev[3 * i + 2]));
    a += t0;
    b += t1;
  }
  if (base_ms) *base_ms = a;
  if (fail_ms) *fail_ms = b;
  if (n) *n = cnt;
  p->timing_n = 0;
  return SPF_OK;
}

spf_status spf_whatif_solve(spf_ctx* c, uint32_t src, const uint32_t* fail_links,
                            uint32_t n_fail, spf_whatif_digest* out, spf_whatif_digest* base) {
  if (!c || !out) return fail(c, SPF_E_INVALID, "spf_whatif_solve: NULL argument");
  spf_whatif_plan* raw = nullptr;
  spf_status st = spf_whatif_plan_create(c, src, fail_links, n_fail, &raw);
  if (st != SPF_OK) return st;
  std::unique_ptr<spf_whatif_plan> p(raw);
  DevBuf<spf_whatif_digest> d_out, d_base;
  HIP_TRY(c, d_out.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, d_base.alloc(1));
  st = spf_whatif_execute(p.get(), d_out.p, d_base.p, c->stream);
  if (st != SPF_OK) return st;
  HIP_TRY(c, hipMemcpyAsync(out, d_out.p, sizeof(spf_whatif_digest) * p->n_fail,
                            hipMemcpyDeviceToHost, c->stream));
  if (base)
    HIP_TRY(c, hipMemcpyAsync(base, d_base.p, sizeof(spf_whatif_digest), hipMemcpyDeviceToHost,
                              c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return spf_device_check(c);
}

spf_status spf_device_check(spf_ctx* c) {
  if (!c) return fail(c, SPF_E_INVALID, "spf_device_check: NULL context");
  HIP_TRY(c, hipSetDevice(c->device));
  // every launch of this context may be on a caller's stream: wait for the
  // device, then read and clear THIS context's fault word only (another
  // context's timeout stays for its own check)
  HIP_TRY(c, hipDeviceSynchronize());
  if (!c->d_fault.p) return SPF_OK;
  uint32_t flag = 0;
  HIP_TRY(c, hipMemcpy(&flag, c->d_fault.p, sizeof flag, hipMemcpyDeviceToHost));
  if (!flag) return SPF_OK;
  HIP_TRY(c, hipMemset(c->d_fault.p, 0, sizeof flag));
  if (flag & 56u) {
    // what-if repair diagnostics: a loop bound (bit 3, phase in bits 8-15), a
    // range check of the profiled instances (bit 4, site in bits 16-23) or a
    // team past its profile region (bit 5, kernel in bits 24-31)
    return fail(c, SPF_E_HIP,
                "what-if repair on device %d: %s%s%s (fault word 0x%08x: loop phase %u, check site %u, "
                "profile kernel %u); the results of this context's launches since the last check are "
                "invalid",
                c->device, (flag & 8u) ? "a repair loop reached its iteration bound " : "",
                (flag & 16u) ? "a scratch index failed its range check " : "",
                (flag & 32u) ? "a team's profile row is outside the profile buffer" : "", flag,
                (flag >> 8) & 0xFFu, (flag >> 16) & 0xFFu, flag >> 24);
  }
  if (flag & 2u) {
    // a team BFS gave up waiting for its members (another process's grid
    // held CUs): this context's plans stop using teams -- each re-derives
    // onto msbfs_kernel at its next execute -- instead of polling again
    c->team_off = true;
    return fail(c, SPF_E_HIP,
                "a team BFS barrier timed out on device %d (workgroups not co-resident): the "
                "results of this context's launches since the last check are invalid; its plans "
                "run msbfs_kernel from their next execute", c->device);
  }
  return fail(c, SPF_E_HIP,
              "a grid barrier timed out on device %d (blocks not co-resident?): the "
              "results of this context's launches since the last check are invalid", c->device);
}

}  // extern "C"
