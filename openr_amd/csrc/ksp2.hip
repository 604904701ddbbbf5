// ============================================================================
//  ksp2.hip -- batched KSP2 (k = 1 and k = 2 edge-disjoint shortest paths)
//  for every (source, destination) pair of a source batch.
//
//  Reference: LinkState::getKthPaths (openr/decision/LinkState.cpp:762-791)
//  with traceOnePath (:398-419) over the pathLinks of runSpf (:808-882):
//    k = 1: trace paths in getSpfResult(src) until the shared visited-link set
//           makes the trace fail;
//    k = 2: linksToIgnore = every link of the k = 1 paths, a fresh
//           runSpf(src, true, linksToIgnore), trace again.
//
//  GPU mapping (one wavefront per pair, 4 pairs in flight per workgroup):
//    * the k = 1 distance row of the workgroup's source (computed by the
//      per-source SSSP kernel beforehand) is staged once in LDS;
//    * traceOnePath is a DFS with an explicit stack; a DFS step evaluates the
//      in-edges of the current node across the lanes and picks the first
//      untried tight one in pathLinks order with a wave min-reduction of the
//      key (dist[tail], edge id) -- the reference iterates pathLinks in
//      Dijkstra pop order (dist, name = id) and then linksFromNode order
//      (= edge id order inside a tail's CSR row).  A link tried once stays in
//      the visited bitmap, exactly like LinkState.cpp:410-416, so "first
//      untried candidate" reproduces the recursion's iteration order;
//    * the k = 2 SPF is a wave-local label-correcting frontier sweep in LDS
//      over the links not ignored, pruned at the destination's tentative
//      distance: a node whose distance is >= d'(dst) can never be a tail of a
//      tight edge on a path to dst (metrics are positive), and tentative
//      values are upper bounds, so every node the trace inspects is exact.
//    * paths go to a pool through a per-wave bump allocator (records
//      [n_links, next, links src->dst]), pairs get a fixed header.
// ============================================================================
#include "engine_internal.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <type_traits>

using namespace spfi;

namespace {

constexpr int kKspThreads = 256;             // 4 waves, one pair each
constexpr int kKspWaves = kKspThreads / 64;
constexpr int kKspLdsMaxThreads = 1024;      // staged-graph kernel: up to 16 waves
constexpr uint32_t kKspChunk = 64;          // sources per workgroup (default; SPF_KSP2_CHUNK)
constexpr uint32_t kPoolGrab = 256;         // words a wave reserves at a time (~ its pairs' paths)
constexpr size_t kMaxLdsKsp = 160 * 1024;
constexpr uint32_t kCompactCap = 512;       // u16-label waves: DFS stack / SPF queue entries
constexpr uint32_t kRedoBlocks = 256;       // workgroups of the u32 redo pass
constexpr uint32_t kProfSlots = 1024;  // SPF_KSP2_PROF: 16-counter slots (by block)
#ifndef KSP2_EDGES
#define KSP2_EDGES 2
#endif
constexpr uint32_t kKspEdges = KSP2_EDGES;  // edges per lane per relaxation step

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Wave-wide minimum of 64-bit keys with DPP moves (row shifts, then row
// broadcasts; a lane with no source keeps ~0) and a lane read: no
// ds_bpermute round trips.  Every lane of the wave must be active.
template <int CTRL, int ROWS, bool BOUND>
__device__ __forceinline__ uint64_t dpp_min64_step(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(~0u, (uint32_t)x, CTRL, ROWS, 0xf, BOUND);
  const uint32_t hi = __builtin_amdgcn_update_dpp(~0u, (uint32_t)(x >> 32), CTRL, ROWS, 0xf, BOUND);
  const uint64_t y = ((uint64_t)hi << 32) | lo;
  return y < x ? y : x;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
  x = dpp_min64_step<0x111, 0xf, false>(x);  // row_shr:1
  x = dpp_min64_step<0x112, 0xf, false>(x);  // row_shr:2
  x = dpp_min64_step<0x114, 0xf, false>(x);  // row_shr:4
  x = dpp_min64_step<0x118, 0xf, false>(x);  // row_shr:8
  x = dpp_min64_step<0x142, 0xa, false>(x);  // row_bcast:15
  x = dpp_min64_step<0x143, 0xc, false>(x);  // row_bcast:31
  return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), 63) << 32) |
         __builtin_amdgcn_readlane((uint32_t)x, 63);
}

__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(~0u, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint64_t wave_min(uint64_t x) { return wave_min64(x); }
__device__ __forceinline__ uint32_t wave_min(uint32_t x) { return wave_min32(x); }

// Exclusive prefix sum over the wave with DPP moves (no LDS round trips):
// row_shr 1/2/4/8 inside each 16-lane row (lanes shifted in from outside the
// row read 0), then row_bcast15 / row_bcast31 carry row totals upwards.
__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t x, uint32_t* total) {
  uint32_t inc = x;
  inc += __builtin_amdgcn_update_dpp(0u, inc, 0x111, 0xf, 0xf, true);  // row_shr:1
  inc += __builtin_amdgcn_update_dpp(0u, inc, 0x112, 0xf, 0xf, true);  // row_shr:2
  inc += __builtin_amdgcn_update_dpp(0u, inc, 0x114, 0xf, 0xf, true);  // row_shr:4
  inc += __builtin_amdgcn_update_dpp(0u, inc, 0x118, 0xf, 0xf, true);  // row_shr:8
  inc += __builtin_amdgcn_update_dpp(0u, inc, 0x142, 0xa, 0xf, false);  // row_bcast:15
  inc += __builtin_amdgcn_update_dpp(0u, inc, 0x143, 0xc, 0xf, false);  // row_bcast:31
  *total = __builtin_amdgcn_readlane(inc, 63);
  return inc - x;
}

// Minimum of the keys held by lanes 0 .. n-1 (n <= 64, wave-uniform): a
// handful of lane reads into scalar registers for small n (*arg = the lane
// holding it), the shuffle reduction otherwise (*arg = 64: unknown).
__device__ __forceinline__ uint64_t lanes_min(uint64_t x, uint32_t n, uint32_t* arg) {
  n = __builtin_amdgcn_readfirstlane(n);
  *arg = 64;
  if (n > 8) return wave_min64(x);
  uint64_t m = ~0ull;
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t y = ((uint64_t)__builtin_amdgcn_readlane(hi, j) << 32) |
                       __builtin_amdgcn_readlane(lo, j);
    if (y < m) {
      m = y;
      *arg = j;
    }
  }
  return m;
}
// 32-bit keys (compact waves: label and edge id both below 2^16): one lane
// read per candidate
__device__ __forceinline__ uint32_t lanes_min(uint32_t x, uint32_t n, uint32_t* arg) {
  n = __builtin_amdgcn_readfirstlane(n);
  *arg = 64;
  if (n > 8) return wave_min32(x);
  uint32_t m = ~0u;
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t y = __builtin_amdgcn_readlane(x, j);
    if (y < m) {
      m = y;
      *arg = j;
    }
  }
  return m;
}

__device__ __forceinline__ bool bit(const uint32_t* bm, uint32_t i) {
  return (bm[i >> 5] >> (i & 31)) & 1u;
}

// The A* heuristic row: u32, or u16 in the staged-graph kernel (0xFFFF =
// dst unreachable; finite distances saturate at 0xFFFE -- still a lower bound)
__device__ __forceinline__ uint32_t hget(const uint32_t* H, uint32_t v) { return H[v]; }
__device__ __forceinline__ uint32_t hget(const uint16_t* H, uint32_t v) {
  const uint32_t x = H[v];
  return x == 0xFFFFu ? kInf : x;
}

// A wave's distance row: u32 labels, or u16 labels on compact plans (0xFFFF
// = unreached or >= 65535; a pair whose labels leave that range is redone
// with u32 labels, see ksp2_pair).
__device__ __forceinline__ uint32_t dget(const uint32_t* D, uint32_t v) { return D[v]; }
__device__ __forceinline__ uint32_t dget(const uint16_t* D, uint32_t v) {
  const uint32_t x = D[v];
  return x == 0xFFFFu ? kInf : x;
}
__device__ __forceinline__ void dput(uint32_t* D, uint32_t v, uint32_t x) { D[v] = x; }
__device__ __forceinline__ void dput(uint16_t* D, uint32_t v, uint32_t x) { D[v] = (uint16_t)x; }
// D[v] = min(D[v], nd); true when the label went down
__device__ __forceinline__ bool dmin(uint32_t* D, uint32_t v, uint32_t nd) {
  return nd < atomicMin(&D[v], nd);
}
__device__ __forceinline__ bool dmin(uint16_t* D, uint32_t v, uint32_t nd) {
  // LDS has no 16-bit min: compare-and-swap on the word holding the label
  uint32_t* w = reinterpret_cast<uint32_t*>(D) + (v >> 1);
  const uint32_t sh = (v & 1u) * 16u;
  uint32_t old = *w;
  for (;;) {
    if (nd >= ((old >> sh) & 0xFFFFu)) return false;
    const uint32_t seen = atomicCAS(w, old, (old & ~(0xFFFFu << sh)) | (nd << sh));
    if (seen == old) return true;
    old = seen;
  }
}
template <class DT>
__device__ __forceinline__ void fill_unreached(DT* D, uint32_t pitch) {
  uint4* o = reinterpret_cast<uint4*>(D);
  for (uint32_t t = __lane_id(); t < pitch * (uint32_t)sizeof(DT) / 16; t += 64)
    o[t] = make_uint4(~0u, ~0u, ~0u, ~0u);
}
// the source's k = 1 row into the wave's labels (u16: saturated at 0xFFFF)
__device__ __forceinline__ void load_row(uint32_t* D, const uint32_t* Drow, uint32_t pitch) {
  const uint4* in = reinterpret_cast<const uint4*>(Drow);
  uint4* o = reinterpret_cast<uint4*>(D);
  for (uint32_t t = __lane_id(); t < pitch / 4; t += 64) o[t] = in[t];
}
__device__ __forceinline__ void load_row(uint16_t* D, const uint32_t* Drow, uint32_t pitch) {
  const uint4* in = reinterpret_cast<const uint4*>(Drow);
  uint2* o = reinterpret_cast<uint2*>(D);
  for (uint32_t t = __lane_id(); t < pitch / 4; t += 64) {
    const uint4 x = in[t];
    o[t] = make_uint2(min(x.x, 0xFFFFu) | (min(x.y, 0xFFFFu) << 16),
                      min(x.z, 0xFFFFu) | (min(x.w, 0xFFFFu) << 16));
  }
}

// Graph accessors: the CSR in HBM (any size), or a 16-bit copy staged in
// LDS by each workgroup (small graphs: every DFS step and relaxation then
// costs LDS latency instead of L2 latency).
struct NodeInfo {
  uint32_t beg, end;  // out-edges [beg, end)
  bool ovl;           // drained (overloaded)
};

struct GGraph {
  const uint32_t* row_ptr;
  const uint32_t* col_;
  const uint32_t* wt;
  const uint32_t* rev_;
  const uint32_t* link_;
  const uint8_t* ovl_;
  uint32_t N;
  __device__ NodeInfo node(uint32_t v) const { return {row_ptr[v], row_ptr[v + 1], ovl_[v] != 0}; }
  __device__ uint32_t col(uint32_t e) const { return col_[e]; }
  __device__ uint32_t w(uint32_t e) const { return wt[e]; }
  __device__ uint32_t rev(uint32_t e) const { return rev_[e]; }
  __device__ uint32_t link(uint32_t e) const { return link_[e]; }  // bitmap index
  __device__ uint32_t link_of(uint32_t e, uint32_t) const { return link_[e]; }  // r = rev(e)
  __device__ uint32_t out_link(uint32_t e) const { return link_[e]; }  // pool record
  __device__ bool ovl(uint32_t v) const { return ovl_[v] != 0; }
  // the ignored-link bitmap: by link id
  __device__ uint32_t ign_at(uint32_t e) const { return link_[e]; }
  __device__ void mark_ign(uint32_t* bm, uint32_t e) const {
    const uint32_t l = link_[e];
    atomicOr(&bm[l >> 5], 1u << (l & 31));
  }
};

// The staged graph indexes its visited-link bitmap by the edge pair
// {e, rev(e)} (min of the two ids) instead of the link id: an up link is
// exactly one such pair (checked when the plan is made), and the 16-bit link
// array then stays out of LDS -- room for one more wave per workgroup.  The
// ignored-link bitmap is indexed by edge id, both directions of a link
// marked, so a relaxation tests it without loading rev(e).  Head and metric
// share one 32-bit word per edge, first edge, degree and the drained flag one
// per node (one LDS read each).
struct LGraph {
  const uint32_t* nd_;      // [N] first edge | degree << 16 | drained << 31 (E < 65536, deg < 32768)
  const uint32_t* cw_;      // head | metric << 16 (metrics < 65536)
  const uint16_t* rev_;
  const uint32_t* glink;    // link ids (HBM): pool records only
  uint32_t N;
  __device__ NodeInfo node(uint32_t v) const {
    const uint32_t x = nd_[v];
    return {x & 0xFFFFu, (x & 0xFFFFu) + ((x >> 16) & 0x7FFFu), (x >> 31) != 0};
  }
  __device__ uint32_t col(uint32_t e) const { return cw_[e] & 0xFFFFu; }
  __device__ uint32_t w(uint32_t e) const { return cw_[e] >> 16; }
  __device__ uint32_t rev(uint32_t e) const { return rev_[e]; }
  __device__ uint32_t link(uint32_t e) const { return min(e, (uint32_t)rev_[e]); }
  __device__ uint32_t link_of(uint32_t e, uint32_t r) const { return min(e, r); }  // r = rev(e)
  __device__ bool ovl(uint32_t v) const { return (nd_[v] >> 31) != 0; }
  __device__ uint32_t ign_at(uint32_t e) const { return e; }
  __device__ uint32_t out_link(uint32_t e) const { return glink[e]; }
  __device__ void mark_ign(uint32_t* bm, uint32_t e) const {
    const uint32_t r = rev_[e];
    atomicOr(&bm[e >> 5], 1u << (e & 31));
    atomicOr(&bm[r >> 5], 1u << (r & 31));
  }
};

// Per-wave bump allocation in the path pool.  Returns the word offset, or
// kInf when the pool is exhausted (the counter keeps counting, so the host
// learns the size it needs).
struct PoolCursor {
  uint64_t cur = 0, end = 0;
  uint32_t grab = kPoolGrab;   // words per reservation (SPF_KSP2_GRAB)
  bool prof = false;
  unsigned long long clk = 0;  // SPF_KSP2_PROF: clocks spent reserving
};

__device__ uint32_t pool_alloc(PoolCursor& pc, uint32_t words, unsigned long long* used,
                               uint64_t cap, uint32_t* overflow) {
  if (pc.cur + words > pc.end) {
    const uint32_t grab = words > pc.grab ? words : pc.grab;
    const unsigned long long t0 = pc.prof ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t base = 0;
    if (__lane_id() == 0) base = atomicAdd(used, (unsigned long long)grab);
    base = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(base >> 32), 0) << 32) |
           __builtin_amdgcn_readlane((uint32_t)base, 0);
    if (pc.prof) pc.clk += __builtin_amdgcn_s_memtime() - t0;
    pc.cur = base;
    pc.end = base + grab;
  }
  const uint64_t at = pc.cur;
  pc.cur += words;
  if (at + words > cap || at + words > 0xFFFFFFF0ull) {
    if (__lane_id() == 0) atomicOr(overflow, 1u);
    return kInf;
  }
  return (uint32_t)at;
}

// traceOnePath (LinkState.cpp:398-419) from dst back to src over the tight
// in-edges of D (tails expanded, links not in `ign` when given, links not in
// `vis`).  On success the stack holds the edges dst-first and *depth their
// count; every link tried is left in `vis`.
// A path deeper than `cap` links sets *ovf (u16-label waves: the pair is
// redone with a full-size stack).
template <class G, class DT, class ST>
__device__ bool trace_one(const G& g, const DT* D, const uint32_t* ign, uint32_t* vis,
                          ST* stack, uint32_t cap, uint32_t src, uint32_t dst, uint32_t* depth,
                          bool* ovf, uint32_t* steps) {
  const uint32_t lane = __lane_id();
  // candidate key (D[tail], edge id): 32 bits in compact waves (both < 2^16)
  using K = typename std::conditional<sizeof(DT) == 2, uint32_t, uint64_t>::type;
  constexpr uint32_t KS = sizeof(K) * 4;  // edge-id bits of a key
  constexpr K KNONE = ~K(0);
  uint32_t k = 0, v = dst, dv = dget(D, dst);
  NodeInfo nv = g.node(dst);
  for (;;) {
    ++*steps;
    if (v == src) {
      *depth = k;
      return true;
    }
    K best = KNONE;
    uint32_t tail = 0, tl = 0;  // this lane's best candidate: tail node, link index
    uint32_t tb = 0, te = 0;    // ... and its in-edge range (the next step's, if it wins)
    const uint32_t e_beg = nv.beg, e_end = nv.end;
    for (uint32_t e = e_beg + lane; e < e_end; e += 64) {
      // in-edge u -> v is the reverse of the out-edge v -> u; every test's
      // load is issued up front (two dependent LDS rounds per step)
      const uint32_t u = g.col(e);
      const uint32_t r = g.rev(e);
      const uint32_t l = g.link_of(e, r);
      const NodeInfo nu = g.node(u);
      const bool drained = nu.ovl && u != src;
      const bool tried = bit(vis, l) || (ign && bit(ign, g.ign_at(e)));
      const uint32_t du = dget(D, u);
      const uint32_t wr = g.w(r);
      if (!drained && !tried && du != kInf && du + wr == dv) {
        const K key = ((K)du << KS) | r;
        if (key < best) {
          best = key;
          tail = u;
          tl = l;
          tb = nu.beg;
          te = nu.end;
        }
      }
    }
    uint32_t arg;
    best = lanes_min(best, min(e_end - e_beg, 64u), &arg);
    if (best == KNONE) {  // every pathLink of v tried: back up one level
      if (k == 0) return false;
      --k;
      v = k == 0 ? dst : g.col(g.rev(stack[k - 1]));
      dv = dget(D, v);
      nv = g.node(v);
      continue;
    }
    const uint32_t r = (uint32_t)(best & ((K(1) << KS) - 1));
    uint32_t l, u;
    if (arg < 64) {  // the winning lane's tail, link and the tail's in-edges
      u = __builtin_amdgcn_readlane(tail, arg);
      l = __builtin_amdgcn_readlane(tl, arg);
      nv.beg = __builtin_amdgcn_readlane(tb, arg);
      nv.end = __builtin_amdgcn_readlane(te, arg);
    } else {
      u = g.col(g.rev(r));
      l = g.link(r);
      nv = g.node(u);
    }
    if (k >= cap) {
      *ovf = true;
      return false;
    }
    if (lane == 0) {
      atomicOr(&vis[l >> 5], 1u << (l & 31));  // ds_or: no read round trip
      stack[k] = (ST)r;
    }
    wave_sync();
    ++k;
    v = u;  // tail of r, D[u] = the key's high part
    dv = (uint32_t)(best >> KS);
  }
}

// Writes the traced path as a pool record [n_links, next, links src->dst],
// chains it after the record at `prev_at` (kInf: first of its list) and
// returns its offset (kInf if the pool overflowed).  Marks the path's links
// in `mark` when given.
template <class G, class ST>
__device__ uint32_t emit_path(const G& g, const ST* stack, uint32_t depth, uint32_t* pool,
                              PoolCursor& pc, unsigned long long* used, uint64_t cap,
                              uint32_t* overflow, uint32_t prev_at, uint32_t* mark) {
  const uint32_t lane = __lane_id();
  const uint32_t at = pool_alloc(pc, depth + 2, used, cap, overflow);
  for (uint32_t j = lane; j < depth; j += 64) {
    const uint32_t e = stack[depth - 1 - j];  // src -> dst order
    if (mark) g.mark_ign(mark, e);
    if (at != kInf) pool[(size_t)at + 2 + j] = g.out_link(e);
  }
  if (at != kInf && lane == 0) {
    pool[at] = depth;
    pool[(size_t)at + 1] = kInf;
    if (prev_at != kInf) pool[(size_t)prev_at + 1] = at;
  }
  wave_sync();
  return at;
}

// Wave-local SPF from src over links not in `ign`, A*-pruned towards dst:
// H[v] = distance from v to dst in the graph with nothing ignored (a
// consistent lower bound of the distance left once links are ignored), so a
// node with D + H > D[dst] lies on no shortest path to dst and is not
// expanded.  Every node with exact D + H <= the final D[dst] -- all the
// nodes a trace to dst can inspect as tight tails -- ends exact (induction
// along its shortest path, whose nodes all satisfy the same bound).
// Expansion is ordered by f = D + H in buckets of width `delta`: a pending
// node with f > T stays pending (its bitmap bit is set again), and when a
// sweep expands nothing T moves to the smallest pending f + the width, which
// doubles on each move.  Without
// the order the sweep is a hop-synchronous Bellman-Ford that reaches dst only
// after expanding every node within dst's hop count (bound D[dst] = inf
// until then); with it, only nodes with f < d2(dst) + delta are expanded.
// The fixpoint -- and so every distance the trace reads -- is the same.
template <class G, class DT, class HT>
__device__ bool wave_sssp(const G& g, DT* D, uint16_t* q, uint32_t qcap, uint32_t* bm,
                          uint32_t bm_words, const uint32_t* ign, uint32_t src, uint32_t dst,
                          uint32_t pitch, const HT* H, uint32_t delta,
                          unsigned long long* prof) {
  // Returns whether a relaxation was dropped because its label did not fit
  // u16 (then an unreached dst proves nothing: the caller redoes the pair).
  // The queue holds at most `qcap` nodes: pending nodes are taken in bitmap
  // order from a cursor that wraps, so a long frontier is worked in chunks
  // (label-correcting: the order changes nothing of the fixpoint); the
  // bucket moves only after a whole round of chunks expanded nothing.
  const uint32_t lane = __lane_id();
  fill_unreached(D, pitch);
  for (uint32_t i = lane; i < bm_words; i += 64) bm[i] = 0;
  wave_sync();
  if (lane == 0) {
    dput(D, src, 0);
    q[0] = (uint16_t)src;
  }
  wave_sync();
  uint32_t qlen = 1;
  uint32_t span = bm_words, cur = 0;  // the chunk's bitmap words; next chunk's first word
  uint32_t idle = 0;                  // bitmap words worked since the last expansion
  // f = D + H in 32 bits in compact waves (labels and heuristic < 2^16; the
  // width stops doubling at 2^24, past every finite f), else in 64
  using F = typename std::conditional<sizeof(DT) == 2, uint32_t, uint64_t>::type;
  constexpr F FNONE = ~F(0);
  constexpr F WMAX = sizeof(DT) == 2 ? F(1u << 24) : F(0xFFFFFFFFull);
  F idle_f = FNONE;  // smallest f deferred since then
  F width = delta;
  F T = (F)hget(H, src) + width;  // expand pending nodes with f <= T
  bool sat = false;
  uint32_t sweeps = 0, raises = 0, pending = 0;  // SPF_KSP2_PROF counters
  while (qlen) {
    ++sweeps;
    pending += qlen;
    // a short frontier gets 2^lg lanes per node, each taking every 2^lg-th
    // edge: the dependent chain per lane is one or two edges, not deg(u)
    const uint32_t lg = qlen <= 16 ? 2u : (qlen <= 32 ? 1u : 0u);
    const uint32_t slot = lane & ((1u << lg) - 1u);
    F defer_f = FNONE;  // smallest f left pending by this lane
    bool expanded = false;
    for (uint32_t i = lane >> lg; i < qlen; i += 64u >> lg) {
      const uint32_t u = q[i];
      const NodeInfo nu = g.node(u);
      const bool drained = nu.ovl && u != src;  // recorded, not expanded
      const uint32_t du = dget(D, u);
      // dst's label now (read per node: a sweep-start copy expanded 6 % more)
      const uint32_t bound = dget(D, dst);
      const uint32_t hu = hget(H, u);
      if (drained || hu == kInf || u == dst) continue;  // (hu unreachable: f past every bound)
      const F f = (F)du + hu;
      if (f > bound) continue;
      if (f > T) {  // a later bucket: stays pending
        if (slot == 0) atomicOr(&bm[u >> 5], 1u << (u & 31));
        defer_f = min(defer_f, f);
        continue;
      }
      expanded = true;
      auto relax = [&](uint32_t v, uint32_t nd, bool ignored, uint32_t hv) {
        if (ignored || hv == kInf || (uint64_t)nd + hv > bound) return;
        if (sizeof(DT) == 2 && nd >= 0xFFFFu) {
          sat = true;
          return;
        }
        if (dmin(D, v, nd)) atomicOr(&bm[v >> 5], 1u << (v & 31));
      };
      // kKspEdges edges per lane and step, each one's loads under its own
      // mask: head, metric, ignored bit and heuristic of all of them in one
      // LDS round each (one edge per step: 117k -> 98k clocks per SPF at two;
      // four: wan_ksp2 76 -> 83 ms, the extra masks and registers)
      const uint32_t st = 1u << lg;
      for (uint32_t e = nu.beg + slot; e < nu.end; e += kKspEdges * st) {
        uint32_t v[kKspEdges], nd[kKspEdges], hv[kKspEdges];
        bool ig[kKspEdges];
#pragma unroll
        for (uint32_t k = 0; k < kKspEdges; ++k) {
          const uint32_t ek = e + k * st;
          v[k] = 0;
          nd[k] = 0;
          ig[k] = true;
          if (k == 0 || ek < nu.end) {
            v[k] = g.col(ek);
            nd[k] = du + g.w(ek);
            ig[k] = bit(ign, g.ign_at(ek));
          }
        }
#pragma unroll
        for (uint32_t k = 0; k < kKspEdges; ++k) hv[k] = (k == 0 || e + k * st < nu.end) ? hget(H, v[k]) : kInf;
#pragma unroll
        for (uint32_t k = 0; k < kKspEdges; ++k)
          if (k == 0 || e + k * st < nu.end) relax(v[k], nd[k], ig[k], hv[k]);
      }
    }
    if (!__ballot(expanded)) {  // everything pending seen lies past T: after a
      idle += span;             // whole round of such chunks the next bucket,
      idle_f = min(idle_f, wave_min(defer_f));  // twice as wide (a long
      if (idle >= bm_words) {                     // detour or an unreachable
        if (idle_f != FNONE) {                    // dst: log2 raises)
          ++raises;
          width = min((F)(2 * width), WMAX);
          T = idle_f + width;
        }
        idle = 0;
        idle_f = FNONE;
      }
    } else {
      idle = 0;
      idle_f = FNONE;
    }
    wave_sync();
    // next chunk: up to qcap pending nodes, bitmap words from `cur` on
    uint32_t n = 0;
    span = bm_words;
    for (uint32_t base = 0; base < bm_words; base += 64) {
      const uint32_t off = base + lane;
      uint32_t i = cur + off;
      if (i >= bm_words) i -= bm_words;
      uint32_t word = off < bm_words ? bm[i] : 0u;
      const uint32_t pc = __popc(word);
      uint32_t tot;
      uint32_t at = n + wave_excl_scan32(pc, &tot);
      const uint64_t cut = __ballot(at + pc > qcap);
      if (word && at < qcap) {
        for (uint32_t take = min(pc, qcap - at); take; --take) {
          const uint32_t b = __ffs(word) - 1;
          word &= word - 1;
          q[at++] = (uint16_t)(i * 32 + b);
        }
        bm[i] = word;  // bits not taken stay pending
      }
      if (cut) {  // the queue is full: the next chunk starts at the first word not taken whole
        const uint32_t first = base + (uint32_t)__ffsll((unsigned long long)cut) - 1;
        span = first;
        cur += first;
        if (cur >= bm_words) cur -= bm_words;
        n = qcap;
        break;
      }
      n += tot;
    }
    wave_sync();
    qlen = n;
  }
  if (prof && __lane_id() == 0) {
    prof += (blockIdx.x & (kProfSlots - 1)) * 16;  // spread: no same-address atomics
    atomicAdd(&prof[4], (unsigned long long)sweeps);
    atomicAdd(&prof[5], (unsigned long long)raises);
    atomicAdd(&prof[6], (unsigned long long)pending);
  }
  return __ballot(sat) != 0;
}

struct KspArgs {
  const uint32_t* Dsrc;   // [n_src][pitch] SPF rows of the sources
  const uint32_t* Hrows;  // [N][pitch] distances TO each node (transposed SPF)
  const uint32_t* srcs;
  uint32_t n_src, pitch, lw, chunks, chunk;
  uint32_t delta;  // bucket width of the k = 2 SPF's f = D + H order
  spf_ksp2_pair* pairs;
  uint32_t* pool;
  uint64_t cap;
  unsigned long long* counters;  // [3] = pairs queued for the u32 redo pass
  unsigned long long* prof;
  unsigned long long* redo;  // [redo_cap] (i << 32 | d) of u16-label pairs to redo
  uint64_t redo_cap;
  uint32_t lw_redo;  // link bitmap words of the redo pass (link ids)
  uint32_t grab;     // pool words a wave reserves at a time
};

// One wave's LDS: labels D [pitch] DT, DFS stack / SPF queue [cap] ST,
// pending bitmap, ign [lw] (the k = 1 links), vis [lw] (links tried).
template <class DT, class ST>
struct WaveLds {
  DT* D;
  ST* stack;
  uint16_t* q;
  uint32_t *bm, *ign, *vis;
  uint32_t cap, lw;
};

template <class DT, class ST>
__host__ __device__ constexpr size_t wave_lds_words(uint32_t pitch, uint32_t cap, uint32_t bm_words,
                                                    uint32_t lw) {
  // rounded to 4 words: each wave's D row starts 16-byte aligned (b128 access)
  return ((pitch * sizeof(DT) + 3) / 4 + (cap * sizeof(ST) + 3) / 4 + bm_words + 2ull * lw + 3) &
         ~3ull;
}

template <class DT, class ST>
__device__ WaveLds<DT, ST> wave_lds(uint32_t* base, uint32_t pitch, uint32_t cap,
                                    uint32_t bm_words, uint32_t lw) {
  WaveLds<DT, ST> m;
  const uint32_t w = threadIdx.x >> 6;
  uint32_t* p = base + (size_t)w * wave_lds_words<DT, ST>(pitch, cap, bm_words, lw);
  m.D = reinterpret_cast<DT*>(p);
  p += (pitch * sizeof(DT) + 3) / 4;
  m.stack = reinterpret_cast<ST*>(p);  // DFS stack ...
  m.q = reinterpret_cast<uint16_t*>(p);  // ... or SPF queue
  p += (cap * sizeof(ST) + 3) / 4;
  m.bm = p;
  m.ign = p + bm_words;
  m.vis = m.ign + lw;
  m.cap = cap;
  m.lw = lw;
  return m;
}

// One (source i, destination d) pair: k = 1 (trace on the source's SPF row
// copied into the wave's D), the k = 2 SPF (into the same D) and k = 2.
// Returns false -- nothing of the pair written, no k = 2 run counted --
// when a u16-label wave meets a label past 65534 that matters or a path
// deeper than its stack: the pair goes to the u32 redo pass.
template <class G, class DT, class ST, class HT>
__device__ bool ksp2_pair(const G& g, const KspArgs& a, const HT* H,
                          const WaveLds<DT, ST>& m, uint32_t i, uint32_t d, PoolCursor& pc,
                          uint32_t* k2_runs) {
  const uint32_t lane = __lane_id(), N = g.N, bm_words = (N + 31) / 32;
  unsigned long long* used = a.counters;
  uint32_t* overflow = reinterpret_cast<uint32_t*>(a.counters + 2);
  const uint32_t s = a.srcs[i];
  const uint32_t* Drow = a.Dsrc + (size_t)i * a.pitch;
  spf_ksp2_pair hdr;
  hdr.first[0] = hdr.first[1] = kInf;
  hdr.n_paths[0] = hdr.n_paths[1] = 0;
  const uint32_t d1 = Drow[d];
  if (d != s && d1 != kInf) {
    if (sizeof(DT) == 2 && d1 >= 0xFFFFu) return false;
    // ---- k = 1: trace in getSpfResult(src) (its row copied to LDS) ----
    load_row(m.D, Drow, a.pitch);
    for (uint32_t j = lane; j < m.lw; j += 64) {
      m.vis[j] = 0;
      m.ign[j] = 0;
    }
    wave_sync();
    uint32_t prev = kInf;
    uint32_t depth = 0;
    uint32_t n1 = 0;
    bool ovf = false;
    uint32_t st1 = 0, st2 = 0;  // SPF_KSP2_PROF: trace steps, emit clocks
    unsigned long long te = 0;
    unsigned long long t0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    while (trace_one(g, m.D, nullptr, m.vis, m.stack, m.cap, s, d, &depth, &ovf, &st1) && depth) {
      const unsigned long long e0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
      prev = emit_path(g, m.stack, depth, a.pool, pc, used, a.cap, overflow, prev, m.ign);
      if (a.prof) te += __builtin_amdgcn_s_memtime() - e0;
      if (n1++ == 0) hdr.first[0] = prev;
    }
    if (ovf) return false;
    hdr.n_paths[0] = n1;
    unsigned long long t1 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long t2 = t1;
    // ---- k = 2: runSpf(src, true, links of the k = 1 paths), trace ----
    if (n1) {
      wave_sync();
      const bool sat = wave_sssp(g, m.D, m.q, m.cap, m.bm, bm_words, m.ign, s, d, a.pitch, H,
                                 a.delta, a.prof);
      if (a.prof) t2 = __builtin_amdgcn_s_memtime();
      const uint32_t d2 = dget(m.D, d);
      if (d2 == kInf && sat) return false;
      if (d2 != kInf) {
        for (uint32_t j = lane; j < m.lw; j += 64) m.vis[j] = 0;
        wave_sync();
        prev = kInf;
        uint32_t n2 = 0;
        while (trace_one(g, m.D, m.ign, m.vis, m.stack, m.cap, s, d, &depth, &ovf, &st2) && depth) {
          const unsigned long long e0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
          prev = emit_path(g, m.stack, depth, a.pool, pc, used, a.cap, overflow, prev, nullptr);
          if (a.prof) te += __builtin_amdgcn_s_memtime() - e0;
          if (n2++ == 0) hdr.first[1] = prev;
        }
        if (ovf) return false;
        hdr.n_paths[1] = n2;
      }
      ++*k2_runs;
    }
    if (a.prof && lane == 0) {
      const unsigned long long t3 = __builtin_amdgcn_s_memtime();
      unsigned long long* P = a.prof + (blockIdx.x & (kProfSlots - 1)) * 16;
      atomicAdd(&P[0], t1 - t0);
      atomicAdd(&P[1], t2 - t1);
      atomicAdd(&P[2], t3 - t2);
      atomicAdd(&P[3], 1ull);
      atomicAdd(&P[7], (unsigned long long)st1);
      atomicAdd(&P[8], (unsigned long long)st2);
      atomicAdd(&P[9], te);
    }
  }
  if (lane == 0) a.pairs[(size_t)i * N + d] = hdr;
  return true;
}

// The pair loop of one workgroup: the block owns one destination d (its
// distances-to-d row H, the A* heuristic, staged in LDS) and a chunk of the
// sources; waves pull sources from a shared counter.
template <class G, class DT, class ST, class HT>
__device__ void ksp2_block(const G& g, const KspArgs& a, const HT* H, uint32_t* ctl,
                           const WaveLds<DT, ST>& m) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t d = blockIdx.x / a.chunks;
  const uint32_t c = blockIdx.x % a.chunks;
  const uint32_t i_end = min(a.n_src, (c + 1) * a.chunk);
  PoolCursor pc;
  pc.grab = a.grab;
  pc.prof = a.prof != nullptr;
  uint32_t k2_runs = 0;
  for (;;) {
    uint32_t i = 0;
    if (lane == 0) i = atomicAdd(&ctl[0], 1u);
    i = __builtin_amdgcn_readlane(i, 0);
    if (i >= i_end) break;
    if (!ksp2_pair(g, a, H, m, i, d, pc, &k2_runs) && lane == 0) {
      const unsigned long long at = atomicAdd(&a.counters[3], 1ull);
      if (at < a.redo_cap) a.redo[at] = ((unsigned long long)i << 32) | d;
      else atomicOr(reinterpret_cast<uint32_t*>(a.counters + 2), 2u);
    }
  }
  if (lane == 0 && k2_runs) atomicAdd(&a.counters[1], (unsigned long long)k2_runs);
  if (a.prof && lane == 0) atomicAdd(&a.prof[(blockIdx.x & (kProfSlots - 1)) * 16 + 10], pc.clk);
}

__device__ void stage_heuristic_row(const KspArgs& a, uint32_t* H, uint32_t* ctl) {
  const uint32_t d = blockIdx.x / a.chunks, c = blockIdx.x % a.chunks;
  const uint4* in = reinterpret_cast<const uint4*>(a.Hrows + (size_t)d * a.pitch);
  uint4* o = reinterpret_cast<uint4*>(H);
  for (uint32_t t = threadIdx.x; t < a.pitch / 4; t += blockDim.x) o[t] = in[t];
  if (threadIdx.x == 0) ctl[0] = c * a.chunk;
}
__device__ __forceinline__ uint32_t h16(uint32_t x) { return x == kInf ? 0xFFFFu : min(x, 0xFFFEu); }
__device__ void stage_heuristic_row(const KspArgs& a, uint16_t* H, uint32_t* ctl) {
  const uint32_t d = blockIdx.x / a.chunks, c = blockIdx.x % a.chunks;
  const uint4* in = reinterpret_cast<const uint4*>(a.Hrows + (size_t)d * a.pitch);
  uint2* o = reinterpret_cast<uint2*>(H);
  for (uint32_t t = threadIdx.x; t < a.pitch / 4; t += blockDim.x) {
    const uint4 x = in[t];
    o[t] = make_uint2(h16(x.x) | (h16(x.y) << 16), h16(x.z) | (h16(x.w) << 16));
  }
  if (threadIdx.x == 0) ctl[0] = c * a.chunk;
}

// Graph in HBM: 4 waves per workgroup, 32-bit DFS stack.
__global__ __launch_bounds__(kKspThreads) void ksp2_kernel(GGraph g, KspArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* H = reinterpret_cast<uint32_t*>(smem);  // [pitch] distances to d
  uint32_t* ctl = H + a.pitch;                      // [4] next source
  stage_heuristic_row(a, H, ctl);
  __syncthreads();
  const auto m = wave_lds<uint32_t, uint32_t>(ctl + 4, a.pitch, a.pitch, (g.N + 31) / 32, a.lw);
  ksp2_block(g, a, H, ctl, m);
}

// Graph staged in LDS as 16-bit arrays; waves per workgroup = blockDim / 64.
// DT = uint16_t: compact labels and a kCompactCap stack / queue per wave.
template <class DT>
__global__ __launch_bounds__(kKspLdsMaxThreads) void ksp2_lds_kernel(GGraph gg, KspArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t N = gg.N;
  uint16_t* H = reinterpret_cast<uint16_t*>(smem);  // [pitch] distances to d (u16)
  uint32_t* ctl = reinterpret_cast<uint32_t*>(H + a.pitch);  // [4] next source
  const uint32_t E = gg.row_ptr[N];
  const uint32_t e_words = (E + 1) / 2;
  uint32_t* cw = ctl + 4;
  uint32_t* nd = cw + E;
  uint16_t* rev = reinterpret_cast<uint16_t*>(nd + N);
  const size_t graph_end = (size_t)(reinterpret_cast<unsigned char*>(rev + 2 * e_words) - smem);
  uint32_t* wave_base = reinterpret_cast<uint32_t*>(smem + ((graph_end + 15) & ~(size_t)15));
  for (uint32_t v = threadIdx.x; v < N; v += blockDim.x) {
    const uint32_t b = gg.row_ptr[v];
    nd[v] = b | ((gg.row_ptr[v + 1] - b) << 16) | ((gg.ovl_[v] ? 1u : 0u) << 31);
  }
  for (uint32_t e = threadIdx.x; e < E; e += blockDim.x) {
    cw[e] = gg.col_[e] | (gg.wt[e] << 16);
    rev[e] = (uint16_t)gg.rev_[e];
  }
  stage_heuristic_row(a, H, ctl);
  __syncthreads();
  const LGraph g{nd, cw, rev, gg.link_, N};
  const uint32_t cap = sizeof(DT) == 2 ? kCompactCap : a.pitch;
  const auto m = wave_lds<DT, uint16_t>(wave_base, a.pitch, cap, (N + 31) / 32, a.lw);
  ksp2_block(g, a, H, ctl, m);
}

// The u32 redo pass of a compact plan: the pairs its u16-label waves handed
// back (counters[3] of them), graph and heuristic rows read from HBM, full
// size stacks.  Exits at once when there are none.
__global__ __launch_bounds__(kKspThreads) void ksp2_redo_kernel(GGraph g, KspArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long n = min((unsigned long long)a.redo_cap, a.counters[3]);
  if (n == 0) return;
  const uint32_t waves = blockDim.x >> 6, w = threadIdx.x >> 6;
  const auto m = wave_lds<uint32_t, uint32_t>(reinterpret_cast<uint32_t*>(smem), a.pitch, a.pitch,
                                              (g.N + 31) / 32, a.lw_redo);
  PoolCursor pc;
  pc.grab = a.grab;
  uint32_t k2_runs = 0;
  for (unsigned long long j = (unsigned long long)blockIdx.x * waves + w; j < n;
       j += (unsigned long long)gridDim.x * waves) {
    const unsigned long long r = a.redo[j];
    const uint32_t i = (uint32_t)(r >> 32), d = (uint32_t)r;
    (void)ksp2_pair(g, a, a.Hrows + (size_t)d * a.pitch, m, i, d, pc, &k2_runs);
  }
  if ((threadIdx.x & 63) == 0 && k2_runs)
    atomicAdd(&a.counters[1], (unsigned long long)k2_runs);
}

size_t ksp2_lds_bytes(uint32_t N, uint32_t pitch, uint32_t lw) {
  const size_t bm_words = (N + 31) / 32;
  return 4ull * (pitch + 4 + kKspWaves * wave_lds_words<uint32_t, uint32_t>(pitch, pitch, bm_words, lw));
}

// LDS bytes of the staged-graph kernel with `waves` waves per workgroup
// (compact: u16 labels)
size_t ksp2_lds_graph_bytes(uint32_t N, uint32_t E, uint32_t pitch, uint32_t lw, uint32_t waves,
                            bool compact) {
  const size_t bm_words = (N + 31) / 32;
  const size_t graph = 4ull * (E + N + (E + 1) / 2);  // cw, nd, rev
  const size_t fixed = (2ull * pitch + 16 + graph + 15) & ~(size_t)15;  // H u16, ctl
  const size_t wave = compact ? wave_lds_words<uint16_t, uint16_t>(pitch, kCompactCap, bm_words, lw)
                              : wave_lds_words<uint32_t, uint16_t>(pitch, pitch, bm_words, lw);
  return fixed + 4ull * waves * wave;
}

size_t ksp2_redo_wave_bytes(uint32_t N, uint32_t pitch, uint32_t lw) {
  return 4ull * wave_lds_words<uint32_t, uint32_t>(pitch, pitch, (N + 31) / 32, lw);
}

}  // namespace

namespace {
__device__ __forceinline__ uint64_t dg_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t dg_fnv(uint64_t h, uint64_t x) { return (h ^ x) * 0x100000001b3ULL; }

// spf_ksp2_digest: one thread per (source, destination) walks the pair's two
// path lists; the per-source sum is commutative (atomic order-free)
__global__ __launch_bounds__(256) void ksp2_digest_kernel(const spf_ksp2_pair* __restrict__ pairs,
                                                          const uint32_t* __restrict__ pool,
                                                          const uint64_t* __restrict__ link_hash,
                                                          uint32_t n_src, uint32_t n,
                                                          unsigned long long* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = blockIdx.y;
  if (i >= n_src || t >= n) return;
  const uint32_t d = (uint32_t)t;
  const uint4 r = reinterpret_cast<const uint4*>(pairs)[(size_t)i * n + d];  // first[2], n_paths[2]
  uint64_t h = 0xcbf29ce484222325ULL;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t np = k ? r.w : r.z;
    h = dg_fnv(h, 0x1000u + np);
    uint32_t at = k ? r.y : r.x;
    for (uint32_t q = 0; q < np; ++q) {
      const uint32_t len = pool[at];
      h = dg_fnv(h, 0x2000u + len);
      for (uint32_t x = 0; x < len; ++x) h = dg_fnv(h, link_hash[pool[at + 2 + x]]);
      at = pool[at + 1];
    }
  }
  atomicAdd(&out[i], (unsigned long long)dg_mix64(h + dg_mix64((uint64_t)d + 1)));
}
}  // namespace

struct spf_ksp2_plan {
  spf_ctx* ctx = nullptr;
  uint32_t n_src = 0, lw = 0;
  uint32_t delta = 0;  // bucket width of the k = 2 SPF (KspArgs::delta)
  uint32_t chunk = kKspChunk;  // sources per workgroup
  uint32_t grab = kPoolGrab;   // pool words per wave reservation
  uint64_t epoch = 0;  // graph state the plan was derived from
  std::vector<uint32_t> srcs;
  DevBuf<uint32_t> d_srcs, d_D, d_H, d_all, d_wt_rev;
  DevBuf<uint8_t> d_no_drain;
  DevBuf<unsigned long long> d_prof;  // SPF_KSP2_PROF diagnostics
  size_t lds = 0;
  uint32_t lds_waves = 0;  // > 0: the staged-graph kernel with this many waves
  bool compact = false;     // ... with u16 labels, and the u32 redo pass behind it
  uint32_t lw_links = 0, redo_waves = 0;
  size_t redo_lds = 0;
  DevBuf<unsigned long long> d_redo;  // [n_src * N] pairs handed to the redo pass
  std::vector<hipEvent_t> ev;
  uint32_t timing_cap = 0, timing_n = 0;
  // outside the batched kernel's envelope (metrics <= 0, u64 labels, more
  // than 65535 nodes or a working set past the LDS): the exact kernel
  std::unique_ptr<spfi::ExactKsp2> exact;
  ~spf_ksp2_plan() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
};

extern "C" {

spf_status spf_ksp2_plan_create(spf_ctx* c, const uint32_t* srcs, uint32_t n_src,
                                spf_ksp2_plan** out) {
  if (!c || !out) return fail(c, SPF_E_INVALID, "spf_ksp2_plan_create: NULL argument");
  *out = nullptr;
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (n_src == 0 || !srcs) return fail(c, SPF_E_INVALID, "empty source list");
  auto p = std::make_unique<spf_ksp2_plan>();
  p->ctx = c;
  p->n_src = n_src;
  p->srcs.assign(srcs, srcs + n_src);
  for (uint32_t i = 0; i < n_src; ++i)
    if (srcs[i] >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", srcs[i]);
  auto go_exact = [&]() -> spf_status {
    HIP_TRY(c, hipSetDevice(c->device));
    p->exact = std::make_unique<spfi::ExactKsp2>();
    const spf_status st = exact_ksp2_prepare(c, p->exact.get(), p->srcs);
    if (st != SPF_OK) return st;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    p->epoch = c->epoch;
    *out = p.release();
    return SPF_OK;
  };
  if (c->nonpos || c->needs64 || c->N > 65535 || std::getenv("SPF_KSP2_EXACT")) return go_exact();
  p->lw = p->lw_links = c->max_link / 32 + 1;
  {  // bucket width: half the mean up-link metric (env SPF_KSP2_DELTA overrides;
     // 4294967295 = no order, the plain hop-synchronous sweep)
    uint64_t sum = 0;
    for (uint32_t e = 0; e < c->E; ++e) sum += c->wt[e];
    // half the mean (wan_ksp2: 74.0 ms at the mean, 73.0 at 200-300, 74.5 at 600)
    p->delta = c->E ? (uint32_t)std::max<uint64_t>(1, sum / c->E / 2) : 1;
    if (const char* env = std::getenv("SPF_KSP2_DELTA")) p->delta = (uint32_t)std::strtoul(env, nullptr, 10);
    if (const char* env = std::getenv("SPF_KSP2_CHUNK")) p->chunk = std::max(1ul, std::strtoul(env, nullptr, 10));
    if (const char* env = std::getenv("SPF_KSP2_GRAB")) p->grab = std::max(64ul, std::strtoul(env, nullptr, 10));
  }
  // graph staged in LDS when its 16-bit copy fits beside >= 2 waves and
  // every up link is one {e, rev(e)} pair (LGraph's bitmap index)
  bool pairs_are_links = c->E < 65536;
  {
    std::vector<uint8_t> seen(c->max_link + 1, 0);
    for (uint32_t e = 0; e < c->E && pairs_are_links; ++e) {
      const uint32_t r = c->rev[e];
      if (r >= c->E || c->rev[r] != e || c->link[r] != c->link[e]) pairs_are_links = false;
      else if (e <= r && seen[c->link[e]]++) pairs_are_links = false;  // one pair per link
    }
  }
  uint32_t max_deg = 0;  // the staged node word holds degrees < 32768
  for (uint32_t v = 0; v < c->N; ++v) max_deg = std::max(max_deg, c->row_ptr[v + 1] - c->row_ptr[v]);
  if (pairs_are_links && c->max_metric < 65536 && max_deg < 32768 && !std::getenv("SPF_KSP2_HBM")) {
    const uint32_t lw_pairs = c->E / 32 + 1;
    auto fit = [&](bool compact) -> uint32_t {
      for (uint32_t w = kKspLdsMaxThreads / 64; w >= 2; --w)
        if (ksp2_lds_graph_bytes(c->N, c->E, c->pitch, lw_pairs, w, compact) <= kMaxLdsKsp) return w;
      return 0;
    };
    const uint32_t w32 = fit(false);
    // u16 labels (SPF_KSP2_U16=0: never, =1: whenever they fit): more waves
    // per CU to hide LDS latency; pairs whose labels pass 65534 or whose
    // paths outgrow the short stack are redone with u32 labels
    const char* u16env = std::getenv("SPF_KSP2_U16");
    const uint32_t redo_wave = (uint32_t)ksp2_redo_wave_bytes(c->N, c->pitch, p->lw_links);
    const uint32_t redo_waves = std::min<uint32_t>(kKspWaves, (uint32_t)(kMaxLdsKsp / redo_wave));
    const uint32_t w16 = (u16env && u16env[0] == '0') || !redo_waves ? 0 : fit(true);
    const bool compact = w16 && (w16 > w32 || (u16env && u16env[0] == '1'));
    const uint32_t w = compact ? w16 : w32;
    if (w) {
      p->lds_waves = w;
      p->compact = compact;
      p->lw = lw_pairs;
      p->lds = ksp2_lds_graph_bytes(c->N, c->E, c->pitch, lw_pairs, w, compact);
      if (compact) {
        p->redo_waves = redo_waves;
        p->redo_lds = (size_t)redo_wave * redo_waves;
      }
    }
  }
  if (!p->lds_waves) p->lds = ksp2_lds_bytes(c->N, c->pitch, p->lw);
  // ~16 pairs per wave and workgroup: the per-workgroup staging and the
  // waves' uneven ends amortised (64 -> 256 sources at 16 waves: 89 -> 84 ms)
  if (!std::getenv("SPF_KSP2_CHUNK"))
    p->chunk = std::max<uint32_t>(kKspChunk, 16 * (p->lds_waves ? p->lds_waves : kKspWaves));
  if (p->lds > kMaxLdsKsp) return go_exact();  // the per-wave rows do not fit the LDS
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipFuncSetAttribute((const void*)ksp2_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsKsp));
  HIP_TRY(c, hipFuncSetAttribute((const void*)ksp2_lds_kernel<uint32_t>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsKsp));
  HIP_TRY(c, hipFuncSetAttribute((const void*)ksp2_lds_kernel<uint16_t>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsKsp));
  HIP_TRY(c, hipFuncSetAttribute((const void*)ksp2_redo_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsKsp));
  {
    const spf_status st = set_lds_limits(c);
    if (st != SPF_OK) return st;
  }
  HIP_TRY(c, p->d_srcs.upload(p->srcs.data(), n_src, c->stream));
  HIP_TRY(c, p->d_D.alloc((size_t)n_src * c->pitch));
  if (p->compact) HIP_TRY(c, p->d_redo.alloc((size_t)n_src * c->N));
  {  // distances TO every node: SPF over transposed metrics, no drains (a
     // lower bound of every drained / link-ignored distance)
    std::vector<uint32_t> all(c->N), wr(c->E);
    for (uint32_t v = 0; v < c->N; ++v) all[v] = v;
    for (uint32_t e = 0; e < c->E; ++e) wr[e] = c->wt[c->rev[e]];
    std::vector<uint8_t> z(c->N, 0);
    HIP_TRY(c, p->d_all.upload(all.data(), c->N, c->stream));
    HIP_TRY(c, p->d_wt_rev.upload(wr.data(), c->E, c->stream));
    HIP_TRY(c, p->d_no_drain.upload(z.data(), c->N, c->stream));
    HIP_TRY(c, p->d_H.alloc((size_t)c->N * c->pitch));
  }
  if (std::getenv("SPF_KSP2_PROF")) {
    HIP_TRY(c, p->d_prof.alloc(16 * kProfSlots));
    HIP_TRY(c, hipMemsetAsync(p->d_prof.p, 0, 128 * kProfSlots, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  p->epoch = c->epoch;
  *out = p.release();
  return SPF_OK;
}

void spf_ksp2_plan_destroy(spf_ksp2_plan* p) { delete p; }
uint32_t spf_ksp2_plan_chunk(const spf_ksp2_plan* p) { return p ? p->chunk : 0u; }

spf_status spf_ksp2_digest(spf_ksp2_plan* p, const spf_ksp2_pair* d_pairs, const uint32_t* d_pool,
                           const uint64_t* d_link_hash, uint64_t* d_out, void* stream) {
  if (!p || !d_pairs || !d_pool || !d_link_hash || !d_out)
    return fail(p ? p->ctx : nullptr, SPF_E_INVALID, "spf_ksp2_digest: NULL argument");
  spf_ctx* c = p->ctx;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  HIP_TRY(c, hipMemsetAsync(d_out, 0, 8ull * p->n_src, s));
  if (!p->n_src || !c->N) return SPF_OK;
  hipLaunchKernelGGL(ksp2_digest_kernel, dim3((c->N + 255) / 256, p->n_src), dim3(256), 0, s, d_pairs,
                     d_pool, d_link_hash, p->n_src, c->N, reinterpret_cast<unsigned long long*>(d_out));
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

spf_status spf_ksp2_execute(spf_ksp2_plan* p, spf_ksp2_pair* d_pairs, uint32_t* d_pool,
                            uint64_t pool_words, uint64_t* d_counters, void* stream) {
  if (!p) return fail(nullptr, SPF_E_INVALID, "spf_ksp2_execute: NULL plan");
  spf_ctx* c = p->ctx;
  if (!c->loaded) return fail(c, SPF_E_STATE, "graph no longer loaded");
  if (p->epoch != c->epoch)
    return fail(c, SPF_E_STATE, "graph changed since the plan was created: recreate it");
  if (!d_pairs || !d_counters || (pool_words && !d_pool))
    return fail(c, SPF_E_INVALID, "spf_ksp2_execute: NULL output buffer");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  hipEvent_t* ev = nullptr;
  if (p->timing_cap) {
    ev = &p->ev[3 * (p->timing_n % p->timing_cap)];
    ++p->timing_n;
    HIP_TRY(c, hipEventRecord(ev[0], s));
  }
  HIP_TRY(c, hipMemsetAsync(d_counters, 0, 4 * sizeof(uint64_t), s));
  if (p->exact) {
    const spf_status st = exact_ksp2_launch(c, p->exact.get(), d_pairs, d_pool, pool_words,
                                            d_counters, s, ev ? ev[1] : nullptr);
    if (st != SPF_OK) return st;
    if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
    c->solves += p->n_src;
    return SPF_OK;
  }
  spf_status st = launch_sssp(c, p->d_srcs.p, p->n_src, false, nullptr, p->d_D.p, s);
  if (st != SPF_OK) return st;
  st = launch_sssp(c, p->d_all.p, c->N, false, nullptr, p->d_H.p, s, p->d_wt_rev.p,
                   p->d_no_drain.p);
  if (st != SPF_OK) return st;
  if (ev) HIP_TRY(c, hipEventRecord(ev[1], s));
  GGraph g{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_rev.p, c->d_link.p, c->d_ovl.p, c->N};
  // blocks: (destination, chunk of p->chunk sources)
  const uint32_t chunks = (p->n_src + p->chunk - 1) / p->chunk;
  KspArgs a{p->d_D.p, p->d_H.p, p->d_srcs.p, p->n_src, c->pitch, p->lw, chunks, p->chunk, p->delta, d_pairs,
            d_pool, pool_words, reinterpret_cast<unsigned long long*>(d_counters), p->d_prof.p,
            p->d_redo.p, (uint64_t)p->d_redo.n, p->lw_links, p->grab};
  if (p->compact)
    hipLaunchKernelGGL(ksp2_lds_kernel<uint16_t>, dim3(c->N * chunks), dim3(64 * p->lds_waves),
                       p->lds, s, g, a);
  else if (p->lds_waves)
    hipLaunchKernelGGL(ksp2_lds_kernel<uint32_t>, dim3(c->N * chunks), dim3(64 * p->lds_waves),
                       p->lds, s, g, a);
  else
    hipLaunchKernelGGL(ksp2_kernel, dim3(c->N * chunks), dim3(kKspThreads), p->lds, s, g, a);
  HIP_TRY(c, hipGetLastError());
  if (p->compact) {  // pairs the u16 waves handed back (usually none: the kernel exits)
    hipLaunchKernelGGL(ksp2_redo_kernel, dim3(kRedoBlocks), dim3(64 * p->redo_waves), p->redo_lds,
                       s, g, a);
    HIP_TRY(c, hipGetLastError());
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
  c->solves += p->n_src;  // k = 2 runs are added by spf_ksp2_solve / the caller
  return SPF_OK;
}

static spf_status ksp2_debug_phases(spf_ksp2_plan* p) {
  if (!p || !p->d_prof.p) return SPF_OK;
  std::vector<unsigned long long> all(16 * kProfSlots);
  HIP_TRY(p->ctx, hipMemcpy(all.data(), p->d_prof.p, 8 * all.size(), hipMemcpyDeviceToHost));
  unsigned long long h[16] = {};
  for (size_t j = 0; j < all.size(); ++j) h[j % 16] += all[j];
  std::fprintf(stderr, "ksp2 phases (clock sums over waves): k1 trace %llu, k2 spf %llu, "
               "k2 trace %llu, pairs %llu; k2 spf sweeps %llu, bucket raises %llu, "
               "queued nodes %llu; trace steps k1 %llu k2 %llu; emit clocks %llu (reserving %llu)\n", h[0], h[1],
               h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9], h[10]);
  const double n = h[3] ? (double)h[3] : 1.0;
  std::fprintf(stderr, "ksp2 per pair: k1 trace %.0f clk (%.1f steps), k2 spf %.0f clk (%.1f sweeps, "
               "%.1f queued), k2 trace %.0f clk (%.1f steps), emit %.0f clk\n", h[0] / n, h[7] / n,
               h[1] / n, h[4] / n, h[6] / n, h[2] / n, h[8] / n, h[9] / n);
  return SPF_OK;
}

spf_status spf_ksp2_enable_timing(spf_ksp2_plan* p, uint32_t max_executes) {
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

spf_status spf_ksp2_timing(spf_ksp2_plan* p, double* spf_ms, double* ksp_ms, uint32_t* n) {
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
  if (spf_ms) *spf_ms = a;
  if (ksp_ms) *ksp_ms = b;
  (void)ksp2_debug_phases(p);
  if (n) *n = cnt;
  p->timing_n = 0;
  return SPF_OK;
}

spf_status spf_ksp2_solve(spf_ctx* c, const uint32_t* srcs, uint32_t n_src,
                          spf_ksp2_pair* pairs_out, uint32_t* pool_out, uint64_t pool_cap,
                          uint64_t* pool_used) {
  if (!c || !pairs_out || !pool_used) return fail(c, SPF_E_INVALID, "spf_ksp2_solve: NULL argument");
  spf_ksp2_plan* raw = nullptr;
  spf_status st = spf_ksp2_plan_create(c, srcs, n_src, &raw);
  if (st != SPF_OK) return st;
  std::unique_ptr<spf_ksp2_plan> p(raw);
  const size_t n_pairs = (size_t)n_src * c->N;
  DevBuf<spf_ksp2_pair> d_pairs;
  DevBuf<uint32_t> d_pool;
  DevBuf<uint64_t> d_cnt;
  HIP_TRY(c, d_pairs.alloc(n_pairs));
  HIP_TRY(c, d_cnt.alloc(4));
  uint64_t cap = std::max<uint64_t>(pool_cap, (uint64_t)n_pairs * 16 + kPoolGrab * 4096ull);
  uint64_t cnt[4] = {0, 0, 0, 0};
  for (int attempt = 0; attempt < 3; ++attempt) {
    HIP_TRY(c, d_pool.alloc(cap));
    st = spf_ksp2_execute(p.get(), d_pairs.p, d_pool.p, cap, d_cnt.p, c->stream);
    if (st != SPF_OK) return st;
    HIP_TRY(c, hipMemcpyAsync(cnt, d_cnt.p, sizeof cnt, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (!(cnt[2] & 1)) break;
    cap = cnt[0] + cnt[0] / 4;  // overflowed: the counter says how much it wanted
  }
  if (cnt[2] & 1) return fail(c, SPF_E_NOMEM, "KSP2 path pool overflow");
  c->solves += cnt[1];
  // The device pool holds the waves' reservations in completion order, with
  // slack at each one's end: repack the records per pair (pair order, k = 1
  // then k = 2, list order) so the layout -- and *pool_used -- is the same on
  // every call (the sizing call's answer fits the second call exactly).
  std::vector<spf_ksp2_pair> hp(n_pairs);
  // cnt[0] counts claimed reservations, a last grab's unused tail included:
  // it can pass the pool's size with no overflow, so copy what the pool holds
  const uint64_t held = std::min<uint64_t>(cnt[0], cap);
  std::vector<uint32_t> pool_h(held);
  HIP_TRY(c, hipMemcpy(hp.data(), d_pairs.p, n_pairs * sizeof(spf_ksp2_pair), hipMemcpyDeviceToHost));
  if (held) HIP_TRY(c, hipMemcpy(pool_h.data(), d_pool.p, held * 4, hipMemcpyDeviceToHost));
  uint64_t dense = 0;
  for (const spf_ksp2_pair& r : hp)
    for (int k = 0; k < 2; ++k)
      for (uint32_t q = 0, at = r.first[k]; q < r.n_paths[k]; ++q, at = pool_h[at + 1]) dense += pool_h[at] + 2ull;
  if (dense > 0xFFFFFFF0ull) return fail(c, SPF_E_NOMEM, "KSP2 paths exceed 32-bit pool offsets");
  *pool_used = dense;
  const bool write = pool_out && pool_cap >= dense;
  uint64_t cur = 0;
  for (spf_ksp2_pair& r : hp)
    for (int k = 0; k < 2; ++k) {
      uint32_t at = r.first[k];
      r.first[k] = r.n_paths[k] ? (uint32_t)cur : kInf;
      for (uint32_t q = 0; q < r.n_paths[k]; ++q) {
        const uint32_t len = pool_h[at];
        if (write) {
          pool_out[cur] = len;
          pool_out[cur + 1] = q + 1 < r.n_paths[k] ? (uint32_t)(cur + len + 2) : kInf;
          std::memcpy(pool_out + cur + 2, pool_h.data() + at + 2, 4ull * len);
        }
        cur += len + 2ull;
        at = pool_h[at + 1];
      }
    }
  std::memcpy(pairs_out, hp.data(), n_pairs * sizeof(spf_ksp2_pair));
  if (pool_out && !write)
    return fail(c, SPF_E_NOMEM, "pool_out holds %llu words, %llu needed",
                (unsigned long long)pool_cap, (unsigned long long)dense);
  return SPF_OK;
}

}  // extern "C"
