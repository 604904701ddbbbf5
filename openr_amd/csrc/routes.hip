// ============================================================================
//  routes.hip -- SpfSolver's next-hop selection for one node and a batch of
//  destination sets (one set per prefix / node label).
//
//  Reference: SpfSolver::SpfSolverImpl in openr/decision/Decision.cpp
//    getMinCostNodes        :1082-1105  closest reachable nodes of the set
//    getNextHopsWithMetric  :1107-1196  shortest-path next hops (+ LFA,
//                                       RFC 5286 condition at :1180)
//    getNextHopsThrift      :1198-1305  one next hop per up link of me towards
//                                       a selected neighbour, metric
//                                       w(link) + dist(neighbour, dst)
//  for a single area and perDestination = false (IP routes and node-label
//  MPLS routes).  The SPF inputs -- dist rows of me and, with LFA, of every
//  neighbour, and me's next-hop bitmaps -- come from one batched plan; the
//  selection runs one wavefront per destination set, lanes over me's links.
// ============================================================================
#include "engine_internal.h"

#include <cstdlib>
#include <memory>

using namespace spfi;

namespace {

constexpr uint64_t kInf64 = ~0ull;

// D rows: row_of[v] = row of v's distances (me and, with LFA, neighbours).
// nh: me's destination bitmaps, bitmap j = neighbour j (ascending id).
__global__ __launch_bounds__(64) void routes_kernel(
    const uint32_t* __restrict__ D, uint32_t pitch, const uint32_t* __restrict__ row_of,
    const uint32_t* __restrict__ nh, uint32_t me, const uint32_t* __restrict__ me_edges_col,
    const uint32_t* __restrict__ me_edges_w, const uint32_t* __restrict__ me_edges_j,
    uint32_t me_deg, const uint32_t* __restrict__ set_ptr, const uint32_t* __restrict__ set_nodes,
    uint32_t lfa, uint64_t* __restrict__ out_min, uint32_t* __restrict__ out_cnt,
    uint32_t* __restrict__ out_edge, uint64_t* __restrict__ out_metric) {
  const uint32_t p = blockIdx.x, lane = threadIdx.x;
  const uint32_t b = set_ptr[p], e = set_ptr[p + 1];
  const uint32_t* Dme = D + (size_t)row_of[me] * pitch;
  const uint32_t wpm = pitch / 32;
  // getMinCostNodes: shortest metric over the reachable members
  uint64_t shortest = kInf64;
  for (uint32_t i = b; i < e; ++i) {
    const uint32_t d = Dme[set_nodes[i]];
    if (d != kInf && d < shortest) shortest = d;
  }
  uint32_t cnt = 0;
  if (shortest != kInf64) {
    for (uint32_t base = 0; base < me_deg; base += 64) {
      const uint32_t k = base + lane;
      bool keep = false;
      uint64_t metric = 0;
      if (k < me_deg) {
        const uint32_t x = me_edges_col[k], j = me_edges_j[k];
        // shortest-path next hop: x in nextHops() of a min-cost member
        // (j == kInf: a dead slot, no link)
        uint64_t val = kInf64;
        for (uint32_t i = b; i < e && j != kInf; ++i) {
          const uint32_t d = set_nodes[i];
          if (Dme[d] != shortest) continue;
          if ((nh[(size_t)j * wpm + (d >> 5)] >> (d & 31)) & 1u) {
            val = shortest - Dme[x];
            break;
          }
        }
        if (lfa && j != kInf) {  // loop-free alternate: d(x, dst) < shortest + d(x, me)
          const uint32_t* Dx = D + (size_t)row_of[x] * pitch;
          const uint64_t back = Dx[me];
          for (uint32_t i = b; i < e; ++i) {
            const uint32_t dxd = Dx[set_nodes[i]];
            if (dxd == kInf || back == kInf) continue;
            if ((uint64_t)dxd < shortest + back && (val == kInf64 || val > dxd)) val = dxd;
          }
        }
        if (val != kInf64) {
          metric = (uint64_t)me_edges_w[k] + val;
          keep = lfa || metric == shortest;
        }
      }
      const uint64_t m = __ballot(keep);
      if (keep) {
        const uint32_t at = cnt + __popcll(m & ((1ull << lane) - 1));
        out_edge[(size_t)p * me_deg + at] = k;
        out_metric[(size_t)p * me_deg + at] = metric;
      }
      cnt += __popcll(m);
    }
  }
  if (lane == 0) {
    out_min[p] = shortest;
    out_cnt[p] = cnt;
  }
}

__device__ __forceinline__ uint64_t rmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Route selection for many `me` nodes over RESIDENT rows (an all-sources
// pass, spf_mplan): a thread per destination set, a run of blocks per me (every
// me value wave-uniform: its CSR row, its distinct neighbours, their rows
// arrive by scalar loads).  Sets of single advertisers sorted by node id make
// consecutive lanes read consecutive entries of me's row and bitmaps.
//   rowp[v] / nhp[v]: device addresses of v's u32 distance row and of its
//   first next-hop bitmap (bitmap j = neighbour j, ascending id, wpm words);
//   0 where v is not resident (a set member never needs it; LFA needs every
//   neighbour of me).
// Per (me, set p) the reference's getMinCostNodes + getNextHopsWithMetric +
// getNextHopsThrift (Decision.cpp:1082-1305, perDestination = false): per up
// link e of me towards x, over = w(e) + via(x) with via(x) = shortest -
// d_me(x) when x is a next hop of a min-cost member, lowered (LFA) to any
// member's d_x(dst) < shortest + d_x(me); kept when LFA or over == shortest.
// MODE:
//   kRsOne     one me: the records of spf_routes (deg(me) slots per set);
//   kRsDigest  digest[slot] += mix(rec + p) over routes with a kept link, rec =
//              mix(K (p + 1) + shortest) + sum over kept links of
//              mix(link_hash[l] + (u32) over);
//   kRsDb      every me's route database materialised (spf_mplan_route_records):
//              hdr[slot * n_sets + p] = offset | count << 32 | 256 << 48, the
//              route's k-th next hop at pool[base[slot] + offset + 256 k], one
//              u64 each = CSR edge | metric << 32, in link order.  A block's
//              256 routes share a [deg(me)][256] tile of me's region: the k-th
//              next hops of consecutive sets sit side by side, so lanes that
//              keep their k-th next hop at the same link -- consecutive
//              destinations of one pod do -- store to one line, and the
//              layout needs no count before the walk (no scan, no atomics, no
//              second walk); a tile's unused slots are never written.  A metric
//              past 2^32 - 1 sets flags bit 1.
constexpr int kRsOne = 0, kRsDigest = 1, kRsDb = 2;
constexpr uint32_t kRsThreads = 256;
constexpr uint32_t kRsGroup = 4;  // consecutive me slots per XCD turn
constexpr uint32_t kRsLinks = 256;  // me's links staged in LDS per pass
template <int MODE>
__global__ __launch_bounds__(kRsThreads) void route_sets_kernel(
    const unsigned long long* __restrict__ rowp, const unsigned long long* __restrict__ nhp,
    uint32_t wpm, const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const uint32_t* __restrict__ wt, const uint32_t* __restrict__ link,
    const uint32_t* __restrict__ edge_nb,
    const uint32_t* __restrict__ me_ids, const uint32_t* __restrict__ set_ptr,
    const uint32_t* __restrict__ set_nodes, uint32_t n_sets, uint32_t lfa,
    const unsigned long long* __restrict__ link_hash, unsigned long long* __restrict__ digest,
    uint64_t* __restrict__ out_min, uint32_t* __restrict__ out_cnt, uint32_t* __restrict__ out_edge,
    uint64_t* __restrict__ out_metric, uint32_t n_me, uint32_t n_chunks, RouteDbOut db) {
  // XCD-aware block order: blocks are dealt to the 8 XCDs round robin
  // (blockIdx % 8); me slots go in groups of kRsGroup consecutive slots, group
  // q to XCD q % 8 (heavy and light nodes of a locality-ordered list spread
  // over the XCDs), every set chunk of one me back to back on its XCD, so
  // me's row and bitmaps and its neighbours' rows (shared by the group's other
  // me) come from that XCD's L2 instead of once per XCD from the MALL
  const uint32_t g = blockIdx.x & 7u, i = blockIdx.x >> 3;
  const uint32_t L = i / n_chunks;  // this XCD's L-th me
  const uint32_t slot = ((L / kRsGroup) * 8 + g) * kRsGroup + L % kRsGroup;
  if (slot >= n_me) return;  // whole block
  const uint32_t me = me_ids[slot];
  const uint32_t chunk = i % n_chunks;
  const uint32_t p = chunk * kRsThreads + threadIdx.x;
  const uint32_t* Dme = reinterpret_cast<const uint32_t*>(rowp[me]);
  const uint32_t* NHme = reinterpret_cast<const uint32_t*>(nhp[me]);
  const uint32_t e0 = row_ptr[me], e1 = row_ptr[me + 1];
  const bool live = p < n_sets;
  const uint32_t b = live ? set_ptr[p] : 0u, e = live ? set_ptr[p + 1] : 0u;
  uint64_t shortest = kInf64;
  for (uint32_t k = b; k < e; ++k) {
    const uint32_t d = Dme[set_nodes[k]];
    if (d != kInf && d < shortest) shortest = d;
  }
  // a one-member set (a loopback, a node label): its node
  const bool one = e == b + 1;
  const uint32_t d0 = one ? set_nodes[b] : 0u;
  // (kRsDb) this block's tile of me's region: [deg][kRsThreads] records
  const uint64_t tile = MODE == kRsDb ? (uint64_t)chunk * kRsThreads * (e1 - e0) : 0ull;
  unsigned long long* const out = MODE == kRsDb ? db.pool + db.base[slot] + tile + threadIdx.x : nullptr;
  // me's up links, kRsLinks at a time, staged in LDS by the whole block: the
  // neighbour's bitmap index, its row's address, d_me(x), d_x(me), the link's
  // metric and hash -- formerly a dependent scalar chain per link and thread
  // (a binary search over me's neighbours, then rowp[x], then d_x(me)); a
  // spine's 173 links made its blocks the pass's tail
  __shared__ uint32_t s_j[kRsLinks], s_dmx[kRsLinks], s_back[kRsLinks], s_w[kRsLinks];
  __shared__ unsigned long long s_row[kRsLinks], s_lh[kRsLinks];
  uint64_t rec = 0;
  uint32_t cnt = 0;
  bool wide = false;
  for (uint32_t c0 = e0; c0 < e1; c0 += kRsLinks) {  // block-uniform
    const uint32_t nl = min(kRsLinks, e1 - c0);
    __syncthreads();  // the previous chunk's reads are done
    for (uint32_t t = threadIdx.x; t < nl; t += kRsThreads) {
      const uint32_t q = c0 + t, x = col[q];
      const unsigned long long rx = lfa && x != me ? rowp[x] : 0ull;
      s_j[t] = edge_nb[q];
      s_dmx[t] = Dme[x];
      s_w[t] = wt[q];
      s_row[t] = rx;
      s_back[t] = rx ? reinterpret_cast<const uint32_t*>(rx)[me] : kInf;
      if constexpr (MODE == kRsDigest) s_lh[t] = link_hash[link[q]];
    }
    __syncthreads();
    if (shortest == kInf64) continue;  // (every thread still meets the barriers)
    for (uint32_t t = 0; t < nl; ++t) {
      if (s_j[t] == kInf) continue;  // a dead slot (no link)
      // getNextHopsWithMetric: x is a shortest-path next hop of a min-cost
      // member (via = shortest - d_me(x)), lowered with LFA to a member's
      // d_x(dst) < shortest + d_x(me)
      uint64_t via = kInf64;
      const uint32_t* bm = NHme + (size_t)s_j[t] * wpm;
      const uint32_t* Dx = reinterpret_cast<const uint32_t*>(s_row[t]);
      const uint64_t back = s_back[t];
      if (one) {  // Dme[d0] == shortest
        const uint32_t bw = bm[d0 >> 5];
        const uint32_t dxd = Dx ? Dx[d0] : kInf;  // (Dx is null without LFA)
        if ((bw >> (d0 & 31)) & 1u) via = shortest - s_dmx[t];
        if (lfa && dxd != kInf && back != kInf && (uint64_t)dxd < shortest + back &&
            (via == kInf64 || via > dxd))
          via = dxd;
      } else {
        for (uint32_t k = b; k < e; ++k) {
          const uint32_t d = set_nodes[k];
          if (Dme[d] != shortest) continue;
          if ((bm[d >> 5] >> (d & 31)) & 1u) {
            via = shortest - s_dmx[t];
            break;
          }
        }
        if (Dx)
          for (uint32_t k = b; k < e; ++k) {
            const uint32_t dxd = Dx[set_nodes[k]];
            if (dxd == kInf || back == kInf) continue;
            if ((uint64_t)dxd < shortest + back && (via == kInf64 || via > dxd)) via = dxd;
          }
      }
      if (via == kInf64) continue;
      const uint64_t over = (uint64_t)s_w[t] + via;
      if (!lfa && over != shortest) continue;
      if constexpr (MODE == kRsDigest) {
        rec += rmix64(s_lh[t] + (uint32_t)over);
      } else if constexpr (MODE == kRsDb) {
        wide |= (over >> 32) != 0;
        __builtin_nontemporal_store((unsigned long long)(c0 + t) | (over << 32),
                                    out + (size_t)cnt * kRsThreads);
      } else {
        const uint32_t deg = e1 - e0;
        out_edge[(size_t)p * deg + cnt] = c0 + t;
        out_metric[(size_t)p * deg + cnt] = over;
      }
      ++cnt;
    }
  }
  if constexpr (MODE == kRsDigest) {
    uint64_t h = (live && cnt) ? rmix64(rmix64(0x9e3779b97f4a7c15ull * (p + 1) + shortest) + rec + p) : 0ull;
    // wave sum, one atomic per wave
    for (int d = 32; d >= 1; d >>= 1) {
      const uint32_t lo2 = __shfl_down((uint32_t)h, d, 64), hi2 = __shfl_down((uint32_t)(h >> 32), d, 64);
      h += ((uint64_t)hi2 << 32) | lo2;
    }
    if ((threadIdx.x & 63) == 0 && h) atomicAdd(&digest[slot], (unsigned long long)h);
  } else if constexpr (MODE == kRsDb) {
    if (wide) atomicOr(db.flags, 2u);
    uint32_t wsum = live ? cnt : 0u;  // the me's record count: one atomic per wave
    for (int d = 32; d >= 1; d >>= 1) wsum += __shfl_down(wsum, d, 64);
    if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&db.count[slot], wsum);
    if (live)
      db.hdr[(size_t)slot * n_sets + p] = (tile + threadIdx.x) | ((unsigned long long)cnt << 32) |
                                          ((unsigned long long)kRsThreads << 48);
  } else {
    if (live) {
      out_min[p] = shortest;
      out_cnt[p] = cnt;
    }
  }
}

// The many-me modes (kRsDigest, kRsDb) with four sets per thread: 1,024 sets
// per block.  When a thread's four sets are single nodes d, d+1, d+2, d+3 (d
// a multiple of 4: every node's loopback, CS-2), one link costs one bitmap
// word and one 16-byte load of d_x(d .. d+3) for all four -- a quarter of the
// load instructions of a thread per set (the selection is bound by them, not
// by bytes: reading u8 rows instead made it slower).  Other sets take the
// per-set path.  kRsDb tiles are [deg(me)][1024].
constexpr uint32_t kRqSets = 4;
constexpr uint32_t kRqPerBlock = kRqSets * kRsThreads;
constexpr bool kRqNt = true;  // streaming 32-byte stores (full lines when a wave's routes agree)
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
template <int MODE, typename Dist>
__global__ __launch_bounds__(kRsThreads) __attribute__((amdgpu_waves_per_eu(MODE == kRsDb && sizeof(Dist) == 4 ? 8 : 1)))
void route_quads_kernel(
    const unsigned long long* __restrict__ rowp, const unsigned long long* __restrict__ nhp,
    uint32_t wpm, const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const uint32_t* __restrict__ wt, const uint32_t* __restrict__ link,
    const uint32_t* __restrict__ edge_nb,
    const uint32_t* __restrict__ me_ids, const uint32_t* __restrict__ set_ptr,
    const uint32_t* __restrict__ set_nodes, uint32_t n_sets, uint32_t lfa,
    const unsigned long long* __restrict__ link_hash, unsigned long long* __restrict__ digest,
    uint32_t n_me, uint32_t n_chunks, RouteDbOut db,
    const unsigned long long* __restrict__ nrowp /* exact u8 rows (LFA loads), or null */) {
  const uint32_t g = blockIdx.x & 7u, i = blockIdx.x >> 3;  // XCD-aware order, as route_sets_kernel
  const uint32_t L = i / n_chunks;
  const uint32_t slot = ((L / kRsGroup) * 8 + g) * kRsGroup + L % kRsGroup;
  if (slot >= n_me) return;  // whole block
  const uint32_t me = me_ids[slot];
  const uint32_t chunk = i % n_chunks;
  const uint32_t p0 = chunk * kRqPerBlock + kRqSets * threadIdx.x;
  const uint32_t* Dme = reinterpret_cast<const uint32_t*>(rowp[me]);
  const uint32_t* NHme = reinterpret_cast<const uint32_t*>(nhp[me]);
  const uint32_t e0 = row_ptr[me], e1 = row_ptr[me + 1];
  // Dist: the selection's sums (d + metric, shortest + d_x(me)) in u64, or
  // in u32 when the host proved every finite sum stays below kInf (fewer
  // VALU instructions: the selection is VALU-bound)
  constexpr Dist kInfD = (Dist)~(Dist)0;
  Dist sh[kRqSets];
  uint64_t rec[kRqSets];
  uint32_t cnt[kRqSets], b[kRqSets], e[kRqSets];
  bool vec = true;
#pragma unroll
  for (uint32_t j = 0; j < kRqSets; ++j) {
    const bool live = p0 + j < n_sets;
    b[j] = live ? set_ptr[p0 + j] : 0u;
    e[j] = live ? set_ptr[p0 + j + 1] : 0u;
    vec &= e[j] == b[j] + 1;
    sh[j] = kInfD;
    rec[j] = 0;
    cnt[j] = 0;
  }
  const uint32_t d0 = vec ? set_nodes[b[0]] : 0u;
  if (vec) {
#pragma unroll
    for (uint32_t j = 1; j < kRqSets; ++j) vec &= set_nodes[b[j]] == d0 + j;
    vec &= (d0 & 3u) == 0u;
  }
  if (vec) {
    const uint4 d4 = *reinterpret_cast<const uint4*>(Dme + d0);
    const uint32_t dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
    for (uint32_t j = 0; j < kRqSets; ++j) sh[j] = dd[j] == kInf ? kInfD : (Dist)dd[j];
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kRqSets; ++j)
      for (uint32_t k = b[j]; k < e[j]; ++k) {
        const uint32_t d = Dme[set_nodes[k]];
        if (d != kInf && d < sh[j]) sh[j] = d;
      }
  }
  bool any_route = false;
#pragma unroll
  for (uint32_t j = 0; j < kRqSets; ++j) any_route |= sh[j] != kInfD;
  const uint64_t tile = MODE == kRsDb ? (uint64_t)chunk * kRqPerBlock * (e1 - e0) : 0ull;
  unsigned long long* const out =
      MODE == kRsDb ? db.pool + db.base[slot] + tile + kRqSets * threadIdx.x : nullptr;
  __shared__ uint32_t s_j[kRsLinks], s_dmx[kRsLinks], s_back[kRsLinks], s_w[kRsLinks];
  __shared__ unsigned long long s_row[kRsLinks], s_lh[kRsLinks], s_row8[kRsLinks];
  bool wide = false;
  for (uint32_t c0 = e0; c0 < e1; c0 += kRsLinks) {  // block-uniform
    const uint32_t nl = min(kRsLinks, e1 - c0);
    __syncthreads();  // the previous chunk's reads are done
    for (uint32_t t = threadIdx.x; t < nl; t += kRsThreads) {
      const uint32_t q = c0 + t, x = col[q];
      const unsigned long long rx = lfa && x != me ? rowp[x] : 0ull;
      s_j[t] = edge_nb[q];
      s_dmx[t] = Dme[x];
      s_w[t] = wt[q];
      s_row[t] = rx;
      s_row8[t] = rx && nrowp ? nrowp[x] : 0ull;
      s_back[t] = rx ? reinterpret_cast<const uint32_t*>(rx)[me] : kInf;
      if constexpr (MODE == kRsDigest) s_lh[t] = link_hash[link[q]];
    }
    __syncthreads();
    if (!any_route) continue;  // (every thread still meets the barriers)
    for (uint32_t t = 0; t < nl; ++t) {
      if (s_j[t] == kInf) continue;  // a dead slot (no link)
      const uint32_t* bm = NHme + (size_t)s_j[t] * wpm;
      const uint32_t* Dx = reinterpret_cast<const uint32_t*>(s_row[t]);
      const Dist back = s_back[t] == kInf ? kInfD : (Dist)s_back[t];
      const uint32_t dmx = s_dmx[t];
      Dist via[kRqSets];
      if (vec) {  // four consecutive single destinations: one word, one 16-byte load
        const uint32_t bw = bm[d0 >> 5];
        uint32_t dx[4] = {kInf, kInf, kInf, kInf};
        if (const uint8_t* Dx8 = reinterpret_cast<const uint8_t*>(s_row8[t])) {
          // the same four distances as bytes (exact: unit metrics, depth < 254)
          const uint32_t b4 = *reinterpret_cast<const uint32_t*>(Dx8 + d0);
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t v = (b4 >> (8 * j)) & 0xFFu;
            dx[j] = v == 0xFFu ? kInf : v;
          }
        } else if (Dx) {
          const uint4 x4 = *reinterpret_cast<const uint4*>(Dx + d0);
          dx[0] = x4.x, dx[1] = x4.y, dx[2] = x4.z, dx[3] = x4.w;
        }
#pragma unroll
        for (uint32_t j = 0; j < kRqSets; ++j) {
          via[j] = kInfD;
          if (sh[j] == kInfD) continue;
          if ((bw >> ((d0 + j) & 31)) & 1u) via[j] = sh[j] - dmx;
          if (lfa && dx[j] != kInf && back != kInfD && (Dist)dx[j] < sh[j] + back &&
              (via[j] == kInfD || via[j] > (Dist)dx[j]))
            via[j] = dx[j];
        }
      } else {
#pragma unroll
        for (uint32_t j = 0; j < kRqSets; ++j) {
          via[j] = kInfD;
          if (sh[j] == kInfD) continue;
          for (uint32_t k = b[j]; k < e[j]; ++k) {
            const uint32_t d = set_nodes[k];
            if (Dme[d] != sh[j]) continue;
            if ((bm[d >> 5] >> (d & 31)) & 1u) {
              via[j] = sh[j] - dmx;
              break;
            }
          }
          if (Dx)
            for (uint32_t k = b[j]; k < e[j]; ++k) {
              const uint32_t dxd = Dx[set_nodes[k]];
              if (dxd == kInf || back == kInfD) continue;
              if ((Dist)dxd < sh[j] + back && (via[j] == kInfD || via[j] > (Dist)dxd)) via[j] = dxd;
            }
        }
      }
      Dist over[kRqSets];
      bool keep[kRqSets];
#pragma unroll
      for (uint32_t j = 0; j < kRqSets; ++j) {
        over[j] = (Dist)s_w[t] + via[j];
        keep[j] = via[j] != kInfD && (lfa || over[j] == sh[j]);
      }
      if constexpr (MODE == kRsDigest) {
#pragma unroll
        for (uint32_t j = 0; j < kRqSets; ++j)
          if (keep[j]) {
            rec[j] += rmix64(s_lh[t] + (uint32_t)over[j]);
            ++cnt[j];
          }
      } else {
        const unsigned long long eb = c0 + t;
        if (keep[0] && keep[1] && keep[2] && keep[3] && cnt[0] == cnt[1] && cnt[1] == cnt[2] &&
            cnt[2] == cnt[3]) {
          // the four routes' next hop at the same position (consecutive
          // destinations of one pod): one 32-byte store
          u64x2* o = reinterpret_cast<u64x2*>(out + (size_t)cnt[0] * kRqPerBlock);
          const u64x2 a = {eb | ((uint64_t)over[0] << 32), eb | ((uint64_t)over[1] << 32)};
          const u64x2 z = {eb | ((uint64_t)over[2] << 32), eb | ((uint64_t)over[3] << 32)};
          if constexpr (kRqNt) {
            __builtin_nontemporal_store(a, o);
            __builtin_nontemporal_store(z, o + 1);
          } else {
            o[0] = a;
            o[1] = z;
          }
#pragma unroll
          for (uint32_t j = 0; j < kRqSets; ++j) {
            wide |= ((uint64_t)over[j] >> 32) != 0;
            ++cnt[j];
          }
        } else {
#pragma unroll
          for (uint32_t j = 0; j < kRqSets; ++j)
            if (keep[j]) {
              wide |= ((uint64_t)over[j] >> 32) != 0;
              out[(size_t)cnt[j] * kRqPerBlock + j] = eb | ((uint64_t)over[j] << 32);
              ++cnt[j];
            }
        }
      }
    }
  }
  if constexpr (MODE == kRsDigest) {
    uint64_t h = 0;
#pragma unroll
    for (uint32_t j = 0; j < kRqSets; ++j) {
      const uint32_t p = p0 + j;
      if (p < n_sets && cnt[j]) h += rmix64(rmix64(0x9e3779b97f4a7c15ull * (p + 1) + sh[j]) + rec[j] + p);
    }
    for (int d = 32; d >= 1; d >>= 1) {  // wave sum, one atomic per wave
      const uint32_t lo2 = __shfl_down((uint32_t)h, d, 64), hi2 = __shfl_down((uint32_t)(h >> 32), d, 64);
      h += ((uint64_t)hi2 << 32) | lo2;
    }
    if ((threadIdx.x & 63) == 0 && h) atomicAdd(&digest[slot], (unsigned long long)h);
  } else {
    if (wide) atomicOr(db.flags, 2u);
    uint32_t wsum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kRqSets; ++j) {
      const uint32_t p = p0 + j;
      if (p >= n_sets) continue;
      wsum += cnt[j];
      db.hdr[(size_t)slot * n_sets + p] = (tile + kRqSets * threadIdx.x + j) | ((unsigned long long)cnt[j] << 32) |
                                          ((unsigned long long)kRqPerBlock << 48);
    }
    for (int d = 32; d >= 1; d >>= 1) wsum += __shfl_down(wsum, d, 64);
    if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&db.count[slot], wsum);
  }
}

}  // namespace

namespace spfi {

uint32_t route_db_tile_sets() { return std::getenv("SPF_ROUTE_SETS1") ? kRsThreads : kRqPerBlock; }

spf_status launch_route_sets(spf_ctx* c, const unsigned long long* d_rowp,
                             const unsigned long long* d_nhp, const uint32_t* d_me, uint32_t n_me,
                             const uint32_t* d_set_ptr, const uint32_t* d_set_nodes, uint32_t n_sets,
                             bool lfa, const unsigned long long* d_link_hash,
                             unsigned long long* d_digest, uint64_t* d_min, uint32_t* d_cnt,
                             uint32_t* d_edge, uint64_t* d_metric, hipStream_t s, const RouteDbOut* db,
                             const unsigned long long* d_nrowp) {
  if (!n_me || !n_sets) return SPF_OK;
  if ((db || d_digest) && !std::getenv("SPF_ROUTE_SETS1")) {  // four sets per thread (SPF_ROUTE_SETS1: one, A/B)
    const uint32_t n_chunks = (n_sets + kRqPerBlock - 1) / kRqPerBlock;
    const uint32_t groups = (n_me + kRsGroup - 1) / kRsGroup;
    const uint64_t blocks = 8ull * ((groups + 7) / 8 * kRsGroup) * n_chunks;
    if (blocks >= (1ull << 31)) return fail(c, SPF_E_INVALID, "route sets: grid too large");
    // u32 sums when no finite one can reach kInf: distances are at most
    // B = max metric x (N - 1), a sum at most 2B + max metric (SPF_ROUTE_U64=1: A/B)
    const uint64_t mm = std::max<uint32_t>(c->max_metric, 1u);
    const uint64_t B = mm * (uint64_t)(c->N ? c->N - 1 : 0);
    const bool n32 = !c->needs64 && 2 * B + mm < (uint64_t)kInf && !std::getenv("SPF_ROUTE_U64");
    const dim3 grid((uint32_t)blocks), block(kRsThreads);
    const uint32_t wpm = c->pitch / 32, lf = lfa ? 1u : 0u;
    if (db && n32)
      hipLaunchKernelGGL((route_quads_kernel<kRsDb, uint32_t>), grid, block, 0, s, d_rowp, d_nhp, wpm,
                         c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p, d_me,
                         d_set_ptr, d_set_nodes, n_sets, lf, nullptr, nullptr, n_me, n_chunks, *db, d_nrowp);
    else if (db)
      hipLaunchKernelGGL((route_quads_kernel<kRsDb, uint64_t>), grid, block, 0, s, d_rowp, d_nhp, wpm,
                         c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p, d_me,
                         d_set_ptr, d_set_nodes, n_sets, lf, nullptr, nullptr, n_me, n_chunks, *db, d_nrowp);
    else if (n32)
      hipLaunchKernelGGL((route_quads_kernel<kRsDigest, uint32_t>), grid, block, 0, s, d_rowp, d_nhp, wpm,
                         c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p, d_me,
                         d_set_ptr, d_set_nodes, n_sets, lf, d_link_hash, d_digest, n_me, n_chunks,
                         RouteDbOut{}, d_nrowp);
    else
      hipLaunchKernelGGL((route_quads_kernel<kRsDigest, uint64_t>), grid, block, 0, s, d_rowp, d_nhp, wpm,
                         c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p, d_me,
                         d_set_ptr, d_set_nodes, n_sets, lf, d_link_hash, d_digest, n_me, n_chunks,
                         RouteDbOut{}, d_nrowp);
    HIP_TRY(c, hipGetLastError());
    return SPF_OK;
  }
  const uint32_t n_chunks = (n_sets + kRsThreads - 1) / kRsThreads;
  const uint32_t groups = (n_me + kRsGroup - 1) / kRsGroup;
  const uint32_t per_xcd = (groups + 7) / 8 * kRsGroup;  // the most me slots any XCD takes
  const uint64_t blocks = 8ull * per_xcd * n_chunks;
  if (blocks >= (1ull << 31)) return fail(c, SPF_E_INVALID, "route sets: grid too large");
  const dim3 grid((uint32_t)blocks);
  if (db)
    hipLaunchKernelGGL(route_sets_kernel<kRsDb>, grid, dim3(kRsThreads), 0, s, d_rowp, d_nhp,
                       c->pitch / 32, c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p,
                       d_me, d_set_ptr, d_set_nodes, n_sets, lfa ? 1u : 0u, nullptr,
                       nullptr, nullptr, nullptr, nullptr, nullptr, n_me, n_chunks, *db);
  else if (d_digest)
    hipLaunchKernelGGL(route_sets_kernel<kRsDigest>, grid, dim3(kRsThreads), 0, s, d_rowp, d_nhp,
                       c->pitch / 32, c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p,
                       d_me, d_set_ptr, d_set_nodes, n_sets, lfa ? 1u : 0u, d_link_hash,
                       d_digest, nullptr, nullptr, nullptr, nullptr, n_me, n_chunks, RouteDbOut{});
  else
    hipLaunchKernelGGL(route_sets_kernel<kRsOne>, grid, dim3(kRsThreads), 0, s, d_rowp, d_nhp,
                       c->pitch / 32, c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_link.p, c->d_edge_nb.p,
                       d_me, d_set_ptr, d_set_nodes, n_sets, lfa ? 1u : 0u, nullptr,
                       nullptr, d_min, d_cnt, d_edge, d_metric, n_me, n_chunks, RouteDbOut{});
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

}  // namespace spfi

extern "C" {

spf_status spf_routes(spf_ctx* c, uint32_t me, const uint32_t* set_ptr,
                      const uint32_t* set_nodes, uint32_t n_sets, uint32_t flags,
                      uint64_t* min_metric, uint32_t* nh_count, uint32_t* nh_edge,
                      uint64_t* nh_metric) {
  if (!c || !set_ptr || !min_metric || !nh_count || !nh_edge || !nh_metric)
    return fail(c, SPF_E_INVALID, "spf_routes: NULL argument");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (me >= c->N) return fail(c, SPF_E_INVALID, "node %u out of range", me);
  const uint32_t N = c->N;
  const uint32_t n_members = set_ptr[n_sets];
  for (uint32_t i = 0; i < n_members; ++i)
    if (set_nodes[i] >= N) return fail(c, SPF_E_INVALID, "set member %u out of range", set_nodes[i]);
  const bool lfa = (flags & SPF_ROUTE_LFA) != 0;
  // sources: me, and with LFA every distinct up neighbour (getSpfResult(nbr),
  // Decision.cpp:1165)
  std::vector<uint32_t> srcs{me};
  const uint32_t nb0 = c->nb_ptr[me], k = c->nb_ptr[me + 1] - nb0;
  if (lfa)
    for (uint32_t j = 0; j < k; ++j) srcs.push_back(c->nb_id[nb0 + j]);
  // the previous call's plan when it solved the same sources on this graph
  // shape (a route build per publication: me and its neighbours again)
  spf_ctx::RouteCache& rc = c->rt;
  spf_status st = SPF_OK;
  if (!rc.plan || rc.shape != c->shape || rc.srcs != srcs) {
    spf_plan_destroy(rc.plan);
    rc.plan = nullptr;
    st = spf_plan_create(c, srcs.data(), (uint32_t)srcs.size(), 0, &rc.plan);
    if (st != SPF_OK) return st;
    rc.srcs = srcs;
    rc.shape = c->shape;
  }
  spf_plan* p = rc.plan;
  // me's up links in linksFromNode order, with the bitmap index of their far end
  const uint32_t e0 = c->row_ptr[me], deg = c->row_ptr[me + 1] - e0;
  std::vector<uint32_t> ecol(deg), ew(deg), ej(deg);
  for (uint32_t i = 0; i < deg; ++i) {
    ecol[i] = c->col[e0 + i];
    ew[i] = c->wt[e0 + i];
    const uint32_t* f = std::lower_bound(c->nb_id.data() + nb0, c->nb_id.data() + nb0 + k, ecol[i]);
    ej[i] = ecol[i] == me ? kInf : (uint32_t)(f - (c->nb_id.data() + nb0));  // dead slot: none
  }
  auto& d_dist = rc.dist;
  auto& d_nh = rc.nh;
  auto& d_ecol = rc.ecol;
  auto& d_ew = rc.ew;
  auto& d_ej = rc.ej;
  auto& d_sp = rc.sp;
  auto& d_sn = rc.sn;
  auto& d_cnt = rc.cnt;
  auto& d_edge = rc.edge;
  auto& d_min = rc.mn;
  auto& d_metric = rc.metric;
  HIP_TRY(c, d_dist.alloc((size_t)srcs.size() * c->pitch));
  HIP_TRY(c, d_nh.alloc(std::max<uint64_t>(1, spf_plan_nh_words(p))));
  HIP_TRY(c, stage_upload(c, d_ecol, ecol.data(), deg));
  HIP_TRY(c, stage_upload(c, d_ew, ew.data(), deg));
  HIP_TRY(c, stage_upload(c, d_ej, ej.data(), deg));
  HIP_TRY(c, stage_upload(c, d_sp, set_ptr, n_sets + 1));
  HIP_TRY(c, stage_upload(c, d_sn, set_nodes, std::max<uint32_t>(1, n_members)));
  const size_t cap = (size_t)n_sets * std::max<uint32_t>(1, deg);
  HIP_TRY(c, d_min.alloc(std::max<uint32_t>(1, n_sets)));
  HIP_TRY(c, d_cnt.alloc(std::max<uint32_t>(1, n_sets)));
  HIP_TRY(c, d_edge.alloc(cap));
  HIP_TRY(c, d_metric.alloc(cap));
  st = spf_plan_execute(p, d_dist.p, d_nh.p, c->stream);
  if (st == SPF_E_STATE) {  // a row patch changed a source's next-hop layout: a new plan
    spf_plan_destroy(rc.plan);
    rc.plan = nullptr;
    st = spf_plan_create(c, srcs.data(), (uint32_t)srcs.size(), 0, &rc.plan);
    if (st != SPF_OK) return st;
    p = rc.plan;
    HIP_TRY(c, d_nh.alloc(std::max<uint64_t>(1, spf_plan_nh_words(p))));
    st = spf_plan_execute(p, d_dist.p, d_nh.p, c->stream);
  }
  if (st != SPF_OK) return st;
  // the plan's D rows: the caller buffer when the source set is closed,
  // otherwise the plan's own closure rows
  const uint32_t* D = p->direct ? d_dist.p : p->d_D.p;
  if (n_sets) {
    hipLaunchKernelGGL(routes_kernel, dim3(n_sets), dim3(64), 0, c->stream, D, c->pitch,
                       p->d_row_of.p, d_nh.p, me, d_ecol.p, d_ew.p, d_ej.p, deg, d_sp.p, d_sn.p,
                       lfa ? 1u : 0u, d_min.p, d_cnt.p, d_edge.p, d_metric.p);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(min_metric, d_min.p, 8ull * n_sets, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(nh_count, d_cnt.p, 4ull * n_sets, hipMemcpyDeviceToHost, c->stream));
    if (deg) {
      HIP_TRY(c, hipMemcpyAsync(nh_edge, d_edge.p, 4ull * cap, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(c, hipMemcpyAsync(nh_metric, d_metric.p, 8ull * cap, hipMemcpyDeviceToHost, c->stream));
    }
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  stage_done(c);
  // out edges are positions in me's CSR row: make them global edge ids
  for (size_t i = 0; i < (size_t)n_sets; ++i)
    for (uint32_t t = 0; t < nh_count[i]; ++t) nh_edge[i * deg + t] += e0;
  return SPF_OK;
}

}  // extern "C"
