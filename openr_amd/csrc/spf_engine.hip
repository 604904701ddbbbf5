// ============================================================================
//  spf_engine.hip -- MI355X (gfx950) all-sources SPF + ECMP engine.
//
//  Implements include/openr_spf.h.  What the reference computes per source in
//  LinkState::runSpf (openr/decision/LinkState.cpp:808-882) is produced here by
//  two data-parallel passes over a CSR graph resident in HBM:
//
//   1. sssp_kernel  -- one workgroup per source row.  Frontier-based
//      Bellman-Ford (== level-synchronous BFS for unit metrics) with the
//      distance array and the frontier queue in LDS; the next frontier is a
//      LDS bitmap compacted with wave ballots/scans.  Writes the distance row
//      D[row][0..N) to HBM.
//
//   2. ecmp_kernel  -- the next-hop pass.  For positive metrics the
//      reference's next-hop union over the shortest-path DAG equals
//         x in nh_s(v)  <=>  (x == v  or  x not overloaded)
//                            and  w(s,x) + d_x(v) == d_s(v)
//      over the distinct up neighbours x of s (w = min metric over s->x
//      links).  Proof sketch in DESIGN.md §3.  So the pass is a streaming
//      compare of D rows: coalesced 16-byte loads, one bit per neighbour,
//      planar u32 words written once.  Blocks are remapped so that the 32 CUs
//      of one XCD walk a contiguous source range and share neighbour rows in
//      their L2.
//
//   3. preds_kernel -- pathLinks of one source (tight in-edges of expanded
//      predecessors, in (dist, node, edge) = Dijkstra pop order).
//
//  Everything is integer.  Distances are u32; spf_graph_load rejects graphs
//  whose longest possible path does not fit (see openr_spf.h).
// ============================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "engine_internal.h"
#include "wave_ops.h"

namespace spfi {

thread_local std::string g_err;

spf_status fail(spf_ctx* c, spf_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  g_err = buf;
  return st;
}

}  // namespace spfi

using namespace spfi;

namespace {

constexpr int kEcmpThreads = 256;
constexpr uint32_t kBigDeg = 24;  // > kBigDeg: expanded by a whole wave
constexpr size_t kMaxLds = 160 * 1024;


// ---------------------------------------------------------------------------
//  device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// wave_excl_scan / wave_or32 / wave_max32 / wave_or64: wave_ops.h

__device__ __forceinline__ bool link_ignored(const uint32_t* ign, uint32_t l) {
  return (ign[l >> 5] >> (l & 31)) & 1u;
}

// LDS control words of the SSSP kernel
enum { C_QLEN = 0, C_NBIG = 1, C_NWORDS = 4 };

// ---------------------------------------------------------------------------
//  1. single-source shortest paths, one workgroup per source row
// ---------------------------------------------------------------------------
//   THREADS: a workgroup's distance row sits in LDS, so a large graph fits
//   only one or two workgroups per CU; those then get 1024 threads, so the
//   CU still holds 32 waves of relaxations in flight (PMC r02_v9, fabric_rtt
//   with 256 threads: 75 % of wave cycles waiting, ~8 waves per CU).
template <typename QT, bool UNIT, int THREADS>
__global__ __launch_bounds__(THREADS) void sssp_kernel(
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const uint32_t* __restrict__ wt, const uint8_t* __restrict__ ovl,
    const uint32_t* __restrict__ link, const uint32_t* __restrict__ ign,
    const uint32_t* __restrict__ rows_src, uint32_t N, uint32_t pitch,
    uint32_t bm_words, uint32_t big_cap, uint32_t* __restrict__ D,
    uint8_t* __restrict__ Dn /* optional u8 copy (npitch == pitch) */,
    const uint32_t* __restrict__ redo /* optional [count, rows...]: redo only those rows */) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* dist = reinterpret_cast<uint32_t*>(smem);  // [pitch]
  uint32_t* bm = dist + pitch;                         // [bm_words] next frontier
  uint32_t* ctl = bm + bm_words;                       // [C_NWORDS]
  uint32_t* big = ctl + C_NWORDS;                      // [big_cap]
  QT* q = reinterpret_cast<QT*>(big + big_cap);        // [N] frontier list

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = tid >> 6;
  constexpr uint32_t kWaves = THREADS / 64;
  uint32_t row = blockIdx.x;
  if (redo) {  // mssp_kernel's overflow rows (launched over all rows, mostly empty)
    if (row >= redo[0]) return;
    row = redo[1 + row];
  }
  const uint32_t src = rows_src[row];

  for (uint32_t v = tid; v < pitch; v += THREADS) dist[v] = kInf;
  for (uint32_t i = tid; i < bm_words; i += THREADS) bm[i] = 0;
  if (tid == 0) {
    ctl[C_QLEN] = 0;
    ctl[C_NBIG] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    dist[src] = 0;
    q[0] = (QT)src;
  }
  __syncthreads();

  uint32_t qlen = 1;
  while (qlen != 0) {
    // ---- expand: small-degree nodes one per thread, big ones per wave ----
    for (uint32_t i = tid; i < qlen; i += THREADS) {
      const uint32_t u = q[i];
      if (ovl[u] && u != src) continue;  // drained node: recorded, not expanded
      const uint32_t b = row_ptr[u], e = row_ptr[u + 1];
      if (e - b > kBigDeg) {
        big[atomicAdd(&ctl[C_NBIG], 1u)] = u;
        continue;
      }
      const uint32_t du = dist[u];
      for (uint32_t k = b; k < e; ++k) {
        if (ign && link_ignored(ign, link[k])) continue;  // KSP linksToIgnore
        const uint32_t v = col[k];
        const uint32_t nd = du + (UNIT ? 1u : wt[k]);
        if (UNIT) {
          // level-synchronous BFS: every writer of v writes the same value
          if (dist[v] > nd) {
            dist[v] = nd;
            atomicOr(&bm[v >> 5], 1u << (v & 31));
          }
        } else {
          if (nd < atomicMin(&dist[v], nd)) atomicOr(&bm[v >> 5], 1u << (v & 31));
        }
      }
    }
    __syncthreads();
    const uint32_t nbig = ctl[C_NBIG];
    for (uint32_t i = wave; i < nbig; i += kWaves) {
      const uint32_t u = big[i];
      const uint32_t du = dist[u];
      const uint32_t e = row_ptr[u + 1];
      for (uint32_t k = row_ptr[u] + lane; k < e; k += 64) {
        if (ign && link_ignored(ign, link[k])) continue;
        const uint32_t v = col[k];
        const uint32_t nd = du + (UNIT ? 1u : wt[k]);
        if (UNIT) {
          if (dist[v] > nd) {
            dist[v] = nd;
            atomicOr(&bm[v >> 5], 1u << (v & 31));
          }
        } else {
          if (nd < atomicMin(&dist[v], nd)) atomicOr(&bm[v >> 5], 1u << (v & 31));
        }
      }
    }
    __syncthreads();
    if (tid == 0) ctl[C_NBIG] = 0;  // every thread has read nbig by now

    // ---- compact the next-frontier bitmap into q (wave ballot/scan) ----
    for (uint32_t base = 0; base < bm_words; base += THREADS) {
      const uint32_t i = base + tid;
      uint32_t word = 0;
      if (i < bm_words) {
        word = bm[i];
        bm[i] = 0;
      }
      uint32_t tot;
      const uint32_t pre = wave_excl_scan(__popc(word), &tot);
      uint32_t at = 0;
      if (lane == 0 && tot) at = atomicAdd(&ctl[C_QLEN], tot);
      at = __builtin_amdgcn_readlane(at, 0) + pre;
      while (word) {
        const uint32_t b = __ffs(word) - 1;
        word &= word - 1;
        q[at++] = (QT)(i * 32 + b);
      }
    }
    __syncthreads();
    qlen = ctl[C_QLEN];
    __syncthreads();
    if (tid == 0) ctl[C_QLEN] = 0;
  }
  __syncthreads();

  // ---- write the distance row (16-byte stores) and, for narrow plans, its
  // u8 copy (min(d, 254), 255 = unreachable) for the next-hop pass ----
  uint4* out = reinterpret_cast<uint4*>(D + (size_t)row * pitch);
  const uint4* in = reinterpret_cast<const uint4*>(dist);
  for (uint32_t i = tid; i < pitch / 4; i += THREADS) {
    const uint4 d = in[i];
    out[i] = d;
    if (Dn) {
      const uint32_t x[4] = {d.x, d.y, d.z, d.w};
      uint32_t b = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) b |= (x[k] == kInf ? 0xFFu : min(x[k], 254u)) << (8 * k);
      reinterpret_cast<uint32_t*>(Dn + (size_t)row * pitch)[i] = b;
    }
  }
}

// ---------------------------------------------------------------------------
//  1b. multi-source BFS for unit metrics: 64 sources per workgroup
// ---------------------------------------------------------------------------
// Every node carries a 64-bit mask, bit s = "source s of this batch".  A level
// is one pull sweep: new(v) = OR_{u in N(v)} F(u) & ~visited(v), where F holds
// the previous level's new masks.  A drained node is recorded but expands only
// as the source (LinkState.cpp:831-838): its producer writes F(v) masked to its
// own source bit, so the consumer loop is branch-free.  One edge sweep serves
// 64 sources, against 64 sweeps for the per-source kernel.
//   * F lives in LDS (8 B/node, F[N] = 0 is the padding target).
//   * visited / new masks of the nodes a thread owns (v = tid + i*1024) live in
//     registers; the 64 lanes of a wave own 64 consecutive nodes = one slice
//     of the sliced-ELL column array, so neighbour j of all 64 nodes is one
//     coalesced 256-byte load (kMsUnroll of them in flight).
//   * distances are written per level as predicated stores over the sources
//     that have new nodes in the wave; one store covers 64 consecutive nodes
//     of one source row.  The u8 narrow copy for the next-hop pass saturates at
//     254.
constexpr int kMsThreads = 1024;
constexpr uint32_t kMsBatch = 64;
constexpr int kMsMaxOwn = 16;
constexpr uint32_t kMsMaxNodes = kMsThreads * kMsMaxOwn;  // 16384 (F: 128 KiB of LDS)
constexpr int kMsUnroll = 8;
constexpr uint32_t kMsLaneStoreRatio = 4;  // per-lane stores when 4 * max per-node count < #sources
constexpr uint32_t kSliceW = 64;  // nodes per sliced-ELL slice (= wave width)
constexpr uint32_t kNoSlice = 0x03FFFFFFu;  // unused slot: its nodes (kNoSlice * 64 + lane) lie past N

// owned slots per thread of msbfs_kernel (the template instances: 1, 2, 4, 8,
// 10, 12, 16) for an N-node graph
inline uint32_t ms_own(uint32_t N) {
  const uint32_t own = (N + kMsThreads - 1) / kMsThreads;
  return own <= 1 ? 1 : own <= 2 ? 2 : own <= 4 ? 4 : own <= 8 ? 8 : own <= 10 ? 10 : own <= 12 ? 12 : 16;
}

// Narrow (u8) distance rows: npitch bytes (a multiple of 1024), node v at
// byte v -- a level's stores are 64 consecutive bytes per (source, slice),
// lane-ordered like the u32 ones (any permutation of the lanes' addresses
// costs the store path measurably).


//   LCOL: the sliced-ELL columns are staged once in LDS as u16 (when they fit
//   beside F -- low-degree graphs such as grids), so the pull sweep issues no
//   global loads: no vmcnt wait, and a level's stores drain in the background
//   instead of stalling the next sweep's first column load.
//   Level 0 is pushed, not pulled: its frontier is the batch's own sources,
//   so each wave ORs its sources' bits into their neighbours' F entries
//   (LDS 64-bit atomics over the sources' CSR rows) where a pull would sweep
//   every column of the graph (~1/5 of a fabric batch's time, r02 stamps).
//   Links are up in both directions or neither, so CSR out-neighbours are
//   the in-neighbours the pull reads.  (Pushing later levels, whose
//   frontiers live in the owners' registers, spilled msbfs_kernel<10>.)
template <int OWN, bool LCOL, bool DB = false>
__global__ __launch_bounds__(kMsThreads) void msbfs_kernel(
    const uint32_t* __restrict__ sell_ptr, const uint32_t* __restrict__ sell_col,
    uint32_t n_col, const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const uint8_t* __restrict__ ovl, const uint32_t* __restrict__ rows_src,
    uint32_t n_rows, uint32_t bs, uint32_t N, uint32_t pitch, uint32_t npitch,
    uint32_t* __restrict__ D, uint8_t* __restrict__ Dn, uint32_t* __restrict__ maxd,
    uint32_t d_from, const uint32_t* __restrict__ smap,
    unsigned long long* __restrict__ stamps /* diagnostics, usually null */) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* F = reinterpret_cast<uint64_t*>(smem);             // [N + 1]
  uint64_t* F2 = F + (DB ? N + 1 : 0);                         // [N + 1] (DB) second frontier
  uint32_t* o_node = reinterpret_cast<uint32_t*>(F2 + N + 1);  // [64] drained batch sources
  uint32_t* o_cnt = o_node + kMsBatch;                         // [1]
  uint32_t* flag = o_cnt + 1;                                  // [3] progress flags
  uint32_t* src_l = flag + 3;                                  // [64] the batch's sources
  uint32_t* e_base = src_l + kMsBatch;                         // [64] their first CSR edge
  uint32_t* e_pre = e_base + kMsBatch;                         // [65] degree prefix sums
  uint16_t* lcol = reinterpret_cast<uint16_t*>(e_pre + kMsBatch + 1);  // [n_col] (LCOL)

  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t row0 = blockIdx.x * bs;  // bs <= 64 sources per workgroup
  // sell_col with its padding columns (spf_graph_load: 32 past the last slice)
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(sell_col), 0, (int)((n_col + 32u * kSliceW) * 4u), 0x00020000);
  const uint32_t nb = min(bs, n_rows - row0);
  const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
  // diagnostics: lane 0 of every wave of workgroup 0 logs phase clocks into
  // stamps[wave * 64 + 1 ..], the count into stamps[wave * 64]
  // (the workgroup logged: stamps[1024], SPF_STAMPS=<workgroup>)
  const bool stamp = stamps && blockIdx.x == (uint32_t)stamps[64 * 16] && lane == 0;
  unsigned long long* my_stamps = stamps + (tid >> 6) * 64;
  uint32_t n_stamp = 0;
#define MS_STAMP()                                                   \
  do {                                                               \
    if (stamp && n_stamp < 63) my_stamps[++n_stamp] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  MS_STAMP();

  for (uint32_t v = tid; v <= N; v += kMsThreads) F[v] = 0;
  if (LCOL)
    for (uint32_t t = tid; t < n_col; t += kMsThreads) lcol[t] = (uint16_t)sell_col[t];
  if (DB)
    for (uint32_t v = N + tid; v <= N; v += kMsThreads) F2[v] = 0;  // the padding target
  if (tid == 0) {
    *o_cnt = 0;
    flag[0] = flag[1] = flag[2] = 0;
  }
  __syncthreads();
  // ---- the batch's sources (wave 0): level 0, drained sources, their CSR
  // rows as one flat edge list (exclusive scan of the degrees), and their own
  // bits marked in F for the owners to pick up ----
  if (tid < 64) {
    uint32_t deg = 0;
    if (tid < nb) {
      const uint32_t src = rows_src[row0 + tid];  // sources of a batch are distinct
      src_l[tid] = src;
      if (ovl[src]) o_node[atomicAdd(o_cnt, 1u)] = src | (tid << 24);
      if (D && d_from == 0) D[(size_t)(row0 + tid) * pitch + src] = 0;  // level 0
      if (Dn) Dn[(size_t)(row0 + tid) * npitch + src] = 0;
      e_base[tid] = row_ptr[src];
      deg = row_ptr[src + 1] - e_base[tid];
      F[src] = 1ull << tid;
    }
    uint32_t total;
    const uint32_t ex = wave_excl_scan(deg, &total);
    e_pre[tid] = ex;
    if (tid == 0) e_pre[64] = total;
  }
  __syncthreads();
  const uint32_t n_osrc = *o_cnt;
  // the part of mask x a drained node v may expand: its own source bit
  auto own_bits = [&](uint32_t v, uint64_t x) {
    uint64_t own = 0;
    for (uint32_t k = 0; k < n_osrc; ++k)
      if ((o_node[k] & 0xFFFFFFu) == v) own = 1ull << (o_node[k] >> 24);
    return x & own;
  };

  // owned slices: slot i of this wave holds slice smap[wave * OWN + i] (the
  // host deals slices to waves balanced by column width; an unused slot's
  // nodes lie past N)
  const uint32_t wv = tid >> 6;
  uint32_t sv[OWN];  // first node of owned slice i (wave-uniform)
  uint64_t vis[OWN], nv[OWN];
  uint32_t drained = 0;  // bit i: owned node i is drained
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    sv[i] = __builtin_amdgcn_readfirstlane(smap[wv * OWN + i]) * kSliceW;
    const uint32_t v = sv[i] + lane;
    vis[i] = v < N ? F[v] : 0ull;  // the node's own source bit, if it is a source
    if (v < N && ovl[v]) drained |= 1u << i;
  }
  __syncthreads();  // the self marks are read
  if (tid < nb) F[src_l[tid]] = 0;
  __syncthreads();
  // ---- level 1 by push: each source's bit ORed into its neighbours' F (a
  // source expands even when drained); the batch's edges dealt over the
  // whole workgroup, their loads all independent ----
  {
    const uint32_t n_e = e_pre[64];
    for (uint32_t t = tid; t < n_e; t += kMsThreads) {
      uint32_t lo = 0, hi = nb;  // the source b with e_pre[b] <= t < e_pre[b + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (e_pre[mid] <= t) lo = mid;
        else hi = mid;
      }
      atomicOr(reinterpret_cast<unsigned long long*>(&F[col[e_base[lo] + t - e_pre[lo]]]),
               1ull << lo);
    }
  }
  __syncthreads();
  uint64_t any1 = 0;
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    const uint32_t v = sv[i] + lane;
    nv[i] = v < N ? F[v] & ~vis[i] : 0ull;  // level 1
    vis[i] |= nv[i];
    any1 |= nv[i];
  }
  __syncthreads();  // every read of the pushed F is done
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    const uint32_t v = sv[i] + lane;
    if (v < N) F[v] = ((drained >> i) & 1u) ? own_bits(v, nv[i]) : nv[i];
  }
  if (any1) flag[0] = 1;  // level 1 is not empty (flag[1] stays 0 for level 1's sweep)
  __syncthreads();
  const bool level1 = flag[0] != 0;  // read before level 1 resets flag[0]

  MS_STAMP();
  // ---- record a level: D[s][v] = L for every new (s, v) of owned slice i
  // (mask x); only the sources with a new node in the slice (wave OR) ----
  auto record = [&](int i, uint64_t x, uint32_t L) {
    // most slices have no new node at a given level: one ballot skips them
    if (__ballot(x != 0ull) == 0ull) return;
    const uint32_t nl = min(L, 254u);
    uint32_t* const DL = L >= d_from ? D : nullptr;  // u32 rows this level (uniform)
    // the wave-uniform mask lives in SGPRs: row addressing is scalar work
    const uint64_t wm = wave_or64(x);
    uint32_t mlo = __builtin_amdgcn_readfirstlane((uint32_t)wm);
    uint32_t mhi = __builtin_amdgcn_readfirstlane((uint32_t)(wm >> 32));
    const uint32_t v = sv[i] + lane;
    // Two ways to cover the (source, node) pairs of the slice: one
    // coalesced store per source (row-major; best when a source discovers
    // many nodes of the slice at once -- dense fabrics), or each lane
    // walking its own new sources (scattered stores; best when every source
    // discovers a node or two per level -- grids, rings).  Trip counts:
    // #sources vs the largest per-node count.
    const uint32_t nsrc = (uint32_t)__popcll(((uint64_t)mhi << 32) | mlo);
    const uint32_t maxpop = wave_max32((uint32_t)__popcll(x));
    if (maxpop * kMsLaneStoreRatio < nsrc) {
      uint64_t m = x;
      for (uint32_t it = 0; it < maxpop; ++it) {
        if (m) {
          const uint32_t s = __ffsll((unsigned long long)m) - 1;
          if (DL) __builtin_nontemporal_store(L, &DL[(size_t)(row0 + s) * pitch + v]);
          if (Dn) Dn[(size_t)(row0 + s) * npitch + v] = (uint8_t)nl;
          m &= m - 1;
        }
      }
      return;
    }
    for (uint64_t m = ((uint64_t)mhi << 32) | mlo; m; m &= m - 1) {
      const uint32_t s = __ffsll((unsigned long long)m) - 1;
      if ((x >> s) & 1ull) {
        if (DL) __builtin_nontemporal_store(L, &DL[(size_t)(row0 + s) * pitch + v]);
        if (Dn) Dn[(size_t)(row0 + s) * npitch + v] = (uint8_t)nl;
      }
    }
  };
  // ---- pull of owned slice i from frontier Fc: the slice's unfinished
  // nodes OR their neighbours' frontier masks; returns the new bits ----
  auto pull = [&](int i, const uint64_t* Fc) -> uint64_t {
    const uint32_t v = sv[i] + lane;
    const bool need = v < N && vis[i] != all;
    uint64_t nx = 0;
    if (__ballot(need)) {  // wave-uniform: the slice has unfinished nodes
      // the slice's column base and width: scalar loads per call (ten
      // slices' pairs held across the level loop spilled SGPRs to VGPR
      // lanes: 110 spills -> 5, fabric_full BFS 0.161 -> 0.157 ms)
      uint32_t sl = sv[i] / kSliceW;
      asm volatile("" : "+s"(sl));
      const uint32_t sbi = sell_ptr[sl];
      const uint32_t w = (sell_ptr[sl + 1] - sbi) / kSliceW;
      const uint32_t* cp = sell_col + sbi + lane;
      const uint16_t* lp = lcol + sbi + lane;
      uint64_t acc = 0;
      uint32_t j = 0;
      if constexpr (!LCOL) {
        // columns from L2: two groups of kMsUnroll loads in flight, issued
        // unconditionally (sell_col is padded past its last slice; columns
        // past w read the next slice's valid ids and are not ORed) -- a load
        // under a branch makes the join's wait count drain the group in
        // flight, one L2 round trip per group
        // buffer loads: the slice's column base in an SGPR, the lane's
        // offset in a VGPR (a 64-bit address pair per owned slice spilled)
        uint32_t ca[kMsUnroll], cb[kMsUnroll];
        auto load = [&](uint32_t j0, uint32_t (&c)[kMsUnroll]) {
#pragma unroll
          for (int u = 0; u < kMsUnroll; ++u)
            c[u] = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(lane * 4u),
                                                        (int)((sbi + (j0 + u) * kSliceW) * 4u), 0);
        };
        auto fold = [&](const uint32_t (&c)[kMsUnroll], uint32_t n) {
          uint64_t f[kMsUnroll];
#pragma unroll
          for (int u = 0; u < kMsUnroll; ++u) f[u] = Fc[c[u]];
#pragma unroll
          for (int u = 0; u < kMsUnroll; ++u)
            if ((uint32_t)u < n) acc |= f[u];
        };
        load(0, ca);
        for (; j < w; j += 2 * kMsUnroll) {
          load(j + kMsUnroll, cb);
          fold(ca, w - j);
          load(j + 2 * kMsUnroll, ca);
          if (j + kMsUnroll < w) fold(cb, w - j - kMsUnroll);
        }
        if (need) {
          nx = acc & ~vis[i];
          vis[i] |= nx;
        }
        return nx;
      }
      // LDS columns: kMsUnroll loads at a time, then the remainder in groups
      // of 4, 2, 1 (w is wave-uniform: scalar branches, no F reads wasted on
      // padding -- the LDS port is what bounds the sweep)
      for (; j + kMsUnroll <= w; j += kMsUnroll) {
        uint32_t c[kMsUnroll];
#pragma unroll
        for (int u = 0; u < kMsUnroll; ++u)
          c[u] = LCOL ? (uint32_t)lp[(j + u) * kSliceW] : cp[(j + u) * kSliceW];
#pragma unroll
        for (int u = 0; u < kMsUnroll; ++u) acc |= Fc[c[u]];
      }
#pragma unroll
      for (int g = kMsUnroll / 2; g >= 1; g >>= 1) {
        if (j + g <= w) {
          uint32_t c[kMsUnroll / 2];
#pragma unroll
          for (int u = 0; u < g; ++u)
            c[u] = LCOL ? (uint32_t)lp[(j + u) * kSliceW] : cp[(j + u) * kSliceW];
#pragma unroll
          for (int u = 0; u < g; ++u) acc |= Fc[c[u]];
          j += g;
        }
      }
      if (need) {
        nx = acc & ~vis[i];
        vis[i] |= nx;
      }
    }
    return nx;
  };
  uint32_t last = 0;  // deepest level of the batch
  if constexpr (DB) {
    // Double-buffered frontier (graphs whose two F arrays fit in LDS): a
    // slice is pulled from level L's frontier, its level L + 1 bits go
    // straight into the other buffer and its stores are issued at once --
    // one barrier per level, no per-slice state kept across it.
    // flag[L mod 3]: set during level L, read after its barrier, cleared
    // during level L + 2's predecessor (its last readers passed a barrier).
#pragma unroll
    for (int i = 0; i < OWN; ++i) record(i, nv[i], 1);
    uint64_t* Fc = F;
    uint64_t* Fn = F2;
    for (uint32_t L = 1; level1; ++L) {
      uint64_t any = 0;
#pragma unroll
      for (int i = 0; i < OWN; ++i) {
        const uint64_t nx = pull(i, Fc);
        const uint32_t v = sv[i] + lane;
        if (v < N) Fn[v] = ((drained >> i) & 1u) ? own_bits(v, nx) : nx;
        any |= nx;
        record(i, nx, L + 1);
      }
      if (any) flag[L % 3] = 1;
      if (tid == 0) flag[(L + 1) % 3] = 0;
      MS_STAMP();
      __syncthreads();
      MS_STAMP();
      if (!flag[L % 3]) {
        last = L;
        break;
      }
      uint64_t* t = Fc;
      Fc = Fn;
      Fn = t;
    }
  } else {
    for (uint32_t L = 1; level1; ++L) {
#pragma unroll
      for (int i = 0; i < OWN; ++i) record(i, nv[i], L);
      MS_STAMP();
      uint64_t any = 0;
      // ---- pull sweep for level L+1 ----
#pragma unroll
      for (int i = 0; i < OWN; ++i) {
        nv[i] = pull(i, F);
        any |= nv[i];
      }
      MS_STAMP();
      __syncthreads();  // every read of F for this level is done
      MS_STAMP();
#pragma unroll
      for (int i = 0; i < OWN; ++i) {
        const uint32_t v = sv[i] + lane;
        if (v < N) F[v] = ((drained >> i) & 1u) ? own_bits(v, nv[i]) : nv[i];  // drained: own source only
      }
      if (any) flag[L & 1] = 1;
      if (tid == 0) flag[(L + 1) & 1] = 0;
      __syncthreads();
      if (!flag[L & 1]) {
        last = L;
        break;
      }
    }
  }
  // the plan's deepest level: how many bit planes the sliced rows need
  if (maxd && tid == 0) atomicMax(maxd, last);
  MS_STAMP();
  // ---- unreachable (s, v) pairs and row padding ----
  uint64_t miss = 0;
#pragma unroll
  for (int i = 0; i < OWN; ++i)
    if (sv[i] + lane < N) miss |= ~vis[i] & all;
  for (uint64_t m = wave_or64(miss); m; m &= m - 1) {
    const uint32_t s = __ffsll((unsigned long long)m) - 1;
    uint32_t* drow = D + (size_t)(row0 + s) * pitch;
    uint8_t* nrow = Dn + (size_t)(row0 + s) * npitch;
#pragma unroll
    for (int i = 0; i < OWN; ++i) {
      const uint32_t v = sv[i] + lane;
      if (v < N && !((vis[i] >> s) & 1ull)) {
        if (D && d_from == 0) __builtin_nontemporal_store(kInf, &drow[v]);
        if (Dn) nrow[v] = 0xFF;
      }
    }
  }
  {  // row padding past N: one flat (row, entry) index over the workgroup
    const uint32_t pw = npitch - N, tot = nb * pw;
    for (uint32_t t = tid; t < tot; t += kMsThreads) {
      const uint32_t s = t / pw, v = N + t % pw;
      if (D && d_from == 0 && v < pitch) __builtin_nontemporal_store(kInf, &D[(size_t)(row0 + s) * pitch + v]);
      if (Dn) Dn[(size_t)(row0 + s) * npitch + v] = 0xFF;
    }
  }
  MS_STAMP();
  if (stamp) my_stamps[0] = n_stamp;
#undef MS_STAMP
}

// ---------------------------------------------------------------------------
//  1c. multi-source BFS with register-resident distances (bit planes)
// ---------------------------------------------------------------------------
// msbfs_kernel writes every (source, node) distance at the level it is found:
// on a large-diameter graph (grid100: 198 levels) a 64-node slice of a source
// row is found over dozens of levels, so its lines leave L2 partially written
// again and again (PMC: 3.1 GB written for a 0.4 GB result).  This variant
// keeps the distances on chip and writes each row once, coalesced:
//   * <= 32 sources per workgroup, u32 masks (F in LDS is 4 B/node);
//   * for every owned node, 8 bit planes: bit s of plane b = bit b of
//     d(source s, node) -- a level L ORs the new mask into the planes of L's
//     set bits (uniform branches, popcount(L) ORs per node);
//   * at the end, per source, lane v assembles its distance from the planes
//     and the wave stores 64 consecutive entries of the row (and of the u8
//     copy when the next-hop pass reads narrow rows).
// Planes hold 255 levels (a window); a search deeper than that flushes the
// window, marks the entries found so far and starts the next window.
// Register budget: 8 planes + visited + new per owned node = 10 VGPRs, so
// OWN <= 10 (N <= 10240); the host picks msbfs_kernel otherwise.
constexpr uint32_t kPlBatch = 32;
constexpr int kPlanes = 8;
constexpr uint32_t kPlWindow = (1u << kPlanes) - 1;  // relative levels 0..254, 255 = marker
//   Columns: SELL-64 packed four u16 byte offsets (4 * id) per lane (uint2), every live slice
//   at least one group wide (padding id N, F[N] == 0), staged in LDS when
//   they fit.  Group 0 of all owned slices is straight-line code (a grid's
//   whole sweep: one 8-byte column load and four F loads per node); lanes
//   whose node is finished read F[N] (a broadcast).
//   F is double-buffered: one barrier per level.

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int OWN, bool LCOL>
__global__ __launch_bounds__(kMsThreads) void msbfs_planes_kernel(
    const uint32_t* __restrict__ sell4_ptr, const uint2* __restrict__ sell4, uint32_t n4,
    const uint8_t* __restrict__ ovl, const uint32_t* __restrict__ rows_src, uint32_t n_rows,
    uint32_t bs, uint32_t N, uint32_t pitch, uint32_t npitch, uint32_t* __restrict__ D,
    uint8_t* __restrict__ Dn, const uint32_t* __restrict__ order /* slot -> row, or null */) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint2* lcol = reinterpret_cast<uint2*>(smem);                   // [n4] (LCOL)
  // F0/F1: one word per owned node slot (OWN * 1024 >= N + 1); slots past
  // N keep F = 0 (their vis is `all`), so every slot is written unconditionally
  constexpr uint32_t kF = OWN * kMsThreads;
  uint32_t* F0 = reinterpret_cast<uint32_t*>(smem + (LCOL ? 8ull * n4 : 0));  // [kF]
  uint32_t* F1 = F0 + kF;                                         // [kF]
  uint32_t* o_node = F1 + kF;                                     // [32] drained batch sources
  uint32_t* o_cnt = o_node + kPlBatch;                            // [1]
  uint32_t* flag = o_cnt + 1;                                     // [3] progress, L mod 3

  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t row0 = blockIdx.x * bs;  // bs <= 32
  const uint32_t nb = min(bs, n_rows - row0);
  const uint32_t all = nb == 32 ? ~0u : ((1u << nb) - 1u);
  // column entries from L2 by buffer loads: the slice's entry base in an
  // SGPR, the lane's offset in a VGPR (per-slice 64-bit addresses spilled)
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint2*>(sell4), 0, (int)(n4 * 8u), 0x00020000);
  auto col4 = [&](uint32_t entry, uint32_t ln) -> uint2 {
    const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(crs, (int)(ln * 8u), (int)(entry * 8u), 0);
    return make_uint2(x.x, x.y);
  };

  for (uint32_t v = tid; v < kF; v += kMsThreads) F0[v] = F1[v] = 0;
  if (LCOL)
    for (uint32_t t = tid; t < n4; t += kMsThreads) lcol[t] = sell4[t];
  if (tid == 0) {
    *o_cnt = 0;
    flag[0] = flag[1] = flag[2] = 0;
  }
  __syncthreads();
  if (tid < nb) {
    const uint32_t src = rows_src[order ? order[row0 + tid] : row0 + tid];
    F0[src] = 1u << tid;  // sources of a batch are distinct
    if (ovl[src]) o_node[atomicAdd(o_cnt, 1u)] = src | (tid << 24);
  }
  __syncthreads();
  const uint32_t n_osrc = *o_cnt;

  uint32_t vis[OWN], P[OWN][kPlanes];
  uint32_t dslices = 0;  // bit i: owned slice i holds a drained node (wave-uniform)
  uint32_t dlane = 0;    // bit i: this lane's node of slot i is drained (no ovl loads per level)
  uint32_t sb[OWN], sg[OWN];  // owned slice i: first packed entry, groups (wave-uniform)
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    const uint32_t v = tid + i * kMsThreads;
    vis[i] = v < N ? F0[v] : all;
#pragma unroll
    for (int b = 0; b < kPlanes; ++b) P[i][b] = 0u;
    const bool dr = v < N && ovl[v];
    dlane |= (uint32_t)dr << i;
    if (__ballot(dr)) dslices |= 1u << i;
    const uint32_t slice = (tid - lane + i * kMsThreads) / kSliceW;
    const bool live = slice * kSliceW < N;
    const uint32_t b = live ? sell4_ptr[slice] : 0u;
    const uint32_t e = live ? sell4_ptr[slice + 1] : kSliceW;
    sb[i] = __builtin_amdgcn_readfirstlane(b);
    sg[i] = __builtin_amdgcn_readfirstlane((e - b) / kSliceW);
  }

  uint32_t base = 0;  // level of relative value 0 in the current window
  for (uint32_t L = 1;; ++L) {
    const uint32_t* Fc = (L & 1) ? F0 : F1;  // frontier of level L - 1
    uint32_t* Fn = (L & 1) ? F1 : F0;        // frontier of level L
    // opaque lane id, recomputed per level: hoisting the owned slices'
    // addresses out of the level loop would spill
    uint32_t ln = tid;
    asm volatile("" : "+v"(ln));
    ln &= 63u;
    const uint32_t rel = L - base;  // relative level recorded in the planes
    uint32_t any = 0;
    const unsigned char* Fb = reinterpret_cast<const unsigned char*>(Fc);
#define PL_F(off) (*reinterpret_cast<const uint32_t*>(Fb + (off)))
    uint2 qn = LCOL ? lcol[sb[0] + ln] : col4(sb[0], ln);
#pragma unroll
    for (int i = 0; i < OWN; ++i) {
      const uint32_t v = tid + i * kMsThreads;
      uint32_t nx = 0;
      const uint2 q = qn;
      // group 0 of slice i + 1 is loaded while slice i waits for its F reads
      if (i + 1 < OWN) qn = LCOL ? lcol[sb[i + 1] + ln] : col4(sb[i + 1], ln);
      // a uniform branch per slice: skips finished slices and keeps the
      // scheduler from hoisting ten slices' loads (register pressure).
      // No per-lane masking: a finished node gets nx = 0 from ~vis, a slot
      // past N has only padding columns (F[N] == 0).
      if (__ballot(vis[i] != all)) {
        // all four reads in flight before the first use (one LDS round trip)
        uint32_t f0 = PL_F(q.x & 0xFFFFu), f1 = PL_F(q.x >> 16), f2 = PL_F(q.y & 0xFFFFu),
                 f3 = PL_F(q.y >> 16);
        asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
        uint32_t acc = f0 | f1 | f2 | f3;
#pragma unroll 1
        for (uint32_t g = 1; g < sg[i]; ++g) {  // wider slices: the remaining groups
          const uint2 r = LCOL ? lcol[sb[i] + g * kSliceW + ln] : col4(sb[i] + g * kSliceW, ln);
          acc |= PL_F(r.x & 0xFFFFu) | PL_F(r.x >> 16) | PL_F(r.y & 0xFFFFu) | PL_F(r.y >> 16);
        }
        nx = acc & ~vis[i];
        vis[i] |= nx;
        any |= nx;
#pragma unroll
        for (int b = 0; b < kPlanes; ++b)
          if ((rel >> b) & 1u) P[i][b] |= nx;
      }
      uint32_t f = nx;
      if ((dslices >> i) & 1u) {  // the slice holds a drained node (uniform test)
        if ((dlane >> i) & 1u) {  // drained: expands only as its own source
          uint32_t own = 0;
          for (uint32_t k = 0; k < n_osrc; ++k)
            if ((o_node[k] & 0xFFFFFFu) == v) own = 1u << (o_node[k] >> 24);
          f &= own;
        }
      }
      Fn[v] = f;
    }
#undef PL_F
    // flag[L mod 3]: set during level L, read after its barrier; cleared
    // during level L - 2 (its last reader finished before barrier L - 1)
    if (any) flag[L % 3] = 1;
    if (tid == 0) flag[(L + 1) % 3] = 0;
    __syncthreads();
    const bool done = !flag[L % 3];
    if (done || rel == kPlWindow - 1) {
      // Flush the window.  The first one writes every entry of the batch's
      // rows (unreached = kInf, row padding); a later one (searches deeper
      // than 254 levels) only the entries found in it -- entries of earlier
      // windows carry the marker value kPlWindow in their planes.
      const bool first = base == 0;
      for (uint32_t s = 0; s < nb; ++s) {
        const uint32_t row = order ? order[row0 + s] : row0 + s;
        uint32_t* drow = D + (size_t)row * pitch;
        uint8_t* nrow = Dn ? Dn + (size_t)row * npitch : nullptr;
#pragma unroll
        for (int i = 0; i < OWN; ++i) {
          const uint32_t v = tid + i * kMsThreads;
          uint32_t r = 0;
#pragma unroll
          for (int b = 0; b < kPlanes; ++b) r |= ((P[i][b] >> s) & 1u) << b;
          const bool seen = v < N && ((vis[i] >> s) & 1u);
          const uint32_t d = seen ? base + r : kInf;
          if (first || (seen && r != kPlWindow)) {
            if (v < pitch) __builtin_nontemporal_store(d, &drow[v]);
            if (nrow && v < npitch) nrow[v] = d == kInf ? 0xFFu : (uint8_t)min(d, 254u);
          }
        }
      }
      if (done) break;
#pragma unroll
      for (int i = 0; i < OWN; ++i)
#pragma unroll
        for (int b = 0; b < kPlanes; ++b) P[i][b] |= vis[i];
      base += kPlWindow;
    }
  }
}

// ---------------------------------------------------------------------------
//  2. next-hop (ECMP) pass
// ---------------------------------------------------------------------------
// Output: per source, one destination bitmap per distinct up neighbour x
// (ascending id): bit v of bitmap j <=> neighbour j is in nh_s(v).  Each wave
// owns a 1024-destination chunk and stores, per neighbour, 32 consecutive u32
// words.
//   NARROW: distances from the u8 copy: lane l loads destinations
//           cbase + 16l .. +15 of the neighbour's row (16 bytes), compares
//           them with the precomputed targets d_s(v) - 1 into a 16-bit mask,
//           and even lanes merge their odd neighbour's half into one word; a
//           wave whose source row holds a saturated entry (>= 254) decides on
//           the exact u32 rows instead.
//   exact:  u32 rows, one coalesced dword load per 64 destinations.

constexpr int kEcmpUnroll = 4;         // neighbour rows per group (two groups in flight)
constexpr uint32_t kEcmpChunk = 1024;  // destinations per wave
constexpr uint32_t kEcmpWaves = kEcmpThreads / 64;
constexpr uint32_t kEcmpRunsPerXcd = 64;  // source runs dealt to each XCD

// Zero-byte flags of x at bit 7 of each byte (exact: no carries cross bytes).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// Byte-equality mask of a lane's 16-byte narrow slice against its packed
// targets: bit n = destination cbase + 16*lane + n.  Dword k byte b is
// destination 4k + b; shifting dword k's zero-byte flags right by 3 - k puts
// it at bit 8b + 4 + k (high nibbles), a shift-or and a byte permute pack the
// nibbles to bit 4b + k, and two delta swaps transpose that 4x4 bit matrix
// to bit 4k + b.
__device__ __forceinline__ uint32_t eq_mask16(const uint4& a, const uint4& t) {
  const uint32_t z = (zero_bytes(a.x ^ t.x) >> 3) | (zero_bytes(a.y ^ t.y) >> 2) |
                     (zero_bytes(a.z ^ t.z) >> 1) | zero_bytes(a.w ^ t.w);
  uint32_t x = __builtin_amdgcn_perm(0u, z | (z << 4), 0x0c0c0301u);
  uint32_t d = (x ^ (x >> 3)) & 0x0A0Au;
  x ^= d ^ (d << 3);
  d = (x ^ (x >> 6)) & 0x00CCu;
  return x ^ d ^ (d << 6);
}

// Weighted narrow match without per-neighbour targets: bit n (eq_mask16's
// order) set iff a_n + w == s_n for the neighbour's byte a_n and the
// source's byte s_n, bytes split into 16-bit halves so the add cannot carry
// (SWAR: ~12 ops per 4 destinations where deriving targets d_s - w per
// neighbour cost ~100 per 16).  No false matches: a = 255 (unreachable,
// drained neighbour's dead row) or 254 (saturated) sums past every
// unsaturated source byte; s = 255 needs a finite a only through a drained
// x, whose row is the dead row; s = 0 (the source) needs w = 0.  w >= 254
// matches nothing in the fast path (the source bytes stay below 254).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t weighted_mask16(const uint4& a4, const uint32_t (&sl)[4],
                                                    const uint32_t (&sh)[4], uint32_t w) {
  if (w >= 0xFEu) return 0u;
  const u16x2 W2 = {(unsigned short)w, (unsigned short)w};
  const u16x2 one = {1, 1};
  const uint32_t a[4] = {a4.x, a4.y, a4.z, a4.w};
  // per word q: bytes 0, 2 and bytes 1, 3 as 16-bit halves (v_perm), a + w
  // and the xor with the source's halves packed (v_pk_add_u16), zero halves
  // -> 1 by a saturating 1 - x (v_pk_sub_u16 clamp); the four result bits
  // land at 4q, 4q + 1 (bytes 0, 1) and 16 + 4q, 17 + 4q (bytes 2, 3)
  uint32_t T = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const u16x2 lo = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, a[q], 0x0c020c00u));
    const u16x2 hi = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, a[q], 0x0c030c01u));
    const uint32_t xl = __builtin_bit_cast(uint32_t, (u16x2)(lo + W2)) ^ sl[q];
    const uint32_t xh = __builtin_bit_cast(uint32_t, (u16x2)(hi + W2)) ^ sh[q];
    const uint32_t zl = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(one, __builtin_bit_cast(u16x2, xl)));
    const uint32_t zh = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(one, __builtin_bit_cast(u16x2, xh)));
    T |= (zl | (zh << 1)) << (4 * q);
  }
  return (T | (T >> 14)) & 0xFFFFu;
}

// nb_row[nb_row_off[i] + j]: byte offset in Dn (row * npitch) of the narrow
// row of the request's source i's neighbour j (ascending id) -- the D row
// itself for plans without narrow rows -- or `dead` if it is drained: the
// offset of an all-0xFF row after the plan's narrow rows (kInf without them).
// Each source's list starts 16-byte aligned and is padded with `dead` to
// roundup(k, 8) + 8 entries (the pipelined loads run one group ahead).  nb_drained[i] counts the drained neighbours.
// Every per-neighbour quantity is wave-uniform and read with scalar loads:
// no LDS staging, no workgroup barriers -- a wave is independent.
template <bool NARROW>
__global__ __launch_bounds__(kEcmpThreads) void ecmp_kernel(
    const uint8_t* __restrict__ Dn, uint32_t npitch, const uint32_t* __restrict__ D,
    uint32_t pitch, uint32_t N, const uint32_t* __restrict__ req_src,
    const uint32_t* __restrict__ row_of, const uint32_t* __restrict__ nb_ptr,
    const uint32_t* __restrict__ nb_id, const uint32_t* __restrict__ nb_w,
    const uint32_t* __restrict__ nb_row, const uint32_t* __restrict__ nb_row_off,
    const uint32_t* __restrict__ nb_drained, uint32_t dead, uint32_t hop, uint32_t weighted,
    const uint64_t* __restrict__ nh_off, uint32_t* __restrict__ nh, uint32_t chunks,
    const uint32_t* __restrict__ slot_src) {
  // Block b runs on XCD b % 8.  slot_src (spf_plan_create) lists each XCD's
  // sources: runs of consecutive request sources (the racks of one pod, the
  // spines of one plane -- the same neighbour rows, shared in that XCD's L2)
  // dealt to the XCDs by work; a source's chunks are consecutive blocks.
  // (Long-lived blocks walking the list were slower at every size tried,
  // profiles/r02_v10_ab_ecmp_blocks.txt.)
  const uint32_t grp = blockIdx.x & 7, pos = blockIdx.x >> 3;
  const uint32_t i = slot_src[(pos / chunks) * 8 + grp];
  const uint32_t c = pos % chunks;
  if (i == kInf) return;
  const uint32_t s = req_src[i];
  const uint32_t nb0 = nb_ptr[s], k = nb_ptr[s + 1] - nb0;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t cbase = (c * kEcmpWaves + (threadIdx.x >> 6)) * kEcmpChunk;
  if (k == 0 || cbase >= N) return;  // whole wave: no barriers below
  const uint32_t srow = row_of[s];
  const uint32_t wpm = pitch / 32;  // u32 words per bitmap
  const uint32_t* offs = nb_row + nb_row_off[i];
  uint32_t* out_w = nh + nh_off[i] + cbase / 32;  // word base of bitmap 0

  // NARROW: the u8 value a neighbour must hold at this lane's 16 slice
  // bytes, packed like the row; 0xFE = none (never held by a non-drained
  // neighbour where the source row is not saturated: d_x(s) = w(x, s) < 0xFE,
  // and a node s cannot reach no neighbour reaches either)
  uint4 tg = make_uint4(0xFEFEFEFEu, 0xFEFEFEFEu, 0xFEFEFEFEu, 0xFEFEFEFEu);
  uint4 raw = tg;  // the source's 16 bytes (weighted matches derive targets per neighbour)
  bool exact = !NARROW;
  if (NARROW) {
    raw = *reinterpret_cast<const uint4*>(Dn + (size_t)srow * npitch + cbase + lane * 16);
    const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
    uint32_t t[4];
    bool sat = false;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      uint32_t o = 0;
#pragma unroll
      for (int bq = 0; bq < 4; ++bq) {
        const uint32_t x = (rw[w] >> (8 * bq)) & 0xFFu;
        sat |= x == 0xFEu;
        o |= ((x == 0u || x >= 0xFEu) ? 0xFEu : x - 1u) << (8 * bq);  // d_x = d_s - 1
      }
      t[w] = o;
    }
    tg = make_uint4(t[0], t[1], t[2], t[3]);
    exact = __ballot(sat) != 0;
  }

  if (!exact) {
    // fast path: lane l stores the 16-bit slice of destinations
    // cbase + 16l .. +15; two groups of kEcmpUnroll neighbour rows in flight
    // (ping-pong); a drained neighbour's row reads as "unreachable" (0xFF
    // never equals a target) and its single possible bit is patched below
    const bool st = cbase / 16 + lane < pitch / 16;
    const uint32_t loff = lane * 16;
    const uint8_t* dn_c = Dn + cbase;
    // weighted: the source's bytes as 16-bit halves (weighted_mask16)
    uint32_t ssl[4], ssh[4];
    {
      const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ssl[q] = rw[q] & 0x00FF00FFu;
        ssh[q] = (rw[q] >> 8) & 0x00FF00FFu;
      }
    }
    // unconditional loads (drained neighbours and list padding point at the
    // all-0xFF dead row), so the waits count exactly: group B's loads stay in
    // flight while group A is matched
    auto load_group = [&](uint32_t j0, uint4* r) {
      const uint4 o4 = *reinterpret_cast<const uint4*>(offs + j0);  // one scalar load
      const uint32_t o[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
      for (int u = 0; u < kEcmpUnroll; ++u) r[u] = *reinterpret_cast<const uint4*>(dn_c + o[u] + loff);
    };
    auto match_group = [&](uint32_t j0, const uint4* r) {
#pragma unroll
      for (int u = 0; u < kEcmpUnroll; ++u) {
        if (j0 + u >= k) break;
        uint32_t m;
        if (weighted) {  // wave-uniform: d_x + w(s, x) == d_s, byte-wise
          m = weighted_mask16(r[u], ssl, ssh, nb_w[nb0 + j0 + u]);
        } else {
          m = eq_mask16(r[u], tg);
        }
        uint16_t* o = reinterpret_cast<uint16_t*>(out_w + (size_t)(j0 + u) * wpm);
        if (st) __builtin_nontemporal_store((uint16_t)m, &o[lane]);
      }
    };
    uint4 ra[kEcmpUnroll], rb[kEcmpUnroll];
    load_group(0, ra);
    for (uint32_t j0 = 0; j0 < k; j0 += 2 * kEcmpUnroll) {
      load_group(j0 + kEcmpUnroll, rb);
      match_group(j0, ra);
      load_group(j0 + 2 * kEcmpUnroll, ra);
      match_group(j0 + kEcmpUnroll, rb);
    }
  } else {
    // exact u32 rows ("wide"): lane l holds the source's distances of
    // destinations cbase + 16l .. +15 in registers and, per neighbour, compares
    // four 16-byte loads of the neighbour's row: bit k set iff
    // d_x(v) + w(s, x) == d_s(v) (d_x finite; then the sum stays below kInf).
    // Same 16-bit lane stores as the narrow path.
    const bool st = cbase / 16 + lane < pitch / 16;
    uint32_t b[16];
    {
      const uint4* Ds = reinterpret_cast<const uint4*>(D + (size_t)srow * pitch + cbase) + lane * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 t = st ? Ds[q] : make_uint4(kInf, kInf, kInf, kInf);
        b[4 * q] = t.x;
        b[4 * q + 1] = t.y;
        b[4 * q + 2] = t.z;
        b[4 * q + 3] = t.w;
      }
    }
    for (uint32_t j = 0; j < k; ++j) {
      const uint32_t oj = offs[j], wj = hop ? 1u : nb_w[nb0 + j];
      uint32_t m = 0;
      if (oj != dead && st) {
        const uint32_t rj = NARROW ? oj / npitch : oj;
        const uint4* Dx = reinterpret_cast<const uint4*>(D + (size_t)rj * pitch + cbase) + lane * 4;
        uint4 t[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = Dx[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t a[4] = {t[q].x, t[q].y, t[q].z, t[q].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            m |= (uint32_t)(a[e] != kInf && a[e] + wj == b[4 * q + e]) << (4 * q + e);
        }
      }
      if (st) __builtin_nontemporal_store((uint16_t)m, &reinterpret_cast<uint16_t*>(out_w + (size_t)j * wpm)[lane]);
    }
  }
  // drained neighbour x: its bitmap is empty except, possibly, x itself --
  // reached directly over the link when d_s(x) == w(s, x)
  if (nb_drained[i]) {
    for (uint32_t j = 0; j < k; ++j) {
      if (offs[j] != dead) continue;
      const uint32_t x = nb_id[nb0 + j];
      if (x < cbase || x >= cbase + kEcmpChunk) continue;
      const uint32_t wj = hop ? 1u : nb_w[nb0 + j];
      if (lane == (x - cbase) / 32 && D[(size_t)srow * pitch + x] == wj)
        out_w[(size_t)j * wpm + lane] = 1u << (x & 31);
    }
  }
}

// ---------------------------------------------------------------------------
//  2b. next-hop pass over bit-sliced rows (msbfs_kernel plans)
// ---------------------------------------------------------------------------
// A row's distances as P bit planes: word w of plane b holds bit b of the
// distances of nodes 32w .. 32w + 31 (bit t = node 32w + t); all-ones =
// unreachable.  P = the bits of maxd + 1 (maxd = the plan's deepest BFS
// level, from msbfs_kernel), so every finite distance stays below the
// all-ones code: a fabric (4-5 levels) needs 3 planes, 3/8 of the u8 row.
// With unit metrics (w(s, x) = 1) the test of 32 destinations against one
// neighbour row is OR_b (x_b ^ t_b) == 0 with t = d_s - 1, decremented
// bit-sliced once per source word: ~2 bit operations per plane and
// neighbour word where the byte compare of narrow rows spends ~30 per 16
// destinations, and the result is already the output word (bit v of word
// v / 32 of bitmap j).  When maxd reaches the u8 copy's saturation (254)
// the planes stay unwritten and the pass decides on the u32 rows.
constexpr uint32_t kSlChunk = 2048;  // destinations per pass of a wave: one word per lane
constexpr uint32_t kSlSlots = 8;     // plane slots per word of a sliced row
constexpr uint32_t kSlSat = 254;     // maxd at which the u8 copy saturates

// Sliced row r starts at S + r * kSlSlots * wpm; word w's P planes sit at
// w * P .. w * P + P - 1, so a lane's planes are one P-dword load and a
// wave's 64 loads cover 64 * P consecutive dwords.

// u8 narrow rows -> bit-sliced rows; one thread per (row, word): two 16-byte
// loads, P words stored.  With D (expand plans, SPF_EXPAND=1, whose BFS
// stores only the u8 rows) the same thread also writes the row's u32
// distances of its 32 nodes:
// byte b < 254 is the distance, 255 unreachable (kInf, also the row padding),
// and 254 -- saturated, level >= 254 -- keeps the exact value the BFS wrote
// into D for those levels only.
__global__ __launch_bounds__(256) void slice_rows_kernel(const uint8_t* __restrict__ Dn,
                                                         uint32_t npitch, uint32_t rows, uint32_t wpm,
                                                         const uint32_t* __restrict__ maxd,
                                                         uint32_t* __restrict__ S,
                                                         uint32_t* __restrict__ D, uint32_t pitch) {
  const uint32_t md = *maxd;
  const bool planes = md < kSlSat;
  if (!planes && !D) return;
  const uint32_t P = 32u - __clz(md + 1u);
  const uint64_t total = (uint64_t)rows * wpm;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = (uint32_t)(t / wpm), w = (uint32_t)(t % wpm);
    const uint4* in = reinterpret_cast<const uint4*>(Dn + (size_t)r * npitch + 32ull * w);
    const uint4 a = in[0], b = in[1];
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if (planes) {
      uint32_t* out = S + (size_t)r * kSlSlots * wpm + (size_t)w * P;
      for (uint32_t pl = 0; pl < P; ++pl) {
        uint32_t word = 0;
        // bit pl of bytes 4q .. 4q + 3 -> bits 4q .. 4q + 3 (the multiply moves
        // byte i's bit to bit 24 + i; no cross term lands in bits 24..31)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          word |= ((((d[q] >> pl) & 0x01010101u) * 0x01020408u) >> 24) << (4 * q);
        out[pl] = word;
      }
    }
    if (D) {
      uint4* o = reinterpret_cast<uint4*>(D + (size_t)r * pitch + 32ull * w);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t y = (d[q] >> (8 * k)) & 0xFFu;
          x[k] = y == 0xFFu ? kInf : y;
        }
        // saturated bytes (254) keep the BFS's exact u32 (rare: deep graphs)
        const uint32_t z = d[q] ^ 0xFEFEFEFEu;  // a zero byte where d[q] holds 254
        if (__builtin_expect(((z - 0x01010101u) & ~z & 0x80808080u) != 0, 0)) {
          const uint4 old = o[q];
          const uint32_t ov[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (((d[q] >> (8 * k)) & 0xFFu) == 0xFEu) x[k] = ov[k];
        }
        o[q] = make_uint4(x[0], x[1], x[2], x[3]);
      }
    }
  }
}

template <int P>
struct Planes {
  uint32_t v[P];
};

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// N consecutive dwords by buffer loads: wave-uniform byte offset in soff (an
// SGPR), the lane's in voff -- no 64-bit vector addresses
template <int N>
__device__ __forceinline__ void bload(uint32_t* d, __amdgpu_buffer_rsrc_t r, uint32_t voff,
                                      uint32_t soff) {
  if constexpr (N >= 4) {
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
    d[0] = a.x, d[1] = a.y, d[2] = a.z, d[3] = a.w;
    if constexpr (N > 4) bload<N - 4>(d + 4, r, voff + 16, soff);
  } else if constexpr (N == 3) {
    const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(r, (int)voff, (int)soff, 0);
    d[0] = a.x, d[1] = a.y, d[2] = a.z;
  } else if constexpr (N == 2) {
    const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
    d[0] = a.x, d[1] = a.y;
  } else {
    d[0] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0);
  }
}

// The sliced match of one 64-word chunk: lane = output word w.  Loads are
// unconditional (rows are padded past the last lane's word), stores
// predicated on `live`.  Two groups of U neighbour rows in flight, one
// P-dword load per row (U * P <= 16 keeps the registers low).
//   rs: the sliced rows (S); ro: the source's bitmaps (nh + nh_off[i]).
//   offs/k: the unit's neighbour range (its row offsets, its length); jb:
//   the range's first neighbour index (the bitmap the first result goes to).
#ifndef SPF_SL_STORE_AUX
#define SPF_SL_STORE_AUX 2
#endif
// bitmap store cache policy: 2 = nt (streaming: the bitmaps are outputs,
// never re-read by the pass; fabric_full next hops 0.102 -> 0.079 ms,
// gpurun_out/r03_nt); 0 = default (build-time A/B)
constexpr int kSlStoreAux = SPF_SL_STORE_AUX;
//   WEIGHTED (weighted plans, wts = the unit's neighbour metrics): the
//   test is d_x + w(s, x) == d_s, the sum formed bit-sliced with w a
//   wave-uniform constant (sum_b = a_b ^ c ^ w_b, carry = a_b c | (a_b ^ c)
//   w_b) -- ~6 bit operations per plane and 32 destinations where the byte
//   rows spend ~65 per 16.  A carry out of the top plane (the sum passes the
//   all-ones code: a drained neighbour's dead row, an unreachable node, or a
//   metric past the planes) matches nothing; an unreachable d_s (all ones)
//   cannot equal a finite d_x + w (d_x finite makes d_s finite).
template <int P, bool WEIGHTED = false, int U = (P <= 4 ? 4 : 2)>
__device__ __forceinline__ void sliced_pass(__amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t ro,
                                            uint32_t wpm, uint32_t srow,
                                            const uint32_t* __restrict__ offs, uint32_t k,
                                            uint32_t jb, uint32_t w, bool live,
                                            const uint32_t* __restrict__ wts = nullptr) {
  const uint32_t wpb = w * P * 4;  // the lane's plane bytes inside any row
  Planes<P> sv;
  bload<P>(sv.v, rs, wpb, srow * kSlSlots * wpm * 4);
  uint32_t t[P];
  uint32_t ones = ~0u, zeros = ~0u, borrow = ~0u;
#pragma unroll
  for (int b = 0; b < P; ++b) {
    const uint32_t x = sv.v[b];
    ones &= x;
    zeros &= ~x;
    t[b] = WEIGHTED ? x : x ^ borrow;  // unit metrics: t = d_s - 1
    borrow &= ~x;
  }
  // the source itself (d = 0) and unreachable destinations take no next hop;
  // elsewhere t is finite and never the all-ones code of a drained (dead) row
  const uint32_t valid = ~(ones | zeros);
  auto load_group = [&](uint32_t j0, Planes<P> (&r)[U]) {
    uint32_t o[U];  // one scalar load of U row offsets
    if constexpr (U == 4) {
      const uint4 o4 = *reinterpret_cast<const uint4*>(offs + j0);
      o[0] = o4.x, o[1] = o4.y, o[2] = o4.z, o[3] = o4.w;
    } else {
      const uint2 o2 = *reinterpret_cast<const uint2*>(offs + j0);
      o[0] = o2.x, o[1] = o2.y;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) bload<P>(r[u].v, rs, wpb, o[u] * 4);
  };
  auto match_group = [&](uint32_t j0, const Planes<P> (&r)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (j0 + u >= k) break;
      uint32_t diff = 0;
      if constexpr (WEIGHTED) {
        const uint32_t wj = wts[j0 + u];  // wave-uniform: a scalar load
        if (wj >> P) {
          diff = ~0u;  // d_x + w past the planes: no finite d_s there
        } else {
          uint32_t c = 0;
#pragma unroll
          for (int b = 0; b < P; ++b) {
            const uint32_t a = r[u].v[b], wb = 0u - ((wj >> b) & 1u), ac = a ^ c;
            diff |= ac ^ wb ^ t[b];
            c = (a & c) | (ac & wb);
          }
          diff |= c;
        }
      } else {
#pragma unroll
        for (int b = 0; b < P; ++b) diff |= r[u].v[b] ^ t[b];
      }
      if (live)
        __builtin_amdgcn_raw_buffer_store_b32(~diff & valid, ro, (int)(w * 4),
                                              (int)((jb + j0 + u) * wpm * 4), kSlStoreAux);
    }
  };
  Planes<P> ra[U], rb[U];
  load_group(0, ra);
  for (uint32_t j0 = 0; j0 < k; j0 += 2 * U) {
    load_group(j0 + U, rb);
    match_group(j0, ra);
    load_group(j0 + 2 * U, ra);
    match_group(j0 + U, rb);
  }
}

// Grouped match (sources with identical neighbour lists: a pod's rack
// switches, a plane's spines): the group's source planes of one 64-word chunk
// stay in registers and every neighbour row is loaded once for all of them
// (the per-source pass loads it once per source -- the next-hop pass is
// bound by those L2 reads).  gs <= kSlGroup sources; lane = output word w.
constexpr uint32_t kSlGroup = 8;
constexpr uint32_t kSlSeg = 4;  // neighbour positions per grouping segment (one uint4 of row offsets)
template <int P>
__device__ __forceinline__ void grouped_pass(__amdgpu_buffer_rsrc_t rs, uint32_t* __restrict__ nh,
                                             const uint64_t* __restrict__ nh_off,
                                             const uint32_t* __restrict__ row_of,
                                             const uint32_t* __restrict__ req_src,
                                             const uint32_t* __restrict__ gm, uint32_t gs,
                                             uint32_t wpm, const uint32_t* __restrict__ offs,
                                             uint32_t j0, uint32_t j1, uint32_t w, bool live) {
  const uint32_t wpb = w * P * 4;
  uint32_t t[kSlGroup][P], valid[kSlGroup];
  uint32_t* out[kSlGroup];
#pragma unroll
  for (uint32_t q = 0; q < kSlGroup; ++q) {
    valid[q] = 0;
    out[q] = nh;
#pragma unroll
    for (int b = 0; b < P; ++b) t[q][b] = 0;
    if (q < gs) {
      const uint32_t i = gm[q];
      out[q] = nh + nh_off[i];
      Planes<P> sv;
      bload<P>(sv.v, rs, wpb, row_of[req_src[i]] * kSlSlots * wpm * 4);
      uint32_t ones = ~0u, zeros = ~0u, borrow = ~0u;
#pragma unroll
      for (int b = 0; b < P; ++b) {
        const uint32_t x = sv.v[b];
        ones &= x;
        zeros &= ~x;
        t[q][b] = x ^ borrow;  // t = d_s - 1
        borrow &= ~x;
      }
      valid[q] = ~(ones | zeros);
    }
  }
  // two groups of 4 neighbour rows in flight (row offset lists are padded:
  // loads past j1 read the dead row)
  constexpr int U = 4;
  offs += j0;
  const uint32_t k = j1 - j0;
  auto load_group = [&](uint32_t jj, Planes<P> (&r)[U]) {
    const uint4 o4 = *reinterpret_cast<const uint4*>(offs + jj);
    const uint32_t o[U] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
    for (int v = 0; v < U; ++v) bload<P>(r[v].v, rs, wpb, o[v] * 4);
  };
  auto match_group = [&](uint32_t jj, const Planes<P> (&r)[U]) {
#pragma unroll
    for (int v = 0; v < U; ++v) {
      if (jj + v >= k) break;
      const size_t at = (size_t)(j0 + jj + v) * wpm + w;
#pragma unroll
      for (uint32_t q = 0; q < kSlGroup; ++q) {
        if (q >= gs) break;  // wave-uniform
        uint32_t diff = 0;
#pragma unroll
        for (int b = 0; b < P; ++b) diff |= r[v].v[b] ^ t[q][b];
        if (live) {
          if constexpr (kSlStoreAux) __builtin_nontemporal_store(~diff & valid[q], &out[q][at]);
          else out[q][at] = ~diff & valid[q];
        }
      }
    }
  };
  Planes<P> ra[U], rb[U];
  load_group(0, ra);
  for (uint32_t jj = 0; jj < k; jj += 2 * U) {
    load_group(jj + U, rb);
    match_group(jj, ra);
    load_group(jj + 2 * U, ra);
    match_group(jj + U, rb);
  }
}

// Work units: (source i, chunks [c0, c1) of 64 words, neighbours [j0, j1)),
// at most about kSlUnit neighbour-chunk matches each (spf_plan_create keeps
// light sources whole and cuts heavy ones per chunk and neighbour range),
// one wave per unit, units of an XCD's source runs on that XCD.  A wave's
// matches are latency-bound (two groups of row loads in flight), so one wave
// per source left the spine switches (173 neighbours x 5 chunks) running
// long after the rest; one wave per (source, chunk) was bound by wave launch;
// persistent waves pulling units through per-XCD atomic counters serialised
// on the counters (r02_v20: 2.4x slower); sc1 bitmap stores (lines leave L2)
// changed nothing (r02_v22).
// neighbour-chunk matches per unit (at most, about): fabric_full's pass 68.5
// us at 128, 66 at 512, 72 at 1024, 92 at 2048 (gpurun_out/r04_s1, r04_s2)
constexpr uint32_t kSlUnit = 512;

__global__ __launch_bounds__(kEcmpThreads) void ecmp_sliced_kernel(
    const uint32_t* __restrict__ S, const uint32_t* __restrict__ maxd,
    const uint32_t* __restrict__ D, uint32_t pitch,
    const uint32_t* __restrict__ req_src, const uint32_t* __restrict__ row_of,
    const uint32_t* __restrict__ nb_ptr, const uint32_t* __restrict__ nb_id,
    const uint32_t* __restrict__ nb_w, const uint32_t* __restrict__ nb_row,
    const uint32_t* __restrict__ nb_row_off, const uint32_t* __restrict__ nb_drained,
    uint32_t dead, uint32_t hop, const uint64_t* __restrict__ nh_off, uint32_t* __restrict__ nh,
    const uint4* __restrict__ units, const uint32_t* __restrict__ unit_off,
    const uint32_t* __restrict__ gtab /* group units: [n, sources...] */, uint32_t s_bytes,
    uint32_t fixed_p /* rows sliced by the BFS itself (sdirect): P planes, maxd unused */,
    uint32_t weighted /* d_x + w(s, x) == d_s (weighted plans) instead of d_x == d_s - 1 */) {
  const uint32_t md = fixed_p ? 0u : *maxd;
  const uint32_t g = blockIdx.x & 7;  // this block's XCD (round-robin placement)
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wpm = pitch / 32;
  const uint32_t P = fixed_p ? fixed_p : md < kSlSat ? 32u - __clz(md + 1u) : 0u;  // 0: saturated
  const uint32_t rstride = kSlSlots * wpm;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(S), 0, (int)s_bytes, 0x00020000);
  // wave-uniform to the compiler too (readfirstlane): the unit's values then
  // live in SGPRs and its row offsets arrive by scalar loads
  const uint32_t t = (blockIdx.x >> 3) * kEcmpWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t u_begin = unit_off[g];
  if (t >= unit_off[g + 1] - u_begin) return;  // whole wave: no barriers below
  // one source's units: chunks [c0, c1), neighbours [j0, j1)
  auto single = [&](const uint32_t i, const uint32_t c0, const uint32_t c1, const uint32_t j0,
                    const uint32_t j1) {
    const uint32_t s = req_src[i];
    const uint32_t nb0 = nb_ptr[s], k = j1 - j0;
    const uint32_t srow = row_of[s];
    const uint32_t* offs = nb_row + nb_row_off[i];
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        nh + nh_off[i], 0, (int)((nb_ptr[s + 1] - nb0) * wpm * 4), 0x00020000);
    for (uint32_t c = c0; c < c1; ++c) {
      const uint32_t w0 = c * 64, w = w0 + lane;
      const bool live = w < wpm;
#define SL_CASE(PV)                                                                          \
  case PV:                                                                                   \
    if (weighted)                                                                            \
      sliced_pass<PV, true>(rs, ro, wpm, srow, offs + j0, k, j0, w, live, nb_w + nb0 + j0);  \
    else                                                                                     \
      sliced_pass<PV>(rs, ro, wpm, srow, offs + j0, k, j0, w, live);                         \
    break;
      switch (P) {
        SL_CASE(1)
        SL_CASE(2)
        SL_CASE(3)
        SL_CASE(4)
        SL_CASE(5)
        SL_CASE(6)
        SL_CASE(7)
        SL_CASE(8)
#undef SL_CASE
        default: {
          uint32_t* out = nh + nh_off[i] + w;
          // saturated: exact u32 rows, 32 destinations per lane (offsets are
          // sliced-row offsets, row = offset / rstride)
          for (uint32_t j = j0; j < j1; ++j) {
            const uint32_t oj = offs[j], wj = hop ? 1u : nb_w[nb0 + j];
            uint32_t m = 0;
            if (oj != dead && live) {
              const uint4* Dx = reinterpret_cast<const uint4*>(D + (size_t)(oj / rstride) * pitch + 32ull * w);
              const uint4* Ds = reinterpret_cast<const uint4*>(D + (size_t)srow * pitch + 32ull * w);
#pragma unroll 1
              for (int q = 0; q < 8; ++q) {
                const uint4 a4 = Dx[q], b4 = Ds[q];
                const uint32_t a[4] = {a4.x, a4.y, a4.z, a4.w}, b[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) m |= (uint32_t)(a[e] != kInf && a[e] + wj == b[e]) << (4 * q + e);
              }
            }
            if (live) out[(size_t)j * wpm] = m;
          }
        }
      }
      // drained neighbour x: only x itself, reached directly when d_s(x) == w(s, x)
      if (nb_drained[i]) {
        uint32_t* out = nh + nh_off[i] + w;
        const uint32_t cbase = w0 * 32;
        for (uint32_t j = j0; j < j1; ++j) {
          if (offs[j] != dead) continue;
          const uint32_t x = nb_id[nb0 + j];
          if (x < cbase || x >= cbase + kSlChunk) continue;
          const uint32_t wj = hop ? 1u : nb_w[nb0 + j];
          if (lane == (x - cbase) / 32 && D[(size_t)srow * pitch + x] == wj)
            out[(size_t)j * wpm] = 1u << (x & 31);
        }
      }
    }
  };
  const uint4 u = units[u_begin + t];
  if (u.y >> 31) {  // a group unit: sources with identical neighbour lists, one chunk
    const uint32_t* gm = gtab + u.x + 1;
    const uint32_t gs = __builtin_amdgcn_readfirstlane(gtab[u.x]), c = u.y & 0xFFFFu;
    const uint32_t* offs = nb_row + nb_row_off[gm[0]];  // the same list for every member
    const uint32_t w = c * 64 + lane;
    const bool live = w < wpm;
    switch (P) {
      case 1: grouped_pass<1>(rs, nh, nh_off, row_of, req_src, gm, gs, wpm, offs, u.z, u.w, w, live); break;
      case 2: grouped_pass<2>(rs, nh, nh_off, row_of, req_src, gm, gs, wpm, offs, u.z, u.w, w, live); break;
      case 3: grouped_pass<3>(rs, nh, nh_off, row_of, req_src, gm, gs, wpm, offs, u.z, u.w, w, live); break;
      case 4: grouped_pass<4>(rs, nh, nh_off, row_of, req_src, gm, gs, wpm, offs, u.z, u.w, w, live); break;
      default:  // deeper planes or saturated rows: member by member
        for (uint32_t q = 0; q < gs; ++q) single(gm[q], c, c + 1, u.z, u.w);
    }
    return;
  }
  single(u.x, u.y & 0xFFFFu, u.y >> 16, u.z, u.w);
}

// ---------------------------------------------------------------------------
//  copy selected D rows into the caller's dense output (non-direct plans)
// ---------------------------------------------------------------------------
// u8 rows (npitch bytes, a multiple of 16): row rows[i] -> out row i
__global__ void gather_rows_u8_kernel(const uint8_t* __restrict__ Dn, uint32_t npitch,
                                      const uint32_t* __restrict__ rows, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.y;
  const uint4* in = reinterpret_cast<const uint4*>(Dn + (size_t)rows[i] * npitch);
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)i * npitch);
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < npitch / 16;
       t += gridDim.x * blockDim.x)
    o[t] = in[t];
}

// practical HBM ceiling (spf_debug_copy_bandwidth): a grid-stride 16-byte
// copy, the float4-copy shape of MI355X_MICROARCH.md's measured 6.29 TB/s
__global__ __launch_bounds__(256) void copy_bw_kernel(const uint4* __restrict__ src,
                                                      uint4* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

__global__ void gather_rows_kernel(const uint32_t* __restrict__ D, uint32_t pitch,
                                   const uint32_t* __restrict__ rows,
                                   uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.y;
  const uint4* in = reinterpret_cast<const uint4*>(D + (size_t)rows[i] * pitch);
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)i * pitch);
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < pitch / 4;
       t += gridDim.x * blockDim.x)
    o[t] = in[t];
}

// ---------------------------------------------------------------------------
//  per-source result digests (spf_plan_digest): the checksum a rank ships
//  instead of its rows when results stay resident on its GPU
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t dg_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Block (chunk of 256 destinations, source i); thread = destination v.  The
// next-hop words of v are assembled 32 neighbours at a time from the planar
// bitmaps (lanes of a wave read the same two words: broadcast loads) and fed
// to FNV-1a in word order; the per-node terms are summed with a wave
// reduction and one 64-bit atomic per wave.
template <bool D64>
__global__ __launch_bounds__(256) void digest_kernel(const void* __restrict__ dist, uint32_t pitch,
                                                     uint32_t N, const uint32_t* __restrict__ nh,
                                                     const uint64_t* __restrict__ nh_off,
                                                     const uint32_t* __restrict__ words,
                                                     unsigned long long* __restrict__ out) {
  const uint32_t i = blockIdx.y;
  const uint32_t v = blockIdx.x * 256 + threadIdx.x;
  uint64_t term = 0;
  if (v < N) {
    const uint64_t d = D64 ? reinterpret_cast<const uint64_t*>(dist)[(size_t)i * pitch + v]
                           : reinterpret_cast<const uint32_t*>(dist)[(size_t)i * pitch + v];
    if (d != (D64 ? ~0ull : (uint64_t)kInf)) {
      const uint32_t k = words[i], wpm = pitch / 32;
      const uint32_t* b = nh + nh_off[i] + v / 32;
      const uint32_t sh = v % 32;
      uint64_t f = 0xcbf29ce484222325ull;
      for (uint32_t j0 = 0; j0 < k; j0 += 32) {
        uint32_t w = 0;
        const uint32_t jn = min(32u, k - j0);
        for (uint32_t j = 0; j < jn; ++j) w |= ((b[(size_t)(j0 + j) * wpm] >> sh) & 1u) << j;
        f ^= w;
        f *= 0x100000001b3ull;
      }
      term = dg_mix64(dg_mix64((uint64_t)v + 1) + d) ^ f;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)term, o, 64), hi = __shfl_xor((uint32_t)(term >> 32), o, 64);
    term += ((uint64_t)hi << 32) | lo;
  }
  if ((threadIdx.x & 63) == 0 && term) atomicAdd(&out[i], (unsigned long long)term);
}

// ---------------------------------------------------------------------------
//  3. predecessor lists (pathLinks) of one source
// ---------------------------------------------------------------------------
// pass 0: count, pass 1: fill sorted by (dist[u], edge id) -- edge ids of one
// tail are contiguous in CSR order and tails appear in id (= name) order, so
// this is the reference's (pop order, linksFromNode order).
template <int PASS>
__global__ void preds_kernel(const uint32_t* __restrict__ dist0,  // [n_src][pitch]
                             uint32_t pitch,
                             const uint32_t* __restrict__ row_ptr,
                             const uint32_t* __restrict__ col,
                             const uint32_t* __restrict__ wt,
                             const uint32_t* __restrict__ rev,
                             const uint8_t* __restrict__ ovl,
                             const uint32_t* __restrict__ link,
                             const uint32_t* __restrict__ ign,
                             const uint32_t* __restrict__ srcs,  // [n_src] (blockIdx.y)
                             uint32_t N, uint32_t hop,
                             uint32_t* __restrict__ cnt_or_ptr0,  // [n_src][N + 1]
                             uint32_t* __restrict__ pred_edge,
                             unsigned long long* __restrict__ pred_key /* PASS 1: sort keys */) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= N) return;
  const uint32_t* dist = dist0 + (size_t)blockIdx.y * pitch;
  uint32_t* cnt_or_ptr = cnt_or_ptr0 + (size_t)blockIdx.y * (N + 1);
  const uint32_t src = srcs[blockIdx.y];
  const uint32_t dv = dist[v];
  uint32_t n = 0;
  uint32_t base = PASS ? cnt_or_ptr[v] : 0;
  if (dv != kInf && v != src) {
    for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
      const uint32_t u = col[e];
      const uint32_t r = rev[e];  // the directed edge u -> v
      if (ovl[u] && u != src) continue;
      if (ign && link_ignored(ign, link[e])) continue;
      const uint32_t du = dist[u];
      if (du == kInf) continue;
      if (du + (hop ? 1u : wt[r]) != dv) continue;
      if (PASS) {
        // insertion into the sorted segment [base, base+n) by (dist of the
        // tail, edge id), the keys kept beside the edges (one load per step
        // where re-deriving a key was three dependent loads)
        const unsigned long long key = ((unsigned long long)du << 32) | r;
        uint32_t p = base + n;
        while (p > base) {
          const unsigned long long pk = pred_key[p - 1];
          if (pk < key) break;
          pred_key[p] = pk;
          pred_edge[p] = (uint32_t)pk;
          --p;
        }
        pred_key[p] = key;
        pred_edge[p] = r;
      }
      ++n;
    }
  }
  if (!PASS) cnt_or_ptr[v] = n;
}

// ---------------------------------------------------------------------------
//  host side
// ---------------------------------------------------------------------------
}  // namespace

namespace {

size_t sssp_lds_bytes(uint32_t N, uint32_t pitch, uint32_t big, bool q16) {
  const uint32_t bm_words = (N + 31) / 32;
  size_t b = 4ull * pitch + 4ull * bm_words + 4ull * C_NWORDS + 4ull * big;
  b += (q16 ? 2ull : 4ull) * N;
  return (b + 15) & ~size_t(15);
}

}  // namespace

extern "C" {

const char* spf_global_error(void) { return g_err.c_str(); }
const char* spf_last_error(const spf_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }
uint64_t spf_solves(const spf_ctx* c) { return c ? c->solves : 0; }
uint32_t spf_row_pitch(const spf_ctx* c) { return c ? c->pitch : 0; }
int spf_graph_has_nonpositive_metric(const spf_ctx* c) { return c && c->nonpos; }
int spf_graph_needs_dist64(const spf_ctx* c) { return c && c->needs64; }

spf_status spf_ctx_create(int device, spf_ctx** out) {
  if (!out) return fail(nullptr, SPF_E_INVALID, "spf_ctx_create: out is NULL");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(nullptr, SPF_E_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n)
    return fail(nullptr, SPF_E_NO_DEVICE, "device %d out of range (%d visible)", device, n);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    return fail(nullptr, SPF_E_NO_DEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(nullptr, SPF_E_NO_DEVICE, "device %d is %s, engine is built for gfx950",
                device, prop.gcnArchName);
  auto c = std::make_unique<spf_ctx>();
  c->device = device;
  c->n_cu = (uint32_t)std::max(1, prop.multiProcessorCount);
  if (hipSetDevice(device) != hipSuccess)
    return fail(nullptr, SPF_E_HIP, "hipSetDevice(%d) failed", device);
  // a BLOCKING stream: work enqueued with stream = NULL ("the context's
  // stream") is ordered after earlier work on the legacy null stream, so a
  // caller's hipMemset / hipMemcpy on the null stream before an execute is
  // seen by it (round 3 lost a plan's first bitmaps to exactly that race
  // with a non-blocking stream)
  if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess)
    return fail(nullptr, SPF_E_HIP, "hipStreamCreate failed");
  if (c->d_fault.alloc(1) != hipSuccess || hipMemset(c->d_fault.p, 0, 4) != hipSuccess)
    return fail(nullptr, SPF_E_HIP, "fault word allocation failed");
  *out = c.release();
  return SPF_OK;
}

void spf_ctx_destroy(spf_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  spfi::resident_forget(c);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  spf_plan_destroy(c->rt.plan);  // spf_routes' cached plan, before its context goes
  c->rt.plan = nullptr;
  if (c->stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
  }
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  if (c->side_fork) (void)hipEventDestroy(c->side_fork);
  if (c->side_join) (void)hipEventDestroy(c->side_join);
  delete c;
}

// Live-edge metric facts (nonpos, needs64, max_metric, unit) from a scan of
// the graph, with the counts a row patch keeps them current by
static void metric_flags(spf_ctx* c) {
  c->nonpos = c->n_nonpos > 0;
  // i32 -> u64 wraps (LinkState.h:22); the longest possible path beyond 32
  // bits takes the exact kernel's u64 labels (SPF_FLAG_DIST64)
  c->needs64 = c->n_neg > 0 || (uint64_t)c->max_metric * (uint64_t)(c->N - 1) >= (uint64_t)kInf;
  c->unit = !c->nonpos && c->max_metric <= 1;
}
static void metric_facts(spf_ctx* c) {
  c->n_nonpos = c->n_neg = c->n_at_max = 0;
  c->max_metric = 0;
  for (uint32_t u = 0; u < c->N; ++u)
    for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e) {
      if (c->col[e] == u) continue;  // dead slot
      c->n_nonpos += c->met[e] <= 0;
      c->n_neg += c->met[e] < 0;
      if (c->wt[e] > c->max_metric) {
        c->max_metric = c->wt[e];
        c->n_at_max = 1;
      } else if (c->wt[e] == c->max_metric) {
        ++c->n_at_max;
      }
    }
  metric_flags(c);
}

spf_status spf_graph_load(spf_ctx* c, const spf_graph* g) {
  if (!c || !g) return fail(c, SPF_E_INVALID, "spf_graph_load: NULL argument");
  const uint32_t N = g->n_nodes, E = g->n_edges;
  if (N == 0) return fail(c, SPF_E_INVALID, "graph has no nodes");
  if (!g->row_ptr || (E && (!g->col || !g->metric || !g->link_id)) || !g->overloaded)
    return fail(c, SPF_E_INVALID, "graph arrays missing");
  if (g->row_ptr[0] != 0 || g->row_ptr[N] != E)
    return fail(c, SPF_E_INVALID, "row_ptr must start at 0 and end at n_edges");
  c->loaded = false;
  c->N = N;
  c->E = E;
  // dist rows / bitmap rows: whole 1024-node chunks, so every next-hop
  // bitmap (pitch / 8 bytes) starts on a 128-byte line and no line of the
  // output is written partially by two waves (SPF_PITCH_ALIGN: A/B only)
  {
    const char* e = std::getenv("SPF_PITCH_ALIGN");
    const uint32_t a = e ? (uint32_t)atoi(e) : 1024u;  // a power of two >= 64
    c->pitch = (N + a - 1) & ~(a - 1);
  }
  c->npitch = (N + 1023) & ~1023u;  // narrow rows: whole 1024-node chunks
  c->row_ptr.assign(g->row_ptr, g->row_ptr + N + 1);
  c->col.assign(g->col, g->col + E);
  c->link.assign(g->link_id, g->link_id + E);
  c->ovl.assign(g->overloaded, g->overloaded + N);
  c->wt.resize(E);
  c->met.assign(g->metric, g->metric + E);
  c->nonpos = false;
  c->needs64 = false;
  c->max_metric = 0;
  for (uint32_t u = 0; u < N; ++u) {
    if (c->row_ptr[u] > c->row_ptr[u + 1])
      return fail(c, SPF_E_INVALID, "row_ptr not monotone at %u", u);
  }
  for (uint32_t u = 0; u < N; ++u)
    for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e) {
      if (c->col[e] >= N) return fail(c, SPF_E_INVALID, "edge %u head %u out of range", e, c->col[e]);
      const int32_t m = g->metric[e];
      c->wt[e] = m > 0 ? (uint32_t)m : 0u;
      if (c->col[e] == u) {  // a dead slot (see openr_spf.h): no edge
        if (m != 1) return fail(c, SPF_E_INVALID, "dead slot %u (a self-loop) must carry metric 1", e);
        continue;
      }
      if (m <= 0) c->nonpos = true;
      if (m < 0) c->needs64 = true;  // i32 -> u64 wraps (LinkState.h:22)
      c->max_metric = std::max(c->max_metric, c->wt[e]);
    }
  metric_facts(c);  // (the same facts, with the counts row patches update)
  // reverse edge of every directed edge (same link id, swapped ends)
  c->rev.assign(E, kInf);
  {
    std::vector<uint32_t> first(0);
    uint32_t max_link = 0;
    for (uint32_t e = 0; e < E; ++e) max_link = std::max(max_link, c->link[e]);
    std::vector<uint32_t> seen((size_t)max_link + 1, kInf);
    for (uint32_t u = 0; u < N; ++u)
      for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e) {
        uint32_t& s = seen[c->link[e]];
        if (s == kInf) {
          s = e;
        } else {
          c->rev[e] = s;
          c->rev[s] = e;
        }
      }
    for (uint32_t e = 0; e < E; ++e)
      if (c->rev[e] == kInf)
        return fail(c, SPF_E_INVALID, "edge %u (link %u) has no reverse edge", e, c->link[e]);
    c->link_slot.assign(2 * ((size_t)max_link + 1), kInf);
    for (uint32_t e = 0; e < E; ++e) {
      uint32_t* ls = &c->link_slot[2 * (size_t)c->link[e]];
      ls[ls[0] == kInf ? 0 : 1] = e;
    }
  }
  // distinct up neighbours per node, ascending id, min metric
  c->nb_ptr.assign(N + 1, 0);
  c->nb_id.clear();
  c->nb_w.clear();
  c->big_nodes = 0;
  std::vector<std::pair<uint32_t, uint32_t>> tmp;
  for (uint32_t u = 0; u < N; ++u) {
    tmp.clear();
    for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
      if (c->col[e] != u) tmp.emplace_back(c->col[e], c->wt[e]);
    if (c->row_ptr[u + 1] - c->row_ptr[u] > kBigDeg) ++c->big_nodes;
    std::sort(tmp.begin(), tmp.end());
    for (size_t i = 0; i < tmp.size(); ++i) {
      if (i && tmp[i].first == tmp[i - 1].first) continue;  // first = min metric
      c->nb_id.push_back(tmp[i].first);
      c->nb_w.push_back(tmp[i].second);
    }
    c->nb_ptr[u + 1] = (uint32_t)c->nb_id.size();
  }
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, c->d_row_ptr.upload(c->row_ptr.data(), N + 1, c->stream));
  HIP_TRY(c, c->d_col.upload(c->col.data(), E, c->stream));
  HIP_TRY(c, c->d_wt.upload(c->wt.data(), E, c->stream));
  HIP_TRY(c, c->d_met.upload(c->met.data(), E, c->stream));
  HIP_TRY(c, c->d_rev.upload(c->rev.data(), E, c->stream));
  HIP_TRY(c, c->d_link.upload(c->link.data(), E, c->stream));
  c->max_link = 0;
  for (uint32_t e = 0; e < E; ++e) c->max_link = std::max(c->max_link, c->link[e]);
  HIP_TRY(c, c->d_ovl.upload(c->ovl.data(), N, c->stream));
  HIP_TRY(c, c->d_nb_ptr.upload(c->nb_ptr.data(), N + 1, c->stream));
  HIP_TRY(c, c->d_nb_id.upload(c->nb_id.data(), c->nb_id.size(), c->stream));
  HIP_TRY(c, c->d_nb_w.upload(c->nb_w.data(), c->nb_w.size(), c->stream));
  {  // per edge: the head's index among the tail's distinct neighbours (the
     // route selection's next-hop bitmap of that neighbour)
    std::vector<uint32_t>& enb = c->edge_nb;
    enb.assign(std::max<uint32_t>(E, 1), kInf);
    for (uint32_t u = 0; u < N; ++u) {
      const auto b = c->nb_id.begin() + c->nb_ptr[u], e = c->nb_id.begin() + c->nb_ptr[u + 1];
      for (uint32_t q = c->row_ptr[u]; q < c->row_ptr[u + 1]; ++q)
        enb[q] = c->col[q] == u ? kInf : (uint32_t)(std::lower_bound(b, e, c->col[q]) - b);
    }
    HIP_TRY(c, c->d_edge_nb.upload(enb.data(), enb.size(), c->stream));
  }
  // sliced ELL (SELL-64): slice = 64 consecutive nodes, width = max degree in
  // the slice, entry (slice, j, lane) = j-th neighbour of node slice*64+lane,
  // padded with N (F[N] == 0 in the BFS kernel)
  {
    const uint32_t n_slices = (N + kSliceW - 1) / kSliceW;
    c->sell_ptr.assign(n_slices + 1, 0);
    for (uint32_t sl = 0; sl < n_slices; ++sl) {
      uint32_t w = 0;
      for (uint32_t v = sl * kSliceW; v < std::min(N, (sl + 1) * kSliceW); ++v)
        w = std::max(w, c->row_ptr[v + 1] - c->row_ptr[v]);
      c->sell_ptr[sl + 1] = c->sell_ptr[sl] + w * kSliceW;
    }
    // + one trailing all-padding group (msbfs_team.hip pads its column streams with it)
    // + padding columns (node N): the trailing all-padding group the team
    // kernel's stream pads with, and the BFS kernels' unconditional loads up
    // to three groups of 8 columns past a slice's last column
    c->sell_col.assign(c->sell_ptr[n_slices] + 32 * kSliceW, N);
    ++c->sell_ver;
    for (uint32_t v = 0; v < N; ++v) {
      const uint32_t sl = v / kSliceW, ln = v % kSliceW;
      for (uint32_t j = 0; j < c->row_ptr[v + 1] - c->row_ptr[v]; ++j) {
        const uint32_t x = c->col[c->row_ptr[v] + j];
        c->sell_col[c->sell_ptr[sl] + j * kSliceW + ln] = x == v ? N : x;  // dead slot: padding
      }
    }
    HIP_TRY(c, c->d_sell_ptr.upload(c->sell_ptr.data(), c->sell_ptr.size(), c->stream));
    HIP_TRY(c, c->d_sell_col.upload(c->sell_col.data(), c->sell_col.size(), c->stream));
    // msbfs_kernel's slices per wave: a level's pull sweep costs each wave the
    // column groups of its slices and the workgroup waits for the slowest, so
    // slices are dealt widest first to the wave with the fewest groups that
    // still has a free slot (OWN slots per wave; unused slots = kNoSlice)
    if (N <= kMsMaxNodes) {
      const uint32_t own = ms_own(N), waves = kMsThreads / 64;
      std::vector<uint32_t> order(n_slices), load(waves, 0), used(waves, 0);
      std::iota(order.begin(), order.end(), 0u);
      auto width = [&](uint32_t sl) { return (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / kSliceW; };
      std::stable_sort(order.begin(), order.end(),
                       [&](uint32_t a, uint32_t b) { return width(a) > width(b); });
      std::vector<uint32_t> smap((size_t)waves * own, kNoSlice);
      for (uint32_t sl : order) {
        uint32_t best = waves;
        for (uint32_t w = 0; w < waves; ++w)
          if (used[w] < own && (best == waves || load[w] < load[best])) best = w;
        smap[(size_t)best * own + used[best]++] = sl;
        load[best] += std::max(1u, width(sl));
      }
      if (std::getenv("SPF_SMAP_STRIDED"))  // A/B: slot i of wave w = slice 16 i + w
        for (uint32_t w = 0; w < waves; ++w)
          for (uint32_t i = 0; i < own; ++i) {
            const uint32_t sl = i * waves + w;
            smap[(size_t)w * own + i] = sl < n_slices ? sl : kNoSlice;
          }
      HIP_TRY(c, c->d_ms_smap.upload(smap.data(), smap.size(), c->stream));
    }
    // the same columns packed four u16 ids per lane (groups of 4 per slice,
    // at least one), for msbfs_planes_kernel (N <= 10240)
    c->sell4_ptr.assign(n_slices + 1, 0);
    c->sell4.clear();
    if (4ull * N < 65536) {
      for (uint32_t sl = 0; sl < n_slices; ++sl) {
        const uint32_t w = (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / kSliceW;
        const uint32_t groups = std::max(1u, (w + 3) / 4);
        c->sell4_ptr[sl + 1] = c->sell4_ptr[sl] + groups * kSliceW;
      }
      c->sell4.assign(2ull * c->sell4_ptr[n_slices], 0);
      for (uint32_t sl = 0; sl < n_slices; ++sl) {
        const uint32_t w = (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / kSliceW;
        const uint32_t groups = (c->sell4_ptr[sl + 1] - c->sell4_ptr[sl]) / kSliceW;
        for (uint32_t g = 0; g < groups; ++g)
          for (uint32_t ln = 0; ln < kSliceW; ++ln) {
            uint32_t id[4];
            for (uint32_t k = 0; k < 4; ++k) {
              const uint32_t j = 4 * g + k;
              id[k] = j < w ? c->sell_col[c->sell_ptr[sl] + j * kSliceW + ln] : N;
            }
            const size_t e = 2ull * (c->sell4_ptr[sl] + g * kSliceW + ln);
            // byte offsets into the BFS frontier array (4 B per node)
            c->sell4[e] = 4 * id[0] | (4 * id[1] << 16);
            c->sell4[e + 1] = 4 * id[2] | (4 * id[3] << 16);
          }
      }
      HIP_TRY(c, c->d_sell4_ptr.upload(c->sell4_ptr.data(), c->sell4_ptr.size(), c->stream));
      HIP_TRY(c, c->d_sell4.upload(c->sell4.data(), c->sell4.size(), c->stream));
    }
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->loaded = true;
  ++c->shape;
  ++c->epoch;
  ++c->layout;
  return SPF_OK;
}

// In-place graph patches.  The reference reacts to
// every adjacency-database publication by re-running updateAdjacencyDatabase
// (LinkState.cpp:564-719) and dropping its SPF memo; the common cases -- a node
// toggling its overload bit (the per-iteration perturbation of
// BM_DecisionFabric, RoutingBenchmarkUtils.cpp:453-479) or a link metric
// change -- leave the CSR structure intact, so only the affected bytes are
// rewritten here instead of a full spf_graph_load.
spf_status spf_graph_set_overload(spf_ctx* c, const uint32_t* nodes, const uint8_t* overloaded,
                                  uint32_t n) {
  if (!c || (n && (!nodes || !overloaded)))
    return fail(c, SPF_E_INVALID, "spf_graph_set_overload: NULL argument");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  for (uint32_t i = 0; i < n; ++i)
    if (nodes[i] >= c->N) return fail(c, SPF_E_INVALID, "node %u out of range", nodes[i]);
  bool changed = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t v = overloaded[i] ? 1 : 0;
    if (c->ovl[nodes[i]] != v) {
      c->ovl[nodes[i]] = v;
      changed = true;
    }
  }
  if (!changed) return SPF_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, stage_upload(c, c->d_ovl, c->ovl.data(), c->N));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  stage_done(c);
  ++c->epoch;
  return SPF_OK;
}

spf_status spf_graph_set_metric(spf_ctx* c, const uint32_t* edges, const int32_t* metric,
                                uint32_t n) {
  if (!c || (n && (!edges || !metric)))
    return fail(c, SPF_E_INVALID, "spf_graph_set_metric: NULL argument");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  for (uint32_t i = 0; i < n; ++i)
    if (edges[i] >= c->E) return fail(c, SPF_E_INVALID, "edge %u out of range", edges[i]);
  std::vector<uint32_t> wt = c->wt;
  std::vector<int32_t> met = c->met;
  bool changed = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t w = metric[i] > 0 ? (uint32_t)metric[i] : 0u;
    changed |= met[edges[i]] != metric[i];
    wt[edges[i]] = w;
    met[edges[i]] = metric[i];
  }
  if (!changed) return SPF_OK;
  c->wt.swap(wt);
  c->met.swap(met);
  metric_facts(c);
  // min metric per distinct neighbour of every tail touched
  std::vector<uint32_t> tails;
  for (uint32_t i = 0; i < n; ++i)
    tails.push_back((uint32_t)(std::upper_bound(c->row_ptr.begin(), c->row_ptr.end(), edges[i]) -
                               c->row_ptr.begin()) - 1);
  std::sort(tails.begin(), tails.end());
  tails.erase(std::unique(tails.begin(), tails.end()), tails.end());
  for (uint32_t u : tails) {
    const uint32_t b = c->nb_ptr[u], e = c->nb_ptr[u + 1];
    for (uint32_t j = b; j < e; ++j) c->nb_w[j] = kInf;
    for (uint32_t k = c->row_ptr[u]; k < c->row_ptr[u + 1]; ++k) {
      if (c->col[k] == u) continue;  // dead slot
      const uint32_t j = (uint32_t)(std::lower_bound(c->nb_id.begin() + b, c->nb_id.begin() + e,
                                                     c->col[k]) - c->nb_id.begin());
      c->nb_w[j] = std::min(c->nb_w[j], c->wt[k]);
    }
  }
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, stage_upload(c, c->d_wt, c->wt.data(), c->E));
  HIP_TRY(c, stage_upload(c, c->d_met, c->met.data(), c->E));
  HIP_TRY(c, stage_upload(c, c->d_nb_w, c->nb_w.data(), c->nb_w.size()));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  stage_done(c);
  ++c->epoch;
  return SPF_OK;
}

// Rows rewritten in place (a link going down or up,
// or an adjacency withdrawn and advertised again, without a reload).  Each
// listed node keeps its row length; a dead slot is a self-loop (col = the
// node, metric 1): no kernel relaxes, pushes or pulls anything over one, the
// distinct-neighbour lists and the route tables skip them.  The derived
// tables of the touched rows are patched: reverse edges (by link id), the
// distinct-neighbour lists (rebuilt when a count changes: plans whose
// sources' next-hop layout changed fail with SPF_E_STATE), the route tables'
// per-edge neighbour index and the sliced-ELL columns.  Plans re-derive at
// their next execute, as after a metric patch.
spf_status spf_graph_patch_rows(spf_ctx* c, const uint32_t* nodes, uint32_t n, const uint32_t* col,
                                const int32_t* metric, const uint32_t* link) {
  if (!c || (n && (!nodes || !col || !metric || !link)))
    return fail(c, SPF_E_INVALID, "spf_graph_patch_rows: NULL argument");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  const uint32_t N = c->N;
  std::vector<uint8_t> touched(N, 0);

  for (uint32_t i = 0; i < n; ++i) {
    if (nodes[i] >= N) return fail(c, SPF_E_INVALID, "node %u out of range", nodes[i]);
    if (touched[nodes[i]]++) return fail(c, SPF_E_INVALID, "node %u listed twice", nodes[i]);

  }
  if (!n) return SPF_OK;
  // validate the new rows before changing anything
  const uint32_t max_link = (uint32_t)(c->link_slot.size() / 2) - 1;
  {
    size_t o = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t u = nodes[i];
      for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e, ++o) {
        if (col[o] >= N) return fail(c, SPF_E_INVALID, "row of %u: head %u out of range", u, col[o]);
        if (link[o] > max_link)
          return fail(c, SPF_E_INVALID, "row of %u: link %u is not a link of the loaded graph", u, link[o]);
        if (col[o] == u && metric[o] != 1)
          return fail(c, SPF_E_INVALID, "row of %u: a dead slot (self-loop) must carry metric 1", u);
      }
    }
  }
  std::vector<uint32_t> old_nb(n);
  for (uint32_t i = 0; i < n; ++i) old_nb[i] = c->nb_ptr[nodes[i] + 1] - c->nb_ptr[nodes[i]];
  // rows (the metric-fact counts lose the old rows' live edges and gain the
  // new ones')
  {
    size_t o = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t u = nodes[i];
      for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
        if (c->col[e] != u) {
          c->n_nonpos -= c->met[e] <= 0;
          c->n_neg -= c->met[e] < 0;
          c->n_at_max -= c->wt[e] == c->max_metric;
        }
    }
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t u = nodes[i];
      for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e, ++o) {
        c->col[e] = col[o];
        c->met[e] = metric[o];
        c->wt[e] = metric[o] > 0 ? (uint32_t)metric[o] : 0u;
        c->link[e] = link[o];
      }
    }
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t u = nodes[i];
      for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
        if (c->col[e] != u) {
          c->n_nonpos += c->met[e] <= 0;
          c->n_neg += c->met[e] < 0;
          if (c->wt[e] > c->max_metric) {
            c->max_metric = c->wt[e];
            c->n_at_max = 1;
          } else if (c->wt[e] == c->max_metric) {
            ++c->n_at_max;
          }
        }
    }
  }
  // link slots and reverse edges: a link's slot in an untouched row keeps its
  // position; its slots in touched rows are where the new rows put them
  auto tail = [&](uint32_t e) {
    return (uint32_t)(std::upper_bound(c->row_ptr.begin(), c->row_ptr.end(), e) - c->row_ptr.begin()) - 1;
  };
  std::unordered_map<uint32_t, std::vector<uint32_t>> moved;  // link -> its slots in touched rows
  std::vector<uint32_t> rev_dirty;  // reverse-edge entries whose value changed
  auto set_rev = [&](uint32_t e, uint32_t r) {
    if (c->rev[e] != r) {
      c->rev[e] = r;
      rev_dirty.push_back(e);
    }
  };
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t e = c->row_ptr[nodes[i]]; e < c->row_ptr[nodes[i] + 1]; ++e) moved[c->link[e]].push_back(e);
  for (auto& [l, es] : moved) {
    uint32_t* ls = &c->link_slot[2 * (size_t)l];
    std::vector<uint32_t> slots = es;
    for (int k = 0; k < 2; ++k)  // its slot in an untouched row, if any, stays
      if (ls[k] != kInf && !touched[tail(ls[k])] && c->link[ls[k]] == l) slots.push_back(ls[k]);
    if (slots.size() != 2)
      return fail(c, SPF_E_INVALID, "link %u has %zu slots after the patch (2 needed)", l, slots.size());
    ls[0] = slots[0];
    ls[1] = slots[1];
    set_rev(slots[0], slots[1]);
    set_rev(slots[1], slots[0]);
    const uint32_t a = tail(slots[0]), b = tail(slots[1]);
    const bool dead0 = c->col[slots[0]] == a, dead1 = c->col[slots[1]] == b;
    if (dead0 != dead1 || (!dead0 && (c->col[slots[0]] != b || c->col[slots[1]] != a)))
      return fail(c, SPF_E_INVALID, "link %u: its two slots are not one link in both directions", l);
  }
  // graph-wide metric facts over live edges: from the counts, unless every
  // edge at the old maximum left (then the maximum fell: one scan)
  if (c->n_at_max == 0) metric_facts(c);
  else metric_flags(c);
  // distinct up neighbours of the touched nodes; the lists are rebuilt (every
  // untouched node's range copied) when a count changes
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> fresh(n);
  bool counts = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t u = nodes[i];
    auto& t = fresh[i];
    for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
      if (c->col[e] != u) t.emplace_back(c->col[e], c->wt[e]);
    std::sort(t.begin(), t.end());
    t.erase(std::unique(t.begin(), t.end(), [](const auto& a, const auto& b) { return a.first == b.first; }),
            t.end());
    counts |= t.size() != old_nb[i];
  }
  if (counts) {
    // the untouched nodes' lists move as whole blocks between touched nodes
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return nodes[a] < nodes[b]; });
    std::vector<uint32_t> ptr(N + 1, 0), id, w;
    id.reserve(c->nb_id.size() + 16);
    w.reserve(c->nb_id.size() + 16);
    uint32_t next = 0;  // first node not yet placed
    auto block = [&](uint32_t to) {  // untouched nodes next .. to - 1
      const uint32_t b = c->nb_ptr[next], e = c->nb_ptr[to];
      const int64_t shift = (int64_t)id.size() - (int64_t)b;
      id.insert(id.end(), c->nb_id.begin() + b, c->nb_id.begin() + e);
      w.insert(w.end(), c->nb_w.begin() + b, c->nb_w.begin() + e);
      for (uint32_t u = next; u < to; ++u) ptr[u + 1] = (uint32_t)((int64_t)c->nb_ptr[u + 1] + shift);
    };
    for (uint32_t oi : order) {
      const uint32_t u = nodes[oi];
      block(u);
      for (const auto& x : fresh[oi]) {
        id.push_back(x.first);
        w.push_back(x.second);
      }
      ptr[u + 1] = (uint32_t)id.size();
      next = u + 1;
    }
    block(N);
    c->nb_ptr.swap(ptr);
    c->nb_id.swap(id);
    c->nb_w.swap(w);
    ++c->layout;
  } else {
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t b = c->nb_ptr[nodes[i]];
      for (size_t k = 0; k < fresh[i].size(); ++k) {
        c->nb_id[b + k] = fresh[i][k].first;
        c->nb_w[b + k] = fresh[i][k].second;
      }
    }
  }
  HIP_TRY(c, hipSetDevice(c->device));
  // the route tables' per-edge neighbour index (touched tails only)
  std::vector<uint32_t>& enb = c->edge_nb;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t u = nodes[i];
    const auto b = c->nb_id.begin() + c->nb_ptr[u], e = c->nb_id.begin() + c->nb_ptr[u + 1];
    for (uint32_t q = c->row_ptr[u]; q < c->row_ptr[u + 1]; ++q)
      enb[q] = c->col[q] == u ? kInf : (uint32_t)(std::lower_bound(b, e, c->col[q]) - b);
  }
  // sliced-ELL columns of the touched nodes (and their packed u16 copies)
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t v = nodes[i], sl = v / kSliceW, ln = v % kSliceW;
    const uint32_t deg = c->row_ptr[v + 1] - c->row_ptr[v];
    for (uint32_t j = 0; j < deg; ++j) {
      const uint32_t x = c->col[c->row_ptr[v] + j];
      c->sell_col[c->sell_ptr[sl] + j * kSliceW + ln] = x == v ? N : x;
    }
    if (!c->sell4.empty()) {
      const uint32_t w = (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / kSliceW;
      const uint32_t groups = (c->sell4_ptr[sl + 1] - c->sell4_ptr[sl]) / kSliceW;
      for (uint32_t g = 0; g < groups; ++g) {
        uint32_t id[4];
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t j = 4 * g + k;
          id[k] = j < w ? c->sell_col[c->sell_ptr[sl] + j * kSliceW + ln] : N;
        }
        const size_t e = 2ull * (c->sell4_ptr[sl] + g * kSliceW + ln);
        c->sell4[e] = 4 * id[0] | (4 * id[1] << 16);
        c->sell4[e + 1] = 4 * id[2] | (4 * id[3] << 16);
      }
    }
  }
  ++c->sell_ver;  // (msbfs_team_prepare's cached tables read sell_col)
  // upload the changed ranges only: the touched rows (merged when adjacent),
  // the partner slots their reverse edges point at, and the touched slices
  std::vector<uint32_t> order(nodes, nodes + n);
  std::sort(order.begin(), order.end());
  std::vector<std::pair<uint32_t, uint32_t>> runs;  // [begin, end) edge ranges
  for (uint32_t u : order) {
    const uint32_t b = c->row_ptr[u], e = c->row_ptr[u + 1];
    if (b == e) continue;
    if (!runs.empty() && runs.back().second == b)
      runs.back().second = e;
    else
      runs.emplace_back(b, e);
  }
  // (uploads through the pinned stage: queued, not a blocking pageable copy each)
  for (const auto& r : runs) {
    const size_t b = r.first, k = r.second - r.first;
    HIP_TRY(c, stage_upload_at(c, c->d_col, c->col.data(), b, k));
    HIP_TRY(c, stage_upload_at(c, c->d_wt, c->wt.data(), b, k));
    HIP_TRY(c, stage_upload_at(c, c->d_met, c->met.data(), b, k));
    HIP_TRY(c, stage_upload_at(c, c->d_rev, c->rev.data(), b, k));
    HIP_TRY(c, stage_upload_at(c, c->d_link, c->link.data(), b, k));
    HIP_TRY(c, stage_upload_at(c, c->d_edge_nb, enb.data(), b, k));
  }
  {  // reverse-edge entries outside the touched rows whose value changed
    std::sort(rev_dirty.begin(), rev_dirty.end());
    rev_dirty.erase(std::unique(rev_dirty.begin(), rev_dirty.end()), rev_dirty.end());
    auto in_runs = [&](uint32_t q) {
      auto it = std::upper_bound(runs.begin(), runs.end(), std::make_pair(q, ~0u));
      return it != runs.begin() && q < std::prev(it)->second;
    };
    for (size_t a = 0; a < rev_dirty.size();) {
      if (in_runs(rev_dirty[a])) {
        ++a;
        continue;
      }
      size_t b = a + 1;
      while (b < rev_dirty.size() && rev_dirty[b] == rev_dirty[b - 1] + 1 && !in_runs(rev_dirty[b])) ++b;
      HIP_TRY(c, stage_upload_at(c, c->d_rev, c->rev.data(), rev_dirty[a], b - a));
      a = b;
    }
  }
  if (counts) {  // the lists moved from the first touched node on
    const uint32_t u0 = order.front();
    const size_t b = c->nb_ptr[u0];
    HIP_TRY(c, stage_upload_at(c, c->d_nb_ptr, c->nb_ptr.data(), u0, N + 1 - u0));
    if (c->d_nb_id.n < c->nb_id.size()) {  // (the lists outgrew the buffers)
      HIP_TRY(c, stage_upload(c, c->d_nb_id, c->nb_id.data(), c->nb_id.size()));
      HIP_TRY(c, stage_upload(c, c->d_nb_w, c->nb_w.data(), c->nb_w.size()));
    } else {
      HIP_TRY(c, stage_upload_at(c, c->d_nb_id, c->nb_id.data(), b, c->nb_id.size() - b));
      HIP_TRY(c, stage_upload_at(c, c->d_nb_w, c->nb_w.data(), b, c->nb_w.size() - b));
    }
  } else {
    for (uint32_t u : order) {
      const size_t b = c->nb_ptr[u], k = c->nb_ptr[u + 1] - b;
      HIP_TRY(c, stage_upload_at(c, c->d_nb_id, c->nb_id.data(), b, k));
      HIP_TRY(c, stage_upload_at(c, c->d_nb_w, c->nb_w.data(), b, k));
    }
  }
  {
    std::vector<uint32_t> slices;
    for (uint32_t u : order) slices.push_back(u / kSliceW);
    slices.erase(std::unique(slices.begin(), slices.end()), slices.end());
    for (uint32_t sl : slices) {
      const size_t b = c->sell_ptr[sl], k = c->sell_ptr[sl + 1] - b;
      HIP_TRY(c, stage_upload_at(c, c->d_sell_col, c->sell_col.data(), b, k));
      if (!c->sell4.empty()) {
        const size_t b4 = 2ull * c->sell4_ptr[sl], k4 = 2ull * (c->sell4_ptr[sl + 1] - c->sell4_ptr[sl]);
        HIP_TRY(c, stage_upload_at(c, c->d_sell4, c->sell4.data(), b4, k4));
      }
    }
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  stage_done(c);
  ++c->epoch;
  return SPF_OK;
}

uint64_t spf_graph_epoch(const spf_ctx* c) { return c ? c->epoch : 0; }
uint64_t spf_graph_loads(const spf_ctx* c) { return c ? c->shape : 0; }

spf_status spf_src_neighbors(const spf_ctx* c, uint32_t src, uint32_t* out,
                             uint32_t cap, uint32_t* count) {
  if (!c || !c->loaded) return SPF_E_STATE;
  if (src >= c->N) return SPF_E_INVALID;
  const uint32_t b = c->nb_ptr[src], k = c->nb_ptr[src + 1] - b;
  if (count) *count = k;
  for (uint32_t i = 0; i < k && i < cap && out; ++i) out[i] = c->nb_id[b + i];
  return SPF_OK;
}

}  // extern "C"

namespace {

// u8 narrow rows for the next-hop pass: 4x fewer bytes per neighbour row
// read, paid for by a second store per (source, slice, level) in
// msbfs_kernel.  Worth it when next-hop work (sum of neighbour counts)
// outweighs the BFS store work, which grows with the number of levels:
// dense fabrics (degree ~23, 5 levels) yes; always with the register-plane
// BFS (one coalesced store per row).  SPF_NARROW=0/1 overrides (experiments).
bool use_planes(const spf_ctx* c);

// Eccentricity estimate of every node (hop counts, drains ignored): the
// largest BFS distance from a few landmarks -- the node farthest from node
// 0, then repeatedly the node farthest from every landmark so far (on a grid:
// the corners, which makes it exact).  Cached per graph epoch.
const std::vector<uint32_t>& ecc_estimate(spf_ctx* c) {
  if (c->ecc_epoch == c->epoch && c->ecc.size() == c->N) return c->ecc;
  const uint32_t N = c->N;
  std::vector<uint32_t> d(N), mind(N, kInf), q;
  c->ecc.assign(N, 0);
  auto bfs = [&](uint32_t r) {
    std::fill(d.begin(), d.end(), kInf);
    d[r] = 0;
    q.assign(1, r);
    for (size_t h = 0; h < q.size(); ++h) {
      const uint32_t u = q[h];
      for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
        if (d[c->col[e]] == kInf) {
          d[c->col[e]] = d[u] + 1;
          q.push_back(c->col[e]);
        }
    }
  };
  uint32_t land = 0;
  for (int j = 0; j < 9 && N; ++j) {
    bfs(land);
    uint32_t far = land, best = 0;
    for (uint32_t v = 0; v < N; ++v) {
      if (d[v] == kInf) continue;
      if (j > 0) c->ecc[v] = std::max(c->ecc[v], d[v]);  // landmark 0 (node 0's far end) onwards
      mind[v] = std::min(mind[v], d[v]);
      if (j == 0 ? d[v] > best : mind[v] > best) {
        best = j == 0 ? d[v] : mind[v];
        far = v;
      }
    }
    if (j == 0) std::fill(mind.begin(), mind.end(), kInf);  // node 0 is no landmark
    land = far;
  }
  c->ecc_epoch = c->epoch;
  return c->ecc;
}

// An upper bound on every hop distance of the graph (any source, drained
// nodes expanded only as the source, LinkState.cpp:831-838): paths run
// s -> x -> ... -> y -> v with x .. y in H = the non-drained nodes, so
// d(s, v) <= 2 + d_H(x, y) <= 2 + 2 ecc_H(r) for any r of x's component of
// H.  One BFS in H per component.  Plans whose rows cannot saturate the u8
// copy (bound < 254) never need u32 rows of non-source closure rows.
uint32_t depth_bound(spf_ctx* c) {
  if (c->dbound_epoch == c->epoch) return c->dbound;
  for (const auto& m : c->dbound_memo)  // the same structure and drain bits as a recent epoch
    if (m.sell_ver == c->sell_ver && m.ovl == c->ovl) {
      c->dbound = m.dbound;
      c->dbound_epoch = c->epoch;
      return c->dbound;
    }
  // one level-synchronous BFS per component over the distinct up neighbours;
  // drained nodes are neither roots nor transit, so they start out seen (one
  // byte test per edge -- recomputed after every patch, on the path of the
  // first plan build of a publication)
  const uint32_t N = c->N;
  std::vector<uint8_t> seen(N);
  for (uint32_t v = 0; v < N; ++v) seen[v] = c->ovl[v] != 0;
  std::vector<uint32_t> q(std::max<uint32_t>(N, 1));
  const uint32_t* nbp = c->nb_ptr.data();
  const uint32_t* nbi = c->nb_id.data();
  uint32_t worst = 0;
  for (uint32_t r = 0; r < N; ++r) {
    if (seen[r]) continue;
    seen[r] = 1;
    size_t head = 0, tail = 0, level_end = 1;
    q[tail++] = r;
    uint32_t ecc = 0;
    while (head < tail) {
      const uint32_t u = q[head++];
      for (uint32_t e = nbp[u]; e < nbp[u + 1]; ++e) {
        const uint32_t x = nbi[e];
        if (!seen[x]) {
          seen[x] = 1;
          q[tail++] = x;
        }
      }
      if (head == level_end && head < tail) {  // the next level starts
        ++ecc;
        level_end = tail;
      }
    }
    worst = std::max(worst, ecc);
  }
  c->dbound = 2 + 2 * worst;
  c->dbound_epoch = c->epoch;
  if (c->dbound_memo.size() >= 4) c->dbound_memo.erase(c->dbound_memo.begin());
  c->dbound_memo.push_back({c->sell_ver, c->ovl, c->dbound});
  return c->dbound;
}

bool use_narrow(const spf_ctx* c, const spf_plan* p) {
  if (const char* e = std::getenv("SPF_NARROW")) return e[0] != '0';
  // the register-plane BFS writes each row once, coalesced: the u8 copy
  // costs one more row store and the next-hop pass reads 4x fewer bytes
  if (use_planes(c)) return true;
  uint64_t nb = 0;
  for (uint32_t i = 0; i < p->n_src; ++i) nb += p->words[i];
  return nb >= 8ull * p->n_src;  // average distinct degree >= 8
}

// Everything a plan derives from the graph's current state (closure over
// non-drained neighbours, narrow/exact mode, next-hop row tables).  Run at
// creation and again by spf_plan_execute after an in-place graph patch
// (spf_graph_set_overload / spf_graph_set_metric); the output layout
// (nh_off, words) depends only on the CSR structure, which patches keep.
spf_status build_plan(spf_ctx* c, spf_plan* p) {
  // SPF_PLAN_DEBUG: per-phase host time of the build on stderr (diagnostics)
  static const bool pd_on = std::getenv("SPF_PLAN_DEBUG") != nullptr;
  auto pd_t0 = std::chrono::steady_clock::now();
  auto PD = [&](const char* what) {
    if (!pd_on) return;
    (void)hipStreamSynchronize(c->stream);
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "build_plan %s %.1f us\n", what, std::chrono::duration<double, std::micro>(t - pd_t0).count());
    pd_t0 = t;
  };
  const uint32_t n_src = p->n_src;
  const uint32_t* srcs = p->srcs.data();
  const bool hop = (p->flags & SPF_FLAG_HOP_COUNT) != 0;
  const bool d64 = (p->flags & SPF_FLAG_DIST64) != 0;
  if (!hop && c->needs64 && !d64)
    return fail(c, SPF_E_UNSUPPORTED,
                "weighted distances of this graph may exceed 32 bits (negative metric or max "
                "metric x hops >= 2^32): create the plan with SPF_FLAG_DIST64");
  const uint32_t N = c->N;
  // the exact kernel replays runSpf step for step: zero-metric plateaus
  // (pop order), u64 labels, and graphs whose distance rows do not fit the
  // LDS-resident kernels
  const bool ms_ok = (hop || c->unit) && N <= kMsMaxNodes;
  const bool lds_ok = sssp_lds_bytes(N, c->pitch, c->big_nodes, N <= 65535) <= kMaxLds;
  p->exact = d64 || (!hop && c->nonpos);
  // graphs beyond the LDS-resident kernels: the whole chip per source
  // (spf_big_kernel); SPF_BIG=0 sends them to the exact kernel, SPF_BIG=1
  // sends every plan it can take there (tests)
  const char* be = std::getenv("SPF_BIG");
  p->big = !p->exact && ((!ms_ok && !lds_ok) ? !(be && be[0] == '0') : (be && be[0] == '1'));
  if (!ms_ok && !lds_ok && !p->big) p->exact = true;
  if (p->exact || p->big) {
    p->closure = p->srcs;
    p->direct = true;
    p->ms = false;
    p->narrow = false;
    p->sliced = false;
    p->expand = false;
    p->nh_off.resize(n_src);
    p->words.resize(n_src);
    uint64_t off = 0;
    p->wmax = 1;
    for (uint32_t i = 0; i < n_src; ++i) {
      const uint32_t k = c->nb_ptr[srcs[i] + 1] - c->nb_ptr[srcs[i]];
      p->words[i] = k;
      p->nh_off[i] = off;
      off += (uint64_t)k * (c->pitch / 32);
      p->wmax = std::max(p->wmax, (k + 31) / 32);
    }
    p->nh_total = off;
    HIP_TRY(c, hipSetDevice(c->device));
    if (p->exact) {
      const spf_status st = exact_reserve(c, &p->xs, n_src, p->wmax);
      if (st != SPF_OK) return st;
    }
    HIP_TRY(c, stage_upload(c, p->d_srcs, p->srcs.data(), n_src));
    HIP_TRY(c, stage_upload(c, p->d_nh_off, p->nh_off.data(), n_src));
    HIP_TRY(c, stage_upload(c, p->d_words, p->words.data(), n_src));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    stage_done(c);
    p->epoch = c->epoch;
    return SPF_OK;
  }
  PD("start");
  p->closure.clear();
  std::vector<uint32_t> row_of(N, kInf);
  bool distinct = true;
  for (uint32_t i = 0; i < n_src; ++i) {
    if (row_of[srcs[i]] != kInf) distinct = false;
    else row_of[srcs[i]] = i;
  }
  // closure: every non-overloaded neighbour's distance row is needed
  bool closed = distinct;
  if (closed) {
    for (uint32_t i = 0; i < n_src && closed; ++i) {
      const uint32_t s = srcs[i];
      for (uint32_t j = c->nb_ptr[s]; j < c->nb_ptr[s + 1]; ++j) {
        const uint32_t x = c->nb_id[j];
        if (!c->ovl[x] && row_of[x] == kInf) {
          closed = false;
          break;
        }
      }
    }
  }
  p->direct = closed;
  if (closed) {
    p->closure = p->srcs;
  } else {
    std::fill(row_of.begin(), row_of.end(), kInf);
    auto add = [&](uint32_t x) {
      if (row_of[x] == kInf) {
        row_of[x] = (uint32_t)p->closure.size();
        p->closure.push_back(x);
      }
    };
    // distinct sources first (rows 0 .. n_src - 1 are the request's rows:
    // kernels that can write a row prefix straight into the caller's buffer
    // do, msbfs_team_kernel), then the neighbours the next-hop pass reads
    if (distinct)
      for (uint32_t i = 0; i < n_src; ++i) add(srcs[i]);
    for (uint32_t i = 0; i < n_src; ++i) {
      const uint32_t s = srcs[i];
      add(s);
      for (uint32_t j = c->nb_ptr[s]; j < c->nb_ptr[s + 1]; ++j)
        if (!c->ovl[c->nb_id[j]]) add(c->nb_id[j]);
    }
  }
  // closure[i] == srcs[i] for i < n_src, and no row can saturate the u8
  // copy (whose saturated entries the next-hop pass reads from u32 rows)
  p->prefix = distinct && depth_bound(c) < kSlSat;
  std::vector<uint32_t> req_rows(n_src);
  for (uint32_t i = 0; i < n_src; ++i) req_rows[i] = row_of[srcs[i]];
  // next-hop layout
  p->nh_off.resize(n_src);
  p->words.resize(n_src);
  uint64_t off = 0;
  for (uint32_t i = 0; i < n_src; ++i) {
    const uint32_t k = c->nb_ptr[srcs[i] + 1] - c->nb_ptr[srcs[i]];
    p->words[i] = k;  // one destination bitmap per distinct up neighbour
    p->nh_off[i] = off;
    off += (uint64_t)k * (c->pitch / 32);
  }
  p->nh_total = off;
  p->q16 = N <= 65535;
  p->lds_bytes = sssp_lds_bytes(N, c->pitch, c->big_nodes, p->q16);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, stage_upload(c, p->d_srcs, p->srcs.data(), n_src));
  HIP_TRY(c, stage_upload(c, p->d_closure, p->closure.data(), p->closure.size()));
  HIP_TRY(c, stage_upload(c, p->d_row_of, row_of.data(), N));
  HIP_TRY(c, stage_upload(c, p->d_req_rows, req_rows.data(), n_src));
  HIP_TRY(c, stage_upload(c, p->d_nh_off, p->nh_off.data(), n_src));
  HIP_TRY(c, stage_upload(c, p->d_words, p->words.data(), n_src));
  p->ms = (hop || c->unit) && N <= kMsMaxNodes;
  // register-plane BFS: batches of similar depth, deepest first (more than
  // one round of batches only; SPF_PL_ORDER=0 keeps the plan order, A/B)
  p->pl_order = false;
  if (p->ms && use_planes(c) && p->closure.size() > (size_t)kPlBatch * c->n_cu) {
    const char* e = std::getenv("SPF_PL_ORDER");
    if (!(e && e[0] == '0')) {
      const std::vector<uint32_t>& ecc = ecc_estimate(c);
      std::vector<uint32_t> order(p->closure.size());
      std::iota(order.begin(), order.end(), 0u);
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return ecc[p->closure[a]] > ecc[p->closure[b]];
      });
      HIP_TRY(c, stage_upload(c, p->d_pl_order, order.data(), order.size()));
      p->pl_order = true;
    }
  }
  // few batches (a rank's share of a multi-GPU pass): teams of workgroups
  // per batch (msbfs_team.hip) instead of one workgroup sweeping everything
  PD("uploads1");
  p->tm_G = 0;
  if (p->ms && !use_planes(c) && !p->expand && !c->team_off) {
    const uint32_t G = msbfs_team_size(c, (uint32_t)p->closure.size());
    if (G) {
      const spf_status st = msbfs_team_prepare(c, p, G);
      if (st != SPF_OK) return st;
    }
  }
  // weighted: S sources per workgroup on mssp_kernel where it applies
  PD("team");
  p->mp = !p->ms && !hop && mssp_words(c) > 0;
  if (p->mp) {
    const spf_status st = mssp_prepare(c);
    if (st != SPF_OK) return st;
    HIP_TRY(c, p->d_redo.alloc(1 + p->closure.size()));
  }
  // weighted plans keep a u8 copy too when the pitches agree (the sssp
  // kernel writes it beside the u32 row; the next-hop pass compares bytes and
  // falls back to u32 rows per wave where the source's row saturates)
  p->narrow = (p->ms || c->pitch == c->npitch) && use_narrow(c, p);
  // bit-sliced rows behind the per-level-store BFS (it reports the deepest
  // level); the register-plane BFS serves deep graphs, where planes would
  // not pay.  SPF_NARROW=1 keeps the byte-row pass (experiments, tests).
  {
    const char* e = std::getenv("SPF_NARROW");
    p->sliced = p->ms && p->narrow && !use_planes(c) && !(e && e[0] == '1');
    // weighted plans on mssp_kernel: its u8 rows sliced too, next hops by
    // bit-sliced sums d_x + w (sliced_pass<P, true>); SPF_WSLICED=0: byte rows
    const char* ws = std::getenv("SPF_WSLICED");
    if (p->mp && p->narrow && !(e && e[0] == '1') && !(ws && ws[0] == '0')) p->sliced = true;
    // SPF_EXPAND=1 (A/B; measured slower): the BFS stores the u8
    // rows only and the slicing pass expands them into the u32 rows.  By
    // default the BFS stores both: its u32 stores drain behind its
    // latency-bound sweeps (+0.06 ms on fabric_full) where a separate
    // streaming pass costs 0.14 ms and a fused one 0.14 ms of the next-hop
    // kernel's time (r02_v25/r02_v26)
    const char* x = std::getenv("SPF_EXPAND");
    p->expand = p->sliced && c->pitch <= c->npitch && x && x[0] == '1';
    // team plans whose depth stays below the planes' all-ones code write the
    // sliced rows themselves: no u8 rows, no slicing pass (SPF_SDIRECT=0: A/B)
    const char* sd = std::getenv("SPF_SDIRECT");
    p->sdirect = p->sliced && p->nh_total && p->tm_G && p->prefix && !p->expand &&
                 depth_bound(c) < (1u << kTeamPlanes) - 1 && !(sd && sd[0] == '0');
  }
  const uint32_t wpm = c->pitch / 32;
  const uint64_t rstride = (uint64_t)kSlSlots * wpm;  // sliced row: words
  {
    // per-source neighbour rows for the next-hop pass (kInf = drained)
    std::vector<uint32_t> nb_row, nb_row_off(n_src), nb_drained(n_src, 0);
    const uint32_t dead = p->sliced   ? (uint32_t)(p->closure.size() * rstride)
                          : p->narrow ? (uint32_t)p->closure.size() * c->npitch
                                      : kInf;
    p->dead = dead;
    for (uint32_t i = 0; i < n_src; ++i) {
      nb_row_off[i] = (uint32_t)nb_row.size();
      for (uint32_t e = c->nb_ptr[srcs[i]]; e < c->nb_ptr[srcs[i] + 1]; ++e) {
        const uint32_t x = c->nb_id[e];
        const bool dr = c->ovl[x] != 0;
        nb_row.push_back(dr          ? dead
                         : p->sliced ? (uint32_t)(row_of[x] * rstride)
                         : p->narrow ? row_of[x] * c->npitch
                                     : row_of[x]);
        nb_drained[i] += dr;
      }
      const size_t k = nb_row.size() - nb_row_off[i];
      nb_row.resize(nb_row_off[i] + (k + 7) / 8 * 8 + 8, dead);
    }
    HIP_TRY(c, stage_upload(c, p->d_nb_row, nb_row.data(), nb_row.size()));
    HIP_TRY(c, stage_upload(c, p->d_nb_row_off, nb_row_off.data(), n_src));
    HIP_TRY(c, stage_upload(c, p->d_nb_drained, nb_drained.data(), n_src));
    // next-hop blocks per XCD: runs of consecutive sources of about
    // 1/(8 * runs) of the work each, every run to the XCD with the least
    // work so far (runs come in request order: the heavy spine and fabric
    // switches first)
    // (a rank's share of a multi-GPU pass -- ~1.3k sources -- does best with
    // two long runs per XCD: 0.097 -> 0.095 ms per world-8 rank, r03_v25)
    const char* env = std::getenv("SPF_ECMP_RUNS");
    const uint32_t runs = env ? (uint32_t)atoi(env) : n_src >= 4096 ? kEcmpRunsPerXcd : 2u;
    std::vector<uint32_t> lists[8];
    if (runs == 0) {  // plain round-robin
      for (uint32_t i = 0; i < n_src; ++i) lists[i % 8].push_back(i);
    } else {
      uint64_t total = 0, load[8] = {};
      for (uint32_t i = 0; i < n_src; ++i) total += p->words[i] + 1;
      const uint64_t target = std::max<uint64_t>(1, total / (8ull * runs));
      for (uint32_t i = 0; i < n_src;) {
        uint32_t e = i;
        uint64_t w = 0;
        while (e < n_src && w < target) w += p->words[e++] + 1;
        const int g = (int)(std::min_element(load, load + 8) - load);
        load[g] += w;
        for (uint32_t t = i; t < e; ++t) lists[g].push_back(t);
        i = e;
      }
    }
    PD("nb_rows");
    if (p->sliced) {
      // sliced-pass work units per XCD, in the XCD's source order: a source
      // whose neighbour-chunk matches fit kSlUnit is one unit, a heavier one
      // is cut per chunk and per neighbour range (multiples of 8: the row
      // offset lists are read 16-byte aligned)
      const uint32_t chunks = (wpm + 63) / 64;
      const char* ue = std::getenv("SPF_SLICED_UNIT");  // A/B knob
      // small plans (a rank's share of a multi-GPU pass) get smaller units so
      // the waves still cover the chip: about 16 units per CU, 16..kSlUnit
      uint64_t matches = 0;
      for (uint32_t i = 0; i < n_src; ++i) matches += (uint64_t)p->words[i] * chunks;
      const uint32_t fill = (uint32_t)std::min<uint64_t>(
          kSlUnit, std::max<uint64_t>(16, matches / (16ull * c->n_cu) / 8 * 8));
      const uint32_t unit = ue ? (uint32_t)atoi(ue) : fill;
      std::vector<uint32_t> units, unit_off(9, 0), gtab;
      // Grouped units: neighbour positions are cut into segments of kSlSeg;
      // sources of one XCD list whose segment q holds the same rows (none
      // drained) share it -- one wave loads each of those rows once for up
      // to kSlGroup sources.  Whole lists match for a pod's rack switches and
      // a plane's spines; a fabric switch's list is [its plane's spines][its
      // pod's rack switches], so the fabric switches of one plane share the
      // first part and those of one pod the second.  Consecutive segments of
      // one member set merge into one range; what no group takes stays with
      // per-source units.  (SPF_SLICED_GROUP=0: no groups, =1: whole
      // identical lists only -- round 3's rule; A/B.)
      const char* ge = std::getenv("SPF_SLICED_GROUP");
      // (weighted plans: no groups -- members share neighbour rows, not metrics)
      const int gmode = p->mp ? 0 : ge ? atoi(ge) : 2;
      p->max_xcd_units = 0;
      for (int g = 0; g < 8; ++g) {
        unit_off[g] = (uint32_t)(units.size() / 4);
        // per source of the list: which segments a group took
        std::map<uint32_t, std::vector<uint8_t>> taken;
        // member set -> segments (q, end position) it shares
        std::map<std::vector<uint32_t>, std::vector<std::pair<uint32_t, uint32_t>>> shared;
        if (gmode) {
          std::map<std::vector<uint32_t>, std::vector<uint32_t>> seg;
          for (uint32_t i : lists[g]) {
            const uint32_t k = p->words[i];
            if (!k) continue;
            const uint32_t* r = nb_row.data() + nb_row_off[i];
            if (gmode == 1) {  // the whole list as one key
              if (nb_drained[i]) continue;
              std::vector<uint32_t> key{0u, k};
              key.insert(key.end(), r, r + k);
              seg[key].push_back(i);
              continue;
            }
            for (uint32_t q = 0; q * kSlSeg < k; ++q) {
              const uint32_t j = q * kSlSeg, e = std::min(k, j + kSlSeg);
              bool dead_in = false;
              for (uint32_t jj = j; jj < e; ++jj) dead_in |= r[jj] == dead;
              if (dead_in) continue;
              std::vector<uint32_t> key{q, e};
              key.insert(key.end(), r + j, r + e);
              seg[key].push_back(i);
            }
          }
          for (auto& kv : seg) {
            const auto& src = kv.second;
            for (size_t a = 0; a + 1 < src.size(); a += kSlGroup) {
              const size_t b = std::min(src.size(), a + kSlGroup);
              if (b - a < 2) break;
              std::vector<uint32_t> m(src.begin() + a, src.begin() + b);
              const uint32_t q = kv.first[0], e = kv.first[1];
              if (gmode == 1) {  // whole list: every segment of it
                for (uint32_t qq = 0; qq * kSlSeg < e; ++qq)
                  shared[m].emplace_back(qq, std::min(e, (qq + 1) * kSlSeg));
              } else {
                shared[m].emplace_back(q, e);
              }
              for (uint32_t i : m) {
                auto& t = taken[i];
                if (t.empty()) t.assign((p->words[i] + kSlSeg - 1) / kSlSeg, 0);
                if (gmode == 1)
                  std::fill(t.begin(), t.end(), 1);
                else
                  t[q] = 1;
              }
            }
          }
        }
        // group units: per member set, runs of consecutive segments, per
        // chunk, ranges of about `unit` matches (multiples of kSlSeg)
        for (auto& kv : shared) {
          auto& segs = kv.second;
          std::sort(segs.begin(), segs.end());
          const uint32_t gs = (uint32_t)kv.first.size();
          const uint32_t goff = (uint32_t)gtab.size();
          gtab.push_back(gs);
          gtab.insert(gtab.end(), kv.first.begin(), kv.first.end());
          for (size_t a = 0; a < segs.size();) {
            size_t b = a + 1;
            while (b < segs.size() && segs[b].first == segs[b - 1].first + 1) ++b;
            const uint32_t j0 = segs[a].first * kSlSeg, j1 = segs[b - 1].second;
            const uint32_t parts = (uint32_t)(((uint64_t)(j1 - j0) * gs + unit - 1) / unit);
            const uint32_t jstep = ((j1 - j0 + parts - 1) / parts + kSlSeg - 1) / kSlSeg * kSlSeg;
            for (uint32_t ch = 0; ch < chunks; ++ch)
              for (uint32_t j = j0; j < j1; j += jstep)
                units.insert(units.end(), {goff, ch | (1u << 31), j, std::min(j1, j + jstep)});
            a = b;
          }
        }
        // per-source units over what no group took
        for (uint32_t i : lists[g]) {
          const uint32_t k = p->words[i];
          if (k == 0) continue;
          const auto it = taken.find(i);
          const std::vector<uint8_t>* t = it == taken.end() ? nullptr : &it->second;
          for (uint32_t q = 0; q * kSlSeg < k;) {
            if (t && (*t)[q]) {
              ++q;
              continue;
            }
            uint32_t q1 = q + 1;
            while (q1 * kSlSeg < k && !(t && (*t)[q1])) ++q1;
            const uint32_t j0 = q * kSlSeg, j1 = std::min(k, q1 * kSlSeg), kr = j1 - j0;
            if ((uint64_t)kr * chunks <= unit) {
              units.insert(units.end(), {i, 0u | (chunks << 16), j0, j1});
            } else {  // per chunk, equal ranges of <= unit neighbours (multiples of kSlSeg)
              const uint32_t parts = (kr + unit - 1) / unit;
              const uint32_t jstep = ((kr + parts - 1) / parts + kSlSeg - 1) / kSlSeg * kSlSeg;
              for (uint32_t ch = 0; ch < chunks; ++ch)
                for (uint32_t j = j0; j < j1; j += jstep)
                  units.insert(units.end(), {i, ch | ((ch + 1) << 16), j, std::min(j1, j + jstep)});
            }
            q = q1;
          }
        }
        p->max_xcd_units = std::max(p->max_xcd_units, (uint32_t)(units.size() / 4) - unit_off[g]);
      }
      unit_off[8] = (uint32_t)(units.size() / 4);
      if (units.empty()) units.assign(4, 0);
      HIP_TRY(c, stage_upload(c, p->d_units, units.data(), units.size()));
      HIP_TRY(c, stage_upload(c, p->d_unit_off, unit_off.data(), 9));
      if (gtab.empty()) gtab.push_back(0);
      HIP_TRY(c, stage_upload(c, p->d_gtab, gtab.data(), gtab.size()));
    }
    size_t most = 0;
    for (auto& l : lists) most = std::max(most, l.size());
    std::vector<uint32_t> slot(most * 8, kInf);
    for (int g = 0; g < 8; ++g)
      for (size_t t = 0; t < lists[g].size(); ++t) slot[t * 8 + g] = lists[g][t];
    p->slots = slot.size();
    if (slot.empty()) slot.push_back(kInf);
    HIP_TRY(c, stage_upload(c, p->d_slot_src, slot.data(), slot.size()));
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // host vectors end here
    stage_done(c);
  }
  PD("units+slots");
  if (!p->direct) HIP_TRY(c, p->d_D.alloc((size_t)p->closure.size() * c->pitch));
  if (p->narrow && !p->sdirect) {  // narrow rows + the dead row (all 0xFF) of the next-hop pass
    HIP_TRY(c, p->d_Dn.alloc((p->closure.size() + 1) * c->npitch));
    HIP_TRY(c, hipMemsetAsync(p->d_Dn.p + p->closure.size() * c->npitch, 0xFF, c->npitch, c->stream));
  }
  if (p->sliced) {  // sliced rows + the dead row (all planes all-ones) + padding
    const size_t rows = p->closure.size();
    // a wave's last chunk reads up to 64 * kSlSlots words past a row's end
    const size_t pad = 64 * kSlSlots + 64;
    if (((rows + 1) * rstride + pad) * 4 >= (1ull << 31))  // buffer byte offsets
      return fail(c, SPF_E_UNSUPPORTED, "sliced rows exceed 32-bit offsets");
    HIP_TRY(c, p->d_S.alloc((rows + 1) * rstride + pad));
    HIP_TRY(c, hipMemsetAsync(p->d_S.p + rows * rstride, 0xFF, (rstride + pad) * 4, c->stream));
    HIP_TRY(c, p->d_maxd.alloc(1));
  }
  {
    const spf_status st = set_lds_limits(c);  // kernels need > 64 KiB of dynamic LDS
    if (st != SPF_OK) return st;
  }
  PD("allocs");
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  stage_done(c);
  p->epoch = c->epoch;
  return SPF_OK;
}

}  // namespace

extern "C" {

spf_status spf_plan_create(spf_ctx* c, const uint32_t* srcs, uint32_t n_src,
                           uint32_t flags, spf_plan** out) {
  if (!c || !out) return fail(c, SPF_E_INVALID, "spf_plan_create: NULL argument");
  *out = nullptr;
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (n_src == 0 || !srcs) return fail(c, SPF_E_INVALID, "empty source list");
  for (uint32_t i = 0; i < n_src; ++i)
    if (srcs[i] >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", srcs[i]);
  auto p = std::make_unique<spf_plan>();
  p->ctx = c;
  p->n_src = n_src;
  p->flags = flags;
  p->srcs.assign(srcs, srcs + n_src);
  p->shape = c->shape;
  p->layout = c->layout;
  const spf_status st = build_plan(c, p.get());
  if (st != SPF_OK) return st;
  *out = p.release();
  return SPF_OK;
}


void spf_plan_destroy(spf_plan* p) { delete p; }
uint64_t spf_plan_nh_words(const spf_plan* p) { return p ? p->nh_total : 0; }
uint32_t spf_plan_closure_rows(const spf_plan* p) { return p ? (uint32_t)p->closure.size() : 0; }

spf_status spf_plan_kernels(const spf_plan* p, uint32_t* bfs, uint32_t* narrow) {
  if (!p || !bfs || !narrow) return SPF_E_INVALID;
  *bfs = p->big ? 4u : p->exact ? 3u : p->mp ? 5u : !p->ms ? 0u : p->tm_G ? 6u
                                                          : use_planes(p->ctx) ? 2u : 1u;
  *narrow = p->sdirect ? 3u : p->sliced ? 2u : p->narrow ? 1u : 0u;
  return SPF_OK;
}

// Bytes each kernel of one execute must move between HBM and the CUs, given
// the kernel's own structure: what `roofline.achieved` in bench.py divides by
// the kernel's measured time (no credit for on-chip reuse).
//   BFS (msbfs / planes): one read of the sliced-ELL columns and the drain
//     bytes per workgroup (a batch of sources shares one sweep per level;
//     repeated levels hit the L2), plus the distance rows (u32, pitch) and,
//     in narrow mode, the u8 rows (npitch) written once.
//   SSSP (weighted, one workgroup per source): one read of row_ptr, col,
//     metric and drain bytes per source, plus the distance row written.
//   ECMP: every distance row it compares read once (u8 rows in narrow mode,
//     u32 rows otherwise) plus the next-hop bitmaps written once.
spf_status spf_plan_traffic(const spf_plan* p, uint64_t* bfs_bytes, uint64_t* ecmp_bytes) {
  if (!p || !bfs_bytes || !ecmp_bytes) return SPF_E_INVALID;
  uint64_t b[3];
  const spf_status st = spf_plan_traffic_phases(p, b);
  if (st != SPF_OK) return st;
  *bfs_bytes = b[0];
  *ecmp_bytes = b[1] + b[2];
  return SPF_OK;
}

//   Slicing (sliced plans): the u8 rows read, P planes per row written (and,
//     in expand plans, the u32 rows); the sliced next-hop pass then reads P
//     planes per row and writes the bitmaps.
spf_status spf_plan_traffic_phases(const spf_plan* p, uint64_t* bytes) {
  if (!p || !bytes) return SPF_E_INVALID;
  uint64_t* bfs_bytes = &bytes[0];
  uint64_t* ecmp_bytes = &bytes[2];
  bytes[1] = 0;
  const spf_ctx* c = p->ctx;
  const uint64_t N = c->N, E = c->E, rows = p->closure.size();
  uint64_t bfs = 0;
  if (p->big) {  // per source: the CSR a few sweeps (counted once), the row, scratch + bitmaps
    *bfs_bytes = rows * (4ull * (N + 1) + 12ull * E + N + 4ull * c->pitch) + 4ull * p->nh_total;
    *ecmp_bytes = 0;
    return SPF_OK;
  }
  if (p->exact) {  // per source: the CSR once, the labels, the outputs
    const uint64_t lab = (p->flags & SPF_FLAG_DIST64) ? 8ull : 4ull;
    *bfs_bytes = rows * (4ull * (N + 1) + 12ull * E + N + 17ull * N + lab * c->pitch) +
                 4ull * p->nh_total;
    *ecmp_bytes = 0;
    return SPF_OK;
  }
  if (p->tm_G) {  // team BFS: each batch sweeps the column stream once (column + meta
                  // words); rows written: u32 for the prefix when direct, u8 or planes
    const uint64_t batches = (rows + p->tm_bs - 1) / p->tm_bs;
    const bool direct = p->prefix && !p->direct && p->narrow;
    const uint64_t wbytes = 4ull * (c->pitch / 32);
    bfs = batches * (8ull * c->sell_ptr.back() + N) + (direct ? p->n_src : rows) * c->pitch * 4ull +
          (p->sdirect ? rows * kTeamPlanes * wbytes : p->narrow ? rows * c->npitch : 0ull);
  } else if (p->ms) {
    const bool planes = use_planes(c);
    const uint32_t batch = planes ? kPlBatch : kMsBatch;
    const uint64_t rounds = (rows + (uint64_t)batch * c->n_cu - 1) / ((uint64_t)batch * c->n_cu);
    const uint64_t bs = std::min<uint64_t>(batch, (rows + rounds * c->n_cu - 1) / (rounds * c->n_cu));
    const uint64_t groups = (rows + bs - 1) / bs;
    const uint64_t n_slices = c->sell_ptr.size() - 1;
    const uint64_t csr = planes ? 8ull * c->sell4_ptr.back() + 4ull * (n_slices + 1)
                                : 4ull * c->sell_ptr.back() + 4ull * (n_slices + 1);
    // expand plans: the u32 rows are written by the slicing pass instead
    bfs = groups * (csr + N) + (p->expand ? 0ull : rows * c->pitch * 4ull) +
          (p->narrow ? rows * c->npitch : 0ull);
  } else if (p->mp) {  // per workgroup: the packed ELL + slice map once; rows written once
    const uint64_t S = mssp_sources(c);
    const uint64_t groups = (rows + S - 1) / S;
    bfs = groups * (4ull * c->sell_ptr.back() + 4ull * c->sell_ptr.size() + 4ull * (N + 1) + N) +
          rows * (4ull * c->pitch + (p->narrow ? c->npitch : 0ull));
  } else {
    bfs = rows * (4ull * (N + 1) + 8ull * E + N + 4ull * c->pitch + (p->narrow ? c->npitch : 0ull));
  }
  *bfs_bytes = bfs;
  if (p->sliced && p->nh_total) {
    // planes in use: from the last execute's deepest level (one 4-byte read)
    // (sdirect: kTeamPlanes planes written by the BFS itself, no slicing pass)
    const uint64_t wbytes = 4ull * (c->pitch / 32);
    if (p->sdirect) {
      *ecmp_bytes = rows * kTeamPlanes * wbytes + 4ull * p->nh_total;
      return SPF_OK;
    }
    uint32_t md = 0;
    HIP_TRY(p->ctx, hipMemcpy(&md, p->d_maxd.p, 4, hipMemcpyDeviceToHost));
    const uint64_t expand = p->expand ? rows * 4ull * c->pitch : 0ull;  // u32 rows written
    if (md < kSlSat) {
      const uint64_t P = 32u - __builtin_clz(md + 1u);
      bytes[1] = rows * c->npitch + rows * P * wbytes + expand;
      *ecmp_bytes = rows * P * wbytes + 4ull * p->nh_total;
    } else {
      bytes[1] = expand ? rows * c->npitch + expand : 0ull;
      *ecmp_bytes = rows * 4ull * c->pitch + 4ull * p->nh_total;
    }
    return SPF_OK;
  }
  const uint64_t row_bytes = p->narrow ? c->npitch : 4ull * c->pitch;
  *ecmp_bytes = p->nh_total ? rows * row_bytes + 4ull * p->nh_total : 0ull;
  return SPF_OK;
}

spf_status spf_plan_nh_layout(const spf_plan* p, uint64_t* nh_off, uint32_t* words) {
  if (!p) return SPF_E_INVALID;
  for (uint32_t i = 0; i < p->n_src; ++i) {
    if (nh_off) nh_off[i] = p->nh_off[i];
    if (words) words[i] = p->words[i];
  }
  return SPF_OK;
}

}  // extern "C"

namespace {

}  // namespace

namespace spfi {

// Launch the SSSP kernel over `rows` closure rows (device list rows_src).
spf_status launch_sssp(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, bool hop,
                       const uint32_t* ign, uint32_t* D, hipStream_t s, const uint32_t* wt,
                       const uint8_t* ovl, uint8_t* Dn, const uint32_t* redo) {
  if (!wt) wt = c->d_wt.p;
  if (!ovl) ovl = c->d_ovl.p;
  const uint32_t N = c->N, pitch = c->pitch, bm_words = (N + 31) / 32;
  const bool q16 = N <= 65535;
  const size_t lds = sssp_lds_bytes(N, pitch, c->big_nodes, q16);
  const bool unit = hop || c->max_metric == 1;
  // threads per workgroup from how many workgroups the LDS row lets a CU hold
  // (SPF_SSSP_THREADS overrides, experiments)
  uint32_t threads = lds > kMaxLds / 3 ? 1024u : lds > kMaxLds / 6 ? 512u : 256u;
  if (const char* e = std::getenv("SPF_SSSP_THREADS")) threads = (uint32_t)atoi(e);
  const dim3 g(rows);
#define SSSP_LAUNCH(QT, U, TH)                                                            \
  hipLaunchKernelGGL((sssp_kernel<QT, U, TH>), g, dim3(TH), lds, s, c->d_row_ptr.p,       \
                     c->d_col.p, wt, ovl, c->d_link.p, ign, rows_src, N, pitch, bm_words,  \
                     c->big_nodes, D, Dn, redo)
#define SSSP_TH(QT, U)                                  \
  do {                                                  \
    if (threads >= 1024) SSSP_LAUNCH(QT, U, 1024);      \
    else if (threads >= 512) SSSP_LAUNCH(QT, U, 512);   \
    else SSSP_LAUNCH(QT, U, 256);                       \
  } while (0)
  if (q16) {
    if (unit) SSSP_TH(uint16_t, true);
    else SSSP_TH(uint16_t, false);
  } else {
    if (unit) SSSP_TH(uint32_t, true);
    else SSSP_TH(uint32_t, false);
  }
#undef SSSP_TH
#undef SSSP_LAUNCH
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

}  // namespace spfi

namespace {

size_t msbfs_lds_bytes(uint32_t N, bool db = false) {
  return 8ull * (N + 1) * (db ? 2 : 1) + 4ull * (4 * kMsBatch + 5);
}

// msbfs_kernel with a double-buffered frontier: when the columns do not fit
// in LDS beside one F array but two F arrays do (SPF_MSBFS_DB=0: single, A/B)
bool ms_double_buffer(const spf_ctx* c) {
  const char* e = std::getenv("SPF_MSBFS_DB");
  if (e && e[0] == '0') return false;
  const size_t n_col = c->sell_ptr.back();
  return msbfs_lds_bytes(c->N) + 2ull * n_col > kMaxLds && msbfs_lds_bytes(c->N, true) <= kMaxLds;
}

template <int OWN>
void msbfs_launch(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, uint32_t* D, uint8_t* Dn,
                  uint32_t* maxd, uint32_t d_from, hipStream_t s) {
  const uint32_t n_col = c->sell_ptr.back();
  const size_t lds = msbfs_lds_bytes(c->N), lds_col = lds + 2ull * n_col;
  const bool lcol = lds_col <= kMaxLds;
  // one workgroup per CU per round: a batch costs one edge sweep per level
  // whatever its size, but its stores scale with it, so spread the sources
  // over every CU rather than fill 64-source batches on fewer CUs
  const uint32_t rounds = (rows + kMsBatch * c->n_cu - 1) / (kMsBatch * c->n_cu);
  const uint32_t bs = std::min<uint32_t>(kMsBatch, (rows + rounds * c->n_cu - 1) / (rounds * c->n_cu));
  if (lcol)
    hipLaunchKernelGGL((msbfs_kernel<OWN, true>), dim3((rows + bs - 1) / bs), dim3(kMsThreads),
                       lds_col, s, c->d_sell_ptr.p, c->d_sell_col.p, n_col, c->d_row_ptr.p, c->d_col.p,
                       c->d_ovl.p, rows_src, rows, bs, c->N, c->pitch, c->npitch, D, Dn,
                       maxd, d_from, c->d_ms_smap.p, c->d_stamps.p);
  else if (ms_double_buffer(c))
    hipLaunchKernelGGL((msbfs_kernel<OWN, false, true>), dim3((rows + bs - 1) / bs), dim3(kMsThreads),
                       msbfs_lds_bytes(c->N, true), s, c->d_sell_ptr.p, c->d_sell_col.p, n_col,
                       c->d_row_ptr.p, c->d_col.p, c->d_ovl.p, rows_src, rows, bs, c->N, c->pitch,
                       c->npitch, D, Dn, maxd, d_from, c->d_ms_smap.p, c->d_stamps.p);
  else
    hipLaunchKernelGGL((msbfs_kernel<OWN, false>), dim3((rows + bs - 1) / bs), dim3(kMsThreads),
                       lds, s, c->d_sell_ptr.p, c->d_sell_col.p, n_col, c->d_row_ptr.p, c->d_col.p,
                       c->d_ovl.p, rows_src, rows, bs, c->N, c->pitch, c->npitch, D, Dn,
                       maxd, d_from, c->d_ms_smap.p, c->d_stamps.p);
}

size_t planes_lds_bytes(uint32_t own) { return 8ull * own * kMsThreads + 4ull * (kPlBatch + 4); }

//   order (optional): rows sorted by estimated eccentricity, deepest first.
//   A batch runs until its deepest source's search ends, so batches of
//   similar depth waste no levels, and the deep ones start first while the
//   shallow ones fill the CUs that free up (grid 100x100: eccentricities
//   100..198; 313 full batches are 1.22 rounds of the chip); without it the
//   batches are spread evenly over rounds.
template <int OWN>
void planes_launch(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, uint32_t* D, uint8_t* Dn,
                   const uint32_t* order, hipStream_t s) {
  const uint32_t n4 = c->sell4_ptr.back();
  const size_t lds = planes_lds_bytes(OWN), lds_col = lds + 8ull * n4;
  const bool lcol = lds_col <= kMaxLds;
  const uint32_t rounds = (rows + kPlBatch * c->n_cu - 1) / (kPlBatch * c->n_cu);
  const uint32_t bs = order ? kPlBatch
                            : std::min<uint32_t>(kPlBatch, (rows + rounds * c->n_cu - 1) / (rounds * c->n_cu));
  const uint2* col4 = reinterpret_cast<const uint2*>(c->d_sell4.p);
  if (lcol)
    hipLaunchKernelGGL((msbfs_planes_kernel<OWN, true>), dim3((rows + bs - 1) / bs), dim3(kMsThreads),
                       lds_col, s, c->d_sell4_ptr.p, col4, n4, c->d_ovl.p, rows_src, rows, bs, c->N,
                       c->pitch, c->npitch, D, Dn, order);
  else
    hipLaunchKernelGGL((msbfs_planes_kernel<OWN, false>), dim3((rows + bs - 1) / bs), dim3(kMsThreads),
                       lds, s, c->d_sell4_ptr.p, col4, n4, c->d_ovl.p, rows_src, rows, bs, c->N,
                       c->pitch, c->npitch, D, Dn, order);
}

// Which BFS variant: the register-plane kernel needs N <= 10240; it wins
// when levels are many (partial-line rewrites dominate msbfs_kernel) and
// loses when the edge sweep dominates (it runs 32 sources per sweep, not
// 64).  SPF_MSBFS=planes|masks overrides (experiments).
bool use_planes(const spf_ctx* c) {
  if (c->N > 10 * (uint32_t)kMsThreads || c->sell4.empty()) return false;
  if (const char* e = std::getenv("SPF_MSBFS")) return e[0] == 'p';
  return c->sell_ptr.back() <= 8ull * c->N;  // sliced-ELL width <= 8 on average
}

spf_status launch_msbfs(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, uint32_t* D,
                        uint8_t* Dn, uint32_t* maxd, hipStream_t s, uint32_t d_from = 0,
                        const uint32_t* order = nullptr) {
  if (!c->d_stamps.p && std::getenv("SPF_STAMPS")) {
    HIP_TRY(c, c->d_stamps.alloc(kStampWords));
    HIP_TRY(c, hipMemsetAsync(c->d_stamps.p, 0, 64 * 16 * 8, s));
    const unsigned long long wg = std::strtoull(std::getenv("SPF_STAMPS"), nullptr, 10);
    HIP_TRY(c, hipMemcpyAsync(c->d_stamps.p + 64 * 16, &wg, 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  const uint32_t own = ms_own(c->N);
  if (use_planes(c)) {
    if (own <= 1) planes_launch<1>(c, rows_src, rows, D, Dn, order, s);
    else if (own <= 2) planes_launch<2>(c, rows_src, rows, D, Dn, order, s);
    else if (own <= 4) planes_launch<4>(c, rows_src, rows, D, Dn, order, s);
    else if (own <= 8) planes_launch<8>(c, rows_src, rows, D, Dn, order, s);
    else planes_launch<10>(c, rows_src, rows, D, Dn, order, s);
    HIP_TRY(c, hipGetLastError());
    return SPF_OK;
  }
  if (own == 1) msbfs_launch<1>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  else if (own == 2) msbfs_launch<2>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  else if (own == 4) msbfs_launch<4>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  else if (own == 8) msbfs_launch<8>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  else if (own == 10) msbfs_launch<10>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  else if (own == 12) msbfs_launch<12>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  else msbfs_launch<16>(c, rows_src, rows, D, Dn, maxd, d_from, s);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

template <bool NARROW>
spf_status launch_ecmp(spf_ctx* c, spf_plan* p, const uint8_t* Dn, const uint32_t* D, bool hop,
                       uint32_t* d_nh, hipStream_t s) {
  const uint32_t per_block = kEcmpChunk * kEcmpWaves;
  const uint32_t chunks = (c->N + per_block - 1) / per_block;
  const uint32_t nb = chunks * (uint32_t)p->slots;
  const uint32_t weighted = NARROW && !hop && !c->unit ? 1u : 0u;
  hipLaunchKernelGGL((ecmp_kernel<NARROW>), dim3(nb), dim3(kEcmpThreads), 0, s, Dn, c->npitch, D,
                     c->pitch, c->N, p->d_srcs.p, p->d_row_of.p, c->d_nb_ptr.p, c->d_nb_id.p,
                     c->d_nb_w.p, p->d_nb_row.p, p->d_nb_row_off.p, p->d_nb_drained.p, p->dead,
                     hop ? 1u : 0u, weighted,
                     p->d_nh_off.p, d_nh, chunks, p->d_slot_src.p);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

spf_status launch_sliced(spf_ctx* c, spf_plan* p, const uint32_t* D, bool hop, uint32_t* d_nh,
                         hipStream_t s) {
  const uint32_t wpm = c->pitch / 32;
  const uint32_t rows = (uint32_t)p->closure.size();
  const uint64_t words = (uint64_t)rows * wpm;
  const uint32_t sb = (uint32_t)std::min<uint64_t>((words + 255) / 256, 16ull * c->n_cu);
  hipLaunchKernelGGL(slice_rows_kernel, dim3(std::max(sb, 1u)), dim3(256), 0, s, p->d_Dn.p, c->npitch,
                     rows, wpm, p->d_maxd.p, p->d_S.p, p->expand ? const_cast<uint32_t*>(D) : nullptr,
                     c->pitch);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

spf_status launch_ecmp_sliced(spf_ctx* c, spf_plan* p, const uint32_t* D, bool hop, uint32_t* d_nh,
                              hipStream_t s) {
  // one wave per unit; block b serves XCD b % 8 (round-robin placement)
  const uint32_t blocks = 8 * std::max(1u, (p->max_xcd_units + kEcmpWaves - 1) / kEcmpWaves);
  hipLaunchKernelGGL(ecmp_sliced_kernel, dim3(blocks), dim3(kEcmpThreads), 0, s, p->d_S.p,
                     p->d_maxd.p, D, c->pitch, p->d_srcs.p, p->d_row_of.p,
                     c->d_nb_ptr.p, c->d_nb_id.p, c->d_nb_w.p, p->d_nb_row.p, p->d_nb_row_off.p,
                     p->d_nb_drained.p, p->dead, hop ? 1u : 0u, p->d_nh_off.p, d_nh,
                     reinterpret_cast<const uint4*>(p->d_units.p), p->d_unit_off.p, p->d_gtab.p,
                     (uint32_t)(p->d_S.n * 4), p->sdirect ? kTeamPlanes : 0u, p->mp ? 1u : 0u);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

}  // namespace

namespace spfi {

spf_status set_lds_limits(spf_ctx* c) {
  static bool done = false;
  if (done) return SPF_OK;
#define SSK(QT, U) (const void*)sssp_kernel<QT, U, 256>, (const void*)sssp_kernel<QT, U, 512>, \
                   (const void*)sssp_kernel<QT, U, 1024>
  const void* fns[] = {SSK(uint16_t, true), SSK(uint16_t, false), SSK(uint32_t, true), SSK(uint32_t, false),
#define MSB(o) (const void*)msbfs_kernel<o, false>, (const void*)msbfs_kernel<o, true>, \
               (const void*)msbfs_kernel<o, false, true>
                       MSB(1), MSB(2), MSB(4), MSB(8), MSB(10), MSB(12), MSB(16),
#define PLB(o) (const void*)msbfs_planes_kernel<o, false>, (const void*)msbfs_planes_kernel<o, true>
                       PLB(1), PLB(2), PLB(4), PLB(8), PLB(10)};
#undef PLB
#undef MSB
#undef SSK
  for (const void* f : fns)
    HIP_TRY(c, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds));
  const spf_status st = mssp_set_lds_limits(c);
  if (st != SPF_OK) return st;
  done = true;
  return SPF_OK;
}

}  // namespace spfi

namespace {

}  // namespace

namespace spfi {

// Process-wide order of the launches whose workgroups wait on each other
// (engine_internal.h resident_order): per device, the stream of the last
// such launch and an event recorded after it.  A launch on another stream
// waits for that event first.
namespace {
struct ResidentSlot {
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
  const spf_ctx* owner = nullptr;  // context whose launch recorded ev
};
std::mutex g_resident_mu;
std::map<int, ResidentSlot> g_resident;
}  // namespace

// (a stream being captured into a hipGraph is skipped: a capture may not
// wait on an event recorded outside it, and the graph's replays are ordered
// by the stream they are launched on)
static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

spf_status resident_order(spf_ctx* c, hipStream_t s) {
  if (capturing(s)) return SPF_OK;
  std::lock_guard<std::mutex> lk(g_resident_mu);
  ResidentSlot& r = g_resident[c->device];
  if (r.ev && r.last != s) HIP_TRY(c, hipStreamWaitEvent(s, r.ev, 0));
  return SPF_OK;
}

spf_status resident_done(spf_ctx* c, hipStream_t s) {
  if (capturing(s)) return SPF_OK;
  std::lock_guard<std::mutex> lk(g_resident_mu);
  ResidentSlot& r = g_resident[c->device];
  if (!r.ev)
    HIP_TRY(c, hipEventCreateWithFlags(&r.ev, hipEventDisableTiming | hipEventDisableSystemFence));
  HIP_TRY(c, hipEventRecord(r.ev, s));
  r.last = s;
  r.owner = c;
  return SPF_OK;
}

// a context going away: its streams may be reused by the runtime, so the
// next launch on any stream waits for the recorded event instead of
// trusting a stale stream handle
void resident_forget(const spf_ctx* c) {
  std::lock_guard<std::mutex> lk(g_resident_mu);
  for (auto& kv : g_resident)
    if (kv.second.owner == c) kv.second.last = nullptr, kv.second.owner = nullptr;
}

// pathLinks of one source from its distance row already on the device
// (d_row = [N] u32, positive metrics or hop counts): counts, host prefix
// sum, then the ordered lists (the batch form is spf_plan_preds).
spf_status preds_from_row(spf_ctx* c, uint32_t src, bool hop, const uint32_t* ign,
                          const uint32_t* d_row, uint32_t* pred_ptr, uint32_t* pred_edge,
                          uint32_t cap, uint32_t* n_preds, hipStream_t s) {
  const uint32_t N = c->N;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, c->d_pred_cnt.alloc(N + 1));
  const dim3 g((N + 255) / 256), b(256);
  HIP_TRY(c, c->d_one_src.upload(&src, 1, s));
  hipLaunchKernelGGL((preds_kernel<0>), g, b, 0, s, d_row, N, c->d_row_ptr.p, c->d_col.p,
                     c->d_wt.p, c->d_rev.p, c->d_ovl.p, c->d_link.p, ign, c->d_one_src.p, N,
                     hop ? 1u : 0u, c->d_pred_cnt.p, (uint32_t*)nullptr,
                     (unsigned long long*)nullptr);
  HIP_TRY(c, hipGetLastError());
  std::vector<uint32_t> cnt(N);
  HIP_TRY(c, hipMemcpyAsync(cnt.data(), c->d_pred_cnt.p, 4ull * N, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  pred_ptr[0] = 0;
  for (uint32_t v = 0; v < N; ++v) pred_ptr[v + 1] = pred_ptr[v] + cnt[v];
  *n_preds = pred_ptr[N];
  if (!pred_edge) return SPF_OK;
  if (cap < pred_ptr[N]) return fail(c, SPF_E_INVALID, "pred_edge capacity %u < %u", cap, pred_ptr[N]);
  HIP_TRY(c, hipMemcpyAsync(c->d_pred_cnt.p, pred_ptr, 4ull * N, hipMemcpyHostToDevice, s));
  HIP_TRY(c, c->d_pred_edge.alloc(std::max<uint32_t>(pred_ptr[N], 1)));
  HIP_TRY(c, c->d_pred_key.alloc(std::max<uint32_t>(pred_ptr[N], 1)));
  hipLaunchKernelGGL((preds_kernel<1>), g, b, 0, s, d_row, N, c->d_row_ptr.p, c->d_col.p,
                     c->d_wt.p, c->d_rev.p, c->d_ovl.p, c->d_link.p, ign, c->d_one_src.p, N,
                     hop ? 1u : 0u, c->d_pred_cnt.p, c->d_pred_edge.p, c->d_pred_key.p);
  HIP_TRY(c, hipGetLastError());
  if (pred_ptr[N])
    HIP_TRY(c, hipMemcpyAsync(pred_edge, c->d_pred_edge.p, 4ull * pred_ptr[N], hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return SPF_OK;
}

// Upload an ignore set (undirected link ids) as a device bitmap; NULL if empty.
spf_status upload_ignore(spf_ctx* c, const uint32_t* ignore, uint32_t n_ignore,
                         const uint32_t** dev) {
  *dev = nullptr;
  if (!ignore || n_ignore == 0) return SPF_OK;
  std::vector<uint32_t> bm(c->max_link / 32 + 1, 0);
  for (uint32_t i = 0; i < n_ignore; ++i)
    if (ignore[i] <= c->max_link) bm[ignore[i] >> 5] |= 1u << (ignore[i] & 31);
  HIP_TRY(c, c->d_ign.upload(bm.data(), bm.size(), c->stream));
  *dev = c->d_ign.p;
  return SPF_OK;
}

}  // namespace spfi

extern "C" {

spf_status spf_plan_execute(spf_plan* p, uint32_t* d_dist, uint32_t* d_nh, void* stream) {
  if (!p) return fail(nullptr, SPF_E_INVALID, "spf_plan_execute: NULL plan");
  spf_ctx* c = p->ctx;
  if (!c->loaded) return fail(c, SPF_E_STATE, "graph no longer loaded");
  if (!d_dist || (p->nh_total && !d_nh))
    return fail(c, SPF_E_INVALID, "spf_plan_execute: NULL output buffer");
  if (p->shape != c->shape)
    return fail(c, SPF_E_STATE, "graph reloaded since the plan was created: recreate it");
  if (p->layout != c->layout) {
    // a row patch changed some node's distinct neighbours: the plan's
    // next-hop layout holds only if none of its sources was one of them
    for (uint32_t i = 0; i < p->n_src; ++i)
      if (c->nb_ptr[p->srcs[i] + 1] - c->nb_ptr[p->srcs[i]] != p->words[i])
        return fail(c, SPF_E_STATE, "source %u's distinct neighbours changed since the plan was "
                                    "created (its next-hop layout): recreate it", p->srcs[i]);
    p->layout = c->layout;
  }
  if (p->epoch != c->epoch || (p->tm_G && c->team_off)) {
    // patched in place, or teams turned off by a timeout: re-derive, same
    // output layout
    const spf_status st = build_plan(c, p);
    if (st != SPF_OK) return st;
  }
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const uint32_t pitch = c->pitch;
  const bool hop = (p->flags & SPF_FLAG_HOP_COUNT) != 0;
  if (p->exact || p->big) {
    hipEvent_t* ev = nullptr;
    if (p->timing_cap) {
      ev = &p->ev[4 * (p->timing_n % p->timing_cap)];
      ++p->timing_n;
      HIP_TRY(c, hipEventRecord(ev[0], s));
    }
    const spf_status st =
        p->big ? launch_big(c, p, d_dist, d_nh, hop, s)
               : launch_exact(c, &p->xs, p->d_srcs.p, p->n_src, p->d_nh_off.p, p->wmax, hop,
                              (p->flags & SPF_FLAG_DIST64) != 0, nullptr, d_dist, d_nh, nullptr, s);
    if (st != SPF_OK) return st;
    if (ev)
      for (int e = 1; e < 4; ++e) HIP_TRY(c, hipEventRecord(ev[e], s));
    c->solves += p->n_src;
    return SPF_OK;
  }
  // team plans whose closure starts with the request's rows write those
  // rows' u32 distances straight into d_dist (and no others): no scratch
  // rows, no gather
  // (u8 or sliced rows only: the u32-row next-hop pass reads the neighbours'
  // u32 rows, which then exist nowhere)
  const bool team_direct = p->tm_G && p->prefix && !p->direct && p->narrow;
  uint32_t* D = (p->direct || team_direct) ? d_dist : p->d_D.p;
  const uint32_t rows = (uint32_t)p->closure.size();
  const bool sliced = p->sliced && p->nh_total;
  if (sliced && !p->sdirect)  // msbfs_kernel's atomicMax target (sdirect plans: planes fixed)
    HIP_TRY(c, hipMemsetAsync(p->d_maxd.p, 0, 4, s));
  hipEvent_t* ev = nullptr;
  if (p->timing_cap) {
    ev = &p->ev[4 * (p->timing_n % p->timing_cap)];
    ++p->timing_n;
    HIP_TRY(c, hipEventRecord(ev[0], s));
  }
  spf_status st =
      p->tm_G ? launch_msbfs_team(c, p, p->d_closure.p, rows, D,
                                  p->narrow && !p->sdirect ? p->d_Dn.p : nullptr,
                                  sliced && !p->sdirect ? p->d_maxd.p : nullptr, s,
                                  team_direct ? p->n_src : rows,
                                  p->sdirect ? p->d_S.p : nullptr,
                                  kSlSlots * (pitch / 32))
      : p->ms ? launch_msbfs(c, p->d_closure.p, rows, D, p->narrow ? p->d_Dn.p : nullptr,
                                       sliced ? p->d_maxd.p : nullptr, s,
                                       sliced && p->expand ? kSlSat : 0u,
                                       p->pl_order ? p->d_pl_order.p : nullptr)
                  : p->mp ? launch_mssp(c, p->d_closure.p, rows, D, p->narrow ? p->d_Dn.p : nullptr,
                                        p->d_redo.p, s, sliced ? p->d_maxd.p : nullptr)
                        : launch_sssp(c, p->d_closure.p, rows, hop, nullptr, D, s, nullptr,
                                      nullptr, p->narrow ? p->d_Dn.p : nullptr);
  if (st != SPF_OK) return st;
  if (ev) HIP_TRY(c, hipEventRecord(ev[1], s));
  if (sliced && !p->sdirect) {
    st = launch_sliced(c, p, D, hop, d_nh, s);
    if (st != SPF_OK) return st;
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
  if (p->nh_total) {
    st = sliced     ? launch_ecmp_sliced(c, p, D, hop, d_nh, s)
         : p->narrow ? launch_ecmp<true>(c, p, p->d_Dn.p, D, hop, d_nh, s)
                     : launch_ecmp<false>(c, p, nullptr, D, hop, d_nh, s);
    if (st != SPF_OK) return st;
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[3], s));
  if (!p->direct && !team_direct) {
    hipLaunchKernelGGL(gather_rows_kernel, dim3(std::min<uint32_t>((pitch / 4 + 255) / 256, 64), p->n_src),
                       dim3(256), 0, s, D, pitch, p->d_req_rows.p, d_dist);
    HIP_TRY(c, hipGetLastError());
  }
  c->solves += p->n_src;
  return SPF_OK;
}

spf_status spf_plan_copy_narrow_rows(spf_plan* p, uint8_t* d_out, void* stream) {
  if (!p || !d_out) return fail(p ? p->ctx : nullptr, SPF_E_INVALID, "spf_plan_copy_narrow_rows: NULL");
  spf_ctx* c = p->ctx;
  if (p->exact || p->big || !p->narrow || !p->d_Dn.p)
    return fail(c, SPF_E_UNSUPPORTED, "spf_plan_copy_narrow_rows: the plan keeps no u8 rows");
  if (c->npitch != c->pitch)
    return fail(c, SPF_E_UNSUPPORTED, "spf_plan_copy_narrow_rows: u8 and u32 row pitches differ");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  hipLaunchKernelGGL(gather_rows_u8_kernel, dim3(std::min<uint32_t>((c->npitch / 16 + 255) / 256, 64), p->n_src),
                     dim3(256), 0, s, p->d_Dn.p, c->npitch, p->d_req_rows.p, d_out);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

spf_status spf_plan_digest(spf_plan* p, const void* d_dist, const uint32_t* d_nh, uint64_t* d_out,
                           void* stream) {
  if (!p || !d_dist || !d_out || (p->nh_total && !d_nh))
    return fail(p ? p->ctx : nullptr, SPF_E_INVALID, "spf_plan_digest: NULL argument");
  spf_ctx* c = p->ctx;
  if (p->shape != c->shape)
    return fail(c, SPF_E_STATE, "graph reloaded since the plan was created: recreate it");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  HIP_TRY(c, hipMemsetAsync(d_out, 0, 8ull * p->n_src, s));
  if (!p->n_src) return SPF_OK;
  const dim3 grid((c->N + 255) / 256, p->n_src);
  const uint32_t* nh = p->nh_total ? d_nh : p->d_words.p;  // never read when every k = 0
  auto* o = reinterpret_cast<unsigned long long*>(d_out);
  if (p->flags & SPF_FLAG_DIST64)
    hipLaunchKernelGGL(digest_kernel<true>, grid, dim3(256), 0, s, d_dist, c->pitch, c->N, nh,
                       p->d_nh_off.p, p->d_words.p, o);
  else
    hipLaunchKernelGGL(digest_kernel<false>, grid, dim3(256), 0, s, d_dist, c->pitch, c->N, nh,
                       p->d_nh_off.p, p->d_words.p, o);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

spf_status spf_plan_enable_timing(spf_plan* p, uint32_t max_executes) {
  if (!p) return SPF_E_INVALID;
  spf_ctx* c = p->ctx;
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  p->ev.assign(4ull * max_executes, nullptr);
  // timing only: no system-scope fence (its L2 writeback + invalidate cost
  // ~5 us per event and left the next kernel a cold L2)
  for (auto& e : p->ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  p->timing_cap = max_executes;
  p->timing_n = 0;
  return SPF_OK;
}

spf_status spf_plan_timing_phases(spf_plan* p, double* ms, uint32_t* n) {
  if (!p || !p->timing_cap || !ms) return SPF_E_STATE;
  spf_ctx* c = p->ctx;
  const uint32_t cnt = std::min(p->timing_n, p->timing_cap);
  ms[0] = ms[1] = ms[2] = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    HIP_TRY(c, hipEventSynchronize(p->ev[4 * i + 3]));
    for (int ph = 0; ph < 3; ++ph) {
      float t = 0;
      HIP_TRY(c, hipEventElapsedTime(&t, p->ev[4 * i + ph], p->ev[4 * i + ph + 1]));
      ms[ph] += t;
    }
  }
  if (n) *n = cnt;
  p->timing_n = 0;
  return SPF_OK;
}

spf_status spf_plan_timing(spf_plan* p, double* sssp_ms, double* ecmp_ms, uint32_t* n) {
  double ms[3];
  const spf_status st = spf_plan_timing_phases(p, ms, n);
  if (st != SPF_OK) return st;
  if (sssp_ms) *sssp_ms = ms[0];
  if (ecmp_ms) *ecmp_ms = ms[1] + ms[2];
  return SPF_OK;
}

spf_status spf_plan_execute_host(spf_plan* p, uint32_t* dist_out, uint32_t* nh_out) {
  if (!p) return fail(nullptr, SPF_E_INVALID, "spf_plan_execute_host: NULL plan");
  spf_ctx* c = p->ctx;
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t lab = (p->flags & SPF_FLAG_DIST64) ? 8 : 4;
  HIP_TRY(c, p->h_dist.alloc((size_t)p->n_src * c->pitch * (lab / 4)));
  HIP_TRY(c, p->h_nh.alloc(std::max<uint64_t>(p->nh_total, 1)));
  const spf_status st = spf_plan_execute(p, p->h_dist.p, p->h_nh.p, nullptr);
  if (st != SPF_OK) return st;
  p->h_epoch = c->epoch;
  if (dist_out) {
    HIP_TRY(c, hipMemcpy2DAsync(dist_out, (size_t)c->N * lab, p->h_dist.p, (size_t)c->pitch * lab,
                                (size_t)c->N * lab, p->n_src, hipMemcpyDeviceToHost, c->stream));
  }
  if (nh_out && p->nh_total) {
    HIP_TRY(c, hipMemcpyAsync(nh_out, p->h_nh.p, p->nh_total * 4, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // grid-resident kernels (spf_big_kernel, the team BFS) report a barrier
  // that gave up (blocks not co-resident) here instead of wrong rows
  return (p->big || p->tm_G) ? spf_device_check(c) : SPF_OK;
}

spf_status spf_solve(spf_ctx* c, const uint32_t* srcs, uint32_t n_src, uint32_t flags,
                     uint32_t* dist_out, uint32_t* nh_out) {
  spf_plan* raw = nullptr;
  spf_status st = spf_plan_create(c, srcs, n_src, flags, &raw);
  if (st != SPF_OK) return st;
  std::unique_ptr<spf_plan> p(raw);
  return spf_plan_execute_host(p.get(), dist_out, nh_out);
}

spf_status spf_debug_copy_bandwidth(spf_ctx* c, uint64_t bytes, uint32_t reps, double* gbs) {
  if (!c || !gbs || bytes < 16 || reps == 0) return fail(c, SPF_E_INVALID, "spf_debug_copy_bandwidth: bad argument");
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t n = bytes / 16;
  DevBuf<uint4> a, b;
  HIP_TRY(c, a.alloc(n));
  HIP_TRY(c, b.alloc(n));
  HIP_TRY(c, hipMemsetAsync(a.p, 1, n * 16, c->stream));
  const dim3 g(c->n_cu * 8), blk(256);
  hipLaunchKernelGGL(copy_bw_kernel, g, blk, 0, c->stream, a.p, b.p, n);  // warm
  HIP_TRY(c, hipGetLastError());
  hipEvent_t e0, e1;
  HIP_TRY(c, hipEventCreate(&e0));
  HIP_TRY(c, hipEventCreate(&e1));
  HIP_TRY(c, hipEventRecord(e0, c->stream));
  for (uint32_t r = 0; r < reps; ++r)
    hipLaunchKernelGGL(copy_bw_kernel, g, blk, 0, c->stream, (r & 1) ? b.p : a.p, (r & 1) ? a.p : b.p, n);
  HIP_TRY(c, hipEventRecord(e1, c->stream));
  HIP_TRY(c, hipEventSynchronize(e1));
  float ms = 0;
  HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *gbs = 2.0 * 16.0 * (double)n * reps / (ms * 1e-3) / 1e9;  // bytes read + written
  return SPF_OK;
}

spf_status spf_debug_stamps(spf_ctx* c, uint64_t* out, uint32_t cap, uint32_t* n) {
  if (!c || !n) return SPF_E_INVALID;
  *n = 0;
  if (!c->d_stamps.p) return SPF_OK;
  std::vector<uint64_t> buf(kStampWords);
  HIP_TRY(c, hipMemcpy(buf.data(), c->d_stamps.p, buf.size() * 8, hipMemcpyDeviceToHost));
  *n = (uint32_t)std::min<size_t>(cap, buf.size());
  std::copy(buf.begin(), buf.begin() + *n, out);
  return SPF_OK;
}

spf_status spf_sssp(spf_ctx* c, uint32_t src, uint32_t flags, const uint32_t* ignore_links,
                    uint32_t n_ignore, uint32_t* dist_out) {
  if (!c || !dist_out) return fail(c, SPF_E_INVALID, "spf_sssp: NULL argument");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (src >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", src);
  const bool hop = (flags & SPF_FLAG_HOP_COUNT) != 0;
  if (!hop && (c->nonpos || c->needs64)) {  // the exact kernel (u32 rows when they fit)
    if (c->needs64)
      return fail(c, SPF_E_UNSUPPORTED, "weighted distances may exceed 32 bits: use spf_solve_exact");
    return spf_solve_exact(c, src, flags, ignore_links, n_ignore, nullptr, dist_out, nullptr,
                           nullptr);
  }
  spf_status st = set_lds_limits(c);
  if (st != SPF_OK) return st;
  const uint32_t* ign = nullptr;
  st = upload_ignore(c, ignore_links, n_ignore, &ign);
  if (st != SPF_OK) return st;
  HIP_TRY(c, c->d_one_src.upload(&src, 1, c->stream));
  HIP_TRY(c, c->d_row.alloc(c->pitch));
  const bool grid_resident = sssp_lds_bytes(c->N, c->pitch, c->big_nodes, c->N <= 65535) > kMaxLds;
  if (grid_resident) {
    st = launch_gsssp(c, src, hop, ign, c->d_row.p, c->stream);
  } else {
    st = launch_sssp(c, c->d_one_src.p, 1, hop, ign, c->d_row.p, c->stream);
  }
  if (st != SPF_OK) return st;
  HIP_TRY(c, hipMemcpyAsync(dist_out, c->d_row.p, 4ull * c->N, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->solves += 1;
  return grid_resident ? spf_device_check(c) : SPF_OK;
}

spf_status spf_solve_exact(spf_ctx* c, uint32_t src, uint32_t flags, const uint32_t* ignore_links,
                           uint32_t n_ignore, uint64_t* dist64_out, uint32_t* dist32_out,
                           uint32_t* nh_out, uint32_t* pop_out) {
  if (!c) return fail(c, SPF_E_INVALID, "spf_solve_exact: NULL context");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (src >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", src);
  const bool hop = (flags & SPF_FLAG_HOP_COUNT) != 0;
  if (dist32_out && !hop && c->needs64)
    return fail(c, SPF_E_UNSUPPORTED, "weighted distances may exceed 32 bits: ask for u64 rows");
  const uint32_t* ign = nullptr;
  spf_status st = upload_ignore(c, ignore_links, n_ignore, &ign);
  if (st != SPF_OK) return st;
  const uint32_t k = c->nb_ptr[src + 1] - c->nb_ptr[src];
  const uint64_t wpm = c->pitch / 32, nh_words = (uint64_t)k * wpm;
  const bool d64 = dist32_out == nullptr;
  DevBuf<uint32_t> d_dist, d_nh, d_pop;
  DevBuf<uint64_t> d_off;
  const uint64_t zero = 0;
  HIP_TRY(c, c->d_one_src.upload(&src, 1, c->stream));
  HIP_TRY(c, d_off.upload(&zero, 1, c->stream));
  HIP_TRY(c, d_dist.alloc((size_t)c->pitch * (d64 ? 2 : 1)));
  HIP_TRY(c, d_nh.alloc(std::max<uint64_t>(nh_words, 1)));
  if (pop_out) HIP_TRY(c, d_pop.alloc(c->pitch));
  const uint32_t wk = std::max<uint32_t>(1, (k + 31) / 32);
  st = exact_reserve(c, &c->exact1, 1, wk);
  if (st != SPF_OK) return st;
  st = launch_exact(c, &c->exact1, c->d_one_src.p, 1, d_off.p, wk, hop, d64, ign, d_dist.p, d_nh.p,
                    pop_out ? d_pop.p : nullptr, c->stream);
  if (st != SPF_OK) return st;
  if (d64 && dist64_out)
    HIP_TRY(c, hipMemcpyAsync(dist64_out, d_dist.p, 8ull * c->N, hipMemcpyDeviceToHost, c->stream));
  if (!d64)
    HIP_TRY(c, hipMemcpyAsync(dist32_out, d_dist.p, 4ull * c->N, hipMemcpyDeviceToHost, c->stream));
  if (nh_out && nh_words)
    HIP_TRY(c, hipMemcpyAsync(nh_out, d_nh.p, 4ull * nh_words, hipMemcpyDeviceToHost, c->stream));
  if (pop_out)
    HIP_TRY(c, hipMemcpyAsync(pop_out, d_pop.p, 4ull * c->N, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->solves += 1;
  return SPF_OK;
}

spf_status spf_preds(spf_ctx* c, uint32_t src, uint32_t flags, const uint32_t* ignore_links,
                     uint32_t n_ignore, const uint32_t* dist, uint32_t* pred_ptr,
                     uint32_t* pred_edge, uint32_t cap, uint32_t* n_preds) {
  if (!c || !dist || !pred_ptr || !n_preds) return fail(c, SPF_E_INVALID, "spf_preds: NULL argument");
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (src >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", src);
  const uint32_t* ign = nullptr;
  spf_status st = upload_ignore(c, ignore_links, n_ignore, &ign);
  if (st != SPF_OK) return st;
  HIP_TRY(c, c->d_row.upload(dist, c->N, c->stream));
  return preds_from_row(c, src, (flags & SPF_FLAG_HOP_COUNT) != 0, ign, c->d_row.p, pred_ptr,
                        pred_edge, cap, n_preds, c->stream);
}

spf_status spf_plan_preds(spf_plan* p, uint32_t* pred_ptr, uint32_t* pred_edge, uint64_t cap,
                          uint64_t* n_preds) {
  if (!p || !pred_ptr || !n_preds) return fail(p ? p->ctx : nullptr, SPF_E_INVALID, "spf_plan_preds: NULL argument");
  spf_ctx* c = p->ctx;
  // positive metrics (or hop counts) with u32 rows: pathLinks follow from the
  // distance row alone, whichever kernel wrote it -- big plans
  // and exact plans of large positive-metric graphs included.  Zero /
  // negative metrics and u64 rows need the pop order (spf_solve_exact).
  const bool hop_only = (p->flags & SPF_FLAG_HOP_COUNT) != 0;
  if ((p->flags & SPF_FLAG_DIST64) || (!hop_only && c->nonpos))
    return fail(c, SPF_E_UNSUPPORTED, "spf_plan_preds: zero / negative metrics and u64 rows order "
                                      "pathLinks by pop rank (spf_solve_exact)");
  if (!p->h_dist.p || p->h_epoch != c->epoch)
    return fail(c, SPF_E_STATE, "spf_plan_preds: no spf_plan_execute_host on the current graph");
  const uint32_t N = c->N, n = p->n_src;
  const bool hop = (p->flags & SPF_FLAG_HOP_COUNT) != 0;
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t slots = (size_t)n * (N + 1);
  HIP_TRY(c, p->h_pcnt.alloc(slots));
  const dim3 g((N + 255) / 256, n), b(256);
  hipLaunchKernelGGL((preds_kernel<0>), g, b, 0, c->stream, p->h_dist.p, c->pitch, c->d_row_ptr.p,
                     c->d_col.p, c->d_wt.p, c->d_rev.p, c->d_ovl.p, c->d_link.p, nullptr,
                     p->d_srcs.p, N, hop ? 1u : 0u, p->h_pcnt.p, (uint32_t*)nullptr,
                     (unsigned long long*)nullptr);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, c->pin_preds.alloc(slots));
  HIP_TRY(c, hipMemcpyAsync(c->pin_preds.p, p->h_pcnt.p, 4ull * slots, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::memcpy(pred_ptr, c->pin_preds.p, 4ull * slots);
  // counts -> absolute offsets: source i's list of v starts at pred_ptr[i*(N+1) + v],
  // pred_ptr[i*(N+1) + N] = the end of source i's lists
  uint64_t at = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t* pp = pred_ptr + (size_t)i * (N + 1);
    for (uint32_t v = 0; v < N; ++v) {
      const uint32_t cnt = pp[v];
      if (at + cnt > 0xFFFFFFFFull) return fail(c, SPF_E_UNSUPPORTED, "spf_plan_preds: > 2^32 entries");
      pp[v] = (uint32_t)at;
      at += cnt;
    }
    pp[N] = (uint32_t)at;
  }
  *n_preds = at;
  if (!pred_edge) return SPF_OK;
  if (cap < at) return fail(c, SPF_E_NOMEM, "spf_plan_preds: capacity %llu < %llu",
                            (unsigned long long)cap, (unsigned long long)at);
  // one staging buffer for the upload and the edges (sized before either copy)
  HIP_TRY(c, c->pin_preds.alloc(std::max<uint64_t>(slots, at)));
  std::memcpy(c->pin_preds.p, pred_ptr, 4ull * slots);
  HIP_TRY(c, hipMemcpyAsync(p->h_pcnt.p, c->pin_preds.p, 4ull * slots, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, p->h_pedge.alloc(std::max<uint64_t>(at, 1)));
  HIP_TRY(c, p->h_pkey.alloc(std::max<uint64_t>(at, 1)));
  hipLaunchKernelGGL((preds_kernel<1>), g, b, 0, c->stream, p->h_dist.p, c->pitch, c->d_row_ptr.p,
                     c->d_col.p, c->d_wt.p, c->d_rev.p, c->d_ovl.p, c->d_link.p, nullptr,
                     p->d_srcs.p, N, hop ? 1u : 0u, p->h_pcnt.p, p->h_pedge.p, p->h_pkey.p);
  HIP_TRY(c, hipGetLastError());
  if (at)
    HIP_TRY(c, hipMemcpyAsync(c->pin_preds.p, p->h_pedge.p, 4ull * at, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (at) std::memcpy(pred_edge, c->pin_preds.p, 4ull * at);
  return SPF_OK;
}

}  // extern "C"
