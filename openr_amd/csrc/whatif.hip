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

#include <memory>

using namespace spfi;

namespace {

constexpr uint32_t kBusy = 0xFFFFFFFEu;
constexpr int kGThreads = 1024;     // global-memory SSSP (one workgroup)
constexpr uint32_t kWaveCap = 4096; // |D| a wave team can hold
constexpr int kBigTeams = 32;       // workgroup teams for large D

__device__ __forceinline__ uint32_t ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t node_hash(uint32_t v, uint32_t d, const uint32_t* nh,
                                              uint32_t W) {
  uint64_t f = 0xcbf29ce484222325ull;
  for (uint32_t w = 0; w < W; ++w) {
    f ^= nh[w];
    f *= 0x100000001b3ull;
  }
  return mix64(mix64((uint64_t)v + 1) + d) ^ f;
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
};

struct WiBase {
  const uint32_t* dist;  // [N] unfailed distances
  const uint32_t* nhb;   // [N][W] unfailed next-hop bitsets
  const unsigned long long* H;  // unfailed hash
};

// ---------------------------------------------------------------------------
//  global-memory SSSP from one source (graphs beyond the LDS kernels)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kGThreads) void gsssp_kernel(
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const uint32_t* __restrict__ wt, const uint8_t* __restrict__ ovl,
    const uint32_t* __restrict__ link, const uint32_t* __restrict__ ign, uint32_t src,
    uint32_t N, uint32_t hop, uint32_t* dist, uint32_t* q, uint32_t* bm) {
  __shared__ uint32_t s_len;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t bm_words = (N + 31) / 32;
  for (uint32_t v = tid; v < N; v += kGThreads) st(&dist[v], v == src ? 0u : kInf);
  for (uint32_t i = tid; i < bm_words; i += kGThreads) st(&bm[i], 0u);
  if (tid == 0) {
    q[0] = src;
    s_len = 0;
  }
  __syncthreads();
  uint32_t qlen = 1;
  while (qlen) {
    for (uint32_t i = tid; i < qlen; i += kGThreads) {
      const uint32_t u = q[i];
      if (ovl[u] && u != src) continue;  // drained: recorded, not expanded
      const uint32_t du = ld(&dist[u]);
      for (uint32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
        if (ign && ((ign[link[e] >> 5] >> (link[e] & 31)) & 1u)) continue;
        const uint32_t v = col[e];
        const uint32_t nd = du + (hop ? 1u : wt[e]);
        if (nd < atomicMin(&dist[v], nd)) atomicOr(&bm[v >> 5], 1u << (v & 31));
      }
    }
    __syncthreads();
    for (uint32_t base = 0; base < bm_words; base += kGThreads) {
      const uint32_t i = base + tid;
      uint32_t word = i < bm_words ? atomicExch(&bm[i], 0u) : 0u;
      // wave scan of the popcounts, one LDS atomic per wave
      uint32_t x = __popc(word), inc = x;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
      const uint32_t tot = __shfl(inc, 63, 64);
      uint32_t at = 0;
      if (lane == 63 && tot) at = atomicAdd(&s_len, tot);
      at = __shfl(at, 63, 64) + inc - x;
      while (word) {
        const uint32_t b = __ffs(word) - 1;
        word &= word - 1;
        q[at++] = i * 32 + b;
      }
    }
    __syncthreads();
    qlen = s_len;
    __syncthreads();
    if (tid == 0) s_len = 0;
  }
}

// ---------------------------------------------------------------------------
//  unfailed next hops: nh(v) = union over tight expanded preds, to fixed point
// ---------------------------------------------------------------------------
__global__ void nh_base_kernel(WiGraph g, const uint32_t* __restrict__ dist, uint32_t* nhb,
                               uint32_t* changed) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (uint64_t)g.N * g.W) return;
  const uint32_t v = (uint32_t)(t / g.W), j = (uint32_t)(t % g.W);
  const uint32_t dv = dist[v];
  if (dv == kInf || v == g.src) return;
  uint32_t acc = 0;
  for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
    const uint32_t u = g.col[e];
    if (g.ovl[u] && u != g.src) continue;
    const uint32_t du = dist[u];
    if (du == kInf || du + g.wt[g.rev[e]] != dv) continue;
    if (u == g.src) {
      const uint32_t jb = g.nbr_bit[v];
      if ((jb >> 5) == j) acc |= 1u << (jb & 31);
    } else {
      acc |= ld(&nhb[(size_t)u * g.W + j]);
    }
  }
  if (acc != ld(&nhb[(size_t)v * g.W + j])) {
    st(&nhb[(size_t)v * g.W + j], acc);
    *changed = 1;
  }
}

__global__ void hash_base_kernel(WiGraph g, const uint32_t* __restrict__ dist,
                                 const uint32_t* __restrict__ nhb, unsigned long long* H) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t h = 0;
  if (v < g.N && dist[v] != kInf) h = node_hash(v, dist[v], nhb + (size_t)v * g.W, g.W);
  // wave sum, one atomic per wave
  uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t l2 = __shfl_down(lo, d, 64), h2 = __shfl_down(hi, d, 64);
    const uint64_t s = ((uint64_t)hi << 32 | lo) + ((uint64_t)h2 << 32 | l2);
    lo = (uint32_t)s;
    hi = (uint32_t)(s >> 32);
  }
  if ((threadIdx.x & 63) == 0) atomicAdd(H, ((unsigned long long)hi << 32) | lo);
}

// ---------------------------------------------------------------------------
//  classify failures: cold -> digest now, hot -> work list (failure, edge)
// ---------------------------------------------------------------------------
__global__ void classify_kernel(WiGraph g, const uint32_t* __restrict__ dist,
                                const unsigned long long* __restrict__ H,
                                const uint32_t* __restrict__ fails, uint32_t n_fail,
                                const uint32_t* __restrict__ link_edge,
                                spf_whatif_digest* out, uint2* hot, uint32_t* n_hot) {
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
  } else {
    hot[atomicAdd(n_hot, 1u)] = make_uint2(f, tight);
  }
}

// ---------------------------------------------------------------------------
//  repair of one hot failure by a team (a wave, or a whole workgroup)
// ---------------------------------------------------------------------------
struct TeamCtl {
  uint32_t n, ovf, flag[3];
  unsigned long long ndist, nnh, dh;
};

template <int TEAM>
__device__ __forceinline__ void team_sync() {
  if (TEAM == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Returns false (nothing written, scratch clean) when |D| exceeds cap.
template <int TEAM>
__device__ bool repair(const WiGraph& g, const WiBase& B, uint32_t* mark, uint32_t* dlist,
                       uint32_t* dnew, uint32_t* nhn, uint32_t cap, TeamCtl* ctl, uint32_t tt,
                       uint32_t e_fail, spf_whatif_digest* out) {
  const uint32_t W = g.W;
  const uint32_t l = g.link[e_fail];
  const uint32_t b = g.col[e_fail];
  if (tt == 0) {
    ctl->n = 1;
    ctl->ovf = 0;
    ctl->flag[0] = ctl->flag[1] = ctl->flag[2] = 0;
    ctl->ndist = ctl->nnh = ctl->dh = 0;
    dlist[0] = b;
    st(&mark[b], 0);
  }
  team_sync<TEAM>();
  // ---- D = descendants of b in the unfailed DAG (level by level) ----
  uint32_t lo = 0;
  for (;;) {
    const uint32_t n = ctl->n;
    team_sync<TEAM>();
    if (lo >= n || ctl->ovf) break;
    for (uint32_t i = lo + tt; i < n; i += TEAM) {
      const uint32_t v = dlist[i];
      if (g.ovl[v]) continue;  // drained (v != src): no DAG children
      const uint32_t dv = B.dist[v];
      for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
        const uint32_t c = g.col[e];
        if (dv + g.wt[e] != B.dist[c]) continue;
        if (atomicCAS(&mark[c], kInf, kBusy) != kInf) continue;
        const uint32_t idx = atomicAdd(&ctl->n, 1u);
        if (idx < cap) {
          dlist[idx] = c;
          st(&mark[c], idx);
        } else {
          st(&mark[c], kInf);
          ctl->ovf = 1;
        }
      }
    }
    lo = n;
    team_sync<TEAM>();
  }
  const uint32_t n = min(ctl->n, cap);
  const bool ovf = ctl->ovf != 0;
  team_sync<TEAM>();
  if (ovf) {
    for (uint32_t i = tt; i < n; i += TEAM) st(&mark[dlist[i]], kInf);
    team_sync<TEAM>();
    return false;
  }
  // ---- seeds: best in-edge from outside D (unchanged distances) ----
  for (uint32_t i = tt; i < n; i += TEAM) {
    const uint32_t v = dlist[i];
    uint32_t best = kInf;
    for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
      if (g.link[e] == l) continue;
      const uint32_t u = g.col[e];
      if (ld(&mark[u]) != kInf) continue;
      if (g.ovl[u] && u != g.src) continue;
      const uint32_t du = B.dist[u];
      if (du == kInf) continue;
      best = min(best, du + g.wt[g.rev[e]]);
    }
    st(&dnew[i], best);
  }
  team_sync<TEAM>();
  // ---- label-correcting sweeps inside D ----
  for (uint32_t it = 0;; ++it) {
    bool any = false;
    for (uint32_t i = tt; i < n; i += TEAM) {
      const uint32_t v = dlist[i];
      const uint32_t dv = ld(&dnew[i]);
      if (dv == kInf || g.ovl[v]) continue;
      for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
        if (g.link[e] == l) continue;
        const uint32_t ic = ld(&mark[g.col[e]]);
        if (ic == kInf) continue;
        const uint32_t nd = dv + g.wt[e];
        if (nd < atomicMin(&dnew[ic], nd)) any = true;
      }
    }
    if (any) ctl->flag[it % 3] = 1;
    if (tt == 0) ctl->flag[(it + 1) % 3] = 0;
    team_sync<TEAM>();
    if (!ctl->flag[it % 3]) break;
  }
  // ---- next hops inside D, to the fixed point ----
  const uint32_t nw = n * W;
  for (uint32_t x = tt; x < nw; x += TEAM) nhn[x] = 0;
  team_sync<TEAM>();
  if (tt == 0) ctl->flag[0] = ctl->flag[1] = ctl->flag[2] = 0;
  team_sync<TEAM>();
  for (uint32_t it = 0;; ++it) {
    bool any = false;
    for (uint32_t x = tt; x < nw; x += TEAM) {
      const uint32_t i = x / W, j = x % W;
      const uint32_t v = dlist[i];
      const uint32_t dv = ld(&dnew[i]);
      if (dv == kInf) continue;
      uint32_t acc = 0;
      for (uint32_t e = g.row_ptr[v]; e < g.row_ptr[v + 1]; ++e) {
        if (g.link[e] == l) continue;
        const uint32_t u = g.col[e];
        if (g.ovl[u] && u != g.src) continue;
        const uint32_t mu = ld(&mark[u]);
        const uint32_t du = mu != kInf ? ld(&dnew[mu]) : B.dist[u];
        if (du == kInf || du + g.wt[g.rev[e]] != dv) continue;
        if (u == g.src) {
          const uint32_t jb = g.nbr_bit[v];
          if ((jb >> 5) == j) acc |= 1u << (jb & 31);
        } else {
          acc |= mu != kInf ? nhn[(size_t)mu * W + j] : B.nhb[(size_t)u * W + j];
        }
      }
      if (acc != nhn[x]) {
        nhn[x] = acc;
        any = true;
      }
    }
    if (any) ctl->flag[it % 3] = 1;
    if (tt == 0) ctl->flag[(it + 1) % 3] = 0;
    team_sync<TEAM>();
    if (!ctl->flag[it % 3]) break;
  }
  // ---- digest delta over D, scratch reset ----
  uint32_t nd_ = 0, nn_ = 0;
  uint64_t dh = 0;
  for (uint32_t i = tt; i < n; i += TEAM) {
    const uint32_t v = dlist[i];
    const uint32_t d1 = ld(&dnew[i]), d0 = B.dist[v];
    const uint32_t* h0 = B.nhb + (size_t)v * W;
    const uint32_t* h1 = nhn + (size_t)i * W;
    nd_ += d1 != d0;
    bool diff = d1 == kInf;
    for (uint32_t w = 0; w < W && !diff; ++w) diff = h0[w] != h1[w];
    nn_ += diff;
    dh += (d1 == kInf ? 0ull : node_hash(v, d1, h1, W)) - node_hash(v, d0, h0, W);
    st(&mark[v], kInf);
  }
  if (nd_) atomicAdd(&ctl->ndist, (unsigned long long)nd_);
  if (nn_) atomicAdd(&ctl->nnh, (unsigned long long)nn_);
  if (dh) atomicAdd(&ctl->dh, (unsigned long long)dh);
  team_sync<TEAM>();
  if (tt == 0)
    *out = spf_whatif_digest{(uint32_t)ctl->ndist, (uint32_t)ctl->nnh,
                             (uint64_t)(*B.H + ctl->dh)};
  team_sync<TEAM>();
  return true;
}

// wave teams over the hot list; failures whose D overflows kWaveCap are
// queued for the workgroup teams
__global__ __launch_bounds__(256) void repair_wave_kernel(
    WiGraph g, WiBase B, const uint2* __restrict__ hot, const uint32_t* __restrict__ n_hot,
    uint32_t* cursor, uint2* big, uint32_t* n_big, uint32_t* mark, uint32_t* dlist, uint32_t* dnew,
    uint32_t* nhn, spf_whatif_digest* out) {
  __shared__ TeamCtl ctl[4];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t team = (size_t)blockIdx.x * 4 + w;
  mark += team * g.N;
  dlist += team * kWaveCap;
  dnew += team * kWaveCap;
  nhn += team * kWaveCap * g.W;
  const uint32_t total = *n_hot;
  for (;;) {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(cursor, 1u);
    k = __shfl(k, 0, 64);
    if (k >= total) break;
    const uint2 h = hot[k];
    if (!repair<64>(g, B, mark, dlist, dnew, nhn, kWaveCap, &ctl[w], lane, h.y, out + h.x)) {
      if (lane == 0) big[atomicAdd(n_big, 1u)] = h;
    }
  }
}

__global__ __launch_bounds__(1024) void repair_block_kernel(
    WiGraph g, WiBase B, const uint2* __restrict__ big, const uint32_t* __restrict__ n_big,
    uint32_t* mark, uint32_t* dlist, uint32_t* dnew, uint32_t* nhn, spf_whatif_digest* out) {
  __shared__ TeamCtl ctl;
  const size_t team = blockIdx.x;
  mark += team * g.N;
  dlist += team * g.N;
  dnew += team * g.N;
  nhn += team * (size_t)g.N * g.W;
  const uint32_t total = *n_big;
  for (uint32_t k = blockIdx.x; k < total; k += gridDim.x) {
    const uint2 h = big[k];
    repair<1024>(g, B, mark, dlist, dnew, nhn, g.N, &ctl, threadIdx.x, h.y, out + h.x);
  }
}

__global__ void base_digest_kernel(spf_whatif_digest* o, const unsigned long long* H) {
  *o = spf_whatif_digest{0u, 0u, (uint64_t)*H};
}

}  // namespace

struct spf_whatif_plan {
  spf_ctx* ctx = nullptr;
  uint32_t src = 0, n_fail = 0, W = 0, wave_teams = 0;
  DevBuf<uint32_t> d_fails, d_link_edge, d_nbr_bit, d_dist, d_q, d_bm, d_nhb, d_flag;
  DevBuf<unsigned long long> d_H;
  DevBuf<uint2> d_hot, d_big;
  DevBuf<uint32_t> d_cnt;  // [0] n_hot, [1] cursor, [2] n_big
  DevBuf<uint32_t> w_mark, w_dlist, w_dnew, w_nhn;  // wave-team scratch
  DevBuf<uint32_t> b_mark, b_dlist, b_dnew, b_nhn;  // workgroup-team scratch
  std::vector<hipEvent_t> ev;
  uint32_t timing_cap = 0, timing_n = 0;
  ~spf_whatif_plan() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
};

namespace spfi {

spf_status launch_gsssp(spf_ctx* c, uint32_t src, bool hop, const uint32_t* ign, uint32_t* dist,
                        uint32_t* q, uint32_t* bm, hipStream_t s) {
  hipLaunchKernelGGL(gsssp_kernel, dim3(1), dim3(kGThreads), 0, s, c->d_row_ptr.p, c->d_col.p,
                     c->d_wt.p, c->d_ovl.p, c->d_link.p, ign, src, c->N, hop ? 1u : 0u, dist, q,
                     bm);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

}  // namespace spfi

extern "C" {

spf_status spf_whatif_plan_create(spf_ctx* c, uint32_t src, const uint32_t* fail_links,
                                  uint32_t n_fail, spf_whatif_plan** out) {
  if (!c || !out) return fail(c, SPF_E_INVALID, "spf_whatif_plan_create: NULL argument");
  *out = nullptr;
  if (!c->loaded) return fail(c, SPF_E_STATE, "no graph loaded");
  if (src >= c->N) return fail(c, SPF_E_INVALID, "source %u out of range", src);
  if (c->nonpos)
    return fail(c, SPF_E_UNSUPPORTED, "graph has up links with metric <= 0 (what-if runs weighted SPF)");
  auto p = std::make_unique<spf_whatif_plan>();
  p->ctx = c;
  p->src = src;
  const uint32_t N = c->N, E = c->E;
  // link -> one of its directed edges
  std::vector<uint32_t> link_edge((size_t)c->max_link + 1, kInf);
  for (uint32_t e = 0; e < E; ++e)
    if (link_edge[c->link[e]] == kInf) link_edge[c->link[e]] = e;
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
  // bit of each distinct up neighbour of src
  std::vector<uint32_t> nbr_bit(N, kInf);
  const uint32_t k = c->nb_ptr[src + 1] - c->nb_ptr[src];
  for (uint32_t j = 0; j < k; ++j) nbr_bit[c->nb_id[c->nb_ptr[src] + j]] = j;
  p->W = std::max<uint32_t>(1, (k + 31) / 32);
  p->wave_teams = 4 * 2 * c->n_cu;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, p->d_fails.upload(fails.data(), fails.size(), c->stream));
  HIP_TRY(c, p->d_link_edge.upload(link_edge.data(), link_edge.size(), c->stream));
  HIP_TRY(c, p->d_nbr_bit.upload(nbr_bit.data(), N, c->stream));
  HIP_TRY(c, p->d_dist.alloc(N));
  HIP_TRY(c, p->d_q.alloc(N));
  HIP_TRY(c, p->d_bm.alloc((N + 31) / 32));
  HIP_TRY(c, p->d_nhb.alloc((size_t)N * p->W));
  HIP_TRY(c, p->d_flag.alloc(1));
  HIP_TRY(c, p->d_H.alloc(1));
  HIP_TRY(c, p->d_hot.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, p->d_big.alloc(std::max<uint32_t>(1, p->n_fail)));
  HIP_TRY(c, p->d_cnt.alloc(4));
  const size_t wt = p->wave_teams;
  HIP_TRY(c, p->w_mark.alloc(wt * N));
  HIP_TRY(c, p->w_dlist.alloc(wt * kWaveCap));
  HIP_TRY(c, p->w_dnew.alloc(wt * kWaveCap));
  HIP_TRY(c, p->w_nhn.alloc(wt * kWaveCap * p->W));
  HIP_TRY(c, p->b_mark.alloc((size_t)kBigTeams * N));
  HIP_TRY(c, p->b_dlist.alloc((size_t)kBigTeams * N));
  HIP_TRY(c, p->b_dnew.alloc((size_t)kBigTeams * N));
  HIP_TRY(c, p->b_nhn.alloc((size_t)kBigTeams * N * p->W));
  // marks start (and are always left) at kInf
  HIP_TRY(c, hipMemsetAsync(p->w_mark.p, 0xFF, wt * N * 4, c->stream));
  HIP_TRY(c, hipMemsetAsync(p->b_mark.p, 0xFF, (size_t)kBigTeams * N * 4, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
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
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const uint32_t N = c->N;
  hipEvent_t* ev = nullptr;
  if (p->timing_cap) {
    ev = &p->ev[3 * (p->timing_n % p->timing_cap)];
    ++p->timing_n;
    HIP_TRY(c, hipEventRecord(ev[0], s));
  }
  WiGraph g{c->d_row_ptr.p, c->d_col.p, c->d_wt.p, c->d_rev.p, c->d_link.p, c->d_ovl.p,
            p->d_nbr_bit.p, N, p->src, p->W};
  // 1. unfailed SPF, next hops, hash
  spf_status st = launch_gsssp(c, p->src, false, nullptr, p->d_dist.p, p->d_q.p, p->d_bm.p, s);
  if (st != SPF_OK) return st;
  HIP_TRY(c, hipMemsetAsync(p->d_nhb.p, 0, 4ull * N * p->W, s));
  const uint64_t items = (uint64_t)N * p->W;
  for (int pass = 0;; ++pass) {
    uint32_t changed = 0;
    HIP_TRY(c, hipMemsetAsync(p->d_flag.p, 0, 4, s));
    hipLaunchKernelGGL(nh_base_kernel, dim3((uint32_t)((items + 255) / 256)), dim3(256), 0, s, g,
                       p->d_dist.p, p->d_nhb.p, p->d_flag.p);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(&changed, p->d_flag.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (!changed) break;
    if (pass > (int)N) return fail(c, SPF_E_HIP, "next-hop propagation did not converge");
  }
  HIP_TRY(c, hipMemsetAsync(p->d_H.p, 0, 8, s));
  hipLaunchKernelGGL(hash_base_kernel, dim3((N + 255) / 256), dim3(256), 0, s, g, p->d_dist.p,
                     p->d_nhb.p, p->d_H.p);
  HIP_TRY(c, hipGetLastError());
  if (ev) HIP_TRY(c, hipEventRecord(ev[1], s));
  // 2. failures
  HIP_TRY(c, hipMemsetAsync(p->d_cnt.p, 0, 16, s));
  if (p->n_fail) {
    hipLaunchKernelGGL(classify_kernel, dim3((p->n_fail + 255) / 256), dim3(256), 0, s, g,
                       p->d_dist.p, p->d_H.p, p->d_fails.p, p->n_fail, p->d_link_edge.p, d_out,
                       p->d_hot.p, p->d_cnt.p);
    HIP_TRY(c, hipGetLastError());
    WiBase B{p->d_dist.p, p->d_nhb.p, p->d_H.p};
    hipLaunchKernelGGL(repair_wave_kernel, dim3(p->wave_teams / 4), dim3(256), 0, s, g, B,
                       p->d_hot.p, p->d_cnt.p, p->d_cnt.p + 1, p->d_big.p, p->d_cnt.p + 2,
                       p->w_mark.p, p->w_dlist.p, p->w_dnew.p, p->w_nhn.p, d_out);
    HIP_TRY(c, hipGetLastError());
    hipLaunchKernelGGL(repair_block_kernel, dim3(kBigTeams), dim3(1024), 0, s, g, B, p->d_big.p,
                       p->d_cnt.p + 2, p->b_mark.p, p->b_dlist.p, p->b_dnew.p, p->b_nhn.p, d_out);
    HIP_TRY(c, hipGetLastError());
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
  uint32_t cnt[4];
  HIP_TRY(c, hipMemcpy(cnt, p->d_cnt.p, sizeof cnt, hipMemcpyDeviceToHost));
  if (n_hot) *n_hot = cnt[0];
  if (n_big) *n_big = cnt[2];
  return SPF_OK;
}

spf_status spf_whatif_enable_timing(spf_whatif_plan* p, uint32_t max_executes) {
  if (!p) return SPF_E_INVALID;
  spf_ctx* c = p->ctx;
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  p->ev.assign(3ull * max_executes, nullptr);
  for (auto& e : p->ev) HIP_TRY(c, hipEventCreate(&e));
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
  return SPF_OK;
}

}  // extern "C"
