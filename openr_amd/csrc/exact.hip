// ============================================================================
//  exact.hip -- the exact-envelope SPF kernel: LinkState::runSpf
//  (openr/decision/LinkState.cpp:808-882) replayed step for step, one
//  wavefront per source, for the inputs the data-parallel kernels of
//  spf_engine.hip do not cover:
//    * zero-metric links: next-hop sets then depend on the heap's pop order
//      among equal-metric nodes (LinkState.h:488-498), which this kernel
//      reproduces exactly -- (metric, node id) with ids ascending by name;
//    * negative metrics (an i32 adjacency metric becomes a huge u64 and the
//      sums wrap, LinkState.h:22, LinkState.cpp:151-152) and graphs whose
//      longest path does not fit 32 bits: u64 labels throughout;
//    * any graph size: all per-source state lives in HBM scratch.
//  Per source the wave keeps an indexed binary heap keyed (u64 metric, id)
//  -- lane 0 owns the heap, the labels and the node states, so they need no
//  cross-lane memory ordering -- pops the minimum, skips the expansion of
//  drained nodes other than the source (:831-838), and relaxes the popped
//  node's up links in linksFromNode order with the reference's rule
//  (:857-873): a strictly better label resets the head's next hops, a better
//  or equal one unions the tail's next hops into them and inserts the head
//  itself when the union is empty (tail = source).  Next-hop words are owned
//  by lane (word % 64), so every read of a word follows that lane's own
//  writes.  The pop rank of every node is recorded (the facade orders
//  pathLinks by it).
// ============================================================================
#include "engine_internal.h"

using namespace spfi;

namespace {

constexpr uint32_t kExactThreads = 256;  // 4 independent waves per block
constexpr uint8_t kUnseen = 0, kOpen = 1, kDone = 2;

struct ExactArgs {
  const uint32_t* row_ptr;
  const uint32_t* col;
  const int32_t* met;  // adjacency metrics as advertised (i32)
  const uint8_t* ovl;
  const uint32_t* link;
  const uint32_t* ign;     // optional link bitmap (linksToIgnore)
  const uint32_t* nb_ptr;  // distinct up neighbours (ascending id): next-hop bit order
  const uint32_t* nb_id;
  const uint32_t* srcs;
  uint32_t n_src, N, pitch, hop, dist64, Wmax;
  void* dist_out;          // [n_src][pitch] u32 or u64
  uint32_t* nh_out;        // planar next-hop bitmaps
  const uint64_t* nh_off;  // [n_src]
  uint32_t* pop_out;       // optional [n_src][pitch] pop rank (kInf = unreached)
  uint8_t* scratch;
  uint64_t per_wave;
  uint32_t* ctr;           // [1] next source
  uint32_t waves;          // waves with scratch; surplus waves of the last block exit
};

struct Scratch {
  uint64_t* key;
  uint32_t* hpos;  // heap position while open, pop rank once done
  uint32_t* heap;
  uint8_t* state;
  uint32_t* nh;  // [N][W]
};

__device__ __forceinline__ bool heap_less(const Scratch& s, uint32_t a, uint32_t b) {
  const uint64_t ka = s.key[a], kb = s.key[b];
  return ka < kb || (ka == kb && a < b);
}

__device__ void sift_up(const Scratch& s, uint32_t pos) {
  const uint32_t x = s.heap[pos];
  while (pos > 0) {
    const uint32_t par = (pos - 1) >> 1;
    const uint32_t y = s.heap[par];
    if (!heap_less(s, x, y)) break;
    s.heap[pos] = y;
    s.hpos[y] = pos;
    pos = par;
  }
  s.heap[pos] = x;
  s.hpos[x] = pos;
}

__device__ void sift_down(const Scratch& s, uint32_t pos, uint32_t size) {
  const uint32_t x = s.heap[pos];
  for (;;) {
    uint32_t c = 2 * pos + 1;
    if (c >= size) break;
    if (c + 1 < size && heap_less(s, s.heap[c + 1], s.heap[c])) ++c;
    const uint32_t y = s.heap[c];
    if (!heap_less(s, y, x)) break;
    s.heap[pos] = y;
    s.hpos[y] = pos;
    pos = c;
  }
  s.heap[pos] = x;
  s.hpos[x] = pos;
}

// bit index of v among src's distinct up neighbours (ascending ids), or kInf
__device__ uint32_t nbr_rank(const ExactArgs& a, uint32_t src, uint32_t v) {
  uint32_t lo = a.nb_ptr[src], hi = a.nb_ptr[src + 1];
  const uint32_t base = lo;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.nb_id[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo < a.nb_ptr[src + 1] && a.nb_id[lo] == v ? lo - base : kInf;
}

enum { kNone = 0, kReset = 1, kUnion = 2 };

__global__ __launch_bounds__(kExactThreads) void exact_spf_kernel(ExactArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (kExactThreads / 64) + (threadIdx.x >> 6);
  if (wave >= a.waves) return;  // wave-uniform: no scratch for it
  uint8_t* base = a.scratch + wave * a.per_wave;
  const uint32_t N = a.N, W = a.Wmax;
  Scratch s;
  s.key = reinterpret_cast<uint64_t*>(base);
  s.hpos = reinterpret_cast<uint32_t*>(base + 8ull * N);
  s.heap = s.hpos + N;
  s.nh = s.heap + N;
  s.state = reinterpret_cast<uint8_t*>(s.nh + (size_t)N * W);
  for (;;) {
    uint32_t i = 0;
    if (lane == 0) i = atomicAdd(a.ctr, 1u);
    i = __shfl(i, 0, 64);
    if (i >= a.n_src) break;
    const uint32_t src = a.srcs[i];
    const uint32_t k = a.nb_ptr[src + 1] - a.nb_ptr[src];
    const uint32_t Wk = (k + 31) / 32;  // words this source uses (<= W)
    for (uint32_t v = lane; v < N; v += 64) s.state[v] = kUnseen;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    uint32_t size = 0, pops = 0;
    if (lane == 0) {
      s.key[src] = 0;
      s.state[src] = kOpen;
      s.heap[0] = src;
      s.hpos[src] = 0;
      size = 1;
    }
    for (uint32_t w = lane; w < Wk; w += 64) s.nh[(size_t)src * W + w] = 0;
    size = __shfl(size, 0, 64);
    while (size > 0) {
      uint32_t u = 0;
      uint64_t du = 0;
      if (lane == 0) {
        u = s.heap[0];
        du = s.key[u];
        --size;
        if (size > 0) {
          s.heap[0] = s.heap[size];
          s.hpos[s.heap[0]] = 0;
          sift_down(s, 0, size);
        }
        s.state[u] = kDone;
        s.hpos[u] = pops;
      }
      ++pops;
      u = __shfl(u, 0, 64);
      du = ((uint64_t)__shfl((uint32_t)(du >> 32), 0, 64) << 32) | __shfl((uint32_t)du, 0, 64);
      size = __shfl(size, 0, 64);
      if (a.ovl[u] && u != src) continue;  // drained: recorded, not expanded
      const uint32_t e0 = a.row_ptr[u], e1 = a.row_ptr[u + 1];
      for (uint32_t eb = e0; eb < e1; eb += 64) {
        const uint32_t e = eb + lane;
        bool cand = e < e1;
        uint32_t v = 0;
        uint64_t nd = 0;
        if (cand) {
          if (a.ign && ((a.ign[a.link[e] >> 5] >> (a.link[e] & 31)) & 1u)) cand = false;
          v = a.col[e];
          nd = du + (a.hop ? 1ull : (uint64_t)(int64_t)a.met[e]);  // u64 wrap as the reference
        }
        for (uint64_t m = __ballot(cand); m; m &= m - 1) {  // linksFromNode order
          const int l = __builtin_ctzll(m);
          const uint32_t hv = __shfl(v, l, 64);
          const uint64_t hd = ((uint64_t)__shfl((uint32_t)(nd >> 32), l, 64) << 32) |
                              __shfl((uint32_t)nd, l, 64);
          int act = kNone;
          if (lane == 0) {
            const uint8_t st = s.state[hv];
            if (st == kUnseen) {
              s.state[hv] = kOpen;
              s.key[hv] = hd;
              s.heap[size] = hv;
              sift_up(s, size);
              ++size;
              act = kReset;
            } else if (st == kOpen) {
              if (hd < s.key[hv]) {
                s.key[hv] = hd;
                sift_up(s, s.hpos[hv]);
                act = kReset;
              } else if (hd == s.key[hv]) {
                act = kUnion;
              }
            }
          }
          act = __shfl(act, 0, 64);
          size = __shfl(size, 0, 64);
          if (act == kNone) continue;
          uint32_t any = 0;
          for (uint32_t w = lane; w < Wk; w += 64) {
            uint32_t* dst = &s.nh[(size_t)hv * W + w];
            uint32_t x = act == kReset ? 0u : *dst;
            if (u != src) x |= s.nh[(size_t)u * W + w];
            *dst = x;
            any |= x;
          }
          if (!__ballot(any != 0)) {  // empty union (tail = source): the head itself
            const uint32_t b = nbr_rank(a, src, hv);
            if (b != kInf && lane == ((b >> 5) & 63)) s.nh[(size_t)hv * W + (b >> 5)] |= 1u << (b & 31);
          }
        }
      }
    }
    // ---- outputs: distances, pop ranks, planar next-hop bitmaps ----
    for (uint32_t v = lane; v < a.pitch; v += 64) {
      const bool done = v < N && s.state[v] == kDone;
      const uint64_t d = done ? s.key[v] : ~0ull;
      if (a.dist64) {
        reinterpret_cast<uint64_t*>(a.dist_out)[(size_t)i * a.pitch + v] = v < N ? d : 0ull;
      } else {
        reinterpret_cast<uint32_t*>(a.dist_out)[(size_t)i * a.pitch + v] =
            v < N ? (done ? (uint32_t)d : kInf) : 0u;
      }
      if (a.pop_out) a.pop_out[(size_t)i * a.pitch + v] = done ? s.hpos[v] : kInf;
    }
    const uint32_t wpm = a.pitch / 32;
    for (uint64_t x = lane; x < (uint64_t)k * wpm; x += 64) {
      const uint32_t j = (uint32_t)(x / wpm), wv = (uint32_t)(x % wpm);
      uint32_t word = 0;
      for (uint32_t b = 0; b < 32; ++b) {
        const uint32_t v = wv * 32 + b;
        if (v < N && s.state[v] == kDone && ((s.nh[(size_t)v * W + (j >> 5)] >> (j & 31)) & 1u))
          word |= 1u << b;
      }
      a.nh_out[a.nh_off[i] + x] = word;
    }
  }
}

}  // namespace

namespace spfi {

// Scratch of the exact kernel for up to `n_src` sources with at most `Wmax`
// next-hop words per node: waves x (16N + 4NW + N) bytes, at most 4 GB, at
// most 16 waves per CU.  Allocation happens here (plan build / one-shot
// solves), never inside spf_plan_execute.
spf_status exact_reserve(spf_ctx* c, ExactScratch* x, uint32_t n_src, uint32_t Wmax) {
  const uint64_t N = c->N;
  const uint64_t W = std::max<uint32_t>(Wmax, 1);
  x->per_wave = ((8 * N + 8 * N + 4 * N * W + N) + 255) & ~uint64_t(255);
  x->wmax = (uint32_t)W;
  constexpr uint64_t kBudget = 4ull << 30;
  uint64_t waves = std::min<uint64_t>(std::max<uint32_t>(n_src, 1), std::max<uint64_t>(1, kBudget / x->per_wave));
  waves = std::min<uint64_t>(waves, 16ull * c->n_cu);
  x->waves = (uint32_t)waves;
  HIP_TRY(c, x->buf.alloc(waves * x->per_wave));
  HIP_TRY(c, x->ctr.alloc(1));
  return SPF_OK;
}

// Enqueue the exact kernel over the plan's sources (include/openr_spf.h
// SPF_FLAG_DIST64, and every plan outside the fast kernels' envelope).  No
// allocation, no host synchronisation: the scratch `x` (reserved for at
// least Wmax words) belongs to the caller -- the plan, or the context for
// the synchronous one-shot solves.
spf_status launch_exact(spf_ctx* c, ExactScratch* x, const uint32_t* d_srcs, uint32_t n_src,
                        const uint64_t* d_nh_off, uint32_t Wmax, bool hop, bool dist64,
                        const uint32_t* ign, void* d_dist, uint32_t* d_nh, uint32_t* d_pop,
                        hipStream_t s) {
  if (!x->buf.p || !x->ctr.p || Wmax > x->wmax)
    return fail(c, SPF_E_STATE, "exact kernel scratch not reserved for %u next-hop words", Wmax);
  HIP_TRY(c, hipMemsetAsync(x->ctr.p, 0, 4, s));
  const uint32_t waves = std::min<uint32_t>(x->waves, std::max<uint32_t>(n_src, 1));
  const uint32_t blocks = (waves + 3) / 4;
  ExactArgs a{c->d_row_ptr.p, c->d_col.p, c->d_met.p, c->d_ovl.p, c->d_link.p, ign,
              c->d_nb_ptr.p, c->d_nb_id.p, d_srcs, n_src, c->N, c->pitch, hop ? 1u : 0u,
              dist64 ? 1u : 0u, x->wmax, d_dist, d_nh, d_nh_off, d_pop, x->buf.p,
              x->per_wave, x->ctr.p, waves};
  hipLaunchKernelGGL(exact_spf_kernel, dim3(blocks), dim3(kExactThreads), 0, s, a);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

}  // namespace spfi
