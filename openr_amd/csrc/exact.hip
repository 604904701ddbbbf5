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

__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t shfl64(uint64_t x, int l) {
  return ((uint64_t)__shfl((uint32_t)(x >> 32), l, 64) << 32) | __shfl((uint32_t)x, l, 64);
}

// runSpf(src, useLinkMetric, linksToIgnore) replayed by one wave in its
// scratch: links in the bitmap `ign` (may be NULL) and the link `skip`
// (kInf: none) are ignored.  NH: maintain the next-hop words (Wk per node)
// -- KSP2 needs only labels and pop ranks.  Afterwards state[v] == kDone for
// every reached node, key[v] = its metric, hpos[v] = its pop rank.
template <bool NH>
__device__ void heap_spf(const ExactArgs& a, const Scratch& s, uint32_t src, uint32_t Wk,
                         const uint32_t* ign, uint32_t skip) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t N = a.N, W = a.Wmax;
  for (uint32_t v = lane; v < N; v += 64) s.state[v] = kUnseen;
  wave_fence();
  uint32_t size = 0, pops = 0;
  if (lane == 0) {
    s.key[src] = 0;
    s.state[src] = kOpen;
    s.heap[0] = src;
    s.hpos[src] = 0;
    size = 1;
  }
  if (NH)
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
    du = shfl64(du, 0);
    size = __shfl(size, 0, 64);
    if (a.ovl[u] && u != src) continue;  // drained: recorded, not expanded
    const uint32_t e0 = a.row_ptr[u], e1 = a.row_ptr[u + 1];
    for (uint32_t eb = e0; eb < e1; eb += 64) {
      const uint32_t e = eb + lane;
      bool cand = e < e1;
      uint32_t v = 0;
      uint64_t nd = 0;
      if (cand) {
        const uint32_t l = a.link[e];
        if ((ign && ((ign[l >> 5] >> (l & 31)) & 1u)) || l == skip) cand = false;
        v = a.col[e];
        nd = du + (a.hop ? 1ull : (uint64_t)(int64_t)a.met[e]);  // u64 wrap as the reference
      }
      for (uint64_t m = __ballot(cand); m; m &= m - 1) {  // linksFromNode order
        const int l = __builtin_ctzll(m);
        const uint32_t hv = __shfl(v, l, 64);
        const uint64_t hd = shfl64(nd, l);
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
        if (!NH || act == kNone) continue;
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
  wave_fence();  // outputs below read other lanes' next-hop words
}

__device__ __forceinline__ Scratch wave_scratch(const ExactArgs& a, uint64_t wave) {
  uint8_t* base = a.scratch + wave * a.per_wave;
  const uint32_t N = a.N;
  Scratch s;
  s.key = reinterpret_cast<uint64_t*>(base);
  s.hpos = reinterpret_cast<uint32_t*>(base + 8ull * N);
  s.heap = s.hpos + N;
  s.nh = s.heap + N;
  s.state = reinterpret_cast<uint8_t*>(s.nh + (size_t)N * a.Wmax);
  return s;
}

__global__ __launch_bounds__(kExactThreads) void exact_spf_kernel(ExactArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (kExactThreads / 64) + (threadIdx.x >> 6);
  if (wave >= a.waves) return;  // wave-uniform: no scratch for it
  const uint32_t N = a.N, W = a.Wmax;
  const Scratch s = wave_scratch(a, wave);
  for (;;) {
    uint32_t i = 0;
    if (lane == 0) i = atomicAdd(a.ctr, 1u);
    i = __shfl(i, 0, 64);
    if (i >= a.n_src) break;
    const uint32_t src = a.srcs[i];
    const uint32_t k = a.nb_ptr[src + 1] - a.nb_ptr[src];
    const uint32_t Wk = (k + 31) / 32;  // words this source uses (<= W)
    heap_spf<true>(a, s, src, Wk, a.ign, kInf);
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
    for (uint64_t x = lane; a.nh_out && x < (uint64_t)k * wpm; x += 64) {
      const uint32_t j = (uint32_t)(x / wpm), wv = (uint32_t)(x % wpm);
      uint32_t word = 0;
      for (uint32_t b = 0; b < 32; ++b) {
        const uint32_t v = wv * 32 + b;
        if (v < N && s.state[v] == kDone && ((s.nh[(size_t)v * W + (j >> 5)] >> (j & 31)) & 1u))
          word |= 1u << b;
      }
      a.nh_out[a.nh_off[i] + x] = word;
    }
    wave_fence();  // the next source's init overwrites the state this read
  }
}

// ---------------------------------------------------------------------------
//  what-if batches outside the positive-metric envelope (zero / negative
//  metrics, u64 labels): runSpf(src, true, {l}) per failed link l replayed by
//  a wave and reduced to the digest of include/openr_spf.h against the
//  unfailed result.  A failure neither direction of which is a pathLink of
//  the unfailed run (tight, tail expanded and popped before the head) leaves
//  the run unchanged: relaxing a link that never sets a final label changes
//  no key a pop reads, so the pop sequence, the labels and the next hops are
//  the same -- its digest is the unfailed one.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ex_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct ExactWiArgs {
  const uint32_t* fails;      // [n_fail] link ids
  const uint32_t* link_edge;  // [max_link + 1] one directed edge of each link
  const uint32_t* rev;        // [E]
  uint32_t n_fail, src;
  uint64_t* base_d;   // [N] unfailed labels (~0 = unreached)
  uint32_t* base_pop; // [N] unfailed pop ranks
  uint32_t* base_nh;  // [N][Wmax] unfailed next-hop words
  spf_whatif_digest* out;  // [n_fail] (base run: the unfailed digest)
  uint32_t base_run;  // 1: the unfailed run, writes base_* and out[0] = {0, 0, H}
};

// is directed edge e = u -> v a pathLink of the unfailed run?
__device__ bool base_tight(const ExactArgs& a, const ExactWiArgs& w, uint32_t e, uint32_t src) {
  uint32_t u = a.col[w.rev[e]];  // tail of e
  const uint32_t v = a.col[e];
  if (a.ovl[u] && u != src) return false;
  if (w.base_pop[u] == kInf || w.base_pop[v] == kInf || w.base_pop[u] >= w.base_pop[v]) return false;
  return w.base_d[u] + (uint64_t)(int64_t)a.met[e] == w.base_d[v];
}

__global__ __launch_bounds__(kExactThreads) void exact_whatif_kernel(ExactArgs a, ExactWiArgs w) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (kExactThreads / 64) + (threadIdx.x >> 6);
  if (wave >= a.waves) return;
  const uint32_t N = a.N, W = a.Wmax, src = w.src;
  const uint32_t k = a.nb_ptr[src + 1] - a.nb_ptr[src];
  const uint32_t Wk = (k + 31) / 32;
  const Scratch s = wave_scratch(a, wave);
  const uint32_t n_tasks = w.base_run ? 1u : w.n_fail;
  for (;;) {
    uint32_t i = 0;
    if (lane == 0) i = atomicAdd(a.ctr, 1u);
    i = __shfl(i, 0, 64);
    if (i >= n_tasks) break;
    const uint32_t l = w.base_run ? kInf : w.fails[i];
    if (!w.base_run) {
      const uint32_t e = w.link_edge[l], r = w.rev[e];
      if (!base_tight(a, w, e, src) && !base_tight(a, w, r, src)) {
        if (lane == 0) w.out[i] = spf_whatif_digest{0u, 0u, 0ull};  // marker: unchanged
        continue;
      }
    }
    heap_spf<true>(a, s, src, Wk, nullptr, l);
    uint64_t h = 0;
    uint32_t nd = 0, nn = 0;
    for (uint32_t v = lane; v < N; v += 64) {
      const bool done = s.state[v] == kDone;
      uint64_t f = 0xcbf29ce484222325ull;
      bool nh_diff = false;
      if (done)
        for (uint32_t x = 0; x < Wk; ++x) {
          const uint32_t word = s.nh[(size_t)v * W + x];
          f ^= word;
          f *= 0x100000001b3ull;
          if (w.base_run) w.base_nh[(size_t)v * W + x] = word;
          else nh_diff |= word != w.base_nh[(size_t)v * W + x];
        }
      const uint64_t d = done ? s.key[v] : ~0ull;
      if (done) h += ex_mix64(ex_mix64((uint64_t)v + 1) + d) ^ f;
      if (w.base_run) {
        w.base_d[v] = d;
        w.base_pop[v] = done ? s.hpos[v] : kInf;
      } else {
        const uint64_t bd = w.base_d[v];
        nd += d != bd;
        nn += (done != (bd != ~0ull)) || nh_diff;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      h += shfl64(h, lane ^ o);
      nd += __shfl_xor(nd, o, 64);
      nn += __shfl_xor(nn, o, 64);
    }
    if (lane == 0) w.out[i] = spf_whatif_digest{nd, nn, h};
    wave_fence();
  }
}

// cold failures were marked {0, 0, 0}: they get the unfailed digest
__global__ void exact_whatif_fill_kernel(spf_whatif_digest* out, uint32_t n,
                                         const spf_whatif_digest* base) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const spf_whatif_digest d = out[i];
  if (d.n_dist_changed == 0 && d.n_nh_changed == 0 && d.hash == 0) out[i] = *base;
}

// ---------------------------------------------------------------------------
//  KSP2 outside the batched kernel's envelope (zero / negative metrics, u64
//  labels, graphs past the LDS): getKthPaths(src, d, 1) and (src, d, 2)
//  (LinkState.cpp:762-791) per pair on one wave.  k = 1 traces the source's
//  run (labels + pop ranks from exact_spf_kernel); k = 2 replays
//  runSpf(src, true, links of the k = 1 paths) in the wave's scratch and
//  traces that.  traceOnePath (:398-419) walks pathLinks in their stored
//  order = pop rank of the tail, then the tail's linksFromNode order (CSR
//  edge order): the DFS step takes the untried tight in-edge u -> v
//  (u expanded, popped before v, label(u) + metric = label(v), u64 wrap)
//  with the smallest (pop(u), edge id); a link tried stays visited.
// ---------------------------------------------------------------------------
struct ExactKspArgs {
  const uint64_t* D;    // [n_src][pitch] k = 1 labels (~0 = unreached)
  const uint32_t* POP;  // [n_src][pitch] k = 1 pop ranks (kInf = unreached)
  const uint32_t* rev;
  uint32_t lw;          // link bitmap words
  spf_ksp2_pair* pairs;
  uint32_t* pool;
  uint64_t cap;
  unsigned long long* counters;  // [0] words claimed, [1] k = 2 runs, [2] bit 0 overflow
};

struct RowAcc {  // labels / pop ranks of a k = 1 row
  const uint64_t* d;
  const uint32_t* pop;
  __device__ uint64_t dist(uint32_t v) const { return d[v]; }
  __device__ uint32_t rank(uint32_t v) const { return pop[v]; }
};
struct ScratchAcc {  // the wave's replayed k = 2 run
  Scratch s;
  __device__ uint64_t dist(uint32_t v) const { return s.key[v]; }
  __device__ uint32_t rank(uint32_t v) const { return s.state[v] == kDone ? s.hpos[v] : kInf; }
};

__device__ __forceinline__ bool test_bit(const uint32_t* bm, uint32_t i) {
  return (bm[i >> 5] >> (i & 31)) & 1u;
}

__device__ __forceinline__ uint64_t wave_min64_ex(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = shfl64(x, (threadIdx.x & 63) ^ o);
    x = y < x ? y : x;
  }
  return x;
}

template <class ACC>
__device__ bool trace_exact(const ExactArgs& a, const ExactKspArgs& k, const ACC& acc,
                            const uint32_t* ign, uint32_t* vis, uint32_t* stack, uint32_t src,
                            uint32_t dst, uint32_t* depth) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t n = 0, v = dst;
  for (;;) {
    if (v == src) {
      *depth = n;
      return true;
    }
    const uint32_t pv = acc.rank(v);
    const uint64_t dv = acc.dist(v);
    uint64_t best = ~0ull;
    const uint32_t e_end = a.row_ptr[v + 1];
    for (uint32_t e = a.row_ptr[v] + lane; e < e_end; e += 64) {
      const uint32_t u = a.col[e], r = k.rev[e], l = a.link[e];
      if (a.ovl[u] && u != src) continue;  // not expanded
      if (test_bit(vis, l) || (ign && test_bit(ign, l))) continue;
      const uint32_t pu = acc.rank(u);
      if (pu == kInf || pu >= pv) continue;
      if (acc.dist(u) + (uint64_t)(int64_t)a.met[r] != dv) continue;
      const uint64_t key = ((uint64_t)pu << 32) | r;
      best = key < best ? key : best;
    }
    best = wave_min64_ex(best);
    if (best == ~0ull) {  // every pathLink of v tried: back up one level
      if (n == 0) return false;
      --n;
      v = n == 0 ? dst : a.col[k.rev[stack[n - 1]]];
      continue;
    }
    const uint32_t r = (uint32_t)best;
    if (lane == 0) {
      const uint32_t l = a.link[r];
      vis[l >> 5] |= 1u << (l & 31);
      stack[n] = r;
    }
    wave_fence();
    ++n;
    v = a.col[k.rev[r]];  // tail of r
  }
}

// pool record [n_links, next, links src->dst] chained after prev_at; marks
// the links in `mark` when given.  Lane 0 writes (the slow envelope).
__device__ uint32_t emit_exact(const ExactArgs& a, const ExactKspArgs& k, const uint32_t* stack,
                               uint32_t depth, uint32_t prev_at, uint32_t* mark) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t at = kInf;
  if (lane == 0) {
    const uint64_t base = atomicAdd(&k.counters[0], (unsigned long long)(depth + 2));
    if (base + depth + 2 > k.cap || base + depth + 2 > 0xFFFFFFF0ull) {
      atomicOr(reinterpret_cast<uint32_t*>(k.counters + 2), 1u);
    } else {
      at = (uint32_t)base;
      k.pool[at] = depth;
      k.pool[(size_t)at + 1] = kInf;
      for (uint32_t j = 0; j < depth; ++j) k.pool[(size_t)at + 2 + j] = a.link[stack[depth - 1 - j]];
      if (prev_at != kInf) k.pool[(size_t)prev_at + 1] = at;
    }
    if (mark)
      for (uint32_t j = 0; j < depth; ++j) {
        const uint32_t l = a.link[stack[j]];
        mark[l >> 5] |= 1u << (l & 31);
      }
  }
  wave_fence();
  return __shfl(at, 0, 64);
}

__global__ __launch_bounds__(kExactThreads) void exact_ksp2_kernel(ExactArgs a, ExactKspArgs k) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (kExactThreads / 64) + (threadIdx.x >> 6);
  if (wave >= a.waves) return;
  const uint32_t N = a.N;
  const Scratch s = wave_scratch(a, wave);
  // behind the heap scratch: vis [lw], ign [lw], stack [N]
  uint32_t* vis = reinterpret_cast<uint32_t*>(a.scratch + wave * a.per_wave + a.per_wave - 4ull * (2ull * k.lw + N));
  uint32_t* ign = vis + k.lw;
  uint32_t* stack = ign + k.lw;
  const uint64_t n_pairs = (uint64_t)a.n_src * N;
  uint32_t k2_runs = 0;
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(a.ctr, 1u);
    t = __shfl(t, 0, 64);
    if (t >= n_pairs) break;
    const uint32_t i = t / N, d = t % N;
    const uint32_t src = a.srcs[i];
    spf_ksp2_pair hdr;
    hdr.first[0] = hdr.first[1] = kInf;
    hdr.n_paths[0] = hdr.n_paths[1] = 0;
    const RowAcc row{k.D + (size_t)i * a.pitch, k.POP + (size_t)i * a.pitch};
    if (d != src && row.rank(d) != kInf) {
      for (uint32_t j = lane; j < k.lw; j += 64) vis[j] = ign[j] = 0;
      wave_fence();
      uint32_t depth = 0, prev = kInf, n1 = 0;
      while (trace_exact(a, k, row, nullptr, vis, stack, src, d, &depth) && depth) {
        prev = emit_exact(a, k, stack, depth, prev, ign);
        if (n1++ == 0) hdr.first[0] = prev;
      }
      hdr.n_paths[0] = n1;
      if (n1) {  // k = 2: runSpf(src, true, links of the k = 1 paths), trace
        ++k2_runs;
        heap_spf<false>(a, s, src, 0, ign, kInf);
        const ScratchAcc acc{s};
        if (acc.rank(d) != kInf) {
          for (uint32_t j = lane; j < k.lw; j += 64) vis[j] = 0;
          wave_fence();
          prev = kInf;
          uint32_t n2 = 0;
          while (trace_exact(a, k, acc, ign, vis, stack, src, d, &depth) && depth) {
            prev = emit_exact(a, k, stack, depth, prev, nullptr);
            if (n2++ == 0) hdr.first[1] = prev;
          }
          hdr.n_paths[1] = n2;
        }
      }
    }
    if (lane == 0) k.pairs[t] = hdr;
    wave_fence();
  }
  if (lane == 0 && k2_runs) atomicAdd(&k.counters[1], (unsigned long long)k2_runs);
}

}  // namespace

namespace spfi {

// Scratch of the exact kernel for up to `n_src` sources with at most `Wmax`
// next-hop words per node: waves x (16N + 4NW + N) bytes, at most 4 GB, at
// most 16 waves per CU.  Allocation happens here (plan build / one-shot
// solves), never inside spf_plan_execute.
spf_status exact_reserve(spf_ctx* c, ExactScratch* x, uint32_t n_src, uint32_t Wmax,
                         uint64_t extra) {
  const uint64_t N = c->N;
  const uint64_t W = std::max<uint32_t>(Wmax, 1);
  // (extra bytes per wave sit at the end of its slice: the KSP2 kernel's
  // bitmaps and DFS stack)
  x->per_wave = ((8 * N + 8 * N + 4 * N * W + N + 15) & ~uint64_t(15)) + ((extra + 255) & ~uint64_t(255));
  x->per_wave = (x->per_wave + 255) & ~uint64_t(255);
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

// ---- what-if on the exact kernel (include/openr_spf.h spf_whatif_*) ----
spf_status exact_whatif_prepare(spf_ctx* c, ExactWhatIf* x, uint32_t src,
                                const std::vector<uint32_t>& fails,
                                const std::vector<uint32_t>& link_edge) {
  const uint32_t k = c->nb_ptr[src + 1] - c->nb_ptr[src];
  x->src = src;
  x->n_fail = (uint32_t)fails.size();
  x->W = std::max<uint32_t>(1, (k + 31) / 32);
  spf_status st = exact_reserve(c, &x->xs, std::max<uint32_t>(1, x->n_fail), x->W, 0);
  if (st != SPF_OK) return st;
  if (fails.empty()) HIP_TRY(c, x->fails.alloc(1));
  else HIP_TRY(c, x->fails.upload(fails.data(), fails.size(), c->stream));
  HIP_TRY(c, x->link_edge.upload(link_edge.data(), link_edge.size(), c->stream));
  HIP_TRY(c, x->base_d.alloc(c->N));
  HIP_TRY(c, x->base_pop.alloc(c->N));
  HIP_TRY(c, x->base_nh.alloc((size_t)c->N * x->xs.wmax));
  HIP_TRY(c, x->base_dig.alloc(1));
  return SPF_OK;
}

spf_status exact_whatif_launch(spf_ctx* c, ExactWhatIf* x, spf_whatif_digest* d_out,
                               spf_whatif_digest* d_base, hipStream_t s, hipEvent_t mid) {
  ExactArgs a{c->d_row_ptr.p, c->d_col.p, c->d_met.p, c->d_ovl.p, c->d_link.p, nullptr,
              c->d_nb_ptr.p, c->d_nb_id.p, nullptr, 0, c->N, c->pitch, 0u, 1u, x->xs.wmax,
              nullptr, nullptr, nullptr, nullptr, x->xs.buf.p, x->xs.per_wave, x->xs.ctr.p, 1u};
  ExactWiArgs w{x->fails.p, x->link_edge.p, c->d_rev.p, x->n_fail, x->src, x->base_d.p,
                x->base_pop.p, x->base_nh.p, x->base_dig.p, 1u};
  HIP_TRY(c, hipMemsetAsync(x->xs.ctr.p, 0, 4, s));
  hipLaunchKernelGGL(exact_whatif_kernel, dim3(1), dim3(kExactThreads), 0, s, a, w);
  HIP_TRY(c, hipGetLastError());
  if (d_base)
    HIP_TRY(c, hipMemcpyAsync(d_base, x->base_dig.p, sizeof(spf_whatif_digest), hipMemcpyDeviceToDevice, s));
  if (mid) HIP_TRY(c, hipEventRecord(mid, s));
  if (x->n_fail == 0) return SPF_OK;
  a.waves = std::min<uint32_t>(x->xs.waves, x->n_fail);
  w.out = d_out;
  w.base_run = 0;
  HIP_TRY(c, hipMemsetAsync(x->xs.ctr.p, 0, 4, s));
  hipLaunchKernelGGL(exact_whatif_kernel, dim3((a.waves + 3) / 4), dim3(kExactThreads), 0, s, a, w);
  HIP_TRY(c, hipGetLastError());
  hipLaunchKernelGGL(exact_whatif_fill_kernel, dim3((x->n_fail + 255) / 256), dim3(256), 0, s, d_out,
                     x->n_fail, x->base_dig.p);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

// ---- KSP2 on the exact kernel (include/openr_spf.h spf_ksp2_*) ----
spf_status exact_ksp2_prepare(spf_ctx* c, ExactKsp2* x, const std::vector<uint32_t>& srcs) {
  x->n_src = (uint32_t)srcs.size();
  x->lw = c->max_link / 32 + 1;
  uint32_t wmax = 1;
  for (uint32_t s : srcs) wmax = std::max(wmax, (c->nb_ptr[s + 1] - c->nb_ptr[s] + 31) / 32);
  spf_status st = exact_reserve(c, &x->xs_a, x->n_src, wmax, 0);
  if (st != SPF_OK) return st;
  const uint64_t pairs = (uint64_t)x->n_src * c->N;
  st = exact_reserve(c, &x->xs_b, (uint32_t)std::min<uint64_t>(pairs, 0xFFFFFFFFull), 1,
                     4ull * (2ull * x->lw + c->N));
  if (st != SPF_OK) return st;
  if (pairs > 0xFFFFFFFFull) return fail(c, SPF_E_UNSUPPORTED, "KSP2: more than 2^32 pairs");
  HIP_TRY(c, x->srcs.upload(srcs.data(), srcs.size(), c->stream));
  HIP_TRY(c, x->D.alloc((size_t)x->n_src * c->pitch));
  HIP_TRY(c, x->POP.alloc((size_t)x->n_src * c->pitch));
  return SPF_OK;
}

spf_status exact_ksp2_launch(spf_ctx* c, ExactKsp2* x, spf_ksp2_pair* d_pairs, uint32_t* d_pool,
                             uint64_t pool_words, uint64_t* d_counters, hipStream_t s,
                             hipEvent_t mid) {
  spf_status st = launch_exact(c, &x->xs_a, x->srcs.p, x->n_src, nullptr, x->xs_a.wmax, false, true,
                               nullptr, x->D.p, nullptr, x->POP.p, s);
  if (st != SPF_OK) return st;
  if (mid) HIP_TRY(c, hipEventRecord(mid, s));
  const uint64_t pairs = (uint64_t)x->n_src * c->N;
  const uint32_t waves = (uint32_t)std::min<uint64_t>(x->xs_b.waves, pairs);
  ExactArgs a{c->d_row_ptr.p, c->d_col.p, c->d_met.p, c->d_ovl.p, c->d_link.p, nullptr,
              c->d_nb_ptr.p, c->d_nb_id.p, x->srcs.p, x->n_src, c->N, c->pitch, 0u, 1u,
              x->xs_b.wmax, nullptr, nullptr, nullptr, nullptr, x->xs_b.buf.p, x->xs_b.per_wave,
              x->xs_b.ctr.p, waves};
  ExactKspArgs k{reinterpret_cast<const uint64_t*>(x->D.p), x->POP.p, c->d_rev.p, x->lw, d_pairs,
                 d_pool, pool_words, reinterpret_cast<unsigned long long*>(d_counters)};
  HIP_TRY(c, hipMemsetAsync(x->xs_b.ctr.p, 0, 4, s));
  hipLaunchKernelGGL(exact_ksp2_kernel, dim3((waves + 3) / 4), dim3(kExactThreads), 0, s, a, k);
  HIP_TRY(c, hipGetLastError());
  return SPF_OK;
}

}  // namespace spfi
