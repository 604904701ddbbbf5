// ============================================================================
//  mssp.hip -- multi-source weighted SPF distances (positive metrics): S
//  sources per workgroup, their distance rows resident in LDS as packed u16
//  pairs, relaxed by min-plus pull sweeps over a sliced-ELL copy of the
//  in-edges until nothing changes.
//
//  Reference: LinkState::runSpf (openr/decision/LinkState.cpp:808-882) with
//  useLinkMetric = true; production metrics are RTT-derived
//  (openr/link-monitor/LinkMonitor.cpp:44-47), so the weighted path is the
//  one a deployment runs.  For positive metrics the final distances are the
//  order-free fixed point
//      d_s(s) = 0,  d_s(v) = min over up in-edges u -> v with u expanded
//                            (u == s or u not drained) of d_s(u) + w(u, v)
//  (DESIGN.md §3), which any sequence of monotone relaxations reaches; the
//  next-hop pass (ecmp_kernel) then works from the rows as for every other
//  distance kernel.
//
//  Layout: LDS row block dist[v][SD] (u32 words, each two u16 labels: source
//  2q in the low half, 2q + 1 in the high half), 0xFFFF = not reached, node N
//  = the all-unreached padding target of the ELL.  One pull sweep: each wave
//  owns whole 64-node slices (dealt by width, mp_smap), lane = node; for
//  every ELL column j the lane's in-neighbour u and in-weight w come in one
//  packed u32 (u | w << 16); a node whose labels did not change since the
//  last sweep it was read in is skipped (3 rotating change bitmaps; a column
//  is skipped by the whole wave when no lane's neighbour changed), otherwise
//  its SD words are read with one LDS load and folded into the lane's
//  accumulators with v_pk_add_u16 (clamp) + v_pk_min_u16: one instruction
//  pair per two sources.  Updates are in place (Gauss-Seidel); every value
//  ever written is the length of a real walk, so the result is exact once a
//  sweep changes nothing.  Drained nodes take labels but never set their
//  change bit, so they are never expanded; each source's own out-edges are
//  applied once at the start (a drained source is expanded, :831-838).
//
//  u8 labels (graphs whose metrics and hop diameter keep distances small:
//  RTT-derived fabric metrics, max(rtt/100, 1) <= 30 over <= 4 hops): four
//  sources per word, twice the sources per LDS byte -- a workgroup takes 4 SD
//  sources instead of 2 SD, so the pass needs half the workgroup rounds.  A
//  word is split into two u16x2 halves by v_perm (sources 0, 2 and 1, 3),
//  folded with the same v_pk_add_u16 clamp / v_pk_min_u16 pair into u16
//  accumulators, and packed back (clamped to 0xFF) when the node updates.
//
//  u16 labels: clamped sums are min(true, 0xFFFF) exactly, so a true
//  distance >= 0xFFFF shows up as some node in [0xFFFF - max metric,
//  0xFFFF) on its path; such rows are listed in `redo` and recomputed by
//  sssp_kernel (u32 labels).  The host skips that launch when the graph's
//  hop diameter bounds every distance below the threshold.
// ============================================================================
#include "engine_internal.h"

using namespace spfi;

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t add_sat2(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, a),
                                                                    __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t min2(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                __builtin_bit_cast(u16x2, b)));
}

constexpr int kMpThreads = 1024;
constexpr uint32_t kMpWaves = kMpThreads / 64;
constexpr uint32_t kMpNoSlice = 0xFFFFFFFFu;
constexpr size_t kMpMaxLds = 160 * 1024;
constexpr size_t kMpStaticLds = 256;  // the kernel's own static LDS (__syncthreads_or)
constexpr uint32_t kMpAhead = 8;      // packed in-edge loads per group (two groups in flight)

// LDS minimum of one label of a word (CAS loop: several sources share a
// word): label `slot` of width B bits (16: two per word, 8: four per word)
template <int B>
__device__ void lds_min_label(uint32_t* p, uint32_t slot, uint32_t val) {
  constexpr uint32_t M = (1u << B) - 1u;
  const uint32_t sh = slot * B;
  val = min(val, M);
  uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (;;) {
    const uint32_t cur = (old >> sh) & M;
    if (val >= cur) return;
    const uint32_t nw = (old & ~(M << sh)) | (val << sh);
    const uint32_t got = atomicCAS(p, old, nw);
    if (got == old) return;
    old = got;
  }
}

// u8 labels: the two u16x2 halves of a word (bytes 0, 2 and bytes 1, 3)
__device__ __forceinline__ uint32_t u8_lo(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c020c00u); }
__device__ __forceinline__ uint32_t u8_hi(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c030c01u); }

template <int SD>
__device__ __forceinline__ void load_words(const uint32_t* p, uint32_t (&d)[SD]) {
  if constexpr (SD == 4) {
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
  } else if constexpr (SD == 2) {
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    d[0] = x.x; d[1] = x.y;
  } else if constexpr (SD == 8) {
    const uint4 x = reinterpret_cast<const uint4*>(p)[0], y = reinterpret_cast<const uint4*>(p)[1];
    d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
    d[4] = y.x; d[5] = y.y; d[6] = y.z; d[7] = y.w;
  } else {
    d[0] = p[0];
  }
}

template <int SD, bool U8>
__global__ __launch_bounds__(kMpThreads) void mssp_kernel(
    const uint32_t* __restrict__ sell_ptr, const uint32_t* __restrict__ ell,
    const uint32_t* __restrict__ smap, uint32_t slots, const uint32_t* __restrict__ row_ptr,
    const uint32_t* __restrict__ col, const uint32_t* __restrict__ wt,
    const uint8_t* __restrict__ ovl, const uint32_t* __restrict__ rows_src, uint32_t n_rows,
    uint32_t N, uint32_t pitch, uint32_t* __restrict__ D, uint8_t* __restrict__ Dn,
    uint32_t ovf_at, uint32_t* __restrict__ redo, uint32_t alt,
    const uint32_t* __restrict__ dep /* [n_slices + 1] offsets, then out-slice lists; null: no skipping */,
    unsigned long long* __restrict__ stats /* diagnostics (SPF_STAMPS): [0] sweeps, [1] max, [2] WGs */,
    uint32_t* __restrict__ maxd /* sliced next-hop plans: largest finite distance (254: saturated) */,
    const uint32_t* __restrict__ cls /* [kMpWaves][n_cls]: first slot of each width class */,
    uint32_t n_cls /* > 1: phased sweeps go class by class, a barrier between */,
    uint32_t phase /* bits 0-7: leading sweeps phased; bit 8: odd phased sweeps narrow class first */) {
  constexpr uint32_t S = (U8 ? 4 : 2) * SD;  // sources per workgroup
  constexpr uint32_t LPW = U8 ? 4 : 2;       // labels per word
  constexpr uint32_t LB = U8 ? 8 : 16;       // label bits
  constexpr uint32_t LM = (1u << LB) - 1u;   // not reached / saturated
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t bw = (N + 32) / 32;  // change-bitmap words (nodes 0..N)
  uint32_t* dist = reinterpret_cast<uint32_t*>(smem);  // [(N + 1) * SD]
  uint32_t* bits = dist + (size_t)(N + 1) * SD;          // [3][bw]
  uint32_t* flag = bits + 3 * bw;                        // [3]
  const uint32_t n_slices = (N + 63) / 64, sw = (n_slices + 31) / 32;
  uint32_t* sbits = flag + 4;                            // [3][sw]: slices to sweep

  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t r0 = blockIdx.x * S;
  const uint32_t nb = min(S, n_rows - r0);

  for (uint32_t i = tid; i < (N + 1) * SD; i += kMpThreads) dist[i] = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < 3 * bw; i += kMpThreads) bits[i] = 0;
  for (uint32_t i = tid; i < 3 * sw; i += kMpThreads) sbits[i] = 0;
  if (tid < 3) flag[tid] = 0;
  __syncthreads();
  if (tid < nb) lds_min_label<LB>(&dist[rows_src[r0 + tid] * SD + tid / LPW], tid % LPW, 0);
  __syncthreads();
  // each source's own out-edges, once (a wave per source): the source is
  // expanded even when drained; its label 0 never changes again
  for (uint32_t si = wave; si < nb; si += kMpWaves) {
    const uint32_t s = rows_src[r0 + si];
    const uint32_t e1 = row_ptr[s + 1];
    for (uint32_t e = row_ptr[s] + lane; e < e1; e += 64) {
      const uint32_t v = col[e];
      lds_min_label<LB>(&dist[v * SD + si / LPW], si % LPW, wt[e]);
      if (!ovl[v]) atomicOr(&bits[v >> 5], 1u << (v & 31));
    }
  }
  __syncthreads();

  // the lane's drained bit of each of its wave's slots (bit k), once: the
  // sweeps test it without a global load
  uint32_t dmask = 0, n_my = 0;  // + the wave's slot count (filled from the front)
  {
    const uint32_t* wm = smap + __builtin_amdgcn_readfirstlane(wave) * slots;
    for (uint32_t k = 0; k < slots; ++k) {
      const uint32_t sl = wm[k];
      if (sl == kMpNoSlice) break;
      n_my = k + 1;
      const uint32_t v = sl * 64 + lane;
      if (k < 32 && v < N && ovl[v]) dmask |= 1u << k;
    }
    n_my = __builtin_amdgcn_readfirstlane(n_my);
  }
  for (uint32_t it = 0;; ++it) {
    // bitmap it % 3: nodes changed in sweep it - 1 or it (read by this
    // sweep; a change sets it and the next sweep's); (it + 2) % 3 is idle
    uint32_t* cur_w = bits + (it % 3) * bw;
    const uint32_t* cur = cur_w;
    uint32_t* nxt = bits + ((it + 1) % 3) * bw;
    uint32_t* old = bits + ((it + 2) % 3) * bw;  // read by nobody this sweep
    for (uint32_t i = tid; i < bw; i += kMpThreads) old[i] = 0;
    // slice-level dirt (dep != null): a slice is swept when one of its
    // in-neighbours changed in the previous sweep or this one (every slice in
    // the first sweep); a slice with a decreased non-drained node marks the
    // slices its out-edges reach
    const uint32_t* scur = sbits + (it % 3) * sw;
    uint32_t* snxt = sbits + ((it + 1) % 3) * sw;
    for (uint32_t i = tid; i < sw; i += kMpThreads) sbits[((it + 2) % 3) * sw + i] = 0;
    if (tid == 0) flag[(it + 1) % 3] = 0;
    bool changed = false;
    // the wave's slot table by scalar loads, the next slot's entry fetched
    // while this slot's columns run (a dependent smap -> sell_ptr chain per
    // slot was ~2 us of every sweep's critical path)
    const uint32_t* wmap = smap + __builtin_amdgcn_readfirstlane(wave) * slots;
    // odd sweeps walk the wave's slots backwards (narrow slices first): a
    // forward sweep carries paths whose hops go from wide to narrow nodes
    // (spine -> fabric -> rack switch), a backward one the opposite turns
    // phased sweeps (the first `phase & 0xFF`): every wave finishes its
    // slices of width class c before any wave starts the next class -- widest
    // first, or (bit 8, odd sweeps) narrowest first -- so labels flow hub ->
    // mid -> leaf (or back) within the sweep: a hop chain in class order
    // lands in one sweep instead of one per order inversion between waves
    const bool phased = n_cls > 1 && it < (phase & 0xFFu);
    const bool rev = phased && (phase & 0x100u) && (it & 1u);
    const bool back = phased ? rev : alt && (it & 1u);
    auto slot_at = [&](uint32_t k) { return back ? n_my - 1u - k : k; };
    uint32_t nsl = n_my ? wmap[slot_at(0)] : kMpNoSlice;
    uint32_t nb0 = nsl == kMpNoSlice ? 0u : sell_ptr[nsl], nb1 = nsl == kMpNoSlice ? 0u : sell_ptr[nsl + 1];
    // class barriers: forward, before the first slot of class pc (pc = 1 ..
    // n_cls - 1); backward, before the first slot below class pc's start
    // (pc = n_cls - 1 .. 1); a wave with no slot of a class meets its
    // barrier at the next class, or at the end
    uint32_t pc = back ? n_cls - 1u : 1u, n_bar = 0;
    const uint32_t* wcls = cls ? cls + __builtin_amdgcn_readfirstlane(wave) * n_cls : nullptr;
    for (uint32_t kk = 0; kk < n_my; ++kk) {
      const uint32_t k = slot_at(kk);
      if (phased) {
        if (!back)
          while (pc < n_cls && k == wcls[pc]) {
            __syncthreads();
            ++pc, ++n_bar;
          }
        else
          while (pc >= 1 && k < wcls[pc]) {
            __syncthreads();
            --pc, ++n_bar;
          }
      }
      const uint32_t sl = nsl;
      const uint32_t b = nb0, w = (nb1 - nb0) / 64;
      nsl = kk + 1 < n_my ? wmap[slot_at(kk + 1)] : kMpNoSlice;
      if (nsl != kMpNoSlice) {
        nb0 = sell_ptr[nsl];
        nb1 = sell_ptr[nsl + 1];
      }
      if (dep && it > 0 &&
          !(__builtin_amdgcn_readfirstlane(scur[sl >> 5] | snxt[sl >> 5]) >> (sl & 31) & 1u))
        continue;  // no in-neighbour changed since this slice's last sweep
      if (stats && lane == 0) {  // slices swept (diagnostics): total, per sweep
        atomicAdd(&stats[3], 1ull);
        atomicAdd(&stats[4 + min(it, 11u)], 1ull);
      }
      const uint32_t v = sl * 64 + lane;
      // u16x2 accumulators: SD of them (u16 labels), 2 SD (u8 labels: the
      // lo / hi halves of each word)
      constexpr int NA = U8 ? 2 * SD : SD;
      uint32_t acc[NA];
#pragma unroll
      for (int q = 0; q < NA; ++q) acc[q] = 0xFFFFFFFFu;
      bool got = false;
      const uint32_t* ep = ell + b + lane;
      // the slice's packed in-edges kMpAhead columns at a time, the next
      // group's loads in flight while this group's labels are folded (one
      // entry in flight made every column an L2 round trip)
      // a group of kMpAhead columns: every change-bit read issued, then
      // every label read of the lanes whose neighbour changed (exec-masked,
      // all in flight), then the folds -- the per-column chain of two
      // dependent LDS round trips bounded the sweep (5.7 sweeps of ~67 us)
      auto fold = [&](const uint32_t (&e)[kMpAhead], uint32_t n) {
        uint32_t cw[kMpAhead];
#pragma unroll
        for (int t = 0; t < (int)kMpAhead; ++t) {
          const uint32_t u = e[t] & 0xFFFFu;
          cw[t] = cur[u >> 5];  // changed in the previous sweep or this one
        }
        uint32_t d[kMpAhead][SD];
        bool c[kMpAhead];
#pragma unroll
        for (int t = 0; t < (int)kMpAhead; ++t) {
          const uint32_t u = e[t] & 0xFFFFu;
          c[t] = (uint32_t)t < n && ((cw[t] >> (u & 31)) & 1u);
          if (c[t]) load_words<SD>(&dist[u * SD], d[t]);
        }
#pragma unroll
        for (int t = 0; t < (int)kMpAhead; ++t)
          if (c[t]) {
            const uint32_t wp = __builtin_amdgcn_perm(e[t], e[t], 0x03020302u);  // w | w << 16
            if constexpr (U8) {
#pragma unroll
              for (int q = 0; q < SD; ++q) {
                acc[2 * q] = min2(acc[2 * q], add_sat2(u8_lo(d[t][q]), wp));
                acc[2 * q + 1] = min2(acc[2 * q + 1], add_sat2(u8_hi(d[t][q]), wp));
              }
            } else {
#pragma unroll
              for (int q = 0; q < SD; ++q) acc[q] = min2(acc[q], add_sat2(d[t][q], wp));
            }
            got = true;
          }
      };
      uint32_t ea[kMpAhead], eb[kMpAhead];
      auto load = [&](uint32_t j0, uint32_t (&e)[kMpAhead]) {
#pragma unroll
        for (int t = 0; t < (int)kMpAhead; ++t) {
          // unconditional (the ELL is padded past its last slice): a
          // branch per column made the compiler drain every load in flight
          // (vmcnt(0)) before each group's folds
          // (columns past the slice's w read the next slice's entries --
          // valid node ids -- and fold() never uses them: t < n)
          e[t] = ep[(j0 + t) * 64];
        }
      };
      // every group load unconditional (the ELL is padded): a load under a
      // branch makes the join's wait count drain the loads in flight
      load(0, ea);
      for (uint32_t j0 = 0; j0 < w; j0 += 2 * kMpAhead) {
        load(j0 + kMpAhead, eb);
        fold(ea, w - j0);
        load(j0 + 2 * kMpAhead, ea);
        if (j0 + kMpAhead < w) fold(eb, w - j0 - kMpAhead);
      }
      bool expands = false;
      if (got && v < N) {
        uint32_t* dv = &dist[v * SD];
        bool dec = false;
#pragma unroll
        for (int q = 0; q < SD; ++q) {
          const uint32_t o = dv[q];
          uint32_t nn;
          if constexpr (U8) {  // per byte min(old, clamp(acc, 0xFF)), packed back
            const uint32_t lo = min2(u8_lo(o), acc[2 * q]), hi = min2(u8_hi(o), acc[2 * q + 1]);
            nn = lo | (hi << 8);
          } else {
            nn = min2(o, acc[q]);
          }
          if (nn != o) {
            dv[q] = nn;
            dec = true;
          }
        }
        if (dec) {
          changed = true;
          if (stats) atomicAdd(&stats[16 + min(it, 11u)], 1ull);  // nodes decreased per sweep
          expands = k < 32 ? !((dmask >> k) & 1u) : !ovl[v];
          if (expands) {  // seen as changed by this sweep and the next
            atomicOr(&cur_w[v >> 5], 1u << (v & 31));
            atomicOr(&nxt[v >> 5], 1u << (v & 31));
          }
        }
      }
      // (whole wave: every lane takes its share of the list)
      if (dep && __builtin_amdgcn_ballot_w64(expands)) {
        const uint32_t d0 = dep[sl], d1 = dep[sl + 1];
        for (uint32_t t = d0 + lane; t < d1; t += 64) {
          const uint32_t o = dep[t];
          atomicOr(&snxt[o >> 5], 1u << (o & 31));
        }
      }
    }
    if (phased)  // the class barriers this wave has no slices for
      for (; n_bar + 1 < n_cls; ++n_bar) __syncthreads();
    if (__builtin_amdgcn_ballot_w64(changed) && lane == 0) flag[it % 3] = 1;
    __syncthreads();
    if (!flag[it % 3]) {
      if (stats && tid == 0) {
        atomicAdd(&stats[0], (unsigned long long)(it + 1));
        atomicMax(&stats[1], (unsigned long long)(it + 1));
        atomicAdd(&stats[2], 1ull);
      }
      break;
    }
  }

  // ---- rows: u32 (kInf = unreached, and past N as sssp_kernel) and the
  // u8 copy next-hop pass; overflow-suspect rows go to `redo` ----
  uint32_t dmax = 0;  // largest finite distance this thread wrote
  for (uint32_t si = 0; si < nb; ++si) {
    const uint32_t row = r0 + si;
    uint32_t ovf = 0;
    for (uint32_t q = tid; q < pitch / 4; q += kMpThreads) {
      uint32_t o[4];
      uint32_t nb8 = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t v = 4 * q + t;
        uint32_t d = kInf;
        if (v < N) {
          const uint32_t x = dist[v * SD + si / LPW];
          const uint32_t h = (x >> ((si % LPW) * LB)) & LM;
          if (h != LM) {
            d = h;
            ovf |= h >= ovf_at;
            dmax = max(dmax, h);
          }
        }
        o[t] = d;
        nb8 |= (d == kInf ? 0xFFu : min(d, 254u)) << (8 * t);
      }
      {  // streaming store: the rows are outputs (the next-hop pass reads the u8 copy)
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u x = {o[0], o[1], o[2], o[3]};
        __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(D + (size_t)row * pitch) + q);
      }
      if (Dn) reinterpret_cast<uint32_t*>(Dn + (size_t)row * pitch)[q] = nb8;
    }
    if (__syncthreads_or(ovf) && tid == 0) {
      if (redo) redo[1 + atomicAdd(redo, 1u)] = row;
      if (maxd) atomicMax(maxd, 254u);  // a redone row may be deep: the bit planes do not apply
    }
  }
  if (maxd) {  // one atomic per wave
    for (int o = 32; o >= 1; o >>= 1) dmax = max(dmax, (uint32_t)__shfl_xor((int)dmax, o));
    if ((tid & 63) == 0 && dmax) atomicMax(maxd, dmax);
  }
}

size_t mp_lds(uint32_t N, uint32_t SD) {
  return 4ull * (N + 1) * SD + 4ull * 3 * ((N + 32) / 32) + 16 + 4ull * 3 * (((N + 63) / 64 + 31) / 32);
}

bool mp_fits(uint32_t N, uint32_t sd) {
  return 4ull * (N + 1) * sd + 4ull * 3 * ((N + 32) / 32) + 16 + 4ull * 3 * (((N + 63) / 64 + 31) / 32) +
             kMpStaticLds <=
         kMpMaxLds;
}

}  // namespace

namespace spfi {

// Dwords per node of mssp_kernel's LDS rows (sources per workgroup / 2) for
// this graph, 0 when the multi-source kernel does not apply: positive
// metrics below 2^16 - 1, node ids below 2^16 (packed ELL entries), rows of
// at least two sources in LDS.  SPF_MSSP=0 turns it off (A/B, tests).
uint32_t mssp_words(const spf_ctx* c) {
  if (const char* e = std::getenv("SPF_MSSP"))
    if (e[0] == '0') return 0;
  if (c->nonpos || c->max_metric >= 0xFFFFu || c->N >= 0xFFFFu) return 0;
  if (const char* e = std::getenv("SPF_MSSP_SD")) {  // A/B: fixed sources per workgroup
    const uint32_t sd = (uint32_t)atoi(e);
    return (sd == 1 || sd == 2 || sd == 4 || sd == 8) && mp_fits(c->N, sd) ? sd : 0;
  }
  for (uint32_t sd : {8u, 4u, 2u, 1u})
    if (mp_fits(c->N, sd)) return sd;
  return 0;
}

// The packed in-edge ELL (u | w(u -> v) << 16 at the sliced-ELL position of
// v's j-th CSR edge, padding N | 0) and the per-wave slice map, rebuilt when
// the graph changed (metrics are patchable in place).  Also the bound that
// decides whether any row can overflow u16 labels.
spf_status mssp_prepare(spf_ctx* c) {
  if (c->mp_epoch == c->epoch && c->d_mp_ell.p) return SPF_OK;
  const uint32_t N = c->N;
  const uint32_t n_slices = (N + 63) / 64;
  // (+ 4 groups of kMpAhead columns of padding: the kernel's column loads
  // run unconditionally up to two groups past a slice's last column)
  std::vector<uint32_t> ell(c->sell_ptr.back() + 4ull * kMpAhead * 64, N);
  for (uint32_t v = 0; v < N; ++v) {
    const uint32_t sl = v / 64, ln = v % 64;
    for (uint32_t j = 0; j < c->row_ptr[v + 1] - c->row_ptr[v]; ++j) {
      const uint32_t e = c->row_ptr[v] + j;
      ell[c->sell_ptr[sl] + j * 64 + ln] = c->col[e] | (c->wt[c->rev[e]] << 16);
    }
  }
  // slices dealt widest first to the wave with the least width so far
  const uint32_t slots = std::max(1u, (n_slices + kMpWaves - 1) / kMpWaves);
  std::vector<uint32_t> order(n_slices), load(kMpWaves, 0), used(kMpWaves, 0);
  for (uint32_t i = 0; i < n_slices; ++i) order[i] = i;
  auto width = [&](uint32_t sl) { return (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / 64; };
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return width(a) > width(b); });
  std::vector<uint32_t> smap((size_t)kMpWaves * slots, kMpNoSlice);
  for (uint32_t sl : order) {
    uint32_t best = kMpWaves;
    for (uint32_t w = 0; w < kMpWaves; ++w)
      if (used[w] < slots && (best == kMpWaves || load[w] < load[best])) best = w;
    smap[(size_t)best * slots + used[best]++] = sl;
    load[best] += std::max(1u, width(sl));
  }
  // width classes (distinct slice widths, widest first; by log2 width when
  // there are more than kMpMaxCls) and, per wave, the first slot of each:
  // the phased first sweep's barriers
  {
    constexpr uint32_t kMpMaxCls = 8;
    std::vector<uint32_t> ws;
    for (uint32_t sl = 0; sl < n_slices; ++sl) ws.push_back(width(sl));
    std::sort(ws.begin(), ws.end(), std::greater<uint32_t>());
    ws.erase(std::unique(ws.begin(), ws.end()), ws.end());
    const bool log_cls = ws.size() > kMpMaxCls;
    auto key = [&](uint32_t w) { return log_cls ? 32u - (uint32_t)__builtin_clz(std::max(w, 1u)) : w; };
    std::vector<uint32_t> keys;
    for (uint32_t w : ws) keys.push_back(key(w));
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());  // descending
    if (keys.size() > kMpMaxCls) keys.resize(kMpMaxCls);  // the narrowest classes merge into the last
    const uint32_t n_cls = (uint32_t)keys.size();
    auto cls_of = [&](uint32_t sl) {
      const uint32_t k = key(width(sl));
      uint32_t c = 0;
      while (c + 1 < n_cls && keys[c] > k) ++c;
      return c;
    };
    std::vector<uint32_t> cl((size_t)kMpWaves * std::max(n_cls, 1u), 0);
    for (uint32_t w = 0; w < kMpWaves; ++w) {
      uint32_t k = 0;
      for (uint32_t c = 0; c < n_cls; ++c) {
        while (k < slots && smap[(size_t)w * slots + k] != kMpNoSlice && cls_of(smap[(size_t)w * slots + k]) < c) ++k;
        cl[(size_t)w * n_cls + c] = k;
      }
    }
    c->mp_ncls = n_cls;
    HIP_TRY(c, c->d_mp_cls.upload(cl.data(), cl.size(), c->stream));
  }
  // per slice: the other slices its nodes' out-edges reach (the mssp
  // kernel's slice-level dirt)
  std::vector<uint32_t> dep(n_slices + 1, 0);
  {
    std::vector<std::vector<uint32_t>> outs(n_slices);
    std::vector<uint32_t> mark(n_slices, kInf);
    for (uint32_t sl = 0; sl < n_slices; ++sl) {
      for (uint32_t u = sl * 64; u < std::min(N, sl * 64 + 64); ++u)
        for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e) {
          const uint32_t o = c->col[e] / 64;
          if (mark[o] != sl) mark[o] = sl, outs[sl].push_back(o);
        }
      std::sort(outs[sl].begin(), outs[sl].end());
    }
    for (uint32_t sl = 0; sl < n_slices; ++sl) dep[sl + 1] = dep[sl] + (uint32_t)outs[sl].size();
    for (uint32_t sl = 0; sl < n_slices; ++sl) dep[sl] += n_slices + 1;
    dep[n_slices] += n_slices + 1;
    for (auto& o : outs) dep.insert(dep.end(), o.begin(), o.end());
  }
  // overflow bound: with no drained node, d(s, v) <= max metric x hops(s, v)
  // <= max metric x 2 ecc(r) for any r of the component (BFS from one node
  // per component); otherwise only the trivial bound (N - 1) x max metric
  uint64_t bound = (uint64_t)(N ? N - 1 : 0) * c->max_metric;
  bool drained = false;
  for (uint32_t v = 0; v < N; ++v) drained |= c->ovl[v] != 0;
  if (!drained) {
    std::vector<uint32_t> hop(N, kInf), q;
    uint32_t ecc = 0;
    for (uint32_t r = 0; r < N; ++r) {
      if (hop[r] != kInf) continue;
      hop[r] = 0;
      q.assign(1, r);
      for (size_t h = 0; h < q.size(); ++h) {
        const uint32_t u = q[h];
        for (uint32_t e = c->row_ptr[u]; e < c->row_ptr[u + 1]; ++e)
          if (hop[c->col[e]] == kInf) {
            hop[c->col[e]] = hop[u] + 1;
            ecc = std::max(ecc, hop[u] + 1);
            q.push_back(c->col[e]);
          }
      }
    }
    bound = std::min<uint64_t>(bound, 2ull * ecc * c->max_metric);
  }
  // u8 labels when distances stay far below 255 on this graph: metrics below
  // 128 and the hop bound under 2 x 255 (rows that still reach the
  // saturation band are redone on u32 labels, as for u16).  SPF_MSSP_U8=0/1
  // forces (A/B, tests).
  {
    uint64_t hop_bound = bound;
    if (drained) hop_bound = ~0ull;
    c->mp_u8 = c->max_metric < 128 && hop_bound < 510;
    if (const char* e = std::getenv("SPF_MSSP_U8")) c->mp_u8 = e[0] == '1' && c->max_metric < 255;
  }
  c->mp_ovf_at = (c->mp_u8 ? 0xFFu : 0xFFFFu) - c->max_metric;
  c->mp_redo = bound >= c->mp_ovf_at;
  c->mp_slots = slots;
  HIP_TRY(c, c->d_mp_ell.upload(ell.data(), ell.size(), c->stream));
  HIP_TRY(c, c->d_mp_smap.upload(smap.data(), smap.size(), c->stream));
  HIP_TRY(c, c->d_mp_dep.upload(dep.data(), dep.size(), c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->mp_epoch = c->epoch;
  return SPF_OK;
}

// sources per workgroup: two labels per LDS word (u16) or four (u8); valid
// once mssp_prepare ran for the current graph epoch
uint32_t mssp_sources(const spf_ctx* c) { return (c->mp_u8 ? 4u : 2u) * mssp_words(c); }

spf_status mssp_set_lds_limits(spf_ctx* c) {
  const int lim = (int)(kMpMaxLds - kMpStaticLds);
  for (const void* f : {(const void*)mssp_kernel<1, false>, (const void*)mssp_kernel<2, false>,
                        (const void*)mssp_kernel<4, false>, (const void*)mssp_kernel<8, false>,
                        (const void*)mssp_kernel<1, true>, (const void*)mssp_kernel<2, true>,
                        (const void*)mssp_kernel<4, true>, (const void*)mssp_kernel<8, true>})
    HIP_TRY(c, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
  return SPF_OK;
}

// Distances of `rows` sources (device list rows_src) into D [rows][pitch]
// (+ the u8 copy Dn): mssp_kernel, then -- when an overflow is possible --
// sssp_kernel over the rows it listed in `redo` ([1 + rows] words).
spf_status launch_mssp(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, uint32_t* D,
                       uint8_t* Dn, uint32_t* redo, hipStream_t s, uint32_t* maxd) {
  const uint32_t sd = mssp_words(c);
  if (!sd) return fail(c, SPF_E_STATE, "mssp kernel does not apply to this graph");
  if (c->mp_epoch != c->epoch) return fail(c, SPF_E_STATE, "mssp tables stale: rebuild the plan");
  if (c->mp_redo) HIP_TRY(c, hipMemsetAsync(redo, 0, 4, s));
  if (!c->d_stamps.p && std::getenv("SPF_STAMPS")) {  // sweep counters (diagnostics)
    HIP_TRY(c, c->d_stamps.alloc(kStampWords));
    HIP_TRY(c, hipMemsetAsync(c->d_stamps.p, 0, (64 * 16 + 1) * 8, s));
  }
  const uint32_t S = mssp_sources(c);
  const dim3 g((rows + S - 1) / S), b(kMpThreads);
  const uint32_t N = c->N;
  uint32_t* rd = c->mp_redo ? redo : nullptr;
  const char* ae = std::getenv("SPF_MSSP_ALT");  // A/B: alternating sweep direction
  const uint32_t alt = ae ? (uint32_t)atoi(ae) : 0u;
  const char* ke = std::getenv("SPF_MSSP_SKIP");  // A/B: slice-level dirt (default on)
  const uint32_t* dep = ke && ke[0] == '0' ? nullptr : c->d_mp_dep.p;
  // class-phased first sweep (default; SPF_MSSP_PHASED=<phase word>: A/B, 0
  // off): fabric_rtt 5.24 -> 4.58 sweeps per workgroup, mssp 1.245 -> 1.131
  // ms (r05_ms2)
  const char* pe = std::getenv("SPF_MSSP_PHASED");
  const uint32_t phase = pe ? (uint32_t)strtoul(pe, nullptr, 0) : 1u;
#define MP_LAUNCH(SDV)                                                                            \
  if (c->mp_u8) {                                                                                 \
    MP_LAUNCH2(SDV, true);                                                                        \
  } else {                                                                                        \
    MP_LAUNCH2(SDV, false);                                                                       \
  }
#define MP_LAUNCH2(SDV, U8V)                                                                      \
  hipLaunchKernelGGL((mssp_kernel<SDV, U8V>), g, b, mp_lds(N, SDV), s, c->d_sell_ptr.p, c->d_mp_ell.p, \
                     c->d_mp_smap.p, c->mp_slots, c->d_row_ptr.p, c->d_col.p, c->d_wt.p,        \
                     c->d_ovl.p, rows_src, rows, N, c->pitch, D, Dn, c->mp_ovf_at, rd, alt, dep, c->d_stamps.p, \
                     maxd, c->d_mp_cls.p, c->mp_ncls, phase)
  switch (sd) {
    case 8: MP_LAUNCH(8); break;
    case 4: MP_LAUNCH(4); break;
    case 2: MP_LAUNCH(2); break;
    default: MP_LAUNCH(1); break;
  }
#undef MP_LAUNCH
#undef MP_LAUNCH2
  HIP_TRY(c, hipGetLastError());
  if (c->mp_redo)
    return launch_sssp(c, rows_src, rows, false, nullptr, D, s, nullptr, nullptr, Dn, redo);
  return SPF_OK;
}

}  // namespace spfi
