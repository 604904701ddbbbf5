// ============================================================================
//  msbfs_team.hip -- multi-source BFS (unit metrics / hop counts) for plans
//  with few sources: a batch of <= 64 sources is shared by a TEAM of G
//  workgroups on one XCD, each owning 1/G of the graph's 64-node slices.
//
//  Reference: LinkState::runSpf (openr/decision/LinkState.cpp:808-882) with
//  unit metrics; same result as msbfs_kernel (spf_engine.hip): per node a
//  64-bit mask (bit = source of the batch), a level = one pull sweep
//  new(v) = OR_{u in N(v)} F(u) & ~visited(v), drained nodes record but
//  expand only as their own source (:831-838).
//
//  Why teams: msbfs_kernel gives a batch one workgroup that sweeps every
//  column of the graph per level, so its time is per-workgroup fixed cost --
//  fine with 10k sources (256 batches fill the chip), but a rank of an 8-GPU
//  run holds ~1250 sources: 20-32 batches, 88 % of the CUs idle and the
//  same time per pass as the whole graph.  Here the batch's sweep is split
//  over G workgroups (G = 256 / next_pow2(batches)); the frontier masks F
//  live in global memory (the team's 2 x 8(N + 1) bytes stay in its XCD's
//  L2) and a level ends at a team barrier (agent-scope release -> arrival
//  counter -> poll -> acquire, MI355X_MICROARCH.md's workgroup hand-off).
//  Teams are persistent (one workgroup per CU, every member resident at
//  once; spins are bounded) and walk their batches; level counters run on
//  across batches, so flags and barriers need no reset between them.
// ============================================================================
#include "engine_internal.h"

using namespace spfi;

namespace {

constexpr int kTmThreads = 1024;
constexpr uint32_t kTmWaves = kTmThreads / 64;
constexpr uint32_t kTmBatch = 64;
constexpr uint32_t kTmNoSlice = 0x03FFFFFFu;  // an unused slot: its nodes lie past N
constexpr uint32_t kTmSpin = 1u << 26;        // ~seconds: never a silent hang
constexpr int kTmUnroll = 8;
constexpr uint32_t kTmBarPad = 32;            // words per team: counter line + 3 flag lines

// set when a team barrier gave up (spf_device_check reads it via msbfs_team_timed_out)
__device__ uint32_t g_team_timeout;

__device__ __forceinline__ uint32_t tm_or32(uint32_t x) {
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true);
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true);
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true);
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true);
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint32_t tm_max32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint64_t tm_or64(uint64_t x) {
  return ((uint64_t)tm_or32((uint32_t)(x >> 32)) << 32) | tm_or32((uint32_t)x);
}

struct TeamArgs {
  const uint32_t* sell_ptr;
  const uint32_t* sell_col;
  const uint32_t* tsmap;  // [G][kTmWaves][own] slice of (member, wave, slot)
  const uint8_t* ovl;
  const uint32_t* rows_src;
  uint32_t n_rows, bs, n_batches, N, pitch, npitch, G, teams_per_xcd;
  uint32_t* D;
  uint8_t* Dn;
  uint32_t* maxd;
  unsigned long long* F;  // [teams][2][N + 1]
  uint32_t* bar;          // [teams][kTmBarPad * 4], zero at launch
};

// team barrier: every member's stores drained and released at agent scope,
// one arrival per member on the team's counter, poll, acquire
__device__ __forceinline__ void team_barrier(uint32_t* cnt, uint32_t G) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t ticket = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = (ticket / G + 1) * G;
    uint32_t k = 0;
    for (; k < kTmSpin && __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++k)
      __builtin_amdgcn_s_sleep(1);
    if (k == kTmSpin) __hip_atomic_store(&g_team_timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

template <int OWN>
__global__ __launch_bounds__(kTmThreads) void msbfs_team_kernel(TeamArgs a) {
  __shared__ uint32_t src_l[kTmBatch];
  __shared__ uint32_t o_node[kTmBatch];
  __shared__ uint32_t o_cnt;
  __shared__ uint32_t any_l;

  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // block -> (XCD, team on it, member): blocks are dealt to the XCDs round
  // robin, so blockIdx % 8 is the XCD; members of a team share its L2
  const uint32_t xcd = blockIdx.x & 7u, j = blockIdx.x >> 3;
  const uint32_t G = a.G;
  const uint32_t member = j % G;
  const uint32_t team = xcd * a.teams_per_xcd + j / G;
  const uint32_t n_teams = 8 * a.teams_per_xcd;
  const uint32_t N = a.N;
  unsigned long long* F0 = a.F + (size_t)team * 2 * (N + 1);
  uint32_t* cnt = a.bar + (size_t)team * kTmBarPad * 4;
  uint32_t* flag = cnt + kTmBarPad;  // flag[L % 3] at flag + (L % 3) * kTmBarPad

  // owned slices (wave-uniform), their columns
  uint32_t sv[OWN], sb[OWN], sw[OWN];
  uint32_t drained = 0;
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    const uint32_t sl = a.tsmap[((size_t)member * kTmWaves + wv) * OWN + i];
    sv[i] = __builtin_amdgcn_readfirstlane(sl * 64u);
    const bool live = sv[i] < N;
    const uint32_t slice = live ? sl : 0u;
    const uint32_t b = live ? a.sell_ptr[slice] : 0u;
    const uint32_t e = live ? a.sell_ptr[slice + 1] : 0u;
    sb[i] = __builtin_amdgcn_readfirstlane(b);
    sw[i] = __builtin_amdgcn_readfirstlane((e - b) / 64u);
    const uint32_t v = sv[i] + lane;
    if (v < N && a.ovl[v]) drained |= 1u << i;
  }
  if (tid == 0) any_l = 0;
  if (member == 0 && tid == 0) {  // the padding target of both buffers stays 0
    F0[N] = 0ull;
    F0[2 * (N + 1) - 1] = 0ull;
  }

  uint32_t L = 0;  // running level counter of the team (flags, buffers)
  for (uint32_t batch = team; batch < a.n_batches; batch += n_teams) {
    const uint32_t row0 = batch * a.bs;
    const uint32_t nb = min(a.bs, a.n_rows - row0);
    const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
    if (tid == 0) o_cnt = 0;
    __syncthreads();
    if (tid < nb) {
      const uint32_t src = a.rows_src[row0 + tid];
      src_l[tid] = src;
      if (a.ovl[src]) o_node[atomicAdd(&o_cnt, 1u)] = src | (tid << 24);
    }
    __syncthreads();
    const uint32_t n_osrc = o_cnt;
    auto own_bits = [&](uint32_t v, uint64_t x) {
      uint64_t own = 0;
      for (uint32_t k = 0; k < n_osrc; ++k)
        if ((o_node[k] & 0xFFFFFFu) == v) own = 1ull << (o_node[k] >> 24);
      return x & own;
    };
    // level 0: a node's own source bits
    uint64_t vis[OWN];
    unsigned long long* Fc = F0 + (size_t)(L & 1u) * (N + 1);
#pragma unroll
    for (int i = 0; i < OWN; ++i) {
      const uint32_t v = sv[i] + lane;
      uint64_t m = 0;
      if (v < N)
        for (uint32_t s = 0; s < nb; ++s) m |= (src_l[s] == v ? 1ull : 0ull) << s;
      vis[i] = m;
      if (v < N) Fc[v] = m;  // a drained source expands as itself: m is its own bit
    }
    // ---- record a level: D[s][v] = lvl for every new (s, v) of slice i ----
    auto record = [&](int i, uint64_t x, uint32_t lvl) {
      if (__ballot(x != 0ull) == 0ull) return;
      const uint32_t nl = min(lvl, 254u);
      const uint64_t wm = tm_or64(x);
      const uint32_t mlo = __builtin_amdgcn_readfirstlane((uint32_t)wm);
      const uint32_t mhi = __builtin_amdgcn_readfirstlane((uint32_t)(wm >> 32));
      const uint32_t v = sv[i] + lane;
      const uint32_t nsrc = (uint32_t)__popcll(((uint64_t)mhi << 32) | mlo);
      const uint32_t maxpop = tm_max32((uint32_t)__popcll(x));
      if (maxpop * 4u < nsrc) {  // few per node: each lane walks its own sources
        uint64_t m = x;
        for (uint32_t it = 0; it < maxpop; ++it) {
          if (m) {
            const uint32_t s = __ffsll((unsigned long long)m) - 1;
            if (a.D) a.D[(size_t)(row0 + s) * a.pitch + v] = lvl;
            if (a.Dn) a.Dn[(size_t)(row0 + s) * a.npitch + v] = (uint8_t)nl;
            m &= m - 1;
          }
        }
        return;
      }
      for (uint64_t m = ((uint64_t)mhi << 32) | mlo; m; m &= m - 1) {  // a store per source
        const uint32_t s = __ffsll((unsigned long long)m) - 1;
        if ((x >> s) & 1ull) {
          if (a.D) a.D[(size_t)(row0 + s) * a.pitch + v] = lvl;
          if (a.Dn) a.Dn[(size_t)(row0 + s) * a.npitch + v] = (uint8_t)nl;
        }
      }
    };
#pragma unroll
    for (int i = 0; i < OWN; ++i) record(i, vis[i], 0);
    team_barrier(cnt, G);
    uint32_t depth = 0;
    for (uint32_t lvl = 1;; ++lvl) {
      ++L;
      const unsigned long long* Fp = F0 + (size_t)((L - 1) & 1u) * (N + 1);  // level lvl - 1
      unsigned long long* Fn = F0 + (size_t)(L & 1u) * (N + 1);
      if (member == 0 && tid == 0)
        __hip_atomic_store(flag + ((L + 1) % 3) * kTmBarPad, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint64_t any = 0;
#pragma unroll
      for (int i = 0; i < OWN; ++i) {
        const uint32_t v = sv[i] + lane;
        const bool need = v < N && vis[i] != all;
        uint64_t nx = 0;
        if (__ballot(need)) {
          const uint32_t* cp = a.sell_col + sb[i] + lane;
          const uint32_t w = sw[i];
          uint64_t acc = 0;
          uint32_t jj = 0;
          for (; jj + kTmUnroll <= w; jj += kTmUnroll) {
            uint32_t c[kTmUnroll];
#pragma unroll
            for (int u = 0; u < kTmUnroll; ++u) c[u] = cp[(jj + u) * 64];
#pragma unroll
            for (int u = 0; u < kTmUnroll; ++u) acc |= Fp[c[u]];
          }
          for (; jj < w; ++jj) acc |= Fp[cp[jj * 64]];
          if (need) {
            nx = acc & ~vis[i];
            vis[i] |= nx;
          }
        }
        if (v < N) Fn[v] = ((drained >> i) & 1u) ? own_bits(v, nx) : nx;
        any |= nx;
        record(i, nx, lvl);
      }
      if (__ballot(any != 0ull) && lane == 0) any_l = 1;
      __syncthreads();
      if (tid == 0) {
        if (any_l)
          __hip_atomic_store(flag + (L % 3) * kTmBarPad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        any_l = 0;  // set again only after the barrier below
      }
      team_barrier(cnt, G);
      if (!__hip_atomic_load(flag + (L % 3) * kTmBarPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        depth = lvl - 1;  // level lvl found nothing: the batch's deepest level
        break;
      }
    }
    if (a.maxd && member == 0 && tid == 0) atomicMax(a.maxd, depth);
    // ---- unreachable (s, v) pairs of the owned slices, row padding ----
    uint64_t miss = 0;
#pragma unroll
    for (int i = 0; i < OWN; ++i)
      if (sv[i] + lane < N) miss |= ~vis[i] & all;
    for (uint64_t m = tm_or64(miss); m; m &= m - 1) {
      const uint32_t s = __ffsll((unsigned long long)m) - 1;
#pragma unroll
      for (int i = 0; i < OWN; ++i) {
        const uint32_t v = sv[i] + lane;
        if (v < N && !((vis[i] >> s) & 1ull)) {
          if (a.D) a.D[(size_t)(row0 + s) * a.pitch + v] = kInf;
          if (a.Dn) a.Dn[(size_t)(row0 + s) * a.npitch + v] = 0xFF;
        }
      }
    }
    for (uint32_t s = 0; s < nb; ++s)  // padding past N, split over the members
      for (uint32_t v = N + member * kTmThreads + tid; v < a.npitch; v += G * kTmThreads) {
        if (a.D && v < a.pitch) a.D[(size_t)(row0 + s) * a.pitch + v] = kInf;
        if (a.Dn) a.Dn[(size_t)(row0 + s) * a.npitch + v] = 0xFF;
      }
  }
}

}  // namespace

namespace spfi {

// Team shape for a plan of `rows` unit-metric rows: G workgroups per batch
// (0: msbfs_kernel's one workgroup per batch is better -- enough batches to
// fill the chip), batch size bs, and per-(member, wave) owned slots.
// SPF_MSBFS_TEAM=0 disables, =G forces a team size (A/B, tests).
uint32_t msbfs_team_size(const spf_ctx* c, uint32_t rows) {
  if (c->n_cu % 8 || rows == 0) return 0;
  const char* e = std::getenv("SPF_MSBFS_TEAM");
  if (e && e[0] == '0') return 0;
  const uint32_t per_xcd = c->n_cu / 8;
  uint32_t G = 0;
  if (e) {
    G = (uint32_t)atoi(e);
  } else {
    const uint32_t batches = (rows + kTmBatch - 1) / kTmBatch;
    if (batches * 2 > c->n_cu) return 0;  // >= half the CUs busy anyway
    // the largest G whose teams still cover every batch in one round
    G = 1;
    while (G * 2 <= per_xcd && (c->n_cu / (G * 2)) >= batches) G *= 2;
  }
  if (G < 2 || G > per_xcd || per_xcd % G) return 0;
  const uint32_t n_slices = (c->N + 63) / 64;
  if ((n_slices + G * kTmWaves - 1) / (G * kTmWaves) > 16) return 0;  // OWN <= 16
  return G;
}

spf_status msbfs_team_prepare(spf_ctx* c, spf_plan* p, uint32_t G) {
  const uint32_t n_slices = (c->N + 63) / 64;
  const uint32_t need = (n_slices + G * kTmWaves - 1) / (G * kTmWaves);
  const uint32_t own = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : need <= 8 ? 8 : 16;
  // slices dealt widest first to the (member, wave) with the least width
  const uint32_t units = G * kTmWaves;
  std::vector<uint32_t> order(n_slices), load(units, 0), used(units, 0);
  for (uint32_t i = 0; i < n_slices; ++i) order[i] = i;
  auto width = [&](uint32_t sl) { return (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / 64; };
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return width(x) > width(y); });
  std::vector<uint32_t> tsmap((size_t)units * own, kTmNoSlice);
  for (uint32_t sl : order) {
    uint32_t best = units;
    for (uint32_t u = 0; u < units; ++u)
      if (used[u] < own && (best == units || load[u] < load[best])) best = u;
    tsmap[(size_t)best * own + used[best]++] = sl;
    load[best] += std::max(1u, width(sl));
  }
  const uint32_t per_xcd = c->n_cu / 8;
  const uint32_t teams = 8 * (per_xcd / G);
  const uint32_t rows = (uint32_t)p->closure.size();
  p->tm_G = G;
  p->tm_own = own;
  p->tm_teams = teams;
  p->tm_bs = std::min<uint32_t>(kTmBatch, (rows + teams - 1) / teams);
  HIP_TRY(c, p->d_tm_map.upload(tsmap.data(), tsmap.size(), c->stream));
  HIP_TRY(c, p->d_tm_F.alloc((size_t)teams * 2 * (c->N + 1) * 2));  // u64 as 2 words
  HIP_TRY(c, p->d_tm_bar.alloc((size_t)teams * kTmBarPad * 4));
  return SPF_OK;
}

spf_status launch_msbfs_team(spf_ctx* c, spf_plan* p, const uint32_t* rows_src, uint32_t rows,
                             uint32_t* D, uint8_t* Dn, uint32_t* maxd, hipStream_t s) {
  HIP_TRY(c, hipMemsetAsync(p->d_tm_bar.p, 0, 4ull * p->tm_teams * kTmBarPad * 4, s));
  TeamArgs a{c->d_sell_ptr.p, c->d_sell_col.p, p->d_tm_map.p, c->d_ovl.p, rows_src, rows,
             p->tm_bs, (rows + p->tm_bs - 1) / p->tm_bs, c->N, c->pitch, c->npitch, p->tm_G,
             (c->n_cu / 8) / p->tm_G, D, Dn, maxd,
             reinterpret_cast<unsigned long long*>(p->d_tm_F.p), p->d_tm_bar.p};
  const uint32_t blocks = p->tm_teams * p->tm_G;  // = n_cu: one persistent workgroup per CU
  void* args[] = {&a};
  const void* k = p->tm_own <= 1   ? (const void*)msbfs_team_kernel<1>
                  : p->tm_own <= 2 ? (const void*)msbfs_team_kernel<2>
                  : p->tm_own <= 4 ? (const void*)msbfs_team_kernel<4>
                  : p->tm_own <= 8 ? (const void*)msbfs_team_kernel<8>
                                   : (const void*)msbfs_team_kernel<16>;
  int fit = 0;
  HIP_TRY(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit, k, kTmThreads, 0));
  if (fit < 1 || (uint64_t)fit * c->n_cu < blocks)
    return fail(c, SPF_E_HIP, "msbfs_team_kernel: %u blocks not co-resident", blocks);
  HIP_TRY(c, hipLaunchKernel(k, dim3(blocks), dim3(kTmThreads), args, 0, s));
  return SPF_OK;
}

// reads and clears the team barriers' timeout flag (spf_device_check)
spf_status msbfs_team_timed_out(spf_ctx* c, bool* out) {
  uint32_t flag = 0;
  const uint32_t zero = 0;
  HIP_TRY(c, hipMemcpyFromSymbol(&flag, HIP_SYMBOL(g_team_timeout), sizeof flag, 0, hipMemcpyDeviceToHost));
  if (flag) HIP_TRY(c, hipMemcpyToSymbol(HIP_SYMBOL(g_team_timeout), &zero, sizeof zero, 0, hipMemcpyHostToDevice));
  *out = flag != 0;
  return SPF_OK;
}

}  // namespace spfi
