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
//  over G workgroups (the largest G whose 256 / G teams still hold every
//  source in one round of <= 64-source batches).
//
//  Per level, each member:
//    * sweeps its share of the column groups with the whole frontier in LDS
//      (Fl, 8 B per node): a member's slices' column groups are cut into 16
//      equal ranges (one per wave), so a fabric's 173-wide spine slices are
//      spread over several waves instead of setting the level's latency;
//      runs of one slice ORed into an LDS accumulator per slice;
//    * finalizes its slices (new = acc & ~visited, stores of the level's
//      distances), writes their next-frontier masks to the team's buffer in
//      global memory (stays in the XCD's L2);
//    * team barrier (agent-scope release -> arrival counter -> poll ->
//      acquire, MI355X_MICROARCH.md's workgroup hand-off);
//    * copies the whole next frontier from L2 into its LDS (80 KB at 10k
//      nodes, uint4 loads).
//  Level 0 needs no exchange (every member marks the sources itself).  A
//  slice whose nodes have every source is skipped by later sweeps, and a
//  level after which every slice is finished ends the batch without the
//  empty level.  Teams are persistent (one workgroup per CU, every member
//  resident at once; spins are bounded) and walk their batches; level
//  counters run on across batches, so flags and barriers need no reset.
// ============================================================================
#include "engine_internal.h"
#include "wave_ops.h"

#include <cstdio>

using namespace spfi;

namespace {

constexpr int kTmThreads = 1024;
constexpr uint32_t kTmWaves = kTmThreads / 64;
constexpr uint32_t kTmBatch = 64;
constexpr uint32_t kTmSpin = 1u << 26;        // ~seconds: never a silent hang
constexpr size_t kTmMaxLds = 160 * 1024;
constexpr int kTmPlanes = 4;                              // distance bit planes per owned node
constexpr uint32_t kTmWindow = (1u << kTmPlanes) - 1;     // levels per window; marker value
static_assert(kTmPlanes == (int)kTeamPlanes, "sdirect rows: the next-hop pass reads kTeamPlanes planes");
constexpr int kTmCopy = 10;                               // uint4 per thread of the frontier copy
constexpr uint32_t kTmRows = 16;                          // sources per flush tile (80 B each per node)
static_assert(kTmRows == 16 && kTmPlanes == 4, "first-window flush: two 4 x 8 plane transposes per tile");
// one flush-tile row of the first window: source r's code from the
// transposed nibbles (see the flush), u32 (kInf if unreached) and u8 (0xF)
__device__ __forceinline__ void flush_code(uint32_t* T32, uint8_t* T8, uint32_t lane, uint32_t r,
                                           uint32_t X0, uint32_t X1) {
  const uint32_t nbl = ((r >> 2) & 1u) | ((r & 1u) << 1) | (((r >> 1) & 1u) << 2);
  const uint32_t q = (((r & 8u) ? X1 : X0) >> (4 * nbl)) & 0xFu;
  T32[r * 64 + lane] = q == 0xFu ? kInf : q;  // first window: base == 0
  T8[r * 64 + lane] = (uint8_t)q;              // q <= kTmWindow - 1 = 14, or 0xF
}
constexpr uint32_t kTmBarPad = 32;            // words per team: counter line + 3 flag lines
constexpr uint32_t kSliceNodes = 64;          // nodes per sliced-ELL slice (= wave width)

struct TeamArgs {
  const uint32_t* sell_col;
  const uint32_t* fin;    // [G][kTmWaves][OWN] finalized slices: slice | slot << 16 (0xFFFF: none)
  const uint32_t* mptr;   // [G * kTmWaves + 1] column-stream ranges of (member, wave), multiples of 16
  const uint8_t* ovl;
  const uint32_t* rows_src;
  uint32_t n_rows, bs, n_batches, N, pitch, npitch, G, teams_per_xcd, n_acc, fwords, front_bytes;
  uint32_t col_bytes;  // sell_col incl. its trailing padding group
  uint32_t d_rows;     // closure rows < d_rows have u32 rows in D (the request's prefix)
  uint32_t* S;         // sdirect: bit-sliced rows (kTmPlanes planes per 32-node word) instead of Dn
  uint32_t s_stride;   // words per sliced row
  uint32_t* D;
  uint8_t* Dn;
  uint32_t* maxd;
  unsigned long long* F;  // [teams][2][fwords]: the levels' frontiers, exchanged through L2
  uint32_t* bar;          // [teams][kTmBarPad * 4]: arrivals, exits | 3 flag lines; zero at launch
  unsigned long long* stamps;  // diagnostics (SPF_STAMPS=<block>), usually null
  const uint32_t* need;        // [G][need_words]: the 64-node frontier slices a member's stream reads
  uint32_t need_words;
  uint32_t* fault;  // the context's barrier-timeout word (spf_device_check)
  const uint32_t* push_off;   // [n_batches + 1]: each batch's level-1 push list
  const uint32_t* push;       // target | source bit << 24 over the batch's sources' CSR rows
  const uint32_t* drained;  // the drained nodes (they keep no level-1 frontier bits)
  uint32_t n_drained;
  uint32_t dbg;     // diagnostics (SPF_TEAM_FLUSH_DBG): bit 0 no u32 row stores, bit 1 no plane
                    // stores, bit 2 no flush at all, bit 3 no row padding, bit 4 no maxd
                    // atomic (the rows are then invalid)
};

// Team hand-off of a level (MI355X_MICROARCH.md, inter-workgroup visibility,
// hand-off row 1 -- no L2 write-back, no L1 invalidate): every member's
// frontier words are stored write-through (sc1) and drained by each storing
// wave (vmcnt(0)), then ONE lane of the member adds its arrival to the
// level's word -- 1 + 256 * (found new nodes) + 65536 * (has unfinished
// slices) -- and polls it with sc1 loads until all G arrived; the frontier
// is read back with sc1 loads only.  Returns the level's word.
// Correctness does not depend on where the members run: this is row 1 of
// MI355X_MICROARCH.md's sc1 hand-off table (one lane per storing workgroup
// adds to an agent-scope counter after every wave's vmcnt(0) and a
// workgroup barrier; the consumer polls with sc1 loads and every load of the
// handed-off bytes is an sc1 load; the payload is stored sc1), which holds
// same-XCD and cross-XCD alike.  blockIdx % 8 groups members for L2
// locality (speed) only.  The launch is ordered after any other
// grid-resident launch of the process on the device (resident_order), so
// its one-workgroup-per-CU grid is not starved of CUs by another waiting
// grid; the spin stays bounded and reports through the context's fault word.
__device__ __forceinline__ uint32_t team_arrive(uint32_t* word, uint32_t G, uint32_t val,
                                                uint32_t* bcast, uint32_t* fault) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t w = 0, k = 0;
    for (; k < kTmSpin; ++k) {
      w = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((w & 0xFFu) >= G) break;
      __builtin_amdgcn_s_sleep(1);
    }
    // 2 = a team barrier: spf_device_check turns team plans off on the context
    if (k == kTmSpin) __hip_atomic_fetch_or(fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *bcast = w;
  }
  __syncthreads();
  return *bcast;
}

// 16-byte write-through (sc1) load: aux bit 4 = sc1 on gfx940+
__device__ __forceinline__ uint4 ld_sc1_16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
  return make_uint4(x.x, x.y, x.z, x.w);
}

// LDS: Fl[fwords] (the whole frontier of the previous level), Acc[n_acc][64]
// (column-stream ORs of the member's slices), the batch's sources.
// Distances stay in registers as kTmPlanes bit planes per owned node (bit s
// of plane b = bit b of d(s, v) - base) and are written once per window.
template <int OWN>
__global__ __launch_bounds__(kTmThreads) void msbfs_team_kernel(TeamArgs a,
                                                                const uint32_t* __restrict__ meta) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* Fl = reinterpret_cast<uint64_t*>(smem);  // [fwords]; the flush tiles reuse it
  uint64_t* Acc = reinterpret_cast<uint64_t*>(smem + a.front_bytes);
  uint32_t* src_l = reinterpret_cast<uint32_t*>(Acc + (size_t)a.n_acc * 64);
  uint32_t* any_l = src_l + kTmBatch;  // [0]: this member's level flags, [1]: broadcast word

  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // test hook (SPF_TEAM_FLUSH_DBG bit 32): report a team-barrier timeout
  if ((a.dbg & 32u) && blockIdx.x == 0 && tid == 0)
    __hip_atomic_fetch_or(a.fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // block -> (XCD, team on it, member): blocks are dealt to the XCDs round
  // robin, so blockIdx % 8 is the XCD; members of a team share its L2
  const uint32_t xcd = blockIdx.x & 7u, j = blockIdx.x >> 3;
  const uint32_t G = a.G;
  const uint32_t member = j % G;
  const uint32_t team = xcd * a.teams_per_xcd + j / G;
  const uint32_t n_teams = 8 * a.teams_per_xcd;
  const uint32_t N = a.N, fw = a.fwords;
  unsigned long long* F0 = a.F + (size_t)team * 2 * fw;
  const __amdgpu_buffer_rsrc_t frs =
      __builtin_amdgcn_make_buffer_rsrc(F0, 0, (int)(16u * fw), 0x00020000);
  uint32_t* cnt = a.bar + (size_t)team * kTmBarPad * 4;  // [0]: unused, [1]: exits
  uint32_t* lvw = cnt + kTmBarPad;  // level word of level L at lvw + (L % 3) * kTmBarPad
  const uint32_t mw = __builtin_amdgcn_readfirstlane(member * kTmWaves + wv);
  const uint32_t m_beg = __builtin_amdgcn_readfirstlane(a.mptr[mw]);
  const uint32_t n_chunks = __builtin_amdgcn_readfirstlane((a.mptr[mw + 1] - m_beg) / 16u);
  const uint32_t* ms = meta + m_beg;
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(a.sell_col), 0, (int)(a.col_bytes), 0x00020000);
  // diagnostics: lane 0 of every wave of block stamps[1024] logs s_memtime at
  // each phase boundary into stamps[wave * 64 + 1 ..], the count at [wave * 64]
  const bool stamp = a.stamps && blockIdx.x == (uint32_t)a.stamps[64 * 16] && lane == 0;
  // block timeline (with stamps on): s_memrealtime (100 MHz, chip-wide) at
  // the start and the end of every block, stamps[1025 + 2 b], [1026 + 2 b]
  if (a.stamps && tid == 0 && blockIdx.x < kStampBlocks)
    a.stamps[64 * 16 + 1 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  uint32_t n_stamp = 0;
#define TM_STAMP()                                                                      \
  do {                                                                                  \
    if (stamp && n_stamp < 63) a.stamps[wv * 64 + ++n_stamp] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  TM_STAMP();

  // finalized slices (wave-uniform): first node, Acc slot
  uint32_t sv[OWN], slot[OWN];
  uint32_t drained = 0;
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    const uint32_t f = a.fin[(size_t)mw * OWN + i];
    const bool live = (f & 0xFFFFu) != 0xFFFFu;
    sv[i] = __builtin_amdgcn_readfirstlane(live ? (f & 0xFFFFu) * 64u : 0x7FFFFFFFu);
    slot[i] = __builtin_amdgcn_readfirstlane(f >> 16);
    const uint32_t v = sv[i] + lane;
    if (v < N && a.ovl[v]) drained |= 1u << i;
  }
  // the frontier copy's 16-byte pieces (2 nodes each, piece t = tid + k *
  // kTmThreads) this member's sweep reads: a member of 8 reads ~1/4 of the
  // frontier's 64-node slices, the others stay stale in its LDS
  uint32_t cpm = 0;
#pragma unroll
  for (int k = 0; k < kTmCopy; ++k) {
    const uint32_t t = tid + k * kTmThreads, sl = t >> 5;
    if (t < fw / 2 && (sl >> 5) < a.need_words &&
        ((a.need[member * a.need_words + (sl >> 5)] >> (sl & 31)) & 1u))
      cpm |= 1u << k;
  }
  if (member == 0 && tid == 0) {  // the padding entries of both buffers stay 0
    for (uint32_t t = N; t < fw; ++t) {
      __hip_atomic_store(&F0[t], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&F0[fw + t], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  for (uint32_t t = tid; t < a.n_acc * 64; t += kTmThreads) Acc[t] = 0ull;

  // ---- one pass over this wave's column stream: 16 column loads per chunk,
  // the next chunk's loads in flight while this chunk's LDS reads run;
  // consecutive groups of one slice ORed in registers, flushed into the
  // slice's accumulator when the slot changes (the stream is slot-sorted) ----
  auto sweep = [&]() {
    uint64_t acc = 0;
    uint32_t cur = 0xFFFFFFFFu;
    constexpr int H = OWN >= 2 ? 4 : 8;  // columns per step, two steps in flight (OWN >= 2: 4 -- x4 / x8 members 3-4 % faster than 8)
    uint32_t ca[H], cb[H];
    // a step's column loads: stream words by scalar loads, group offset in
    // an SGPR, lane offset in a VGPR
    auto load = [&](uint32_t k, uint32_t (&c)[H]) {
#pragma unroll
      for (int u = 0; u < H; ++u) {
        const uint32_t g = __builtin_amdgcn_readfirstlane(ms[k * H + u]) & 0xFFFFFu;
        c[u] = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(lane * 4u), (int)(g * 256u), 0);
      }
    };
    // the step's stream words and frontier gathers all issued before the
    // first is used (a scalar load between them serialized one LDS round
    // trip per column: both count on lgkmcnt)
    auto proc = [&](uint32_t k, const uint32_t (&c)[H]) {
      uint32_t m[H];
      uint64_t f[H];
#pragma unroll
      for (int u = 0; u < H; ++u) m[u] = __builtin_amdgcn_readfirstlane(ms[k * H + u]);
#pragma unroll
      for (int u = 0; u < H; ++u) f[u] = Fl[c[u]];
#pragma unroll
      for (int u = 0; u < H; ++u) {
        const uint32_t sl = m[u] >> 20;
        if (sl != cur) {
          if (cur != 0xFFFFFFFFu && acc)
            atomicOr(reinterpret_cast<unsigned long long*>(&Acc[cur * 64 + lane]), acc);
          cur = sl;
          acc = 0;
        }
        acc |= f[u];
      }
    };
    const uint32_t n_steps = n_chunks * (16 / H);
    if (n_steps == 0) return;
    // loads unconditional (the stream table is padded with two chunks of the
    // all-padding group; past a wave's range they read the next wave's
    // groups, never processed): a load under a branch made the join's wait
    // count drain the next step's loads before every step's gathers
    load(0, ca);
    for (uint32_t k = 0; k < n_steps; k += 2) {
      load(k + 1, cb);
      proc(k, ca);
      load(k + 2, ca);
      if (k + 1 < n_steps) proc(k + 1, cb);
    }
    if (acc) atomicOr(reinterpret_cast<unsigned long long*>(&Acc[cur * 64 + lane]), acc);
  };

  uint32_t L = 0;  // running level counter of the team (flags, buffers)
  TM_STAMP();  // prologue done
  for (uint32_t batch = team; batch < a.n_batches; batch += n_teams) {
    const uint32_t row0 = batch * a.bs;
    const uint32_t nb = min(a.bs, a.n_rows - row0);
    const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
    for (uint32_t t = tid; t < fw / 2; t += kTmThreads)
      reinterpret_cast<uint4*>(Fl)[t] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // level 0, computed by every member alone: the sources' own bits (a
    // drained source expands as itself)
    if (tid < nb) {
      const uint32_t src = a.rows_src[row0 + tid];
      src_l[tid] = src;
      atomicOr(reinterpret_cast<unsigned long long*>(&Fl[src]), 1ull << tid);
    }
    __syncthreads();
    uint64_t vis[OWN], P[OWN][kTmPlanes];
#pragma unroll
    for (int i = 0; i < OWN; ++i) {
      const uint32_t v = sv[i] + lane;
      vis[i] = v < N ? Fl[v] : 0ull;
#pragma unroll
      for (int b = 0; b < kTmPlanes; ++b) P[i][b] = 0ull;
    }
    __syncthreads();  // the self marks are read
    if (tid < nb) Fl[src_l[tid]] = 0ull;
    __syncthreads();
    // ---- level 1 by push, by every member for the whole graph (no
    // exchange): each source's bit ORed into its neighbours' entries, the
    // batch's edges dealt over the workgroup, their loads independent.
    // Links are up in both directions or neither, so the CSR out-neighbours
    // are the in-neighbours a pull would read.  The first pull sweep, its
    // hand-off and frontier copy are gone (msbfs_kernel pushes level 1 too) ----
    // The batch's push list (target | source bit << 24, built at plan time
    // from the closure's CSR rows) dealt over the workgroup, four entries
    // per thread in flight before their LDS ORs.  (A thread per flat edge
    // finding its source by binary search cost ~10 us on spine batches,
    // a wave per source ~6, r05_t3 / r05_t4 stamps.)
    TM_STAMP();  // level 0 done
    const uint32_t p0 = a.push_off[batch], p1 = a.push_off[batch + 1];
    const uint32_t n_e = p1 - p0;
    for (uint32_t t = p0 + tid; t < p1; t += 4 * kTmThreads) {
      uint32_t x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = t + q * kTmThreads < p1 ? a.push[t + q * kTmThreads] : ~0u;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (x[q] != ~0u)
          atomicOr(reinterpret_cast<unsigned long long*>(&Fl[x[q] & 0xFFFFFFu]), 1ull << (x[q] >> 24));
    }
    __syncthreads();
    // level 1 of the owned slices (drained nodes included: recorded, not expanded)
#pragma unroll
    for (int i = 0; i < OWN; ++i) {
      const uint32_t v = sv[i] + lane;
      const uint64_t nx = v < N && sv[i] < N ? Fl[v] & ~vis[i] : 0ull;
      vis[i] |= nx;
      P[i][0] |= nx;  // relative level 1: plane 0
    }
    TM_STAMP();  // push + level-1 finalize done
    if (a.n_drained) {  // a drained node keeps no level-1 frontier bits
      __syncthreads();  // every owned read of the pushed entries is done
      for (uint32_t t = tid; t < a.n_drained; t += kTmThreads) Fl[a.drained[t]] = 0ull;
    }
    __syncthreads();
    // ---- write the window's distances: every (s, v) of the owned slices
    // in the first window (unreached = kInf), later only those found in it
    // (entries of earlier windows carry the marker kTmWindow in the planes) ----
    uint32_t base = 0;
    // the first window's flush covers every (s, v) and goes through a
    // per-wave LDS tile (the frontier's space, free by then): d of kTmRows
    // sources x 64 nodes, read back as 16-byte row pieces -- one dwordx4
    // store per 4 u32 rows and per 16 u8 rows instead of a dword and a byte
    // store per row (the store issue rate bounded the per-row form)
    auto flush = [&]() {
      if (a.dbg & 4u) return;
      if (base == 0) {
        uint32_t* T32 = reinterpret_cast<uint32_t*>(smem) + (size_t)wv * kTmRows * 80;
        uint8_t* T8 = reinterpret_cast<uint8_t*>(T32 + kTmRows * 64);
#pragma unroll
        for (int i = 0; i < OWN; ++i) {
          if (sv[i] >= N) continue;  // wave-uniform
          const uint32_t v = sv[i] + lane;
          for (uint32_t g0 = 0; g0 < nb; g0 += kTmRows) {
            const uint32_t gn = __builtin_amdgcn_readfirstlane(min(kTmRows, nb - g0));
            // the group's codes as nibbles, by a 4 x 8 bit-matrix transpose per
            // half: W = byte h of the four planes (bit 8b + r), two delta swaps
            // (index bits 0 <-> 3, 1 <-> 4) put plane b of source 8h + r at bit
            // 4 nbl(r) + b, nbl(r) = r2 + 2 r0 + 4 r1; a row then costs one
            // constant bit-field extract (the per-row gather of four plane bits
            // made the flush VALU-bound).  Unreached entries: all planes set
            // (code 0xF; the planes hold no bit of an unreached node)
            uint32_t X0, X1;
            {
              auto dswap = [](uint32_t x, uint32_t m, int d) {
                const uint32_t t = ((x >> d) ^ x) & m;
                return x ^ t ^ (t << d);
              };
              const uint32_t un = v < N ? ~(uint32_t)(vis[i] >> g0) : ~0u;
              uint32_t pw[kTmPlanes];
#pragma unroll
              for (int b = 0; b < kTmPlanes; ++b) pw[b] = (uint32_t)(P[i][b] >> g0) | un;
              auto half = [&](int h) {
                const uint32_t w = ((pw[0] >> (8 * h)) & 0xFFu) | (((pw[1] >> (8 * h)) & 0xFFu) << 8) |
                                   (((pw[2] >> (8 * h)) & 0xFFu) << 16) | (((pw[3] >> (8 * h)) & 0xFFu) << 24);
                return dswap(dswap(w, 0x00AA00AAu, 7), 0x0000CCCCu, 14);
              };
              X0 = half(0);
              X1 = half(1);
            }
            if (gn == kTmRows) {
#pragma unroll
              for (uint32_t r = 0; r < kTmRows; ++r) flush_code(T32, T8, lane, r, X0, X1);
            } else {
              for (uint32_t r = 0; r < gn; ++r) flush_code(T32, T8, lane, r, X0, X1);
            }
            if (a.D && !(a.dbg & 1u))
              for (uint32_t r4 = 0; r4 < gn; r4 += 4) {
                const uint32_t r = r4 + (lane >> 4);
                if (r < gn && row0 + g0 + r < a.d_rows) {
                  // streaming (nt) store: the u32 rows are outputs, never re-read here
                  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                  const v4u x = *reinterpret_cast<const v4u*>(T32 + r * 64 + (lane & 15) * 4);
                  __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(a.D + (size_t)(row0 + g0 + r) * a.pitch +
                                                                       sv[i] + (lane & 15) * 4));
                }
              }
            if (a.S && !(a.dbg & 2u)) {
              // the sliced rows (ecmp_sliced_kernel's layout with P =
              // kTmPlanes): word w of row r holds plane b at w * P + b, bit t
              // = node 32w + t; code all-ones = unreachable (tile byte 0x0F; nodes
              // past N too).  From the byte tile: lane (row r = lane / 4,
              // quarter q = lane % 4) turns its 16 bytes into a 16-bit piece
              // of each plane (slice_rows_kernel's multiply gather), lanes
              // q and q ^ 1 join their pieces into the word (DPP quad swap),
              // even quarters store their word's P planes as one dwordx4
              const uint32_t r = lane >> 2;
              const uint4 x = *reinterpret_cast<const uint4*>(T8 + (r < gn ? r : 0) * 64 + (lane & 3) * 16);
              const uint32_t dw[4] = {x.x, x.y, x.z, x.w};
              uint32_t wd[kTmPlanes];
#pragma unroll
              for (int b = 0; b < kTmPlanes; ++b) {
                uint32_t h = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  h |= ((((dw[q] >> b) & 0x01010101u) * 0x01020408u) >> 24) << (4 * q);
                const uint32_t o = (uint32_t)__builtin_amdgcn_mov_dpp((int)h, 0xB1, 0xF, 0xF, false);  // quad_perm(1,0,3,2)
                wd[b] = h | (o << 16);  // even quarter: its own piece low, the odd neighbour's high
              }
              if (r < gn && (lane & 1) == 0) {
                uint4* o = reinterpret_cast<uint4*>(a.S + (size_t)(row0 + g0 + r) * a.s_stride +
                                                    (sv[i] / 32u + ((lane >> 1) & 1)) * kTmPlanes);
                *o = make_uint4(wd[0], wd[1], wd[2], wd[3]);
              }
            }
            if (a.Dn) {
              const uint32_t r = lane >> 2;
              if (r < gn) {
                uint4 x = *reinterpret_cast<const uint4*>(T8 + r * 64 + (lane & 3) * 16);
                auto unreached = [](uint32_t w) {  // byte 0x0F (tile) -> 0xFF (u8 rows)
                  const uint32_t m = w & (w >> 1) & (w >> 2) & (w >> 3) & 0x01010101u;
                  return w | ((m << 8) - (m << 4));
                };
                x = make_uint4(unreached(x.x), unreached(x.y), unreached(x.z), unreached(x.w));
                *reinterpret_cast<uint4*>(a.Dn + (size_t)(row0 + g0 + r) * a.npitch + sv[i] +
                                          (lane & 3) * 16) = x;
              }
            }
          }
        }
        return;
      }
      // later windows (searches deeper than the planes): the entries found
      // in the window, one store per lane
      for (uint32_t s = 0; s < nb; ++s) {
        uint32_t* drow = a.D && row0 + s < a.d_rows ? a.D + (size_t)(row0 + s) * a.pitch : nullptr;
        uint8_t* nrow = a.Dn ? a.Dn + (size_t)(row0 + s) * a.npitch : nullptr;
#pragma unroll
        for (int i = 0; i < OWN; ++i) {
          if (sv[i] >= N) continue;  // wave-uniform
          const uint32_t v = sv[i] + lane;
          uint32_t q = 0;
#pragma unroll
          for (int b = 0; b < kTmPlanes; ++b) q |= (uint32_t)((P[i][b] >> s) & 1ull) << b;
          const bool seen = v < N && ((vis[i] >> s) & 1ull);
          if (seen && q != kTmWindow) {
            if (drow) drow[v] = base + q;
            if (nrow) nrow[v] = (uint8_t)min(base + q, 254u);
          }
        }
      }
    };
    uint32_t depth = n_e ? 1u : 0u;
    for (uint32_t lvl = 2; n_e; ++lvl) {
      ++L;
      unsigned long long* Fn = F0 + (size_t)(L & 1u) * fw;
      if (member == 0 && tid == 0)  // the word of level L + 1 (its last readers passed level L - 1)
        __hip_atomic_store(lvw + ((L + 1) % 3) * kTmBarPad, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sweep();
      TM_STAMP();
      __syncthreads();
      TM_STAMP();
      // ---- finalize the owned slices: new bits, planes, next frontier
      // (write-through: the hand-off's payload) ----
      const uint32_t rel = lvl - base;  // 1 .. kTmWindow - 1
      uint64_t any = 0;
      bool open = false;
#pragma unroll
      for (int i = 0; i < OWN; ++i) {
        const uint32_t v = sv[i] + lane;
        if (sv[i] >= N) continue;  // wave-uniform
        const uint64_t x = Acc[slot[i] * 64 + lane];
        Acc[slot[i] * 64 + lane] = 0ull;
        const uint64_t nx = v < N ? x & ~vis[i] : 0ull;
        vis[i] |= nx;
#pragma unroll
        for (int b = 0; b < kTmPlanes; ++b)
          if ((rel >> b) & 1u) P[i][b] |= nx;
        if (v < N)  // drained: expands as its own source only (level 0)
          __hip_atomic_store(&Fn[v], ((drained >> i) & 1u) ? 0ull : nx, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        any |= nx;
        if (__ballot(v < N && vis[i] != all)) open = true;
      }
      if (__ballot(any != 0ull) && lane == 0) atomicOr(any_l, 1u);
      if (open && lane == 0) atomicOr(any_l, 2u);
      __syncthreads();
      const uint32_t mine = *any_l;
      TM_STAMP();
      const uint32_t w = team_arrive(lvw + (L % 3) * kTmBarPad, G,
                                     1u + ((mine & 1u) << 8) + ((mine & 2u) << 15), any_l + 1,
                                     a.fault);
      if (tid == 0) *any_l = 0;  // read by every thread before team_arrive's second barrier
      TM_STAMP();
      if (((w >> 8) & 0xFFu) == 0) {
        depth = lvl - 1;  // level lvl found nothing: the batch's deepest level
        break;
      }
      if (((w >> 16) & 0xFFu) == 0) {
        depth = lvl;  // every node has every source: level lvl is the last
        break;
      }
      if (rel == kTmWindow - 1) {  // window full: write it, mark its entries, next window
        flush();
#pragma unroll
        for (int i = 0; i < OWN; ++i)
#pragma unroll
          for (int b = 0; b < kTmPlanes; ++b) P[i][b] |= vis[i];
        base += kTmWindow;
        __syncthreads();  // the flush's LDS tiles are read before the copy below
      }
      // ---- the next level's frontier into LDS: sc1 loads (L2-served, no
      // invalidate needed), every load issued before the stores ----
      {
        const uint32_t fo = (L & 1u) * fw * 8u;
        uint4* dst4 = reinterpret_cast<uint4*>(Fl);
#pragma unroll
        for (int h = 0; h < kTmCopy; h += kTmCopy / 2) {  // two halves: registers
          uint4 t4[kTmCopy / 2];
#pragma unroll
          for (int q = 0; q < kTmCopy / 2; ++q) {
            const uint32_t t = tid + (h + q) * kTmThreads;
            if ((cpm >> (h + q)) & 1u) t4[q] = ld_sc1_16(frs, fo + 16u * t);
          }
#pragma unroll
          for (int q = 0; q < kTmCopy / 2; ++q) {
            const uint32_t t = tid + (h + q) * kTmThreads;
            if ((cpm >> (h + q)) & 1u) dst4[t] = t4[q];
          }
        }
      }
      __syncthreads();
      TM_STAMP();
    }
    __syncthreads();  // every wave past its last frontier read: the tiles may overwrite Fl
    flush();
    if (a.maxd && member == 0 && tid == 0 && !(a.dbg & 16u)) atomicMax(a.maxd, depth);
    // row padding: the entries past the slices' end (the flush covered every
    // slice, nodes past N included) -- one flat (row, entry) index dealt to
    // every thread of every member.  A loop per row, as before, cost ~9 us per
    // batch in loop overhead at 57 rows (r04_g5 stamps, SPF_TEAM_FLUSH_DBG=8).
    if (!(a.dbg & 8u)) {
      const uint32_t v0 = (N + kSliceNodes - 1u) / kSliceNodes * kSliceNodes;
      const uint32_t pw = a.npitch - v0, tot = nb * pw;
      for (uint32_t t = member * kTmThreads + tid; t < tot; t += G * kTmThreads) {
        const uint32_t s = t / pw, v = v0 + t % pw;
        if (a.D && v < a.pitch && row0 + s < a.d_rows)
          __builtin_nontemporal_store(kInf, &a.D[(size_t)(row0 + s) * a.pitch + v]);
        if (a.Dn) a.Dn[(size_t)(row0 + s) * a.npitch + v] = 0xFF;
      }
    }
    __syncthreads();  // Fl, src_l are reset by the next batch
    TM_STAMP();
  }
  if (stamp) a.stamps[wv * 64] = n_stamp;
  if (a.stamps && tid == 0 && blockIdx.x < kStampBlocks)
    a.stamps[64 * 16 + 2 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#undef TM_STAMP
  // the team's last member out zeroes its barrier words for the next launch
  // (no memset per execute; every member passes here, timed-out ones too)
  __syncthreads();
  if (tid == 0) {
    if (__hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
      for (uint32_t k = 0; k < 3; ++k)
        __hip_atomic_store(lvw + k * kTmBarPad, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

namespace spfi {

// Team shape for a plan of `rows` unit-metric rows: G workgroups per batch
// (0: msbfs_kernel's one workgroup per batch is better -- enough batches to
// fill the chip).  SPF_MSBFS_TEAM=0 disables, =G forces a team size (A/B, tests).
static size_t team_lds(uint32_t fwords, uint32_t n_acc) {
  const size_t front = std::max<size_t>(8ull * fwords, (size_t)kTmWaves * kTmRows * 80 * 4);
  return front + 8ull * 64 * n_acc + 4ull * (kTmBatch + 2) + 16;
}

static const void* team_kernel(uint32_t own) {
  return own <= 1 ? (const void*)msbfs_team_kernel<1>
         : own <= 2 ? (const void*)msbfs_team_kernel<2>
                    : (const void*)msbfs_team_kernel<4>;
}

static uint32_t team_fwords(uint32_t N) { return (N + 2) & ~1u; }  // >= N + 1, even (uint4 copies)

uint32_t msbfs_team_size(const spf_ctx* c, uint32_t rows) {
  if (c->n_cu % 8 || rows == 0) return 0;
  const char* e = std::getenv("SPF_MSBFS_TEAM");
  if (e && e[0] == '0') return 0;
  const uint32_t per_xcd = c->n_cu / 8;
  const uint32_t n_slices = (c->N + 63) / 64;
  if (n_slices >= 0xFFFFu) return 0;
  auto valid = [&](uint32_t G) {
    if (G < 2 || G > per_xcd || per_xcd % G) return false;
    // LDS: the frontier plus the slice accumulators of the largest member;
    // registers: OWN <= 4 finalized slices per wave
    const uint32_t per_member = (n_slices + G - 1) / G + 2;
    return team_lds(team_fwords(c->N), per_member) <= kTmMaxLds &&
           (per_member + kTmWaves - 1) / kTmWaves <= 4;
  };
  if (e) {
    const uint32_t G = (uint32_t)atoi(e);
    return valid(G) ? G : 0;
  }
  // per-level cost model (us), fitted to fabric_full stamps and kernel
  // times (r03_v11..v14): msbfs_kernel sweeps every column group with one
  // workgroup (16 waves, ~6.5 groups per us per wave, +20 % for its
  // per-level stores); a team of G sweeps 1/G of them (~4 groups per us per
  // wave: column loads, LDS gathers and the accumulator ORs) plus ~5 us per
  // level (write-through hand-off, arrival word, frontier copy) and takes
  // ceil(batches / teams) rounds.  SPF_TEAM_LEVEL_US tunes the fixed part.
  const double groups = (double)(c->sell_ptr.back() / 64);
  const char* lu = std::getenv("SPF_TEAM_LEVEL_US");
  const double level_us = lu ? atof(lu) : 5.0;
  const double single = groups / kTmWaves / 6.5 * 1.2;
  const uint64_t batches = (rows + kTmBatch - 1) / kTmBatch;
  uint32_t best = 0;
  double best_cost = single;
  for (uint32_t G = 2; G <= per_xcd; G *= 2) {
    if (!valid(G)) continue;
    const uint64_t teams = c->n_cu / G;
    const double rounds = (double)((batches + teams - 1) / teams);
    const double cost = rounds * (groups / (kTmWaves * G) / 4.0 + level_us);
    if (cost < best_cost) best_cost = cost, best = G;
  }
  return best;
}

spf_status msbfs_team_prepare(spf_ctx* c, spf_plan* p, uint32_t G) {
  const uint32_t n_slices = (c->N + 63) / 64;
  auto width = [&](uint32_t sl) { return (c->sell_ptr[sl + 1] - c->sell_ptr[sl]) / 64; };
  const char* ne = std::getenv("SPF_TEAM_FULLCOPY");  // A/B: copy the whole frontier
  const bool full_copy = ne && ne[0] == '1';
  spf_ctx::TeamTables& T = c->tm_tab;
  // the graph-derived tables: computed once per sliced-ELL state and team
  // size (a plan re-derived after an overload or metric patch, or a new
  // single-source plan per query, reuses them -- the need pass alone walks
  // every column of the graph)
  if (T.ver != c->sell_ver || T.G != G || T.full_copy != full_copy) {
    T.ver = ~0ull;
    // slices to members, widest first to the least-loaded member (column
    // groups + a slice's finalize cost)
    std::vector<uint32_t> order(n_slices);
    for (uint32_t i = 0; i < n_slices; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return width(x) > width(y); });
    std::vector<std::vector<uint32_t>> mem(G);
    std::vector<uint64_t> load(G, 0);
    for (uint32_t sl : order) {
      uint32_t best = 0;
      for (uint32_t m = 1; m < G; ++m)
        if (load[m] < load[best] || (load[m] == load[best] && mem[m].size() < mem[best].size())) best = m;
      mem[best].push_back(sl);
      load[best] += width(sl) + 2;
    }
    uint32_t n_acc = 1;
    for (auto& v : mem) n_acc = std::max<uint32_t>(n_acc, (uint32_t)v.size());
    const uint32_t need = (n_acc + kTmWaves - 1) / kTmWaves;
    const uint32_t own = need <= 1 ? 1 : need <= 2 ? 2 : 4;
    if (need > 4 || team_lds(team_fwords(c->N), n_acc) > kTmMaxLds)
      return fail(c, SPF_E_INVALID, "msbfs_team: %u slices per member do not fit", n_acc);
    // per member: finalize slots dealt round robin to the waves; the member's
    // column groups (its slices' in order) cut into kTmWaves equal ranges, each
    // range a stream of {group | slot << 20}, padded to whole chunks of 16 with
    // the all-padding group after the last slice (sell_col's tail)
    const uint32_t units = G * kTmWaves;
    const uint32_t dummy = c->sell_ptr.back() / 64;
    if (dummy >= (1u << 20) || n_acc >= (1u << 12))
      return fail(c, SPF_E_INVALID, "msbfs_team: column groups exceed the stream encoding");
    std::vector<uint32_t>& fin = T.fin;
    std::vector<uint32_t>& mptr = T.mptr;
    std::vector<uint32_t>& meta = T.meta;
    fin.assign((size_t)units * own, 0xFFFFu);
    mptr.assign(units + 1, 0);
    meta.clear();
    for (uint32_t m = 0; m < G; ++m) {
      const auto& S = mem[m];
      for (uint32_t k = 0; k < S.size(); ++k)
        fin[((size_t)m * kTmWaves + k % kTmWaves) * own + k / kTmWaves] = S[k] | (k << 16);
      std::vector<uint32_t> all;  // the member's stream
      for (uint32_t k = 0; k < S.size(); ++k)
        for (uint32_t g = 0; g < width(S[k]); ++g) all.push_back((c->sell_ptr[S[k]] / 64 + g) | (k << 20));
      const uint64_t Tn = all.size();
      for (uint32_t w = 0; w < kTmWaves; ++w) {
        mptr[m * kTmWaves + w] = (uint32_t)meta.size();
        const uint64_t b = Tn * w / kTmWaves, e = Tn * (w + 1) / kTmWaves;
        for (uint64_t t = b; t < e; ++t) meta.push_back(all[t]);
        if (e > b)
          while (meta.size() % 16) meta.push_back(dummy | (all[e - 1] & 0xFFF00000u));
      }
    }
    mptr[units] = (uint32_t)meta.size();
    // per member: the 64-node slices its stream's columns read (frontier copy)
    const uint32_t fslices = (team_fwords(c->N) + 63) / 64;
    const uint32_t nw = (fslices + 31) / 32;
    T.need.assign((size_t)G * nw, full_copy ? ~0u : 0u);
    if (!full_copy)
      for (uint32_t m = 0; m < G; ++m)
        for (uint32_t sl : mem[m])
          for (uint32_t e = c->sell_ptr[sl]; e < c->sell_ptr[sl + 1]; ++e) {
            const uint32_t x = c->sell_col[e] / 64;
            T.need[(size_t)m * nw + x / 32] |= 1u << (x % 32);
          }
    T.need_words = nw;
    T.n_acc = n_acc;
    T.own = own;
    T.G = G;
    T.full_copy = full_copy;
    T.ver = c->sell_ver;
  }
  const uint32_t n_acc = T.n_acc, own = T.own;
  const std::vector<uint32_t>& fin = T.fin;
  const std::vector<uint32_t>& mptr = T.mptr;
  const std::vector<uint32_t>& meta = T.meta;
  const uint32_t dummy = c->sell_ptr.back() / 64;
  const uint32_t per_xcd = c->n_cu / 8;
  const uint32_t teams = 8 * (per_xcd / G);
  const uint32_t rows = (uint32_t)p->closure.size();
  const uint32_t fw = team_fwords(c->N);
  {  // every member must be resident at once (one workgroup per CU): else
     // the plan keeps msbfs_kernel (tm_G stays 0; spf_plan_kernels tells)
    const void* k = team_kernel(own);
    HIP_TRY(c, hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTmMaxLds));
    // one block per CU needs: the block's registers (compiled for 1024
    // threads: maxThreadsPerBlock), its LDS within the CU's 160 KiB, and
    // one block per CU in the grid (teams * G == n_cu).  (The occupancy API
    // answered 0 for this kernel on some boxes and 1 on others with the same
    // image and the same arguments; these static facts decide instead.)
    hipFuncAttributes fa{};
    HIP_TRY(c, hipFuncGetAttributes(&fa, k));
    const size_t lds = team_lds(fw, n_acc) + fa.sharedSizeBytes;
    if (fa.maxThreadsPerBlock < (int)kTmThreads || lds > kTmMaxLds || (uint64_t)teams * G > c->n_cu) {
      if (std::getenv("SPF_TEAM_DEBUG"))
        std::fprintf(stderr, "msbfs_team: <%u> not co-resident (max threads %d, %zu B LDS, G %u): msbfs_kernel\n",
                     own, fa.maxThreadsPerBlock, lds, G);
      p->tm_G = 0;
      return SPF_OK;
    }
    if (std::getenv("SPF_TEAM_DEBUG")) {
      int fit = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit, k, kTmThreads, team_lds(fw, n_acc));
      std::fprintf(stderr, "msbfs_team: <%u> G %u, %zu B LDS, occupancy API %d per CU\n", own, G, lds, fit);
    }
  }
  p->tm_G = G;
  p->tm_own = own;
  p->tm_teams = teams;
  p->tm_nacc = n_acc;
  {  // equal batches over whole rounds of the teams
    const uint32_t rounds = (rows + kTmBatch * teams - 1) / (kTmBatch * teams);
    p->tm_bs = std::min<uint32_t>(kTmBatch, (rows + teams * rounds - 1) / (teams * rounds));
  }
  std::vector<uint32_t> tab;  // fin | mptr | (16-entry aligned) meta, one upload
  tab.insert(tab.end(), fin.begin(), fin.end());
  p->tm_rptr_at = (uint32_t)tab.size();
  tab.insert(tab.end(), mptr.begin(), mptr.end());
  while (tab.size() % 16) tab.push_back(0);
  p->tm_runs_at = (uint32_t)tab.size();
  tab.insert(tab.end(), meta.begin(), meta.end());
  tab.insert(tab.end(), 32, dummy);  // the sweep's loads run up to two chunks past a range
  {  // per member: the frontier slices its stream reads (cached above)
    p->tm_need_at = (uint32_t)tab.size();
    p->tm_need_words = T.need_words;
    tab.insert(tab.end(), T.need.begin(), T.need.end());
  }
  // the drained nodes (level 1 is pushed into every node's entry; these
  // keep none of it as frontier)
  p->tm_drained_at = (uint32_t)tab.size();
  for (uint32_t v = 0; v < c->N; ++v)
    if (c->ovl[v]) tab.push_back(v);
  p->tm_n_drained = (uint32_t)tab.size() - p->tm_drained_at;
  tab.push_back(0);  // never empty past the offset
  {  // per batch: its sources' CSR rows as (target | bit << 24), the level-1 push
    const uint32_t nbat = (rows + p->tm_bs - 1) / p->tm_bs;
    p->tm_push_n = nbat + 1;
    p->tm_push_at = (uint32_t)tab.size();
    tab.resize(tab.size() + nbat + 1, 0u);
    std::vector<uint32_t> lst;
    for (uint32_t k = 0; k < nbat; ++k) {
      tab[p->tm_push_at + k] = (uint32_t)lst.size();
      for (uint32_t b = 0; b < p->tm_bs && k * p->tm_bs + b < rows; ++b) {
        const uint32_t src = p->closure[k * p->tm_bs + b];
        for (uint32_t e = c->row_ptr[src]; e < c->row_ptr[src + 1]; ++e)
          if (c->col[e] != src) lst.push_back(c->col[e] | (b << 24));  // (not a dead slot)
      }
    }
    tab[p->tm_push_at + nbat] = (uint32_t)lst.size();
    if (c->N >= (1u << 24) || tab.size() + lst.size() >= (1ull << 32))
      return fail(c, SPF_E_INVALID, "msbfs_team: push list exceeds its encoding");
    tab.insert(tab.end(), lst.begin(), lst.end());
  }
  HIP_TRY(c, stage_upload(c, p->d_tm_map, tab.data(), tab.size()));
  HIP_TRY(c, p->d_tm_F.alloc((size_t)teams * 2 * fw * 2));  // u64 as 2 words
  HIP_TRY(c, p->d_tm_bar.alloc((size_t)teams * kTmBarPad * 4));
  // zeroed once: every launch leaves them zero (the kernel's exit protocol)
  HIP_TRY(c, hipMemsetAsync(p->d_tm_bar.p, 0, 4ull * teams * kTmBarPad * 4, c->stream));
  return SPF_OK;
}

spf_status launch_msbfs_team(spf_ctx* c, spf_plan* p, const uint32_t* rows_src, uint32_t rows,
                             uint32_t* D, uint8_t* Dn, uint32_t* maxd, hipStream_t s,
                             uint32_t d_rows, uint32_t* S, uint32_t s_stride) {
  if (!c->d_stamps.p && std::getenv("SPF_STAMPS")) {
    HIP_TRY(c, c->d_stamps.alloc(kStampWords));
    HIP_TRY(c, hipMemsetAsync(c->d_stamps.p, 0, kStampWords * 8, s));
    const unsigned long long wg = std::strtoull(std::getenv("SPF_STAMPS"), nullptr, 10);
    HIP_TRY(c, hipMemcpyAsync(c->d_stamps.p + 64 * 16, &wg, 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  const uint32_t fw = team_fwords(c->N);
  TeamArgs a{c->d_sell_col.p, p->d_tm_map.p, p->d_tm_map.p + p->tm_rptr_at, c->d_ovl.p, rows_src,
             rows, p->tm_bs, (rows + p->tm_bs - 1) / p->tm_bs, c->N, c->pitch, c->npitch, p->tm_G,
             (c->n_cu / 8) / p->tm_G, p->tm_nacc, fw,
             (uint32_t)std::max<size_t>(8ull * fw, (size_t)kTmWaves * kTmRows * 80 * 4),
             (uint32_t)(4ull * c->sell_col.size()), d_rows, S, s_stride, D, Dn, maxd,
             reinterpret_cast<unsigned long long*>(p->d_tm_F.p), p->d_tm_bar.p, c->d_stamps.p,
             p->d_tm_map.p + p->tm_need_at, p->tm_need_words, c->d_fault.p,
             p->d_tm_map.p + p->tm_push_at, p->d_tm_map.p + p->tm_push_at + p->tm_push_n,
             p->d_tm_map.p + p->tm_drained_at, p->tm_n_drained, 0u};
  if (const char* e = std::getenv("SPF_TEAM_FLUSH_DBG")) a.dbg = (uint32_t)atoi(e);
  const uint32_t* meta = p->d_tm_map.p + p->tm_runs_at;
  const uint32_t blocks = p->tm_teams * p->tm_G;  // = n_cu: one persistent workgroup per CU
  const size_t lds = team_lds(fw, p->tm_nacc);
  void* args[] = {&a, &meta};
  if (const spf_status st = resident_order(c, s); st != SPF_OK) return st;
  HIP_TRY(c, hipLaunchKernel(team_kernel(p->tm_own), dim3(blocks), dim3(kTmThreads), args, lds, s));
  return resident_done(c, s);
}

}  // namespace spfi
