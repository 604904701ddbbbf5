// ============================================================================
//  engine_internal.h -- state shared by the engine's translation units
//  (spf_engine.hip: SPF/ECMP plans; ksp2.hip: batched KSP2).  Not part of the
//  C-ABI: include/openr_spf.h is the boundary.
// ============================================================================
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "openr_spf.h"

namespace spfi {

constexpr uint32_t kInf = SPF_UNREACHABLE;
// diagnostics buffer (SPF_STAMPS): 16 waves x 64 phase stamps of one block,
// the block selector, then a start / end s_memrealtime pair per block
constexpr uint32_t kStampBlocks = 1024;
constexpr uint32_t kStampWords = 64 * 16 + 1 + 2 * kStampBlocks;

extern thread_local std::string g_err;

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { reset(); }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    reset();
    const hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) n = count;
    return e;
  }
  hipError_t upload(const T* h, size_t count, hipStream_t s) {
    hipError_t e = alloc(count);
    if (e != hipSuccess || count == 0) return e;
    return hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s);
  }
  // h[off, off + count) into the allocated buffer at the same offset
  hipError_t upload_at(const T* h, size_t off, size_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (!p || off + count > n) return hipErrorInvalidValue;
    return hipMemcpyAsync(p + off, h + off, count * sizeof(T), hipMemcpyHostToDevice, s);
  }
};

// Pinned host staging (hipHostMalloc): device-to-host copies at PCIe rate
// instead of the runtime's chunked pageable path.
template <typename T>
struct PinBuf {
  T* p = nullptr;
  size_t n = 0;
  PinBuf() = default;
  PinBuf(const PinBuf&) = delete;
  PinBuf& operator=(const PinBuf&) = delete;
  ~PinBuf() { reset(); }
  void reset() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    reset();
    const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T),
                                       hipHostMallocDefault);
    if (e == hipSuccess) n = count;
    return e;
  }
};

// exact_spf_kernel scratch (exact.hip): per-wave heap, labels, next hops.
struct ExactScratch {
  DevBuf<uint8_t> buf;
  DevBuf<uint32_t> ctr;  // next source
  uint64_t per_wave = 0;
  uint32_t waves = 0, wmax = 0;
};

// What-if batches on the exact kernel (zero / negative metrics, u64): one
// replayed runSpf per failure that touches a pathLink, digests vs the
// unfailed run (exact.hip).
struct ExactWhatIf {
  ExactScratch xs;
  DevBuf<uint32_t> fails, link_edge, base_pop, base_nh;
  DevBuf<uint64_t> base_d;
  DevBuf<spf_whatif_digest> base_dig;
  uint32_t src = 0, n_fail = 0, W = 1;
};

// KSP2 on the exact kernel: the sources' runs (labels, pop ranks), then a
// wave per pair tracing k = 1 and replaying k = 2 (exact.hip).
struct ExactKsp2 {
  ExactScratch xs_a, xs_b;
  DevBuf<uint32_t> srcs, POP;
  DevBuf<uint64_t> D;
  uint32_t n_src = 0, lw = 0;
};

}  // namespace spfi

struct spf_ctx {
  int device = 0;
  uint32_t n_cu = 256;  // compute units (BFS batch sizing)
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;  // what-if workgroup teams (lazily created, lives with the ctx)
  hipEvent_t side_fork = nullptr, side_join = nullptr;
  // barrier-timeout word of this context's grid-resident / team launches
  // (spf_device_check reads and clears it)
  spfi::DevBuf<uint32_t> d_fault;
  bool team_off = false;  // a team barrier timed out: plans keep msbfs_kernel
  std::string err;
  uint64_t solves = 0;
  uint64_t shape = 0;  // bumped by spf_graph_load (CSR structure)
  uint64_t epoch = 0;  // bumped by every graph change (load or in-place patch)
  // bumped when a patch changes some node's distinct-neighbour count (a
  // plan's next-hop layout); plans of the old layout fail with SPF_E_STATE
  uint64_t layout = 0;
  // the two CSR slots of every link id (kInf: none), kept by spf_graph_patch_rows
  std::vector<uint32_t> link_slot;
  // graph
  bool loaded = false;
  uint32_t N = 0, E = 0, pitch = 0;
  bool nonpos = false;
  bool needs64 = false;  // a negative metric or max metric x (N-1) >= 2^32 - 1: u64 labels
  uint32_t max_metric = 0;
  // live directed edges with metric <= 0, < 0, and weight == max_metric: a
  // row patch updates the metric facts from these without a graph scan
  uint64_t n_nonpos = 0, n_neg = 0, n_at_max = 0;
  std::vector<uint32_t> row_ptr, col, wt, rev, link;
  std::vector<int32_t> met;  // metrics as advertised (exact kernel)
  spfi::DevBuf<int32_t> d_met;
  spfi::ExactScratch exact1;  // spf_solve_exact (synchronous one-shot solves) only
  std::vector<uint8_t> ovl;
  std::vector<uint32_t> nb_ptr, nb_id, nb_w;  // distinct up neighbours
  uint32_t big_nodes = 0;                    // nodes with degree > kBigDeg
  uint32_t max_link = 0;
  bool unit = false;                         // every up edge has metric 1
  uint32_t npitch = 0;                       // narrow (u8) row pitch
  std::vector<uint32_t> sell_ptr, sell_col;  // sliced-ELL columns (64-node slices)
  uint64_t sell_ver = 0;  // bumped whenever sell_ptr / sell_col change (load, row patch)
  // msbfs_team_prepare's graph-derived tables for one team size (slices to
  // members, finalize slots, column streams, frontier slices each member
  // reads): valid while sell_ver holds, shared by every plan of the context
  struct TeamTables {
    uint64_t ver = ~0ull;
    uint32_t G = 0, own = 0, n_acc = 0, need_words = 0;
    bool full_copy = false;
    std::vector<uint32_t> fin, mptr, meta, need;
  } tm_tab;
  spfi::DevBuf<uint32_t> d_sell_ptr, d_sell_col;
  spfi::DevBuf<uint32_t> d_ms_smap;  // msbfs_kernel: slice of (wave, slot), balanced by width
  std::vector<uint32_t> sell4_ptr, sell4;  // packed u16x4 columns (uint2 entries), planes BFS
  spfi::DevBuf<uint32_t> d_sell4_ptr, d_sell4;
  spfi::DevBuf<uint32_t> d_row_ptr, d_col, d_wt, d_rev, d_nb_ptr, d_nb_id, d_nb_w;
  std::vector<uint32_t> edge_nb;     // host copy of d_edge_nb (patched in place)
  spfi::DevBuf<uint32_t> d_edge_nb;  // per CSR edge: its head's index among the tail's distinct neighbours
  spfi::DevBuf<uint8_t> d_ovl;
  // scratch for spf_preds
  spfi::DevBuf<uint32_t> d_pred_cnt, d_pred_edge, d_link, d_ign, d_one_src, d_row;
  spfi::DevBuf<unsigned long long> d_pred_key;
  spfi::DevBuf<uint32_t> d_gq, d_gq2, d_gbm, d_gctr;  // global-memory SSSP scratch
  spfi::DevBuf<uint32_t> d_gbar;  // its grid-barrier counters (whatif.hip XGrid)
  // per-node eccentricity estimates (planes BFS batch order), for ecc_epoch
  std::vector<uint32_t> ecc;
  uint64_t ecc_epoch = ~0ull;
  uint32_t dbound = 0;  // hop-distance upper bound (depth_bound), for dbound_epoch
  // recent bounds by (sliced-ELL structure version, drain bits): a drain bit
  // toggled back and forth (the BM_DecisionFabric publication) or a metric
  // patch (the bound counts hops) finds its bound again without a BFS
  struct DboundMemo {
    uint64_t sell_ver;
    std::vector<uint8_t> ovl;
    uint32_t dbound;
  };
  std::vector<DboundMemo> dbound_memo;
  uint64_t dbound_epoch = ~0ull;
  // mssp_kernel tables (mssp.hip), valid for graph epoch mp_epoch
  spfi::DevBuf<uint32_t> d_mp_ell, d_mp_smap;
  spfi::DevBuf<uint32_t> d_mp_dep;  // per slice: the slices its nodes' out-edges reach (CSR)
  spfi::DevBuf<uint32_t> d_mp_cls;  // per wave: first slot of each width class (phased first sweep)
  uint32_t mp_ncls = 0;
  uint32_t mp_slots = 0, mp_ovf_at = 0;
  bool mp_redo = true;
  bool mp_u8 = false;  // u8 labels (four sources per LDS word)
  uint64_t mp_epoch = ~0ull;
  spfi::DevBuf<unsigned long long> d_stamps;  // BFS kernel phase stamps (SPF_STAMPS=1)
  // spf_plan_preds' pinned staging: lives with the context (the facade makes
  // a plan per query; pinning per plan cost more than it saved)
  spfi::PinBuf<uint32_t> pin_preds;
  // plan builds' host-to-device uploads (spfi::stage_upload): one pinned
  // buffer, copies queued on `stream`, reused once `stream` has synchronised
  spfi::PinBuf<uint8_t> stage;
  size_t stage_used = 0;
  // spf_routes' (routes.hip) last plan, kept while its sources and the graph
  // shape hold (executes re-derive it after in-place patches), and its
  // buffers, which only grow: a route build per publication allocates nothing
  struct RouteCache {
    spf_plan* plan = nullptr;
    std::vector<uint32_t> srcs;
    uint64_t shape = ~0ull;
    spfi::DevBuf<uint32_t> dist, nh, ecol, ew, ej, sp, sn, cnt, edge;
    spfi::DevBuf<uint64_t> mn, metric;
  } rt;
};

namespace spfi {
// A plan build's uploads (build_plan, msbfs_team_prepare) through the
// context's pinned stage: a pageable hipMemcpyAsync is a blocking staged copy
// (~35 us each on MI355X boxes, a dozen per build_plan), a pinned one is only
// queued.  Copies go on c->stream; the stage is reused after that stream has
// synchronised (here when it runs full, and stage_done after a build's final
// synchronize).  Payloads above kStageMax take the plain path.
constexpr size_t kStageMax = 8u << 20;
// bytes from host memory to device memory through the stage (queued on c->stream)
inline hipError_t stage_copy(spf_ctx* c, void* dst, const void* h, size_t bytes) {
  if (bytes == 0) return hipSuccess;
  if (bytes > kStageMax) return hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, c->stream);
  size_t at = (c->stage_used + 255) & ~(size_t)255;
  if (!c->stage.p || at + bytes > c->stage.n) {
    if (c->stage_used) {
      const hipError_t e = hipStreamSynchronize(c->stream);  // every copy out of the stage has landed
      if (e != hipSuccess) return e;
    }
    c->stage_used = at = 0;
    if (bytes > c->stage.n || !c->stage.p) {
      const hipError_t e = c->stage.alloc(std::max<size_t>(std::max<size_t>(bytes, 2 * c->stage.n), 1u << 20));
      if (e != hipSuccess) return e;
    }
  }
  std::memcpy(c->stage.p + at, h, bytes);
  c->stage_used = at + bytes;
  return hipMemcpyAsync(dst, c->stage.p + at, bytes, hipMemcpyHostToDevice, c->stream);
}
template <typename T>
hipError_t stage_upload(spf_ctx* c, DevBuf<T>& d, const T* h, size_t count) {
  const hipError_t e = d.alloc(count);
  if (e != hipSuccess || count == 0) return e;
  return stage_copy(c, d.p, h, count * sizeof(T));
}
// h[off, off + count) into the allocated buffer at the same offset
template <typename T>
hipError_t stage_upload_at(spf_ctx* c, DevBuf<T>& d, const T* h, size_t off, size_t count) {
  if (count == 0) return hipSuccess;
  if (!d.p || off + count > d.n) return hipErrorInvalidValue;
  return stage_copy(c, d.p + off, h + off, count * sizeof(T));
}
// after a synchronize of c->stream: the stage's copies are done
inline void stage_done(spf_ctx* c) { c->stage_used = 0; }
}  // namespace spfi

struct spf_plan {
  spf_ctx* ctx = nullptr;
  uint32_t n_src = 0, flags = 0;
  uint64_t shape = 0, epoch = 0;  // graph state the plan was derived from
  uint64_t layout = 0;             // c->layout its next-hop layout was taken at
  std::vector<uint32_t> srcs, closure;
  std::vector<uint64_t> nh_off;
  std::vector<uint32_t> words;
  uint64_t nh_total = 0;
  bool direct = false;  // closure == srcs: D is the caller's dist buffer
  bool prefix = false;  // closure[i] == srcs[i] for i < n_src (distinct sources)
  bool ms = false;      // unit metrics: multi-source BFS
  bool narrow = false;  // ... writing the u8 narrow copy for the next-hop pass
  bool sliced = false;  // ... and the next-hop pass on its bit-sliced form
  bool expand = false;  // ... the u32 rows expanded from the u8 ones (BFS stores bytes only)
  bool exact = false;   // exact_spf_kernel (exact.hip): zero/negative metrics, u64, any size
  bool mp = false;      // weighted: mssp_kernel (mssp.hip), S sources per workgroup
  bool pl_order = false;  // planes BFS: rows batched deepest-first (d_pl_order)
  bool sdirect = false;   // team plan writing the sliced rows itself (kTeamPlanes planes, no u8 rows)
  // msbfs_team_kernel (msbfs_team.hip): G workgroups per batch when the plan
  // has too few batches to fill the chip (tm_G == 0: msbfs_kernel)
  uint32_t tm_G = 0, tm_own = 0, tm_teams = 0, tm_bs = 0, tm_nacc = 0;
  uint32_t tm_rptr_at = 0, tm_runs_at = 0;  // d_tm_map = finalize slots | stream ranges | streams
  uint32_t tm_need_at = 0, tm_need_words = 0;  // ... | per-member frontier slice masks
  uint32_t tm_drained_at = 0, tm_n_drained = 0;  // ... | the drained nodes
  uint32_t tm_push_at = 0, tm_push_n = 0;  // ... | batch push offsets [tm_push_n] | push lists
  spfi::DevBuf<uint32_t> d_tm_map, d_tm_F, d_tm_bar;
  spfi::DevBuf<uint32_t> d_pl_order;
  spfi::DevBuf<uint32_t> d_redo;  // mp: rows whose u16 labels may have overflowed
  uint32_t wmax = 0;    // exact: max next-hop words per node over the plan's sources
  spfi::ExactScratch xs;  // exact: the kernel's scratch, reserved by build_plan
  spfi::DevBuf<uint32_t> d_srcs, d_closure, d_row_of, d_req_rows, d_D;
  spfi::DevBuf<uint8_t> d_Dn;
  spfi::DevBuf<uint32_t> d_S, d_maxd;  // sliced rows (+ dead row); deepest BFS level + 8 counters
  spfi::DevBuf<uint32_t> d_units, d_unit_off;  // sliced pass: uint4 work units per XCD
  spfi::DevBuf<uint32_t> d_gtab;  // sliced pass: source groups ([n, sources...] each)
  uint32_t max_xcd_units = 0;
  bool big = false;  // spf_big_kernel (whatif.hip): graphs beyond the LDS kernels
  spfi::DevBuf<uint32_t> b_q, b_q2, b_bm, b_ctr, b_nbr_bit, b_nhb, b_lvl, b_order, b_misc, b_parent;
  spfi::DevBuf<uint32_t> b_bar;  // spf_big_kernel's grid-barrier counters
  spfi::DevBuf<uint64_t> d_nh_off;
  spfi::DevBuf<uint32_t> d_words;  // [n_src] next-hop bitmaps per source (spf_plan_digest)
  spfi::DevBuf<uint32_t> d_nb_row, d_nb_row_off, d_nb_drained;  // next-hop pass inputs
  uint32_t dead = 0;  // nb_row value of a drained neighbour
  spfi::DevBuf<uint32_t> d_slot_src;  // next-hop blocks: source per (slot, XCD)
  spfi::DevBuf<uint32_t> h_dist, h_nh;  // spf_plan_execute_host staging
  uint64_t h_epoch = ~0ull;              // graph epoch of the rows in h_dist
  spfi::DevBuf<uint32_t> h_pcnt, h_pedge;  // spf_plan_preds scratch
  spfi::DevBuf<unsigned long long> h_pkey;  // ... its sort keys
  size_t slots = 0;
  size_t lds_bytes = 0;
  bool q16 = true;
  // optional per-kernel timing: 4 events per execute (before the distance
  // kernel, after it, after the row slicing, after ECMP), ring of
  // `timing_cap` executes
  std::vector<hipEvent_t> ev;
  uint32_t timing_cap = 0, timing_n = 0;
  ~spf_plan() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
};

namespace spfi {

spf_status fail(spf_ctx* c, spf_status st, const char* fmt, ...);

#define HIP_TRY(ctx, expr)                                                   \
  do {                                                                       \
    const hipError_t e_ = (expr);                                            \
    if (e_ != hipSuccess)                                                    \
      return fail(ctx, e_ == hipErrorOutOfMemory ? SPF_E_NOMEM : SPF_E_HIP,   \
                  "%s: %s (%s:%d)", #expr,                                   \
                  hipGetErrorString(e_), __FILE__, __LINE__);                \
  } while (0)

// Upload an ignore set (undirected link ids) as a device bitmap; NULL if empty.
spf_status upload_ignore(spf_ctx* c, const uint32_t* ignore, uint32_t n_ignore,
                         const uint32_t** dev);

// Launch the per-source SSSP kernel (distances only) over `rows` sources
// (device list rows_src), writing rows [rows][pitch] of D.
// wt / ovl override the graph's metrics / drain bits (e.g. transposed
// metrics and no drains for distances TO the rows' nodes).
spf_status launch_sssp(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, bool hop,
                       const uint32_t* ign, uint32_t* D, hipStream_t s,
                       const uint32_t* wt = nullptr, const uint8_t* ovl = nullptr,
                       uint8_t* Dn = nullptr, const uint32_t* redo = nullptr);
// Multi-source weighted distances (mssp.hip): mssp_words() = LDS words per
// node (0: does not apply), mssp_prepare() builds its tables for the current
// graph epoch (plan build), launch_mssp() enqueues it (+ the overflow redo
// pass over `redo` = [1 + rows] words of plan scratch).
uint32_t mssp_words(const spf_ctx* c);
uint32_t mssp_sources(const spf_ctx* c);
// Team BFS (msbfs_team.hip): the team size for a unit plan of `rows` rows
// (0: not used), its tables, its launch, its barrier-timeout flag.
uint32_t msbfs_team_size(const spf_ctx* c, uint32_t rows);
spf_status msbfs_team_prepare(spf_ctx* c, spf_plan* p, uint32_t G);
spf_status launch_msbfs_team(spf_ctx* c, spf_plan* p, const uint32_t* rows_src, uint32_t rows,
                             uint32_t* D, uint8_t* Dn, uint32_t* maxd, hipStream_t s,
                             uint32_t d_rows,  // u32 rows written: closure rows < d_rows
                             uint32_t* S = nullptr, uint32_t s_stride = 0);  // sdirect planes
// planes per word of the rows msbfs_team_kernel slices itself (sdirect plans)
constexpr uint32_t kTeamPlanes = 4;
spf_status mssp_prepare(spf_ctx* c);
spf_status mssp_set_lds_limits(spf_ctx* c);
spf_status launch_mssp(spf_ctx* c, const uint32_t* rows_src, uint32_t rows, uint32_t* D,
                       uint8_t* Dn, uint32_t* redo, hipStream_t s, uint32_t* maxd = nullptr);
// Single-source SSSP in global memory, one cooperative grid (any graph
// size); scratch lives in the context.  dist = [N].
spf_status launch_gsssp(spf_ctx* c, uint32_t src, bool hop, const uint32_t* ign, uint32_t* dist,
                        hipStream_t s);
// The exact kernel (exact.hip) over n_src sources: dist rows (u32 or u64,
// pitch entries), planar next-hop bitmaps at nh_off, optional pop ranks.
spf_status exact_reserve(spf_ctx* c, ExactScratch* x, uint32_t n_src, uint32_t Wmax,
                         uint64_t extra = 0);
spf_status exact_whatif_prepare(spf_ctx* c, ExactWhatIf* x, uint32_t src,
                                const std::vector<uint32_t>& fails,
                                const std::vector<uint32_t>& link_edge);
spf_status exact_whatif_launch(spf_ctx* c, ExactWhatIf* x, spf_whatif_digest* d_out,
                               spf_whatif_digest* d_base, hipStream_t s, hipEvent_t mid);
spf_status exact_ksp2_prepare(spf_ctx* c, ExactKsp2* x, const std::vector<uint32_t>& srcs);
spf_status exact_ksp2_launch(spf_ctx* c, ExactKsp2* x, spf_ksp2_pair* d_pairs, uint32_t* d_pool,
                             uint64_t pool_words, uint64_t* d_counters, hipStream_t s,
                             hipEvent_t mid);
spf_status launch_exact(spf_ctx* c, ExactScratch* x, const uint32_t* d_srcs, uint32_t n_src,
                        const uint64_t* d_nh_off, uint32_t Wmax, bool hop, bool dist64,
                        const uint32_t* ign, void* d_dist, uint32_t* d_nh, uint32_t* d_pop,
                        hipStream_t s);
// spf_big_kernel (whatif.hip): the plan's sources one after another on the
// whole chip -- frontier SSSP into the dist rows, next hops in distance
// order, transposed into the plan's bitmaps.  Positive metrics or hop counts.
spf_status launch_big(spf_ctx* c, spf_plan* p, uint32_t* d_dist, uint32_t* d_nh, bool hop,
                      hipStream_t s);
// Raise the dynamic-LDS limit of the engine's LDS-resident kernels.
spf_status set_lds_limits(spf_ctx* c);
// Order a launch whose workgroups wait on each other (grid barriers, team
// BFS) on stream s after the previous such launch of this process on the
// same device, whatever context or stream that was on: two of them running
// at once could each hold part of the CUs the other's members need (each
// waits for members that cannot become resident until it exits).  Call
// before the launch, then resident_done(c, s) after it.
spf_status resident_order(spf_ctx* c, hipStream_t s);
spf_status resident_done(spf_ctx* c, hipStream_t s);
void resident_forget(const spf_ctx* c);
// Materialised route databases of many `me` (routes.hip kRsDb): per me slot
// its headers (n_sets words), where its region of the record pool starts
// (n_chunks x 256 x deg(me) records), its record count (zeroed before the
// launch, added to) and the error flags.
struct RouteDbOut {
  unsigned long long* hdr = nullptr;
  unsigned long long* pool = nullptr;
  const unsigned long long* base = nullptr;
  uint32_t* count = nullptr;
  uint32_t* flags = nullptr;
};
// sets per kRsDb tile (the [deg][sets] tiles of a route database region)
uint32_t route_db_tile_sets();
// Route selection over resident rows for many `me` (routes.hip): digests per
// me (d_digest, n_me slots, added to), their route databases (db), or
// spf_routes' records of ONE me.
spf_status launch_route_sets(spf_ctx* c, const unsigned long long* d_rowp,
                             const unsigned long long* d_nhp, const uint32_t* d_me, uint32_t n_me,
                             const uint32_t* d_set_ptr, const uint32_t* d_set_nodes, uint32_t n_sets,
                             bool lfa, const unsigned long long* d_link_hash,
                             unsigned long long* d_digest, uint64_t* d_min, uint32_t* d_cnt,
                             uint32_t* d_edge, uint64_t* d_metric, hipStream_t s,
                             const RouteDbOut* db = nullptr,
                             const unsigned long long* d_nrowp = nullptr);
// pathLinks of `src` from its u32 distance row on the device (spf_preds
// without the upload; spf_mplan_preds reads a resident row).
spf_status preds_from_row(spf_ctx* c, uint32_t src, bool hop, const uint32_t* ign,
                          const uint32_t* d_row, uint32_t* pred_ptr, uint32_t* pred_edge,
                          uint32_t cap, uint32_t* n_preds, hipStream_t s);

}  // namespace spfi
