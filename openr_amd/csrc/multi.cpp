// ============================================================================
//  multi.cpp -- several GPUs behind one C-ABI context (include/openr_spf.h,
//  "multi-device context").
//
//  Open/R's Decision is one process on one event-base thread
//  (openr/decision/Decision.cpp:1484): the LinkState it owns must reach every
//  GPU of the node from that thread, not through a process per GPU.  An
//  spf_mctx holds one engine context (spf_ctx) per listed device, each with
//  its own replica of the graph (the CSR is small and
//  replicated); an spf_mplan splits a batch of sources over the members --
//  the locality partition (a source's next hops need its neighbours' rows,
//  so a member solves its sources' neighbours too: keep that closure small)
//  or contiguous blocks -- and keeps every member's distance rows and
//  next-hop bitmaps resident in that member's HBM.  Queries
//  (spf_mplan_read / spf_mplan_preds / spf_mplan_digest) are answered by the
//  owning member: the way Decision::getDecisionRouteDb(node) for every node
//  (Decision.cpp:1480-1500) reads an all-sources pass.
//
//  Device ids may repeat (one GPU holding several members, e.g. for tests on
//  a one-GPU machine): members of one device share that device's execute
//  stream, so their executes run one after another there, exactly as they
//  would run side by side on separate GPUs.
// ============================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <numeric>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine_internal.h"

using namespace spfi;

namespace {

// a source's cost in next-hop bitmaps: its k bitmaps plus its distance rows
// (u32 + the u8 copy = 5N bytes = 40 bitmaps of N/8 bytes); the same
// constant as openr_amd/sharding.py AllSourcesLayout.ROW_COST
constexpr double kRowCost = 40.0;
constexpr uint32_t kLocalityMaxNodes = 1u << 16;

// closure sizes of a partition: per part, its sources plus their neighbours
std::vector<uint32_t> closure_sizes(const uint32_t* nb_ptr, const uint32_t* nb_id, uint32_t n_nodes,
                                    const uint32_t* srcs, uint32_t n_src, const uint32_t* part,
                                    uint32_t n_parts) {
  std::vector<uint32_t> out(n_parts, 0);
  std::vector<uint32_t> mark(n_nodes, 0xFFFFFFFFu);
  for (uint32_t r = 0; r < n_parts; ++r) {
    uint32_t cnt = 0;
    auto add = [&](uint32_t x) {
      if (mark[x] != r) mark[x] = r, ++cnt;
    };
    for (uint32_t i = 0; i < n_src; ++i) {
      if (part[i] != r) continue;
      add(srcs[i]);
      for (uint32_t e = nb_ptr[srcs[i]]; e < nb_ptr[srcs[i] + 1]; ++e) add(nb_id[e]);
    }
    out[r] = cnt;
  }
  return out;
}

// contiguous blocks of the request order balanced by cost (k + kRowCost):
// block r ends at the first prefix cost above total * (r+1) / n_parts
void contiguous_parts(const uint32_t* nb_ptr, const uint32_t* srcs, uint32_t n_src,
                      uint32_t n_parts, uint32_t* part) {
  std::vector<double> cum(n_src);
  double acc = 0;
  for (uint32_t i = 0; i < n_src; ++i) {
    acc += (double)(nb_ptr[srcs[i] + 1] - nb_ptr[srcs[i]]) + kRowCost;
    cum[i] = acc;
  }
  std::vector<uint32_t> bounds(n_parts + 1, 0);
  bounds[n_parts] = n_src;
  for (uint32_t r = 1; r < n_parts; ++r)
    bounds[r] = (uint32_t)(std::upper_bound(cum.begin(), cum.end(), acc * r / n_parts) - cum.begin());
  for (uint32_t r = 0; r < n_parts; ++r)
    for (uint32_t i = bounds[r]; i < std::max(bounds[r], bounds[r + 1]); ++i) part[i] = r;
}

// One-pass streaming partition (linear deterministic greedy): sources in
// ascending (degree, position), each to the part whose closure it grows
// least among the parts whose cost stays within 3 % of the mean, ties to
// the least loaded, then the lowest part.  Low-degree nodes first: a
// fabric's rack switches gather by pod, the fabric switches follow their
// pod, a plane's spines land together.  Same rule as sharding.py
// locality_partition (tests/test_partition.py checks they agree).
void locality_parts(const uint32_t* nb_ptr, const uint32_t* nb_id, uint32_t n_nodes,
                    const uint32_t* srcs, uint32_t n_src, uint32_t n_parts, uint32_t* part) {
  std::vector<uint32_t> order(n_src);
  std::iota(order.begin(), order.end(), 0u);
  auto deg = [&](uint32_t i) { return nb_ptr[srcs[i] + 1] - nb_ptr[srcs[i]]; };
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return deg(a) < deg(b); });
  double total = 0;
  for (uint32_t i = 0; i < n_src; ++i) total += (double)deg(i) + kRowCost;
  const double cap = total / n_parts * (1.0 + 0.03);  // sharding.py: sum / world * (1 + slack)
  std::vector<uint8_t> clo((size_t)n_parts * n_nodes, 0);
  std::vector<double> load(n_parts, 0.0);
  std::vector<double> grow(n_parts);
  for (uint32_t i : order) {
    const uint32_t v = srcs[i];
    const double cost = (double)deg(i) + kRowCost;
    bool any_ok = false;
    for (uint32_t r = 0; r < n_parts; ++r) any_ok |= load[r] + cost <= cap;
    for (uint32_t r = 0; r < n_parts; ++r) {
      if (any_ok && !(load[r] + cost <= cap)) {
        grow[r] = std::numeric_limits<double>::infinity();
        continue;
      }
      const uint8_t* c = clo.data() + (size_t)r * n_nodes;
      uint32_t g = c[v] ? 0u : 1u;
      for (uint32_t e = nb_ptr[v]; e < nb_ptr[v + 1]; ++e) g += c[nb_id[e]] ? 0u : 1u;
      grow[r] = g;
    }
    const double best = *std::min_element(grow.begin(), grow.end());
    uint32_t pick = n_parts;
    for (uint32_t r = 0; r < n_parts; ++r)
      if (grow[r] == best && (pick == n_parts || load[r] < load[pick])) pick = r;
    part[i] = pick;
    uint8_t* c = clo.data() + (size_t)pick * n_nodes;
    c[v] = 1;
    for (uint32_t e = nb_ptr[v]; e < nb_ptr[v + 1]; ++e) c[nb_id[e]] = 1;
    load[pick] += cost;
  }
}

uint32_t partition(const uint32_t* nb_ptr, const uint32_t* nb_id, uint32_t n_nodes,
                   const uint32_t* srcs, uint32_t n_src, uint32_t n_parts, uint32_t mode,
                   uint32_t* part) {
  contiguous_parts(nb_ptr, srcs, n_src, n_parts, part);
  if (mode == SPF_PARTITION_CONTIGUOUS || n_parts <= 1) return SPF_PARTITION_CONTIGUOUS;
  if (mode == SPF_PARTITION_AUTO && n_nodes > kLocalityMaxNodes) return SPF_PARTITION_CONTIGUOUS;
  std::vector<uint32_t> loc(n_src);
  locality_parts(nb_ptr, nb_id, n_nodes, srcs, n_src, n_parts, loc.data());
  if (mode == SPF_PARTITION_AUTO) {
    const auto a = closure_sizes(nb_ptr, nb_id, n_nodes, srcs, n_src, part, n_parts);
    const auto b = closure_sizes(nb_ptr, nb_id, n_nodes, srcs, n_src, loc.data(), n_parts);
    if (*std::max_element(b.begin(), b.end()) >= *std::max_element(a.begin(), a.end()))
      return SPF_PARTITION_CONTIGUOUS;
  }
  std::copy(loc.begin(), loc.end(), part);
  return SPF_PARTITION_LOCALITY;
}

}  // namespace

struct spf_mctx {
  std::vector<spf_ctx*> members;
  std::vector<hipStream_t> exec;  // per member: its device's execute stream (shared by repeats)
  std::string err;
  ~spf_mctx() {
    for (spf_ctx* c : members) spf_ctx_destroy(c);
  }
};

struct spf_mplan {
  spf_mctx* m = nullptr;
  uint32_t n_src = 0, flags = 0, mode = 0;
  std::vector<uint32_t> srcs, owner, row;  // per request index: member, row in its plan
  struct Part {
    spf_plan* plan = nullptr;
    std::vector<uint32_t> req;  // request indices in plan order
    std::vector<uint64_t> nh_off;
    std::vector<uint32_t> words;
    DevBuf<uint32_t> dist, nh;
    DevBuf<unsigned long long> dig;
    hipGraphExec_t gexec = nullptr;
    hipGraph_t graph = nullptr;
    uint64_t g_epoch = ~0ull;  // graph epoch the captured executes belong to
    bool g_team_off = false;   // ... and the context's team switch
    std::vector<hipEvent_t> ev;  // timing: [2 * cap] start / end per execute
    // route selection over the resident pass (spf_mplan_route_digests /
    // spf_mplan_routes): every resident row's device address, the request's
    // sets, its me list and outputs on this member's device
    DevBuf<unsigned long long> rowp, nhp, lh, rdig, rmin, rmetric;
    DevBuf<unsigned long long> nrowp;  // every resident node's exact u8 row (u8 LFA loads), or none
    DevBuf<uint32_t> rsp, rsn, rme, rcnt, redge;
    std::vector<uint32_t> h_rsp, h_rsn;  // host copies of the uploaded sets (re-upload only on change)
    std::vector<uint64_t> h_lh;
    uint64_t r_epoch = ~0ull;  // execute count the address tables belong to
    // materialised route databases (spf_mplan_route_records): per me slot
    // [n_sets] headers, its region of the record pool, reservation cursors
    DevBuf<unsigned long long> dbhdr, dbpool, dbbase;
    DevBuf<uint32_t> dbcnt, dbflags;
    std::vector<uint32_t> db_me, h_dbcnt;
    std::vector<unsigned long long> h_dbbase;
    uint64_t db_tiles = 0;  // sets rounded up to whole 256-set tiles
  };
  // the last spf_mplan_route_records: request t -> (member, slot), sets
  std::vector<std::pair<uint32_t, uint32_t>> db_loc;
  uint32_t db_sets = 0;
  std::vector<unsigned long long> h_rowp, h_nhp;  // the address tables (host; uploads read them)
  std::vector<unsigned long long> h_nrowp;  // u8 rows, when every member's are exact (else empty)
  std::unique_ptr<Part[]> parts;  // [n_parts]
  uint32_t n_parts = 0;
  bool graphs = false;
  uint32_t timing_cap = 0, timing_n = 0;
  uint64_t executes = 0;   // bumps on every spf_mplan_execute (route tables follow it)
  int peer = -1;           // 1: every member can read every other member's HBM
  // host enqueue: per member, ns from the execute's start until its launches
  // were enqueued (the last execute; spf_mplan_enqueue_ns)
  std::vector<uint64_t> enq_ns;
  // per-member enqueue threads (spf_mplan_set_enqueue_threads): each member's
  // launches issued from its own host thread, so the last GPU does not start
  // n_members - 1 enqueues after the first
  struct Pool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> gen{0};
    std::atomic<uint32_t> pending{0};
    std::atomic<bool> stop{false};
    std::vector<spf_status> st;
    std::chrono::steady_clock::time_point t0;
  };
  std::unique_ptr<Pool> pool;
  int threads_mode = -1;  // -1: automatic (distinct devices), 0 off, 1 on
  void stop_pool() {
    if (!pool) return;
    {
      std::lock_guard<std::mutex> lk(pool->mu);
      pool->stop = true;
    }
    pool->cv.notify_all();
    for (auto& t : pool->th) t.join();
    pool.reset();
  }
  ~spf_mplan() {
    stop_pool();
    for (size_t i = 0; i < n_parts; ++i) {
      Part& p = parts[i];
      if (!p.plan) continue;
      (void)hipSetDevice(m->members[i]->device);
      (void)hipStreamSynchronize(m->exec[i]);
      if (p.gexec) (void)hipGraphExecDestroy(p.gexec);
      if (p.graph) (void)hipGraphDestroy(p.graph);
      for (hipEvent_t e : p.ev) (void)hipEventDestroy(e);
      spf_plan_destroy(p.plan);
      p.dist.reset();
      p.nh.reset();
      p.dig.reset();
    }
  }
};

namespace {

std::mutex g_err_mu;  // member errors may come from the enqueue threads

spf_status mfail(spf_mctx* m, spf_status st, const char* fmt, ...) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (m) m->err = buf;
  g_err = buf;
  return st;
}

spf_status member_fail(spf_mctx* m, uint32_t i, spf_status st) {
  return mfail(m, st, "member %u (device %d): %s", i, m->members[i]->device,
               spf_last_error(m->members[i]));
}

#define M_HIP(m, expr)                                                                   \
  do {                                                                                   \
    const hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                                \
      return mfail(m, e_ == hipErrorOutOfMemory ? SPF_E_NOMEM : SPF_E_HIP, "%s: %s (%s:%d)", \
                   #expr, hipGetErrorString(e_), __FILE__, __LINE__);                     \
  } while (0)

// One member's execute on its device's stream: a replay of the captured
// graph when one matches the member's graph epoch, else the plan's execute
// (which re-derives the plan after an in-place patch) -- captured then for
// the next call when graphs are on.
spf_status run_part(spf_mplan* mp, uint32_t i) {
  spf_mctx* m = mp->m;
  spf_ctx* c = m->members[i];
  spf_mplan::Part& p = mp->parts[i];
  const hipStream_t s = m->exec[i];
  M_HIP(m, hipSetDevice(c->device));
  hipEvent_t* ev = nullptr;
  if (mp->timing_cap) {
    ev = &p.ev[2 * (mp->timing_n % mp->timing_cap)];
    M_HIP(m, hipEventRecord(ev[0], s));
  }
  // (a capture made before a team timeout turned teams off is stale too)
  if (p.gexec && p.g_epoch == spf_graph_epoch(c) && p.g_team_off == c->team_off) {
    // A replay bypasses the plan's own resident_order / resident_done (they
    // skip a capturing stream): a plan with grid-resident launches (team BFS,
    // big-graph kernel) orders the replay itself, so it never splits the CUs
    // with another context's resident launch on this device.
    const bool resident = p.plan->tm_G || p.plan->big;
    if (resident) {
      const spf_status st = resident_order(c, s);
      if (st != SPF_OK) return member_fail(m, i, st);
    }
    M_HIP(m, hipGraphLaunch(p.gexec, s));
    if (resident) {
      const spf_status st = resident_done(c, s);
      if (st != SPF_OK) return member_fail(m, i, st);
    }
  } else {
    if (p.gexec) {
      (void)hipGraphExecDestroy(p.gexec);
      (void)hipGraphDestroy(p.graph);
      p.gexec = nullptr;
      p.graph = nullptr;
    }
    // A re-derive (graph patched, teams turned off) rebuilds the plan's
    // tables on the member's own stream; a member whose execute runs on a
    // shared stream (repeated device id) waits for what is in flight there
    // first, so the rebuild never overwrites tables a queued kernel reads.
    if (s != c->stream && (p.plan->epoch != c->epoch || (p.plan->tm_G && c->team_off)))
      M_HIP(m, hipStreamSynchronize(s));
    spf_status st = spf_plan_execute(p.plan, p.dist.p, p.nh.p, s);
    if (st != SPF_OK) return member_fail(m, i, st);
    if (mp->graphs) {  // the plan is derived for this epoch now: capture its launches
      M_HIP(m, hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
      st = spf_plan_execute(p.plan, p.dist.p, p.nh.p, s);
      hipGraph_t g = nullptr;
      const hipError_t e = hipStreamEndCapture(s, &g);
      if (st != SPF_OK) {
        if (g) (void)hipGraphDestroy(g);
        return member_fail(m, i, st);
      }
      M_HIP(m, e);
      M_HIP(m, hipGraphInstantiate(&p.gexec, g, nullptr, nullptr, 0));
      p.graph = g;
      p.g_epoch = spf_graph_epoch(c);
      p.g_team_off = c->team_off;
    }
  }
  if (ev) M_HIP(m, hipEventRecord(ev[1], s));
  return SPF_OK;
}

}  // namespace

extern "C" {

spf_status spf_partition_sources(const uint32_t* nb_ptr, const uint32_t* nb_id, uint32_t n_nodes,
                                 const uint32_t* srcs, uint32_t n_src, uint32_t n_parts,
                                 uint32_t mode, uint32_t* part_out, uint32_t* mode_used) {
  if (!nb_ptr || (n_src && (!srcs || !part_out)) || n_parts == 0 || mode > SPF_PARTITION_LOCALITY)
    return mfail(nullptr, SPF_E_INVALID, "spf_partition_sources: bad argument");
  if (nb_ptr[n_nodes] && !nb_id) return mfail(nullptr, SPF_E_INVALID, "spf_partition_sources: nb_id NULL");
  for (uint32_t i = 0; i < n_src; ++i)
    if (srcs[i] >= n_nodes) return mfail(nullptr, SPF_E_INVALID, "source %u out of range", srcs[i]);
  const uint32_t used = partition(nb_ptr, nb_id, n_nodes, srcs, n_src, n_parts, mode, part_out);
  if (mode_used) *mode_used = used;
  return SPF_OK;
}

spf_status spf_mctx_create(const int* gpu_ids, uint32_t n, spf_mctx** out) {
  if (!out || !gpu_ids || n == 0) return mfail(nullptr, SPF_E_INVALID, "spf_mctx_create: bad argument");
  *out = nullptr;
  auto m = std::make_unique<spf_mctx>();
  std::map<int, hipStream_t> dev_stream;
  for (uint32_t i = 0; i < n; ++i) {
    spf_ctx* c = nullptr;
    const spf_status st = spf_ctx_create(gpu_ids[i], &c);
    if (st != SPF_OK) return mfail(nullptr, st, "member %u: %s", i, spf_global_error());
    m->members.push_back(c);
    auto it = dev_stream.find(gpu_ids[i]);
    if (it == dev_stream.end()) it = dev_stream.emplace(gpu_ids[i], c->stream).first;
    m->exec.push_back(it->second);
  }
  *out = m.release();
  return SPF_OK;
}

void spf_mctx_destroy(spf_mctx* m) { delete m; }
const char* spf_mctx_last_error(const spf_mctx* m) { return m ? m->err.c_str() : g_err.c_str(); }
uint32_t spf_mctx_size(const spf_mctx* m) { return m ? (uint32_t)m->members.size() : 0; }
spf_ctx* spf_mctx_member(spf_mctx* m, uint32_t i) {
  return m && i < m->members.size() ? m->members[i] : nullptr;
}
int spf_mctx_device(const spf_mctx* m, uint32_t i) {
  return m && i < m->members.size() ? m->members[i]->device : -1;
}

// Patches upload on each member's own stream, while a member of a repeated
// device id executes on that device's shared stream: wait for every execute
// stream first, so a patch never rewrites the drain bytes / metrics a queued
// execute still reads (spf_mplan_execute returns before its kernels run).
static spf_status drain_exec(spf_mctx* m) {
  for (uint32_t i = 0; i < m->members.size(); ++i) {
    M_HIP(m, hipSetDevice(m->members[i]->device));
    M_HIP(m, hipStreamSynchronize(m->exec[i]));
  }
  return SPF_OK;
}

spf_status spf_mctx_graph_load(spf_mctx* m, const spf_graph* g) {
  if (!m || !g) return mfail(m, SPF_E_INVALID, "spf_mctx_graph_load: NULL argument");
  if (const spf_status st = drain_exec(m); st != SPF_OK) return st;
  for (uint32_t i = 0; i < m->members.size(); ++i) {
    const spf_status st = spf_graph_load(m->members[i], g);
    if (st != SPF_OK) return member_fail(m, i, st);
  }
  return SPF_OK;
}

spf_status spf_mctx_graph_set_overload(spf_mctx* m, const uint32_t* nodes, const uint8_t* overloaded,
                                       uint32_t n) {
  if (!m) return mfail(m, SPF_E_INVALID, "spf_mctx_graph_set_overload: NULL context");
  if (const spf_status st = drain_exec(m); st != SPF_OK) return st;
  for (uint32_t i = 0; i < m->members.size(); ++i) {
    const spf_status st = spf_graph_set_overload(m->members[i], nodes, overloaded, n);
    if (st != SPF_OK) return member_fail(m, i, st);
  }
  return SPF_OK;
}

spf_status spf_mctx_graph_set_metric(spf_mctx* m, const uint32_t* edges, const int32_t* metric,
                                     uint32_t n) {
  if (!m) return mfail(m, SPF_E_INVALID, "spf_mctx_graph_set_metric: NULL context");
  if (const spf_status st = drain_exec(m); st != SPF_OK) return st;
  for (uint32_t i = 0; i < m->members.size(); ++i) {
    const spf_status st = spf_graph_set_metric(m->members[i], edges, metric, n);
    if (st != SPF_OK) return member_fail(m, i, st);
  }
  return SPF_OK;
}

spf_status spf_mctx_graph_patch_rows(spf_mctx* m, const uint32_t* nodes, uint32_t n,
                                     const uint32_t* col, const int32_t* metric, const uint32_t* link) {
  if (!m) return mfail(m, SPF_E_INVALID, "spf_mctx_graph_patch_rows: NULL context");
  if (const spf_status st = drain_exec(m); st != SPF_OK) return st;
  for (uint32_t i = 0; i < m->members.size(); ++i) {
    const spf_status st = spf_graph_patch_rows(m->members[i], nodes, n, col, metric, link);
    if (st != SPF_OK) return member_fail(m, i, st);
  }
  return SPF_OK;
}

spf_status spf_mplan_create(spf_mctx* m, const uint32_t* srcs, uint32_t n_src, uint32_t flags,
                            uint32_t mode, spf_mplan** out) {
  if (!m || !out || !srcs || n_src == 0 || mode > SPF_PARTITION_LOCALITY)
    return mfail(m, SPF_E_INVALID, "spf_mplan_create: bad argument");
  *out = nullptr;
  spf_ctx* c0 = m->members[0];
  for (spf_ctx* c : m->members)
    if (!c->loaded || c->shape == 0 || c->N != c0->N)
      return mfail(m, SPF_E_STATE, "spf_mplan_create: load the graph with spf_mctx_graph_load first");
  for (uint32_t i = 0; i < n_src; ++i)
    if (srcs[i] >= c0->N) return mfail(m, SPF_E_INVALID, "source %u out of range", srcs[i]);
  const uint32_t P = (uint32_t)m->members.size();
  auto mp = std::make_unique<spf_mplan>();
  mp->m = m;
  mp->n_src = n_src;
  mp->flags = flags;
  mp->srcs.assign(srcs, srcs + n_src);
  mp->owner.resize(n_src);
  mp->row.resize(n_src);
  mp->mode = partition(c0->nb_ptr.data(), c0->nb_id.data(), c0->N, srcs, n_src, P, mode,
                       mp->owner.data());
  mp->parts.reset(new spf_mplan::Part[P]);
  mp->n_parts = P;
  for (uint32_t i = 0; i < n_src; ++i) {
    spf_mplan::Part& p = mp->parts[mp->owner[i]];
    mp->row[i] = (uint32_t)p.req.size();
    p.req.push_back(i);
  }
  const uint32_t pitch = c0->pitch;
  const size_t lab = (flags & SPF_FLAG_DIST64) ? 2 : 1;
  for (uint32_t r = 0; r < P; ++r) {
    spf_mplan::Part& p = mp->parts[r];
    if (p.req.empty()) continue;
    spf_ctx* c = m->members[r];
    std::vector<uint32_t> ps(p.req.size());
    for (size_t t = 0; t < ps.size(); ++t) ps[t] = srcs[p.req[t]];
    spf_status st = spf_plan_create(c, ps.data(), (uint32_t)ps.size(), flags, &p.plan);
    if (st != SPF_OK) return member_fail(m, r, st);
    p.nh_off.resize(ps.size());
    p.words.resize(ps.size());
    spf_plan_nh_layout(p.plan, p.nh_off.data(), p.words.data());
    M_HIP(m, hipSetDevice(c->device));
    M_HIP(m, p.dist.alloc(ps.size() * pitch * lab));
    M_HIP(m, p.nh.alloc(std::max<uint64_t>(spf_plan_nh_words(p.plan), 1)));
    M_HIP(m, p.dig.alloc(ps.size()));
  }
  *out = mp.release();
  return SPF_OK;
}

void spf_mplan_destroy(spf_mplan* mp) { delete mp; }

uint32_t spf_mplan_partition(const spf_mplan* mp) { return mp ? mp->mode : 0; }

spf_status spf_mplan_owner(const spf_mplan* mp, uint32_t i, uint32_t* member, uint32_t* row) {
  if (!mp || i >= mp->n_src) return SPF_E_INVALID;
  if (member) *member = mp->owner[i];
  if (row) *row = mp->row[i];
  return SPF_OK;
}

spf_status spf_mplan_shard(spf_mplan* mp, uint32_t member, uint32_t* n_src, spf_plan** plan,
                           void** d_dist, uint32_t** d_nh) {
  if (!mp || member >= mp->n_parts) return SPF_E_INVALID;
  spf_mplan::Part& p = mp->parts[member];
  if (n_src) *n_src = (uint32_t)p.req.size();
  if (plan) *plan = p.plan;
  if (d_dist) *d_dist = p.dist.p;
  if (d_nh) *d_nh = p.nh.p;
  return SPF_OK;
}

spf_status spf_mplan_set_graphs(spf_mplan* mp, int enable) {
  if (!mp) return SPF_E_INVALID;
  mp->graphs = enable != 0;
  return SPF_OK;
}

namespace {

// enqueue threads wanted: on when asked, or -- automatically -- when the
// members with work sit on two or more distinct devices (members of one
// device share its stream: nothing to overlap)
bool want_threads(const spf_mplan* mp) {
  if (mp->threads_mode >= 0) return mp->threads_mode == 1;
  std::vector<int> devs;
  for (uint32_t i = 0; i < mp->n_parts; ++i)
    if (mp->parts[i].plan) devs.push_back(mp->m->members[i]->device);
  std::sort(devs.begin(), devs.end());
  return std::unique(devs.begin(), devs.end()) - devs.begin() > 1;
}

void enqueue_worker(spf_mplan* mp, uint32_t i) {
  spf_mplan::Pool& P = *mp->pool;
  uint64_t seen = 0;
  for (;;) {
    // spin briefly (back-to-back executes), then sleep until the next one
    uint64_t g = P.gen.load(std::memory_order_acquire);
    for (int k = 0; g == seen && k < 20000 && !P.stop.load(std::memory_order_relaxed); ++k) {
      __builtin_ia32_pause();
      g = P.gen.load(std::memory_order_acquire);
    }
    if (g == seen) {
      std::unique_lock<std::mutex> lk(P.mu);
      P.cv.wait(lk, [&] { return P.stop || P.gen.load(std::memory_order_acquire) != seen; });
      if (P.stop) return;
      g = P.gen.load(std::memory_order_acquire);
    }
    if (P.stop) return;
    seen = g;
    if (mp->parts[i].plan) {
      P.st[i] = run_part(mp, i);
      mp->enq_ns[i] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now() - P.t0).count();
    }
    P.pending.fetch_sub(1, std::memory_order_acq_rel);
  }
}

}  // namespace

spf_status spf_mplan_set_enqueue_threads(spf_mplan* mp, int mode) {
  if (!mp || mode < -1 || mode > 1) return SPF_E_INVALID;
  mp->threads_mode = mode;
  if (!want_threads(mp)) mp->stop_pool();
  return SPF_OK;
}

spf_status spf_mplan_enqueue_ns(const spf_mplan* mp, uint64_t* out, uint32_t n, int* threaded) {
  if (!mp || (n && !out)) return SPF_E_INVALID;
  for (uint32_t i = 0; i < n && i < mp->n_parts; ++i) out[i] = i < mp->enq_ns.size() ? mp->enq_ns[i] : 0;
  if (threaded) *threaded = mp->pool ? 1 : 0;
  return SPF_OK;
}

spf_status spf_mplan_execute(spf_mplan* mp) {
  if (!mp) return mfail(nullptr, SPF_E_INVALID, "spf_mplan_execute: NULL plan");
  mp->enq_ns.assign(mp->n_parts, 0);
  const auto t0 = std::chrono::steady_clock::now();
  if (want_threads(mp)) {
    if (!mp->pool) {
      mp->pool = std::make_unique<spf_mplan::Pool>();
      mp->pool->st.assign(mp->n_parts, SPF_OK);
      for (uint32_t i = 0; i < mp->n_parts; ++i) mp->pool->th.emplace_back(enqueue_worker, mp, i);
    }
    spf_mplan::Pool& P = *mp->pool;
    P.t0 = t0;
    P.pending.store(mp->n_parts, std::memory_order_release);
    {
      std::lock_guard<std::mutex> lk(P.mu);
      P.gen.fetch_add(1, std::memory_order_acq_rel);
    }
    P.cv.notify_all();
    while (P.pending.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    for (uint32_t i = 0; i < mp->n_parts; ++i)
      if (P.st[i] != SPF_OK) return P.st[i];
  } else {
    for (uint32_t i = 0; i < mp->n_parts; ++i) {
      if (!mp->parts[i].plan) continue;
      const spf_status st = run_part(mp, i);
      if (st != SPF_OK) return st;
      mp->enq_ns[i] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now() - t0).count();
    }
  }
  if (mp->timing_cap) ++mp->timing_n;
  ++mp->executes;
  return SPF_OK;
}

spf_status spf_mplan_synchronize(spf_mplan* mp) {
  if (!mp) return mfail(nullptr, SPF_E_INVALID, "spf_mplan_synchronize: NULL plan");
  spf_mctx* m = mp->m;
  for (uint32_t i = 0; i < mp->n_parts; ++i) {
    if (!mp->parts[i].plan) continue;
    M_HIP(m, hipSetDevice(m->members[i]->device));
    M_HIP(m, hipStreamSynchronize(m->exec[i]));
    const spf_status st = spf_device_check(m->members[i]);
    if (st != SPF_OK) return member_fail(m, i, st);
  }
  return SPF_OK;
}

spf_status spf_mplan_digest(spf_mplan* mp, uint64_t* out) {
  if (!mp || !out) return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_digest: NULL argument");
  spf_mctx* m = mp->m;
  std::vector<std::vector<uint64_t>> h(mp->n_parts);
  for (uint32_t i = 0; i < mp->n_parts; ++i) {
    spf_mplan::Part& p = mp->parts[i];
    if (!p.plan) continue;
    M_HIP(m, hipSetDevice(m->members[i]->device));
    spf_status st = spf_plan_digest(p.plan, p.dist.p, p.nh.p, reinterpret_cast<uint64_t*>(p.dig.p),
                                    m->exec[i]);
    if (st != SPF_OK) return member_fail(m, i, st);
    h[i].resize(p.req.size());
    M_HIP(m, hipMemcpyAsync(h[i].data(), p.dig.p, 8 * p.req.size(), hipMemcpyDeviceToHost, m->exec[i]));
  }
  const spf_status st = spf_mplan_synchronize(mp);
  if (st != SPF_OK) return st;
  for (uint32_t i = 0; i < mp->n_parts; ++i)
    for (size_t t = 0; t < mp->parts[i].req.size(); ++t) out[mp->parts[i].req[t]] = h[i][t];
  return SPF_OK;
}

spf_status spf_mplan_read(spf_mplan* mp, uint32_t i, void* dist, uint32_t* nh) {
  if (!mp || i >= mp->n_src) return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_read: bad argument");
  spf_mctx* m = mp->m;
  const uint32_t r = mp->owner[i], row = mp->row[i];
  spf_mplan::Part& p = mp->parts[r];
  spf_ctx* c = m->members[r];
  const size_t lab = (mp->flags & SPF_FLAG_DIST64) ? 8 : 4;
  M_HIP(m, hipSetDevice(c->device));
  if (dist)
    M_HIP(m, hipMemcpyAsync(dist, reinterpret_cast<const uint8_t*>(p.dist.p) + (size_t)row * c->pitch * lab,
                            (size_t)c->N * lab, hipMemcpyDeviceToHost, m->exec[r]));
  const uint64_t words = (uint64_t)p.words[row] * (c->pitch / 32);
  if (nh && words)
    M_HIP(m, hipMemcpyAsync(nh, p.nh.p + p.nh_off[row], 4 * words, hipMemcpyDeviceToHost, m->exec[r]));
  M_HIP(m, hipStreamSynchronize(m->exec[r]));
  return SPF_OK;
}

spf_status spf_mplan_preds(spf_mplan* mp, uint32_t i, uint32_t* pred_ptr, uint32_t* pred_edge,
                           uint32_t cap, uint32_t* n_preds) {
  if (!mp || i >= mp->n_src || !pred_ptr || !n_preds)
    return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_preds: bad argument");
  spf_mctx* m = mp->m;
  const uint32_t r = mp->owner[i];
  spf_ctx* c = m->members[r];
  const bool hop = (mp->flags & SPF_FLAG_HOP_COUNT) != 0;
  if ((mp->flags & SPF_FLAG_DIST64) || (!hop && c->nonpos))
    return mfail(m, SPF_E_UNSUPPORTED, "spf_mplan_preds: zero / negative metrics and u64 rows "
                                       "order pathLinks by pop rank (spf_solve_exact)");
  const uint32_t* d_row = mp->parts[r].dist.p + (size_t)mp->row[i] * c->pitch;
  const spf_status st = preds_from_row(c, mp->srcs[i], hop, nullptr, d_row, pred_ptr, pred_edge,
                                       cap, n_preds, m->exec[r]);
  return st == SPF_OK ? SPF_OK : member_fail(m, r, st);
}

// ---- route selection over the resident pass ------------------------------
namespace {

// Every member's table of each resident row's (and bitmap set's) device
// address, plus the sets, on that member's device.  Rows of another device
// are read through peer access (xGMI): enabled here once, required for LFA
// (neighbours' rows) when the members span devices.
// Streams a route call has queued work on (copies into the caller's or the
// call's own host memory, timing events): on any early return they are
// drained and the events destroyed before that memory goes away.
struct IssuedGuard {
  spf_mctx* m;
  std::vector<uint32_t> members;
  std::vector<hipEvent_t>* ev = nullptr;
  ~IssuedGuard() {
    for (uint32_t r : members) {
      (void)hipSetDevice(m->members[r]->device);
      (void)hipStreamSynchronize(m->exec[r]);
    }
    if (ev)
      for (hipEvent_t e : *ev)
        if (e) (void)hipEventDestroy(e);
  }
};

spf_status route_prepare(spf_mplan* mp, const uint32_t* set_ptr, const uint32_t* set_nodes,
                         uint32_t n_sets, bool lfa, const uint64_t* link_hash, uint32_t n_links,
                         const uint32_t* me_req, uint32_t n_me) {
  spf_mctx* m = mp->m;
  spf_ctx* c0 = m->members[0];
  const uint32_t N = c0->N;
  if (mp->flags & SPF_FLAG_DIST64)
    return mfail(m, SPF_E_UNSUPPORTED, "route selection reads u32 rows (SPF_FLAG_DIST64 plan)");
  if (mp->flags & SPF_FLAG_HOP_COUNT)
    return mfail(m, SPF_E_UNSUPPORTED, "route selection needs link-metric rows (useLinkMetric)");
  for (uint32_t i = 0; i < set_ptr[n_sets]; ++i)
    if (set_nodes[i] >= N) return mfail(m, SPF_E_INVALID, "set member %u out of range", set_nodes[i]);
  if (mp->peer < 0) {
    mp->peer = 1;
    for (uint32_t a = 0; a < mp->n_parts; ++a)
      for (uint32_t b = 0; b < mp->n_parts; ++b) {
        const int da = m->members[a]->device, db = m->members[b]->device;
        if (da == db) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, da, db) != hipSuccess || !can) {
          mp->peer = 0;
          continue;
        }
        M_HIP(m, hipSetDevice(da));
        const hipError_t e = hipDeviceEnablePeerAccess(db, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) mp->peer = 0;
        (void)hipGetLastError();
      }
  }
  bool stale = false;
  for (uint32_t r = 0; r < mp->n_parts; ++r) stale |= mp->parts[r].plan && mp->parts[r].r_epoch != mp->executes;
  std::vector<unsigned long long>& rowp = mp->h_rowp;
  std::vector<unsigned long long>& nhp = mp->h_nhp;
  std::vector<int> dev_of(N, -1);
  if (stale) {  // no upload of the old tables may still be reading them
    for (uint32_t r = 0; r < mp->n_parts; ++r)
      if (mp->parts[r].plan) {
        M_HIP(m, hipSetDevice(m->members[r]->device));
        M_HIP(m, hipStreamSynchronize(m->exec[r]));
      }
    rowp.assign(N, 0);
    nhp.assign(N, 0);
    // the members' u8 row copies (the BFS's narrow rows, closure order) are
    // exact distances when every metric is 1 and no row reached 254: the
    // records kernel's LFA then loads 4 bytes for 4 destinations instead of
    // 16 (it is bound by HBM bytes: 3.94 -> 3.77 ms on fabric_full,
    // profiles/r06_routes/u8lfa).  SPF_ROUTE_U8=0: u32 loads (A/B)
    mp->h_nrowp.clear();
    const char* ue = std::getenv("SPF_ROUTE_U8");
    bool u8 = c0->unit && !(ue && ue[0] == '0');
    for (uint32_t r = 0; r < mp->n_parts && u8; ++r) {
      const spf_plan* pl = mp->parts[r].plan;
      if (!pl) continue;
      u8 = pl->narrow && pl->sliced && !pl->sdirect && !pl->expand && pl->d_Dn.p && pl->d_maxd.p;
      if (!u8) break;
      uint32_t md = ~0u;
      M_HIP(m, hipSetDevice(m->members[r]->device));
      M_HIP(m, hipMemcpy(&md, pl->d_maxd.p, 4, hipMemcpyDeviceToHost));
      u8 = md < 254;
    }
    if (u8) {
      mp->h_nrowp.assign(N, 0);
      for (uint32_t r = 0; r < mp->n_parts; ++r) {
        const spf_plan* pl = mp->parts[r].plan;
        if (!pl) continue;
        const uint32_t np = m->members[r]->npitch;
        for (size_t ci = 0; ci < pl->closure.size(); ++ci)
          mp->h_nrowp[pl->closure[ci]] = (unsigned long long)(uintptr_t)(pl->d_Dn.p + ci * np);
      }
    }
  }
  for (uint32_t i = 0; i < mp->n_src; ++i) {
    const uint32_t v = mp->srcs[i], r = mp->owner[i], row = mp->row[i];
    const spf_mplan::Part& p = mp->parts[r];
    if (stale) {
      rowp[v] = (unsigned long long)(uintptr_t)(p.dist.p + (size_t)row * c0->pitch);
      nhp[v] = (unsigned long long)(uintptr_t)(p.nh.p + p.nh_off[row]);
    }
    dev_of[v] = m->members[r]->device;
  }
  if (lfa) {
    // LFA reads every neighbour's row: a partial plan without one of them
    // would silently drop that neighbour's LFA candidates
    for (uint32_t t = 0; t < n_me; ++t) {
      const uint32_t v = mp->srcs[me_req[t]];
      for (uint32_t e = c0->nb_ptr[v]; e < c0->nb_ptr[v + 1]; ++e)
        if (!rowp[c0->nb_id[e]])
          return mfail(m, SPF_E_UNSUPPORTED,
                       "LFA route selection for node %u needs its neighbour %u resident in the plan",
                       v, c0->nb_id[e]);
    }
  }
  if (lfa && !mp->peer) {
    // members on distinct devices without peer access: every neighbour of a
    // member's me must then live on that member's device
    for (uint32_t i = 0; i < mp->n_src; ++i) {
      const uint32_t v = mp->srcs[i];
      for (uint32_t e = c0->nb_ptr[v]; e < c0->nb_ptr[v + 1]; ++e)
        if (dev_of[c0->nb_id[e]] != dev_of[v])
          return mfail(m, SPF_E_UNSUPPORTED, "LFA route selection across devices needs peer access");
    }
  }
  for (uint32_t r = 0; r < mp->n_parts; ++r) {
    spf_mplan::Part& p = mp->parts[r];
    if (!p.plan) continue;
    spf_ctx* c = m->members[r];
    M_HIP(m, hipSetDevice(c->device));
    const hipStream_t s = m->exec[r];
    if (p.r_epoch != mp->executes) {
      M_HIP(m, p.rowp.upload(rowp.data(), N, s));
      M_HIP(m, p.nhp.upload(nhp.data(), N, s));
      if (!mp->h_nrowp.empty()) M_HIP(m, p.nrowp.upload(mp->h_nrowp.data(), N, s));
      p.r_epoch = mp->executes;
    }
    // the sets and link hashes of a call are usually the previous call's
    // (every route build of a node list): uploaded only when they changed
    const uint32_t n_mem = std::max<uint32_t>(1, set_ptr[n_sets]);
    auto same = [](const auto& v, const auto* x, size_t n) {
      return v.size() == n && std::equal(v.begin(), v.end(), x);
    };
    const bool up = !same(p.h_rsp, set_ptr, n_sets + 1) || !same(p.h_rsn, set_nodes, n_mem) ||
                    (link_hash && !same(p.h_lh, link_hash, std::max<uint32_t>(1, n_links)));
    if (up) M_HIP(m, hipStreamSynchronize(s));  // no upload still reads the host copies
    if (!same(p.h_rsp, set_ptr, n_sets + 1)) {
      p.h_rsp.assign(set_ptr, set_ptr + n_sets + 1);
      M_HIP(m, p.rsp.upload(p.h_rsp.data(), n_sets + 1, s));
    }
    if (!same(p.h_rsn, set_nodes, n_mem)) {
      p.h_rsn.assign(set_nodes, set_nodes + n_mem);
      M_HIP(m, p.rsn.upload(p.h_rsn.data(), n_mem, s));
    }
    if (link_hash && !same(p.h_lh, link_hash, std::max<uint32_t>(1, n_links))) {
      p.h_lh.assign(link_hash, link_hash + std::max<uint32_t>(1, n_links));
      M_HIP(m, p.lh.upload(reinterpret_cast<const unsigned long long*>(p.h_lh.data()), p.h_lh.size(), s));
    }
    // (uploads read the host copies, which outlive the call)
  }
  return SPF_OK;
}

}  // namespace

spf_status spf_mplan_route_digests(spf_mplan* mp, const uint32_t* me_req, uint32_t n_me,
                                   const uint32_t* set_ptr, const uint32_t* set_nodes, uint32_t n_sets,
                                   uint32_t flags, const uint64_t* link_hash, uint32_t n_links,
                                   uint64_t* digests, double* kernel_ms) {
  if (!mp || (n_me && (!me_req || !digests)) || !set_ptr || !link_hash)
    return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_route_digests: NULL argument");
  spf_mctx* m = mp->m;
  spf_ctx* c0 = m->members[0];
  for (uint32_t t = 0; t < n_me; ++t)
    if (me_req[t] >= mp->n_src) return mfail(m, SPF_E_INVALID, "me %u is not a request index", me_req[t]);
  for (uint32_t e = 0; e < c0->E; ++e)
    if (c0->link[e] >= n_links) return mfail(m, SPF_E_INVALID, "link_hash shorter than the link ids");
  const bool lfa = (flags & SPF_ROUTE_LFA) != 0;
  if (const spf_status st = route_prepare(mp, set_ptr, set_nodes, n_sets, lfa, link_hash, n_links,
                                         me_req, n_me);
      st != SPF_OK)
    return st;
  std::vector<std::vector<uint32_t>> mine(mp->n_parts), slot(mp->n_parts);
  for (uint32_t t = 0; t < n_me; ++t) {
    const uint32_t r = mp->owner[me_req[t]];
    mine[r].push_back(mp->srcs[me_req[t]]);
    slot[r].push_back(t);
  }
  std::vector<hipEvent_t> ev(2 * mp->n_parts, nullptr);
  std::vector<std::vector<uint64_t>> got(mp->n_parts);
  IssuedGuard guard{m, {}, &ev};  // declared after got: drains before got is freed
  for (uint32_t r = 0; r < mp->n_parts; ++r) {
    spf_mplan::Part& p = mp->parts[r];
    if (mine[r].empty()) continue;
    spf_ctx* c = m->members[r];
    M_HIP(m, hipSetDevice(c->device));
    guard.members.push_back(r);
    const hipStream_t s = m->exec[r];
    const uint32_t n = (uint32_t)mine[r].size();
    M_HIP(m, p.rme.upload(mine[r].data(), n, s));
    M_HIP(m, p.rdig.alloc(n));
    M_HIP(m, hipMemsetAsync(p.rdig.p, 0, 8ull * n, s));
    if (kernel_ms) {
      M_HIP(m, hipEventCreate(&ev[2 * r]));
      M_HIP(m, hipEventCreate(&ev[2 * r + 1]));
      M_HIP(m, hipEventRecord(ev[2 * r], s));
    }
    const spf_status st = launch_route_sets(c, p.rowp.p, p.nhp.p, p.rme.p, n, p.rsp.p, p.rsn.p, n_sets,
                                            lfa, p.lh.p, p.rdig.p, nullptr, nullptr, nullptr, nullptr, s);
    // (u8 LFA loads only for the records kernel: the digest kernel is
    // VALU-bound and the byte unpacking made it slower, 2.33 -> 2.42 ms)
    if (st != SPF_OK) return member_fail(m, r, st);
    if (kernel_ms) M_HIP(m, hipEventRecord(ev[2 * r + 1], s));
    got[r].resize(n);
    M_HIP(m, hipMemcpyAsync(got[r].data(), p.rdig.p, 8ull * n, hipMemcpyDeviceToHost, s));
  }
  double worst = 0;
  for (uint32_t r = 0; r < mp->n_parts; ++r) {
    if (mine[r].empty()) continue;
    M_HIP(m, hipSetDevice(m->members[r]->device));
    M_HIP(m, hipStreamSynchronize(m->exec[r]));
    if (kernel_ms) {
      float t = 0;
      M_HIP(m, hipEventElapsedTime(&t, ev[2 * r], ev[2 * r + 1]));
      worst = std::max(worst, (double)t);
    }
    for (size_t q = 0; q < got[r].size(); ++q) digests[slot[r][q]] = got[r][q];
  }
  if (kernel_ms) *kernel_ms = worst;
  return SPF_OK;
}

spf_status spf_mplan_route_records(spf_mplan* mp, const uint32_t* me_req, uint32_t n_me,
                                   const uint32_t* set_ptr, const uint32_t* set_nodes, uint32_t n_sets,
                                   uint32_t flags, uint64_t* n_records, double* kernel_ms) {
  if (!mp || (n_me && !me_req) || !set_ptr)
    return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_route_records: NULL argument");
  spf_mctx* m = mp->m;
  spf_ctx* c0 = m->members[0];
  for (uint32_t t = 0; t < n_me; ++t)
    if (me_req[t] >= mp->n_src) return mfail(m, SPF_E_INVALID, "me %u is not a request index", me_req[t]);
  const bool lfa = (flags & SPF_ROUTE_LFA) != 0;
  if (const spf_status st = route_prepare(mp, set_ptr, set_nodes, n_sets, lfa, nullptr, 0, me_req, n_me);
      st != SPF_OK)
    return st;
  mp->db_loc.assign(n_me, {0u, 0u});
  mp->db_sets = n_sets;
  std::vector<std::vector<uint32_t>> mine(mp->n_parts);
  for (uint32_t t = 0; t < n_me; ++t) {
    const uint32_t r = mp->owner[me_req[t]];
    mp->db_loc[t] = {r, (uint32_t)mine[r].size()};
    mine[r].push_back(mp->srcs[me_req[t]]);
  }
  // me's region: one [deg(me)][ts] tile per chunk of ts sets (route_quads_kernel<kRsDb>)
  const uint64_t ts = route_db_tile_sets();
  const uint64_t tiles = ((uint64_t)n_sets + ts - 1) / ts * ts;
  std::vector<hipEvent_t> ev(2 * mp->n_parts, nullptr);
  std::vector<std::vector<uint32_t>> fl(mp->n_parts);
  IssuedGuard guard{m, {}, &ev};  // declared after fl: drains before it is freed
  for (uint32_t r = 0; r < mp->n_parts; ++r) {
    spf_mplan::Part& p = mp->parts[r];
    if (mine[r].empty()) continue;
    spf_ctx* c = m->members[r];
    M_HIP(m, hipSetDevice(c->device));
    guard.members.push_back(r);
    const hipStream_t s = m->exec[r];
    const uint32_t n = (uint32_t)mine[r].size();
    if (p.db_me != mine[r] || p.db_tiles != tiles) {
      M_HIP(m, hipStreamSynchronize(s));  // no queued upload still reads the host tables
      p.db_me = mine[r];
      p.db_tiles = tiles;
      p.h_dbbase.assign(n, 0);
      unsigned long long tot = 0;
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t v = mine[r][k];
        const uint64_t region = tiles * (c0->row_ptr[v + 1] - c0->row_ptr[v]);
        if (region >= (1ull << 32))
          return mfail(m, SPF_E_UNSUPPORTED, "route database of node %u: %llu record slots (2^32 max)", v,
                       (unsigned long long)region);
        p.h_dbbase[k] = tot;
        tot += region;
      }
      M_HIP(m, p.dbpool.alloc(std::max<unsigned long long>(tot, 1)));
      M_HIP(m, p.dbbase.upload(p.h_dbbase.data(), n, s));
    }
    M_HIP(m, p.rme.upload(p.db_me.data(), n, s));
    M_HIP(m, p.dbhdr.alloc(std::max<size_t>(1, (size_t)n * n_sets)));
    M_HIP(m, p.dbcnt.alloc(n));
    M_HIP(m, p.dbflags.alloc(1));
    M_HIP(m, hipMemsetAsync(p.dbcnt.p, 0, 4ull * n, s));
    M_HIP(m, hipMemsetAsync(p.dbflags.p, 0, 4, s));
    if (kernel_ms) {
      M_HIP(m, hipEventCreate(&ev[2 * r]));
      M_HIP(m, hipEventCreate(&ev[2 * r + 1]));
      M_HIP(m, hipEventRecord(ev[2 * r], s));
    }
    RouteDbOut db;
    db.hdr = p.dbhdr.p;
    db.pool = p.dbpool.p;
    db.base = p.dbbase.p;
    db.count = p.dbcnt.p;
    db.flags = p.dbflags.p;
    const spf_status st = launch_route_sets(c, p.rowp.p, p.nhp.p, p.rme.p, n, p.rsp.p, p.rsn.p, n_sets, lfa,
                                            nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, s, &db,
                                            mp->h_nrowp.empty() ? nullptr : p.nrowp.p);
    if (st != SPF_OK) return member_fail(m, r, st);
    if (kernel_ms) M_HIP(m, hipEventRecord(ev[2 * r + 1], s));
    fl[r].resize(n + 1);
    M_HIP(m, hipMemcpyAsync(fl[r].data(), p.dbcnt.p, 4ull * n, hipMemcpyDeviceToHost, s));
    M_HIP(m, hipMemcpyAsync(fl[r].data() + n, p.dbflags.p, 4, hipMemcpyDeviceToHost, s));
  }
  double worst = 0;
  uint64_t total = 0;
  for (uint32_t r = 0; r < mp->n_parts; ++r) {
    spf_mplan::Part& p = mp->parts[r];
    if (mine[r].empty()) continue;
    M_HIP(m, hipSetDevice(m->members[r]->device));
    M_HIP(m, hipStreamSynchronize(m->exec[r]));
    const uint32_t n = (uint32_t)mine[r].size();
    if (fl[r][n] & 2u) return mfail(m, SPF_E_UNSUPPORTED, "a next-hop metric exceeds 2^32 - 1");
    p.h_dbcnt.assign(fl[r].begin(), fl[r].begin() + n);
    for (uint32_t k = 0; k < n; ++k) total += p.h_dbcnt[k];
    if (kernel_ms) {
      float t = 0;
      M_HIP(m, hipEventElapsedTime(&t, ev[2 * r], ev[2 * r + 1]));
      worst = std::max(worst, (double)t);
    }
  }
  if (n_records) *n_records = total;
  if (kernel_ms) *kernel_ms = worst;
  return SPF_OK;
}

spf_status spf_mplan_route_db(spf_mplan* mp, uint32_t t, uint64_t* hdr, uint64_t* rec, uint64_t cap,
                              uint64_t* n) {
  if (!mp || t >= mp->db_loc.size())
    return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_route_db: no such me (call spf_mplan_route_records)");
  spf_mctx* m = mp->m;
  const auto [r, k] = mp->db_loc[t];
  spf_mplan::Part& p = mp->parts[r];
  const uint32_t cnt = p.h_dbcnt[k];
  if (n) *n = cnt;
  if (!hdr && !rec) return SPF_OK;
  if (rec && cap < cnt)
    return mfail(m, SPF_E_NOMEM, "route db of %u records, room for %llu", cnt, (unsigned long long)cap);
  // the device headers and me's tiled region, compacted here: route p's
  // records contiguous from its header's offset, in set order
  const uint32_t S = mp->db_sets;
  std::vector<uint64_t> h(S);
  const uint32_t me = p.db_me[k];
  const uint64_t region = p.db_tiles * (mp->m->members[r]->row_ptr[me + 1] - mp->m->members[r]->row_ptr[me]);
  std::vector<uint64_t> tile(std::max<uint64_t>(region, 1));
  M_HIP(m, hipSetDevice(m->members[r]->device));
  const hipStream_t s = m->exec[r];
  if (S) M_HIP(m, hipMemcpyAsync(h.data(), p.dbhdr.p + (size_t)k * S, 8ull * S, hipMemcpyDeviceToHost, s));
  if (rec && region)
    M_HIP(m, hipMemcpyAsync(tile.data(), p.dbpool.p + p.h_dbbase[k], 8ull * region, hipMemcpyDeviceToHost, s));
  M_HIP(m, hipStreamSynchronize(s));
  uint64_t at = 0;
  for (uint32_t q = 0; q < S; ++q) {
    const uint64_t off = h[q] & 0xFFFFFFFFull, c = (h[q] >> 32) & 0xFFFFull, stride = h[q] >> 48;
    if (rec)
      for (uint64_t j = 0; j < c; ++j) rec[at + j] = tile[off + j * stride];
    if (hdr) hdr[q] = at | (c << 32);
    at += c;
  }
  return SPF_OK;
}

spf_status spf_mplan_routes(spf_mplan* mp, uint32_t me_req, const uint32_t* set_ptr,
                            const uint32_t* set_nodes, uint32_t n_sets, uint32_t flags,
                            uint64_t* min_metric, uint32_t* nh_count, uint32_t* nh_edge,
                            uint64_t* nh_metric) {
  if (!mp || !set_ptr || !min_metric || !nh_count || !nh_edge || !nh_metric)
    return mfail(mp ? mp->m : nullptr, SPF_E_INVALID, "spf_mplan_routes: NULL argument");
  spf_mctx* m = mp->m;
  if (me_req >= mp->n_src) return mfail(m, SPF_E_INVALID, "me %u is not a request index", me_req);
  const bool lfa = (flags & SPF_ROUTE_LFA) != 0;
  if (const spf_status st = route_prepare(mp, set_ptr, set_nodes, n_sets, lfa, nullptr, 0, &me_req, 1);
      st != SPF_OK)
    return st;
  const uint32_t r = mp->owner[me_req];
  spf_mplan::Part& p = mp->parts[r];
  spf_ctx* c = m->members[r];
  const uint32_t me = mp->srcs[me_req];
  const uint32_t deg = c->row_ptr[me + 1] - c->row_ptr[me];
  const size_t cap = (size_t)n_sets * std::max<uint32_t>(1, deg);
  M_HIP(m, hipSetDevice(c->device));
  const hipStream_t s = m->exec[r];
  IssuedGuard guard{m, {r}};  // &me and the caller's outputs outlive every queued copy
  M_HIP(m, p.rme.upload(&me, 1, s));
  M_HIP(m, p.rmin.alloc(std::max<uint32_t>(1, n_sets)));
  M_HIP(m, p.rcnt.alloc(std::max<uint32_t>(1, n_sets)));
  M_HIP(m, p.redge.alloc(cap));
  M_HIP(m, p.rmetric.alloc(cap));
  const spf_status st = launch_route_sets(c, p.rowp.p, p.nhp.p, p.rme.p, 1, p.rsp.p, p.rsn.p, n_sets, lfa,
                                          nullptr, nullptr, reinterpret_cast<uint64_t*>(p.rmin.p),
                                          p.rcnt.p, p.redge.p, reinterpret_cast<uint64_t*>(p.rmetric.p), s);
  if (st != SPF_OK) return member_fail(m, r, st);
  if (n_sets) {
    M_HIP(m, hipMemcpyAsync(min_metric, p.rmin.p, 8ull * n_sets, hipMemcpyDeviceToHost, s));
    M_HIP(m, hipMemcpyAsync(nh_count, p.rcnt.p, 4ull * n_sets, hipMemcpyDeviceToHost, s));
    if (deg) {
      M_HIP(m, hipMemcpyAsync(nh_edge, p.redge.p, 4ull * cap, hipMemcpyDeviceToHost, s));
      M_HIP(m, hipMemcpyAsync(nh_metric, p.rmetric.p, 8ull * cap, hipMemcpyDeviceToHost, s));
    }
  }
  M_HIP(m, hipStreamSynchronize(s));
  return SPF_OK;
}

uint32_t spf_mplan_closure_rows(const spf_mplan* mp, uint32_t member) {
  if (!mp || member >= mp->n_parts || !mp->parts[member].plan) return 0;
  return spf_plan_closure_rows(mp->parts[member].plan);
}

spf_status spf_mplan_enable_timing(spf_mplan* mp, uint32_t max_executes) {
  if (!mp) return SPF_E_INVALID;
  spf_mctx* m = mp->m;
  for (uint32_t i = 0; i < mp->n_parts; ++i) {
    spf_mplan::Part& p = mp->parts[i];
    if (!p.plan) continue;
    M_HIP(m, hipSetDevice(m->members[i]->device));
    for (hipEvent_t e : p.ev) (void)hipEventDestroy(e);
    p.ev.assign(2ull * max_executes, nullptr);
    for (auto& e : p.ev) M_HIP(m, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  }
  mp->timing_cap = max_executes;
  mp->timing_n = 0;
  return SPF_OK;
}

// per member: summed milliseconds of its executes (start to end on its
// stream), and the number of executes
spf_status spf_mplan_timing(spf_mplan* mp, double* ms, uint32_t* n) {
  if (!mp || !mp->timing_cap || !ms) return SPF_E_STATE;
  spf_mctx* m = mp->m;
  const uint32_t cnt = std::min(mp->timing_n, mp->timing_cap);
  for (uint32_t i = 0; i < mp->n_parts; ++i) {
    ms[i] = 0;
    spf_mplan::Part& p = mp->parts[i];
    if (!p.plan) continue;
    M_HIP(m, hipSetDevice(m->members[i]->device));
    for (uint32_t k = 0; k < cnt; ++k) {
      float t = 0;
      M_HIP(m, hipEventSynchronize(p.ev[2 * k + 1]));
      M_HIP(m, hipEventElapsedTime(&t, p.ev[2 * k], p.ev[2 * k + 1]));
      ms[i] += t;
    }
  }
  if (n) *n = cnt;
  mp->timing_n = 0;
  return SPF_OK;
}

}  // extern "C"
