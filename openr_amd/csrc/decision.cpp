// ============================================================================
//  decision.cpp -- the SpfSolver drop-in (openr_decision.h), in C++ over the
//  LinkState facade's C-ABI (openr_linkstate.h) and the engine's batched
//  route selection (openr_spf.h).
//
//  Reference: openr/decision/Decision.cpp SpfSolver::SpfSolverImpl
//  (createRouteForPrefix :389-555, buildRouteDb :556-722, selectBestRoutes /
//  runBestPathSelectionBgp / maybeFilterDrainedNodes :724-832,
//  selectBestPathsSpf / selectBestPathsKsp2 / addBestPaths :834-1080,
//  getMinCostNodes / getNextHopsWithMetric / getNextHopsThrift :1082-1305),
//  PrefixState (PrefixState.cpp:17-84), the best-route helpers of
//  openr/common/Util.{h,cpp} (selectBestPrefixMetrics :540-571,
//  selectBestNodeArea :1028-1040, MetricVectorUtils :1074-1217) and
//  createNextHop (Util.cpp:907-922).
//
//  One area: every SP_ECMP / IP prefix and node label of a build is one set
//  of ONE batched selection (spf_mplan_routes over a resident all-sources
//  pass, else spf_routes); the records are assembled here, routes whose
//  selections are equal share one record range.  Several areas, SR_MPLS and
//  KSP2_ED_ECMP prefixes take the reference's per-prefix walk over the
//  memoised SPF results / KSP2 paths of every area.
// ============================================================================
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <array>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "openr_decision.h"

namespace {

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

constexpr uint64_t kInf64 = ~0ull;

// folly::hash::hash_128_to_64: folly's std::hash<std::pair<A, B>> combiner
inline uint64_t folly_mix(uint64_t upper, uint64_t lower) {
  constexpr uint64_t kMul = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lower ^ upper) * kMul;
  a ^= a >> 47;
  uint64_t b = (upper ^ a) * kMul;
  b ^= b >> 47;
  return b * kMul;
}

using NodeArea = std::pair<std::string, std::string>;
struct NodeAreaHash {  // std::hash<NodeAndArea> with folly's pair specialisation
  size_t operator()(const NodeArea& k) const {
    return folly_mix(std::hash<std::string>()(k.first), std::hash<std::string>()(k.second));
  }
};

struct MetricEntity {
  int64_t type = 0, priority = 0;
  uint32_t op = DC_WIN_IF_PRESENT;
  bool tie_breaker = false;
  std::vector<int64_t> metric;
};
struct MetricVector {
  int32_t version = 0;
  std::vector<MetricEntity> metrics;
};

struct Entry {
  bool v4 = false, bgp = false;
  uint8_t ftype = DC_FWD_IP, falgo = DC_ALGO_SP_ECMP;
  std::optional<int32_t> prepend;
  std::optional<int64_t> min_nexthop;
  int32_t pp = 0, sp = 0, distance = 0;
  std::optional<MetricVector> mv;
  // the advertiser's name id in the LinkState with serial id_serial (a
  // cache: ids are stable per state)
  mutable uint64_t id_serial = 0;
  mutable uint32_t id = 0;
};
// PrefixEntries (openr/common/Types.h:24): the reference's container
using Entries = std::unordered_map<NodeArea, Entry, NodeAreaHash>;

bool mpls_label_valid(int64_t l) { return l >= 0 && l <= (1 << 20) - 1; }  // isMplsLabelValid

// ---- MetricVectorUtils (openr/common/Util.cpp:1074-1217) ----------------------
enum CmpResult { WINNER, TIE_WINNER, TIE, TIE_LOOSER, LOOSER, ERROR };
CmpResult inverse(CmpResult r) {
  switch (r) {
    case WINNER: return LOOSER;
    case TIE_WINNER: return TIE_LOOSER;
    case TIE_LOOSER: return TIE_WINNER;
    case LOOSER: return WINNER;
    default: return r;
  }
}
bool decisive(CmpResult r) { return r == WINNER || r == LOOSER || r == ERROR; }
CmpResult compare_metrics(const std::vector<int64_t>& l, const std::vector<int64_t>& r, bool tb) {
  if (l.size() != r.size()) return ERROR;
  for (size_t i = 0; i < l.size(); ++i) {
    if (l[i] > r[i]) return tb ? TIE_WINNER : WINNER;
    if (l[i] < r[i]) return tb ? TIE_LOOSER : LOOSER;
  }
  return TIE;
}
CmpResult result_for_loner(const MetricEntity& e) {
  if (e.op == DC_WIN_IF_PRESENT) return e.tie_breaker ? TIE_WINNER : WINNER;
  if (e.op == DC_WIN_IF_NOT_PRESENT) return e.tie_breaker ? TIE_LOOSER : LOOSER;
  return TIE;  // IGNORE_IF_NOT_PRESENT
}
// sortMetricVector (Util.cpp:1120-1133): decreasing priority, in place
void sort_metric_vector(MetricVector& mv) {
  auto& m = mv.metrics;
  bool sorted = true;
  for (size_t i = 0; i + 1 < m.size(); ++i) sorted &= m[i].priority >= m[i + 1].priority;
  if (!sorted)
    std::stable_sort(m.begin(), m.end(),
                     [](const MetricEntity& a, const MetricEntity& b) { return a.priority > b.priority; });
}
CmpResult compare_metric_vectors(MetricVector& l, MetricVector& r) {
  CmpResult result = TIE;
  auto upd = [&](CmpResult u) {
    if (decisive(u) || result == TIE) result = u;
  };
  if (l.version != r.version) return ERROR;
  sort_metric_vector(l);
  sort_metric_vector(r);
  const auto &L = l.metrics, &R = r.metrics;
  size_t i = 0, j = 0;
  while (!decisive(result) && i < L.size() && j < R.size()) {
    const MetricEntity &a = L[i], &b = R[j];
    if (a.type == b.type) {
      if (a.tie_breaker != b.tie_breaker) upd(ERROR);
      else upd(compare_metrics(a.metric, b.metric, a.tie_breaker));
      ++i;
      ++j;
    } else if (a.priority > b.priority) {
      upd(result_for_loner(a));
      ++i;
    } else if (a.priority < b.priority) {
      upd(inverse(result_for_loner(b)));
      ++j;
    } else {
      upd(ERROR);  // same priority, different types
    }
  }
  while (!decisive(result) && i < L.size()) upd(result_for_loner(L[i++]));
  while (!decisive(result) && j < R.size()) upd(inverse(result_for_loner(R[j++])));
  return result;
}

using EntryRef = const std::pair<const NodeArea, Entry>*;

// BestRouteSelectionResult (openr/decision/RibEntry.h); allNodeAreas is a std::set
struct BestRoute {
  bool success = false;
  std::vector<NodeArea> all;  // ascending
  std::optional<NodeArea> best;
  std::vector<EntryRef> refs;  // all[i]'s entry in the build's PrefixEntries (not cached)
  uint64_t gen = 0;            // the build that stored it (dc_solver::build_gen)
  bool has_node(const std::string& n) const {
    for (const auto& na : all)
      if (na.first == n) return true;
    return false;
  }
};

// A next hop under construction (createNextHop, Util.cpp:907-922)
struct NH {
  std::array<uint8_t, 16> addr{};
  uint8_t addr_len = 16;
  uint8_t action = DC_MPLS_NONE;
  int32_t metric = 0;
  int32_t swap = 0;
  std::vector<int32_t> push;
  std::optional<std::string> ifname, area, neighbor;
  auto key() const { return std::tie(addr, addr_len, action, metric, swap, push, ifname, area, neighbor); }
  bool operator<(const NH& o) const { return key() < o.key(); }
  bool operator==(const NH& o) const { return key() == o.key(); }
};
int32_t i32_metric(uint64_t m) { return (int32_t)(uint32_t)(m & 0xFFFFFFFFull); }

// me's side of one link of a LinkState (Link accessors, LinkState.h:82-175)
struct MyLink {
  uint32_t id;
  std::string nb;
  std::string ifname;
  uint64_t metric;
  int32_t adj_label;
  bool up;
  std::array<uint8_t, 4> v4;
  std::array<uint8_t, 16> v6;
};

}  // namespace

// ---- PrefixState ---------------------------------------------------------------
struct dc_prefix_state {
  std::unordered_map<std::string, Entries> prefixes;  // prefixes_ (PrefixState.h:69)
};

// ---- DecisionRouteDb -------------------------------------------------------------
struct dc_route_db {
  // the string table: NUL-terminated strings back to back in one arena, by
  // offset (a route's prefix is one append, not one allocation; the arena
  // stops growing when the build returns, so dc_route_db_string's pointers
  // stay valid)
  std::string arena;
  std::vector<uint32_t> str_off;
  std::unordered_map<std::string, uint32_t> sid;
  std::vector<dc_nexthop> nhs;
  std::vector<int32_t> labels;
  std::vector<uint32_t> uni;   // rows of 6
  std::vector<uint32_t> mpls;  // rows of 3
  // label -> its row in mpls: open addressing, (label, row + 1) per slot, row
  // + 1 == 0 empty (a build adds one per node label: no node allocation each)
  std::vector<std::pair<uint32_t, uint32_t>> lrow;
  size_t lrow_used = 0;

  void reserve_labels(size_t n) {
    size_t want = 64;
    while (want < 2 * (lrow_used + n)) want *= 2;
    if (want <= lrow.size()) return;
    std::vector<std::pair<uint32_t, uint32_t>> old(want, {0u, 0u});
    old.swap(lrow);
    for (const auto& kv : old)
      if (kv.second) lrow[lrow_slot(kv.first)] = kv;
  }
  size_t lrow_slot(uint32_t label) const {  // the label's slot, or the empty one ending its probe
    const size_t mask = lrow.size() - 1;
    size_t h = (size_t)(label * 0x9E3779B1u) & mask;
    while (lrow[h].second && lrow[h].first != label) h = (h + 1) & mask;
    return h;
  }

  uint32_t intern(const std::string& s) {
    auto it = sid.find(s);
    if (it != sid.end()) return it->second;
    const uint32_t id = push_unique(s);
    sid.emplace(s, id);
    return id;
  }
  uint32_t opt(const std::optional<std::string>& s) { return s ? intern(*s) : DC_NONE; }
  // a string no other record shares (a route's prefix): no lookup
  uint32_t push_unique(const std::string& s) {
    str_off.push_back((uint32_t)arena.size());
    arena.append(s.data(), s.size());
    arena.push_back('\0');
    return (uint32_t)str_off.size() - 1;
  }
  const char* str(uint32_t id) const { return arena.data() + str_off[id]; }
  // a next-hop set (sorted, unique) appended; returns [begin, end)
  std::pair<uint32_t, uint32_t> add_set(std::vector<NH>& set) {
    std::sort(set.begin(), set.end());
    set.erase(std::unique(set.begin(), set.end()), set.end());
    const uint32_t b = (uint32_t)nhs.size();
    for (const NH& h : set) {
      dc_nexthop r{};
      std::memcpy(r.address, h.addr.data(), 16);
      r.address_len = h.addr_len;
      r.mpls_action = h.action;
      r.metric = h.metric;
      r.swap_label = h.swap;
      r.n_push = (uint8_t)h.push.size();
      r.push_off = h.push.empty() ? 0u : (uint32_t)labels.size();
      labels.insert(labels.end(), h.push.begin(), h.push.end());
      r.ifname = opt(h.ifname);
      r.area = opt(h.area);
      r.neighbor = opt(h.neighbor);
      nhs.push_back(r);
    }
    return {b, (uint32_t)nhs.size()};
  }
  // POD records (the kernel path's next hops: no PUSH labels) as a set
  // records ordered as memcmp orders their bytes (the canonical order of a
  // route's next hops), compared inline as big-endian words: a label route
  // sorts its ~3 records per build, and memcmp calls were most of the
  // route assembly's time
  static int rec_cmp(const dc_nexthop& a, const dc_nexthop& b) {
    static_assert(sizeof(dc_nexthop) == 44, "five 8-byte words and a 4-byte one");
    const unsigned char* x = reinterpret_cast<const unsigned char*>(&a);
    const unsigned char* y = reinterpret_cast<const unsigned char*>(&b);
    for (int w = 0; w < 5; ++w) {
      uint64_t p, q;
      std::memcpy(&p, x + 8 * w, 8);
      std::memcpy(&q, y + 8 * w, 8);
      if (p != q) return __builtin_bswap64(p) < __builtin_bswap64(q) ? -1 : 1;
    }
    uint32_t p, q;
    std::memcpy(&p, x + 40, 4);
    std::memcpy(&q, y + 40, 4);
    if (p != q) return __builtin_bswap32(p) < __builtin_bswap32(q) ? -1 : 1;
    return 0;
  }
  std::pair<uint32_t, uint32_t> add_records(std::vector<dc_nexthop>& v) {
    auto lt = [](const dc_nexthop& a, const dc_nexthop& b) { return rec_cmp(a, b) < 0; };
    auto eq = [](const dc_nexthop& a, const dc_nexthop& b) { return rec_cmp(a, b) == 0; };
    if (v.size() <= 16) {  // insertion sort: a route's few records
      for (size_t i = 1; i < v.size(); ++i)
        for (size_t j = i; j > 0 && lt(v[j], v[j - 1]); --j) std::swap(v[j], v[j - 1]);
    } else {
      std::sort(v.begin(), v.end(), lt);
    }
    v.erase(std::unique(v.begin(), v.end(), eq), v.end());
    const uint32_t b = (uint32_t)nhs.size();
    nhs.insert(nhs.end(), v.begin(), v.end());
    return {b, (uint32_t)nhs.size()};
  }
  void add_unicast(const std::string& prefix, const NodeArea& best, bool dni,
                   std::pair<uint32_t, uint32_t> r) {
    uni.insert(uni.end(), {intern(prefix), intern(best.first), intern(best.second), (uint32_t)dni,
                           r.first, r.second});
  }
  // dict assignment, as the restatement's DecisionRouteDb (the reference
  // CHECKs that a label is added once, Decision.h:116-120)
  void add_mpls(int32_t label, std::pair<uint32_t, uint32_t> r) {
    reserve_labels(1);
    auto& slot = lrow[lrow_slot((uint32_t)label)];
    if (slot.second) {  // a later route for the label replaces the earlier one
      mpls[slot.second - 1 + 1] = r.first;
      mpls[slot.second - 1 + 2] = r.second;
      return;
    }
    slot = {(uint32_t)label, (uint32_t)mpls.size() + 1};
    ++lrow_used;
    mpls.insert(mpls.end(), {(uint32_t)label, r.first, r.second});
  }
};

// ---- SpfSolver ---------------------------------------------------------------------
namespace {

// one SPF result with a name-id index
struct SpfIdx {
  ls_spf_view v{};
  std::vector<int32_t> pos;  // name id -> entry, -1 absent
  int find(uint32_t id) const { return id < pos.size() ? pos[id] : -1; }
};

// per-LinkState caches that outlive a build while its flattened graph holds
struct GraphCache {
  uint64_t epoch = ~0ull;
  std::vector<uint32_t> csr_name, csr_of, row_ptr, link_id;
};

}  // namespace

// the single-area batched selection: one spf_mplan_routes / spf_routes call
// (kept by the solver: a build of the same shape resizes nothing)
struct Selection {
  uint32_t deg = 1;
  std::vector<uint64_t> mins, metric;
  std::vector<uint32_t> cnt, edge;
};

struct dc_solver {
  Selection sel;  // the last build's batched selection buffers
  std::string me;
  bool enable_v4 = false, lfa = false, bgp_dry_run = false, best_route_selection = false;
  std::string err;
  std::map<std::string, uint64_t> counters;
  std::map<int32_t, std::vector<NH>> static_mpls;  // staticMplsRoutes_
  std::unordered_map<std::string, BestRoute> best_cache;  // bestRoutesCache_
  uint64_t build_gen = 0;  // bumped per build: entries it did not store are swept
  std::unordered_map<ls_state*, GraphCache> graphs;
  // build cost by phase, ns since creation (dc_debug_phase_ns)
  uint64_t phase_ns[6] = {0, 0, 0, 0, 0, 0};

  void bump(const char* k) { ++counters[k]; }
};

namespace {

spf_status sfail(dc_solver* s, spf_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (s) s->err = buf;
  return st;
}

// One area of a build: its LinkState and the lookups the walk needs, filled lazily.
struct Area {
  std::string name;
  ls_state* ls = nullptr;
  uint64_t serial = 0;  // ls_serial
  uint32_t me_id = 0;
  std::vector<uint32_t> db_sid;  // name id -> route-db string id (+1; 0 = not yet)
  uint32_t area_sid = DC_NONE;
  std::unordered_map<uint32_t, std::unique_ptr<SpfIdx>> spf;  // name id -> SPF result
  bool links_done = false;
  std::vector<MyLink> links;  // linksFromNode(me), in its order
  bool labels_done = false;
  std::unordered_map<uint32_t, int32_t> labels;  // getAdjacencyDatabases(): node -> node label

  uint32_t id(const std::string& n) { return ls_name_id(ls, n.c_str()); }
  uint32_t id(const std::pair<const NodeArea, Entry>& kv) {  // cached in the entry
    const Entry& e = kv.second;
    if (e.id_serial != serial) {
      e.id = id(kv.first.first);
      e.id_serial = serial;
    }
    return e.id;
  }
  uint32_t sid(dc_route_db* db, uint32_t name_id, const std::string& name) {
    if (name_id >= db_sid.size()) db_sid.resize(std::max<size_t>(name_id + 1, 2 * db_sid.size()), 0);
    // (one table entry per name and build: no lookup among the other strings)
    if (!db_sid[name_id]) db_sid[name_id] = db->push_unique(name) + 1;
    return db_sid[name_id] - 1;
  }
  std::string name_of(uint32_t i) const { return ls_name(ls, i); }
};

struct Build {
  dc_solver* s;
  const std::string& me;
  std::vector<std::unique_ptr<Area>> areas;  // in the reference's map order
  std::unordered_map<std::string, Area*> by_name;
  dc_route_db* db;
  spf_status st = SPF_OK;

  bool ok() const { return st == SPF_OK; }
  Area* area_of(const std::string& name) {
    if (areas.size() == 1) return areas[0]->name == name ? areas[0].get() : nullptr;
    auto it = by_name.find(name);
    return it == by_name.end() ? nullptr : it->second;
  }
  spf_status ls_err(Area& a, spf_status code) {
    st = sfail(s, code, "LinkState of area %s: %s", a.name.c_str(), ls_last_error(a.ls));
    return st;
  }

  // getSpfResult(node) of an area (memoised by the LinkState; indexed here)
  const SpfIdx* spf(Area& a, uint32_t node) {
    auto it = a.spf.find(node);
    if (it != a.spf.end()) return it->second.get();
    auto x = std::make_unique<SpfIdx>();
    const spf_status code = ls_get_spf_metrics(a.ls, a.name_of(node).c_str(), 1, &x->v);
    if (code != SPF_OK) {
      ls_err(a, code);
      return nullptr;
    }
    uint32_t mx = 0;
    for (uint32_t i = 0; i < x->v.n; ++i) mx = std::max(mx, x->v.node[i] + 1);
    x->pos.assign(mx, -1);
    for (uint32_t i = 0; i < x->v.n; ++i) x->pos[x->v.node[i]] = (int32_t)i;
    return a.spf.emplace(node, std::move(x)).first->second.get();
  }

  const std::vector<MyLink>& links(Area& a) {
    if (a.links_done) return a.links;
    a.links_done = true;
    uint32_t n = 0;
    ls_links_from_node(a.ls, me.c_str(), nullptr, 0, &n);
    std::vector<uint32_t> ids(n);
    ls_links_from_node(a.ls, me.c_str(), ids.data(), n, &n);
    for (uint32_t id : ids) {
      ls_link_desc d{};
      if (ls_link_info(a.ls, id, &d) != SPF_OK) continue;
      const int side = d.node1 == a.me_id ? 0 : 1;
      MyLink l;
      l.id = id;
      l.nb = a.name_of(side ? d.node1 : d.node2);
      l.ifname = side ? d.if2 : d.if1;
      l.metric = side ? d.metric2 : d.metric1;
      l.adj_label = side ? d.adj_label2 : d.adj_label1;
      l.up = d.is_up != 0;
      std::memcpy(l.v4.data(), side ? d.nh_v4_2 : d.nh_v4_1, 4);
      std::memcpy(l.v6.data(), side ? d.nh_v6_2 : d.nh_v6_1, 16);
      a.links.push_back(std::move(l));
    }
    return a.links;
  }

  const std::unordered_map<uint32_t, int32_t>& labels(Area& a) {
    if (a.labels_done) return a.labels;
    a.labels_done = true;
    uint32_t n = 0;
    ls_adjacency_databases(a.ls, nullptr, nullptr, 0, &n);
    std::vector<uint32_t> ids(n);
    std::vector<int32_t> lab(n);
    ls_adjacency_databases(a.ls, ids.data(), lab.data(), n, &n);
    for (uint32_t i = 0; i < n; ++i) a.labels.emplace(ids[i], lab[i]);
    return a.labels;
  }

  NH link_nh(const MyLink& l, const Area& a, bool v4, uint64_t metric) const {
    NH h;
    if (v4) {
      std::copy(l.v4.begin(), l.v4.end(), h.addr.begin());
      h.addr_len = 4;
    } else {
      h.addr = l.v6;
      h.addr_len = 16;
    }
    h.ifname = l.ifname;
    h.metric = i32_metric(metric);
    h.area = a.name;
    h.neighbor = l.nb;
    return h;
  }

  // ---- best-route selection (Decision.cpp:724-832) ----
  std::optional<BestRoute> filter_drained(BestRoute r) {  // maybeFilterDrainedNodes :766-789
    auto is_drained = [&](size_t i, bool& bad) {
      const NodeArea& na = r.all[i];
      Area* a = area_of(na.second);
      if (!a) {  // areaLinkStates.at(area) throws
        st = sfail(s, SPF_E_INVALID, "advertiser %s in area %s, which has no LinkState",
                   na.first.c_str(), na.second.c_str());
        bad = true;
        return false;
      }
      return ls_is_node_overloaded_id(a->ls, a->id(*r.refs[i])) != 0;
    };
    bool any = false, bad = false;
    for (size_t i = 0; i < r.all.size() && !any; ++i) any = is_drained(i, bad);
    if (bad) return std::nullopt;
    if (!any) return r;
    std::vector<char> drained(r.all.size(), 0);
    for (size_t i = 0; i < r.all.size(); ++i) drained[i] = is_drained(i, bad);
    BestRoute f;
    f.success = r.success;
    f.best = r.best;
    for (size_t i = 0; i < r.all.size(); ++i)
      if (!drained[i]) {
        f.all.push_back(r.all[i]);
        f.refs.push_back(r.refs[i]);
      }
    // (the filtered copy keeps the unfiltered bestNodeArea: the reference
    // compares the copy's bestNodeArea with its source's)
    return f.all.empty() ? r : f;
  }

  std::optional<BestRoute> bgp_walk(const Entries& ents) {  // runBestPathSelectionBgp :791-832
    BestRoute ret;
    std::optional<MetricVector> best_v;
    std::vector<EntryRef> chosen;
    auto by_key = [](EntryRef a, EntryRef b) { return a->first < b->first; };
    auto set_all = [&]() {
      std::sort(chosen.begin(), chosen.end(), by_key);
      for (EntryRef x : chosen) ret.all.push_back(x->first);
      ret.refs = chosen;
    };
    for (const auto& kv : ents) {
      MetricVector mv = *kv.second.mv;  // the reference's entries are a copy (Decision.cpp:409)
      const CmpResult r = best_v ? compare_metric_vectors(mv, *best_v) : WINNER;
      if (r == WINNER) chosen.clear();
      if (r == WINNER || r == TIE_WINNER) {
        best_v = mv;
        ret.best = kv.first;
      }
      if (r == WINNER || r == TIE_WINNER || r == TIE_LOOSER) {
        chosen.push_back(&kv);
      } else if (r == TIE || r == ERROR) {
        set_all();
        return ret;  // success false: no route
      }
    }
    set_all();
    ret.success = true;
    return filter_drained(std::move(ret));
  }

  // `ret`: an empty result whose vectors may hold capacity (the cache slot's)
  std::optional<BestRoute> select_best(const Entries& ents, bool bgp, BestRoute ret = {}) {  // selectBestRoutes :728-748
    if (s->best_route_selection) {
      // selectBestPrefixMetrics (Util.h:540-571): best (pp, sp, -distance) from (0, 0, 0)
      std::tuple<int64_t, int64_t, int64_t> bt{0, 0, 0};
      for (const auto& kv : ents) {
        const Entry& e = kv.second;
        const std::tuple<int64_t, int64_t, int64_t> t{e.pp, e.sp, -(int64_t)e.distance};
        if (t < bt) continue;
        if (t > bt) {
          bt = t;
          ret.refs.clear();
        }
        ret.refs.push_back(&kv);
      }
      std::sort(ret.refs.begin(), ret.refs.end(), [](EntryRef a, EntryRef b) { return a->first < b->first; });
      for (EntryRef x : ret.refs) ret.all.push_back(x->first);
      if (!ret.all.empty()) {  // selectBestNodeArea (Util.cpp:1028-1040)
        ret.best = ret.all[0];
        for (const auto& na : ret.all)
          if (na.first == me) {
            ret.best = na;
            break;
          }
      }
      ret.success = true;
    } else if (bgp) {
      auto r = bgp_walk(ents);
      if (!r) return std::nullopt;
      ret = std::move(*r);
    } else {  // openr routes: every advertiser is best
      for (const auto& kv : ents) ret.refs.push_back(&kv);
      if (ret.refs.size() > 1)
        std::sort(ret.refs.begin(), ret.refs.end(), [](EntryRef a, EntryRef b) { return a->first < b->first; });
      for (EntryRef x : ret.refs) ret.all.push_back(x->first);
      ret.best = ret.all[0];
      ret.success = true;
    }
    return filter_drained(std::move(ret));
  }

  // ---- getMinCostNodes / getNextHopsWithMetric / getNextHopsThrift ----
  // (Decision.cpp:1082-1305) over the areas in map order
  using NhKey = std::pair<std::string, std::string>;  // (next-hop node, destination or "")

  std::pair<uint64_t, std::map<NhKey, uint64_t>> nexthops_with_metric(std::vector<NodeArea> dsts,
                                                                       bool per_dest) {
    std::sort(dsts.begin(), dsts.end());
    uint64_t shortest = kInf64;
    std::map<NhKey, uint64_t> nh;
    for (auto& ap : areas) {
      Area& a = *ap;
      const SpfIdx* here = spf(a, a.me_id);
      if (!here) return {};
      // getMinCostNodes (:1082-1105; a node of the set reached in any area counts)
      uint64_t mcm = kInf64;
      std::vector<std::pair<std::string, int>> mc;  // (node, entry)
      for (const auto& [d, _] : dsts) {
        const int p = here->find(a.id(d));
        if (p < 0) continue;
        const uint64_t m = here->v.metric[p];
        if (mcm >= m) {
          if (mcm > m) {
            mcm = m;
            mc.clear();
          }
          const std::string& dd = d;
          if (std::find_if(mc.begin(), mc.end(), [&](const auto& x) { return x.first == dd; }) == mc.end())
            mc.emplace_back(d, p);
        }
      }
      if (shortest < mcm) continue;
      if (shortest > mcm) {
        shortest = mcm;
        nh.clear();
      }
      if (mc.empty()) continue;
      for (const auto& [d, p] : mc) {
        const std::string ref = per_dest ? d : std::string();
        for (uint32_t q = here->v.nh_ptr[p]; q < here->v.nh_ptr[p + 1]; ++q) {
          const uint32_t hop = here->v.nh_node[q];
          const int hp = here->find(hop);  // getMetricFromAToB(me, hop)
          const uint64_t mh = hp < 0 ? 0 : here->v.metric[hp];
          nh[{a.name_of(hop), ref}] = shortest - mh;
        }
      }
      if (s->lfa) {
        const auto& ls_links = links(a);
        std::vector<std::string> nbs{me};  // me + every neighbour in one batched plan
        for (const MyLink& l : ls_links)
          if (l.up) nbs.push_back(l.nb);
        std::vector<const char*> cn;
        for (const auto& x : nbs) cn.push_back(x.c_str());
        if (const spf_status code = ls_prefetch_spf_results(a.ls, cn.data(), (uint32_t)cn.size(), 1);
            code != SPF_OK) {
          ls_err(a, code);
          return {};
        }
        for (const MyLink& l : ls_links) {
          if (!l.up) continue;
          const SpfIdx* from_nb = spf(a, a.id(l.nb));
          if (!from_nb) return {};
          const int pme = from_nb->find(a.me_id);
          if (pme < 0) continue;  // (an up link: me is reached from nb)
          const uint64_t nb_to_here = from_nb->v.metric[pme];
          for (const auto& [d, d_area] : dsts) {
            if (a.name != d_area) continue;
            const int pd = from_nb->find(a.id(d));
            if (pd < 0) continue;
            const uint64_t dn = from_nb->v.metric[pd];
            if (dn < shortest + nb_to_here) {  // RFC 5286 (:1180), u64 arithmetic
              const NhKey key{l.nb, per_dest ? d : std::string()};
              auto it = nh.find(key);
              if (it == nh.end() || it->second > dn) nh[key] = dn;
            }
          }
        }
      }
    }
    return {shortest, std::move(nh)};
  }

  // getNextHopsThrift (:1198-1305); ents may be null when !per_dest
  std::vector<NH> nexthops_thrift(const std::vector<NodeArea>& dst_areas, bool v4, bool per_dest,
                                  uint64_t min_metric, const std::map<NhKey, uint64_t>& nhn,
                                  std::optional<int32_t> swap, const Entries* ents) {
    std::vector<NodeArea> dsts;
    if (per_dest) {
      dsts = dst_areas;
      std::sort(dsts.begin(), dsts.end());
    } else {
      dsts.emplace_back();
    }
    std::set<NodeArea> dst_set(dst_areas.begin(), dst_areas.end());
    std::vector<NH> out;
    for (auto& ap : areas) {
      Area& a = *ap;
      for (const MyLink& l : links(a)) {
        for (const auto& [d, d_area] : dsts) {
          if (!d_area.empty() && a.name != d_area) continue;
          auto it = nhn.find({l.nb, d});
          if (it == nhn.end() || !l.up) continue;
          if (!d.empty() && dst_set.count({l.nb, a.name}) && l.nb != d) continue;
          const uint64_t over = l.metric + it->second;
          if (!s->lfa && over != min_metric) continue;
          NH h = link_nh(l, a, v4, over);
          if (swap) {
            if (dst_set.count({l.nb, a.name})) {
              h.action = DC_MPLS_PHP;
            } else {
              h.action = DC_MPLS_SWAP;
              h.swap = *swap;
            }
          }
          if (!d.empty()) {
            std::vector<int32_t> push;
            const auto pe = ents->find({d, a.name});
            if (pe == ents->end()) {
              st = sfail(s, SPF_E_INVALID, "prefixEntries.at((%s, %s))", d.c_str(), a.name.c_str());
              return {};
            }
            if (pe->second.prepend) {
              push.push_back(*pe->second.prepend);
              if (!mpls_label_valid(push.back())) continue;
            }
            if (d != l.nb) {
              const auto& lab = labels(a);
              auto li = lab.find(a.id(d));
              if (li == lab.end()) {  // getAdjacencyDatabases().at(dstNode)
                st = sfail(s, SPF_E_INVALID, "no adjacency database of %s in area %s", d.c_str(),
                           a.name.c_str());
                return {};
              }
              push.push_back(li->second);
              if (!mpls_label_valid(push.back())) continue;
            }
            if (!push.empty()) {
              h.action = DC_MPLS_PUSH;
              h.swap = 0;
              h.push = std::move(push);
            }
          }
          out.push_back(std::move(h));
        }
      }
    }
    return out;
  }

  // addBestPaths (:1020-1080)
  bool add_best_paths(const std::string& prefix, const BestRoute& res, const Entries& ents, bool bgp,
                      std::vector<NH> nhs) {
    std::sort(nhs.begin(), nhs.end());
    nhs.erase(std::unique(nhs.begin(), nhs.end()), nhs.end());
    std::optional<int64_t> need;  // getMinNextHopThreshold
    for (const auto& na : res.all) {
      const Entry& e = ents.at(na);
      if (e.min_nexthop && (!need || *e.min_nexthop > *need)) need = e.min_nexthop;
    }
    if (need && *need > (int64_t)nhs.size()) return false;  // min-nexthop requirement not met
    if (res.has_node(me)) {
      std::optional<int32_t> prepend;
      for (const auto& [na, e] : ents)  // map order
        if (na.first == me && e.prepend) {
          prepend = e.prepend;
          break;
        }
      if (!prepend) {  // CHECK(prependLabel.has_value())
        st = sfail(s, SPF_E_INVALID, "self route %s must carry a prepend label", prefix.c_str());
        return false;
      }
      auto it = s->static_mpls.find(*prepend);
      if (it != s->static_mpls.end())
        for (const NH& x : it->second) {
          NH h;  // createNextHop(address, nullopt, 0, nullopt)
          h.addr = x.addr;
          h.addr_len = x.addr_len;
          nhs.push_back(std::move(h));
        }
    }
    db->add_unicast(prefix, *res.best, bgp && s->bgp_dry_run, db->add_set(nhs));
    return true;
  }

  // selectBestPathsSpf (:834-893)
  void best_paths_spf(const std::string& prefix, const BestRoute& res, const Entries& ents, bool bgp,
                      uint8_t ftype, bool v4) {
    const bool per_dest = ftype == DC_FWD_SR_MPLS;
    std::vector<NodeArea> filtered = res.all;
    if (res.has_node(me) && per_dest)
      for (const auto& [na, e] : ents)  // map order (:855-862)
        if (na.first == me && e.prepend) {
          filtered.erase(std::remove(filtered.begin(), filtered.end(), na), filtered.end());
          break;
        }
    auto [mn, nhn] = nexthops_with_metric(filtered, per_dest);
    if (!ok()) return;
    if (nhn.empty()) {
      s->bump("decision.no_route_to_prefix");
      return;
    }
    std::vector<NH> nhs = nexthops_thrift(res.all, v4, per_dest, mn, nhn, std::nullopt, &ents);
    if (!ok()) return;
    add_best_paths(prefix, res, ents, bgp, std::move(nhs));
  }

  // selectBestPathsKsp2 (:895-1018)
  void best_paths_ksp2(const std::string& prefix, const BestRoute& res, const Entries& ents, bool bgp,
                       uint8_t ftype, bool v4) {
    if (ftype != DC_FWD_SR_MPLS) {
      s->bump("decision.incompatible_forwarding_type");
      return;
    }
    struct Path {
      Area* area;
      std::vector<uint32_t> links;
    };
    std::vector<Path> paths;
    for (auto& ap : areas) {
      Area& a = *ap;
      for (const auto& [node, best_area] : res.all) {
        if (node == me && best_area == a.name) continue;
        ls_paths_view pv{};
        if (const spf_status c = ls_get_kth_paths(a.ls, me.c_str(), node.c_str(), 1, &pv); c != SPF_OK) {
          ls_err(a, c);
          return;
        }
        for (uint32_t p = 0; p < pv.n_paths; ++p)
          paths.push_back({&a, std::vector<uint32_t>(pv.link + pv.path_ptr[p], pv.link + pv.path_ptr[p + 1])});
      }
      const size_t first = paths.size();
      for (const auto& [node, best_area] : res.all) {
        if (a.name != best_area) continue;
        ls_paths_view pv{};
        if (const spf_status c = ls_get_kth_paths(a.ls, me.c_str(), node.c_str(), 2, &pv); c != SPF_OK) {
          ls_err(a, c);
          return;
        }
        for (uint32_t p = 0; p < pv.n_paths; ++p) {
          const uint32_t* sec = pv.link + pv.path_ptr[p];
          const uint32_t ns = pv.path_ptr[p + 1] - pv.path_ptr[p];
          bool add = true;
          for (size_t i = 0; i < first && add; ++i)  // anycast: pathAInPathB
            if (paths[i].area == &a &&
                ls_path_a_in_path_b(paths[i].links.data(), (uint32_t)paths[i].links.size(), sec, ns))
              add = false;
          if (add) paths.push_back({&a, std::vector<uint32_t>(sec, sec + ns)});
        }
      }
    }
    if (paths.empty()) return;
    std::vector<NH> out;
    for (const Path& path : paths) {
      Area& pa = *path.area;  // the links belong to this area's LinkState
      for (auto& ap : areas) {
        Area& a = *ap;
        uint64_t cost = 0;
        std::vector<int32_t> stack;  // pushed at the front: built reversed
        std::string nxt = me;
        const auto& lab = labels(a);
        for (uint32_t lid : path.links) {
          ls_link_desc d{};
          if (const spf_status c = ls_link_info(pa.ls, lid, &d); c != SPF_OK) {
            ls_err(pa, c);
            return;
          }
          const uint32_t nid = pa.id(nxt);
          const bool side1 = d.node1 == nid;
          cost += side1 ? d.metric1 : d.metric2;
          nxt = pa.name_of(side1 ? d.node2 : d.node1);
          auto li = lab.find(a.id(nxt));
          if (li == lab.end()) {
            st = sfail(s, SPF_E_INVALID, "no adjacency database of %s in area %s", nxt.c_str(),
                       a.name.c_str());
            return;
          }
          stack.push_back(li->second);
        }
        // labels.push_front per hop, pop_back (the first hop's label: PHP),
        // prepend label pushed at the front (bottom of the stack)
        std::vector<int32_t> labels_list(stack.rbegin(), stack.rend());
        labels_list.pop_back();
        auto pe = ents.find({nxt, a.name});
        if (pe == ents.end()) {
          st = sfail(s, SPF_E_INVALID, "prefixEntries.at((%s, %s))", nxt.c_str(), a.name.c_str());
          return;
        }
        if (pe->second.prepend) labels_list.insert(labels_list.begin(), *pe->second.prepend);
        ls_link_desc h{};
        if (const spf_status c = ls_link_info(pa.ls, path.links[0], &h); c != SPF_OK) {
          ls_err(pa, c);
          return;
        }
        const bool side1 = h.node1 == pa.me_id;
        NH x;
        if (v4) {
          std::memcpy(x.addr.data(), side1 ? h.nh_v4_1 : h.nh_v4_2, 4);
          x.addr_len = 4;
        } else {
          std::memcpy(x.addr.data(), side1 ? h.nh_v6_1 : h.nh_v6_2, 16);
          x.addr_len = 16;
        }
        x.ifname = std::string(side1 ? h.if1 : h.if2);
        x.metric = i32_metric(cost);
        if (!labels_list.empty()) {
          x.action = DC_MPLS_PUSH;
          x.push = std::move(labels_list);
        }
        x.area = pa.name;
        x.neighbor = pa.name_of(side1 ? h.node2 : h.node1);
        out.push_back(std::move(x));
      }
    }
    add_best_paths(prefix, res, ents, bgp, std::move(out));
  }
};


spf_status graph_cache(dc_solver* s, ls_state* ls, GraphCache*& out) {
  uint32_t N = 0, E = 0;
  spf_status st = ls_flatten(ls, &N, &E);
  if (st != SPF_OK) return sfail(s, st, "flatten: %s", ls_last_error(ls));
  GraphCache& g = s->graphs[ls];
  const uint64_t ep = ls_graph_epoch(ls);
  if (g.epoch != ep) {
    g.csr_name.resize(N);
    g.row_ptr.resize(N + 1);
    g.link_id.resize(std::max<uint32_t>(E, 1));
    st = ls_graph_node_names(ls, g.csr_name.data());
    if (st == SPF_OK) st = ls_graph_csr(ls, g.row_ptr.data(), nullptr, nullptr, g.link_id.data(), nullptr);
    if (st != SPF_OK) return sfail(s, st, "graph: %s", ls_last_error(ls));
    uint32_t mx = 0;
    for (uint32_t n : g.csr_name) mx = std::max(mx, n + 1);
    g.csr_of.assign(mx, ~0u);
    for (uint32_t i = 0; i < N; ++i) g.csr_of[g.csr_name[i]] = i;
    g.epoch = ep;
  }
  out = &g;
  return SPF_OK;
}

}  // namespace

// ---- C-ABI ------------------------------------------------------------------------
extern "C" {

dc_prefix_state* dc_prefix_state_create(void) { return new dc_prefix_state(); }
void dc_prefix_state_destroy(dc_prefix_state* ps) { delete ps; }

spf_status dc_prefix_update(dc_prefix_state* ps, const char* node, const char* area,
                            const dc_prefix_entry* in) {
  if (!ps || !node || !area || !in || !in->prefix) return SPF_E_INVALID;
  Entry e;
  e.v4 = in->is_v4 != 0;
  e.bgp = in->is_bgp != 0;
  e.ftype = in->forwarding_type;
  e.falgo = in->forwarding_algorithm;
  if (in->has_prepend_label) e.prepend = in->prepend_label;
  if (in->has_min_nexthop) e.min_nexthop = in->min_nexthop;
  e.pp = in->path_preference;
  e.sp = in->source_preference;
  e.distance = in->distance;
  if (in->has_mv) {
    MetricVector mv;
    mv.version = in->mv_version;
    for (uint32_t i = 0; i < in->n_mv; ++i) {
      const dc_metric_entity& x = in->mv[i];
      MetricEntity m;
      m.type = x.type;
      m.priority = x.priority;
      m.op = x.op;
      m.tie_breaker = x.is_tie_breaker != 0;
      m.metric.assign(x.metric, x.metric + x.n_metric);
      mv.metrics.push_back(std::move(m));
    }
    e.mv = std::move(mv);
  }
  // entriesByOriginator.emplace, or assignment of an existing key (:55-68)
  Entries& ents = ps->prefixes[in->prefix];
  auto [it, inserted] = ents.emplace(NodeArea(node, area), e);
  if (!inserted) it->second = std::move(e);
  return SPF_OK;
}

spf_status dc_prefix_delete(dc_prefix_state* ps, const char* node, const char* area,
                            const char* prefix) {
  if (!ps || !node || !area || !prefix) return SPF_E_INVALID;
  auto it = ps->prefixes.find(prefix);
  if (it == ps->prefixes.end()) return SPF_OK;
  it->second.erase(NodeArea(node, area));
  if (it->second.empty()) ps->prefixes.erase(it);  // PrefixState.cpp:49-50
  return SPF_OK;
}

spf_status dc_prefix_entries(const dc_prefix_state* ps, const char* prefix, const char** nodes,
                             const char** areas, uint32_t cap, uint32_t* count) {
  if (!ps || !prefix || !count) return SPF_E_INVALID;
  *count = 0;
  auto it = ps->prefixes.find(prefix);
  if (it == ps->prefixes.end()) return SPF_OK;
  uint32_t k = 0;
  for (const auto& kv : it->second) {
    if (k < cap) {
      if (nodes) nodes[k] = kv.first.first.c_str();
      if (areas) areas[k] = kv.first.second.c_str();
    }
    ++k;
  }
  *count = k;
  return SPF_OK;
}

spf_status dc_solver_create(const char* my_node, int enable_v4, int compute_lfa_paths,
                            int bgp_dry_run, int enable_best_route_selection, dc_solver** out) {
  if (!my_node || !out) return SPF_E_INVALID;
  auto s = std::make_unique<dc_solver>();
  s->me = my_node;
  s->enable_v4 = enable_v4 != 0;
  s->lfa = compute_lfa_paths != 0;
  s->bgp_dry_run = bgp_dry_run != 0;
  s->best_route_selection = enable_best_route_selection != 0;
  *out = s.release();
  return SPF_OK;
}
void dc_solver_destroy(dc_solver* s) { delete s; }
const char* dc_last_error(const dc_solver* s) { return s ? s->err.c_str() : "NULL solver"; }

spf_status dc_static_mpls_route_set(dc_solver* s, int32_t label, const dc_nexthop* nhs, uint32_t n,
                                    const char* const* strings, const int32_t* labels) {
  if (!s || (n && !nhs)) return SPF_E_INVALID;
  std::vector<NH> v;
  for (uint32_t i = 0; i < n; ++i) {
    const dc_nexthop& r = nhs[i];
    NH h;
    std::memcpy(h.addr.data(), r.address, 16);
    h.addr_len = r.address_len;
    h.action = r.mpls_action;
    h.metric = r.metric;
    h.swap = r.swap_label;
    if (r.n_push) {
      if (!labels) return sfail(s, SPF_E_INVALID, "static route %d: PUSH labels missing", label);
      h.push.assign(labels + r.push_off, labels + r.push_off + r.n_push);
    }
    auto str = [&](uint32_t id) -> std::optional<std::string> {
      if (id == DC_NONE) return std::nullopt;
      return std::string(strings ? strings[id] : "");
    };
    h.ifname = str(r.ifname);
    h.area = str(r.area);
    h.neighbor = str(r.neighbor);
    v.push_back(std::move(h));
  }
  s->static_mpls[label] = std::move(v);
  return SPF_OK;
}

spf_status dc_static_mpls_route_delete(dc_solver* s, int32_t label) {
  if (!s) return SPF_E_INVALID;
  s->static_mpls.erase(label);
  return SPF_OK;
}

uint64_t dc_counter(const dc_solver* s, const char* name) {
  if (!s || !name) return 0;
  auto it = s->counters.find(name);
  return it == s->counters.end() ? 0 : it->second;
}

spf_status dc_best_route(const dc_solver* s, const char* prefix, int* found, int* success,
                         const char** best_node, const char** best_area, const char** nodes,
                         const char** areas, uint32_t cap, uint32_t* count) {
  if (!s || !prefix || !found) return SPF_E_INVALID;
  auto it = s->best_cache.find(prefix);
  *found = it != s->best_cache.end();
  if (!*found) return SPF_OK;
  const BestRoute& r = it->second;
  if (success) *success = r.success;
  if (best_node) *best_node = r.best ? r.best->first.c_str() : nullptr;
  if (best_area) *best_area = r.best ? r.best->second.c_str() : nullptr;
  for (uint32_t i = 0; i < r.all.size() && i < cap; ++i) {
    if (nodes) nodes[i] = r.all[i].first.c_str();
    if (areas) areas[i] = r.all[i].second.c_str();
  }
  if (count) *count = (uint32_t)r.all.size();
  return SPF_OK;
}

spf_status dc_build_route_db(dc_solver* s, const char* const* area_names, ls_state* const* area_ls,
                             uint32_t n_areas, const dc_prefix_state* ps, dc_route_db** out) {
  if (!s || !ps || !out || (n_areas && (!area_names || !area_ls)))
    return sfail(s, SPF_E_INVALID, "dc_build_route_db: NULL argument");
  *out = nullptr;
  const std::string& me = s->me;
  // std::unordered_map<std::string, LinkState> emplaced in the given order
  std::unordered_map<std::string, ls_state*> amap;
  for (uint32_t i = 0; i < n_areas; ++i) {
    if (!area_names[i] || !area_ls[i]) return sfail(s, SPF_E_INVALID, "area %u: NULL", i);
    amap.emplace(area_names[i], area_ls[i]);
  }
  auto db = std::make_unique<dc_route_db>();
  Build b{s, me, {}, {}, db.get()};
  bool exists = false;
  for (const auto& [name, ls] : amap) {
    auto a = std::make_unique<Area>();
    a->name = name;
    a->ls = ls;
    a->serial = ls_serial(ls);
    a->me_id = ls_name_id(ls, me.c_str());
    exists |= ls_has_node(ls, me.c_str()) != 0;
    b.by_name.emplace(name, a.get());
    b.areas.push_back(std::move(a));
  }
  if (!exists) return SPF_OK;  // std::nullopt
  uint64_t t_ph = now_ns();
  auto phase = [&](int k) {
    const uint64_t t = now_ns();
    s->phase_ns[k] += t - t_ph;
    t_ph = t;
  };
  // bestRoutesCache_.clear() (Decision.cpp:575): entries this build does not store again
  // are swept when it ends; stored ones reuse their node and key (no string
  // allocation per prefix and build)
  const uint64_t gen = ++s->build_gen;
  struct Sweep {
    dc_solver* s;
    uint64_t gen;
    ~Sweep() {
      for (auto it = s->best_cache.begin(); it != s->best_cache.end();) {
        if (it->second.gen != gen) {
          it = s->best_cache.erase(it);
        } else {
          it->second.refs.clear();  // (they pointed into this build)
          ++it;
        }
      }
    }
  } sweep{s, gen};
  s->best_cache.reserve(ps->prefixes.size());
  const bool single = b.areas.size() == 1;
  std::vector<const SpfIdx*> mine;
  for (auto& a : b.areas) {
    mine.push_back(b.spf(*a, a->me_id));
    if (!b.ok()) return b.st;
  }

  phase(0);
  // ---- unicast: createRouteForPrefix (:389-555) ----
  struct Uni {
    const std::string* prefix;
    const Entries* ents;
    std::unique_ptr<Entries> own;  // the filtered copy, when an entry was dropped
    const BestRoute* res;           // in the solver's best-routes cache
    bool bgp, v4;
  };
  std::vector<Uni> uni;
  uni.reserve(ps->prefixes.size());
  bool ksp_fetched = false;
  std::unordered_map<const Area*, size_t> area_idx;
  for (size_t i = 0; i < b.areas.size(); ++i) area_idx.emplace(b.areas[i].get(), i);
  // an advertiser survives the reachability filter unless its area has a
  // LinkState in which my SPF does not reach it
  auto reached = [&](const std::pair<const NodeArea, Entry>& kv) {
    Area* a = b.area_of(kv.first.second);
    if (!a) return true;
    return mine[single ? 0 : area_idx.at(a)]->find(a->id(kv)) >= 0;
  };
  for (const auto& [prefix, all] : ps->prefixes) {
    // entries of nodes unreachable in their own area dropped (:409-420): the
    // copy's erasures keep the survivors' order; no copy when none drops
    std::unique_ptr<Entries> own;
    const Entries* ep = &all;
    for (const auto& kv : all)
      if (!reached(kv)) {
        own = std::make_unique<Entries>(all);
        for (auto it = own->begin(); it != own->end();) {
          if (reached(*it)) ++it;
          else it = own->erase(it);
        }
        ep = own.get();
        break;
      }
    const Entries& ents = *ep;
    if (ents.empty()) {
      s->bump("decision.no_route_to_prefix");
      continue;
    }
    const bool v4 = ents.begin()->second.v4;
    if (v4 && !s->enable_v4) {
      s->bump("decision.skipped_unicast_route");
      continue;
    }
    bool has_bgp = false, has_non_bgp = false, missing_mv = false, self_prepend = true;
    for (const auto& [na, e] : ents) {
      has_bgp |= e.bgp;
      has_non_bgp |= !e.bgp;
      if (na.first == me) self_prepend &= e.prepend.has_value();
      if (e.bgp && !e.mv) missing_mv = true;
    }
    if (has_bgp && ((has_non_bgp && !s->best_route_selection) || missing_mv)) {
      s->bump("decision.skipped_unicast_route");
      continue;
    }
    // bestRoutesCache_ (its refs point into this build's entries: cleared
    // when the build ends); the selection starts from the slot's vectors, so
    // a prefix re-selected every build allocates nothing (a slot this build
    // does not fill keeps an old generation and is swept)
    BestRoute& slot = s->best_cache[prefix];
    BestRoute scratch;
    scratch.all.swap(slot.all);
    scratch.refs.swap(slot.refs);
    scratch.all.clear();
    scratch.refs.clear();
    auto sel = b.select_best(ents, has_bgp, std::move(scratch));
    if (!b.ok()) return b.st;
    if (!sel->success) continue;
    if (sel->all.empty()) {
      s->bump("decision.no_route_to_prefix");
      continue;
    }
    slot = std::move(*sel);
    slot.gen = gen;
    const BestRoute& res = slot;
    if (res.has_node(me) && !self_prepend) continue;  // self-advertised
    // getPrefixForwardingTypeAndAlgorithm (Util.cpp:617-643)
    uint8_t ftype = DC_FWD_SR_MPLS, falgo = DC_ALGO_KSP2_ED_ECMP;
    for (const auto& kv : ents) {  // (walked in map order, as the reference)
      if (std::find(res.refs.begin(), res.refs.end(), &kv) == res.refs.end()) continue;
      ftype = std::min(ftype, kv.second.ftype);
      falgo = std::min(falgo, kv.second.falgo);
      if (ftype == DC_FWD_IP && falgo == DC_ALGO_SP_ECMP) break;
    }
    if (single && falgo == DC_ALGO_SP_ECMP && ftype == DC_FWD_IP) {
      uni.push_back({&prefix, ep, std::move(own), &res, has_bgp, v4});
      continue;
    }
    if (single && falgo == DC_ALGO_KSP2_ED_ECMP && !ksp_fetched) {
      // one batched KSP2 launch for every advertiser (ls_prefetch_kth_paths)
      ksp_fetched = true;
      if (const spf_status c = ls_prefetch_kth_paths(b.areas[0]->ls, me.c_str()); c != SPF_OK)
        return b.ls_err(*b.areas[0], c);
    }
    if (falgo == DC_ALGO_SP_ECMP) b.best_paths_spf(prefix, res, ents, has_bgp, ftype, v4);
    else b.best_paths_ksp2(prefix, res, ents, has_bgp, ftype, v4);
    if (!b.ok()) return b.st;
  }

  phase(1);
  // ---- node labels (:583-664) ----
  // label -> (node, area), the collision rule of :605-617 (the smaller name wins)
  struct LabelOwner {
    uint32_t node;  // name id in `area`
    Area* area;
    std::string name() const { return ls_name(area->ls, node); }
  };
  // labels in first-seen order with their owners; label -> position by open
  // addressing (one slot per label, no node allocation per label)
  std::vector<int32_t> label_order;
  std::vector<LabelOwner> owner;
  std::vector<uint32_t> lpos;  // position + 1, 0 = empty
  auto lslot = [&](int32_t top) {
    const size_t mask = lpos.size() - 1;
    size_t h = (size_t)((uint32_t)top * 0x9E3779B1u) & mask;
    while (lpos[h] && label_order[lpos[h] - 1] != top) h = (h + 1) & mask;
    return h;
  };
  for (auto& ap : b.areas) {
    Area& a = *ap;
    uint32_t n = 0;
    ls_adjacency_databases(a.ls, nullptr, nullptr, 0, &n);
    std::vector<uint32_t> ids(n);
    std::vector<int32_t> lab(n);
    ls_adjacency_databases(a.ls, ids.data(), lab.data(), n, &n);
    {  // room for every label of this area at <= 1/2 load
      size_t want = 64;
      while (want < 2 * (label_order.size() + n)) want *= 2;
      if (want > lpos.size()) {
        lpos.assign(want, 0u);
        for (uint32_t k = 0; k < label_order.size(); ++k) lpos[lslot(label_order[k])] = k + 1;
      }
    }
    for (uint32_t i = 0; i < n; ++i) {
      const int32_t top = lab[i];
      if (top == 0 || !mpls_label_valid(top)) continue;
      uint32_t& pos = lpos[lslot(top)];
      if (!pos) {
        label_order.push_back(top);
        owner.push_back({ids[i], &a});
        pos = (uint32_t)label_order.size();
      } else {
        LabelOwner& o = owner[pos - 1];
        if (!(std::strcmp(ls_name(o.area->ls, o.node), ls_name(a.ls, ids[i])) < 0))
          o = {ids[i], &a};  // the collision's smaller name wins (a tie: the later area)
      }
    }
  }

  if (single) {
    // ---- one batched selection: IP prefixes, then node labels ----
    Area& a = *b.areas[0];
    GraphCache* g = nullptr;
    if (const spf_status c = graph_cache(s, a.ls, g); c != SPF_OK) return c;
    std::vector<uint32_t> set_ptr{0}, set_nodes;
    set_ptr.reserve(uni.size() + label_order.size() + 1);
    set_nodes.reserve(uni.size() + label_order.size());
    auto add_node = [&](uint32_t id) {
      if (id < g->csr_of.size() && g->csr_of[id] != ~0u) set_nodes.push_back(g->csr_of[id]);
    };
    for (const Uni& u : uni) {
      for (EntryRef r : u.res->refs) add_node(a.id(*r));
      set_ptr.push_back((uint32_t)set_nodes.size());
    }
    for (const LabelOwner& o : owner) {  // labels needing a selection, in set order
      if (o.node == a.me_id) continue;
      add_node(o.node);
      set_ptr.push_back((uint32_t)set_nodes.size());
    }
    const uint32_t n_sets = (uint32_t)set_ptr.size() - 1;
    phase(2);
    Selection& sel = s->sel;
    const uint32_t m = a.me_id < g->csr_of.size() ? g->csr_of[a.me_id] : ~0u;
    if (m != ~0u && n_sets) {
      // every min and count is written by the selection, and a set's first
      // count edges and metrics: no fill (the same sizes resize nothing)
      sel.deg = std::max<uint32_t>(1, g->row_ptr[m + 1] - g->row_ptr[m]);
      sel.mins.resize(n_sets);
      sel.cnt.resize(n_sets);
      sel.edge.resize((size_t)n_sets * sel.deg);
      sel.metric.resize((size_t)n_sets * sel.deg);
      if (set_nodes.empty()) set_nodes.push_back(0);
      const uint32_t flags = s->lfa ? SPF_ROUTE_LFA : 0u;
      spf_status c = SPF_E_UNSUPPORTED;
      if (spf_mplan* mp = ls_all_sources_plan(a.ls)) {
        // a resident all-sources pass answers from me's owner, no new plan
        c = spf_mplan_routes(mp, m, set_ptr.data(), set_nodes.data(), n_sets, flags, sel.mins.data(),
                             sel.cnt.data(), sel.edge.data(), sel.metric.data());
        if (c != SPF_OK && c != SPF_E_UNSUPPORTED)
          return sfail(s, c, "spf_mplan_routes: %s", spf_global_error());
      }
      if (c != SPF_OK) {
        spf_ctx* eng = ls_engine(a.ls);
        c = spf_routes(eng, m, set_ptr.data(), set_nodes.data(), n_sets, flags, sel.mins.data(),
                       sel.cnt.data(), sel.edge.data(), sel.metric.data());
        if (c != SPF_OK) return sfail(s, c, "spf_routes: %s", spf_last_error(eng));
      }
    } else {
      sel.cnt.assign(n_sets, 0);
    }
    phase(3);
    // me's links by link id (the selection's edges), and each link's
    // createNextHop record with its strings interned once
    struct LinkRec {
      const MyLink* l;
      uint32_t nb_id;
      dc_nexthop v4, v6;
    };
    std::unordered_map<uint32_t, LinkRec> by_link;
    for (const MyLink& l : b.links(a)) {
      LinkRec r{&l, a.id(l.nb), {}, {}};
      r.v6.address_len = 16;
      std::memcpy(r.v6.address, l.v6.data(), 16);
      r.v4.address_len = 4;
      std::memcpy(r.v4.address, l.v4.data(), 4);
      for (dc_nexthop* x : {&r.v4, &r.v6}) {
        x->ifname = db->intern(l.ifname);
        x->area = db->intern(a.name);
        x->neighbor = db->intern(l.nb);
      }
      by_link.emplace(l.id, r);
    }
    // me's CSR edges -> their link's record (the selection returns edges of me's row)
    const uint32_t e0 = m != ~0u ? g->row_ptr[m] : 0u, e1 = m != ~0u ? g->row_ptr[m + 1] : 0u;
    std::vector<const LinkRec*> rec_at(e1 - e0, nullptr);
    for (uint32_t e = e0; e < e1; ++e) {
      auto it = by_link.find(g->link_id[e]);
      rec_at[e - e0] = it == by_link.end() ? nullptr : &it->second;
    }
    auto edge_rec = [&](uint32_t e) -> const LinkRec* {
      if (e - e0 < rec_at.size()) return rec_at[e - e0];
      auto it = by_link.find(g->link_id[e]);
      return it == by_link.end() ? nullptr : &it->second;
    };
    // IP routes: equal selections (edges, metrics, family) share one record range
    std::unordered_map<std::string, std::pair<uint32_t, uint32_t>> shared;
    db->str_off.reserve(db->str_off.size() + 2 * uni.size());
    db->arena.reserve(db->arena.size() + 24 * uni.size());
    db->uni.reserve(db->uni.size() + 6 * uni.size());
    std::vector<dc_nexthop> recs;
    std::string key;
    for (uint32_t i = 0; i < uni.size(); ++i) {
      const Uni& u = uni[i];
      const uint32_t c = sel.cnt[i];
      if (!c) {
        s->bump("decision.no_route_to_prefix");
        continue;
      }
      const size_t o = (size_t)i * sel.deg;
      if (u.res->has_node(me)) {  // self-advertised with a prepend label: addBestPaths' static hops
        std::vector<NH> v;
        for (uint32_t q = 0; q < c; ++q) {
          const LinkRec* r = edge_rec(sel.edge[o + q]);
          if (!r) return sfail(s, SPF_E_INVALID, "selected edge %u is not a link of %s", sel.edge[o + q], me.c_str());
          v.push_back(b.link_nh(*r->l, a, u.v4, sel.metric[o + q]));
        }
        b.add_best_paths(*u.prefix, *u.res, *u.ents, u.bgp, std::move(v));
        if (!b.ok()) return b.st;
        continue;
      }
      key.assign(reinterpret_cast<const char*>(sel.edge.data() + o), 4ull * c);
      key.append(reinterpret_cast<const char*>(sel.metric.data() + o), 8ull * c);
      key.push_back(u.v4 ? 1 : 0);
      auto it = shared.find(key);
      if (it == shared.end()) {
        recs.clear();
        for (uint32_t q = 0; q < c; ++q) {
          const LinkRec* r = edge_rec(sel.edge[o + q]);
          if (!r) return sfail(s, SPF_E_INVALID, "selected edge %u is not a link of %s", sel.edge[o + q], me.c_str());
          dc_nexthop x = u.v4 ? r->v4 : r->v6;
          x.metric = i32_metric(sel.metric[o + q]);
          recs.push_back(x);
        }
        it = shared.emplace(key, db->add_records(recs)).first;
      }
      // addBestPaths (:1020-1080), one remote advertiser set: the min-nexthop check
      std::optional<int64_t> need;
      EntryRef best = nullptr;
      for (EntryRef r : u.res->refs) {
        const Entry& e = r->second;
        if (e.min_nexthop && (!need || *e.min_nexthop > *need)) need = e.min_nexthop;
        if (r->first == *u.res->best) best = r;
      }
      if (need && *need > (int64_t)(it->second.second - it->second.first)) continue;
      if (best && best->first.second == a.name) {  // strings from the per-name cache
        if (a.area_sid == DC_NONE) a.area_sid = db->intern(a.name);
        db->uni.insert(db->uni.end(), {db->push_unique(*u.prefix), a.sid(db.get(), a.id(*best), best->first.first),
                                       a.area_sid, (uint32_t)(u.bgp && s->bgp_dry_run), it->second.first,
                                       it->second.second});
      } else {  // (the drained filter kept an unfiltered bestNodeArea)
        db->add_unicast(*u.prefix, *u.res->best, u.bgp && s->bgp_dry_run, it->second);
      }
    }
    // node-label routes (selection sets after the IP ones, in label order)
    uint32_t k = (uint32_t)uni.size();
    db->reserve_labels(label_order.size());
    db->mpls.reserve(db->mpls.size() + 3 * label_order.size());
    for (size_t li = 0; li < label_order.size(); ++li) {
      const int32_t top = label_order[li];
      const LabelOwner& own = owner[li];
      if (own.node == a.me_id) {
        NH h;  // POP_AND_LOOKUP, address "::"
        h.action = DC_MPLS_POP_AND_LOOKUP;
        h.area = own.area->name;
        std::vector<NH> v{h};
        db->add_mpls(top, db->add_set(v));
        continue;
      }
      const uint32_t i = k++;
      const uint32_t c = sel.cnt[i];
      if (!c) {
        s->bump("decision.no_route_to_label");
        continue;
      }
      const size_t o = (size_t)i * sel.deg;
      recs.clear();
      for (uint32_t q = 0; q < c; ++q) {
        const LinkRec* r = edge_rec(sel.edge[o + q]);
        if (!r) return sfail(s, SPF_E_INVALID, "selected edge %u is not a link of %s", sel.edge[o + q], me.c_str());
        dc_nexthop x = r->v6;
        x.metric = i32_metric(sel.metric[o + q]);
        if (r->nb_id == own.node) {
          x.mpls_action = DC_MPLS_PHP;
        } else {
          x.mpls_action = DC_MPLS_SWAP;
          x.swap_label = top;
        }
        recs.push_back(x);
      }
      db->add_mpls(top, db->add_records(recs));
    }
  } else {
    for (size_t li = 0; li < label_order.size(); ++li) {
      const int32_t top = label_order[li];
      const LabelOwner& own = owner[li];
      const std::string node = own.name();
      if (node == me) {
        NH h;
        h.action = DC_MPLS_POP_AND_LOOKUP;
        h.area = own.area->name;
        std::vector<NH> v{h};
        db->add_mpls(top, db->add_set(v));
        continue;
      }
      const std::vector<NodeArea> dst{{node, own.area->name}};
      auto [mn, nhn] = b.nexthops_with_metric(dst, false);
      if (!b.ok()) return b.st;
      if (nhn.empty()) {
        s->bump("decision.no_route_to_label");
        continue;
      }
      std::vector<NH> v = b.nexthops_thrift(dst, false, false, mn, nhn, top, nullptr);
      if (!b.ok()) return b.st;
      db->add_mpls(top, db->add_set(v));
    }
  }

  phase(4);
  // ---- adjacency labels of every area (:667-698) ----
  for (auto& ap : b.areas) {
    Area& a = *ap;
    for (const MyLink& l : b.links(a)) {
      const int32_t top = l.adj_label;
      if (top == 0 || !mpls_label_valid(top)) continue;
      NH h = b.link_nh(l, a, false, l.metric);
      h.action = DC_MPLS_PHP;
      std::vector<NH> v{h};
      db->add_mpls(top, db->add_set(v));
    }
  }
  // ---- static MPLS routes (:700-707) ----
  for (auto& [top, nhs] : s->static_mpls) {
    std::vector<NH> v = nhs;
    db->add_mpls(top, db->add_set(v));
  }
  phase(5);
  *out = db.release();
  return SPF_OK;
}

void dc_debug_phase_ns(const dc_solver* s, uint64_t* out) {
  for (int i = 0; i < 6; ++i) out[i] = s ? s->phase_ns[i] : 0;
}

void dc_route_db_destroy(dc_route_db* db) { delete db; }
uint32_t dc_route_db_strings(const dc_route_db* db) { return db ? (uint32_t)db->str_off.size() : 0; }
const char* dc_route_db_string(const dc_route_db* db, uint32_t id) {
  return db && id < db->str_off.size() ? db->str(id) : nullptr;
}
const dc_nexthop* dc_route_db_nexthops(const dc_route_db* db, uint32_t* n) {
  if (n) *n = db ? (uint32_t)db->nhs.size() : 0;
  return db ? db->nhs.data() : nullptr;
}
const int32_t* dc_route_db_labels(const dc_route_db* db, uint32_t* n) {
  if (n) *n = db ? (uint32_t)db->labels.size() : 0;
  return db ? db->labels.data() : nullptr;
}
uint32_t dc_route_db_unicast_count(const dc_route_db* db) { return db ? (uint32_t)db->uni.size() / 6 : 0; }
spf_status dc_route_db_unicast(const dc_route_db* db, uint32_t i, uint32_t* prefix, uint32_t* best_node,
                               uint32_t* best_area, int* do_not_install, uint32_t* nh_begin,
                               uint32_t* nh_end) {
  if (!db || i >= db->uni.size() / 6) return SPF_E_INVALID;
  const uint32_t* r = db->uni.data() + 6ull * i;
  if (prefix) *prefix = r[0];
  if (best_node) *best_node = r[1];
  if (best_area) *best_area = r[2];
  if (do_not_install) *do_not_install = (int)r[3];
  if (nh_begin) *nh_begin = r[4];
  if (nh_end) *nh_end = r[5];
  return SPF_OK;
}
uint32_t dc_route_db_mpls_count(const dc_route_db* db) { return db ? (uint32_t)db->mpls.size() / 3 : 0; }
spf_status dc_route_db_mpls(const dc_route_db* db, uint32_t i, int32_t* label, uint32_t* nh_begin,
                            uint32_t* nh_end) {
  if (!db || i >= db->mpls.size() / 3) return SPF_E_INVALID;
  const uint32_t* r = db->mpls.data() + 3ull * i;
  if (label) *label = (int32_t)r[0];
  if (nh_begin) *nh_begin = r[1];
  if (nh_end) *nh_end = r[2];
  return SPF_OK;
}
const uint32_t* dc_route_db_unicast_table(const dc_route_db* db, uint32_t* n) {
  if (n) *n = dc_route_db_unicast_count(db);
  return db ? db->uni.data() : nullptr;
}
const uint32_t* dc_route_db_mpls_table(const dc_route_db* db, uint32_t* n) {
  if (n) *n = dc_route_db_mpls_count(db);
  return db ? db->mpls.data() : nullptr;
}

}  // extern "C"
