// ============================================================================
//  link_state.cpp -- host side of the LinkState drop-in (openr_linkstate.h).
//
//  Two halves:
//   * LSDB bookkeeping with the reference's semantics -- bidirectional-link
//     check (reference openr/decision/LinkState.cpp:531-547), ordered merge of
//     old/new links (:564-719), ordered-FIB holds (HoldableValue, :54-125),
//     link / node overload (:233-236, :480-498), deletion (:721-738).
//     Links of a node are kept in a std::unordered_set hashed exactly like
//     the reference's LinkSet (folly pair hash of the ordered (node, ifName)
//     names, LinkState.cpp:138-142), so that its iteration order -- which the
//     reference's Dijkstra uses to order parallel links in pathLinks -- is
//     reproduced; the CSR lists each node's edges in that order.
//   * Shortest paths: flatten the up links into a CSR once per topology
//     version and run every SPF on the MI355X engine (spf_engine.hip).  Results
//     are memoised per (node, useLinkMetric) and per (src, dst, k) and
//     invalidated on topology changes, as LinkState.h:271-301 does.
// ============================================================================
#include <algorithm>
#include <chrono>
#include <array>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <numeric>
#include <optional>
#include <thread>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "openr_linkstate.h"

namespace openr_amd {
namespace {

using Metric = uint64_t;
constexpr uint32_t kNone = 0xFFFFFFFFu;

// folly::hash::hash_128_to_64, the combiner behind folly's
// std::hash<std::pair<A, B>> (= mix(std::hash<A>(a), std::hash<B>(b))).
inline uint64_t folly_mix(uint64_t upper, uint64_t lower) {
  constexpr uint64_t kMul = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lower ^ upper) * kMul;
  a ^= a >> 47;
  uint64_t b = (upper ^ a) * kMul;
  b ^= b >> 47;
  return b * kMul;
}

// Ordered-FIB holdable value (rfc 6976), reference LinkState.h:36-58.
template <class T>
struct Holdable {
  T val;
  std::optional<T> held;
  Metric ttl = 0;
  explicit Holdable(T v) : val(v) {}
  void set(T v) {  // plain assignment: clears any hold
    val = v;
    held.reset();
    ttl = 0;
  }
  const T& get() const { return held ? *held : val; }
  bool has_hold() const { return held.has_value(); }
  bool tick() {
    if (!held) return false;
    if (--ttl != 0) return false;
    held.reset();
    return true;
  }
  bool bring_up(T v) const;
  // returns true when the effective value changes now
  bool update(T v, Metric up, Metric down) {
    if (v == val) return false;
    if (held) {
      held.reset();
      ttl = 0;
    } else {
      ttl = bring_up(v) ? up : down;
      if (ttl) held = val;
    }
    val = v;
    return !held;
  }
};
template <>
bool Holdable<bool>::bring_up(bool v) const { return val && !v; }
template <>
bool Holdable<Metric>::bring_up(Metric v) const { return v < val; }

using OrderedNames =
    std::pair<std::pair<std::string, std::string>, std::pair<std::string, std::string>>;

struct Side {
  uint32_t node;
  std::string ifname;
  Holdable<Metric> metric{1};
  Holdable<bool> overload{false};
  int32_t label = 0;
  std::array<uint8_t, 4> v4{};
  std::array<uint8_t, 16> v6{};
};

struct LinkObj {
  uint32_t id = kNone;
  Side s[2];
  Metric hold_up = 0;
  OrderedNames names;
  uint64_t hash = 0;

  int side_of(uint32_t n) const { return s[0].node == n ? 0 : (s[1].node == n ? 1 : -1); }
  Side& from(uint32_t n) { return s[side_of(n)]; }
  const Side& from(uint32_t n) const { return s[side_of(n)]; }
  uint32_t other(uint32_t n) const { return s[0].node == n ? s[1].node : s[0].node; }
  bool up() const { return hold_up == 0 && !s[0].overload.get() && !s[1].overload.get(); }
  bool before(const LinkObj& o) const {  // Link::operator< (LinkState.cpp:347-353)
    return hash != o.hash ? hash < o.hash : names < o.names;
  }
  bool same(const LinkObj& o) const { return hash == o.hash && names == o.names; }
  bool tick() {
    bool expired = false;
    if (hold_up) expired |= (--hold_up == 0);
    for (auto& x : s) {
      expired |= x.metric.tick();
      expired |= x.overload.tick();
    }
    return expired;
  }
  bool holds() const {
    return hold_up || s[0].metric.has_hold() || s[1].metric.has_hold() ||
           s[0].overload.has_hold() || s[1].overload.has_hold();
  }
};

// NB: not noexcept, as the reference's LinkPtrHash -- keeps libstdc++'s node
// layout (cached hash codes) identical; iteration order depends only on the
// hash values and the insert/erase sequence.
struct LinkHash {
  size_t operator()(const LinkObj* l) const { return l->hash; }
};
struct LinkEq {
  bool operator()(const LinkObj* a, const LinkObj* b) const { return a->same(*b); }
};
using LinkBag = std::unordered_set<LinkObj*, LinkHash, LinkEq>;

struct AdjIn {
  uint32_t other;
  std::string ifname, other_if;
  int32_t metric, label;
  bool overload;
  std::array<uint8_t, 4> v4;
  std::array<uint8_t, 16> v6;
};
struct DbIn {
  bool overload = false;
  int32_t node_label = 0;
  std::vector<AdjIn> adjs;
};

struct SpfMemo {
  std::vector<uint32_t> node, nh_ptr{0}, nh_node, pl_ptr{0}, pl_link, pl_prev;
  std::vector<uint64_t> metric;
  // csr-indexed predecessor lists for path tracing
  std::vector<uint32_t> pred_ptr, pred_edge;
  std::vector<uint32_t> dist;  // csr-indexed (empty for an off-graph source)
  // filled by ls_prefetch_spf_results: the reference's runSpf (and its
  // decision.spf_runs count) happens on the first getSpfResult
  uint8_t pending = 0;
  // metrics and next hops only (ls_get_spf_metrics): pathLinks are derived
  // on the first call that asks for them, without counting another run
  uint8_t pl_missing = 0;
};
struct PathMemo {
  std::vector<uint32_t> path_ptr{0}, link;
  // filled by ls_prefetch_kth_paths: the reference's side effects of
  // computing it (getSpfResult(src) for k = 1, one runSpf for k = 2 with
  // k = 1 paths) are applied on first access, so spf_runs counts as if the
  // pair had been queried alone
  uint8_t pending = 0;
};

}  // namespace
}  // namespace openr_amd

using namespace openr_amd;

static uint64_t next_ls_serial() {
  static std::atomic<uint64_t> n{0};
  return ++n;
}

struct ls_state {
  std::string area;
  int device = 0;
  std::string err;
  const uint64_t serial = next_ls_serial();  // process-unique (ls_serial)
  spf_ctx* eng = nullptr;
  // several GPUs (ls_create_multi): eng is member 0 of meng (single-source
  // queries), `all` the resident all-sources pass of ls_prefetch_all_sources
  spf_mctx* meng = nullptr;
  spf_mplan* all = nullptr;
  bool all_valid = false;  // `all` holds results of the current graph
  int all_ulm = 1;
  uint64_t spf_runs = 0;

  // names
  std::vector<std::string> names;
  std::unordered_map<std::string, uint32_t> name_ids;

  // LSDB
  std::unordered_map<uint32_t, DbIn> dbs;
  std::vector<uint32_t> db_order;  // dbs' node ids by ascending name (ls_adjacency_databases)
  bool db_order_valid = false;
  std::unordered_map<uint32_t, LinkBag> link_map;
  LinkBag all_links;
  std::unordered_map<uint32_t, Holdable<bool>> node_ovl;
  std::vector<std::unique_ptr<LinkObj>> slab;
  std::vector<uint32_t> free_ids;
  // link ids holding slots of the flattened CSR (in_csr) are not reused until
  // the next full flatten: a withdrawn link leaves a dead slot under its id
  // (ghost), and gets the same id -- the same slots -- when it comes back
  std::vector<uint8_t> in_csr;
  std::map<OrderedNames, uint32_t> ghost;
  uint64_t row_patches = 0;  // flattens that patched rows in place (ls_debug_row_patches)
  // nodes whose links changed since the last flatten (the rows a patch
  // rewrites); touched_all: unknown, every row is compared
  std::vector<uint32_t> touched;
  bool touched_all = true;
  void touch(const LinkObj* l) {
    touched.push_back(l->s[0].node);
    touched.push_back(l->s[1].node);
  }

  // flattened graph
  bool dirty = true;                 // links changed: re-flatten (patch or reload)
  uint64_t flat_epoch = 0;           // bumped whenever the flattened CSR structure is rebuilt
  bool engine_loaded = false;        // the engine holds the flattened graph below
  std::vector<uint32_t> pending_ovl;  // name ids whose overload bit flipped since the last flatten
  std::vector<uint32_t> csr_name;   // csr id -> name id
  std::vector<uint32_t> csr_of;     // name id -> csr id (kNone)
  std::vector<uint32_t> row_ptr, col, link_id, edge_tail;
  std::vector<int32_t> metric;
  std::vector<uint8_t> ovl;

  // memo
  std::map<std::pair<uint32_t, int>, SpfMemo> spf_memo;
  // getSpfResult cost by phase, ns (ls_debug_phase_ns): plan build, GPU
  // execute + copy back, pathLinks, host result assembly
  uint64_t phase_ns[4] = {0, 0, 0, 0};
  // pathLinks scratch: one directed edge per predecessor at most, so a
  // buffer of every edge takes them in one preds call (no sizing call)
  std::vector<uint32_t> pred_scratch;
  std::map<std::tuple<uint32_t, uint32_t, uint64_t>, PathMemo> ksp_memo;

  uint32_t intern(const std::string& s) {
    auto it = name_ids.find(s);
    if (it != name_ids.end()) return it->second;
    const uint32_t id = (uint32_t)names.size();
    names.push_back(s);
    name_ids.emplace(s, id);
    return id;
  }
  const uint32_t* find_name(const std::string& s) const {
    auto it = name_ids.find(s);
    return it == name_ids.end() ? nullptr : &it->second;
  }
};

namespace {

spf_status lfail(ls_state* ls, spf_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ls) ls->err = buf;
  return st;
}

spf_status eng_fail(ls_state* ls, spf_status st) {
  ls->err = std::string("engine: ") + (ls->meng ? spf_mctx_last_error(ls->meng) : "") +
            (ls->meng ? " / " : "") + spf_last_error(ls->eng);
  return st;
}

void clear_results(ls_state* ls) {
  ls->spf_memo.clear();
  ls->ksp_memo.clear();
  ls->all_valid = false;  // the resident pass answered the old graph
}

// graph to the engine: every member's replica when several GPUs serve it
spf_status eng_load(ls_state* ls, const spf_graph* g) {
  if (ls->all) {  // bound to the old CSR structure
    spf_mplan_destroy(ls->all);
    ls->all = nullptr;
  }
  return ls->meng ? spf_mctx_graph_load(ls->meng, g) : spf_graph_load(ls->eng, g);
}
spf_status eng_set_overload(ls_state* ls, const uint32_t* nodes, const uint8_t* v, uint32_t n) {
  return ls->meng ? spf_mctx_graph_set_overload(ls->meng, nodes, v, n)
                  : spf_graph_set_overload(ls->eng, nodes, v, n);
}
spf_status eng_patch_rows(ls_state* ls, const uint32_t* nodes, uint32_t n, const uint32_t* col,
                          const int32_t* m, const uint32_t* link) {
  return ls->meng ? spf_mctx_graph_patch_rows(ls->meng, nodes, n, col, m, link)
                  : spf_graph_patch_rows(ls->eng, nodes, n, col, m, link);
}
spf_status eng_set_metric(ls_state* ls, const uint32_t* edges, const int32_t* m, uint32_t n) {
  return ls->meng ? spf_mctx_graph_set_metric(ls->meng, edges, m, n)
                  : spf_graph_set_metric(ls->eng, edges, m, n);
}

void clear_memo(ls_state* ls) {
  clear_results(ls);
  ls->dirty = true;
}

void put_change(ls_change* out, bool topo, bool attrs, bool label) {
  if (!out) return;
  out->topology_changed = topo;
  out->link_attributes_changed = attrs;
  out->node_label_changed = label;
  out->pad = 0;
}

std::unique_ptr<LinkObj> make_link(ls_state* ls, uint32_t n1, const AdjIn& a1, uint32_t n2,
                                   const AdjIn& a2) {
  auto l = std::make_unique<LinkObj>();
  const AdjIn* in[2] = {&a1, &a2};
  const uint32_t nodes[2] = {n1, n2};
  for (int i = 0; i < 2; ++i) {
    Side& s = l->s[i];
    s.node = nodes[i];
    s.ifname = in[i]->ifname;
    s.metric.set((Metric)(int64_t)in[i]->metric);  // i32 -> u64 like the reference
    s.overload.set(in[i]->overload);
    s.label = in[i]->label;
    s.v4 = in[i]->v4;
    s.v6 = in[i]->v6;
  }
  l->names = std::minmax(std::make_pair(ls->names[n1], a1.ifname),
                         std::make_pair(ls->names[n2], a2.ifname));
  const auto& nm = l->names;
  l->hash = folly_mix(folly_mix(std::hash<std::string>()(nm.first.first),
                                std::hash<std::string>()(nm.first.second)),
                      folly_mix(std::hash<std::string>()(nm.second.first),
                                std::hash<std::string>()(nm.second.second)));
  return l;
}

uint32_t first_node(const ls_state* ls, const LinkObj& l) {
  return ls->name_ids.at(l.names.first.first);
}
uint32_t second_node(const ls_state* ls, const LinkObj& l) {
  return ls->name_ids.at(l.names.second.first);
}

// maybeMakeLink (LinkState.cpp:531-547): only bidirectional adjacencies
std::unique_ptr<LinkObj> bidir(ls_state* ls, uint32_t node, const AdjIn& a) {
  auto it = ls->dbs.find(a.other);
  if (it == ls->dbs.end()) return nullptr;
  for (const AdjIn& b : it->second.adjs) {
    if (b.other == node && a.other_if == b.ifname && a.ifname == b.other_if)
      return make_link(ls, node, a, a.other, b);
  }
  return nullptr;
}

LinkObj* adopt(ls_state* ls, std::unique_ptr<LinkObj> l) {
  uint32_t id;
  if (auto g = ls->ghost.find(l->names); g != ls->ghost.end()) {  // back in its old slots
    id = g->second;
    ls->ghost.erase(g);
  } else if (!ls->free_ids.empty()) {
    id = ls->free_ids.back();
    ls->free_ids.pop_back();
  } else {
    id = (uint32_t)ls->slab.size();
    ls->slab.emplace_back();
  }
  l->id = id;
  ls->slab[id] = std::move(l);
  return ls->slab[id].get();
}

void release(ls_state* ls, LinkObj* l) {
  const uint32_t id = l->id;
  if (id < ls->in_csr.size() && ls->in_csr[id]) ls->ghost[l->names] = id;  // keeps its slots
  else ls->free_ids.push_back(id);
  ls->slab[id].reset();
}

bool add_link(ls_state* ls, LinkObj* l) {
  bool ok = ls->link_map[first_node(ls, *l)].insert(l).second;
  ok &= ls->link_map[second_node(ls, *l)].insert(l).second;
  ok &= ls->all_links.insert(l).second;
  return ok;
}

bool set_node_overload(ls_state* ls, uint32_t node, bool o, Metric up, Metric down) {
  auto it = ls->node_ovl.find(node);
  if (it != ls->node_ovl.end()) return it->second.update(o, up, down);
  ls->node_ovl.emplace(node, Holdable<bool>(o));
  return false;  // a node seen for the first time never signals a change
}

bool node_overloaded(const ls_state* ls, uint32_t node) {
  auto it = ls->node_ovl.find(node);
  return it != ls->node_ovl.end() && it->second.get();
}

// updateAdjacencyDatabase (LinkState.cpp:564-719)
spf_status apply_db(ls_state* ls, uint32_t node, DbIn&& db, Metric up, Metric down,
                    ls_change* out) {
  bool topo = false, attrs = false, label;
  const bool known = ls->dbs.count(node) != 0;
  if (!known) ls->db_order_valid = false;
  DbIn& slot = ls->dbs[node];
  const int32_t prior_label = slot.node_label;
  slot = std::move(db);
  const DbIn& cur = slot;

  std::vector<LinkObj*> old_links;
  if (auto it = ls->link_map.find(node); it != ls->link_map.end())
    old_links.assign(it->second.begin(), it->second.end());
  auto by_order = [](const LinkObj* a, const LinkObj* b) { return a->before(*b); };
  std::sort(old_links.begin(), old_links.end(), by_order);

  std::vector<std::unique_ptr<LinkObj>> fresh;
  for (const AdjIn& a : cur.adjs)
    if (auto l = bidir(ls, node, a)) fresh.push_back(std::move(l));
  std::sort(fresh.begin(), fresh.end(),
            [](const std::unique_ptr<LinkObj>& a, const std::unique_ptr<LinkObj>& b) {
              return a->before(*b);
            });

  // a node overload flip alone keeps the CSR: the engine patches one byte
  const bool node_flip = set_node_overload(ls, node, cur.overload, up, down);
  label = prior_label != cur.node_label;

  size_t i = 0, j = 0;
  while (i < fresh.size() || j < old_links.size()) {
    if (i < fresh.size() && (j == old_links.size() || fresh[i]->before(*old_links[j]))) {
      fresh[i]->hold_up = up;
      topo |= fresh[i]->up();
      ls->touch(fresh[i].get());
      LinkObj* l = adopt(ls, std::move(fresh[i]));
      if (!add_link(ls, l))
        return lfail(ls, SPF_E_INVALID, "duplicate link while adding adjacency of %s",
                     ls->names[node].c_str());
      ++i;
      continue;
    }
    if (j < old_links.size() && (i == fresh.size() || old_links[j]->before(*fresh[i]))) {
      LinkObj* l = old_links[j];
      topo |= l->up();
      ls->touch(l);
      ls->link_map.at(first_node(ls, *l)).erase(l);
      ls->link_map.at(second_node(ls, *l)).erase(l);
      ls->all_links.erase(l);
      release(ls, l);
      ++j;
      continue;
    }
    // same link: apply this node's side of the attributes
    Side& o = old_links[j]->from(node);
    const Side& n = fresh[i]->from(node);
    if (n.metric.get() != o.metric.get()) {
      topo |= o.metric.update(n.metric.get(), up, down);
      ls->touch(old_links[j]);
    }
    if (n.overload.get() != o.overload.get()) {
      ls->touch(old_links[j]);
      const bool was_up = old_links[j]->up();
      o.overload.update(n.overload.get(), up, down);
      topo |= was_up != old_links[j]->up();
    }
    if (n.label != o.label) {
      attrs = true;
      o.label = n.label;
    }
    if (n.v4 != o.v4) {
      attrs = true;
      o.v4 = n.v4;
    }
    if (n.v6 != o.v6) {
      attrs = true;
      o.v6 = n.v6;
    }
    ++i;
    ++j;
  }
  if (topo) {
    clear_memo(ls);
  } else if (node_flip) {
    clear_results(ls);
  }
  // (the flatten patches these nodes' overload bits, with or without rows)
  if (node_flip) ls->pending_ovl.push_back(node);
  // a new node joins the CSR on the next flatten; like the reference, its
  // first database signals no topology change and keeps the memo
  if (!known) ls->dirty = true;
  put_change(out, topo || node_flip, attrs, label);
  return SPF_OK;
}

// CSR flatten: ids in ascending name order, edges in linksFromNode order.
spf_status flatten(ls_state* ls) {
  if (!ls->dirty) {
    // only node overload bits changed: patch them in place
    std::vector<uint32_t> nodes;
    std::vector<uint8_t> vals;
    for (uint32_t nm : ls->pending_ovl) {
      const uint32_t u = nm < ls->csr_of.size() ? ls->csr_of[nm] : kNone;
      if (u == kNone) continue;
      const uint8_t v = node_overloaded(ls, nm);
      if (ls->ovl[u] == v) continue;
      ls->ovl[u] = v;
      nodes.push_back(u);
      vals.push_back(v);
    }
    ls->pending_ovl.clear();
    if (!nodes.empty() && ls->eng && ls->engine_loaded) {
      const spf_status st = eng_set_overload(ls, nodes.data(), vals.data(), (uint32_t)nodes.size());
      if (st != SPF_OK) return eng_fail(ls, st);
    }
    return SPF_OK;
  }
  const std::vector<uint32_t> povl = std::move(ls->pending_ovl);
  ls->pending_ovl.clear();
  // the node order: the last flatten's when the node set is the same (no
  // string sort per publication), else every name sorted again
  bool same_nodes = ls->dbs.size() == ls->csr_name.size();
  if (same_nodes)
    for (const auto& kv : ls->dbs)
      if (kv.first >= ls->csr_of.size() || ls->csr_of[kv.first] == kNone) {
        same_nodes = false;
        break;
      }
  std::vector<uint32_t> ids;
  if (same_nodes) {
    ids = ls->csr_name;
  } else {
    ids.reserve(ls->dbs.size());
    for (const auto& kv : ls->dbs) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end(),
              [&](uint32_t a, uint32_t b) { return ls->names[a] < ls->names[b]; });
  }
  const uint32_t N = (uint32_t)ids.size();
  // Every link of a node -- up or down -- has a slot in its row, in
  // linksFromNode order; a down link's slot is dead (a self-loop of metric 1,
  // openr_spf.h), so a link going down or up changes the row in place.  A
  // withdrawn link keeps dead slots under its id (ghost) until the next full
  // flatten.  When every node's links still fit the slots of its row (no new
  // link identity), the changed rows are patched (spf_graph_patch_rows,
  // spf_graph_set_metric, spf_graph_set_overload); otherwise the graph reloads.
  auto slot_of = [&](const LinkObj* l, uint32_t u_name, uint32_t& col, int32_t& met) {
    if (l->up()) {
      col = ls->csr_of[l->other(u_name)];
      met = (int32_t)(uint32_t)l->from(u_name).metric.get();
    } else {
      col = ls->csr_of[u_name];
      met = 1;
    }
  };
  if (N > 0 && ls->eng && ls->engine_loaded && ids == ls->csr_name) {
    bool fits = true;
    // overload bits: only nodes whose database flipped one can differ
    std::vector<uint8_t> new_ovl(ls->ovl);
    for (uint32_t nm : povl)
      if (nm < ls->csr_of.size() && ls->csr_of[nm] != kNone) new_ovl[ls->csr_of[nm]] = node_overloaded(ls, nm);
    // the rows to rebuild: the touched nodes' (every row when unknown)
    std::vector<uint32_t> cand;
    if (ls->touched_all) {
      cand.resize(N);
      std::iota(cand.begin(), cand.end(), 0u);
    } else {
      for (uint32_t nm : ls->touched)
        if (nm < ls->csr_of.size() && ls->csr_of[nm] != kNone) cand.push_back(ls->csr_of[nm]);
      std::sort(cand.begin(), cand.end());
      cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
    }
    // the candidate rows' new slots, back to back in candidate order (the
    // CSR arrays themselves change only once the engine took the patch)
    std::vector<uint32_t> nc, nl;
    std::vector<int32_t> nmt;
    std::vector<uint8_t> used;
    for (uint32_t u : cand) {
      if (!fits) break;
      const uint32_t nm = ids[u];
      const uint32_t b = ls->row_ptr[u], e = ls->row_ptr[u + 1];
      const size_t k0 = nc.size();
      nc.resize(k0 + (e - b));
      nl.resize(k0 + (e - b));
      nmt.resize(k0 + (e - b));
      size_t k = k0;
      used.assign(e - b, 0);
      auto it = ls->link_map.find(nm);
      if (it != ls->link_map.end())
        for (const LinkObj* l : it->second) {
          uint32_t at = e;  // this link's slot in the old row
          for (uint32_t q = b; q < e; ++q)
            if (ls->link_id[q] == l->id && !used[q - b]) {
              at = q;
              break;
            }
          const uint32_t o = l->other(nm);
          if (at == e || k == k0 + (e - b) || o >= ls->csr_of.size() || ls->csr_of[o] == kNone) {
            fits = false;  // a new link, or more links than slots: reload
            break;
          }
          used[at - b] = 1;
          slot_of(l, nm, nc[k], nmt[k]);
          nl[k++] = l->id;
        }
      for (uint32_t q = b; q < e && fits; ++q)  // the withdrawn links' dead slots, in their old order
        if (!used[q - b]) {
          nc[k] = u;
          nmt[k] = 1;
          nl[k++] = ls->link_id[q];
        }
    }
    if (fits) {
      std::vector<uint32_t> rows, rcol, rlid, medges, onodes;
      std::vector<int32_t> rmet, mmet;
      std::vector<uint8_t> ovals;
      for (uint32_t nm : povl) {
        const uint32_t u = nm < ls->csr_of.size() ? ls->csr_of[nm] : kNone;
        if (u == kNone || new_ovl[u] == ls->ovl[u]) continue;
        if (std::find(onodes.begin(), onodes.end(), u) != onodes.end()) continue;
        onodes.push_back(u);
        ovals.push_back(new_ovl[u]);
      }
      size_t k0 = 0;
      for (uint32_t u : cand) {
        const uint32_t b = ls->row_ptr[u], e = ls->row_ptr[u + 1];
        bool structural = false;
        for (uint32_t q = b; q < e; ++q)
          structural |= nc[k0 + q - b] != ls->col[q] || nl[k0 + q - b] != ls->link_id[q];
        if (structural) {
          rows.push_back(u);
          rcol.insert(rcol.end(), nc.begin() + k0, nc.begin() + k0 + (e - b));
          rmet.insert(rmet.end(), nmt.begin() + k0, nmt.begin() + k0 + (e - b));
          rlid.insert(rlid.end(), nl.begin() + k0, nl.begin() + k0 + (e - b));
        } else {
          for (uint32_t q = b; q < e; ++q)
            if (nmt[k0 + q - b] != ls->metric[q]) {
              medges.push_back(q);
              mmet.push_back(nmt[k0 + q - b]);
            }
        }
        k0 += e - b;
      }
      spf_status st = SPF_OK;
      if (!rows.empty())
        st = eng_patch_rows(ls, rows.data(), (uint32_t)rows.size(), rcol.data(), rmet.data(), rlid.data());
      if (st == SPF_OK && !medges.empty())
        st = eng_set_metric(ls, medges.data(), mmet.data(), (uint32_t)medges.size());
      if (st == SPF_OK && !onodes.empty())
        st = eng_set_overload(ls, onodes.data(), ovals.data(), (uint32_t)onodes.size());
      if (st != SPF_OK) {
        ls->engine_loaded = false;
        return eng_fail(ls, st);
      }
      k0 = 0;  // the engine has the patch: the host CSR follows
      for (uint32_t u : cand) {
        const uint32_t b = ls->row_ptr[u], e = ls->row_ptr[u + 1];
        std::copy(nc.begin() + k0, nc.begin() + k0 + (e - b), ls->col.begin() + b);
        std::copy(nmt.begin() + k0, nmt.begin() + k0 + (e - b), ls->metric.begin() + b);
        std::copy(nl.begin() + k0, nl.begin() + k0 + (e - b), ls->link_id.begin() + b);
        k0 += e - b;
      }
      ls->ovl.swap(new_ovl);
      if (!rows.empty()) {
        ++ls->row_patches;
        static std::atomic<uint64_t> next_patch_epoch{1ull << 62};
        ls->flat_epoch = ++next_patch_epoch;  // link ids / cols of rows moved (ls_graph_epoch)
        if (ls->all) {  // the resident pass's layout may have changed: rebuilt on demand
          spf_mplan_destroy(ls->all);
          ls->all = nullptr;
        }
      }
      ls->dirty = false;
      ls->touched.clear();
      ls->touched_all = false;
      return SPF_OK;
    }
  }
  ls->touched.clear();
  ls->touched_all = false;
  // full flatten: every link in a slot, no ghosts (their ids are free again)
  for (const auto& g : ls->ghost) ls->free_ids.push_back(g.second);
  ls->ghost.clear();
  ls->csr_name = ids;
  ls->csr_of.assign(ls->names.size(), kNone);
  for (uint32_t i = 0; i < ids.size(); ++i) ls->csr_of[ids[i]] = i;
  ls->row_ptr.assign(N + 1, 0);
  ls->col.clear();
  ls->metric.clear();
  ls->link_id.clear();
  ls->edge_tail.clear();
  ls->ovl.assign(N, 0);
  ls->in_csr.assign(ls->slab.size(), 0);
  for (uint32_t u = 0; u < N; ++u) {
    const uint32_t nm = ids[u];
    ls->ovl[u] = node_overloaded(ls, nm);
    auto it = ls->link_map.find(nm);
    if (it != ls->link_map.end()) {
      for (const LinkObj* l : it->second) {
        const uint32_t v = ls->csr_of[l->other(nm)];
        if (v == kNone) return lfail(ls, SPF_E_INVALID, "link to node without a database");
        uint32_t c;
        int32_t m;
        slot_of(l, nm, c, m);
        ls->col.push_back(c);
        ls->metric.push_back(m);
        ls->link_id.push_back(l->id);
        ls->edge_tail.push_back(u);
        ls->in_csr[l->id] = 1;
      }
    }
    ls->row_ptr[u + 1] = (uint32_t)ls->col.size();
  }
  ls->engine_loaded = false;
  // names, row_ptr, col or link ids changed: a process-wide counter, so no
  // two flattened graphs of any two states share an epoch
  static std::atomic<uint64_t> next_epoch{0};
  ls->flat_epoch = ++next_epoch;
  if (N > 0 && ls->eng) {
    spf_graph g;
    g.n_nodes = N;
    g.n_edges = (uint32_t)ls->col.size();
    g.row_ptr = ls->row_ptr.data();
    g.col = ls->col.data();
    g.metric = ls->metric.data();
    g.link_id = ls->link_id.data();
    g.overloaded = ls->ovl.data();
    const spf_status st = eng_load(ls, &g);
    if (st != SPF_OK) return eng_fail(ls, st);
    ls->engine_loaded = true;
  }
  ls->dirty = false;
  return SPF_OK;
}

void fill_view(const SpfMemo& m, ls_spf_view* out) {
  out->n = (uint32_t)m.node.size();
  out->node = m.node.data();
  out->metric = m.metric.data();
  out->nh_ptr = m.nh_ptr.data();
  out->nh_node = m.nh_node.data();
  out->pl_ptr = m.pl_ptr.data();
  out->pl_link = m.pl_link.data();
  out->pl_prev = m.pl_prev.data();
}

// Weighted solves the data-parallel kernels cannot answer exactly (zero or
// negative metrics, u64 distances) run the engine's exact kernel, which also
// reports the Dijkstra pop order; pathLinks follow from it.
bool needs_exact(const ls_state* ls, bool ulm) {
  return ulm && (spf_graph_has_nonpositive_metric(ls->eng) || spf_graph_needs_dist64(ls->eng));
}

// runSpf(s, ulm, ignore) on the exact kernel: u64 distances (UINT64_MAX =
// unreachable), next-hop bitmaps (nh may be NULL) and pathLinks as csr edge
// ids: the tight up in-edges (u -> v) of expanded u popped before v, in
// (pop order of u, linksFromNode order) -- LinkState.cpp:857-873.
spf_status exact_spf(ls_state* ls, uint32_t s, bool ulm, const std::vector<uint32_t>& ignore,
                     std::vector<uint64_t>& dist, std::vector<uint32_t>* nh,
                     std::vector<uint32_t>& pred_ptr, std::vector<uint32_t>& pred_edge) {
  const uint32_t N = (uint32_t)ls->csr_name.size();
  const uint32_t flags = ulm ? 0u : SPF_FLAG_HOP_COUNT;
  std::vector<uint32_t> pop(N);
  dist.assign(N, 0);
  spf_status st = spf_solve_exact(ls->eng, s, flags, ignore.empty() ? nullptr : ignore.data(),
                                  (uint32_t)ignore.size(), dist.data(), nullptr,
                                  nh ? nh->data() : nullptr, pop.data());
  if (st != SPF_OK) return eng_fail(ls, st);
  std::unordered_set<uint32_t> ign(ignore.begin(), ignore.end());
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> in(N);  // (pop(u), edge)
  for (uint32_t u = 0; u < N; ++u) {
    if (pop[u] == SPF_UNREACHABLE || (ls->ovl[u] && u != s)) continue;  // not expanded
    for (uint32_t e = ls->row_ptr[u]; e < ls->row_ptr[u + 1]; ++e) {
      const uint32_t v = ls->col[e];
      if (pop[v] == SPF_UNREACHABLE || pop[v] <= pop[u] || ign.count(ls->link_id[e])) continue;
      const uint64_t w = ulm ? (uint64_t)(int64_t)ls->metric[e] : 1ull;
      if (dist[u] + w == dist[v]) in[v].emplace_back(pop[u], e);
    }
  }
  pred_ptr.assign(N + 1, 0);
  pred_edge.clear();
  for (uint32_t v = 0; v < N; ++v) {
    std::sort(in[v].begin(), in[v].end());
    for (const auto& pe : in[v]) pred_edge.push_back(pe.second);
    pred_ptr[v + 1] = (uint32_t)pred_edge.size();
  }
  return SPF_OK;
}

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// A source's memo entry from its engine output: csr distance row, its
// next-hop bitmaps (k of pitch/32 words, bitmap j = destinations routed via
// neighbour nbr[j]) and its pathLinks (csr-indexed pred_ptr / pred_edge;
// d64 = u64 distances of exact solves, else empty).
void fill_memo(const ls_state* ls, const uint32_t* dist, const std::vector<uint64_t>& d64,
               const uint32_t* nh, uint32_t k, uint32_t wpm, const std::vector<uint32_t>& nbr,
               const uint32_t* pred_ptr, const uint32_t* pred_edge, SpfMemo& m) {
  const uint32_t N = (uint32_t)ls->csr_name.size();
  // next hops per destination from the per-neighbour bitmaps: set bits
  // counted, then placed in neighbour order -- O(k * N/32 + bits), not O(k * N)
  const uint32_t nw = (N + 31) / 32, nv = nw * 32;  // bitmap words / nodes they cover
  std::vector<uint32_t> at(nv + 1, 0);
  for (uint32_t j = 0; j < k; ++j)
    for (uint32_t w = 0; w < nw; ++w)
      for (uint32_t x = nh[(size_t)j * wpm + w]; x; x &= x - 1) ++at[w * 32 + __builtin_ctz(x) + 1];
  for (uint32_t v = 0; v < nv; ++v) at[v + 1] += at[v];
  std::vector<uint32_t> nh_of(at[nv]);
  {
    std::vector<uint32_t> fill(at.begin(), at.end() - 1);
    for (uint32_t j = 0; j < k; ++j)
      for (uint32_t w = 0; w < nw; ++w)
        for (uint32_t x = nh[(size_t)j * wpm + w]; x; x &= x - 1) nh_of[fill[w * 32 + __builtin_ctz(x)]++] = j;
  }
  m.node.reserve(N);
  m.metric.reserve(N);
  m.nh_ptr.reserve(N + 1);
  m.pl_ptr.reserve(N + 1);
  m.nh_node.reserve(at[nv]);
  for (uint32_t v = 0; v < N; ++v) {
    if (dist[v] == SPF_UNREACHABLE) continue;
    m.node.push_back(ls->csr_name[v]);
    m.metric.push_back(d64.empty() ? (uint64_t)dist[v] : d64[v]);
    for (uint32_t t = at[v]; t < at[v + 1]; ++t) m.nh_node.push_back(ls->csr_name[nbr[nh_of[t]]]);
    m.nh_ptr.push_back((uint32_t)m.nh_node.size());
    if (pred_ptr)
      for (uint32_t p = pred_ptr[v]; p < pred_ptr[v + 1]; ++p) {
        const uint32_t e = pred_edge[p];
        m.pl_link.push_back(ls->link_id[e]);
        m.pl_prev.push_back(ls->csr_name[ls->edge_tail[e]]);
      }
    m.pl_ptr.push_back((uint32_t)m.pl_link.size());
  }
}

std::vector<uint32_t> src_neighbors(const ls_state* ls, uint32_t s) {
  uint32_t k = 0;
  spf_src_neighbors(ls->eng, s, nullptr, 0, &k);
  std::vector<uint32_t> nbr(k);
  spf_src_neighbors(ls->eng, s, nbr.data(), k, &k);
  return nbr;
}

// pathLinks of a memo entry made without them (ls_get_spf_metrics): the
// predecessor lists from the resident row, or from one more solve of the same
// source on the unchanged graph (the memo is dropped on any change) -- the
// same run as far as decision.spf_runs goes
spf_status fill_pathlinks(ls_state* ls, uint32_t node, bool ulm, SpfMemo& m) {
  const uint32_t s = node < ls->csr_of.size() ? ls->csr_of[node] : kNone;
  m.pl_missing = 0;
  if (s == kNone) return SPF_OK;  // off-graph source: no pathLinks
  const uint32_t N = (uint32_t)ls->csr_name.size();
  m.pred_ptr.resize(N + 1);
  ls->pred_scratch.resize(std::max<size_t>(ls->edge_tail.size(), 1));
  spf_status st;
  if (ls->all && ls->all_valid && ls->all_ulm == (ulm ? 1 : 0)) {
    uint32_t npred = 0;
    st = spf_mplan_preds(ls->all, s, m.pred_ptr.data(), ls->pred_scratch.data(),
                         (uint32_t)ls->pred_scratch.size(), &npred);
    if (st != SPF_OK) return eng_fail(ls, st);
    m.pred_edge.assign(ls->pred_scratch.begin(), ls->pred_scratch.begin() + npred);
  } else {
    spf_plan* raw = nullptr;
    st = spf_plan_create(ls->eng, &s, 1, ulm ? 0u : SPF_FLAG_HOP_COUNT, &raw);
    if (st != SPF_OK) return eng_fail(ls, st);
    std::unique_ptr<spf_plan, void (*)(spf_plan*)> plan(raw, spf_plan_destroy);
    std::vector<uint32_t> dist(N), nh(std::max<uint64_t>(spf_plan_nh_words(plan.get()), 1));
    st = spf_plan_execute_host(plan.get(), dist.data(), nh.data());
    if (st != SPF_OK) return eng_fail(ls, st);
    uint64_t npred = 0;
    st = spf_plan_preds(plan.get(), m.pred_ptr.data(), ls->pred_scratch.data(), ls->pred_scratch.size(),
                        &npred);
    if (st != SPF_OK) return eng_fail(ls, st);
    m.pred_edge.assign(ls->pred_scratch.begin(), ls->pred_scratch.begin() + npred);
  }
  m.pl_ptr.assign(1, 0);
  m.pl_link.clear();
  m.pl_prev.clear();
  for (uint32_t v = 0; v < N; ++v) {
    if (m.dist[v] == SPF_UNREACHABLE) continue;  // m.node's order: reached csr ids ascending
    for (uint32_t p = m.pred_ptr[v]; p < m.pred_ptr[v + 1]; ++p) {
      const uint32_t e = m.pred_edge[p];
      m.pl_link.push_back(ls->link_id[e]);
      m.pl_prev.push_back(ls->csr_name[ls->edge_tail[e]]);
    }
    m.pl_ptr.push_back((uint32_t)m.pl_link.size());
  }
  return SPF_OK;
}

// getSpfResult (LinkState.cpp:793-803) -> memo entry; need_pl = false leaves
// the pathLinks of a new entry to the first caller that needs them
spf_status spf_result(ls_state* ls, uint32_t node, bool ulm, const SpfMemo** out, bool need_pl = true) {
  auto key = std::make_pair(node, (int)ulm);
  auto it = ls->spf_memo.find(key);
  if (it != ls->spf_memo.end()) {
    if (it->second.pending) {  // prefetched: this is the reference's runSpf call
      it->second.pending = 0;
      ls->spf_runs++;
    }
    if (need_pl && it->second.pl_missing) {
      const spf_status st = fill_pathlinks(ls, node, ulm, it->second);
      if (st != SPF_OK) return st;
    }
    *out = &it->second;
    return SPF_OK;
  }
  spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  if (!ls->eng) return lfail(ls, SPF_E_NO_DEVICE, "LinkState created host-only (device < 0)");
  SpfMemo m;
  ls->spf_runs++;  // decision.spf_runs (LinkState.cpp:815)
  const uint32_t s = node < ls->csr_of.size() ? ls->csr_of[node] : kNone;
  if (s == kNone) {
    // not in the graph: the reference's Dijkstra records only the source
    m.node.push_back(node);
    m.metric.push_back(0);
    m.nh_ptr.push_back(0);
    m.pl_ptr.push_back(0);
  } else {
    const uint32_t N = (uint32_t)ls->csr_name.size();
    const uint32_t flags = ulm ? 0u : SPF_FLAG_HOP_COUNT;
    const std::vector<uint32_t> nbr = src_neighbors(ls, s);
    const uint32_t k = (uint32_t)nbr.size();
    const uint32_t pitch = spf_row_pitch(ls->eng);
    const uint32_t wpm = pitch / 32;  // u32 words per destination bitmap
    const uint64_t words = (uint64_t)k * wpm;
    m.dist.resize(N);
    std::vector<uint32_t> nh(std::max<uint64_t>(words, 1));
    std::vector<uint64_t> d64;
    uint64_t t0 = now_ns();
    if (ls->all && ls->all_valid && ls->all_ulm == (ulm ? 1 : 0)) {
      // answered by the GPU holding the resident all-sources pass (every
      // csr node is a source of `all`, request index = csr id)
      st = spf_mplan_read(ls->all, s, m.dist.data(), nh.data());
      if (st != SPF_OK) return eng_fail(ls, st);
      uint64_t t1 = now_ns();
      ls->phase_ns[1] += t1 - t0;
      if (need_pl) {
        m.pred_ptr.resize(N + 1);
        uint32_t npred = 0;
        ls->pred_scratch.resize(std::max<size_t>(ls->edge_tail.size(), 1));
        st = spf_mplan_preds(ls->all, s, m.pred_ptr.data(), ls->pred_scratch.data(),
                             (uint32_t)ls->pred_scratch.size(), &npred);
        if (st != SPF_OK) return eng_fail(ls, st);
        m.pred_edge.assign(ls->pred_scratch.begin(), ls->pred_scratch.begin() + npred);
      } else {
        m.pl_missing = 1;
      }
      t0 = now_ns();
      ls->phase_ns[2] += t0 - t1;
    } else if (needs_exact(ls, ulm)) {
      st = exact_spf(ls, s, ulm, {}, d64, &nh, m.pred_ptr, m.pred_edge);
      if (st != SPF_OK) return st;
      for (uint32_t v = 0; v < N; ++v)  // csr-indexed reachability for path tracing
        m.dist[v] = d64[v] == SPF_UNREACHABLE64 ? SPF_UNREACHABLE : 0u;
      ls->phase_ns[1] += now_ns() - t0;
    } else {
      spf_plan* raw = nullptr;
      st = spf_plan_create(ls->eng, &s, 1, flags, &raw);
      if (st != SPF_OK) return eng_fail(ls, st);
      std::unique_ptr<spf_plan, void (*)(spf_plan*)> plan(raw, spf_plan_destroy);
      uint64_t t1 = now_ns();
      ls->phase_ns[0] += t1 - t0;
      st = spf_plan_execute_host(plan.get(), m.dist.data(), nh.data());
      if (st != SPF_OK) return eng_fail(ls, st);
      t0 = now_ns();
      ls->phase_ns[1] += t0 - t1;
      if (need_pl) {
        m.pred_ptr.resize(N + 1);
        uint64_t npred = 0;
        ls->pred_scratch.resize(std::max<size_t>(ls->edge_tail.size(), 1));
        st = spf_plan_preds(plan.get(), m.pred_ptr.data(), ls->pred_scratch.data(),
                            ls->pred_scratch.size(), &npred);
        if (st != SPF_OK) return eng_fail(ls, st);
        m.pred_edge.assign(ls->pred_scratch.begin(), ls->pred_scratch.begin() + npred);
      } else {
        m.pl_missing = 1;
      }
      ls->phase_ns[2] += now_ns() - t0;
    }
    t0 = now_ns();
    fill_memo(ls, m.dist.data(), d64, nh.data(), k, wpm, nbr,
              m.pred_ptr.empty() ? nullptr : m.pred_ptr.data(), m.pred_edge.data(), m);
    ls->phase_ns[3] += now_ns() - t0;
  }
  *out = &ls->spf_memo.emplace(key, std::move(m)).first->second;
  return SPF_OK;
}

// traceOnePath (LinkState.cpp:398-419) over csr predecessor lists
bool trace(const ls_state* ls, uint32_t src, uint32_t dst, const std::vector<uint32_t>& pred_ptr,
           const std::vector<uint32_t>& pred_edge, std::unordered_set<uint32_t>& used,
           std::vector<uint32_t>& path) {
  if (src == dst) return true;
  for (uint32_t p = pred_ptr[dst]; p < pred_ptr[dst + 1]; ++p) {
    const uint32_t e = pred_edge[p];
    if (!used.insert(ls->link_id[e]).second) continue;
    if (trace(ls, src, ls->edge_tail[e], pred_ptr, pred_edge, used, path)) {
      path.push_back(ls->link_id[e]);
      return true;
    }
  }
  return false;
}

spf_status kth_paths(ls_state* ls, uint32_t src, uint32_t dst, uint64_t k, const PathMemo** out) {
  auto key = std::make_tuple(src, dst, k);
  auto it = ls->ksp_memo.find(key);
  if (it != ls->ksp_memo.end()) {
    PathMemo& m = it->second;
    if (m.pending) {  // prefetched: settle the reference's side effects
      m.pending = 0;
      if (k == 1) {
        const SpfMemo* sm = nullptr;
        const spf_status st = spf_result(ls, src, true, &sm);
        if (st != SPF_OK) return st;
      } else {
        const PathMemo* k1 = nullptr;
        const spf_status st = kth_paths(ls, src, dst, 1, &k1);
        if (st != SPF_OK) return st;
        if (!k1->link.empty()) ls->spf_runs++;  // LinkState.cpp:778-779
      }
    }
    *out = &m;
    return SPF_OK;
  }
  std::vector<uint32_t> ignore;
  {
    std::unordered_set<uint32_t> seen;
    for (uint64_t i = 1; i < k; ++i) {
      const PathMemo* pm = nullptr;
      const spf_status st = kth_paths(ls, src, dst, i, &pm);
      if (st != SPF_OK) return st;
      for (uint32_t l : pm->link)
        if (seen.insert(l).second) ignore.push_back(l);
    }
  }
  PathMemo res;
  const std::vector<uint32_t>* pptr = nullptr;
  const std::vector<uint32_t>* pedge = nullptr;
  std::vector<uint32_t> dist, my_ptr, my_edge;
  bool reachable = false;
  uint32_t s = kNone, d = kNone;
  if (ignore.empty()) {
    const SpfMemo* m = nullptr;
    const spf_status st = spf_result(ls, src, true, &m);
    if (st != SPF_OK) return st;
    s = src < ls->csr_of.size() ? ls->csr_of[src] : kNone;
    d = dst < ls->csr_of.size() ? ls->csr_of[dst] : kNone;
    if (s != kNone && d != kNone) {
      reachable = m->dist[d] != SPF_UNREACHABLE;
      pptr = &m->pred_ptr;
      pedge = &m->pred_edge;
    }
  } else {
    spf_status st = flatten(ls);
    if (st != SPF_OK) return st;
    if (!ls->eng) return lfail(ls, SPF_E_NO_DEVICE, "LinkState created host-only (device < 0)");
    s = ls->csr_of[src];
    d = ls->csr_of[dst];
    ls->spf_runs++;  // the un-memoised runSpf of LinkState.cpp:778-779
    const uint32_t N = (uint32_t)ls->csr_name.size();
    dist.resize(N);
    if (needs_exact(ls, true)) {
      std::vector<uint64_t> d64;
      st = exact_spf(ls, s, true, ignore, d64, nullptr, my_ptr, my_edge);
      if (st != SPF_OK) return st;
      reachable = d64[d] != SPF_UNREACHABLE64;
      pptr = &my_ptr;
      pedge = &my_edge;
    } else {
      st = spf_sssp(ls->eng, s, 0, ignore.data(), (uint32_t)ignore.size(), dist.data());
      if (st != SPF_OK) return eng_fail(ls, st);
      reachable = dist[d] != SPF_UNREACHABLE;
    }
    if (reachable && !pptr) {
      uint32_t np = 0;
      my_ptr.resize(N + 1);
      st = spf_preds(ls->eng, s, 0, ignore.data(), (uint32_t)ignore.size(), dist.data(),
                     my_ptr.data(), nullptr, 0, &np);
      if (st != SPF_OK) return eng_fail(ls, st);
      my_edge.resize(np);
      st = spf_preds(ls->eng, s, 0, ignore.data(), (uint32_t)ignore.size(), dist.data(),
                     my_ptr.data(), my_edge.data(), np, &np);
      if (st != SPF_OK) return eng_fail(ls, st);
      pptr = &my_ptr;
      pedge = &my_edge;
    }
  }
  if (reachable && s != d) {
    std::unordered_set<uint32_t> used;
    for (;;) {
      std::vector<uint32_t> path;
      if (!trace(ls, s, d, *pptr, *pedge, used, path) || path.empty()) break;
      res.link.insert(res.link.end(), path.begin(), path.end());
      res.path_ptr.push_back((uint32_t)res.link.size());
    }
  }
  *out = &ls->ksp_memo.emplace(key, std::move(res)).first->second;
  return SPF_OK;
}

spf_status read_lsdb(ls_state* ls, const openr_lsdb* in, uint32_t d, uint32_t* node, DbIn* db) {
  const openr_db_rec& r = in->dbs[d];
  *node = ls->intern(std::string(in->blob + r.name_off, r.name_len));
  db->overload = r.is_overloaded != 0;
  db->node_label = r.node_label;
  db->adjs.clear();
  db->adjs.reserve(r.adj_count);
  for (uint32_t k = 0; k < r.adj_count; ++k) {
    const openr_adj_rec& a = in->adjs[r.adj_begin + k];
    AdjIn x;
    x.other = ls->intern(std::string(in->blob + a.other_off, a.other_len));
    x.ifname.assign(in->blob + a.if_off, a.if_len);
    x.other_if.assign(in->blob + a.oif_off, a.oif_len);
    x.metric = a.metric;
    x.label = a.adj_label;
    x.overload = a.is_overloaded != 0;
    std::memcpy(x.v4.data(), a.nh_v4, 4);
    std::memcpy(x.v6.data(), a.nh_v6, 16);
    db->adjs.push_back(std::move(x));
  }
  return SPF_OK;
}

}  // namespace

extern "C" {

spf_status ls_create_multi(const char* area, const int* gpu_ids, uint32_t n, ls_state** out) {
  if (!out || !gpu_ids || n == 0) return SPF_E_INVALID;
  *out = nullptr;
  auto ls = std::make_unique<ls_state>();
  ls->area = area ? area : "0";
  ls->device = gpu_ids[0];
  const spf_status st = spf_mctx_create(gpu_ids, n, &ls->meng);
  if (st != SPF_OK) return st;  // spf_global_error() has the reason
  ls->eng = spf_mctx_member(ls->meng, 0);
  *out = ls.release();
  return SPF_OK;
}

// getSpfResult for every node, as Decision::getDecisionRouteDb asks for each
// node of the area (Decision.cpp:1480-1500): one all-sources pass split over
// the GPUs, results resident on the owning GPU until the next graph change.
spf_status ls_prefetch_all_sources(ls_state* ls, int ulm) {
  if (!ls) return SPF_E_INVALID;
  spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  if (!ls->eng) return lfail(ls, SPF_E_NO_DEVICE, "LinkState created host-only (device < 0)");
  if (!ls->meng) return lfail(ls, SPF_E_STATE, "ls_prefetch_all_sources needs ls_create_multi");
  if (needs_exact(ls, ulm != 0)) return SPF_OK;  // the exact kernel answers node by node
  const uint32_t N = (uint32_t)ls->csr_name.size();
  if (N == 0) return SPF_OK;
  const uint32_t flags = ulm ? 0u : SPF_FLAG_HOP_COUNT;
  if (ls->all && ls->all_ulm != (ulm != 0 ? 1 : 0)) {
    spf_mplan_destroy(ls->all);
    ls->all = nullptr;
  }
  if (!ls->all) {
    std::vector<uint32_t> srcs(N);
    std::iota(srcs.begin(), srcs.end(), 0u);
    st = spf_mplan_create(ls->meng, srcs.data(), N, flags, SPF_PARTITION_AUTO, &ls->all);
    if (st != SPF_OK) return eng_fail(ls, st);
    ls->all_ulm = ulm != 0 ? 1 : 0;
  }
  ls->all_valid = false;
  st = spf_mplan_execute(ls->all);
  if (st == SPF_OK) st = spf_mplan_synchronize(ls->all);
  if (st != SPF_OK) return eng_fail(ls, st);
  ls->all_valid = true;
  return SPF_OK;
}

spf_mplan* ls_all_sources_plan(ls_state* ls) { return ls && ls->all_valid ? ls->all : nullptr; }

spf_status ls_create(const char* area, int device, ls_state** out) {
  if (!out) return SPF_E_INVALID;
  *out = nullptr;
  auto ls = std::make_unique<ls_state>();
  ls->area = area ? area : "0";
  ls->device = device;
  if (device >= 0) {  // device < 0: host-only (LSDB + flatten, no solves)
    const spf_status st = spf_ctx_create(device, &ls->eng);
    if (st != SPF_OK) return st;  // spf_global_error() has the reason
  }
  *out = ls.release();
  return SPF_OK;
}

void ls_destroy(ls_state* ls) {
  if (!ls) return;
  spf_mplan_destroy(ls->all);
  if (ls->meng)
    spf_mctx_destroy(ls->meng);  // owns eng
  else
    spf_ctx_destroy(ls->eng);
  delete ls;
}

const char* ls_last_error(const ls_state* ls) {
  return ls ? ls->err.c_str() : spf_global_error();
}

const char* ls_get_area(const ls_state* ls) { return ls ? ls->area.c_str() : nullptr; }

spf_status ls_update_adjacency_databases(ls_state* ls, const openr_lsdb* lsdb, uint64_t up,
                                         uint64_t down, ls_change* changes) {
  if (!ls || !lsdb) return SPF_E_INVALID;
  for (uint32_t d = 0; d < lsdb->n_dbs; ++d) {
    uint32_t node;
    DbIn db;
    spf_status st = read_lsdb(ls, lsdb, d, &node, &db);
    if (st != SPF_OK) return st;
    st = apply_db(ls, node, std::move(db), up, down, changes ? changes + d : nullptr);
    if (st != SPF_OK) return st;
  }
  return SPF_OK;
}

// deleteAdjacencyDatabase (LinkState.cpp:721-738) + removeNode (:436-455)
spf_status ls_delete_adjacency_database(ls_state* ls, const char* node, ls_change* change) {
  if (!ls || !node) return SPF_E_INVALID;
  const uint32_t* id = ls->find_name(node);
  if (!id || !ls->dbs.count(*id)) {
    put_change(change, false, false, false);
    return SPF_OK;
  }
  const uint32_t n = *id;
  auto it = ls->link_map.find(n);
  if (it != ls->link_map.end()) {
    std::vector<LinkObj*> doomed(it->second.begin(), it->second.end());
    for (LinkObj* l : it->second) {
      ls->link_map.at(l->other(n)).erase(l);
      ls->all_links.erase(l);
    }
    ls->link_map.erase(it);
    ls->node_ovl.erase(n);
    for (LinkObj* l : doomed) release(ls, l);
  }
  ls->dbs.erase(n);
  ls->db_order_valid = false;
  ls->touched_all = true;
  clear_memo(ls);
  put_change(change, true, false, false);
  return SPF_OK;
}

spf_status ls_decrement_holds(ls_state* ls, ls_change* change) {
  if (!ls) return SPF_E_INVALID;
  bool topo = false;
  for (LinkObj* l : ls->all_links)
    if (l->tick()) {
      topo = true;
      ls->touch(l);
    }
  for (auto& kv : ls->node_ovl) topo |= kv.second.tick();
  if (topo) clear_memo(ls);
  put_change(change, topo, false, false);
  return SPF_OK;
}

int ls_has_holds(const ls_state* ls) {
  for (const LinkObj* l : ls->all_links)
    if (l->holds()) return 1;
  for (const auto& kv : ls->node_ovl)
    if (kv.second.has_hold()) return 1;
  return 0;
}
uint64_t ls_num_links(const ls_state* ls) { return ls->all_links.size(); }
uint64_t ls_num_nodes(const ls_state* ls) { return ls->link_map.size(); }
int ls_has_node(const ls_state* ls, const char* node) {
  const uint32_t* id = ls->find_name(node);
  return id && ls->dbs.count(*id);
}
spf_status ls_adjacency_databases(const ls_state* ls, uint32_t* name_ids, int32_t* node_labels,
                                  uint32_t cap, uint32_t* count) {
  if (!ls || !count) return SPF_E_INVALID;
  if (!ls->db_order_valid) {  // re-sorted only when a database appears or goes
    auto* mls = const_cast<ls_state*>(ls);
    mls->db_order.clear();
    mls->db_order.reserve(ls->dbs.size());
    for (const auto& kv : ls->dbs) mls->db_order.push_back(kv.first);
    std::sort(mls->db_order.begin(), mls->db_order.end(),
              [&](uint32_t a, uint32_t b) { return ls->names[a] < ls->names[b]; });
    mls->db_order_valid = true;
  }
  const std::vector<uint32_t>& ids = ls->db_order;
  *count = (uint32_t)ids.size();
  for (uint32_t i = 0; i < ids.size() && i < cap; ++i) {
    if (name_ids) name_ids[i] = ids[i];
    if (node_labels) node_labels[i] = ls->dbs.at(ids[i]).node_label;
  }
  return SPF_OK;
}

int ls_is_node_overloaded(const ls_state* ls, const char* node) {
  const uint32_t* id = ls->find_name(node);
  return id && node_overloaded(ls, *id);
}
int ls_is_node_overloaded_id(const ls_state* ls, uint32_t id) { return ls && node_overloaded(ls, id); }
uint32_t ls_name_id(ls_state* ls, const char* name) { return ls->intern(name); }
const char* ls_name(const ls_state* ls, uint32_t id) {
  return id < ls->names.size() ? ls->names[id].c_str() : nullptr;
}

spf_status ls_links_from_node(const ls_state* ls, const char* node, uint32_t* ids, uint32_t cap,
                              uint32_t* count) {
  if (!ls || !node || !count) return SPF_E_INVALID;
  *count = 0;
  const uint32_t* id = ls->find_name(node);
  if (!id) return SPF_OK;
  auto it = ls->link_map.find(*id);
  if (it == ls->link_map.end()) return SPF_OK;
  uint32_t n = 0;
  for (const LinkObj* l : it->second) {
    if (ids && n < cap) ids[n] = l->id;
    ++n;
  }
  *count = n;
  return SPF_OK;
}

spf_status ls_link_info(const ls_state* ls, uint32_t link_id, ls_link_desc* out) {
  if (!ls || !out) return SPF_E_INVALID;
  if (link_id >= ls->slab.size() || !ls->slab[link_id]) return SPF_E_INVALID;
  const LinkObj& l = *ls->slab[link_id];
  out->node1 = l.s[0].node;
  out->node2 = l.s[1].node;
  out->if1 = l.s[0].ifname.c_str();
  out->if2 = l.s[1].ifname.c_str();
  out->first_node = first_node(ls, l);
  out->second_node = second_node(ls, l);
  out->metric1 = l.s[0].metric.get();
  out->metric2 = l.s[1].metric.get();
  out->adj_label1 = l.s[0].label;
  out->adj_label2 = l.s[1].label;
  out->overload1 = l.s[0].overload.get();
  out->overload2 = l.s[1].overload.get();
  out->is_up = l.up();
  out->pad = 0;
  out->hash = l.hash;
  out->nh_v4_1 = l.s[0].v4.data();
  out->nh_v4_2 = l.s[1].v4.data();
  out->nh_v6_1 = l.s[0].v6.data();
  out->nh_v6_2 = l.s[1].v6.data();
  return SPF_OK;
}

spf_status ls_get_spf_result(ls_state* ls, const char* node, int ulm, ls_spf_view* out) {
  if (!ls || !node || !out) return SPF_E_INVALID;
  const SpfMemo* m = nullptr;
  const spf_status st = spf_result(ls, ls->intern(node), ulm != 0, &m);
  if (st != SPF_OK) return st;
  fill_view(*m, out);
  return SPF_OK;
}

spf_status ls_get_spf_metrics(ls_state* ls, const char* node, int ulm, ls_spf_view* out) {
  if (!ls || !node || !out) return SPF_E_INVALID;
  const SpfMemo* m = nullptr;
  const spf_status st = spf_result(ls, ls->intern(node), ulm != 0, &m, false);
  if (st != SPF_OK) return st;
  fill_view(*m, out);
  if (m->pl_missing) out->pl_ptr = out->pl_link = out->pl_prev = nullptr;
  return SPF_OK;
}

spf_status ls_get_kth_paths(ls_state* ls, const char* src, const char* dst, uint64_t k,
                            ls_paths_view* out) {
  if (!ls || !src || !dst || !out) return SPF_E_INVALID;
  if (k < 1) return lfail(ls, SPF_E_INVALID, "getKthPaths: k must be >= 1 (CHECK_GE, LinkState.cpp:765)");
  const PathMemo* pm = nullptr;
  const spf_status st = kth_paths(ls, ls->intern(src), ls->intern(dst), k, &pm);
  if (st != SPF_OK) return st;
  out->n_paths = (uint32_t)pm->path_ptr.size() - 1;
  out->path_ptr = pm->path_ptr.data();
  out->link = pm->link.data();
  return SPF_OK;
}

// getKthPaths(src, d, 1) and (src, d, 2) for every node d in one batched
// KSP2 launch (spf_ksp2_solve), stored in the memo; SpfSolver calls it
// before building KSP2_ED_ECMP routes (Decision.cpp:895-1018 queries every
// advertiser of every such prefix).
spf_status ls_prefetch_kth_paths(ls_state* ls, const char* src_c) {
  if (!ls || !src_c) return SPF_E_INVALID;
  spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  if (!ls->eng) return lfail(ls, SPF_E_NO_DEVICE, "LinkState created host-only (device < 0)");
  const uint32_t src = ls->intern(src_c);
  const uint32_t s = src < ls->csr_of.size() ? ls->csr_of[src] : kNone;
  if (s == kNone) return SPF_OK;  // not in the graph: every query is empty anyway
  // (zero / negative metrics, u64 labels, big graphs: the engine's KSP2
  // plan runs on the exact kernel, same output)
  const uint32_t N = (uint32_t)ls->csr_name.size();
  std::vector<spf_ksp2_pair> pairs(N);
  std::vector<uint32_t> pool;
  uint64_t used = 0;
  st = spf_ksp2_solve(ls->eng, &s, 1, pairs.data(), nullptr, 0, &used);
  if (st != SPF_OK && st != SPF_E_NOMEM) return eng_fail(ls, st);
  pool.resize(std::max<uint64_t>(used, 1));
  st = spf_ksp2_solve(ls->eng, &s, 1, pairs.data(), pool.data(), pool.size(), &used);
  if (st != SPF_OK) return eng_fail(ls, st);
  for (uint32_t d = 0; d < N; ++d) {
    const uint32_t dst = ls->csr_name[d];
    for (uint32_t k = 1; k <= 2; ++k) {
      auto key = std::make_tuple(src, dst, (uint64_t)k);
      if (ls->ksp_memo.count(key)) continue;
      PathMemo m;
      uint32_t at = pairs[d].first[k - 1];
      for (uint32_t p = 0; p < pairs[d].n_paths[k - 1] && at != SPF_KSP2_NONE; ++p) {
        const uint32_t n = pool[at], next = pool[at + 1];
        m.link.insert(m.link.end(), pool.begin() + at + 2, pool.begin() + at + 2 + n);
        m.path_ptr.push_back((uint32_t)m.link.size());
        at = next;
      }
      m.pending = 1;
      ls->ksp_memo.emplace(key, std::move(m));
    }
  }
  return SPF_OK;
}

// getSpfResult for several nodes in one batched plan (the SPF analogue of
// ls_prefetch_kth_paths): SpfSolver's LFA asks for getSpfResult(me) and then
// getSpfResult(n) for every neighbour n (Decision.cpp:1158-1165).  The memo
// entries are marked pending: decision.spf_runs is counted when each is
// first read, as if it had been computed then.
spf_status ls_prefetch_spf_results(ls_state* ls, const char* const* nodes, uint32_t n, int ulm) {
  if (!ls || (n && !nodes)) return SPF_E_INVALID;
  spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  if (!ls->eng) return lfail(ls, SPF_E_NO_DEVICE, "LinkState created host-only (device < 0)");
  if (needs_exact(ls, ulm != 0)) return SPF_OK;  // the exact kernel answers node by node
  std::vector<uint32_t> srcs, ids;
  std::unordered_set<uint32_t> seen;
  for (uint32_t i = 0; i < n; ++i) {
    if (!nodes[i]) return lfail(ls, SPF_E_INVALID, "ls_prefetch_spf_results: NULL node name");
    const uint32_t id = ls->intern(nodes[i]);
    const uint32_t s = id < ls->csr_of.size() ? ls->csr_of[id] : kNone;
    if (s == kNone || ls->spf_memo.count(std::make_pair(id, ulm != 0 ? 1 : 0)) || !seen.insert(s).second)
      continue;  // off-graph sources are trivial; memoised ones are done
    srcs.push_back(s);
    ids.push_back(id);
  }
  if (srcs.empty()) return SPF_OK;
  const uint32_t N = (uint32_t)ls->csr_name.size();
  const uint32_t flags = ulm ? 0u : SPF_FLAG_HOP_COUNT;
  uint64_t t0 = now_ns();
  spf_plan* raw = nullptr;
  st = spf_plan_create(ls->eng, srcs.data(), (uint32_t)srcs.size(), flags, &raw);
  if (st != SPF_OK) return eng_fail(ls, st);
  std::unique_ptr<spf_plan, void (*)(spf_plan*)> plan(raw, spf_plan_destroy);
  const uint32_t m = (uint32_t)srcs.size();
  std::vector<uint64_t> nh_off(m);
  std::vector<uint32_t> kk(m);
  spf_plan_nh_layout(plan.get(), nh_off.data(), kk.data());
  std::vector<uint32_t> dist((size_t)m * N);
  std::vector<uint32_t> nh(std::max<uint64_t>(spf_plan_nh_words(plan.get()), 1));
  uint64_t t1 = now_ns();
  ls->phase_ns[0] += t1 - t0;
  st = spf_plan_execute_host(plan.get(), dist.data(), nh.data());
  if (st != SPF_OK) return eng_fail(ls, st);
  t0 = now_ns();
  ls->phase_ns[1] += t0 - t1;
  std::vector<uint32_t> pred_ptr((size_t)m * (N + 1));
  uint64_t npred = 0;
  // every in-edge at most once per source; left uninitialised (8 MB of
  // zeroing for a fabric's me + 8 neighbours otherwise)
  const size_t pred_cap = (size_t)m * ls->col.size() + 1;
  std::unique_ptr<uint32_t[]> pred_edge(new uint32_t[pred_cap]);
  st = spf_plan_preds(plan.get(), pred_ptr.data(), pred_edge.get(), pred_cap, &npred);
  if (st != SPF_OK) return eng_fail(ls, st);
  t1 = now_ns();
  ls->phase_ns[2] += t1 - t0;
  const uint32_t wpm = spf_row_pitch(ls->eng) / 32;
  const std::vector<uint64_t> none;
  std::vector<SpfMemo> memos(m);
  std::vector<std::vector<uint32_t>> nbrs(m);
  for (uint32_t i = 0; i < m; ++i) nbrs[i] = src_neighbors(ls, srcs[i]);
  // the host assembly of each source's result is independent (read-only
  // LinkState tables): one thread per source, at most 16
  auto build = [&](uint32_t i) {
    SpfMemo& e = memos[i];
    e.dist.assign(dist.begin() + (size_t)i * N, dist.begin() + (size_t)(i + 1) * N);
    const uint32_t* pp = pred_ptr.data() + (size_t)i * (N + 1);
    // csr-indexed predecessor lists of this source, offsets rebased to 0
    e.pred_ptr.resize(N + 1);
    for (uint32_t v = 0; v <= N; ++v) e.pred_ptr[v] = pp[v] - pp[0];
    e.pred_edge.assign(pred_edge.get() + pp[0], pred_edge.get() + pp[N]);
    fill_memo(ls, e.dist.data(), none, nh.data() + nh_off[i], kk[i], wpm, nbrs[i],
              e.pred_ptr.data(), e.pred_edge.data(), e);
    e.pending = 1;
  };
  const uint32_t nt = std::min<uint32_t>(m, std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  if (nt <= 1) {
    for (uint32_t i = 0; i < m; ++i) build(i);
  } else {
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < nt; ++t)
      pool.emplace_back([&, t]() {
        for (uint32_t i = t; i < m; i += nt) build(i);
      });
    for (auto& th : pool) th.join();
  }
  for (uint32_t i = 0; i < m; ++i)
    ls->spf_memo.emplace(std::make_pair(ids[i], ulm != 0 ? 1 : 0), std::move(memos[i]));
  ls->phase_ns[3] += now_ns() - t1;
  return SPF_OK;
}

// Cumulative getSpfResult cost by phase in ns: [0] plan build, [1] GPU
// execute + copy back, [2] pathLinks, [3] host result assembly.
void ls_debug_phase_ns(const ls_state* ls, uint64_t* out) {
  for (int i = 0; i < 4; ++i) out[i] = ls ? ls->phase_ns[i] : 0;
}

// getMetricFromAToB (LinkState.cpp:740-751)
spf_status ls_get_metric_a_to_b(ls_state* ls, const char* a, const char* b, int ulm,
                                uint64_t* metric, int* has) {
  if (!ls || !a || !b || !metric || !has) return SPF_E_INVALID;
  *has = 0;
  if (std::strcmp(a, b) == 0) {
    *metric = 0;
    *has = 1;
    return SPF_OK;
  }
  const SpfMemo* m = nullptr;
  const spf_status st = spf_result(ls, ls->intern(a), ulm != 0, &m);
  if (st != SPF_OK) return st;
  const uint32_t bid = ls->intern(b);
  for (size_t i = 0; i < m->node.size(); ++i)
    if (m->node[i] == bid) {
      *metric = m->metric[i];
      *has = 1;
      break;
    }
  return SPF_OK;
}

// getMaxHopsToNode (LinkState.cpp:753-760)
spf_status ls_get_max_hops_to_node(ls_state* ls, const char* node, uint64_t* out) {
  if (!ls || !node || !out) return SPF_E_INVALID;
  const SpfMemo* m = nullptr;
  const spf_status st = spf_result(ls, ls->intern(node), false, &m);
  if (st != SPF_OK) return st;
  uint64_t mx = 0;
  for (uint64_t v : m->metric) mx = std::max(mx, v);
  *out = mx;
  return SPF_OK;
}

uint64_t ls_spf_runs(const ls_state* ls) { return ls ? ls->spf_runs : 0; }

spf_ctx* ls_engine(ls_state* ls) { return ls ? ls->eng : nullptr; }

uint64_t ls_graph_epoch(const ls_state* ls) { return ls ? ls->flat_epoch : 0; }
uint64_t ls_serial(const ls_state* ls) { return ls ? ls->serial : 0; }
uint64_t ls_debug_row_patches(const ls_state* ls) { return ls ? ls->row_patches : 0; }

spf_status ls_flatten(ls_state* ls, uint32_t* n_nodes, uint32_t* n_edges) {
  if (!ls) return SPF_E_INVALID;
  const spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  if (n_nodes) *n_nodes = (uint32_t)ls->csr_name.size();
  if (n_edges) *n_edges = (uint32_t)ls->col.size();
  return SPF_OK;
}

spf_status ls_graph_csr(ls_state* ls, uint32_t* row_ptr, uint32_t* col, int32_t* metric,
                        uint32_t* link_id, uint8_t* overloaded) {
  if (!ls) return SPF_E_INVALID;
  const spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  if (row_ptr) std::copy(ls->row_ptr.begin(), ls->row_ptr.end(), row_ptr);
  if (col) std::copy(ls->col.begin(), ls->col.end(), col);
  if (metric) std::copy(ls->metric.begin(), ls->metric.end(), metric);
  if (link_id) std::copy(ls->link_id.begin(), ls->link_id.end(), link_id);
  if (overloaded) std::copy(ls->ovl.begin(), ls->ovl.end(), overloaded);
  return SPF_OK;
}

spf_status ls_graph_node_names(ls_state* ls, uint32_t* name_ids) {
  if (!ls || !name_ids) return SPF_E_INVALID;
  const spf_status st = flatten(ls);
  if (st != SPF_OK) return st;
  std::copy(ls->csr_name.begin(), ls->csr_name.end(), name_ids);
  return SPF_OK;
}


// ---- standalone Link / HoldableValue / pathAInPathB (LinkState.h) ------------
struct ls_link {
  std::string area;
  std::string name[2];
  LinkObj obj;
  int side(const char* n) const {
    if (name[0] == n) return 0;
    if (name[1] == n) return 1;
    return -1;
  }
};

struct ls_holdable {
  bool is_bool;
  Holdable<bool> b{false};
  Holdable<Metric> m{0};
};

spf_status ls_link_create(const char* area, const char* node1, const char* if1, int32_t metric1,
                          int32_t adj_label1, int overload1, const char* node2, const char* if2,
                          int32_t metric2, int32_t adj_label2, int overload2, ls_link** out) {
  if (!area || !node1 || !if1 || !node2 || !if2 || !out) return SPF_E_INVALID;
  auto l = std::make_unique<ls_link>();
  l->area = area;
  l->name[0] = node1;
  l->name[1] = node2;
  const char* ifs[2] = {if1, if2};
  const int32_t met[2] = {metric1, metric2}, lab[2] = {adj_label1, adj_label2};
  const int ovl[2] = {overload1, overload2};
  for (int i = 0; i < 2; ++i) {
    Side& sd = l->obj.s[i];
    sd.node = (uint32_t)i;
    sd.ifname = ifs[i];
    sd.metric.set((Metric)(int64_t)met[i]);  // i32 -> u64 like the reference
    sd.overload.set(ovl[i] != 0);
    sd.label = lab[i];
  }
  l->obj.names = std::minmax(std::make_pair(l->name[0], std::string(if1)),
                             std::make_pair(l->name[1], std::string(if2)));
  const auto& nm = l->obj.names;
  l->obj.hash = folly_mix(folly_mix(std::hash<std::string>()(nm.first.first),
                                    std::hash<std::string>()(nm.first.second)),
                          folly_mix(std::hash<std::string>()(nm.second.first),
                                    std::hash<std::string>()(nm.second.second)));
  *out = l.release();
  return SPF_OK;
}
void ls_link_destroy(ls_link* l) { delete l; }
const char* ls_link_area(const ls_link* l) { return l ? l->area.c_str() : nullptr; }
uint64_t ls_link_hash(const ls_link* l) { return l ? l->obj.hash : 0; }
int ls_link_is_up(const ls_link* l) { return l && l->obj.up(); }
int ls_link_equal(const ls_link* a, const ls_link* b) { return a && b && a->obj.same(b->obj); }
int ls_link_less(const ls_link* a, const ls_link* b) { return a && b && a->obj.before(b->obj); }

#define LS_SIDE(l, node)                                   \
  const int sd_ = (l && node) ? (l)->side(node) : -1;       \
  if (sd_ < 0) return SPF_E_INVALID; /* std::invalid_argument */

spf_status ls_link_other_node(const ls_link* l, const char* node, const char** out) {
  LS_SIDE(l, node);
  *out = l->name[1 - sd_].c_str();
  return SPF_OK;
}
spf_status ls_link_iface(const ls_link* l, const char* node, const char** out) {
  LS_SIDE(l, node);
  *out = l->obj.s[sd_].ifname.c_str();
  return SPF_OK;
}
spf_status ls_link_metric(const ls_link* l, const char* node, uint64_t* out) {
  LS_SIDE(l, node);
  *out = l->obj.s[sd_].metric.get();
  return SPF_OK;
}
spf_status ls_link_adj_label(const ls_link* l, const char* node, int32_t* out) {
  LS_SIDE(l, node);
  *out = l->obj.s[sd_].label;
  return SPF_OK;
}
spf_status ls_link_overload(const ls_link* l, const char* node, int* out) {
  LS_SIDE(l, node);
  *out = l->obj.s[sd_].overload.get() ? 1 : 0;
  return SPF_OK;
}
// Link::setMetricFromNode / setOverloadFromNode (LinkState.cpp:253-286):
// *changed = the metric changed now / the link's up-state changed
spf_status ls_link_set_metric(ls_link* l, const char* node, uint64_t metric, uint64_t hold_up,
                              uint64_t hold_down, int* changed) {
  LS_SIDE(l, node);
  const bool c = l->obj.s[sd_].metric.update(metric, hold_up, hold_down);
  if (changed) *changed = c;
  return SPF_OK;
}
spf_status ls_link_set_overload(ls_link* l, const char* node, int overload, uint64_t hold_up,
                                uint64_t hold_down, int* changed) {
  LS_SIDE(l, node);
  const bool was_up = l->obj.up();
  l->obj.s[sd_].overload.update(overload != 0, hold_up, hold_down);
  if (changed) *changed = was_up != l->obj.up();
  return SPF_OK;
}
#undef LS_SIDE

// LinkState::pathAInPathB (LinkState.h:395-410): a occurs in b as a contiguous
// run of equal links (Link::operator==; link ids of one LinkState identify
// links).
spf_status ls_string_map_order(const char* const* keys, uint32_t n, uint32_t* order,
                               uint32_t* n_out) {
  if ((n && (!keys || !order)) || !n_out) return SPF_E_INVALID;
  std::unordered_map<std::string, uint32_t> m;  // the same container as the reference's
  for (uint32_t i = 0; i < n; ++i) {
    if (!keys[i]) return SPF_E_INVALID;
    m.emplace(keys[i], i);
  }
  uint32_t k = 0;
  for (const auto& kv : m) order[k++] = kv.second;
  *n_out = k;
  return SPF_OK;
}

// PrefixEntries = std::unordered_map<NodeAndArea, PrefixEntry> (Types.h:24):
// the same container, hashed by folly's std::hash<std::pair> (hash_128_to_64
// of the two std::hash<std::string>), replayed through the emplace / erase
// history PrefixState::updatePrefixDatabase applied (PrefixState.cpp:47-60).
namespace {
struct NodeAreaHash {
  size_t operator()(const std::pair<std::string, std::string>& k) const {
    return folly_mix(std::hash<std::string>()(k.first), std::hash<std::string>()(k.second));
  }
};
}  // namespace

spf_status ls_node_area_map_order(const char* const* nodes, const char* const* areas,
                                  const uint8_t* ops, uint32_t n_ops, uint32_t* order,
                                  uint32_t* n_out) {
  if ((n_ops && (!nodes || !areas || !ops || !order)) || !n_out) return SPF_E_INVALID;
  std::unordered_map<std::pair<std::string, std::string>, uint32_t, NodeAreaHash> m;
  for (uint32_t i = 0; i < n_ops; ++i) {
    if (!nodes[i] || !areas[i] || ops[i] > 1) return SPF_E_INVALID;
    std::pair<std::string, std::string> key(nodes[i], areas[i]);
    if (ops[i]) m.emplace(std::move(key), i);
    else m.erase(key);
  }
  uint32_t k = 0;
  for (const auto& kv : m) order[k++] = kv.second;
  *n_out = k;
  return SPF_OK;
}

int ls_path_a_in_path_b(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb) {
  if (na > nb) return 0;
  for (uint32_t i = 0; i < nb - na + 1; ++i) {
    uint32_t ai = 0, bi = i;
    while (ai < na && a[ai] == b[bi]) {
      ++ai;
      ++bi;
    }
    if (ai == na) return 1;
  }
  return 0;
}

ls_holdable* ls_holdable_create(int is_bool, uint64_t value) {
  auto* h = new ls_holdable{is_bool != 0};
  if (h->is_bool) h->b.set(value != 0);
  else h->m.set(value);
  return h;
}
void ls_holdable_destroy(ls_holdable* h) { delete h; }
uint64_t ls_holdable_value(const ls_holdable* h) {
  return h->is_bool ? (uint64_t)h->b.get() : h->m.get();
}
int ls_holdable_has_hold(const ls_holdable* h) { return h->is_bool ? h->b.has_hold() : h->m.has_hold(); }
int ls_holdable_decrement_ttl(ls_holdable* h) { return h->is_bool ? h->b.tick() : h->m.tick(); }
int ls_holdable_update_value(ls_holdable* h, uint64_t v, uint64_t hold_up, uint64_t hold_down) {
  return h->is_bool ? h->b.update(v != 0, hold_up, hold_down) : h->m.update(v, hold_up, hold_down);
}

}  // extern "C"
