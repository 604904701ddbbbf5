/*
 * openr_linkstate.h -- C-ABI of the LinkState drop-in facade (libopenr_spf.so).
 *
 * Replaces the reference's C++ class openr::LinkState
 * (openr/decision/LinkState.h:177-469) for its consumer SpfSolver
 * (openr/decision/Decision.cpp:413, 926, 939, 1126, 1153, 1165).  Method for
 * method:
 *
 *   LinkState::updateAdjacencyDatabase  (LinkState.h:330-333) -> ls_update_adjacency_databases
 *   LinkState::deleteAdjacencyDatabase  (LinkState.h:337)     -> ls_delete_adjacency_database
 *   LinkState::decrementHolds           (LinkState.h:327)     -> ls_decrement_holds
 *   LinkState::hasHolds / numLinks / numNodes / hasNode / isNodeOverloaded
 *                                        (LinkState.h:361-380) -> ls_has_holds, ls_num_links, ...
 *   LinkState::linksFromNode            (LinkState.h:366)     -> ls_links_from_node
 *   LinkState::getSpfResult             (LinkState.h:271-272) -> ls_get_spf_result
 *   LinkState::getKthPaths              (LinkState.h:293-294) -> ls_get_kth_paths
 *   LinkState::getMetricFromAToB / getHopsFromAToB / getMaxHopsToNode
 *                                        (LinkState.h:343-354) -> ls_get_metric_a_to_b, ls_get_max_hops_to_node
 *   fb303 counter decision.spf_runs     (LinkState.cpp:815)   -> ls_spf_runs
 *
 * The LSDB bookkeeping (bidirectional-link check, ordered-FIB holds, link and
 * node overload) runs on the host exactly as the reference's; every shortest
 * path computation is a batch on the MI355X engine (openr_spf.h).
 *
 * Ownership: views returned by ls_get_spf_result / ls_get_kth_paths point into
 * memo storage owned by the ls_state and stay valid until the next call that
 * reports topology_changed (the reference's memo invalidation,
 * LinkState.cpp:509-512, 714-717, 730-731) or ls_destroy.
 * Names are interned: ls_name_id()/ls_name() map between names and stable ids.
 * Errors: spf_status codes + ls_last_error(); no exceptions cross the ABI.
 */
#ifndef OPENR_LINKSTATE_H_
#define OPENR_LINKSTATE_H_

#include <stdint.h>

#include "openr_lsdb.h"
#include "openr_spf.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ls_state ls_state;

/* LinkState::LinkStateChange (LinkState.h:306-325) */
typedef struct ls_change {
  uint8_t topology_changed;
  uint8_t link_attributes_changed;
  uint8_t node_label_changed;
  uint8_t pad;
} ls_change;

/* Snapshot of one Link (LinkState.h:82-175). */
typedef struct ls_link_desc {
  uint32_t node1, node2;      /* name ids, in construction order (n1_, n2_) */
  const char* if1;            /* interface on node1 */
  const char* if2;            /* interface on node2 */
  uint32_t first_node;        /* orderedNames_.first.first  (name id) */
  uint32_t second_node;       /* orderedNames_.second.first (name id) */
  uint64_t metric1, metric2;  /* getMetricFromNode(node1/node2) (held value) */
  int32_t adj_label1, adj_label2;
  uint8_t overload1, overload2, is_up, pad;
  uint64_t hash;              /* Link::hash */
  const uint8_t* nh_v4_1;     /* 4 bytes each */
  const uint8_t* nh_v4_2;
  const uint8_t* nh_v6_1;     /* 16 bytes each */
  const uint8_t* nh_v6_2;
} ls_link_desc;

/* LinkState::SpfResult: one entry per reached node (source included). */
typedef struct ls_spf_view {
  uint32_t n;
  const uint32_t* node;      /* [n] name ids                              */
  const uint64_t* metric;    /* [n] NodeSpfResult::metric()               */
  const uint32_t* nh_ptr;    /* [n+1] into nh_node                        */
  const uint32_t* nh_node;   /* next-hop name ids (ascending name)        */
  const uint32_t* pl_ptr;    /* [n+1] into pl_link / pl_prev              */
  const uint32_t* pl_link;   /* pathLinks().link  (link ids)              */
  const uint32_t* pl_prev;   /* pathLinks().prevNode (name ids)           */
} ls_spf_view;

/* std::vector<LinkState::Path>: path p = link[path_ptr[p] .. path_ptr[p+1]) */
typedef struct ls_paths_view {
  uint32_t n_paths;
  const uint32_t* path_ptr;
  const uint32_t* link;
} ls_paths_view;

/* device < 0 creates a host-only state: LSDB bookkeeping and CSR flatten work,
 * shortest-path queries fail with SPF_E_NO_DEVICE (used by CPU-only tests). */
spf_status ls_create(const char* area, int device, ls_state** out);
/* A LinkState served by several GPUs of the node (spf_mctx over gpu_ids; ids
 * may repeat): the graph is replicated to every one; single-source queries
 * run on the first; ls_prefetch_all_sources splits an all-sources pass over
 * all of them.  Open/R's Decision reaches every GPU from its one thread
 * (Decision.cpp:1484). */
spf_status ls_create_multi(const char* area, const int* gpu_ids, uint32_t n, ls_state** out);
void ls_destroy(ls_state* ls);
const char* ls_last_error(const ls_state* ls);
/* LinkState::getArea (LinkState.h:356-359) */
const char* ls_get_area(const ls_state* ls);

spf_status ls_update_adjacency_databases(ls_state* ls, const openr_lsdb* lsdb,
                                         uint64_t hold_up_ttl,
                                         uint64_t hold_down_ttl,
                                         ls_change* changes /* [n_dbs] */);
spf_status ls_delete_adjacency_database(ls_state* ls, const char* node,
                                        ls_change* change);
spf_status ls_decrement_holds(ls_state* ls, ls_change* change);

int ls_has_holds(const ls_state* ls);
uint64_t ls_num_links(const ls_state* ls);
uint64_t ls_num_nodes(const ls_state* ls);
int ls_has_node(const ls_state* ls, const char* node);
int ls_is_node_overloaded(const ls_state* ls, const char* node);
/* the same by interned name id (ls_name_id) */
int ls_is_node_overloaded_id(const ls_state* ls, uint32_t node_id);

uint32_t ls_name_id(ls_state* ls, const char* name);
const char* ls_name(const ls_state* ls, uint32_t id);

/* getAdjacencyDatabases() (LinkState.h:357-359) reduced to what SpfSolver
 * reads from it: the nodes that advertised a database (name ids, ascending
 * name) and their node labels.  Call with cap 0 to size (*count). */
spf_status ls_adjacency_databases(const ls_state* ls, uint32_t* name_ids, int32_t* node_labels,
                                  uint32_t cap, uint32_t* count);
spf_status ls_links_from_node(const ls_state* ls, const char* node,
                              uint32_t* link_ids, uint32_t cap, uint32_t* count);
spf_status ls_link_info(const ls_state* ls, uint32_t link_id, ls_link_desc* out);

spf_status ls_get_spf_result(ls_state* ls, const char* node, int use_link_metric,
                             ls_spf_view* out);
/* getSpfResult for callers that read metrics and next hops only (SpfSolver's
 * route selection): the same memo entry and the same decision.spf_runs count,
 * its pathLinks derived on the first later call that needs them (the view's
 * pl_* are NULL until then). */
spf_status ls_get_spf_metrics(ls_state* ls, const char* node, int use_link_metric,
                              ls_spf_view* out);
spf_status ls_get_kth_paths(ls_state* ls, const char* src, const char* dst,
                            uint64_t k, ls_paths_view* out);
/* Batch fill of the getKthPaths memo: (src, d, 1) and (src, d, 2) for every
 * node d in one KSP2 launch.  Later ls_get_kth_paths calls for src return the
 * prefetched paths; spf_runs still counts as if each pair were queried on its
 * own (LinkState.cpp:778-779, 815).  Used by SpfSolver's KSP2_ED_ECMP route
 * build (Decision.cpp:895-1018). */
spf_status ls_prefetch_kth_paths(ls_state* ls, const char* src);
/* Batch fill of the getSpfResult memo for `n` nodes (use_link_metric as in
 * ls_get_spf_result) with one plan: one GPU execute, one copy back, one
 * batched pathLinks launch -- what SpfSolver's LFA needs before it asks for
 * getSpfResult(me) and getSpfResult(n) of every neighbour n
 * (Decision.cpp:1158-1165).  Results equal the one-by-one queries; spf_runs
 * counts each entry when it is first read (LinkState.cpp:815), so counts match
 * the reference whether or not a caller prefetches.  Nodes already memoised,
 * duplicates and off-graph nodes are skipped; graphs needing the exact kernel
 * (zero / negative metrics, u64) are left to the per-node path. */
spf_status ls_prefetch_spf_results(ls_state* ls, const char* const* nodes, uint32_t n,
                                   int use_link_metric);
/* getSpfResult for EVERY node of the graph -- what
 * Decision::getDecisionRouteDb does node by node (Decision.cpp:1480-1500) --
 * as one all-sources pass split over the GPUs of an ls_create_multi state
 * (SPF_E_STATE for a single-device state).  Results stay resident on the GPU
 * that computed them; a later ls_get_spf_result(node) (same use_link_metric)
 * reads node's row and next-hop bitmaps from its owner and computes its
 * pathLinks there, and counts decision.spf_runs then (LinkState.cpp:815), as
 * the reference's lazy getSpfResult would.  Any topology change drops the
 * pass (the memo invalidation, LinkState.cpp:509-512, 714-717, 730-731).
 * Graphs needing the exact kernel (zero / negative metrics, u64) are left to
 * the per-node path. */
spf_status ls_prefetch_all_sources(ls_state* ls, int use_link_metric);
/* The resident pass (NULL when none is valid): per-source digests
 * (spf_mplan_digest), owners, device buffers. */
spf_mplan* ls_all_sources_plan(ls_state* ls);
/* Cumulative getSpfResult cost by phase in ns since creation: out[0] plan
 * build, [1] GPU execute + copy back, [2] pathLinks, [3] host result
 * assembly (diagnostics; no reference counterpart). */
void ls_debug_phase_ns(const ls_state* ls, uint64_t* out);
spf_status ls_get_metric_a_to_b(ls_state* ls, const char* a, const char* b,
                                int use_link_metric, uint64_t* metric,
                                int* has_value);
spf_status ls_get_max_hops_to_node(ls_state* ls, const char* node, uint64_t* out);

uint64_t ls_spf_runs(const ls_state* ls);

/* The flattened CSR handed to the engine (for inspection / batch callers):
 * node ids are ascending-name ranks; returns the engine context. */
spf_ctx* ls_engine(ls_state* ls);
spf_status ls_flatten(ls_state* ls, uint32_t* n_nodes, uint32_t* n_edges);
/* Version of the flattened CSR structure (node ids, row_ptr, col, link ids):
 * changes whenever ls_flatten rebuilds it or rewrites rows in place (a link
 * down or up), not when it patches metrics or overload bits.  Callers caching per-graph tables key them on it. */
uint64_t ls_graph_epoch(const ls_state* ls);
/* A process-unique id of the state (never reused, unlike its address): name
 * ids (ls_name_id) are stable per state, so callers may cache them by it. */
uint64_t ls_serial(const ls_state* ls);
/* Flattens since creation that patched rows in place (a link down / up, an
 * adjacency withdrawn / advertised again) instead of reloading the graph
 * (diagnostics; spf_graph_loads counts the reloads). */
uint64_t ls_debug_row_patches(const ls_state* ls);
/* Flattens since creation that patched rows in place (a link down / up, an
 * adjacency withdrawn / advertised again) instead of reloading the graph
 * (diagnostics; spf_graph_loads counts the reloads). */
uint64_t ls_debug_row_patches(const ls_state* ls);
spf_status ls_graph_node_names(ls_state* ls, uint32_t* name_ids /* [n_nodes] */);
/* Copy of the flattened CSR (sizes from ls_flatten); any pointer may be NULL. */
spf_status ls_graph_csr(ls_state* ls, uint32_t* row_ptr, uint32_t* col, int32_t* metric,
                        uint32_t* link_id, uint8_t* overloaded);

/* ---- standalone value types of LinkState.h ------------------------------ */
/* openr::Link (LinkState.h:82-175): a link built outside a LinkState, as
 * LinkTest constructs one -- Link(area, node1, adj1, node2, adj2),
 * LinkState.cpp:127-186.  Side accessors take a node name and fail with
 * SPF_E_INVALID for a node not on the link (the reference throws
 * std::invalid_argument, LinkState.cpp:163-172). */
typedef struct ls_link ls_link;
spf_status ls_link_create(const char* area, const char* node1, const char* if1, int32_t metric1,
                          int32_t adj_label1, int overload1, const char* node2, const char* if2,
                          int32_t metric2, int32_t adj_label2, int overload2, ls_link** out);
void ls_link_destroy(ls_link* link);
const char* ls_link_area(const ls_link* link);                 /* getArea           */
uint64_t ls_link_hash(const ls_link* link);                    /* Link::hash        */
int ls_link_is_up(const ls_link* link);                        /* isUp              */
int ls_link_equal(const ls_link* a, const ls_link* b);         /* operator==        */
int ls_link_less(const ls_link* a, const ls_link* b);          /* operator<         */
spf_status ls_link_other_node(const ls_link* link, const char* node, const char** out);
spf_status ls_link_iface(const ls_link* link, const char* node, const char** out);
spf_status ls_link_metric(const ls_link* link, const char* node, uint64_t* out);
spf_status ls_link_adj_label(const ls_link* link, const char* node, int32_t* out);
spf_status ls_link_overload(const ls_link* link, const char* node, int* out);
/* setMetricFromNode / setOverloadFromNode (LinkState.cpp:253-286): *changed =
 * the effective metric changed now / the link's up state changed. */
spf_status ls_link_set_metric(ls_link* link, const char* node, uint64_t metric,
                              uint64_t hold_up, uint64_t hold_down, int* changed);
spf_status ls_link_set_overload(ls_link* link, const char* node, int overload,
                                uint64_t hold_up, uint64_t hold_down, int* changed);

/* LinkState::pathAInPathB (static, LinkState.h:395-410) over paths given as
 * link ids of one LinkState (ls_get_kth_paths): 1 when a is a contiguous
 * run of b. */
int ls_path_a_in_path_b(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb);

/* Iteration order of a std::unordered_map<std::string, V> after emplacing
 * keys[0..n) in that order (duplicates ignored, as emplace does):
 * order[i] = the index in keys of the i-th key visited; *n_out = distinct
 * keys.  SpfSolver walks its areaLinkStates map this way
 * (Decision.cpp:411-412, 574-576, 1124, 1212), and with several areas that
 * order decides ties (getNextHopsWithMetric's running shortest metric, the
 * node-label entry of a node present in two areas). */
spf_status ls_string_map_order(const char* const* keys, uint32_t n, uint32_t* order,
                               uint32_t* n_out);

/* Iteration order of a PrefixEntries map, std::unordered_map<NodeAndArea,
 * PrefixEntry> (openr/common/Types.h:24, folly's std::hash<std::pair>), after
 * the history PrefixState applied to it (PrefixState.cpp:47-60): op i emplaces
 * (ops[i] = 1; an existing key is left where it is) or erases (ops[i] = 0)
 * the key (nodes[i], areas[i]).  order[j] = the op index that inserted the
 * j-th surviving key; *n_out = surviving keys.  runBestPathSelectionBgp
 * (Decision.cpp:795-832) and addBestPaths' prepend-label walk (:1047-1053)
 * visit the entries in this order. */
spf_status ls_node_area_map_order(const char* const* nodes, const char* const* areas,
                                  const uint8_t* ops, uint32_t n_ops, uint32_t* order,
                                  uint32_t* n_out);

/* HoldableValue<bool> / HoldableValue<LinkStateMetric> (LinkState.h:36-58,
 * LinkState.cpp:54-125). */
typedef struct ls_holdable ls_holdable;
ls_holdable* ls_holdable_create(int is_bool, uint64_t value);
void ls_holdable_destroy(ls_holdable* h);
uint64_t ls_holdable_value(const ls_holdable* h);
int ls_holdable_has_hold(const ls_holdable* h);
int ls_holdable_decrement_ttl(ls_holdable* h);
int ls_holdable_update_value(ls_holdable* h, uint64_t value, uint64_t hold_up_ttl,
                             uint64_t hold_down_ttl);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_LINKSTATE_H_ */
