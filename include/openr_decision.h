/*
 * openr_decision.h -- C-ABI of the SpfSolver drop-in (libopenr_spf.so).
 *
 * Replaces the reference's route computation, openr::SpfSolver
 * (openr/decision/Decision.h, SpfSolver::SpfSolverImpl in
 * openr/decision/Decision.cpp:389-1305) and the PrefixState it reads
 * (openr/decision/PrefixState.{h,cpp}), for a C++ Decision that owns one
 * LinkState per area (openr_linkstate.h):
 *
 *   PrefixState::updatePrefixDatabase  (PrefixState.cpp:17-84) -> dc_prefix_update / dc_prefix_delete
 *   SpfSolver::buildRouteDb            (Decision.cpp:556-722)   -> dc_build_route_db
 *   SpfSolver::createRouteForPrefix    (Decision.cpp:389-555)     (inside)
 *   SpfSolver::selectBestRoutes / runBestPathSelectionBgp / maybeFilterDrainedNodes
 *                                      (Decision.cpp:724-832)     (inside)
 *   SpfSolver::selectBestPathsSpf / selectBestPathsKsp2 / addBestPaths
 *                                      (Decision.cpp:834-1080)    (inside)
 *   SpfSolver::getNextHopsWithMetric / getNextHopsThrift
 *                                      (Decision.cpp:1082-1305)   (inside)
 *   SpfSolver::updateStaticMplsRoutes  (Decision.cpp:354-387)   -> dc_static_mpls_route_set / _delete
 *   SpfSolver::getBestRoutesCache      (Decision.h)             -> dc_best_route
 *   fb303 counters decision.*          (Decision.cpp)           -> dc_counter
 *
 * One area: the SP_ECMP / IP prefixes and node labels of a build are one
 * batched next-hop selection on the GPU (spf_routes, or spf_mplan_routes
 * from a resident all-sources pass), the records assembled here.  Several
 * areas, SR_MPLS and KSP2_ED_ECMP prefixes: the reference's per-prefix walk
 * over the LinkStates' memoised (GPU) SPF results and batched KSP2 paths.
 * PrefixEntries maps are the reference's container (std::unordered_map over
 * NodeAndArea with folly's pair hash), so every walk that depends on their
 * order (runBestPathSelectionBgp, the prepend-label searches) visits the
 * entries as the reference does.
 *
 * Ownership: a dc_route_db is owned by the caller (dc_route_db_destroy);
 * its views stay valid until then.  Errors: spf_status + dc_last_error();
 * no exceptions cross the ABI.  Single-threaded, like the reference
 * (Decision.cpp:1484).
 */
#ifndef OPENR_DECISION_H_
#define OPENR_DECISION_H_

#include <stdint.h>

#include "openr_linkstate.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dc_prefix_state dc_prefix_state;
typedef struct dc_solver dc_solver;
typedef struct dc_route_db dc_route_db;

/* thrift::PrefixForwardingType / PrefixForwardingAlgorithm (OpenrConfig.thrift) */
#define DC_FWD_IP 0u
#define DC_FWD_SR_MPLS 1u
#define DC_ALGO_SP_ECMP 0u
#define DC_ALGO_KSP2_ED_ECMP 1u
/* thrift::CompareType (Lsdb.thrift:171-180) */
#define DC_WIN_IF_PRESENT 0u
#define DC_WIN_IF_NOT_PRESENT 1u
#define DC_IGNORE_IF_NOT_PRESENT 2u
/* thrift::MplsActionCode (Network.thrift) */
#define DC_MPLS_NONE 0u
#define DC_MPLS_PUSH 1u
#define DC_MPLS_SWAP 2u
#define DC_MPLS_PHP 3u
#define DC_MPLS_POP_AND_LOOKUP 4u

/* thrift::MetricEntity (Lsdb.thrift:182-204) */
typedef struct dc_metric_entity {
  int64_t type;
  int64_t priority;
  uint32_t op;                 /* DC_WIN_IF_PRESENT ... */
  uint32_t is_tie_breaker;
  uint32_t n_metric;
  const int64_t* metric;       /* [n_metric] */
} dc_metric_entity;

/* The fields of thrift::PrefixEntry (Lsdb.thrift:214-268) route building reads. */
typedef struct dc_prefix_entry {
  const char* prefix;          /* textual prefix: the route key */
  uint8_t is_v4;               /* IPv4 prefix (createRouteForPrefix's v4 checks) */
  uint8_t is_bgp;              /* type == BGP */
  uint8_t forwarding_type;     /* DC_FWD_* */
  uint8_t forwarding_algorithm;/* DC_ALGO_* */
  uint8_t has_prepend_label, has_min_nexthop, has_mv, pad;
  int32_t prepend_label;
  int64_t min_nexthop;
  int32_t path_preference, source_preference, distance; /* thrift::PrefixMetrics */
  int32_t mv_version;          /* thrift::MetricVector */
  uint32_t n_mv;
  const dc_metric_entity* mv;  /* [n_mv] */
} dc_prefix_entry;

/* thrift::NextHopThrift (Network.thrift:65-86) as createNextHop builds it
 * (openr/common/Util.cpp:907-922).  Strings are ids into the route db's
 * string table (dc_route_db_string); DC_NONE = unset optional field. */
#define DC_NONE 0xFFFFFFFFu
typedef struct dc_nexthop {
  uint8_t address[16];
  uint8_t address_len;         /* 4 or 16 */
  uint8_t mpls_action;         /* DC_MPLS_* */
  uint8_t n_push;              /* PUSH: labels at push_off in the label pool */
  uint8_t pad;
  int32_t metric;              /* i32, as the thrift field */
  int32_t swap_label;          /* SWAP */
  uint32_t push_off;
  uint32_t ifname, area, neighbor;
} dc_nexthop;

/* ---- PrefixState -------------------------------------------------------- */
dc_prefix_state* dc_prefix_state_create(void);
void dc_prefix_state_destroy(dc_prefix_state* ps);
/* entriesByOriginator.emplace / assignment (PrefixState.cpp:55-68) and
 * erase (:41-52): the prefix's map is dropped with its last advertiser. */
spf_status dc_prefix_update(dc_prefix_state* ps, const char* node, const char* area,
                            const dc_prefix_entry* entry);
spf_status dc_prefix_delete(dc_prefix_state* ps, const char* node, const char* area,
                            const char* prefix);
/* The advertisers of `prefix` in the map's iteration order: node / area
 * pointers valid until the prefix's map changes.  cap 0 sizes (*count). */
spf_status dc_prefix_entries(const dc_prefix_state* ps, const char* prefix, const char** nodes,
                             const char** areas, uint32_t cap, uint32_t* count);

/* ---- SpfSolver ---------------------------------------------------------- */
/* SpfSolver(myNodeName, enableV4, computeLfaPaths, enableOrderedFib,
 * bgpDryRun, enableBestRouteSelection) (Decision.h) */
spf_status dc_solver_create(const char* my_node, int enable_v4, int compute_lfa_paths,
                            int bgp_dry_run, int enable_best_route_selection, dc_solver** out);
void dc_solver_destroy(dc_solver* s);
const char* dc_last_error(const dc_solver* s);
/* updateStaticMplsRoutes: label -> next hops; the records' string ids index
 * `strings`, their PUSH labels `labels` (either may be NULL when unused) */
spf_status dc_static_mpls_route_set(dc_solver* s, int32_t label, const dc_nexthop* nhs, uint32_t n,
                                    const char* const* strings, const int32_t* labels);
spf_status dc_static_mpls_route_delete(dc_solver* s, int32_t label);

/* buildRouteDb(myNodeName, areaLinkStates, prefixState): areas[i] is the
 * LinkState of area_names[i]; the areas are walked in the order of the
 * reference's std::unordered_map<std::string, LinkState> emplaced in this
 * order.  *out = NULL (and SPF_OK) when no area has my node (the reference's
 * std::nullopt). */
spf_status dc_build_route_db(dc_solver* s, const char* const* area_names, ls_state* const* areas,
                             uint32_t n_areas, const dc_prefix_state* ps, dc_route_db** out);

/* fb303 counter `name` (decision.no_route_to_prefix, ...) since creation */
uint64_t dc_counter(const dc_solver* s, const char* name);
/* getBestRoutesCache()[prefix]: *found = 0 when the last build cached none;
 * success, bestNodeArea and the allNodeAreas set (ascending) */
spf_status dc_best_route(const dc_solver* s, const char* prefix, int* found, int* success,
                         const char** best_node, const char** best_area, const char** nodes,
                         const char** areas, uint32_t cap, uint32_t* count);

/* Cumulative dc_build_route_db cost by phase in ns since creation (diagnostics;
 * no reference counterpart): [0] area setup + getSpfResult(me), [1] the
 * prefix walk (createRouteForPrefix; per-prefix SR / KSP2 / several-area
 * routes included), [2] node-label collection + set layout, [3] the batched
 * selection (spf_mplan_routes / spf_routes), [4] route assembly from it,
 * [5] adjacency-label and static routes. */
void dc_debug_phase_ns(const dc_solver* s, uint64_t* out);

/* ---- DecisionRouteDb ---------------------------------------------------- */
void dc_route_db_destroy(dc_route_db* db);
/* the string table (interface names, areas, neighbours, prefixes) */
uint32_t dc_route_db_strings(const dc_route_db* db);
const char* dc_route_db_string(const dc_route_db* db, uint32_t id);
/* every next-hop record and the label pool of PUSH actions */
const dc_nexthop* dc_route_db_nexthops(const dc_route_db* db, uint32_t* n);
const int32_t* dc_route_db_labels(const dc_route_db* db, uint32_t* n);
/* RibUnicastEntry i: prefix, bestPrefixEntry's (node, area), doNotInstall,
 * next hops [nh_begin, nh_end) of dc_route_db_nexthops (a set: no two equal) */
uint32_t dc_route_db_unicast_count(const dc_route_db* db);
spf_status dc_route_db_unicast(const dc_route_db* db, uint32_t i, uint32_t* prefix,
                               uint32_t* best_node, uint32_t* best_area, int* do_not_install,
                               uint32_t* nh_begin, uint32_t* nh_end);
/* RibMplsEntry i: label, next hops [nh_begin, nh_end) */
uint32_t dc_route_db_mpls_count(const dc_route_db* db);
spf_status dc_route_db_mpls(const dc_route_db* db, uint32_t i, int32_t* label, uint32_t* nh_begin,
                            uint32_t* nh_end);
/* Whole-db tables in one call each (bindings that materialise every route):
 * unicast rows of 6 u32 (prefix, best node, best area, doNotInstall,
 * nh_begin, nh_end), mpls rows of 3 (label, nh_begin, nh_end). */
const uint32_t* dc_route_db_unicast_table(const dc_route_db* db, uint32_t* n);
const uint32_t* dc_route_db_mpls_table(const dc_route_db* db, uint32_t* n);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_DECISION_H_ */
