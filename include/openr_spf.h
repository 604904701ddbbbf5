/*
 * openr_spf.h -- C-ABI of the MI355X SPF engine (libopenr_spf.so).
 *
 * Graph-level interface: the caller (the LinkState facade of
 * openr_linkstate.h, or a host program that already has a CSR) hands over a
 * flattened link-state graph once, then asks for batches of single-source
 * shortest-path-first solves.  Each solve reproduces, bit for bit, what the
 * reference computes in LinkState::runSpf (openr/decision/LinkState.cpp:808-882):
 *   - dist[v]  = NodeSpfResult::metric() of v, or SPF_UNREACHABLE
 *   - nh bits  = NodeSpfResult::nextHops() of v as a bitset over the source's
 *                distinct up neighbours (ascending node id = ascending name)
 * The reference entry points this replaces are LinkState::getSpfResult
 * (LinkState.h:271-272, LinkState.cpp:793-803) for a batch of sources at once.
 *
 * Conventions
 *   - Node ids 0..n_nodes-1 MUST be assigned in ascending std::string order of
 *     the node names: the reference's Dijkstra queue breaks metric ties by
 *     node name (LinkState.h:488-498) and the engine breaks them by node id.
 *   - A directed edge u->v exists for every *up* link (Link::isUp,
 *     LinkState.cpp:233-236); its metric is the metric advertised by u
 *     (Link::getMetricFromNode(u), LinkState.cpp:195-204).  Edges of one node
 *     appear in linksFromNode(u) iteration order.
 *   - overloaded[u] != 0: u is recorded but never expanded unless it is the
 *     source (LinkState.cpp:831-838).
 *   - Distances are u32 unless the plan asks for SPF_FLAG_DIST64 (u64, the
 *     reference's LinkStateMetric).  Weighted solves of graphs whose longest
 *     possible path (max metric x (n_nodes-1)) does not fit 32 bits, or with
 *     a negative metric (the reference's i32 -> u64 conversion wraps), need
 *     SPF_FLAG_DIST64.
 *   - Zero or negative metrics, u64 distances and graphs too large for the
 *     LDS-resident kernels run the exact kernel (exact.hip): runSpf replayed
 *     step for step, one wavefront per source, heap pop order (metric, id)
 *     reproduced -- the next-hop sets under zero-cost plateaus depend on it.
 *   - Row pitch: dist and next-hop rows are stored with pitch
 *     spf_row_pitch() = n_nodes rounded up to a multiple of 1024 (every
 *     next-hop bitmap then starts on a 128-byte line).
 *
 * Errors: every call returns spf_status; spf_last_error() describes the last
 * failure.  No exceptions cross the ABI.  All calls on one context must come
 * from one host thread (the reference is single-threaded too,
 * openr/decision/Decision.cpp:1484).
 */
#ifndef OPENR_SPF_H_
#define OPENR_SPF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum spf_status {
  SPF_OK = 0,
  SPF_E_INVALID = 1,     /* bad argument / malformed graph            */
  SPF_E_UNSUPPORTED = 2, /* input outside the exact-parity envelope   */
  SPF_E_HIP = 3,         /* HIP runtime failure                       */
  SPF_E_NO_DEVICE = 4,   /* no usable gfx950 device                   */
  SPF_E_NOMEM = 5,
  SPF_E_STATE = 6        /* call out of order (e.g. no graph loaded)  */
} spf_status;

#define SPF_UNREACHABLE 0xFFFFFFFFu

/* solve flags */
#define SPF_FLAG_HOP_COUNT 0x1u /* useLinkMetric == false: every edge costs 1 */
/* Distance rows are u64 (LinkStateMetric, LinkState.h:22): pitch entries of
 * 8 bytes, UINT64_MAX = unreachable.  Required for weighted solves of graphs
 * with a negative metric or max metric x (n_nodes-1) >= 2^32 - 1. */
#define SPF_FLAG_DIST64 0x2u
#define SPF_UNREACHABLE64 0xFFFFFFFFFFFFFFFFull

typedef struct spf_ctx spf_ctx;
typedef struct spf_plan spf_plan;

/* Dead slots: an edge u -> u (a self-loop) with metric 1 stands for no edge
 * -- a link of u that is down, or withdrawn, kept in place so that a later
 * change of that link patches the row instead of reloading the graph
 * (spf_graph_patch_rows).  Both slots of such a link are self-loops sharing
 * its link id.  No kernel relaxes, pushes or pulls over one; they are not
 * distinct neighbours and never next hops or pathLinks. */
typedef struct spf_graph {
  uint32_t n_nodes;
  uint32_t n_edges;             /* directed up edges (and dead slots)           */
  const uint32_t* row_ptr;      /* [n_nodes+1]                                  */
  const uint32_t* col;          /* [n_edges] head node of edge                  */
  const int32_t* metric;        /* [n_edges] metric advertised by the tail      */
  const uint32_t* link_id;      /* [n_edges] undirected link id (shared by both directions) */
  const uint8_t* overloaded;    /* [n_nodes]                                    */
} spf_graph;

/* ---- context ------------------------------------------------------------ */
spf_status spf_ctx_create(int device, spf_ctx** out);
void spf_ctx_destroy(spf_ctx* ctx);
const char* spf_last_error(const spf_ctx* ctx);
/* Thread-local message for failures before a context exists. */
const char* spf_global_error(void);

/* Copies the graph to the device (replaces any previous graph). */
spf_status spf_graph_load(spf_ctx* ctx, const spf_graph* g);

/* In-place patches of the loaded graph: the CSR
 * structure (nodes, up edges, their order) stays, so no spf_graph_load is
 * needed when an adjacency-database update only toggles node overload bits or
 * changes metrics of up links -- the reference re-runs updateAdjacencyDatabase
 * (openr/decision/LinkState.cpp:564-719) and clears its SPF memo
 * (:509-512, :714-717) on every such publication.
 *   spf_graph_set_overload: overloaded[i] != 0 drains node nodes[i]
 *     (LinkState::updateNodeOverloaded, LinkState.cpp:480-493).
 *   spf_graph_set_metric: new metric of directed edge edges[i] (CSR edge id),
 *     i.e. Link::getMetricFromNode of its tail (LinkState.cpp:195-204).
 * Every change bumps spf_graph_epoch(); SPF plans (spf_plan_*) re-derive
 * their internal state on their next execute (same output layout); KSP2 and
 * what-if plans return SPF_E_STATE and must be recreated; any plan returns
 * SPF_E_STATE after a spf_graph_load. */
spf_status spf_graph_set_overload(spf_ctx* ctx, const uint32_t* nodes, const uint8_t* overloaded,
                                  uint32_t n);
spf_status spf_graph_set_metric(spf_ctx* ctx, const uint32_t* edges, const int32_t* metric,
                                uint32_t n);
/* Rows of nodes[0..n) rewritten in place, each with its current length:
 * col / metric / link hold the new rows back to back (a dead slot: col = the
 * node, metric 1).  What a link going down or up, or an adjacency withdrawn
 * and advertised again, does to the CSR (LinkState::updateAdjacencyDatabase,
 * LinkState.cpp:564-719; Link::isUp, :233-236) when every link id keeps its
 * two slots.  Reverse edges, distinct-neighbour lists and the kernels' tables
 * are patched; plans re-derive on their next execute, except a plan one of
 * whose sources gained or lost a distinct neighbour (its next-hop layout):
 * that one returns SPF_E_STATE and must be recreated. */
spf_status spf_graph_patch_rows(spf_ctx* ctx, const uint32_t* nodes, uint32_t n, const uint32_t* col,
                                const int32_t* metric, const uint32_t* link);
uint64_t spf_graph_epoch(const spf_ctx* ctx);
/* Number of spf_graph_load calls so far (patches do not count). */
uint64_t spf_graph_loads(const spf_ctx* ctx);
uint32_t spf_row_pitch(const spf_ctx* ctx);
/* 1 when the loaded graph has an up edge with metric <= 0 (weighted solves
 * of such graphs run the exact kernel, which reproduces the heap pop order the
 * reference's next-hop sets depend on under zero-cost plateaus). */
int spf_graph_has_nonpositive_metric(const spf_ctx* ctx);
/* 1 when weighted solves need u64 distances (SPF_FLAG_DIST64). */
int spf_graph_needs_dist64(const spf_ctx* ctx);

/* Distinct up neighbours of `src` in ascending id: the bit order of its
 * next-hop sets.  Writes min(count, cap) ids; *count = total. */
spf_status spf_src_neighbors(const spf_ctx* ctx, uint32_t src, uint32_t* out,
                             uint32_t cap, uint32_t* count);

/* ---- plans: a fixed batch of sources, executable many times ------------- */
/* Next-hop layout of source i of the plan: one destination bitmap per
 * distinct up neighbour (k_i bitmaps, neighbours in ascending id), each of
 * pitch/32 32-bit words:
 *   neighbour j in nextHops(v)  <=>  nh[nh_off[i] + j*(pitch/32) + v/32] bit (v%32).
 * spf_plan_nh_layout reports nh_off[i] and k_i ("words" = bitmaps). */
spf_status spf_plan_create(spf_ctx* ctx, const uint32_t* srcs, uint32_t n_src,
                           uint32_t flags, spf_plan** out);
void spf_plan_destroy(spf_plan* plan);
uint64_t spf_plan_nh_words(const spf_plan* plan);     /* total u32 words   */
spf_status spf_plan_nh_layout(const spf_plan* plan, uint64_t* nh_off,
                              uint32_t* words);       /* n_src entries each */
uint32_t spf_plan_closure_rows(const spf_plan* plan); /* sources actually solved */
/* Which kernels the next execute runs (diagnostics, benchmarks):
 * *bfs = 0 sssp_kernel (weighted, per source), 1 msbfs_kernel (64 sources per
 * sweep, per-level stores), 2 msbfs_planes_kernel (32 sources, register bit
 * planes, rows written once), 3 exact_spf_kernel, 4 spf_big_kernel (graphs
 * beyond the LDS-resident kernels: one source at a time on the whole chip,
 * next hops inside), 5 mssp_kernel (weighted, positive metrics: 2-16 sources
 * per workgroup, u16 labels in LDS, min-plus sweeps), 6 msbfs_team_kernel (unit
 * metrics, plans with few sources: each batch's sweep split over a team of
 * workgroups on one XCD); *narrow = 0 when the
 * next-hop pass (ecmp_kernel) reads the u32 rows, 1 when it reads u8 rows,
 * 2 when slice_rows_kernel turns the u8 rows into bit planes and
 * ecmp_sliced_kernel matches those, 3 when msbfs_team_kernel writes the bit
 * planes itself (4 per word; no u8 rows, no slicing pass).
 * No reference counterpart (engine introspection). */
spf_status spf_plan_kernels(const spf_plan* plan, uint32_t* bfs, uint32_t* narrow);
/* Bytes the distance kernel and the next-hop kernel of one execute must move
 * to or from HBM (compulsory traffic given each kernel's structure: one
 * column sweep per BFS workgroup or per SSSP source, every output written
 * once, every compared distance row read once).  Denominator-free roofline
 * input for benchmarks; no reference counterpart. */
spf_status spf_plan_traffic(const spf_plan* plan, uint64_t* bfs_bytes, uint64_t* ecmp_bytes);
/* The same per phase: bytes[0] distance kernel, bytes[1] row slicing (0
 * unless *narrow == 2), bytes[2] next-hop kernel.  For sliced plans the
 * plane count comes from the last execute's deepest level (a 4-byte read). */
spf_status spf_plan_traffic_phases(const spf_plan* plan, uint64_t* bytes);

/* Execute on device buffers: d_dist = [n_src][pitch] u32, d_nh = nh words.
 * Enqueued on `stream` (a hipStream_t); NULL = the context's stream, a
 * BLOCKING stream, so work the caller put on the legacy null stream before
 * (a hipMemset / hipMemcpy of the outputs) is ordered before the execute.  A
 * caller's own non-blocking stream gets no such ordering: order it yourself.
 * Steady state (same graph epoch as the previous execute of the plan): no
 * host synchronisation, no allocation -- capturable into a hipGraph
 * (spf_mplan_set_graphs does).  The FIRST execute after an in-place patch
 * (spf_graph_set_overload / _metric) re-derives the plan on the host and
 * uploads its tables with a stream synchronisation, and a big plan's first
 * execute allocates its scratch: run one execute on a new epoch before
 * capturing.  Launches whose workgroups wait on each other (team BFS, grid
 * barriers) are ordered after any other such launch of the process on the
 * same device (see spf_device_check). */
spf_status spf_plan_execute(spf_plan* plan, uint32_t* d_dist, uint32_t* d_nh,
                            void* stream);
/* Per-source digests of an execute's output (d_dist / d_nh as passed to
 * spf_plan_execute), enqueued on `stream`: d_out[i] (u64) = sum mod 2^64 over
 * reachable v of mix(mix(v + 1) + dist(v)) ^ fnv1a64(nh(v) as u32 words),
 * mix = splitmix64's finaliser, nh(v) = v's next-hop set as a bitset over the
 * source's distinct up neighbours (the what-if digest's node term).  What a
 * rank ships when its rows stay resident on its GPU (multi-GPU all-sources),
 * and what the parity tests compare with the oracle's digests.  No
 * reference counterpart. */
spf_status spf_plan_digest(spf_plan* plan, const void* d_dist, const uint32_t* d_nh,
                           uint64_t* d_out, void* stream);
/* The narrow (u8) distance rows of the plan's last execute, for plans whose
 * distance kernel keeps them (spf_plan_kernels: *narrow != 0): row i (source
 * srcs[i]) byte v = d(srcs[i], v) when below 254, 254 when d >= 254, 255
 * when unreachable or v >= n_nodes -- lossless when every finite distance of
 * the execute is below 254 (unit-metric fabrics: 4 levels; grid 100x100:
 * 198).  n_src rows of spf_row_pitch bytes are copied to d_out on `stream`
 * (after the execute on that stream).  SPF_E_UNSUPPORTED for plans without
 * them.  Used to ship rows compactly (multi-GPU gather); no reference
 * counterpart (the reference's metric is u64, LinkState.h:22). */
spf_status spf_plan_copy_narrow_rows(spf_plan* plan, uint8_t* d_out, void* stream);
/* spf_plan_execute into host buffers: dist [n_src][n_nodes] (dense, no row
 * padding) and the next-hop words (spf_plan_nh_words of them); either may be
 * NULL.  Device staging is owned by the plan. */
spf_status spf_plan_execute_host(spf_plan* plan, uint32_t* dist, uint32_t* nh);
/* (with SPF_FLAG_DIST64, `dist` is read as uint64_t[n_src][n_nodes]) */
/* pathLinks of every source of the plan's last spf_plan_execute_host, one
 * batched launch (the batch form of spf_preds): pred_ptr = [n_src][n_nodes+1]
 * absolute offsets into pred_edge (source i's list for v is
 * pred_edge[pred_ptr[i*(n+1)+v] .. pred_ptr[i*(n+1)+v+1]), directed CSR edge
 * ids in the reference's order, LinkState.cpp:857-873); *n_preds = total.
 * With pred_edge == NULL only the offsets are written; SPF_E_NOMEM when cap <
 * *n_preds.  SPF_E_UNSUPPORTED for exact / big plans (spf_solve_exact's pop
 * ranks order those). */
spf_status spf_plan_preds(spf_plan* plan, uint32_t* pred_ptr, uint32_t* pred_edge, uint64_t cap,
                          uint64_t* n_preds);

/* Kernel timing with HIP events recorded on the execute stream: after
 * spf_plan_enable_timing(plan, K), each of the next K executes records events
 * around its SSSP and ECMP kernels; spf_plan_timing() waits for them and
 * returns the summed milliseconds of each kernel and the number of executes
 * (then resets the count). */
spf_status spf_plan_enable_timing(spf_plan* plan, uint32_t max_executes);
spf_status spf_plan_timing(spf_plan* plan, double* sssp_ms, double* ecmp_ms, uint32_t* n);
/* The same per phase: ms[0] distance kernel, ms[1] row slicing, ms[2]
 * next-hop kernel (spf_plan_timing's ecmp_ms = ms[1] + ms[2]). */
spf_status spf_plan_timing_phases(spf_plan* plan, double* ms, uint32_t* n);

/* Convenience: plan + execute + copy back to host buffers.
 * dist_out = [n_src][n_nodes] (dense, no pitch); nh_out sized by
 * spf_plan_nh_words with the planar layout above (pitch = spf_row_pitch). */
spf_status spf_solve(spf_ctx* ctx, const uint32_t* srcs, uint32_t n_src,
                     uint32_t flags, uint32_t* dist_out, uint32_t* nh_out);

/* ---- single-source primitives (LinkState facade, KSP) -------------------- */
/* Distances of one source with an optional set of undirected link ids to
 * ignore -- the reference's runSpf(src, true, linksToIgnore) used by
 * getKthPaths (LinkState.cpp:776-779).  dist_out = [n_nodes]. */
spf_status spf_sssp(spf_ctx* ctx, uint32_t src, uint32_t flags,
                    const uint32_t* ignore_links, uint32_t n_ignore,
                    uint32_t* dist_out);

/* runSpf(src, useLinkMetric, linksToIgnore) on the exact kernel, into host
 * buffers: distances as u64 (dist64_out, UINT64_MAX unreachable) when
 * dist32_out is NULL, else as u32; next-hop bitmaps in the plan layout
 * (spf_src_neighbors(src) bitmaps of pitch/32 words); pop_out[v] = the
 * position of v in the reference's Dijkstra pop order (UINT32_MAX
 * unreachable), from which pathLinks follow: the tight up in-edges (u -> v)
 * of expanded u with pop(u) < pop(v), ordered by (pop(u), linksFromNode
 * order).  Any pointer but one distance buffer may be NULL. */
spf_status spf_solve_exact(spf_ctx* ctx, uint32_t src, uint32_t flags,
                           const uint32_t* ignore_links, uint32_t n_ignore,
                           uint64_t* dist64_out, uint32_t* dist32_out, uint32_t* nh_out,
                           uint32_t* pop_out);

/* Predecessor ("pathLinks") lists of one source given its distance row `dist`
 * (from spf_solve / spf_sssp with the same flags and ignore set), in the
 * reference's order (LinkState.cpp:857-873: predecessors u in Dijkstra pop
 * order, then u's links in linksFromNode(u) order).  Entries are directed
 * edge ids u->v.  pred_ptr = [n_nodes+1]; call with pred_edge == NULL first
 * to size (*n_preds). */
spf_status spf_preds(spf_ctx* ctx, uint32_t src, uint32_t flags,
                     const uint32_t* ignore_links, uint32_t n_ignore,
                     const uint32_t* dist, uint32_t* pred_ptr,
                     uint32_t* pred_edge, uint32_t cap, uint32_t* n_preds);

/* ---- batched KSP2: getKthPaths(src, dst, 1) and (src, dst, 2) ------------ */
/* For every pair (srcs[i], d), d = 0..n_nodes-1, the k = 1 and k = 2 paths the
 * reference returns from LinkState::getKthPaths (LinkState.cpp:762-791): k = 1
 * traces edge-disjoint paths in the SPF of src (traceOnePath, :398-419, with
 * the shared visited-link set); k = 2 re-runs SPF from src ignoring every link
 * of the k = 1 paths and traces again.  Paths are lists of undirected link
 * ids (spf_graph.link_id) in src -> dst order, in the reference's discovery
 * order.  src == dst and unreachable pairs have no paths.
 *
 * Output: pairs[i * n_nodes + d] (below) and a pool of u32 words holding path
 * records [n_links, next record offset (SPF_KSP2_NONE = last), link ids...];
 * the k = 1 and k = 2 lists of a pair start at first[0] / first[1].
 * Graphs with a metric <= 0, u64 labels, more than 65535 nodes or a
 * working set past the LDS run on the exact kernel (runSpf replayed in pop
 * order per pair, HBM scratch): same output, far slower. */
#define SPF_KSP2_NONE 0xFFFFFFFFu
typedef struct spf_ksp2_pair {
  uint32_t first[2];   /* pool offset of the first k = 1 / k = 2 record */
  uint32_t n_paths[2]; /* number of k = 1 / k = 2 paths                  */
} spf_ksp2_pair;

typedef struct spf_ksp2_plan spf_ksp2_plan;
spf_status spf_ksp2_plan_create(spf_ctx* ctx, const uint32_t* srcs, uint32_t n_src,
                                spf_ksp2_plan** out);
void spf_ksp2_plan_destroy(spf_ksp2_plan* plan);
/* Sources per KSP2 workgroup (a block is one destination x this many
 * sources; the graph is staged once per block): for traffic accounting. */
uint32_t spf_ksp2_plan_chunk(const spf_ksp2_plan* plan);
/* Enqueue on `stream` (NULL = context stream).  d_pairs = [n_src * n_nodes],
 * d_pool = pool_words u32, d_counters = 4 u64 zeroed by the call:
 *   [0] pool words claimed, reservations' unused tails included (may
 *       exceed pool_words without an overflow: bit 0 of [2] is the only
 *       overflow signal; the written words are at most min([0], pool_words)),
 *   [1] k = 2 SPF runs (the reference's un-memoised runSpf calls, :778-779),
 *   [2] bit 0 = overflow (bit 1: redo list full, never on plans made by
 *       spf_ksp2_plan_create, which size it for every pair),
 *   [3] pairs the u16-label waves of a compact plan handed to the u32 redo
 *       pass (labels past 65534 or paths deeper than 512 links; 0 otherwise).
 * No host synchronisation, no allocation. */
spf_status spf_ksp2_execute(spf_ksp2_plan* plan, spf_ksp2_pair* d_pairs, uint32_t* d_pool,
                            uint64_t pool_words, uint64_t* d_counters, void* stream);
/* Per-source digests of an execute's output, on the GPU (enqueued on
 * `stream`): d_out[i] = sum mod 2^64 over destinations d of
 * mix(h(i, d) + mix(d + 1)), h = FNV-1a over (0x1000 + n_paths[k], then per path
 * 0x2000 + length and link_hash[link] of each link) for k = 1, 2 and mix =
 * splitmix64's finaliser.  link_hash[id] identifies link `id` by value (the
 * caller hashes its ordered (node, ifname) key), so digests compare across
 * engines and the oracle.  What the parity checks of all-pairs KSP2 compare;
 * no reference counterpart. */
spf_status spf_ksp2_digest(spf_ksp2_plan* plan, const spf_ksp2_pair* d_pairs, const uint32_t* d_pool,
                           const uint64_t* d_link_hash, uint64_t* d_out, void* stream);
/* HIP-event kernel timing of the next `max_executes` executes: summed ms of
 * the k = 1 SPF kernel and of the KSP2 kernel. */
spf_status spf_ksp2_enable_timing(spf_ksp2_plan* plan, uint32_t max_executes);
spf_status spf_ksp2_timing(spf_ksp2_plan* plan, double* spf_ms, double* ksp_ms, uint32_t* n);
/* Convenience: plan + execute (growing the device pool on overflow) + copy
 * back.  pairs_out = [n_src * n_nodes]; the records are repacked densely in
 * pair order (k = 1 then k = 2, list order), so *pool_used -- the packed
 * size -- is the same on every call.  With pool_out == NULL or pool_cap <
 * *pool_used only the pairs are copied (the latter returns SPF_E_NOMEM): call
 * again with a pool of *pool_used words. */
spf_status spf_ksp2_solve(spf_ctx* ctx, const uint32_t* srcs, uint32_t n_src,
                          spf_ksp2_pair* pairs_out, uint32_t* pool_out, uint64_t pool_cap,
                          uint64_t* pool_used);

/* ---- what-if batches: one source, every single-link failure -------------- */
/* For each failed link l of the list: the reference's
 * runSpf(src, true, {l}) (LinkState.cpp:808-882 with linksToIgnore = {l}),
 * reduced to a digest against the unfailed runSpf(src):
 *   n_dist_changed  nodes whose metric changed (incl. becoming unreachable)
 *   n_nh_changed    nodes whose nextHops() changed (incl. becoming unreachable)
 *   hash            sum over reachable v of
 *                     mix(mix(v + 1) + metric(v)) ^ fnv1a64(nh(v) as u32 words)
 *                   mod 2^64, mix = splitmix64's finaliser, nh(v) = bitset over
 *                   the distinct up neighbours of src in the unfailed graph
 *                   (ascending id), ceil(k/32) words.
 * The unfailed result's digest is {0, 0, hash}.  Global-memory kernels, no
 * LDS size limit: repair scratch is sized from fixed HBM budgets (8 GB of
 * wave teams, 8 GB of workgroup teams, fewer teams on bigger graphs) plus
 * O(N) per plan; an allocation failure returns SPF_E_NOMEM.  Graphs with a
 * metric <= 0 or u64 labels run on the exact kernel: the unfailed run
 * replayed in pop order, and for every failure one of whose directions is a
 * pathLink of it, runSpf(src, true, {l}) replayed by one wavefront (the
 * others keep the unfailed digest). */
typedef struct spf_whatif_digest {
  uint32_t n_dist_changed;
  uint32_t n_nh_changed;
  uint64_t hash;
} spf_whatif_digest;

typedef struct spf_whatif_plan spf_whatif_plan;
/* fail_links: undirected link ids (spf_graph.link_id) of up links; NULL =
 * every up link of the graph in ascending id order. */
spf_status spf_whatif_plan_create(spf_ctx* ctx, uint32_t src, const uint32_t* fail_links,
                                  uint32_t n_fail, spf_whatif_plan** out);
void spf_whatif_plan_destroy(spf_whatif_plan* plan);
uint32_t spf_whatif_plan_failures(const spf_whatif_plan* plan);
spf_status spf_whatif_plan_links(const spf_whatif_plan* plan, uint32_t* links /* [n_fail] */);
/* d_out = [n_fail] digests, d_base = 1 digest (may be NULL).  Enqueued on
 * `stream` (a grid-resident launch for the unfailed solve); no host
 * synchronisation.  Failures with a large affected region are repaired on a
 * side stream owned by the ctx, forked from and joined back into `stream`
 * with events, so all work is ordered after earlier work on `stream` and
 * complete before later work on it.  Executes of plans sharing one ctx must
 * not overlap (one host thread per ctx, as elsewhere). */
spf_status spf_whatif_execute(spf_whatif_plan* plan, spf_whatif_digest* d_out,
                              spf_whatif_digest* d_base, void* stream);
/* After an execute: failures that needed a re-solve (tight links) and those
 * re-solved by whole workgroups (large affected region).  Waits for the last
 * execute's stream (SPF_E_STATE before the first execute). */
spf_status spf_whatif_stats(spf_whatif_plan* plan, uint32_t* n_hot, uint32_t* n_big);
spf_status spf_whatif_enable_timing(spf_whatif_plan* plan, uint32_t max_executes);
/* summed ms of the unfailed solve (SPF + next hops + hash) and of the failures */
spf_status spf_whatif_timing(spf_whatif_plan* plan, double* base_ms, double* fail_ms,
                             uint32_t* n);
/* Convenience: plan + execute + copy back. out = [n_fail] (n_fail = number of
 * up links when fail_links is NULL), base may be NULL. */
spf_status spf_whatif_solve(spf_ctx* ctx, uint32_t src, const uint32_t* fail_links,
                            uint32_t n_fail, spf_whatif_digest* out, spf_whatif_digest* base);

/* ---- SpfSolver next-hop selection (Decision.cpp:1082-1305) -------------- */
/* For node `me` and n_sets destination sets (set i = set_nodes[set_ptr[i] ..
 * set_ptr[i+1]), the advertisers of one prefix or the owner of one node
 * label, already filtered for reachability / drain as buildRouteDb does):
 *   getMinCostNodes      -> min_metric[i] (UINT64_MAX: no member reachable)
 *   getNextHopsWithMetric + getNextHopsThrift (single area, perDestination
 *   false) -> nh_count[i] next hops, each an up link of me (nh_edge = the
 *   directed CSR edge me -> neighbour, so link_id[] and the metric advertised
 *   by me come with it) and its metric w(link) + dist(neighbour, dst)
 *   (nh_metric).  Without SPF_ROUTE_LFA only links on shortest paths are
 *   kept; with it every neighbour passing the RFC 5286 condition of
 *   Decision.cpp:1180 is added.
 * nh_edge / nh_metric hold deg(me) entries per set: [n_sets * deg(me)], where
 * deg(me) = row_ptr[me+1] - row_ptr[me]. */
#define SPF_ROUTE_LFA 0x1u
spf_status spf_routes(spf_ctx* ctx, uint32_t me, const uint32_t* set_ptr,
                      const uint32_t* set_nodes, uint32_t n_sets, uint32_t flags,
                      uint64_t* min_metric, uint32_t* nh_count, uint32_t* nh_edge,
                      uint64_t* nh_metric);

/* ---- multi-device context: several GPUs behind one host thread ----------- */
/* SURVEY.md §8(b)'s spf_ctx_create(gpu_ids, ngpu): Open/R's Decision runs in
 * one process on one event-base thread (Decision.cpp:1484), so the GPUs of a
 * node are reached from one context, not a process per GPU.  An spf_mctx
 * holds one member engine context per listed device id (ids may repeat: the
 * members of one device share its execute stream and run one after another
 * there), each with a replica of the graph.  An spf_mplan splits a batch of
 * sources over the members and keeps each member's distance rows and
 * next-hop bitmaps resident in that member's HBM; queries are answered by the
 * owning member.  Results are bit-identical to one spf_plan over the batch.
 *
 * Partition of the sources (also usable on its own, host only):
 *   SPF_PARTITION_CONTIGUOUS  blocks of the request order balanced by the
 *                             bytes each source's results take (k + 40
 *                             bitmaps, k = distinct up neighbours)
 *   SPF_PARTITION_LOCALITY    a streaming partition keeping each member's
 *                             closure (sources + their neighbours, whose rows
 *                             the next-hop pass reads) small: a fabric's pods
 *                             and planes stay together
 *   SPF_PARTITION_AUTO        locality when its largest closure is smaller
 *                             (graphs up to 65,536 nodes), else contiguous */
#define SPF_PARTITION_AUTO 0u
#define SPF_PARTITION_CONTIGUOUS 1u
#define SPF_PARTITION_LOCALITY 2u
/* nb_ptr/nb_id: distinct up neighbours per node (spf_src_neighbors of every
 * node, CSR form); part_out[i] = part of srcs[i]; *mode_used = the rule taken. */
spf_status spf_partition_sources(const uint32_t* nb_ptr, const uint32_t* nb_id, uint32_t n_nodes,
                                 const uint32_t* srcs, uint32_t n_src, uint32_t n_parts,
                                 uint32_t mode, uint32_t* part_out, uint32_t* mode_used);

typedef struct spf_mctx spf_mctx;
typedef struct spf_mplan spf_mplan;
spf_status spf_mctx_create(const int* gpu_ids, uint32_t n, spf_mctx** out);
void spf_mctx_destroy(spf_mctx* m);
const char* spf_mctx_last_error(const spf_mctx* m);
uint32_t spf_mctx_size(const spf_mctx* m);
/* member i's engine context (owned by the mctx; every single-context call
 * works on it) and its device id */
spf_ctx* spf_mctx_member(spf_mctx* m, uint32_t i);
int spf_mctx_device(const spf_mctx* m, uint32_t i);
/* graph replicated to every member; patches applied to every replica */
spf_status spf_mctx_graph_load(spf_mctx* m, const spf_graph* g);
spf_status spf_mctx_graph_set_overload(spf_mctx* m, const uint32_t* nodes,
                                       const uint8_t* overloaded, uint32_t n);
spf_status spf_mctx_graph_patch_rows(spf_mctx* m, const uint32_t* nodes, uint32_t n,
                                     const uint32_t* col, const int32_t* metric, const uint32_t* link);
spf_status spf_mctx_graph_set_metric(spf_mctx* m, const uint32_t* edges, const int32_t* metric,
                                     uint32_t n);

/* A batch of sources split over the members (partition `mode`), result
 * buffers owned by the plan on each member's device. */
spf_status spf_mplan_create(spf_mctx* m, const uint32_t* srcs, uint32_t n_src, uint32_t flags,
                            uint32_t mode, spf_mplan** out);
void spf_mplan_destroy(spf_mplan* mp);
uint32_t spf_mplan_partition(const spf_mplan* mp);   /* SPF_PARTITION_* taken */
/* request index i (srcs[i]) -> owning member, row in that member's plan */
spf_status spf_mplan_owner(const spf_mplan* mp, uint32_t i, uint32_t* member, uint32_t* row);
/* member's share: its plan (spf_plan_nh_layout etc.), its resident device
 * buffers ([n][pitch] rows, next-hop words) -- for device-side consumers */
spf_status spf_mplan_shard(spf_mplan* mp, uint32_t member, uint32_t* n_src, spf_plan** plan,
                           void** d_dist, uint32_t** d_nh);
uint32_t spf_mplan_closure_rows(const spf_mplan* mp, uint32_t member);
/* enable != 0: each member's execute is captured into a hipGraph after the
 * first execute of a graph epoch and replayed after that (re-captured after
 * an in-place patch) */
spf_status spf_mplan_set_graphs(spf_mplan* mp, int enable);
/* Host enqueue threads: mode 1 issues each member's execute from its own host
 * thread (spinning briefly between back-to-back executes, then sleeping), 0
 * from the caller's thread one member after another, -1 (default) threads
 * when the members with work sit on two or more distinct devices. */
spf_status spf_mplan_set_enqueue_threads(spf_mplan* mp, int mode);
/* The last execute's host enqueue: out[i] = ns from the execute's start until
 * member i's launches were enqueued (0 for members without work); *threaded =
 * 1 when it used the enqueue threads.  The spread of out[] is the start
 * stagger the members' GPUs see. */
spf_status spf_mplan_enqueue_ns(const spf_mplan* mp, uint64_t* out, uint32_t n, int* threaded);
/* Enqueue every member's execute on its device's stream; no host wait. */
spf_status spf_mplan_execute(spf_mplan* mp);
/* Wait for every member and check its grid / team barriers (spf_device_check). */
spf_status spf_mplan_synchronize(spf_mplan* mp);
/* Per-source digests (spf_plan_digest's hash) in request order, computed on
 * each owning device; waits. */
spf_status spf_mplan_digest(spf_mplan* mp, uint64_t* out);
/* Source i's result from its owner: dist = [n_nodes] (u32, u64 with
 * SPF_FLAG_DIST64), nh = k bitmaps of spf_row_pitch/32 words (k = distinct up
 * neighbours of srcs[i]); either may be NULL.  Waits for the owner's stream. */
spf_status spf_mplan_read(spf_mplan* mp, uint32_t i, void* dist, uint32_t* nh);
/* pathLinks of source i (spf_preds' output) from the resident row on its
 * owning device; SPF_E_UNSUPPORTED for zero / negative metrics and u64 rows. */
spf_status spf_mplan_preds(spf_mplan* mp, uint32_t i, uint32_t* pred_ptr, uint32_t* pred_edge,
                           uint32_t cap, uint32_t* n_preds);
/* Route selection of many nodes from the resident pass (no new SPF): the
 * reference's getNextHopsWithMetric + getNextHopsThrift (Decision.cpp:
 * 1082-1305, perDestination = false, one area) of every me = srcs[me_req[t]]
 * towards every destination set p (set_ptr / set_nodes as spf_routes),
 * evaluated on me's owning device from its resident row and bitmaps (LFA:
 * every neighbour's resident row, read over peer access when it lives on
 * another device).  What Decision::getDecisionRouteDb(node) for every node
 * (Decision.cpp:1480-1500) computes, minus the thrift formatting.
 * spf_mplan_route_digests: per me, digests[t] = sum over sets p with a kept
 * next hop of mix(mix(0x9e3779b97f4a7c15 (p+1) + shortest) + sum over kept
 * links of mix(link_hash[link id] + (u32) metric) + p) (mix = splitmix64's
 * finaliser; link_hash[id] identifies link `id` by value, as for
 * spf_ksp2_digest); *kernel_ms (optional) = the slowest member's kernel time.
 * spf_mplan_routes: one me's records in spf_routes' layout.  Rows must be u32
 * link-metric rows (not SPF_FLAG_HOP_COUNT / SPF_FLAG_DIST64). */
spf_status spf_mplan_route_digests(spf_mplan* mp, const uint32_t* me_req, uint32_t n_me,
                                   const uint32_t* set_ptr, const uint32_t* set_nodes,
                                   uint32_t n_sets, uint32_t flags, const uint64_t* link_hash,
                                   uint32_t n_links, uint64_t* digests, double* kernel_ms);
spf_status spf_mplan_routes(spf_mplan* mp, uint32_t me_req, const uint32_t* set_ptr,
                            const uint32_t* set_nodes, uint32_t n_sets, uint32_t flags,
                            uint64_t* min_metric, uint32_t* nh_count, uint32_t* nh_edge,
                            uint64_t* nh_metric);
/* Every me's route database materialised on its owning device (the same
 * selection as spf_mplan_route_digests, written out instead of hashed): what
 * Decision::getDecisionRouteDb(node) returns for every node (Decision.cpp:
 * 1480-1500 -> buildRouteDb :556-722, one area), in device memory.  Per me t
 * and set p a header word = offset | count << 32 | stride << 48: the route's
 * k-th next hop (k < count) is record offset + k * stride of me's region, a
 * u64 = CSR edge (me -> neighbour: link id, interface, neighbour and the
 * metric me advertises come with it) | metric << 32 (w(link) +
 * dist(neighbour, dst)), in me's link order -- getNextHopsThrift's next
 * hops.  Device layout: me's region is one [deg(me)][1024] tile per 1024
 * sets (stride 1024), so consecutive routes' k-th next hops are adjacent; a
 * region holds ceil(n_sets / 1024) * 1024 * deg(me) record slots (unused ones
 * are never written).  Sets without a kept next hop have count 0.
 * SPF_E_UNSUPPORTED when a metric exceeds 2^32 - 1 or a region 2^32 slots.
 * *n_records (optional) = records over every me; *kernel_ms (optional) = the
 * slowest member's kernel.  The databases stay resident until the next call. */
spf_status spf_mplan_route_records(spf_mplan* mp, const uint32_t* me_req, uint32_t n_me,
                                   const uint32_t* set_ptr, const uint32_t* set_nodes, uint32_t n_sets,
                                   uint32_t flags, uint64_t* n_records, double* kernel_ms);
/* me t's database from the last spf_mplan_route_records, compacted on the
 * host: hdr = [n_sets] headers offset | count << 32 (stride 1: route p's next
 * hops contiguous, routes in set order; may be NULL), rec = its records (cap
 * entries; SPF_E_NOMEM when fewer than *n; may be NULL), *n = its record
 * count.  Waits. */
spf_status spf_mplan_route_db(spf_mplan* mp, uint32_t t, uint64_t* hdr, uint64_t* rec, uint64_t cap,
                              uint64_t* n);
/* HIP-event time of each member's executes: ms[member] summed over the last
 * executes since enable / the last call, *n = executes. */
spf_status spf_mplan_enable_timing(spf_mplan* mp, uint32_t max_executes);
spf_status spf_mplan_timing(spf_mplan* mp, double* ms, uint32_t* n);

/* ---- diagnostics ---------------------------------------------------------- */
/* With SPF_STAMPS set in the environment, the multi-source BFS kernel records
 * s_memtime clocks of workgroup 0 at its phase boundaries (init, then per level:
 * distance stores, pull sweep, barrier; end), per wave: out[w*64] = count,
 * out[w*64 + 1 ..] = clocks of wave w (16 waves).  Copies up to cap words. */
spf_status spf_debug_stamps(spf_ctx* ctx, uint64_t* out, uint32_t cap, uint32_t* n);
/* The device's practical HBM ceiling: a 16-byte grid-stride copy of `bytes`
 * (read + written per rep, `reps` reps timed with HIP events) -> *gbs in
 * GB/s of bytes moved.  What bench.py reports beside the 8 TB/s peak
 * (BASELINE.md §4).  No reference counterpart. */
spf_status spf_debug_copy_bandwidth(spf_ctx* ctx, uint64_t bytes, uint32_t reps, double* gbs);

/* Waits for every launch on the context's device and reports whether a
 * grid-resident kernel's barrier of THIS context (spf_big_kernel, the
 * what-if unfailed pass, the global-memory SSSP, the what-if group teams,
 * the team BFS) gave up waiting: its spin is bounded so a block that never
 * arrives cannot hang the GPU, and the outputs of that launch are then
 * invalid.  Each context has its own fault word, so another context's
 * timeout is neither reported nor cleared here.  SPF_E_HIP (and the word is
 * cleared) when one did; SPF_OK otherwise.  Such launches of one process
 * are serialised per device (one cannot starve another of CUs), so a timeout
 * means a fault or a foreign process holding the CUs.  The synchronous
 * convenience calls (spf_solve, spf_whatif_solve, spf_whatif_stats, ...)
 * check it themselves.  No reference counterpart. */
spf_status spf_device_check(spf_ctx* ctx);

/* ---- counters ----------------------------------------------------------- */
/* Logical single-source solves executed (the reference's decision.spf_runs,
 * LinkState.cpp:815) and kernel time of the last execute in ms. */
uint64_t spf_solves(const spf_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_SPF_H_ */
