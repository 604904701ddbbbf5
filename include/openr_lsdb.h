/*
 * openr_lsdb.h -- packed link-state-database layout shared by every C-ABI
 * entry point that ingests adjacency databases.
 *
 * It carries the fields of the reference's thrift input types
 *   thrift::Adjacency          (reference openr/if/Lsdb.thrift:71-105)
 *   thrift::AdjacencyDatabase  (reference openr/if/Lsdb.thrift:109-129)
 * without thrift: every string lives in one byte blob and is referenced by
 * (offset, length); databases and adjacencies are fixed-size records.
 * openr_amd/lsdb.py builds this layout with numpy (DB_DTYPE / ADJ_DTYPE).
 */
#ifndef OPENR_LSDB_H_
#define OPENR_LSDB_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One thrift::AdjacencyDatabase (32 bytes). */
typedef struct openr_db_rec {
  uint32_t name_off, name_len;   /* thisNodeName                          */
  uint32_t area_off, area_len;   /* area                                  */
  int32_t is_overloaded;         /* isOverloaded (node drain bit)         */
  int32_t node_label;            /* nodeLabel                             */
  uint32_t adj_begin, adj_count; /* adjacencies = adj[adj_begin .. +count) */
} openr_db_rec;

/* One thrift::Adjacency (80 bytes). */
typedef struct openr_adj_rec {
  uint32_t other_off, other_len; /* otherNodeName */
  uint32_t if_off, if_len;       /* ifName        */
  uint32_t oif_off, oif_len;     /* otherIfName   */
  int32_t metric;                /* metric (i32; the link metric from this side) */
  int32_t adj_label;             /* adjLabel      */
  int32_t is_overloaded;         /* isOverloaded  (link drain bit from this side) */
  int32_t rtt;                   /* rtt           */
  int64_t timestamp;             /* timestamp     */
  int64_t weight;                /* weight        */
  uint8_t nh_v6[16];             /* nextHopV6 address bytes */
  uint8_t nh_v4[4];              /* nextHopV4 address bytes */
  uint8_t pad[4];
} openr_adj_rec;

/* A packed batch of adjacency databases. */
typedef struct openr_lsdb {
  const char* blob;              /* all strings, referenced by offset */
  const openr_db_rec* dbs;
  uint32_t n_dbs;
  const openr_adj_rec* adjs;     /* indexed by openr_db_rec.adj_begin */
} openr_lsdb;

#ifdef __cplusplus
}
#endif
#endif /* OPENR_LSDB_H_ */
