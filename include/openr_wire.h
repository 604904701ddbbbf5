/*
 * openr_wire.h -- LSDB wire ingest (libopenr_spf.so): the thrift
 * CompactProtocol values Decision reads from KvStore publications, decoded
 * into the packed LSDB of openr_lsdb.h.
 *
 * Reference interfaces replaced:
 *   fbzmq::util::readThriftObjStr<thrift::AdjacencyDatabase>(value,
 *       apache::thrift::CompactSerializer)     (openr/decision/Decision.cpp:1743-1745)
 *                                              -> openr_wire_decode_adjdb
 *   the link-state half of Decision::processPublication
 *       (openr/decision/Decision.cpp:1709-1760 "adj:" updates,
 *        :1806-1817 expired "adj:" keys)       -> openr_wire_decode_publication,
 *                                                 ls_apply_publication
 * Schemas: thrift::Publication / thrift::Value (openr/if/KvStore.thrift:21-41,
 * 226-247), thrift::AdjacencyDatabase / thrift::Adjacency
 * (openr/if/Lsdb.thrift:71-129), thrift::BinaryAddress (Network.thrift:55-58).
 * Unknown fields are skipped, absent fields take the IDL defaults
 * (adjLabel 0, isOverloaded false, weight 1, otherIfName "", area "0").
 *
 * Errors: spf_status codes; openr_wire_last_error() describes the last
 * failure of the calling thread.  A value that does not decode is skipped and
 * counted (the reference logs and continues, Decision.cpp:1799-1802); a
 * database whose thisNodeName differs from its key's node name fails the
 * whole publication (the reference CHECK-fails, :1746).
 */
#ifndef OPENR_WIRE_H_
#define OPENR_WIRE_H_

#include <stddef.h>
#include <stdint.h>

#include "openr_linkstate.h"
#include "openr_lsdb.h"
#include "openr_spf.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Decoded databases (packed view) + expired adjacency keys; owned by the
 * caller, freed with openr_wire_free. */
typedef struct openr_wire_lsdb openr_wire_lsdb;

/* One serialized thrift::AdjacencyDatabase. */
spf_status openr_wire_decode_adjdb(const uint8_t* buf, size_t len, openr_wire_lsdb** out);

/* One serialized thrift::Publication: every keyVals entry whose key starts
 * with "adj:" and carries a value becomes a database (area = the
 * publication's area); every expired "adj:" key contributes its node name
 * (getNodeNameFromKey, openr/common/Util.cpp:1013-1020).  Other keys
 * (prefix:, fibTime:) are not link state and are ignored.  Databases come
 * out in the iteration order of the keyVals container the reference
 * deserialises into (std::unordered_map<std::string, Value>,
 * KvStore.thrift:43-44, reserved for the map size and filled in wire order),
 * which is the order Decision::processPublication applies them in
 * (Decision.cpp:1726). */
spf_status openr_wire_decode_publication(const uint8_t* buf, size_t len,
                                         openr_wire_lsdb** out);

const openr_lsdb* openr_wire_view(const openr_wire_lsdb* w);
const char* openr_wire_area(const openr_wire_lsdb* w);
uint32_t openr_wire_n_expired(const openr_wire_lsdb* w);
const char* openr_wire_expired(const openr_wire_lsdb* w, uint32_t i);
uint32_t openr_wire_n_skipped(const openr_wire_lsdb* w); /* values that failed to decode */
void openr_wire_free(openr_wire_lsdb* w);
const char* openr_wire_last_error(void);

/* Decision::processPublication for one area's LinkState: decode, apply every
 * adjacency database (updateAdjacencyDatabase, holds 0/0), then delete the
 * expired ones (deleteAdjacencyDatabase).  The publication's area must be the
 * LinkState's.  *agg ORs the LinkStateChange flags of every step;
 * *n_updated / *n_deleted count them (any pointer may be NULL). */
spf_status ls_apply_publication(ls_state* ls, const uint8_t* buf, size_t len,
                                uint32_t* n_updated, uint32_t* n_deleted, ls_change* agg);
/* The same with enable_ordered_fib_programming (Decision.cpp:1750-1758):
 * my_node != NULL applies the databases one at a time, each with hold-up
 * TTL = getHopsFromAToB(my_node, originator) and hold-down TTL =
 * getMaxHopsToNode(originator) - hold-up (0/0 when the originator is not
 * reachable), read before that database is applied; needs a device-backed
 * LinkState.  my_node == NULL is ls_apply_publication. */
spf_status ls_apply_publication_ordered(ls_state* ls, const uint8_t* buf, size_t len,
                                        const char* my_node, uint32_t* n_updated,
                                        uint32_t* n_deleted, ls_change* agg);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_WIRE_H_ */
