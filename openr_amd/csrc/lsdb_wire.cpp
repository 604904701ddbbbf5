// ============================================================================
//  lsdb_wire.cpp -- LSDB wire ingest (include/openr_wire.h).
//
//  Decision reads adjacency databases out of KvStore publications as thrift
//  CompactProtocol blobs (reference openr/decision/Decision.cpp:1726-1760,
//  CompactSerializer).  This file decodes them straight into the packed LSDB
//  the engine ingests (openr_lsdb.h) -- one string blob, fixed-size records --
//  with no thrift runtime: a bounds-checked CompactProtocol reader, one
//  decoder per struct of the schema (Lsdb.thrift:71-129, KvStore.thrift:21-41,
//  226-247, Network.thrift:55-58) that keeps the fields the LinkState needs and
//  skips everything else generically.
//
//  CompactProtocol, as the decoder reads it:
//    field header  byte (delta << 4 | type); delta 0 = a zigzag-varint i16
//                  field id follows; 0x00 ends a struct; bool fields carry
//                  their value in the type (1 true, 2 false)
//    i16/i32/i64   zigzag varint          double  8 bytes LE   float  4 bytes
//    binary        varint length + bytes
//    list/set      byte (size << 4 | elem type), size 15 = varint size follows
//                  (bool elements: one byte each)
//    map           varint size; if > 0, byte (key type << 4 | value type)
//  Types: 1/2 bool, 3 byte, 4 i16, 5 i32, 6 i64, 7 double, 8 binary, 9 list,
//  10 set, 11 map, 12 struct, 13 float.
// ============================================================================
#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "openr_wire.h"

namespace {

thread_local std::string g_wire_err;

enum : int {
  kBoolTrue = 1, kBoolFalse = 2, kByte = 3, kI16 = 4, kI32 = 5, kI64 = 6, kDouble = 7,
  kBinary = 8, kList = 9, kSet = 10, kMap = 11, kStruct = 12, kFloat = 13
};
constexpr int kMaxDepth = 64;

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;

  bool fail() { return ok = false; }
  uint8_t byte() {
    if (p >= end) { fail(); return 0; }
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      const uint8_t b = byte();
      if (!ok) return 0;
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
    }
    fail();
    return 0;
  }
  int64_t zz64() {
    const uint64_t u = varint();
    return (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
  }
  int32_t zz32() { return (int32_t)zz64(); }
  std::string_view binary() {
    const uint64_t n = varint();
    if (!ok || n > (uint64_t)(end - p)) { fail(); return {}; }
    std::string_view s(reinterpret_cast<const char*>(p), (size_t)n);
    p += n;
    return s;
  }
  void skip_bytes(uint64_t n) {
    if (n > (uint64_t)(end - p)) { fail(); return; }
    p += n;
  }
  // Field header; false at the struct's STOP byte (or on error).
  bool field(int16_t& id, int& type) {
    const uint8_t b = byte();
    if (!ok || b == 0) return false;
    type = b & 0x0F;
    const int delta = b >> 4;
    id = delta ? (int16_t)(id + delta) : (int16_t)zz32();
    return ok;
  }
  // list/set header
  void list(uint32_t& n, int& etype) {
    const uint8_t b = byte();
    etype = b & 0x0F;
    uint64_t size = b >> 4;
    if (size == 15) size = varint();
    if (size > (uint64_t)(end - p)) fail();  // every element takes >= 1 byte
    n = ok ? (uint32_t)size : 0;
  }
  bool read_bool(int type, bool in_container) {
    if (in_container) return byte() == kBoolTrue;
    return type == kBoolTrue;
  }
  // Skip a value of `type` (in_container: bools take a byte).
  void skip(int type, bool in_container, int depth = 0) {
    if (depth > kMaxDepth) { fail(); return; }
    switch (type) {
      case kBoolTrue:
      case kBoolFalse:
        if (in_container) byte();
        return;
      case kByte: byte(); return;
      case kI16: case kI32: case kI64: varint(); return;
      case kDouble: skip_bytes(8); return;
      case kFloat: skip_bytes(4); return;
      case kBinary: binary(); return;
      case kList:
      case kSet: {
        uint32_t n; int et;
        list(n, et);
        for (uint32_t i = 0; i < n && ok; ++i) skip(et, true, depth + 1);
        return;
      }
      case kMap: {
        const uint64_t n = varint();
        if (!ok || n == 0) return;
        if (n > (uint64_t)(end - p)) { fail(); return; }
        const uint8_t kv = byte();
        for (uint64_t i = 0; i < n && ok; ++i) {
          skip(kv >> 4, true, depth + 1);
          skip(kv & 0x0F, true, depth + 1);
        }
        return;
      }
      case kStruct: {
        int16_t id = 0; int t;
        while (ok && field(id, t)) skip(t, false, depth + 1);
        return;
      }
      default: fail(); return;
    }
  }
};

// Decoded databases in the packed layout of openr_lsdb.h.
struct Packed {
  std::string blob;
  std::vector<openr_db_rec> dbs;
  std::vector<openr_adj_rec> adjs;

  void str(std::string_view s, uint32_t* off, uint32_t* len) {
    *off = (uint32_t)blob.size();
    *len = (uint32_t)s.size();
    if (!s.empty()) blob.append(s.data(), s.size());
  }
};

// thrift::BinaryAddress (Network.thrift:55-58): the address bytes
void decode_address(Reader& r, uint8_t* out, size_t width) {
  std::memset(out, 0, width);
  int16_t id = 0; int t;
  while (r.ok && r.field(id, t)) {
    if (id == 1 && t == kBinary) {
      const std::string_view a = r.binary();
      if (!a.empty()) std::memcpy(out, a.data(), std::min(a.size(), width));
    } else {
      r.skip(t, false);
    }
  }
}

// thrift::Adjacency (Lsdb.thrift:71-105)
void decode_adjacency(Reader& r, Packed& pk, openr_adj_rec& a) {
  std::memset(&a, 0, sizeof a);
  a.weight = 1;  // IDL default (10: i64 weight = 1)
  std::string_view other, ifn, oif;
  int16_t id = 0; int t;
  while (r.ok && r.field(id, t)) {
    switch (id) {
      case 1: if (t == kBinary) { other = r.binary(); continue; } break;
      case 2: if (t == kBinary) { ifn = r.binary(); continue; } break;
      case 3: if (t == kStruct) { decode_address(r, a.nh_v6, 16); continue; } break;
      case 5: if (t == kStruct) { decode_address(r, a.nh_v4, 4); continue; } break;
      case 4: if (t == kI32) { a.metric = r.zz32(); continue; } break;
      case 6: if (t == kI32) { a.adj_label = r.zz32(); continue; } break;
      case 7: if (t == kBoolTrue || t == kBoolFalse) { a.is_overloaded = r.read_bool(t, false); continue; } break;
      case 8: if (t == kI32) { a.rtt = r.zz32(); continue; } break;
      case 9: if (t == kI64) { a.timestamp = r.zz64(); continue; } break;
      case 10: if (t == kI64) { a.weight = r.zz64(); continue; } break;
      case 11: if (t == kBinary) { oif = r.binary(); continue; } break;
      default: break;
    }
    r.skip(t, false);  // unknown field, or a known id with a foreign type
  }
  pk.str(other, &a.other_off, &a.other_len);
  pk.str(ifn, &a.if_off, &a.if_len);
  pk.str(oif, &a.oif_off, &a.oif_len);
}

// thrift::AdjacencyDatabase (Lsdb.thrift:109-129) -> one db record + its
// adjacencies appended to pk.  Returns the node name (for the key check).
std::string decode_adjdb(Reader& r, Packed& pk, const std::string* area_override) {
  openr_db_rec d{};
  std::string_view name, area;  // 6: string area, no declared default (Lsdb.thrift:128)
  std::vector<openr_adj_rec> adjs;
  int16_t id = 0; int t;
  while (r.ok && r.field(id, t)) {
    switch (id) {
      case 1: if (t == kBinary) { name = r.binary(); continue; } break;
      case 2: if (t == kBoolTrue || t == kBoolFalse) { d.is_overloaded = r.read_bool(t, false); continue; } break;
      case 3:
        if (t == kList) {
          uint32_t n; int et;
          r.list(n, et);
          if (et != kStruct && n) { r.fail(); continue; }
          adjs.resize(n);
          for (uint32_t k = 0; k < n && r.ok; ++k) decode_adjacency(r, pk, adjs[k]);
          continue;
        }
        break;
      case 4: if (t == kI32) { d.node_label = r.zz32(); continue; } break;
      case 6: if (t == kBinary) { area = r.binary(); continue; } break;
      default: break;  // 5: optional PerfEvents perfEvents -- not link state
    }
    r.skip(t, false);
  }
  if (!r.ok) return {};
  pk.str(name, &d.name_off, &d.name_len);
  pk.str(area_override ? std::string_view(*area_override) : area, &d.area_off, &d.area_len);
  d.adj_begin = (uint32_t)pk.adjs.size();
  d.adj_count = (uint32_t)adjs.size();
  pk.adjs.insert(pk.adjs.end(), adjs.begin(), adjs.end());
  pk.dbs.push_back(d);
  return std::string(name);
}

// getNodeNameFromKey (openr/common/Util.cpp:1013-1020): the second
// ':'-separated token, "" when there is none.
std::string node_from_key(std::string_view key) {
  const size_t a = key.find(':');
  if (a == std::string_view::npos) return {};
  const size_t b = key.find(':', a + 1);
  return std::string(key.substr(a + 1, b == std::string_view::npos ? std::string_view::npos : b - a - 1));
}

constexpr std::string_view kAdjDbMarker = "adj:";  // Constants.h:201

spf_status wire_fail(spf_status st, const std::string& msg) {
  g_wire_err = msg;
  return st;
}

}  // namespace

struct openr_wire_lsdb {
  Packed pk;
  std::string area = "0";
  std::vector<std::string> expired;
  uint32_t skipped = 0;
  openr_lsdb view{};

  void finish() {
    view.blob = pk.blob.data();
    view.dbs = pk.dbs.data();
    view.n_dbs = (uint32_t)pk.dbs.size();
    view.adjs = pk.adjs.data();
  }
};

extern "C" {

spf_status openr_wire_decode_adjdb(const uint8_t* buf, size_t len, openr_wire_lsdb** out) {
  if (!out || (!buf && len)) return wire_fail(SPF_E_INVALID, "null argument");
  *out = nullptr;
  auto w = std::make_unique<openr_wire_lsdb>();
  Reader r{buf, buf + len};
  decode_adjdb(r, w->pk, nullptr);
  if (!r.ok) return wire_fail(SPF_E_INVALID, "malformed thrift::AdjacencyDatabase (CompactProtocol)");
  w->area.assign(w->pk.blob.data() + w->pk.dbs[0].area_off, w->pk.dbs[0].area_len);
  w->finish();
  *out = w.release();
  return SPF_OK;
}

spf_status openr_wire_decode_publication(const uint8_t* buf, size_t len, openr_wire_lsdb** out) {
  if (!out || (!buf && len)) return wire_fail(SPF_E_INVALID, "null argument");
  *out = nullptr;
  auto w = std::make_unique<openr_wire_lsdb>();
  // Values are decoded after the whole publication is read: the area
  // (field 7) may follow the key-values (field 2).
  struct AdjVal { std::string node; std::string_view value; };
  std::vector<AdjVal> vals;
  Reader r{buf, buf + len};
  int16_t id = 0; int t;
  while (r.ok && r.field(id, t)) {
    if (id == 2 && t == kMap) {  // keyVals: map<string, Value>
      const uint64_t n = r.varint();
      if (!r.ok || n == 0) continue;
      const uint8_t kv = r.byte();
      if ((kv >> 4) != kBinary || (kv & 0x0F) != kStruct) { r.fail(); break; }
      // The reference walks keyVals as the std::unordered_map<std::string,
      // Value> fbthrift deserialises it into (KvStore.thrift:43-44,
      // Decision.cpp:1726): reserved for the map's size, then filled in wire
      // order.  The order databases are applied decides the order links
      // enter the per-node link sets, hence linksFromNode order and the
      // KSP2 / pathLinks tie-breaks -- so build the same container here
      // (libstdc++ on both sides) and iterate it.
      struct Entry { bool adj = false, has_value = false; std::string_view value; };
      std::unordered_map<std::string, Entry> key_vals;
      key_vals.reserve(n);
      for (uint64_t i = 0; i < n && r.ok; ++i) {
        const std::string_view key = r.binary();
        Entry e;
        int16_t vid = 0; int vt;
        while (r.ok && r.field(vid, vt)) {  // thrift::Value (KvStore.thrift:21-41)
          if (vid == 2 && vt == kBinary) {
            e.value = r.binary();
            e.has_value = true;
          } else {
            r.skip(vt, false);
          }
        }
        e.adj = key.substr(0, kAdjDbMarker.size()) == kAdjDbMarker;
        if (r.ok) key_vals.emplace(std::string(key), e);
      }
      for (const auto& kvp : key_vals)  // a TTL update carries no value (Decision.cpp:1728-1732)
        if (kvp.second.adj && kvp.second.has_value)
          vals.push_back({node_from_key(kvp.first), kvp.second.value});
    } else if (id == 3 && t == kList) {  // expiredKeys: list<string>
      uint32_t n; int et;
      r.list(n, et);
      for (uint32_t i = 0; i < n && r.ok; ++i) {
        if (et != kBinary) { r.skip(et, true); continue; }
        const std::string_view key = r.binary();
        if (r.ok && key.substr(0, kAdjDbMarker.size()) == kAdjDbMarker)
          w->expired.push_back(node_from_key(key));
      }
    } else if (id == 7 && t == kBinary) {  // area
      w->area = std::string(r.binary());
    } else {
      r.skip(t, false);  // nodeIds, tobeUpdatedKeys, floodRootId
    }
  }
  if (!r.ok) return wire_fail(SPF_E_INVALID, "malformed thrift::Publication (CompactProtocol)");
  if (w->area.empty())  // CHECK(not thriftPub.area_ref()->empty()), Decision.cpp:1711
    return wire_fail(SPF_E_INVALID, "publication with an empty area");
  for (const AdjVal& v : vals) {
    Reader vr{reinterpret_cast<const uint8_t*>(v.value.data()),
              reinterpret_cast<const uint8_t*>(v.value.data()) + v.value.size()};
    const size_t blob0 = w->pk.blob.size(), adj0 = w->pk.adjs.size(), db0 = w->pk.dbs.size();
    const std::string name = decode_adjdb(vr, w->pk, &w->area);
    if (!vr.ok) {  // Decision logs "Failed to deserialize" and moves on
      w->pk.blob.resize(blob0);
      w->pk.adjs.resize(adj0);
      w->pk.dbs.resize(db0);
      ++w->skipped;
      continue;
    }
    if (name != v.node)  // CHECK_EQ(nodeName, thisNodeName), Decision.cpp:1746
      return wire_fail(SPF_E_INVALID, "adj:" + v.node + " carries the database of node '" + name + "'");
  }
  w->finish();
  *out = w.release();
  return SPF_OK;
}

const openr_lsdb* openr_wire_view(const openr_wire_lsdb* w) { return w ? &w->view : nullptr; }
const char* openr_wire_area(const openr_wire_lsdb* w) { return w ? w->area.c_str() : nullptr; }
uint32_t openr_wire_n_expired(const openr_wire_lsdb* w) { return w ? (uint32_t)w->expired.size() : 0; }
const char* openr_wire_expired(const openr_wire_lsdb* w, uint32_t i) {
  return w && i < w->expired.size() ? w->expired[i].c_str() : nullptr;
}
uint32_t openr_wire_n_skipped(const openr_wire_lsdb* w) { return w ? w->skipped : 0; }
void openr_wire_free(openr_wire_lsdb* w) { delete w; }
const char* openr_wire_last_error(void) { return g_wire_err.c_str(); }

spf_status ls_apply_publication_ordered(ls_state* ls, const uint8_t* buf, size_t len,
                                        const char* my_node, uint32_t* n_updated,
                                        uint32_t* n_deleted, ls_change* agg) {
  if (!ls) return wire_fail(SPF_E_INVALID, "null LinkState");
  openr_wire_lsdb* w = nullptr;
  spf_status st = openr_wire_decode_publication(buf, len, &w);
  if (st != SPF_OK) return st;
  std::unique_ptr<openr_wire_lsdb> hold(w);
  if (agg) std::memset(agg, 0, sizeof *agg);
  const char* ls_area = ls_get_area(ls);
  if (w->area != ls_area)
    return wire_fail(SPF_E_INVALID, "publication of area '" + w->area +
                                        "' applied to the LinkState of area '" + ls_area + "'");
  const uint32_t n = w->view.n_dbs;
  std::vector<ls_change> ch(n ? n : 1);
  if (!my_node) {
    st = ls_update_adjacency_databases(ls, &w->view, 0, 0, ch.data());
    if (st != SPF_OK) return wire_fail(st, ls_last_error(ls));
  } else {
    // enable_ordered_fib_programming (Decision.cpp:1750-1758): each database
    // is held for the hop count from this node to its originator (hold up)
    // and the rest of the originator's eccentricity (hold down), both read
    // from the link state as it stands before that database is applied.
    for (uint32_t i = 0; i < n; ++i) {
      const openr_db_rec& d = w->view.dbs[i];
      const std::string node(w->view.blob + d.name_off, d.name_len);
      uint64_t up = 0, down = 0, hops = 0, max_hops = 0;
      int has = 0;
      st = ls_get_metric_a_to_b(ls, my_node, node.c_str(), 0, &hops, &has);
      if (st != SPF_OK) return wire_fail(st, ls_last_error(ls));
      if (has) {
        st = ls_get_max_hops_to_node(ls, node.c_str(), &max_hops);
        if (st != SPF_OK) return wire_fail(st, ls_last_error(ls));
        up = hops;
        down = max_hops - hops;
      }
      openr_lsdb one = w->view;
      one.dbs = w->view.dbs + i;
      one.n_dbs = 1;
      st = ls_update_adjacency_databases(ls, &one, up, down, &ch[i]);
      if (st != SPF_OK) return wire_fail(st, ls_last_error(ls));
    }
  }
  ls_change one{};
  for (const std::string& node : w->expired) {
    st = ls_delete_adjacency_database(ls, node.c_str(), &one);
    if (st != SPF_OK) return wire_fail(st, ls_last_error(ls));
    ch.push_back(one);
  }
  if (agg)
    for (const ls_change& c : ch) {
      agg->topology_changed |= c.topology_changed;
      agg->link_attributes_changed |= c.link_attributes_changed;
      agg->node_label_changed |= c.node_label_changed;
    }
  if (n_updated) *n_updated = n;
  if (n_deleted) *n_deleted = (uint32_t)w->expired.size();
  return SPF_OK;
}

spf_status ls_apply_publication(ls_state* ls, const uint8_t* buf, size_t len, uint32_t* n_updated,
                                uint32_t* n_deleted, ls_change* agg) {
  return ls_apply_publication_ordered(ls, buf, len, nullptr, n_updated, n_deleted, agg);
}

}  // extern "C"
