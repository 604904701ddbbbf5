"""ctypes binding of libopenr_spf.so (include/openr_spf.h, openr_linkstate.h).

The library is built in-tree by ``python -m openr_amd.build`` (or
``__graft_entry__.build()``) into ``openr_amd/lib/libopenr_spf.so``.  There is
no fallback: if the library is missing, importing this module raises.
"""

from __future__ import annotations

import atexit
import ctypes as C
import os
import weakref
from pathlib import Path

import numpy as np

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libopenr_spf.so"
if os.environ.get("OPENR_SPF_LIB"):  # experiments: an alternative in-tree build
    LIB_PATH = Path(os.environ["OPENR_SPF_LIB"]).resolve()

SPF_OK = 0
SPF_E_INVALID = 1
SPF_E_UNSUPPORTED = 2
SPF_E_HIP = 3
SPF_E_NO_DEVICE = 4
SPF_E_NOMEM = 5
SPF_E_STATE = 6
SPF_UNREACHABLE = 0xFFFFFFFF
SPF_FLAG_HOP_COUNT = 0x1
SPF_FLAG_DIST64 = 0x2
SPF_UNREACHABLE64 = 0xFFFFFFFFFFFFFFFF
SPF_KSP2_NONE = 0xFFFFFFFF
SPF_ROUTE_LFA = 0x1
SPF_PARTITION_AUTO = 0
SPF_PARTITION_CONTIGUOUS = 1
SPF_PARTITION_LOCALITY = 2
PARTITION_NAMES = {SPF_PARTITION_CONTIGUOUS: "contiguous", SPF_PARTITION_LOCALITY: "locality"}

_STATUS_NAMES = {
    SPF_E_INVALID: "SPF_E_INVALID",
    SPF_E_UNSUPPORTED: "SPF_E_UNSUPPORTED",
    SPF_E_HIP: "SPF_E_HIP",
    SPF_E_NO_DEVICE: "SPF_E_NO_DEVICE",
    SPF_E_NOMEM: "SPF_E_NOMEM",
    SPF_E_STATE: "SPF_E_STATE",
}


class SpfError(RuntimeError):
    def __init__(self, status: int, msg: str) -> None:
        super().__init__(f"{_STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class UnsupportedInput(SpfError):
    """Input outside the engine's exact-parity envelope (SPF_E_UNSUPPORTED)."""


class NoDevice(SpfError):
    """No gfx950 device (SPF_E_NO_DEVICE)."""


def raise_for(status: int, msg: str) -> None:
    if status == SPF_OK:
        return
    if status == SPF_E_UNSUPPORTED:
        raise UnsupportedInput(status, msg)
    if status == SPF_E_NO_DEVICE:
        raise NoDevice(status, msg)
    raise SpfError(status, msg)


# ---- structs -----------------------------------------------------------------
class SpfGraph(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("n_edges", C.c_uint32),
        ("row_ptr", C.POINTER(C.c_uint32)),
        ("col", C.POINTER(C.c_uint32)),
        ("metric", C.POINTER(C.c_int32)),
        ("link_id", C.POINTER(C.c_uint32)),
        ("overloaded", C.POINTER(C.c_uint8)),
    ]


class OpenrLsdb(C.Structure):
    _fields_ = [
        ("blob", C.c_char_p),
        ("dbs", C.c_void_p),
        ("n_dbs", C.c_uint32),
        ("adjs", C.c_void_p),
    ]


class LsChange(C.Structure):
    _fields_ = [
        ("topology_changed", C.c_uint8),
        ("link_attributes_changed", C.c_uint8),
        ("node_label_changed", C.c_uint8),
        ("pad", C.c_uint8),
    ]


class LsLinkDesc(C.Structure):
    _fields_ = [
        ("node1", C.c_uint32), ("node2", C.c_uint32),
        ("if1", C.c_char_p), ("if2", C.c_char_p),
        ("first_node", C.c_uint32), ("second_node", C.c_uint32),
        ("metric1", C.c_uint64), ("metric2", C.c_uint64),
        ("adj_label1", C.c_int32), ("adj_label2", C.c_int32),
        ("overload1", C.c_uint8), ("overload2", C.c_uint8),
        ("is_up", C.c_uint8), ("pad", C.c_uint8),
        ("hash", C.c_uint64),
        ("nh_v4_1", C.POINTER(C.c_uint8)), ("nh_v4_2", C.POINTER(C.c_uint8)),
        ("nh_v6_1", C.POINTER(C.c_uint8)), ("nh_v6_2", C.POINTER(C.c_uint8)),
    ]


class LsSpfView(C.Structure):
    _fields_ = [
        ("n", C.c_uint32),
        ("node", C.POINTER(C.c_uint32)),
        ("metric", C.POINTER(C.c_uint64)),
        ("nh_ptr", C.POINTER(C.c_uint32)),
        ("nh_node", C.POINTER(C.c_uint32)),
        ("pl_ptr", C.POINTER(C.c_uint32)),
        ("pl_link", C.POINTER(C.c_uint32)),
        ("pl_prev", C.POINTER(C.c_uint32)),
    ]


class LsPathsView(C.Structure):
    _fields_ = [
        ("n_paths", C.c_uint32),
        ("path_ptr", C.POINTER(C.c_uint32)),
        ("link", C.POINTER(C.c_uint32)),
    ]


class DcMetricEntity(C.Structure):  # openr_decision.h dc_metric_entity
    _fields_ = [("type", C.c_int64), ("priority", C.c_int64), ("op", C.c_uint32),
                ("is_tie_breaker", C.c_uint32), ("n_metric", C.c_uint32),
                ("metric", C.POINTER(C.c_int64))]


class DcPrefixEntry(C.Structure):  # openr_decision.h dc_prefix_entry
    _fields_ = [("prefix", C.c_char_p), ("is_v4", C.c_uint8), ("is_bgp", C.c_uint8),
                ("forwarding_type", C.c_uint8), ("forwarding_algorithm", C.c_uint8),
                ("has_prepend_label", C.c_uint8), ("has_min_nexthop", C.c_uint8),
                ("has_mv", C.c_uint8), ("pad", C.c_uint8), ("prepend_label", C.c_int32),
                ("min_nexthop", C.c_int64), ("path_preference", C.c_int32),
                ("source_preference", C.c_int32), ("distance", C.c_int32),
                ("mv_version", C.c_int32), ("n_mv", C.c_uint32),
                ("mv", C.POINTER(DcMetricEntity))]


class DcNexthop(C.Structure):  # openr_decision.h dc_nexthop
    _fields_ = [("address", C.c_uint8 * 16), ("address_len", C.c_uint8),
                ("mpls_action", C.c_uint8), ("n_push", C.c_uint8), ("pad", C.c_uint8),
                ("metric", C.c_int32), ("swap_label", C.c_int32), ("push_off", C.c_uint32),
                ("ifname", C.c_uint32), ("area", C.c_uint32), ("neighbor", C.c_uint32)]


# numpy view of dc_nexthop records (the route db's table, read in one copy)
DC_NEXTHOP_DTYPE = np.dtype([("address", "u1", (16,)), ("address_len", "u1"),
                             ("mpls_action", "u1"), ("n_push", "u1"), ("pad", "u1"),
                             ("metric", "<i4"), ("swap_label", "<i4"), ("push_off", "<u4"),
                             ("ifname", "<u4"), ("area", "<u4"), ("neighbor", "<u4")])
DC_NONE = 0xFFFFFFFF
DC_MPLS_ACTIONS = (None, "PUSH", "SWAP", "PHP", "POP_AND_LOOKUP")

_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p

# name -> (restype, argtypes); also the list of exported symbols checked by tests
PROTOTYPES = {
    # engine (openr_spf.h)
    "spf_ctx_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "spf_ctx_destroy": (None, [_vp]),
    "spf_last_error": (C.c_char_p, [_vp]),
    "spf_global_error": (C.c_char_p, []),
    "spf_graph_load": (C.c_int, [_vp, C.POINTER(SpfGraph)]),
    "spf_graph_set_overload": (C.c_int, [_vp, _u32p, _u8p, C.c_uint32]),
    "spf_graph_set_metric": (C.c_int, [_vp, _u32p, _i32p, C.c_uint32]),
    "spf_graph_patch_rows": (C.c_int, [_vp, _u32p, C.c_uint32, _u32p, _i32p, _u32p]),
    "spf_mctx_graph_patch_rows": (C.c_int, [_vp, _u32p, C.c_uint32, _u32p, _i32p, _u32p]),
    "spf_graph_epoch": (C.c_uint64, [_vp]),
    "spf_graph_loads": (C.c_uint64, [_vp]),
    "spf_row_pitch": (C.c_uint32, [_vp]),
    "spf_graph_has_nonpositive_metric": (C.c_int, [_vp]),
    "spf_src_neighbors": (C.c_int, [_vp, C.c_uint32, _u32p, C.c_uint32, _u32p]),
    "spf_plan_create": (C.c_int, [_vp, _u32p, C.c_uint32, C.c_uint32, C.POINTER(_vp)]),
    "spf_plan_destroy": (None, [_vp]),
    "spf_plan_nh_words": (C.c_uint64, [_vp]),
    "spf_plan_nh_layout": (C.c_int, [_vp, _u64p, _u32p]),
    "spf_plan_closure_rows": (C.c_uint32, [_vp]),
    "spf_plan_kernels": (C.c_int, [_vp, _u32p, _u32p]),
    "spf_plan_traffic": (C.c_int, [_vp, _u64p, _u64p]),
    "spf_plan_traffic_phases": (C.c_int, [_vp, _u64p]),
    "spf_plan_execute": (C.c_int, [_vp, _vp, _vp, _vp]),
    "spf_plan_copy_narrow_rows": (C.c_int, [_vp, _vp, _vp]),
    "spf_plan_digest": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "spf_plan_execute_host": (C.c_int, [_vp, _u32p, _u32p]),
    "spf_plan_enable_timing": (C.c_int, [_vp, C.c_uint32]),
    "spf_plan_timing": (C.c_int, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double), _u32p]),
    "spf_plan_timing_phases": (C.c_int, [_vp, C.POINTER(C.c_double), _u32p]),
    "spf_solve": (C.c_int, [_vp, _u32p, C.c_uint32, C.c_uint32, _u32p, _u32p]),
    "spf_sssp": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _u32p, C.c_uint32, _u32p]),
    "spf_solve_exact": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _u32p, C.c_uint32, _u64p, _u32p,
                                  _u32p, _u32p]),
    "spf_graph_needs_dist64": (C.c_int, [_vp]),
    "spf_preds": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _u32p, C.c_uint32, _u32p,
                            _u32p, _u32p, C.c_uint32, _u32p]),
    "spf_solves": (C.c_uint64, [_vp]),
    "spf_device_check": (C.c_int, [_vp]),
    "spf_debug_stamps": (C.c_int, [_vp, _u64p, C.c_uint32, _u32p]),
    "spf_debug_copy_bandwidth": (C.c_int, [_vp, C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]),
    "spf_ksp2_plan_create": (C.c_int, [_vp, _u32p, C.c_uint32, C.POINTER(_vp)]),
    "spf_ksp2_plan_destroy": (None, [_vp]),
    "spf_ksp2_plan_chunk": (C.c_uint32, [_vp]),
    "spf_ksp2_execute": (C.c_int, [_vp, _vp, _vp, C.c_uint64, _vp, _vp]),
    "spf_ksp2_digest": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "spf_ksp2_enable_timing": (C.c_int, [_vp, C.c_uint32]),
    "spf_ksp2_timing": (C.c_int, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double), _u32p]),
    "spf_ksp2_solve": (C.c_int, [_vp, _u32p, C.c_uint32, _u32p, _u32p, C.c_uint64, _u64p]),
    "spf_whatif_plan_create": (C.c_int, [_vp, C.c_uint32, _u32p, C.c_uint32, C.POINTER(_vp)]),
    "spf_whatif_plan_destroy": (None, [_vp]),
    "spf_whatif_plan_failures": (C.c_uint32, [_vp]),
    "spf_whatif_plan_links": (C.c_int, [_vp, _u32p]),
    "spf_whatif_execute": (C.c_int, [_vp, _vp, _vp, _vp]),
    "spf_whatif_stats": (C.c_int, [_vp, _u32p, _u32p]),
    "spf_whatif_enable_timing": (C.c_int, [_vp, C.c_uint32]),
    "spf_whatif_timing": (C.c_int, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double), _u32p]),
    "spf_whatif_solve": (C.c_int, [_vp, C.c_uint32, _u32p, C.c_uint32, _vp, _vp]),
    "spf_routes": (C.c_int, [_vp, C.c_uint32, _u32p, _u32p, C.c_uint32, C.c_uint32, _u64p,
                             _u32p, _u32p, _u64p]),
    # multi-device context (openr_spf.h)
    "spf_partition_sources": (C.c_int, [_u32p, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                        C.c_uint32, _u32p, _u32p]),
    "spf_mctx_create": (C.c_int, [C.POINTER(C.c_int), C.c_uint32, C.POINTER(_vp)]),
    "spf_mctx_destroy": (None, [_vp]),
    "spf_mctx_last_error": (C.c_char_p, [_vp]),
    "spf_mctx_size": (C.c_uint32, [_vp]),
    "spf_mctx_member": (_vp, [_vp, C.c_uint32]),
    "spf_mctx_device": (C.c_int, [_vp, C.c_uint32]),
    "spf_mctx_graph_load": (C.c_int, [_vp, C.POINTER(SpfGraph)]),
    "spf_mctx_graph_set_overload": (C.c_int, [_vp, _u32p, _u8p, C.c_uint32]),
    "spf_mctx_graph_set_metric": (C.c_int, [_vp, _u32p, _i32p, C.c_uint32]),
    "spf_mplan_create": (C.c_int, [_vp, _u32p, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.POINTER(_vp)]),
    "spf_mplan_destroy": (None, [_vp]),
    "spf_mplan_partition": (C.c_uint32, [_vp]),
    "spf_mplan_owner": (C.c_int, [_vp, C.c_uint32, _u32p, _u32p]),
    "spf_mplan_shard": (C.c_int, [_vp, C.c_uint32, _u32p, C.POINTER(_vp), C.POINTER(_vp),
                                  C.POINTER(_vp)]),
    "spf_mplan_closure_rows": (C.c_uint32, [_vp, C.c_uint32]),
    "spf_mplan_set_graphs": (C.c_int, [_vp, C.c_int]),
    "spf_mplan_set_enqueue_threads": (C.c_int, [_vp, C.c_int]),
    "spf_mplan_route_records": (C.c_int, [_vp, _u32p, C.c_uint32, _u32p, _u32p, C.c_uint32, C.c_uint32,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
    "spf_mplan_route_db": (C.c_int, [_vp, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                     C.c_uint64, C.POINTER(C.c_uint64)]),
    "spf_mplan_enqueue_ns": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_int)]),
    "spf_mplan_execute": (C.c_int, [_vp]),
    "spf_mplan_synchronize": (C.c_int, [_vp]),
    "spf_mplan_digest": (C.c_int, [_vp, _u64p]),
    "spf_mplan_read": (C.c_int, [_vp, C.c_uint32, _vp, _u32p]),
    "spf_mplan_route_digests": (C.c_int, [_vp, _u32p, C.c_uint32, _u32p, _u32p, C.c_uint32, C.c_uint32,
                                          _u64p, C.c_uint32, _u64p, C.POINTER(C.c_double)]),
    "spf_mplan_routes": (C.c_int, [_vp, C.c_uint32, _u32p, _u32p, C.c_uint32, C.c_uint32, _u64p, _u32p,
                                   _u32p, _u64p]),
    "spf_mplan_preds": (C.c_int, [_vp, C.c_uint32, _u32p, _u32p, C.c_uint32, _u32p]),
    "spf_mplan_enable_timing": (C.c_int, [_vp, C.c_uint32]),
    "spf_mplan_timing": (C.c_int, [_vp, C.POINTER(C.c_double), _u32p]),
    # LinkState facade (openr_linkstate.h)
    "ls_create": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_vp)]),
    "ls_create_multi": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.c_uint32, C.POINTER(_vp)]),
    "ls_prefetch_all_sources": (C.c_int, [_vp, C.c_int]),
    "ls_all_sources_plan": (_vp, [_vp]),
    "ls_destroy": (None, [_vp]),
    "ls_last_error": (C.c_char_p, [_vp]),
    "ls_get_area": (C.c_char_p, [_vp]),
    "ls_update_adjacency_databases": (C.c_int, [_vp, C.POINTER(OpenrLsdb), C.c_uint64,
                                                C.c_uint64, C.POINTER(LsChange)]),
    "ls_delete_adjacency_database": (C.c_int, [_vp, C.c_char_p, C.POINTER(LsChange)]),
    "ls_decrement_holds": (C.c_int, [_vp, C.POINTER(LsChange)]),
    "ls_has_holds": (C.c_int, [_vp]),
    "ls_num_links": (C.c_uint64, [_vp]),
    "ls_num_nodes": (C.c_uint64, [_vp]),
    "ls_has_node": (C.c_int, [_vp, C.c_char_p]),
    "ls_is_node_overloaded": (C.c_int, [_vp, C.c_char_p]),
    "ls_name_id": (C.c_uint32, [_vp, C.c_char_p]),
    "ls_name": (C.c_char_p, [_vp, C.c_uint32]),
    "ls_adjacency_databases": (C.c_int, [_vp, _u32p, _i32p, C.c_uint32, _u32p]),
    "ls_links_from_node": (C.c_int, [_vp, C.c_char_p, _u32p, C.c_uint32, _u32p]),
    "ls_link_info": (C.c_int, [_vp, C.c_uint32, C.POINTER(LsLinkDesc)]),
    "ls_get_spf_result": (C.c_int, [_vp, C.c_char_p, C.c_int, C.POINTER(LsSpfView)]),
    "ls_prefetch_kth_paths": (C.c_int, [_vp, C.c_char_p]),
    "ls_prefetch_spf_results": (C.c_int, [_vp, _vp, C.c_uint32, C.c_int]),
    "ls_debug_phase_ns": (None, [_vp, _vp]),
    "spf_plan_preds": (C.c_int, [_vp, _vp, _vp, C.c_uint64, _vp]),
    "ls_get_kth_paths": (C.c_int, [_vp, C.c_char_p, C.c_char_p, C.c_uint64,
                                   C.POINTER(LsPathsView)]),
    "ls_get_metric_a_to_b": (C.c_int, [_vp, C.c_char_p, C.c_char_p, C.c_int, _u64p,
                                       C.POINTER(C.c_int)]),
    "ls_get_max_hops_to_node": (C.c_int, [_vp, C.c_char_p, _u64p]),
    "ls_spf_runs": (C.c_uint64, [_vp]),
    "ls_engine": (_vp, [_vp]),
    "ls_flatten": (C.c_int, [_vp, _u32p, _u32p]),
    "ls_graph_node_names": (C.c_int, [_vp, _u32p]),
    "ls_graph_csr": (C.c_int, [_vp, _u32p, _u32p, _i32p, _u32p, _u8p]),
    # LSDB wire ingest (openr_wire.h)
    "openr_wire_decode_adjdb": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_vp)]),
    "openr_wire_decode_publication": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_vp)]),
    "openr_wire_view": (C.POINTER(OpenrLsdb), [_vp]),
    "openr_wire_area": (C.c_char_p, [_vp]),
    "openr_wire_n_expired": (C.c_uint32, [_vp]),
    "openr_wire_expired": (C.c_char_p, [_vp, C.c_uint32]),
    "openr_wire_n_skipped": (C.c_uint32, [_vp]),
    "openr_wire_free": (None, [_vp]),
    "openr_wire_last_error": (C.c_char_p, []),
    "ls_apply_publication": (C.c_int, [_vp, C.c_char_p, C.c_size_t, _u32p, _u32p,
                                       C.POINTER(LsChange)]),
    "ls_link_create": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int32, C.c_int32,
                                 C.c_int, C.c_char_p, C.c_char_p, C.c_int32, C.c_int32, C.c_int,
                                 C.POINTER(_vp)]),
    "ls_link_destroy": (None, [_vp]),
    "ls_link_area": (C.c_char_p, [_vp]),
    "ls_link_hash": (C.c_uint64, [_vp]),
    "ls_link_is_up": (C.c_int, [_vp]),
    "ls_link_equal": (C.c_int, [_vp, _vp]),
    "ls_link_less": (C.c_int, [_vp, _vp]),
    "ls_link_other_node": (C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_char_p)]),
    "ls_link_iface": (C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_char_p)]),
    "ls_link_metric": (C.c_int, [_vp, C.c_char_p, _u64p]),
    "ls_link_adj_label": (C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_int32)]),
    "ls_link_overload": (C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_int)]),
    "ls_link_set_metric": (C.c_int, [_vp, C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                     C.POINTER(C.c_int)]),
    "ls_link_set_overload": (C.c_int, [_vp, C.c_char_p, C.c_int, C.c_uint64, C.c_uint64,
                                       C.POINTER(C.c_int)]),
    "ls_path_a_in_path_b": (C.c_int, [_u32p, C.c_uint32, _u32p, C.c_uint32]),
    "ls_string_map_order": (C.c_int, [C.POINTER(C.c_char_p), C.c_uint32, _u32p, _u32p]),
    "ls_node_area_map_order": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                         C.POINTER(C.c_uint8), C.c_uint32, _u32p, _u32p]),
    "ls_graph_epoch": (C.c_uint64, [_vp]),
    "ls_get_spf_metrics": (C.c_int, [_vp, C.c_char_p, C.c_int, C.POINTER(LsSpfView)]),
    "ls_serial": (C.c_uint64, [_vp]),
    "ls_debug_row_patches": (C.c_uint64, [_vp]),
    "ls_is_node_overloaded_id": (C.c_int, [_vp, C.c_uint32]),
    # SpfSolver / PrefixState (include/openr_decision.h)
    "dc_prefix_state_create": (_vp, []),
    "dc_prefix_state_destroy": (None, [_vp]),
    "dc_prefix_update": (C.c_int, [_vp, C.c_char_p, C.c_char_p, C.POINTER(DcPrefixEntry)]),
    "dc_prefix_delete": (C.c_int, [_vp, C.c_char_p, C.c_char_p, C.c_char_p]),
    "dc_prefix_entries": (C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                    C.c_uint32, _u32p]),
    "dc_solver_create": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.POINTER(C.c_void_p)]),
    "dc_solver_destroy": (None, [_vp]),
    "dc_last_error": (C.c_char_p, [_vp]),
    "dc_static_mpls_route_set": (C.c_int, [_vp, C.c_int32, C.POINTER(DcNexthop), C.c_uint32,
                                           C.POINTER(C.c_char_p), C.POINTER(C.c_int32)]),
    "dc_static_mpls_route_delete": (C.c_int, [_vp, C.c_int32]),
    "dc_build_route_db": (C.c_int, [_vp, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p), C.c_uint32,
                                    _vp, C.POINTER(C.c_void_p)]),
    "dc_counter": (C.c_uint64, [_vp, C.c_char_p]),
    "dc_best_route": (C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_uint32, _u32p]),
    "dc_debug_phase_ns": (None, [_vp, _u64p]),
    "dc_route_db_destroy": (None, [_vp]),
    "dc_route_db_strings": (C.c_uint32, [_vp]),
    "dc_route_db_string": (C.c_char_p, [_vp, C.c_uint32]),
    "dc_route_db_nexthops": (C.c_void_p, [_vp, _u32p]),
    "dc_route_db_labels": (C.c_void_p, [_vp, _u32p]),
    "dc_route_db_unicast_count": (C.c_uint32, [_vp]),
    "dc_route_db_unicast": (C.c_int, [_vp, C.c_uint32, _u32p, _u32p, _u32p, C.POINTER(C.c_int),
                                      _u32p, _u32p]),
    "dc_route_db_mpls_count": (C.c_uint32, [_vp]),
    "dc_route_db_mpls": (C.c_int, [_vp, C.c_uint32, _i32p, _u32p, _u32p]),
    "dc_route_db_unicast_table": (C.c_void_p, [_vp, _u32p]),
    "dc_route_db_mpls_table": (C.c_void_p, [_vp, _u32p]),
    "ls_holdable_create": (_vp, [C.c_int, C.c_uint64]),
    "ls_holdable_destroy": (None, [_vp]),
    "ls_holdable_value": (C.c_uint64, [_vp]),
    "ls_holdable_has_hold": (C.c_int, [_vp]),
    "ls_holdable_decrement_ttl": (C.c_int, [_vp]),
    "ls_holdable_update_value": (C.c_int, [_vp, C.c_uint64, C.c_uint64, C.c_uint64]),
    "ls_apply_publication_ordered": (C.c_int, [_vp, C.c_char_p, C.c_size_t, C.c_char_p, _u32p,
                                               _u32p, C.POINTER(LsChange)]),
}


def _load() -> C.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -m openr_amd.build` "
            "(the SPF path has no CPU fallback)"
        )
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def ptr(a: np.ndarray, ctype=C.c_uint32):
    """ctypes pointer to a C-contiguous numpy array (caller keeps it alive)."""
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(ctype))


def global_error() -> str:
    return (lib.spf_global_error() or b"").decode()


def lsdb_struct(packed) -> OpenrLsdb:
    """OpenrLsdb view of a PackedLsdb (keep `packed` alive while in use)."""
    s = OpenrLsdb()
    s.blob = packed.blob
    s.dbs = packed.dbs.ctypes.data
    s.n_dbs = len(packed.dbs)
    s.adjs = packed.adjs.ctypes.data if len(packed.adjs) else None
    return s


# ---- lifetime of native handles -------------------------------------------------
class NativeHandle:
    """Owner of one C-ABI object (plan or context) with an explicit close().

    Device memory, streams and events are released by close() -- or by the
    context manager -- in a defined order: plans before the context they were
    created on.  Handles still open when the interpreter exits are closed by
    an atexit hook in the same order, before the HIP runtime's own teardown
    runs (destroying them from a garbage-collector finaliser after that point
    is what crashed profiled runs at exit)."""

    _LEVEL = 0  # closed in ascending level at exit: plans 0, contexts 1
    _destroy = ""

    def _adopt(self, h: C.c_void_p) -> None:
        self._h = h
        _LIVE.add(self)

    def close(self) -> None:
        h = getattr(self, "_h", None)
        lib = globals().get("lib")  # None during interpreter shutdown
        if h is not None and h.value and lib is not None and getattr(self, "_owned", True):
            getattr(lib, self._destroy)(h)
        self._h = C.c_void_p()
        _LIVE.discard(self)

    @property
    def closed(self) -> bool:
        h = getattr(self, "_h", None)
        return h is None or not h.value

    def __enter__(self):
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self) -> None:
        self.close()


_LIVE: "weakref.WeakSet[NativeHandle]" = weakref.WeakSet()


def close_all() -> None:
    """Close every open plan, then every open context (registered atexit)."""
    for obj in sorted(list(_LIVE), key=lambda o: o._LEVEL):
        obj.close()


atexit.register(close_all)
