"""openr_amd -- MI355X-native SPF engine for Open/R's Decision module.

The hot path of the reference (``LinkState::getSpfResult`` / ``getKthPaths``,
openr/decision/LinkState.cpp:762-882) re-designed as batched HIP kernels for
gfx950 behind a C-ABI (include/openr_spf.h, include/openr_linkstate.h).

Modules:
  lsdb        thrift-equivalent input types + packed C-ABI layout
  topology    synthetic topologies (reference grid/fabric generators, WAN, BA)
  link_state  drop-in ``LinkState`` (reference API) over the engine
  engine      batched all-sources API on device buffers
"""

__all__ = ["lsdb", "topology", "link_state", "engine"]
