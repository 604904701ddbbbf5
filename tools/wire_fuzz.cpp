// Host-only sanitizer fuzz of the LSDB wire decoder (csrc/lsdb_wire.cpp):
// truncations and byte flips of encoded databases / publications must decode
// or be refused, never read out of bounds.  The LinkState entry points that
// ls_apply_publication calls are stubbed.  Run: bash tools/wire_fuzz.sh
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include "openr_wire.h"
extern "C" {
const char* ls_get_area(const ls_state*) { return "a"; }
const char* ls_last_error(const ls_state*) { return ""; }
spf_status ls_update_adjacency_databases(ls_state*, const openr_lsdb*, uint64_t, uint64_t, ls_change*) { return SPF_OK; }
spf_status ls_delete_adjacency_database(ls_state*, const char*, ls_change*) { return SPF_OK; }
}
int main() {
  FILE* f = fopen("corpus.bin", "rb");
  std::vector<std::vector<uint8_t>> c;
  uint32_t n;
  while (fread(&n, 4, 1, f) == 1) {
    std::vector<uint8_t> b(n);
    if (fread(b.data(), 1, n, f) != n) return 1;
    c.push_back(b);
  }
  std::mt19937 rng(1);
  long ok = 0, bad = 0;
  for (int it = 0; it < 200000; ++it) {
    std::vector<uint8_t> b = c[it % c.size()];
    int mode = rng() % 3;
    if (mode == 0 && !b.empty()) b.resize(rng() % b.size());
    else if (mode == 1) for (int k = 0; k < 1 + (int)(rng() % 4); ++k) if (!b.empty()) b[rng() % b.size()] = rng();
    openr_wire_lsdb* w = nullptr;
    spf_status st = (it & 1) ? openr_wire_decode_publication(b.data(), b.size(), &w)
                             : openr_wire_decode_adjdb(b.data(), b.size(), &w);
    if (st == SPF_OK) { ++ok; const openr_lsdb* v = openr_wire_view(w); volatile uint32_t s = 0; for (uint32_t d = 0; d < v->n_dbs; ++d) s += v->dbs[d].adj_count; openr_wire_free(w); } else ++bad;
    ls_change ch;
    ls_apply_publication((ls_state*)&ch, b.data(), b.size(), nullptr, nullptr, &ch);
  }
  printf("ok %ld bad %ld\n", ok, bad);
}
