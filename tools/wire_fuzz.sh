#!/bin/bash
# Build tools/wire_fuzz.cpp with ASan + UBSan (host code only) and run it on
# a corpus of CompactProtocol buffers from tests/thrift_compact.py.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d)
cd "$T"
python3 - "$ROOT" <<'PY'
import sys
import numpy as np
root = sys.argv[1]
sys.path[:0] = [root + "/tests", root]
from thrift_compact import encode_adjacency_database, encode_publication
from test_wire import _random_db
rng = np.random.default_rng(5)
with open("corpus.bin", "wb") as f:
    for n in (0, 3, 20):
        b = encode_adjacency_database(_random_db(rng, f"x{n}", n), unknown=True, perf_events=True)
        p = encode_publication([(f"adj:x{n}", b), ("adj:y", None)], expired=["adj:z"], area="a")
        for x in (b, p):
            f.write(len(x).to_bytes(4, "little") + x)
PY
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -I"$ROOT/include" \
    "$ROOT/tools/wire_fuzz.cpp" "$ROOT/openr_amd/csrc/lsdb_wire.cpp" -o wire_fuzz
./wire_fuzz
