"""Build libopenr_spf.so in-tree for gfx950 (hipcc, no JIT cache).

    python -m openr_amd.build [--force]

Sources: every openr_amd/csrc/*.hip (HIP kernels + engine C-ABI) and *.cpp
(link_state.cpp: LinkState facade C-ABI; lsdb_wire.cpp: LSDB wire ingest);
headers in include/.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OUT = PKG / "lib" / "libopenr_spf.so"
SOURCES = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
INTERNAL = sorted(CSRC.glob("*.h"))
HEADERS = sorted((ROOT / "include").glob("*.h"))


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not OUT.exists():
        return True
    t = OUT.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS + INTERNAL)


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return OUT
    OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = OUT.with_suffix(".so.tmp")
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", f"-I{ROOT / 'include'}", *map(str, SOURCES), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    tmp.replace(OUT)
    return OUT


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
