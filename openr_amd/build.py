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
    """Compile every source to an object in parallel (hipcc -c, one process
    per file, at most 8), then link the shared library."""
    from concurrent.futures import ThreadPoolExecutor

    if not force and not needs_build():
        return OUT
    OUT.parent.mkdir(parents=True, exist_ok=True)
    obj_dir = OUT.parent / "obj"
    obj_dir.mkdir(exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
             f"-I{ROOT / 'include'}"]

    def compile_one(src: Path) -> Path:
        obj = obj_dir / (src.name + ".o")
        cmd = [hipcc(), *flags, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")), 8))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = OUT.with_suffix(".so.tmp")
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", *map(str, objs), "-o",
           str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    tmp.replace(OUT)
    return OUT


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
