"""The C-ABI library loads and exports every function include/*.h declares
(no device needed: nothing is computed)."""

import ctypes
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    names = set()
    for h in sorted((ROOT / "include").glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b([a-z][a-z0-9_]*)\s*\(", text, re.M):
            name = m.group(1)
            if name in ("if", "defined", "sizeof"):
                continue
            names.add(name)
    return names


def test_headers_declare_expected_entry_points():
    names = declared_functions()
    for must in ("spf_ctx_create", "spf_graph_load", "spf_plan_execute", "spf_solve",
                 "spf_sssp", "spf_preds", "ls_create", "ls_update_adjacency_databases",
                 "ls_get_spf_result", "ls_get_kth_paths"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from openr_amd import _native

    lib = ctypes.CDLL(str(_native.LIB_PATH))
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding declares a prototype for each of them
    assert declared_functions() <= set(_native.PROTOTYPES), (
        declared_functions() - set(_native.PROTOTYPES))


def test_no_device_is_reported_not_faked():
    """Without a GPU the engine refuses loudly instead of falling back."""
    import torch

    if torch.cuda.is_available():
        return
    from openr_amd import _native as N

    h = ctypes.c_void_p()
    st = N.lib.spf_ctx_create(0, ctypes.byref(h))
    assert st == N.SPF_E_NO_DEVICE
    assert N.global_error()
