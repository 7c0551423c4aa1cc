"""The C-ABI library loads and exports every function include/prysm_hip.h declares (no GPU
needed: nothing is called except the version query)."""
import ctypes
import os
import re

from prysm_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "prysm_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pz_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    dll = ctypes.CDLL(_lib.library_path)
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(dll, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(declared_functions()) <= set(_lib.SIGNATURES)


def test_version():
    assert _lib.lib.dll.pz_version() == 1


def test_epoch_batch_struct_layout():
    # pz_epoch_batch is passed by pointer from ctypes: field order/packing must match the header
    src = open(os.path.join(ROOT, "include", "prysm_hip.h")).read()
    body = src[src.index("typedef struct pz_epoch_batch"):src.index("} pz_epoch_batch;")]
    body = re.sub(r"/\*.*?\*/", "", body.split("{", 1)[1], flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:
            first, *rest = decl.split(",")
            fields += [first.split()[-1].lstrip("*")] + [r.strip().lstrip("*") for r in rest]
    assert fields == [f for f, _ in _lib.EpochBatch._fields_]
