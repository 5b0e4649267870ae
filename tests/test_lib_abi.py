"""CPU checks of the C-ABI boundary: the library builds/loads and exports every symbol the
header declares; ctypes signatures cover them.  No GPU work."""
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "alignn_hip.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(alignn_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    for must in ("alignn_gemm_f32", "alignn_graph_prep", "alignn_tconv_fwd", "alignn_tconv_bwd_dst",
                 "alignn_tconv_bwd_src", "alignn_gate_ln_fwd", "alignn_gate_ln_bwd", "alignn_hetero_nll"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from alignn_mi355x import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_declared()) == set(_lib.EXPORTED)
    assert lib.alignn_version() >= 1
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in _declared():
        assert re.search(rf"\bT {name}\b", out), name


def test_library_is_gfx950():
    from alignn_mi355x import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
