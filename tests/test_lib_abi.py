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
    assert lib.alignn_version() == 3  # ALIGNN_ABI_VERSION (include/alignn_hip.h)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in _declared():
        assert re.search(rf"\bT {name}\b", out), name


def test_library_is_gfx950():
    from alignn_mi355x import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_gemm_plan_workspace_query_on_host():
    """alignn_gemm_workspace runs the C-side plan without touching a GPU (no device: 256 CUs
    assumed, the MI355X count): 64x64 tiles, split-K toward one workgroup per CU for long K or a
    tiny grid, each split >= 32 deep (gemm.hip make_plan)."""
    import ctypes
    from alignn_mi355x import _lib
    lib = _lib.load()

    def ws(M, N, K, batch=1, split=0, reduce_batch=0, tile=0):
        a = _lib.GemmArgs()
        a.M, a.N, a.K, a.batch = M, N, K, batch
        a.sam, a.sak, a.sbk, a.sbn, a.scm, a.scn = K, 1, 1, K, N, 1
        a.split_k, a.reduce_batch, a.tile = split, reduce_batch, tile
        return lib.alignn_gemm_workspace(ctypes.byref(a))

    # dW of a line-graph projection: 4 tiles of 64x64, K = 23040 -> 63 chunks of 368
    assert ws(64, 256, 23040) == 63 * 64 * 256
    assert ws(256, 256, 256) == 8 * 256 * 256        # 16 tiles: split to 8 chunks of 32
    assert ws(512, 256, 256) == 0                    # short K on >= 32 tiles does not split
    assert ws(2580, 768, 256) == 0                   # enough tiles
    assert ws(1920, 256, 1024) == 2 * 1920 * 256     # 120 tiles, long K: 2 splits
    assert ws(256, 256, 4096, split=4) == 4 * 256 * 256
    assert ws(256, 256, 4096, split=1) == 0
    assert ws(64, 64, 4096, tile=4 | 64) == ws(64, 64, 4096, tile=4)   # bf16 flag leaves the plan alone
    assert ws(-1, 4, 4) == -1


def test_precision_flags_match_header():
    from alignn_mi355x import ops
    src = open(HEADER).read()
    assert re.search(rf"#define ALIGNN_GEMM_BF16 {ops.GEMM_BF16}\b", src)
    assert re.search(r"#define ALIGNN_GEMM_BK32 16\b", src)
    assert re.search(r"#define ALIGNN_GEMM_BK64 128\b", src)
