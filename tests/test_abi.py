"""CPU-side checks of the C-ABI library: it loads and exports every symbol include/esgpt_amd.h declares."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "esgpt_amd.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(esgpt_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    fns = declared_functions()
    for must in ("esgpt_embed_joint_fwd", "esgpt_embed_bag_bwd", "esgpt_attn_fwd", "esgpt_attn_bwd",
                 "esgpt_output_loss", "esgpt_embed_split_bags_fwd", "esgpt_embed_epilogue_fwd"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    from eventstreamgpt_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # the binding's table covers every declared function
    assert set(declared_functions()) <= set(_lib.SIGNATURES), set(declared_functions()) - set(_lib.SIGNATURES)
    lib.esgpt_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.esgpt_version()


def test_workspace_queries_without_gpu():
    from eventstreamgpt_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load(require_device=False)
    # MFMA backward: f32 dQ accumulator beyond one 256-key block + the dK/dV exchange slabs of the query-split pairs
    assert lib.esgpt_attn_bwd_workspace(2, 4, 256, 256, 64) == 4 * (2 * 4 * 1) * 2 * 256 * 64
    # two key blocks: one f32 dQ partial per key block + the dK / dV exchange slabs
    assert lib.esgpt_attn_bwd_workspace(2, 4, 512, 512, 64) == 2 * 4 * 2 * 4 * 512 * 64 + 4 * (2 * 4 * 2) * 2 * 256 * 64
    # hd 16 past one key block and hd 128 take the split dK/dV + dQ kernels: no MFMA workspace (the generic kernels'
    # delta buffer, B*H*Lq floats, remains the floor)
    assert lib.esgpt_attn_bwd_workspace(2, 4, 512, 512, 16) == 4 * 2 * 4 * 512
    assert lib.esgpt_attn_bwd_counters(2, 4, 512) == 2 * 2 * 4 * 2
    b = _lib.EsgptBatch()
    b.B, b.L, b.M, b.S = 32, 256, 16, 2
    assert lib.esgpt_embed_bag_bwd_workspace(ctypes.byref(b), 1, 1210, 256) > 32 * 256 * 16 * 16
    assert lib.esgpt_output_loss_workspace(32, 256, 5) > 0
    # GEMM split-K plans: forward products never split; weight gradients split the token dimension
    assert lib.esgpt_gemm_counters(8192, 1624) == 128 * 26
    assert lib.esgpt_linear_bwd_workspace(8192, 256, 256, 1) == 4 * (8 * 256 * 256 + 8 * 256)
    assert lib.esgpt_linear_bwd_workspace(64, 256, 256, 1) == 0


def test_product_path_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from eventstreamgpt_amd.kernels import BatchView
    from eventstreamgpt_amd.synthetic import CONFIGS
    from eventstreamgpt_amd._lib import HipExtensionMissing

    with pytest.raises(HipExtensionMissing):
        BatchView(CONFIGS["C1"].batch(0, batch_size=2))


def test_product_libraries_carry_no_tuning_hooks():
    """Kernel selection and numerics depend on the call's arguments alone: the in-tree product libraries contain none
    of the tools build's environment switches (make TUNING=1 builds them into eventstreamgpt_amd/tuning/)."""
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "eventstreamgpt_amd")
    names = [b"ESGPT_GEMM_", b"ESGPT_ATTN_BWD_NSPLIT", b"ESGPT_LN_FWD_ROWS", b"ESGPT_LN_BWD_ROWS",
             b"ESGPT_LOSS_ROW_STAGE", b"ESGPT_ATTN_GENERIC"]
    checked = 0
    for lib in ("libesgpt_amd.so", "libesgpt_torch.so"):
        path = os.path.join(here, lib)
        if not os.path.exists(path):
            continue
        data = open(path, "rb").read()
        for n in names:
            assert n not in data, (lib, n)
        checked += 1
    if not checked:
        pytest.skip("libraries not built")
