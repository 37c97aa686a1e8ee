"""C-ABI library: loads on a machine without a GPU and exports every entry point include/pcnerf_hip.h declares."""
import os
import re

import pytest

from conftest import REPO


def declared_functions():
    txt = open(os.path.join(REPO, "include", "pcnerf_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pcnerf_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_header_symbols():
    from nof import _hip
    L = _hip.lib()
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_hip.exported_symbols()), set(names) ^ set(_hip.exported_symbols())
    assert L.pcnerf_abi_version() == 1


def test_size_queries_without_gpu():
    from nof import _hip
    L = _hip.lib()
    # the fp32 image, 16 floats of split-image scales, the split image (120 k-steps x 8 x 2 x 64 f16x8)
    assert L.pcnerf_nof_eval_packed_floats() == 2 * 16384 + 7 * 65536 + 8 * 256 + 256 + 4 + 16 + 120 * 8 * 2 * 64 * 4
    # two chunk-sized activation buffers dominate the train workspace
    assert L.pcnerf_nof_train_workspace_bytes(262144) >= 2 * 262144 * 256 * 4
    assert L.pcnerf_child_loss_workspace_bytes(15333) == 15333 * 3 * 8


def test_argument_errors_are_reported_before_launch():
    from nof import _hip
    L = _hip.lib()
    rc = L.pcnerf_composite(None, None, 0, 0, None, 0.0, 0.0, None, 0, 0, 0, 0, None, None, None, None, None, None,
                            None)
    assert rc != 0
    assert b"null" in L.pcnerf_last_error()


def test_render_refuses_cpu_tensors():
    import pytest
    import torch
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_val
    with pytest.raises(RuntimeError, match="no CPU path"):
        with torch.no_grad():
            render_rays_val(NOF_coarse(), NOF_fine(), Embedding(3, 10), torch.zeros(4, 15))


def test_state_dict_keys_match_reference_layout():
    from nof import synthetic as syn
    from nof.networks import NOF_coarse
    keys = set(NOF_coarse().state_dict())
    assert keys == set(syn.init_nof_params(0))


def test_math_switches_without_gpu():
    """pcnerf_set_train_math / pcnerf_set_eval_math: process-wide selectors, previous mode returned, invalid modes
    refused with a message (no GPU call involved)."""
    from nof import _ops, _hip
    assert _ops.get_train_math() == "f16x2_3_fused" and _ops.get_eval_math() == "f16x2_3"
    assert _ops.set_train_math("f16x2_3") == "f16x2_3_fused"
    assert _ops.set_train_math("fp32") == "f16x2_3"
    assert _ops.set_train_math("f16x2_3_fused") == "fp32"
    assert _ops.get_train_math() == "f16x2_3_fused"
    assert _ops.set_eval_math("fp32") == "f16x2_3"
    assert _ops.set_eval_math("f16x2_3") == "fp32"
    assert _hip.lib().pcnerf_set_eval_math(7) == -1
    assert b"eval_math" in _hip.lib().pcnerf_last_error()
    with pytest.raises(ValueError):
        _ops.set_eval_math("bf16")
    assert _ops.get_eval_math() == "f16x2_3"


def test_activation_store_skips_chunks_beyond_32bit_layer_offsets(monkeypatch):
    """the fused query addresses a stored layer with a 32-bit byte offset, so under the default
    train math a chunk whose layer region reaches 4 GiB (>= 4,194,304 samples) is not stored -- the store holds no
    chunk and every chunk is recomputed -- instead of the forward failing, however large the budget."""
    import torch
    from nof import _ops
    gib = 1 << 30
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (280 * gib, 288 * gib))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda dev=None: 0)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda dev=None: 0)
    monkeypatch.delenv("PCNERF_ACT_STORE", raising=False)
    prev = _ops.set_activation_store_budget(1 << 62)
    prev_math = _ops.set_train_math("f16x2_3_fused")
    try:
        big = 1 << 22
        st = _ops.ActivationStore("cuda:0", 2 * big, big, 0)
        assert st.n_chunks == 0 and st.buf is None
    finally:
        _ops.set_activation_store_budget(prev)
        _ops.set_train_math(prev_math)


def test_activation_store_default_is_bounded(monkeypatch):
    """The drop-in's default activation-store budget is DEFAULT_STORE_CAP (32 GiB) however much HBM is free, at most
    half of what is free, and callers opt into more (set_activation_store_budget / PCNERF_ACT_STORE_GB)."""
    import torch
    from nof import _ops
    gib = 1 << 30
    free = {"v": 280 * gib}
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (free["v"], 288 * gib))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda dev=None: 0)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda dev=None: 0)
    monkeypatch.delenv("PCNERF_ACT_STORE", raising=False)
    monkeypatch.delenv("PCNERF_ACT_STORE_GB", raising=False)
    prev = _ops.set_activation_store_budget(None)
    try:
        assert _ops.DEFAULT_STORE_CAP == 32 * gib
        assert _ops.store_budget("cuda:0", 4 * gib) == 32 * gib
        free["v"] = 40 * gib   # little free: half of what is left after the reserve
        assert _ops.store_budget("cuda:0", 4 * gib) == 18 * gib
        free["v"] = 280 * gib
        monkeypatch.setenv("PCNERF_ACT_STORE_GB", "100")
        assert _ops.store_budget("cuda:0", 4 * gib) == 100 * gib
        _ops.set_activation_store_budget(1 << 62)   # bench.py's opt-in: everything but the reserve
        assert _ops.store_budget("cuda:0", 4 * gib) == 276 * gib
        monkeypatch.setenv("PCNERF_ACT_STORE", "0")
        assert _ops.store_budget("cuda:0", 4 * gib) == 0
    finally:
        _ops.set_activation_store_budget(prev)
