"""C-ABI boundary checks that need no GPU (the library is loaded, nothing is launched).

- every function include/rlmd_abi.h declares is exported by librlmd_amd.so;
- rlmd_amd/_abi.py binds a signature for every declared function (and only those);
- the structs the facade passes by pointer have the header's sizes;
- host-only entry points behave as documented (layout arithmetic, error strings).
"""
import ctypes as C
import os
import subprocess

import pytest

from rlmd_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_abi.LIB_PATH):
        pytest.skip("librlmd_amd.so not built (run __graft_entry__.build())")
    return _abi.load()


def test_every_header_symbol_is_exported(lib):
    names = _abi.header_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared in rlmd_abi.h but not exported: {missing}"


def test_dynamic_symbol_table_matches_header(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T rlmd_" in ln}
    declared = set(_abi.header_symbols())
    assert declared <= exported
    # nothing rlmd_* leaks out that the header does not declare (experiment builds excluded)
    assert exported - declared <= {"rlmd_debug_ts"}, exported - declared


def test_bindings_cover_header():
    assert set(_abi.SIGNATURES) == set(_abi.header_symbols())


def test_struct_sizes():
    # rlmd_env_cfg: 10 x i32 + u64; rlmd_train_cfg: i64 + 4 x i32
    assert C.sizeof(_abi.EnvCfg) == 48
    assert C.sizeof(_abi.TrainCfg) == 24
    # rlmd_agent_cfg: 13 x i32, 16 x f32, (pad) u64
    assert C.sizeof(_abi.AgentCfg) == 15 * 4 + 16 * 4 + 4 + 8  # 15 int32, 16 f32, pad, u64 seed


def test_layout_is_host_only_and_matches_torch_order(lib):
    cfg = _abi.AgentCfg()
    cfg.algo, cfg.state_dim, cfg.action_dim, cfg.h1, cfg.h2 = 0, 5, 1, 256, 256
    n, oa, o1, o2 = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    _abi.check(lib.rlmd_agent_layout(C.byref(cfg), C.byref(n), C.byref(oa), C.byref(o1), C.byref(o2)))
    actor = 5 * 256 + 256 + 256 * 256 + 256 + 2 * (256 + 1)   # fc1, fc2, pi, log_scale
    critic = 6 * 256 + 256 + 256 * 256 + 256 + 256 + 1        # fc1, fc2, q_value
    assert (oa.value, o1.value, o2.value, n.value) == (0, actor, actor + critic, actor + 2 * critic)


def test_errors_are_reported_not_raised(lib):
    rc = lib.rlmd_agent_layout(None, None, None, None, None)
    assert rc != 0
    assert b"null" in lib.rlmd_last_error()
