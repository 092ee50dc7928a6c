"""CPU checks of the C ABI boundary: libsgmm.so loads without a GPU and
exports exactly the functions include/sgmm.h declares; ctypes mirrors of the
ABI structs have the header's sizes/offsets."""
import ctypes
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "sgmm.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sgmm_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ("sgmm_rollout_fitness", "sgmm_rollout_trace", "sgmm_env_step_batch",
                 "sgmm_policy_forward", "sgmm_ga_ask", "sgmm_ga_tell", "sgmm_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(sgmm):
    from sgmm_amd import _lib
    L = _lib.load()
    lib_path = _lib.LIB_PATH
    nm = subprocess.run(["nm", "-D", "--defined-only", str(lib_path)], capture_output=True, text=True,
                        check=True).stdout
    exported = set(re.findall(r" T (sgmm_[a-z_0-9]+)", nm))
    declared = set(declared_functions())
    assert declared <= exported, declared - exported
    assert exported <= declared, exported - declared  # nothing undocumented
    assert set(_lib.SIGNATURES) == declared            # the binding covers the header
    assert L.sgmm_abi_version() == 5


def test_struct_layouts_match_header(sgmm):
    from sgmm_amd import _lib
    assert ctypes.sizeof(_lib.EnvParams) == 48
    assert ctypes.sizeof(_lib.GAState) == 80 and _lib.GAState.decay.offset == 72
    assert ctypes.sizeof(_lib.GAHistory) == 40
    assert _lib.Episodes.genome.offset == 24 and ctypes.sizeof(_lib.Episodes) == 80
    assert ctypes.sizeof(_lib.Ticks) == 56
    assert ctypes.sizeof(_lib.AskedPopulation) == 40 and _lib.AskedPopulation.i0.offset == 32
    assert _lib.GAState.arrivals.offset == 68
    assert ctypes.sizeof(_lib.DayStreams) == 104 and _lib.DayStreams.snap_off.offset == 16
    assert ctypes.sizeof(_lib.EventBars) == 88 and _lib.EventBars.vwap_num.offset == 80
    # ABI 5: the writable walk order is its own member (train_eps->order stays read-only)
    assert ctypes.sizeof(_lib.Populations) == 72 and _lib.Populations.walk_order.offset == 64
    text = HEADER.read_text()
    assert "const int32_t *order;" in text and "int32_t *walk_order;" in text


def test_argument_errors_need_no_gpu(sgmm):
    """Validation happens before any HIP call: bad arguments fail cleanly on CPU."""
    from sgmm_amd import _lib
    L = _lib.load()
    rc = L.sgmm_policy_forward(None, 0, 16, None, None, None, 10, None)
    assert rc == -1 and b"null" in L.sgmm_last_error()
    rc = L.sgmm_policy_forward(ctypes.c_void_p(8), 370, 12, None, ctypes.c_void_p(8), ctypes.c_void_p(8), 1, None)
    assert rc == -1 and b"hidden" in L.sgmm_last_error()
    # H = 64 genomes (4546 floats) overflow the GA step's LDS master stage: rejected
    # before launch by every multi-population GA entry point
    v = ctypes.c_void_p(8)
    pops = _lib.Populations(1, 8, 64, 0, 8, 8, None, None, 8, None, None)
    for rc in (L.sgmm_ga_step_multi(ctypes.byref(pops), v, v, v, v, 0, 0, 0, 0, None),
               L.sgmm_ga_tell_multi(ctypes.byref(pops), v, v, 0, 0, 0, 0, None)):
        assert rc == -1 and b"genome too large" in L.sgmm_last_error()
    # no adversary: u64 chunk maps + chunk trade counts + frontier merge info + f64 path planes,
    # 256-aligned sections sized for both the table (1000/64 + 4 + 1 chunk slots) and the
    # frontier kernel (64 G chunk records per episode -- G = 8 groups of 64 chunks at 4
    # episodes, the default rule's cap: u64 map, u32[8] counts, u32 merge info) (planes:
    # 1000 ticks + 4 x (256 G + 16) padding rows of the frontier layout -- 128-byte aligned
    # episode blocks -- rounded to 32: 9280); u32 slots per frontier wave (64 per episode);
    # u32 spill entries per frontier wave (64 per episode: <= 16 groups x 4 waves); the
    # fused scan's u32 arrival words and 16-byte chain hand-offs (one each per episode,
    # 256-aligned)
    assert L.sgmm_rollout_workspace_size(4, 1000, 5) == (4 * 512 * 8 + 4 * 512 * 32 + 4 * 512 * 4
                                                         + 4 * 64 * 4 + 4 * 64 * 4 + 256 + 256 + 5 * 9280 * 8)
    # bundle builder: group starts (i32) + times (i64), 256-aligned, + 7 f64 stats per tick
    assert L.sgmm_event_bars_workspace_size(1000) == 4096 + 8192 + 56000
    rc = L.sgmm_event_bars_build(None, None, None, 0, None)
    assert rc == -1 and b"null" in L.sgmm_last_error()
    ev = _lib.EventBars()
    rc = L.sgmm_bar_windows(ctypes.byref(ev), 1, ctypes.c_void_p(8), ctypes.c_void_p(8), ctypes.c_void_p(8),
                            ctypes.c_void_p(8), ctypes.c_void_p(8), 5000, None)
    assert rc == -1 and b"bars per day" in L.sgmm_last_error()
    # adversary (20 states): u64 fill words + per-state f64 reward planes (stride
    # 1000 rounded to 32: table rows only, no frontier padding); the scan derives
    # the chunk transducers itself
    assert L.sgmm_rollout_workspace_size(4, 1000, 20) == 8192 + 20 * 1024 * 8
    # ABI 4: the adversary flag is explicit, so 1 or 2 inventory values (4 or 8
    # states) get the adversary layout, not the no-adversary one of the same state count
    assert L.sgmm_rollout_workspace_bytes(4, 1000, 5, 1) == L.sgmm_rollout_workspace_size(4, 1000, 20)
    assert L.sgmm_rollout_workspace_bytes(4, 1000, 5, 0) == L.sgmm_rollout_workspace_size(4, 1000, 5)
    for nsi in (1, 2):
        assert L.sgmm_rollout_workspace_bytes(4, 1000, nsi, 1) == 8192 + 4 * nsi * 1024 * 8
    # the worked example: one 5000-tick ARL episode with 2 inventory values (8
    # states) has the adversary layout, not the 8-inventory no-adversary one
    assert L.sgmm_rollout_workspace_bytes(1, 5000, 2, 1) == 40192 + 8 * 5024 * 8
    assert L.sgmm_rollout_workspace_bytes(1, 5000, 2, 1) != L.sgmm_rollout_workspace_size(1, 5000, 8)
    assert L.sgmm_rollout_workspace_bytes(4, 1000, 9, 0) == 0  # more than 8 inventory values


def test_gpu_entry_points_fail_loudly_without_gpu(sgmm):
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        sgmm.RolloutEngine("cuda")


PLAN_ENV = {"SGMM_TABLE_PATH": "frontier", "SGMM_FRONTIER_NW": "3", "SGMM_FRONTIER_LS": "2",
            "SGMM_FRONTIER_TAIL": "0", "SGMM_FRONTIER_FOUR": "0", "SGMM_FRONTIER_MIN_EPS": "4",
            "SGMM_TABLE_SP": "1", "SGMM_SCAN_THREADS": "256", "SGMM_REORDER_WEIGHTS": "5,5",
            "SGMM_FRONTIER_SPILL": "0", "SGMM_FRONTIER_REORDER": "0", "SGMM_SEQ_SUM": "1",
            "SGMM_FUSED_SCAN": "0", "SGMM_LANES_SCAN": "0"}


def test_shipped_library_reads_no_plan_environment(sgmm):
    """The shipped libsgmm.so takes its launch plan from the measured rules and
    the explicit sgmm_plan_set overrides only: with every experiment variable of
    the A/B builds set, each knob still reads -1 (the default rule) and the
    workspace size is the default plan's; the variable names are not even in
    the binary (they are compiled only into -DSGMM_EXPERIMENTS variants)."""
    import os
    import sys
    from sgmm_amd import _lib
    blob = _lib.LIB_PATH.read_bytes()
    for name in PLAN_ENV:
        assert name.encode() not in blob, name
    assert b"getenv" not in blob
    code = ("import sgmm_pkg; sgmm_pkg.load(); from sgmm_amd import _lib; L = _lib.load(); "
            "print([L.sgmm_plan_get(k) for k in range(13)], L.sgmm_rollout_workspace_bytes(2560, 2560 * 4560, 5, 0), "
            "L.sgmm_plan_get(13))")
    env = dict(os.environ)
    clean = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                           check=True).stdout.split("\n")[-2]
    env.update(PLAN_ENV)
    dirty = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                           check=True).stdout.split("\n")[-2]
    assert dirty == clean
    assert clean.startswith("[" + ", ".join(["-1"] * 13) + "]")
    assert clean.endswith(str(-2**31))  # unknown knob


def test_plan_overrides_round_trip(sgmm):
    """sgmm_plan_set / sgmm_plan_get (no GPU needed): a knob reads back what was
    set, a negative value restores the default rule, unknown knobs are
    rejected; the workspace size follows a groups override (records and plane
    padding are laid out for the launch's chunk groups)."""
    from sgmm_amd import _lib
    L = _lib.load()
    base = L.sgmm_rollout_workspace_bytes(4, 1000, 5, 0)
    with _lib.plan(groups=16, policy_path="valu"):
        assert L.sgmm_plan_get(_lib.PLAN_KNOBS["groups"]) == 16
        assert L.sgmm_plan_get(_lib.PLAN_KNOBS["policy_path"]) == 3
        assert L.sgmm_rollout_workspace_bytes(4, 1000, 5, 0) > base
    assert L.sgmm_plan_get(_lib.PLAN_KNOBS["groups"]) == -1
    assert L.sgmm_rollout_workspace_bytes(4, 1000, 5, 0) == base
    assert L.sgmm_plan_set(99, 1) == -1 and b"unknown plan knob" in L.sgmm_last_error()
