"""CPU checks of the drop-in boundary: libmapf.so loads, exports every symbol
include/mapf.h declares, and the ctypes structs match the C layout."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mapf.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mapf_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from mapf_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    assert L.mapf_abi_version() == 1


def test_struct_layout_matches_c(tmp_path):
    from mapf_amd import _lib
    from mapf_amd.config import MapfConfig
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mapf.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(mapf_config),'
                   ' offsetof(mapf_config, seed), offsetof(mapf_config, goal_reward), sizeof(mapf_reset_spec),'
                   ' offsetof(mapf_reset_spec, seed), sizeof(mapf_step_out), sizeof(mapf_state), sizeof(mapf_mapgen_spec),'
                   ' offsetof(mapf_mapgen_spec, density), offsetof(mapf_mapgen_spec, seed));'
                   ' printf("%zu %zu\\n", sizeof(mapf_tuning), offsetof(mapf_tuning, diag_exp)); return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(MapfConfig), MapfConfig.seed.offset, MapfConfig.goal_reward.offset,
            ctypes.sizeof(_lib.ResetSpec), _lib.ResetSpec.seed.offset, ctypes.sizeof(_lib.StepOut),
            ctypes.sizeof(_lib.State), ctypes.sizeof(_lib.MapGenSpec), _lib.MapGenSpec.density.offset,
            _lib.MapGenSpec.seed.offset, ctypes.sizeof(_lib.Tuning), _lib.Tuning.diag_exp.offset]
    assert got == want


def test_oracle_config_layout_matches_product():
    from mapf_amd.config import MapfConfig
    from oracle.oracle import OracleConfig
    assert [f[0] for f in OracleConfig._fields_] == [f[0] for f in MapfConfig._fields_]
    assert ctypes.sizeof(OracleConfig) == ctypes.sizeof(MapfConfig)


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mapf_amd.env import BatchedMapfGym
    with pytest.raises(RuntimeError):
        BatchedMapfGym(num_envs=1, height=10, width=10)


def test_invalid_config_rejected_without_touching_gpu():
    """mapf_create validates before any device call."""
    from mapf_amd import _lib
    from mapf_amd.config import make_config
    cfg = make_config(1, 10, 10, num_agents=65)
    h = ctypes.c_void_p()
    rc = _lib.lib().mapf_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc == -1 and b"num_agents" in _lib.lib().mapf_last_error()


def test_tuning_defaults_and_validation_without_gpu():
    """mapf_tuning_default fills the documented (measured) forms; mapf_set_tuning rejects a
    null handle before any device call."""
    from mapf_amd import _lib
    t = _lib.Tuning()
    _lib.lib().mapf_tuning_default(ctypes.byref(t))
    got = {n: getattr(t, n) for n in _lib.TUNING_FIELDS}
    assert got == dict(roll_occ=0, roll_group=-1, roll_fair=-1, roll_slack=1, wide_nt=-1, wide_pipe=1, wide_grid=1,
                       wide_overlap=1, wide_obs=2, wide_epw=0, wide_pair=0, wide_slack=1, wide_fair=0, wide_prio=1,
                       wide_bfsobs=1, xcd_remap=1, obs_envs=0, step_block=256, search_blocks=64, band_blocks=0,
                       agent_lanes=0, serial_search=0, no_defer=0, diag_exp=0)
    assert _lib.lib().mapf_set_tuning(None, ctypes.byref(t)) == -1


def test_no_process_environment_in_the_library():
    """Kernel forms come from the handle's mapf_tuning only: no source of libmapf.so reads the
    process environment (a user's stray variable must not change which kernel runs)."""
    csrc = os.path.join(ROOT, "primal-ppo_amd", "csrc")
    hits = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h", ".cpp")):
            for k, line in enumerate(open(os.path.join(csrc, f)), 1):
                if re.search(r"\b(getenv|secure_getenv|environ)\b", line):
                    hits.append(f"{f}:{k}")
    assert not hits, hits
