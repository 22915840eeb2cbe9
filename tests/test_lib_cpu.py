"""CPU-side checks of the product library and host code (no GPU needed, no kernels run)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest
import torch

from marlnav import _lib
from marlnav import scenario as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "gridenv.h")
HEADERS = [HEADER, os.path.join(REPO, "include", "learner_ops.h"), os.path.join(REPO, "include", "actor_ops.h"),
           os.path.join(REPO, "include", "rollout_ops.h")]


def declared_functions():
    text = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:gw_status|const char|void|int64_t)\s*\*?\s*(gw_\w+)\s*\(", text, re.M)))


def test_library_builds_and_exports_every_declared_symbol():
    path = _lib.build()
    assert os.path.exists(path)
    lib = C.CDLL(path)
    names = declared_functions()
    assert set(names) == set(_lib.EXPORTS), (names, _lib.EXPORTS)
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", out), f"{n} not exported"


def test_library_targets_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


MEASURE_SWITCHES = ("GW_ACT_AB", "GW_CNN_AB", "GW_PATCH_PROBE", "GW_PATCH_PB", "GW_PATCH_MODE", "GW_WCNN_STAT",
                    "GW_RARE_STAMP", "GW_LEARN_STAMP")


def test_release_library_ignores_measurement_switches():
    """the kernels' work-skipping A/B and probe switches (GW_ACT_AB drops layer 2,
    GW_PATCH_PROBE stores zeros, ...) exist only in the -DGW_MEASURE build (csrc/measure.h).  The
    release library never reads them: their names are not even in the binary, so no stale export
    can change what the product computes.  The env knobs it does read are result-neutral
    scheduling choices or the tested precision variant."""
    assert not _lib.MEASURE
    blob = open(_lib.build(), "rb").read()
    for name in MEASURE_SWITCHES:
        assert name.encode() not in blob, f"{name} is read by the release library"
    # the sources read every one of them only through GW_MEASURE_ENV
    csrc = os.path.join(REPO, "marl-responsible-nav_amd", "csrc")
    for fn in os.listdir(csrc):
        if fn.endswith((".hip", ".h")):
            text = open(os.path.join(csrc, fn)).read()
            for name in MEASURE_SWITCHES:
                assert f'getenv("{name}")' not in text.replace("GW_MEASURE_ENV", ""), (fn, name)
    known = {"GW_KERNEL", "GW_MERGE_BYTES", "GW_FEAR_BE", "GW_OBS_CHUNKS", "GW_OBS_STREAMS", "GW_ACT_V",
             "GW_ACT_WAVES", "GW_WCNN_LIST"}
    for fn in os.listdir(csrc):
        if fn.endswith((".hip", ".h")):
            for name in re.findall(r'std::getenv\("(\w+)"\)', open(os.path.join(csrc, fn)).read()):
                assert name in known, (fn, name)


STRUCTS = {
    "gw_scenario": (_lib.GwScenario, ["H", "W", "region", "policy_id", "n_policies", "policy_cdf", "mdr", "apples"]),
    "gw_config": (_lib.GwConfig, ["N", "K", "num_envs", "env_offset", "fear", "fear_weight", "max_steps",
                                  "auto_reset", "seed"]),
    "gw_step_out": (_lib.GwStepOut, _lib.STEP_OUT_FIELDS),
    "gw_state": (_lib.GwState, _lib.STATE_FIELDS),
    "gw_obs_source": (_lib.GwObsSource, ["desc", "base", "apples", "N", "K", "H", "W", "variant", "E", "env_offset"]),
    "gw_mlp_actors": (_lib.GwMlpActors, ["K", "in_dim", "hidden", "n_actions", "layer_norm", *_lib.MLP_PARAM_FIELDS]),
}


def test_ctypes_layout_matches_header():
    """sizeof/offsetof of every ABI struct, compiled from include/gridenv.h with gcc."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gridenv.h"', '#include "actor_ops.h"',
             "int main(void){"]
    for s, (_, fields) in STRUCTS.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f in fields:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "l.c")
        open(src, "w").write("\n".join(lines))
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", f"-I{os.path.dirname(HEADER)}", src, "-o", exe], check=True)
        res = dict(l.rsplit(" ", 1) for l in subprocess.run([exe], capture_output=True, text=True).stdout.splitlines())
    for s, (cls, fields) in STRUCTS.items():
        assert int(res[s]) == C.sizeof(cls), s
        for f in fields:
            assert int(res[f"{s}.{f}"]) == getattr(cls, f).offset, f"{s}.{f}"


def test_no_cpu_fallback():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from marlnav.vec_env import VecGridEnv
    with pytest.raises(_lib.GwError):
        VecGridEnv("grid32", num_envs=4)


@pytest.mark.parametrize("name", sorted(S.BUILTIN))
def test_builtin_scenarios_compile(name):
    sc = S.builtin(name)
    H, W, N, K = S.BUILTIN[name]
    assert (sc.H, sc.W, sc.N, sc.K) == (H, W, N, K)
    assert sc.free_cells.size >= N
    assert np.allclose(sc.policy_p.sum(-1), 1.0)
    assert np.all(sc.policy_cdf[..., -1] == 1.0)
    for k in range(K):  # apples sit on roads
        assert sc.region[sc.apples[k]] == 1
    # okmask agrees with the region
    for c in range(sc.HW):
        r, q = divmod(c, sc.W)
        for d, (dr, dc) in enumerate(((-1, 0), (1, 0), (0, -1), (0, 1))):
            rr, cc = r + dr, q + dc
            ok = 0 <= rr < sc.H and 0 <= cc < sc.W and sc.region[rr * sc.W + cc] == 1
            assert bool(sc.okmask[c] >> d & 1) == ok


def test_scenario_rejects_bad_input():
    sc = S.level3_like(10, 16)
    with pytest.raises(ValueError):
        S.compile_scenario(sc, n_agents=9)
    bad = dict(sc)
    bad["Apples"] = {"apple_0": [50, 0], "apple_1": [0, 0]}
    with pytest.raises(ValueError):
        S.compile_scenario(bad)
