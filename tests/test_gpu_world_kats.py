"""The HIP world update (UpdateGWorld + collision resolution, custom/grid_world.py:233-563) on the
reference's own known-answer cases (tests/golden/transition.npz, recorded from the reference by
tests/golden/make_golden.py): every case of a group is one env of a batch, spawned at the case's
cells (replay mode) and stepped once with the case's joint action through the C ABI.  Crash and
restricted bits and the final cells must equal the reference's, on the FeAR-off step (N <= 4: the
unrolled pair rules; N > 4: the per-lane pair lists) and on the FeAR-on step (the env's own sim in
step_v2's task phase).  Apples do not move agents, so the env's fixed apples stand in for the
cases' ones (the oracle KATs in test_oracle_golden.py check the apple scan)."""
import dataclasses
import os

import numpy as np
import pytest
import torch

from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _groups():
    z = np.load(os.path.join(GOLD, "transition.npz"))
    return sorted({k.split("/")[0] for k in z.files if "/" in k})


def _scenario(region2d: np.ndarray, N: int) -> S.CompiledScenario:
    """A scenario on the case's map: one (unused) scripted policy, MdR stay, K = 1."""
    base = S.builtin("level3")
    H, W = region2d.shape
    return dataclasses.replace(
        base, name="kat", H=H, W=W, N=N, K=1, region=(region2d != 0).astype(np.uint8).reshape(-1),
        policy_id=np.zeros(H * W, np.uint8), policy_keys=base.policy_keys[:1], policy_p=base.policy_p[:1],
        policy_cdf=base.policy_cdf[:1], mdr=np.zeros(H * W, np.uint8), apples=np.zeros(1, np.int32),
        free_cells=np.flatnonzero(region2d.reshape(-1) == 1).astype(np.int32),
        okmask=S.okmask_table(region2d), action_mask=S.action_mask_table(region2d))


@pytest.mark.parametrize("fear", [False, True])
@pytest.mark.parametrize("group", _groups())
def test_world_update_matches_reference_kats(group, fear):
    z = np.load(os.path.join(GOLD, "transition.npz"))
    g = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(group + "/")}
    region = np.asarray(g["region"])
    loc = np.asarray(g["loc"], np.int64)                    # [n, N] (row, col) or cells
    act = np.asarray(g["act"], np.int32)                    # [n, N]
    n, N = act.shape
    H, W = region.shape
    cells = loc if loc.ndim == 2 else loc[..., 0] * W + loc[..., 1]
    fin_ref = np.asarray(g["final"], np.int64)
    fin_ref = fin_ref if fin_ref.ndim == 2 else fin_ref[..., 0] * W + fin_ref[..., 1]
    env = VecGridEnv(_scenario(region, N), num_envs=n, fear=fear, fear_weight=-5.0, max_steps=1000,
                     debug=True)
    env.reset(spawn=torch.as_tensor(cells.astype(np.int32)))
    r = env.step(act[:, :1].copy(), act[:, 1:].copy() if N > 1 else None)
    torch.cuda.synchronize()
    bits = lambda b: ((b.cpu().numpy().astype(np.int64)[:, None] >> np.arange(N)) & 1).astype(bool)
    np.testing.assert_array_equal(bits(r.crash_bits), np.asarray(g["crash"]).astype(bool), err_msg=f"{group} crash")
    np.testing.assert_array_equal(bits(r.restr_bits), np.asarray(g["restricted"]).astype(bool),
                                  err_msg=f"{group} restricted")
    np.testing.assert_array_equal(r.final_pos.cpu().numpy(), fin_ref, err_msg=f"{group} final cells")
    assert N == 1 or bits(r.crash_bits).any()  # the group exercises the collision rules
    env.close()
