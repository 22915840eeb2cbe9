"""FeAR's block width (gw_set_fear_blocks, include/gridenv.h): an env without a full-obs writer
(``VecGridEnv(obs=False)``: the window rollouts) runs FeAR on 32-env blocks, every other env on
64-env blocks.  The width only changes the launch shape: FeAR, shaped rewards, returns, positions,
dones are bit-identical and the statistics totals equal up to the f64 sum's grouping to the 64-env blocks (``GW_FEAR_BE=wide`` forces
them), and the width cannot change after the first reset (it fixes the stats-row layout)."""
import pytest
import torch

from marlnav import _lib
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu

E, T = 4096, 24


def _run(wide: bool):
    mp = pytest.MonkeyPatch()
    mp.setenv("GW_KERNEL", "defer")  # the world update + fear_v2 path (merged runs FeAR inline)
    if wide:
        mp.setenv("GW_FEAR_BE", "wide")
    try:
        env = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=-5.0, max_steps=16, seed=5, obs=False,
                         stats=True, debug=True)
    finally:
        mp.undo()
    env.reset()
    acc = torch.zeros_like(env.out["stats"])
    rec = {n: [] for n in ("fear", "shaped", "ep_return", "final_pos", "done")}
    for _ in range(T):
        r = env.step(into={"stats_acc": acc})
        for n in rec:
            rec[n].append(getattr(r, n).clone())
    torch.cuda.synchronize()
    out = {n: torch.stack(v) for n, v in rec.items()}
    out["totals"] = acc.sum(0).cpu()
    out["rows"] = int(env.lib.gw_stats_rows(env.handle))
    with pytest.raises(_lib.GwError):  # after the first reset the width is fixed
        _lib.check(env.lib.gw_set_fear_blocks(env.handle, 1), "gw_set_fear_blocks")
    env.close()
    return out


def test_fear_block_width_is_result_neutral():
    narrow, wide = _run(False), _run(True)
    assert narrow["rows"] > wide["rows"]  # twice the FeAR blocks: their stats rows
    for n in ("fear", "shaped", "ep_return", "final_pos", "done"):
        assert torch.equal(narrow[n], wide[n]), n
    assert int(narrow["done"].sum()) > 0
    # the totals sum the blocks' rows: another grouping of the same f64 terms
    torch.testing.assert_close(narrow["totals"], wide["totals"], rtol=1e-12, atol=1e-9)
