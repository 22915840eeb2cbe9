"""The descriptor replay ring (``ReplayRing(desc=True)``, ``gw_obs_desc_copy`` +
``gw_replay_gather_desc``, include/rollout_ops.h): the learner's sampled rows expanded from the
48-byte obs descriptors of each ring slot must be bit for bit the rows of the dense obs /
final-obs slots the obs writer filled (MultiAgentReplayBuffer.sample of the reference's
memory, maddpg/agent.py:199-224; obs encodings ma_customenv.py:197-209 reset, :303-322 step).

Covered: step and reset encodings, terminal obs of done envs (auto-reset, a short episode cap),
a wrapped ring, both obs-writer pipelines (eager on the merged path, lazy on the split path),
the unjoined FeAR, the single-agent variant, and a whole training run (the learner on
descriptor rows == the learner on dense rows, every weight bit for bit)."""
import pytest
import torch

from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _compare(ro, batch=4096, seed=0):
    rp = ro.replay
    ro.fence()  # the dense slots are complete
    assert rp.use_desc
    outs = []
    for use_desc in (True, False):
        g = torch.Generator(device="cuda").manual_seed(seed)
        outs.append(rp._sample_hip(batch, g, True, critic_in=True, use_desc=use_desc))
    torch.cuda.synchronize()
    a, b = outs
    for x, y in zip(a[:5], b[:5]):
        assert torch.equal(x, y)
    assert torch.equal(a[5][0], b[5][0]) and torch.equal(a[5][1], b[5][1])  # (tr, env)
    kh = rp.K * rp.obs.shape[-2] * rp.obs.shape[-1]  # x_next's action slots are left to the learner
    assert torch.equal(a[6][0], b[6][0]) and torch.equal(a[6][1][:, :kh], b[6][1][:, :kh])  # critic rows
    tr, env = a[5]
    done = rp.done[tr, env].bool()
    return int(done.sum())


@pytest.mark.parametrize("scen,E,fear,obs_async,fear_async,cap", [
    ("grid32", 1024, True, "lazy", False, 9),
    ("grid32", 1024, True, True, True, 7),
    ("grid32", 4096, False, True, False, 11),
    ("level3", 333, True, False, False, 5),
    ("level3_single", 500, False, "lazy", False, 6),
])
def test_desc_rows_equal_dense_rows(scen, E, fear, obs_async, fear_async, cap):
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    sc = S.builtin(scen)
    variant = "single" if scen.endswith("single") else None
    kw = dict(variant=variant) if variant else {}
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=3, max_steps=cap, auto_reset=True,
                     stats=True, **kw)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=1)
    ro = Rollout(env, actors, replay_slots=8, training=True, seed=4, obs_async=obs_async,
                 fear_async=fear_async, desc_ring=True)
    assert ro.fused and ro.replay.desc is not None
    ro.reset()
    dones = 0
    for t in range(1, 30):
        ro.step()
        if t in (1, 2, 7, 8, 9, 17, 29):  # before / at / after the ring wraps
            dones += _compare(ro, seed=t)
    assert dones > 0  # terminal rows were sampled
    env.close()


def test_resume_falls_back_to_dense_rows():
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=512, fear=False, seed=5, max_steps=8, auto_reset=True)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=2)
    ro = Rollout(env, actors, replay_slots=6, training=True, seed=1, obs_async=True, desc_ring=True)
    ro.reset()
    for _ in range(5):
        ro.step()
    assert ro.replay.use_desc
    ro.resume()
    assert not ro.replay.use_desc  # the carried-over terminal obs has no descriptor
    ro.step()
    ro.reset()
    assert ro.replay.use_desc
    env.close()


def test_training_on_desc_rows_equals_dense_rows(monkeypatch):
    """Two trainers from the same seeds, one sampling the descriptor ring (the default with the
    fused actor), one the dense slots, both with the dense-row learner (GW_DESC_LEARN=0; the
    descriptor learner has its own tests, tests/test_gpu_desc_learner.py): after 24 env steps with
    updates every weight is equal."""
    monkeypatch.setenv("GW_DESC_LEARN", "0")
    from marlnav.maddpg import MADDPG
    from marlnav.train import MADDPGTrainer
    sc = S.builtin("grid32")
    states = []
    for desc in (True, False):
        torch.manual_seed(5)  # the captured update draws from the default generators
        env = VecGridEnv(sc, num_envs=256, fear=True, fear_weight=-5.0, stats=True, seed=7, max_steps=10)
        m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
        tr = MADDPGTrainer(env, m, memory_size=2048, updates_per_step=1, graph=True, seed=3)
        if not desc:
            tr.rollout.replay.desc = None
        tr.reset()
        assert tr.rollout.replay.use_desc == desc
        tr.train(24)
        torch.cuda.synchronize()
        assert tr.updates > 10
        states.append({k: v.clone() for k, v in m.state_dict().items()})
        env.close()
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k


@pytest.mark.parametrize("desc_learner", ["1", "0"])
def test_update_as_recorded_launches_equals_graph_replay(monkeypatch, desc_learner):
    """MADDPG.capture(launches=True): the captured update re-issued as its recorded C-ABI
    launches (_lib.LaunchRecorder) == the HIP graph replay, every weight bit for bit (same
    seeds, in-kernel draws), and the replayed launches really ran (the weights moved); with the
    descriptor learner (one gw_maddpg_desc_update_img call, which also leaves the fused actor's
    workspace: no gw_actor_prepare) and with the dense-row update."""
    monkeypatch.setenv("GW_DESC_LEARN", desc_learner)
    first = "gw_maddpg_desc_update_img" if desc_learner == "1" else "gw_replay_gather_desc"
    from marlnav.maddpg import MADDPG
    from marlnav.train import MADDPGTrainer
    sc = S.builtin("grid32")
    states = []
    for mode in ("launches", True):
        env = VecGridEnv(sc, num_envs=256, fear=True, fear_weight=-5.0, stats=True, seed=7, max_steps=10)
        m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
        tr = MADDPGTrainer(env, m, memory_size=2048, updates_per_step=1, graph=mode, seed=3)
        tr.reset()
        tr.train(6)
        assert m._graph is not None and (m._launches is not None) == (mode == "launches")
        if mode == "launches":
            names = [c[0] for c in m._launches.calls]
            assert names[0] == first and ("gw_actor_prepare" in names) == (desc_learner == "0"), names
        before = m.actors.net.flat_params().clone()
        tr.train(18)
        torch.cuda.synchronize()
        assert not torch.equal(before, m.actors.net.flat_params())
        states.append({k: v.clone() for k, v in m.state_dict().items()})
        env.close()
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k


def test_capture_follows_the_rings_row_mode():
    """a capture made while the ring served dense rows (after resume) must not be
    replayed once a reset switched the ring back to descriptor rows (its fence would then skip the
    obs writer the captured dense gather reads): the trainer re-captures on the new mode."""
    from marlnav.maddpg import MADDPG
    from marlnav.train import MADDPGTrainer
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=256, fear=True, fear_weight=-5.0, stats=True, seed=7, max_steps=10)
    m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
    tr = MADDPGTrainer(env, m, memory_size=2048, updates_per_step=1, graph="launches", seed=3)
    tr.reset()
    tr.train(4)
    tr.rollout.resume()
    assert not tr.rollout.replay.use_desc
    tr.train(3)
    assert m._graph is not None and m._capture_desc is False
    names = [c[0] for c in m._launches.calls]
    assert names[0] == "gw_replay_gather", names
    tr.reset()
    assert tr.rollout.replay.use_desc and not m.capture_matches(tr.rollout.replay)
    tr.train(3)
    assert m._capture_desc is True and m.capture_matches(tr.rollout.replay)
    assert [c[0] for c in m._launches.calls][0] == "gw_maddpg_desc_update_img"
    env.close()


def test_launch_recorder_refuses_torch_kernels():
    """A torch op that launches a GPU kernel inside a recording would be missing from every
    replay: LaunchRecorder raises instead (views and allocations pass)."""
    from marlnav import _lib
    x = torch.zeros(8, device="cuda")
    rec = _lib.LaunchRecorder(torch.cuda.current_stream().cuda_stream)
    with rec:
        x.view(2, 4)[1]
        torch.empty(16, device="cuda")
    with pytest.raises(_lib.RecordingError):
        with _lib.LaunchRecorder(torch.cuda.current_stream().cuda_stream):
            x.add_(1)
