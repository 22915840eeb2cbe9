"""The no-code checkpoint reader (marlnav/checkpoint.py) and the shipped trained actors.

The reference evaluates agents it loads from agilerl checkpoints (customeval.py:39-64,
maddpg/agent.py:279-281).  Those pickles need dill / numpy globals, so they are read by replaying
their pickle opcodes (pickletools) into inert records -- nothing in the file is imported or run.

CPU tests:
* the reader against torch's own writer: tensors (incl. an offset / strided view) that
  ``torch.save`` wrote come back bit for bit, nested in dicts / lists / OrderedDicts;
* a pickle that would call ``os.system`` when unpickled yields an inert record and runs nothing;
* the reference's shipped checkpoints (when /root/reference is present, i.e. here) read to the
  committed fixture tests/golden/ckpt_actors.npz bit for bit (tests/golden/make_golden_checkpoint.py);
* the loaded MLP actor (marlnav MultiAgentActors) == an independent float64 restatement of
  agilerl's EvolvableMLP forward (Linear - LayerNorm(eps 1e-5) - ReLU x2 - Linear) on the obs of the
  reference's single-agent trajectories (tests/golden/single_traj.npz), within f32 rounding.
"""
import collections
import io
import os
import zipfile

import numpy as np
import pytest
import torch

from marlnav import checkpoint as ck

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_MODELS = "/root/reference/models/custom/single/level3"


def test_reader_matches_torch_save(tmp_path):
    g = torch.Generator().manual_seed(0)
    big = torch.randn(6, 10, generator=g)
    sd = collections.OrderedDict([("a.weight", torch.randn(4, 3, generator=g)), ("a.bias", torch.arange(5.0)),
                                  ("view", big[2:5, 1:8:2]), ("d", torch.randn(3, generator=g, dtype=torch.float64)),
                                  ("i", torch.arange(7, dtype=torch.int64))])
    obj = {"actors_state_dict": [sd], "steps": [12345], "name": "MADDPG", "nested": {"x": [big.t()]}}
    path = str(tmp_path / "ck.pt")
    torch.save(obj, path)
    r = ck.read_checkpoint(path)
    assert r["steps"] == [12345] and r["name"] == "MADDPG"
    got = ck.state_dict_tensors(r["actors_state_dict"][0])
    assert list(got) == list(sd)
    for k, v in sd.items():
        assert got[k].dtype == v.numpy().dtype and np.array_equal(got[k], v.numpy()), k
    np.testing.assert_array_equal(r["nested"]["x"][0].data, big.t().numpy())


def test_reader_runs_nothing(tmp_path):
    marker = tmp_path / "ran"
    # protocol-0 pickle of os.system("touch <marker>"): unpickling it would run the command
    payload = f"cos\nsystem\n(V touch {marker}\ntR.".encode()
    path = str(tmp_path / "evil.pt")
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("evil/data.pkl", payload)
    r = ck.read_checkpoint(path)
    assert isinstance(r, ck.Call) and r.func == ck.Global("os", "system")
    assert not marker.exists()


class _Storage:
    """A storage marker the crafted pickler below writes as a persistent id."""


def _crafted_checkpoint(path, numel, offset, size, stride):
    """A torch-zip checkpoint whose one tensor is `_rebuild_tensor_v2(storage of numel floats,
    offset, size, stride)` with the given (possibly hostile) view arguments."""
    import pickle
    st = _Storage()

    class P(pickle.Pickler):
        def persistent_id(self, obj):
            return ("storage", torch.FloatStorage, "0", "cpu", numel) if obj is st else None

    class T:
        def __reduce__(self):
            return torch._utils._rebuild_tensor_v2, (st, offset, size, stride, False, collections.OrderedDict())

    buf = io.BytesIO()
    P(buf, protocol=2).dump({"t": T()})
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("ck/data.pkl", buf.getvalue())
        z.writestr("ck/data/0", np.arange(numel, dtype="<f4").tobytes())


def test_reader_rejects_out_of_bounds_views(tmp_path):
    path = str(tmp_path / "ok.pt")
    _crafted_checkpoint(path, 12, 2, (2, 3), (4, 1))  # in bounds: elements 2..8
    r = ck.read_checkpoint(path)
    np.testing.assert_array_equal(r["t"].data, np.array([[2, 3, 4], [6, 7, 8]], np.float32))
    bad = {"offset past the end": (12, (1,), (1,)), "oversized shape": (0, (4, 4), (4, 1)),
           "oversized stride": (0, (2, 3), (40, 1)), "negative stride": (5, (3,), (-1,)),
           "negative offset": (-1, (2,), (1,)), "negative size": (0, (-2, 3), (3, 1))}
    for what, (off, size, stride) in bad.items():
        p = str(tmp_path / "bad.pt")
        _crafted_checkpoint(p, 12, off, size, stride)
        with pytest.raises(ValueError):
            ck.read_checkpoint(p)
            pytest.fail(what)
    # an empty view reads nothing and is accepted
    _crafted_checkpoint(path, 12, 0, (0, 5), (5, 1))
    assert ck.read_checkpoint(path)["t"].data.shape == (0, 5)


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference checkpoints not present (GPU box)")
def test_shipped_checkpoints_match_fixture():
    z = np.load(os.path.join(GOLD, "ckpt_actors.npz"))
    for tag, rel in (("level3_fear_4k", "fear/Single_MADDPG_4k.pt"), ("level3_wofear", "wo_fear/Single_MADDPG.pt")):
        st = ck.actor_state(os.path.join(REF_MODELS, rel))
        want = ck.actor_state(z, tag=tag)
        assert sorted(st) == sorted(want)
        for k in st:
            assert np.array_equal(st[k], want[k]), (tag, k)


def _f64_forward(st, x):
    """agilerl 1.0.15 EvolvableMLP forward (feature_net: linear, layer norm, ReLU per hidden
    layer, then linear_layer_output; the GumbelSoftmax output activation is applied by
    get_action), float64."""
    def ln(h, w, b):
        m = h.mean(-1, keepdims=True)
        v = ((h - m) ** 2).mean(-1, keepdims=True)
        return (h - m) / np.sqrt(v + 1e-5) * w + b
    f = lambda n: st[n].astype(np.float64)
    h = x.astype(np.float64)
    for i in range(2):
        h = np.maximum(ln(h @ f(f"linear_layer_{i}.weight").T + f(f"linear_layer_{i}.bias"),
                          f(f"layer_norm_{i}.weight"), f(f"layer_norm_{i}.bias")), 0.0)
    return h @ f("linear_layer_output.weight").T + f("linear_layer_output.bias")


@pytest.mark.parametrize("tag", ["level3_fear_4k", "level3_wofear"])
def test_loaded_actor_matches_f64_forward(tag):
    z = np.load(os.path.join(GOLD, "ckpt_actors.npz"))
    st = ck.actor_state(z, tag=tag)
    actors = ck.load_actors([st], 10, 16)
    t = np.load(os.path.join(GOLD, "single_traj.npz"))
    obs = np.concatenate([t[k] for k in t.files if k.endswith("/obs")]).astype(np.float32) / 2  # int8 half-units
    with torch.no_grad():
        got = actors(torch.from_numpy(obs).reshape(1, -1, 10, 16))[0].double().numpy()
    want = _f64_forward(st, obs.reshape(-1, 160))
    err = np.abs(got - want) / (1 + np.abs(want))
    # f32 forward of a 160-128-128-9 MLP with two LayerNorms: measured max 1.4e-5 (fear_4k) and
    # 1.5e-4 (wofear: rows whose hidden pre-activations have a small spread, which LayerNorm
    # scales up), median ~1e-6
    assert err.max() < 1e-3 and np.median(err) < 1e-5, (err.max(), np.median(err))
    # the trained policy is not degenerate: several actions are the argmax somewhere
    assert len(np.unique(want.argmax(-1))) >= 2
