"""No-code reader of the reference's agilerl checkpoints (``models/custom/**/*.pt``).

The reference saves its trained agents with agilerl's ``MADDPG.saveCheckpoint`` (a
``torch.save`` zip: ``<name>/data.pkl`` + raw little-endian storages ``<name>/data/<key>``) and
evaluates them with ``agents.load_wo_memory(path, filename)`` (``customeval.py:39-64``,
``maddpg/agent.py:279-281``).  Those pickles name dill / numpy globals, so
``torch.load(weights_only=True)`` refuses them, and they must never be unpickled (nothing from the
file may run).  This module reads them WITHOUT unpickling:

* ``pickletools.genops`` disassembles ``data.pkl`` into opcodes (it constructs nothing);
* a symbolic stack machine replays those opcodes into inert Python data: a GLOBAL is a
  ``Global(module, name)`` record (never imported or looked up), a REDUCE / NEWOBJ is a ``Call``
  record, a BUILD attaches its state to an ``Obj`` record, a persistent id is a ``PersId`` record;
* tensors are the ``Call(torch._utils._rebuild_tensor_v2, (PersId(('storage', dtype, key, device,
  numel)), offset, size, stride, ...))`` records; their bytes are read from the zip member
  ``data/<key>`` with ``numpy.frombuffer`` (f32 / f64 / int64 storages only).

``read_checkpoint(path)`` returns the dict the checkpoint holds with every tensor as a numpy array
and every other leaf as plain data; ``actor_weights(ckpt, agent)`` names the agilerl EvolvableMLP
actor's layers (``feature_net.linear_layer_0.weight (128, 160)``, ``layer_norm_0``,
``linear_layer_1``, ``layer_norm_1``, ``linear_layer_output (9, 128)``) for
``marlnav.actor``'s MLP actors.
"""
from __future__ import annotations

import pickletools
import zipfile
from dataclasses import dataclass, field

import numpy as np


@dataclass(frozen=True)
class Global:
    """A GLOBAL opcode's (module, name): recorded, never imported."""
    module: str
    name: str


@dataclass
class Call:
    """REDUCE / NEWOBJ of an inert callable on inert arguments."""
    func: object
    args: tuple


@dataclass
class Obj:
    """An object a BUILD gave state to (e.g. an nn.Module with its __dict__)."""
    base: object
    state: object = None


@dataclass(frozen=True)
class PersId:
    pid: tuple


@dataclass
class Tensor:
    """A tensor record: storage key, dtype name, element offset, shape, strides (elements)."""
    key: str
    dtype: str
    offset: int
    shape: tuple
    stride: tuple
    data: np.ndarray = field(default=None, repr=False)


_STORAGE_DTYPES = {"FloatStorage": np.float32, "DoubleStorage": np.float64, "LongStorage": np.int64,
                   "IntStorage": np.int32, "HalfStorage": np.float16, "ByteStorage": np.uint8,
                   "BoolStorage": np.bool_}

_MARK = object()


def _replay(data: bytes):
    """Evaluate the opcode stream into inert records (no object of the file is constructed)."""
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("EMPTY_DICT",):
            stack.append({})
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_SET":
            stack.append(set())
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "DICT":
            items = pop_mark()
            stack.append({_hashable(items[i]): items[i + 1] for i in range(0, len(items), 2)})
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            _setitem(stack[-1], k, v)
        elif n == "SETITEMS":
            items = pop_mark()
            for i in range(0, len(items), 2):
                _setitem(stack[-1], items[i], items[i + 1])
        elif n == "APPEND":
            v = stack.pop()
            _append(stack[-1], [v])
        elif n == "APPENDS":
            _append(stack[-1], pop_mark())
        elif n == "ADDITEMS":
            items = pop_mark()
            if isinstance(stack[-1], set):
                stack[-1].update(_hashable(x) for x in items)
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n in ("GLOBAL",):
            mod, name = arg.split(" ", 1)
            stack.append(Global(mod, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(Global(mod, name))
        elif n in ("REDUCE",):
            args = stack.pop()
            func = stack.pop()
            stack.append(_call(func, args))
        elif n == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(Call(cls, tuple(args)))
        elif n == "NEWOBJ_EX":
            kw = stack.pop()
            args = stack.pop()
            cls = stack.pop()
            stack.append(Call(cls, tuple(args) + (kw,)))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, Obj):
                obj.state = state
            elif isinstance(obj, dict):
                pass  # an OrderedDict's own attributes (a state_dict's _metadata): not needed
            else:
                stack[-1] = Obj(obj, state)
        elif n == "BINPERSID":
            stack.append(PersId(_freeze(stack.pop())))
        elif n == "POP":
            stack.pop()
        elif n == "POP_MARK":
            pop_mark()
        elif n == "DUP":
            stack.append(stack[-1])
        elif n in ("NONE",):
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n in ("BININT", "BININT1", "BININT2", "INT", "LONG", "LONG1", "LONG4", "BINFLOAT", "FLOAT",
                   "BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "UNICODE", "STRING", "BINSTRING",
                   "SHORT_BINSTRING", "BINBYTES", "SHORT_BINBYTES", "BINBYTES8", "BYTEARRAY8"):
            stack.append(arg)
        else:
            raise ValueError(f"checkpoint reader: unsupported pickle opcode {n}")
    if len(stack) != 1:
        raise ValueError("checkpoint reader: malformed pickle stream")
    return stack[0]


def _freeze(x):
    if isinstance(x, list):
        return tuple(_freeze(v) for v in x)
    if isinstance(x, tuple):
        return tuple(_freeze(v) for v in x)
    return x


def _hashable(k):
    try:
        hash(k)
        return k
    except TypeError:
        return repr(k)


def _setitem(target, k, v):
    if isinstance(target, dict):
        target[_hashable(k)] = v
    elif isinstance(target, Call):  # e.g. OrderedDict() then SETITEMS: keep the items on the record
        if not target.args or not isinstance(target.args[-1], dict) or not getattr(target, "_items", False):
            target.args = tuple(target.args) + ({},)
            target._items = True
        target.args[-1][_hashable(k)] = v


def _append(target, items):
    if isinstance(target, list):
        target.extend(items)
    elif isinstance(target, Call):
        if not getattr(target, "_list", False):
            target.args = tuple(target.args) + ([],)
            target._list = True
        target.args[-1].extend(items)


def _call(func, args):
    """REDUCE: tensors become Tensor records, OrderedDict() an (ordered) dict, other calls stay
    inert Call records.  Nothing is imported or executed."""
    args = tuple(args) if isinstance(args, (tuple, list)) else (args,)
    if func == Global("torch._utils", "_rebuild_tensor_v2") or func == Global("torch._utils", "_rebuild_tensor"):
        pid, offset, size, stride = args[0], args[1], args[2], args[3]
        if not isinstance(pid, PersId) or pid.pid[0] != "storage":
            raise ValueError("checkpoint reader: tensor without a storage id")
        stype = pid.pid[1]
        dtype = stype.name if isinstance(stype, Global) else str(stype)
        return Tensor(key=str(pid.pid[2]), dtype=dtype, offset=int(offset), shape=tuple(size), stride=tuple(stride))
    if func == Global("collections", "OrderedDict"):
        d = {}
        if args and isinstance(args[0], (list, tuple)):
            for kv in args[0]:
                d[_hashable(kv[0])] = kv[1]
        return d
    return Call(func, args)


def _check_view(t: "Tensor", numel: int):
    """Reject a tensor record whose (offset, shape, stride) would read outside its storage of
    `numel` elements: the values come from the (untrusted) file and feed as_strided."""
    ints = (t.offset,) + tuple(t.shape) + tuple(t.stride)
    if not all(isinstance(v, int) and not isinstance(v, bool) for v in ints):
        raise ValueError(f"checkpoint reader: non-integer view of storage {t.key}")
    if len(t.shape) != len(t.stride):
        raise ValueError(f"checkpoint reader: shape / stride rank mismatch in storage {t.key}")
    if t.offset < 0 or any(n < 0 for n in t.shape) or any(s < 0 for s in t.stride):
        raise ValueError(f"checkpoint reader: negative offset, size or stride in storage {t.key}")
    if any(n == 0 for n in t.shape):
        return  # empty view: nothing is read
    last = t.offset + sum((n - 1) * s for n, s in zip(t.shape, t.stride))
    if last >= numel:
        raise ValueError(f"checkpoint reader: view of storage {t.key} reaches element {last} "
                         f"of {numel}")


def _attach(obj, z: zipfile.ZipFile, prefix: str, seen=None):
    """Read every Tensor record's bytes from its storage member (depth-first, shared records once)."""
    seen = set() if seen is None else seen
    if id(obj) in seen:
        return
    seen.add(id(obj))
    if isinstance(obj, Tensor):
        dt = _STORAGE_DTYPES.get(obj.dtype)
        if dt is None:
            raise ValueError(f"checkpoint reader: unsupported storage type {obj.dtype}")
        raw = np.frombuffer(z.read(f"{prefix}data/{obj.key}"), dtype=np.dtype(dt).newbyteorder("<"))
        _check_view(obj, len(raw))
        itemsize = raw.itemsize
        if any(n == 0 for n in obj.shape):
            view = np.zeros(obj.shape, dtype=dt)
        elif obj.shape:
            view = np.lib.stride_tricks.as_strided(raw[obj.offset:], shape=obj.shape,
                                                   strides=tuple(s * itemsize for s in obj.stride))
        else:
            view = raw[obj.offset:obj.offset + 1].reshape(())
        obj.data = np.array(view, dtype=dt)  # a contiguous copy
        return
    if isinstance(obj, dict):
        for v in obj.values():
            _attach(v, z, prefix, seen)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _attach(v, z, prefix, seen)
    elif isinstance(obj, Call):
        _attach(obj.args, z, prefix, seen)
    elif isinstance(obj, Obj):
        _attach(obj.base, z, prefix, seen)
        _attach(obj.state, z, prefix, seen)


def read_checkpoint(path: str):
    """The checkpoint's top-level object as inert data, tensors as ``Tensor`` records carrying
    numpy arrays.  Raises ValueError for anything but a torch zip checkpoint."""
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
        pkl = [n for n in names if n.endswith("data.pkl")]
        if len(pkl) != 1:
            raise ValueError(f"{path}: not a torch zip checkpoint (data.pkl members: {len(pkl)})")
        prefix = pkl[0][: -len("data.pkl")]
        root = _replay(z.read(pkl[0]))
        _attach(root, z, prefix)
    return root


def module_tensors(obj, prefix: str = "") -> dict:
    """name -> numpy array of every parameter / buffer under an nn.Module record (its BUILD state's
    ``_parameters``, ``_buffers`` and, recursively, ``_modules``), torch's state_dict naming."""
    out = {}
    st = obj.state if isinstance(obj, Obj) else obj
    if isinstance(st, tuple) and st and isinstance(st[0], dict):  # (dict state, slot state)
        st = st[0]
    if not isinstance(st, dict):
        return out
    for group in ("_parameters", "_buffers"):
        for name, t in (st.get(group) or {}).items():
            t = t.base if isinstance(t, Obj) else t
            if isinstance(t, Call) and t.args and isinstance(t.args[0], Tensor):  # Parameter(tensor, ...)
                t = t.args[0]
            if isinstance(t, Tensor):
                out[prefix + name] = t.data
    for name, sub in (st.get("_modules") or {}).items():
        if sub is not None:
            out.update(module_tensors(sub, prefix + name + "."))
    return out


def state_dict_tensors(d) -> dict:
    """name -> numpy array of a state-dict (an OrderedDict of tensors)."""
    return {k: (v.data if isinstance(v, Tensor) else v) for k, v in d.items() if isinstance(v, Tensor)}


# agilerl 1.0.15 EvolvableMLP layer names -> (layer index, kind)
_MLP_LAYERS = [("feature_net.linear_layer_0", "linear", 0), ("feature_net.layer_norm_0", "ln", 0),
               ("feature_net.linear_layer_1", "linear", 1), ("feature_net.layer_norm_1", "ln", 1),
               ("feature_net.linear_layer_output", "linear", 2)]


def actor_weights(ckpt, agent: int = 0) -> dict:
    """The agilerl MLP actor of `agent` as {"weights": [W1, W2, W3], "biases": [...], "ln_w": [...],
    "ln_b": [...]} (numpy f32; W as (out, in), torch's layout).  Looks in the checkpoint's
    ``actors_state_dict`` list, else in its ``actor_networks`` module records."""
    if not isinstance(ckpt, dict):
        raise ValueError("checkpoint reader: the checkpoint is not a dict")
    sd = None
    if isinstance(ckpt.get("actors_state_dict"), (list, tuple)) and len(ckpt["actors_state_dict"]) > agent:
        sd = state_dict_tensors(ckpt["actors_state_dict"][agent])
    if not sd and isinstance(ckpt.get("actor_networks"), (list, tuple)) and len(ckpt["actor_networks"]) > agent:
        sd = module_tensors(ckpt["actor_networks"][agent])
    if not sd:
        raise ValueError("checkpoint reader: no actor weights found")
    out = {"weights": [None] * 3, "biases": [None] * 3, "ln_w": [None] * 2, "ln_b": [None] * 2}
    for name, kind, i in _MLP_LAYERS:
        w, b = sd.get(name + ".weight"), sd.get(name + ".bias")
        if w is None or b is None:
            raise ValueError(f"checkpoint reader: actor layer {name} missing (have {sorted(sd)[:8]} ...)")
        if kind == "linear":
            out["weights"][i], out["biases"][i] = w.astype(np.float32), b.astype(np.float32)
        else:
            out["ln_w"][i], out["ln_b"][i] = w.astype(np.float32), b.astype(np.float32)
    return out


def net_config(ckpt) -> dict:
    """The plain-data entries of the checkpoint's ``net_config`` / ``actors_init_dict`` (arch,
    hidden sizes, output activation) for a consistency check; {} if absent."""
    out = {}
    for key in ("net_config", "actors_init_dict"):
        v = ckpt.get(key) if isinstance(ckpt, dict) else None
        if isinstance(v, list) and v:
            v = v[0]
        if isinstance(v, dict):
            out.update({k: x for k, x in v.items() if isinstance(x, (str, int, float, bool, list, tuple))})
    return out


def actor_state(source, agent: int = 0, tag: str | None = None) -> dict:
    """One agent's actor in the checkpoint's naming without the ``feature_net.`` prefix
    (``linear_layer_0.weight`` (out, in), ...; ``StackedMLPActors.load_agent``'s input), from
    a reference ``.pt`` checkpoint (read with ``read_checkpoint``) or from a mapping of
    ``[<tag>/]feature_net.<layer>.<param>`` arrays (tests/golden/ckpt_actors.npz)."""
    if isinstance(source, str) and source.endswith(".pt"):
        c = read_checkpoint(source)
        sd = None
        if isinstance(c.get("actors_state_dict"), (list, tuple)) and len(c["actors_state_dict"]) > agent:
            sd = state_dict_tensors(c["actors_state_dict"][agent])
        if not sd:
            w = actor_weights(c, agent)
            sd = {}
            for (name, kind, i) in _MLP_LAYERS:
                src_w, src_b = (w["weights"], w["biases"]) if kind == "linear" else (w["ln_w"], w["ln_b"])
                sd[name + ".weight"], sd[name + ".bias"] = src_w[i], src_b[i]
    else:
        pre = f"{tag}/" if tag else ""
        sd = {k[len(pre):]: np.asarray(v) for k, v in dict(source).items() if k.startswith(pre)}
    out = {k[len("feature_net."):]: np.asarray(v, dtype=np.float32) for k, v in sd.items()
           if k.startswith("feature_net.")}
    if "linear_layer_0.weight" not in out:
        raise ValueError("checkpoint reader: no feature_net actor layers")
    return out


def load_actors(states: list, H: int, W: int, device=None):
    """MultiAgentActors (MLP, K = len(states)) holding the given per-agent actor states
    (``actor_state``): what ``agents.load_wo_memory`` restores for evaluation
    (maddpg/agent.py:279-281, customeval.py:63).  The input width must be H * W."""
    from .actor import MultiAgentActors
    K = len(states)
    hidden = tuple(int(states[0][f"linear_layer_{i}.weight"].shape[0])
                   for i in range(sum(1 for k in states[0] if k.startswith("linear_layer_") and k.endswith(".weight")
                                      and k != "linear_layer_output.weight")))
    in_dim = int(states[0]["linear_layer_0.weight"].shape[1])
    if in_dim != H * W:
        raise ValueError(f"checkpoint actor input {in_dim} != H * W = {H * W}")
    actors = MultiAgentActors(K, H, W, "mlp", hidden=hidden, device=device)
    for k, st in enumerate(states):
        actors.net.load_agent(k, st)
    actors.mark_updated()
    return actors
