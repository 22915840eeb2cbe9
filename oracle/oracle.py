"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The C restatement of the reference algorithm (see gw_oracle.h).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker or the timed
CPU baseline, never as the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
MAXN = 8


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "gw_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE, "-B" if force else "liboracle.so"], check=True)
    return LIB_PATH


class World(C.Structure):
    _fields_ = [("H", C.c_int32), ("W", C.c_int32), ("N", C.c_int32), ("K", C.c_int32),
                ("region", C.c_void_p), ("policy_id", C.c_void_p), ("policy_cdf", C.c_void_p),
                ("mdr", C.c_void_p), ("apples", C.c_void_p), ("n_free", C.c_int32),
                ("free_cells", C.c_void_p), ("fear", C.c_int32), ("fear_weight", C.c_double),
                ("max_steps", C.c_int32), ("seed", C.c_uint64), ("env_offset", C.c_int64),
                ("variant", C.c_int32)]


class Env(C.Structure):
    _fields_ = [("pos", C.c_int32 * MAXN), ("apples", C.c_uint32), ("term", C.c_uint32),
                ("trunc", C.c_uint32), ("prev_dist", C.c_int32 * MAXN), ("t", C.c_int32),
                ("episode", C.c_uint32), ("score", C.c_double), ("fear_score", C.c_double)]


class StepOut(C.Structure):
    _fields_ = [("actions", C.c_int32 * MAXN), ("mdr", C.c_int32 * MAXN),
                ("final_pos", C.c_int32 * MAXN), ("crash_bits", C.c_uint32),
                ("restricted_bits", C.c_uint32), ("reward", C.c_double * MAXN),
                ("fear", C.c_double * MAXN), ("shaped", C.c_double * MAXN),
                ("term", C.c_uint8 * MAXN), ("trunc", C.c_uint8 * MAXN),
                ("mask", C.c_uint16 * MAXN), ("crashes", C.c_int32),
                ("apples_caught", C.c_int32), ("done", C.c_uint8), ("ep_return", C.c_double),
                ("ep_fear", C.c_double), ("ep_len", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        p = C.c_void_p
        L.orc_philox4x32_10.argtypes = [p, p, p]
        L.orc_np_sum.argtypes = [p, C.c_int]
        L.orc_np_sum.restype = C.c_double
        L.orc_update_world.argtypes = [C.c_int, C.c_int, p, C.c_int, p, p, C.c_int, p, p, p, p, p, p]
        L.orc_update_world.restype = C.c_int
        L.orc_fear_one_actor.argtypes = [C.c_int, C.c_int, p, C.c_int, p, C.c_int, p, p, p, C.c_int, p, p, p]
        L.orc_fear_one_actor.restype = C.c_double
        L.orc_fear_matrix.argtypes = [C.c_int, C.c_int, p, C.c_int, p, C.c_int, p, p, p, p, p, p]
        L.orc_fear_matrix.restype = None
        L.orc_feal.argtypes = [C.c_int, C.c_int, p, C.c_int, p, C.c_int, p, p, p, p, p, p]
        L.orc_feal.restype = None
        L.orc_action_mask.argtypes = [C.c_int, C.c_int, p, C.c_int]
        L.orc_action_mask.restype = C.c_uint16
        L.orc_env_reset.argtypes = [p, C.c_int64, p, p, p, p]
        L.orc_env_step.argtypes = [p, C.c_int64, p, p, p, p, C.c_int, p, p, p]
        L.orc_vec_step.argtypes = [p, p, C.c_int64, p, C.c_int, p, p, C.c_int]
        L.orc_vec_step_final.argtypes = [p, p, C.c_int64, p, C.c_int, p, p, p, C.c_int]
        L.orc_vec_reset.argtypes = [p, p, C.c_int64, p, C.c_int]
        L.orc_sizeof_env.restype = C.c_int
        L.orc_sizeof_step_out.restype = C.c_int
        assert L.orc_sizeof_env() == C.sizeof(Env), "orc_env layout mismatch"
        assert L.orc_sizeof_step_out() == C.sizeof(StepOut), "orc_step_out layout mismatch"
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags.c_contiguous
    return a.ctypes.data


def philox(ctr, key) -> np.ndarray:
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().orc_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def np_sum(a) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
    return lib().orc_np_sum(_ptr(a), a.size)


def update_world(H, W, region, loc, act, apple_cells=None):
    """GWorld.UpdateGWorld; returns (crash[N], restricted[N], final[N], caught[(agent, apple)], loops)."""
    region = np.ascontiguousarray(region, dtype=np.uint8).reshape(-1)
    loc = np.ascontiguousarray(loc, dtype=np.int32)
    act = np.ascontiguousarray(act, dtype=np.int32)
    N = loc.size
    crash = np.zeros(N, np.uint8)
    restr = np.zeros(N, np.uint8)
    fin = np.zeros(N, np.int32)
    caught = np.zeros(2 * 4 * MAXN * MAXN, np.int32)
    nc = np.zeros(1, np.int32)
    ap = None if apple_cells is None else np.ascontiguousarray(apple_cells, dtype=np.int32)
    loops = lib().orc_update_world(H, W, _ptr(region), N, _ptr(loc), _ptr(act),
                                   0 if ap is None else ap.size, _ptr(ap), _ptr(crash), _ptr(restr),
                                   _ptr(fin), _ptr(caught), _ptr(nc))
    pairs = [(int(caught[2 * i]), int(caught[2 * i + 1])) for i in range(int(nc[0]))]
    return crash.astype(bool), restr.astype(bool), fin, pairs, loops


def fear_one_actor(H, W, region, loc, list_ids, list_acts, mdr_acts, actor):
    region = np.ascontiguousarray(region, dtype=np.uint8).reshape(-1)
    loc = np.ascontiguousarray(loc, dtype=np.int32)
    N = loc.size
    ids = np.ascontiguousarray(list_ids, dtype=np.int32)
    acts = np.ascontiguousarray(list_acts, dtype=np.int32)
    mdr = np.ascontiguousarray(mdr_acts, dtype=np.int32)
    resp = np.zeros(N * N, np.float64)
    vm = np.zeros(N, np.int32)
    va = np.zeros(N, np.int32)
    s = lib().orc_fear_one_actor(H, W, _ptr(region), N, _ptr(loc), ids.size, _ptr(ids), _ptr(acts),
                                 _ptr(mdr), int(actor), _ptr(resp), _ptr(vm), _ptr(va))
    return s, resp.reshape(N, N), vm, va


class OracleEnvs:
    """E independent envs stepped by the C restatement (replay or native-RNG mode)."""

    def __init__(self, sc, E: int, fear: bool, fear_weight: float = -5.0, max_steps: int = 150,
                 seed: int = 42, env_offset: int = 0, reset: bool = True, variant: int = 0):
        self.sc = sc
        self.E = int(E)
        self._keep = dict(region=np.ascontiguousarray(sc.region, np.uint8),
                          policy_id=np.ascontiguousarray(sc.policy_id, np.uint8),
                          cdf=np.ascontiguousarray(sc.policy_cdf, np.float64),
                          mdr=np.ascontiguousarray(sc.mdr, np.uint8),
                          apples=np.ascontiguousarray(sc.apples, np.int32),
                          free=np.ascontiguousarray(sc.free_cells, np.int32))
        k = self._keep
        self.world = World(sc.H, sc.W, sc.N, sc.K, _ptr(k["region"]), _ptr(k["policy_id"]),
                           _ptr(k["cdf"]), _ptr(k["mdr"]), _ptr(k["apples"]), k["free"].size,
                           _ptr(k["free"]), int(bool(fear)), float(fear_weight), int(max_steps),
                           int(seed) & 0xFFFFFFFFFFFFFFFF, int(env_offset), int(variant))
        self.envs = (Env * self.E)()
        self.env_offset = int(env_offset)
        if reset:
            self.reset_all()

    def reset_all(self, obs: np.ndarray | None = None, nthreads: int = 1):
        lib().orc_vec_reset(C.byref(self.world), self.envs, self.E, _ptr(obs), nthreads)

    def reset_one(self, e: int, spawn=None, episode: int | None = None):
        sc = self.sc
        obs = np.zeros((sc.K, sc.HW), np.float32)
        mask = np.zeros(sc.K, np.uint16)
        if episode is not None:
            self.envs[e].episode = episode
        sp = None if spawn is None else np.ascontiguousarray(spawn, np.int32)
        lib().orc_env_reset(C.byref(self.world), self.env_offset + e, C.byref(self.envs[e]), _ptr(sp),
                            _ptr(obs), _ptr(mask))
        return obs, mask

    def step_one(self, e: int, rl_act=None, scripted=None, spawn=None, auto_reset: bool = True):
        sc = self.sc
        obs = np.zeros((sc.K, sc.HW), np.float32)
        final_obs = np.full((sc.K, sc.HW), np.nan, np.float32)
        out = StepOut()
        ra = None if rl_act is None else np.ascontiguousarray(rl_act, np.int32)
        sa = None if scripted is None else np.ascontiguousarray(scripted, np.int32)
        sp = None if spawn is None else np.ascontiguousarray(spawn, np.int32)
        lib().orc_env_step(C.byref(self.world), self.env_offset + e, C.byref(self.envs[e]), _ptr(ra),
                           _ptr(sa), _ptr(sp), int(auto_reset), _ptr(obs), _ptr(final_obs),
                           C.byref(out))
        return obs, final_obs, out

    def vec_step(self, rl_act=None, obs: np.ndarray | None = None, outs=None, nthreads: int = 1,
                 auto_reset: bool = True, final_obs: np.ndarray | None = None):
        """obs / final_obs: [K, E, H*W] float32 (final_obs rows written for the envs that ended)."""
        ra = None if rl_act is None else np.ascontiguousarray(rl_act, np.int32)
        lib().orc_vec_step_final(C.byref(self.world), self.envs, self.E, _ptr(ra), int(auto_reset),
                                 _ptr(obs), _ptr(final_obs), outs, nthreads)

    def state(self, e: int) -> Env:
        return self.envs[e]

    def positions(self) -> np.ndarray:
        N = self.sc.N
        return np.array([[self.envs[e].pos[n] for n in range(N)] for e in range(self.E)], np.int32)


def fear_matrix(H, W, region, loc, acts, mdr, in_list=None):
    """Responsibility.FeAR + FeAL of one world snapshot (C restatement).  in_list: which agents
    are in ActionID4Agents (the others take 'stay' and ignore swaps); None = all.
    -> dict resp [N,N], vm, va [N,N], feal [N], feal_vm, feal_va [N]."""
    N = len(loc)
    region = np.ascontiguousarray(region, np.uint8).reshape(-1)
    loc = np.ascontiguousarray(loc, np.int32)
    mdr = np.ascontiguousarray(mdr, np.int32)
    ids = np.array([n for n in range(N) if in_list is None or in_list[n]], np.int32)
    la = np.ascontiguousarray(np.asarray(acts, np.int32)[ids])
    out = dict(resp=np.zeros((N, N)), vm=np.zeros((N, N), np.int32), va=np.zeros((N, N), np.int32),
               feal=np.zeros(N), feal_vm=np.zeros(N, np.int32), feal_va=np.zeros(N, np.int32))
    lib().orc_fear_matrix(H, W, _ptr(region), N, _ptr(loc), len(ids), _ptr(ids), _ptr(la), _ptr(mdr),
                          _ptr(out["resp"]), _ptr(out["vm"]), _ptr(out["va"]))
    lib().orc_feal(H, W, _ptr(region), N, _ptr(loc), len(ids), _ptr(ids), _ptr(la), _ptr(mdr),
                   _ptr(out["feal"]), _ptr(out["feal_vm"]), _ptr(out["feal_va"]))
    return out
