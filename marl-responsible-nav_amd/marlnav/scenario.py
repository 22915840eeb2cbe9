"""Scenario loading and compilation into the static device tables of the grid world.

A scenario uses the reference's JSON schema (``custom/Scenarios.json``: ``Map.Region``,
``Map.Walls``, ``Map.OneWays``, ``Policies``/``MdRs`` with ``slicex``/``slicey`` triples,
``N_Agents``, ``defaultAction``) plus two optional keys of ours: ``Apples``
(``{"apple_k": [r, c]}``) and ``N_Intelligent`` (K, the RL agents).

Compilation follows the reference exactly:

* slices -> ``slice(a, b, None if step == 0 else step)``      custom/grid_world.py:621-651
* ``policy_map[slicex, slicey] = key`` in key order, later keys override earlier ones;
  a cell's policy is ``str(policy_map[r, c]).zfill(2)``       custom/ma_customenv.py:346-354,438
* the same for the MdR map                                   custom/ma_customenv.py:357-365,445
* ``GeneratePolicy(stepWeights, directionWeights)``:
  ``p = [sw0] + [sw_k * dw for k >= 1]`` normalised          custom/custom_agent.py:181-197
  and the 25 % branch ``directionWeights = None`` -> [1,1,1,1] custom/ma_customenv.py:441-443
* numpy legacy ``choice(p=...)``: ``cdf = cumsum(p); cdf /= cdf[-1]``, sampled by
  ``searchsorted(cdf, u, 'right')``.
* action masks                                               custom/ma_customenv.py:467-506
* apples default to Level 3's ``{"apple_0": (9, 0), "apple_1": (5, 10)}`` (:422).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np

N_ACTIONS = 9
# custom/custom_agent.py:41-178 (rows grow downward): Stay, Up1, Down1, Left1, Right1, Up2, ...
ACTION_NAMES = ["Stay", "Up1", "Down1", "Left1", "Right1", "Up2", "Down2", "Left2", "Right2"]
MOVE_LEN = np.array([1, 1, 1, 1, 1, 2, 2, 2, 2], dtype=np.int32)
MOVE_DR = np.array([0, -1, 1, 0, 0, -1, 1, 0, 0], dtype=np.int32)
MOVE_DC = np.array([0, 0, 0, -1, 1, 0, 0, -1, 1], dtype=np.int32)
LEVEL3_APPLES = {"apple_0": (9, 0), "apple_1": (5, 10)}

_HERE = os.path.dirname(os.path.abspath(__file__))
SCENARIO_DIR = os.path.join(os.path.dirname(_HERE), "scenarios")
MAX_AGENTS = 8


@dataclass
class CompiledScenario:
    name: str
    H: int
    W: int
    N: int
    K: int
    region: np.ndarray        # uint8 [H*W], 1 road / 0 inactive
    policy_id: np.ndarray     # uint8 [H*W], index into policy_keys
    policy_keys: list
    policy_p: np.ndarray      # f64 [P, 2, 9]  ([.,0] scenario weights, [.,1] uniform-direction)
    policy_cdf: np.ndarray    # f64 [P, 2, 9]
    mdr: np.ndarray           # uint8 [H*W], MdR action per cell
    apples: np.ndarray        # int32 [K], apple cell of RL agent k
    free_cells: np.ndarray    # int32 [F], road cells in row-major order
    okmask: np.ndarray        # uint8 [H*W], bit d: unit move d (0 U, 1 D, 2 L, 3 R) allowed
    action_mask: np.ndarray   # uint16 [H*W], 9-bit get_action_mask per cell
    default_action: str = "random"
    source: dict = field(default_factory=dict, repr=False)

    @property
    def HW(self) -> int:
        return self.H * self.W

    def policy_map(self) -> np.ndarray:
        """Integer policy map exactly as ``CustomMAEnv.policy_map`` holds it."""
        keys = np.array([int(k) for k in self.policy_keys], dtype=np.int64)
        return keys[self.policy_id].reshape(self.H, self.W)

    def mdr_map_actions(self) -> np.ndarray:
        return self.mdr.reshape(self.H, self.W).astype(np.int64)

    def cell(self, r: int, c: int) -> int:
        return int(r) * self.W + int(c)

    def rc(self, cell: int):
        return int(cell) // self.W, int(cell) % self.W


def _to_slice(triple):
    a, b, s = triple
    return slice(a, b, None if s == 0 else s)


def generate_policy(step_weights, direction_weights=None) -> np.ndarray:
    """custom/custom_agent.py:181-197."""
    if step_weights is None:
        step_weights = [5, 4, 3, 2, 1]
    if direction_weights is None:
        direction_weights = [1, 1, 1, 1]
    p = [step_weights[0]]
    for sw in step_weights[1:]:
        p = p + [sw * x for x in direction_weights]
    p = np.array(p)
    return p / p.sum()


def legacy_choice_cdf(p: np.ndarray) -> np.ndarray:
    cdf = np.asarray(p, dtype=np.float64).cumsum()
    cdf /= cdf[-1]
    return cdf


def action_mask_table(region2d: np.ndarray) -> np.ndarray:
    """get_action_mask (custom/ma_customenv.py:467-506) for every cell."""
    H, W = region2d.shape
    out = np.zeros(H * W, dtype=np.uint16)
    for x in range(H):
        for y in range(W):
            m = 0x1FF
            if x - 1 < 0 or region2d[x - 1][y] == 0: m &= ~(1 << 1)
            if x + 1 >= H or region2d[x + 1][y] == 0: m &= ~(1 << 2)
            if y - 1 < 0 or region2d[x][y - 1] == 0: m &= ~(1 << 3)
            if y + 1 >= W or region2d[x][y + 1] == 0: m &= ~(1 << 4)
            if x - 2 < 0 or region2d[x - 2][y] == 0: m &= ~(1 << 5)
            if x + 2 >= H or region2d[x + 2][y] == 0: m &= ~(1 << 6)
            if y - 2 < 0 or region2d[x][y - 2] == 0: m &= ~(1 << 7)
            if y + 2 >= W or region2d[x][y + 2] == 0: m &= ~(1 << 8)
            out[x * W + y] = m
    return out


def okmask_table(region2d: np.ndarray) -> np.ndarray:
    """Per cell, which unit moves (U, D, L, R) stay on the grid and land on an active cell
    (the clip + ``WorldState[new] >= 0`` tests of custom/grid_world.py:486-518)."""
    H, W = region2d.shape
    out = np.zeros(H * W, dtype=np.uint8)
    for r in range(H):
        for c in range(W):
            m = 0
            for d, (dr, dc) in enumerate(((-1, 0), (1, 0), (0, -1), (0, 1))):
                rr, cc = r + dr, c + dc
                if 0 <= rr < H and 0 <= cc < W and region2d[rr, cc] != 0:
                    m |= 1 << d
            out[r * W + c] = m
    return out


def compile_scenario(sc: dict, name: str = "scenario", n_agents: int | None = None,
                     n_rl: int | None = None, apples: dict | None = None) -> CompiledScenario:
    region2d = np.array(sc["Map"]["Region"])
    H, W = region2d.shape
    if sc["Map"].get("Walls") or sc["Map"].get("OneWays"):
        # Loaded from JSON, the reference's wall entries are lists and never match the tuple
        # paths tested at custom/grid_world.py:498 -- walls are inert on the env path.
        pass
    N = int(n_agents if n_agents is not None else sc["N_Agents"])
    K = int(n_rl if n_rl is not None else sc.get("N_Intelligent", 2))
    if not (1 <= K <= N <= MAX_AGENTS):
        raise ValueError(f"need 1 <= K <= N <= {MAX_AGENTS}, got K={K} N={N}")
    if W < 2:
        raise ValueError("grid width must be >= 2")
    if sc.get("AgentLocations"):
        raise NotImplementedError("fixed AgentLocations are not supported (all scenarios spawn randomly)")
    if sc.get("SpecificAction4Agents"):
        raise NotImplementedError("SpecificAction4Agents is not supported")
    if sc.get("defaultAction", "random") != "random":
        raise NotImplementedError("only defaultAction='random' is supported")

    policies = sc["Policies"]
    policy_map = np.zeros((H, W), dtype=int)
    for key in policies:
        policy_map[_to_slice(policies[key]["slicex"]), _to_slice(policies[key]["slicey"])] = int(key)
    mdrs = sc["MdRs"]
    mdr_key_map = np.zeros((H, W), dtype=int)
    for key in mdrs:
        mdr_key_map[_to_slice(mdrs[key]["slicex"]), _to_slice(mdrs[key]["slicey"])] = int(key)

    keys = list(policies.keys())
    key_index = {k: i for i, k in enumerate(keys)}
    if len(keys) > 255:
        raise ValueError("at most 255 policies")
    policy_id = np.zeros(H * W, dtype=np.uint8)
    mdr = np.zeros(H * W, dtype=np.uint8)
    for r in range(H):
        for c in range(W):
            pk = str(policy_map[r, c]).zfill(2)
            mk = str(mdr_key_map[r, c]).zfill(2)
            policy_id[r * W + c] = key_index[pk]
            a = int(mdrs[mk]["mdr"])
            if not 0 <= a < N_ACTIONS:
                raise ValueError(f"MdR action {a} out of range")
            mdr[r * W + c] = a
    P = len(keys)
    policy_p = np.zeros((P, 2, N_ACTIONS), dtype=np.float64)
    policy_cdf = np.zeros((P, 2, N_ACTIONS), dtype=np.float64)
    for i, k in enumerate(keys):
        sw = policies[k]["stepWeights"]
        dw = policies[k]["directionWeights"]
        for v, d in enumerate((dw, None)):
            p = generate_policy(sw, d)
            if p.shape != (N_ACTIONS,) or not np.all(np.isfinite(p)):
                raise ValueError(f"policy {k} does not give 9 finite probabilities")
            policy_p[i, v] = p
            policy_cdf[i, v] = legacy_choice_cdf(p)

    region = (region2d != 0).astype(np.uint8).reshape(-1)
    free = np.flatnonzero(region2d.reshape(-1) == 1).astype(np.int32)
    if free.size < N:
        raise ValueError("fewer road cells than agents")
    if apples is None:
        apples = sc.get("Apples", LEVEL3_APPLES)
    apple_cells = np.zeros(K, dtype=np.int32)
    for k in range(K):
        r, c = apples[f"apple_{k}"]
        if not (0 <= r < H and 0 <= c < W):
            raise ValueError(f"apple_{k} outside the grid")
        apple_cells[k] = r * W + c
    return CompiledScenario(
        name=name, H=H, W=W, N=N, K=K, region=region, policy_id=policy_id, policy_keys=keys,
        policy_p=policy_p, policy_cdf=policy_cdf, mdr=mdr, apples=apple_cells, free_cells=free,
        okmask=okmask_table(region2d), action_mask=action_mask_table(region2d),
        default_action=sc.get("defaultAction", "random"), source=sc)


def load_scenario_json(path: str, scenario_name: str) -> dict:
    """LoadJsonScenario (custom/grid_world.py:621-674) without the slice conversion
    (compile_scenario converts the ``[a, b, step]`` triples itself)."""
    with open(path) as f:
        return json.load(f)[scenario_name]


def level3_like(H: int, W: int, n_agents: int = 4, n_rl: int = 2) -> dict:
    """A scenario with Level 3's topology scaled to H x W.

    Level 3 (custom/Scenarios.json:64-103) is an outer clockwise ring of 2-step roads, two
    vertical connectors at columns W//3 and 2W//3, and an inner anticlockwise 1-step loop on
    rows H//5 and H-3; MdR = the 1-step version of the ring direction.  level3_like(10, 16)
    reproduces Level 3's region, policy map and MdR map exactly (tests/test_scenario.py)."""
    if H < 8 or W < 8:
        raise ValueError("level3_like needs H, W >= 8")
    a, b = W // 3, (2 * W) // 3
    r1, r2 = H // 5, H - 3
    region = np.zeros((H, W))
    region[0, :] = region[H - 1, :] = 1
    region[:, 0] = region[:, W - 1] = 1
    region[:, a] = region[:, b] = 1
    region[r1, a:b + 1] = region[r2, a:b + 1] = 1

    def pol(sw, dw, sx, sy):
        return {"directionWeights": dw, "slicex": sx, "slicey": sy, "stepWeights": sw}

    R2, R1 = [0, 0, 1], [0, 1, 0]
    U, D, L, Rt = [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]
    policies = {
        "00": pol([1, 1, 0], [1, 1, 1, 1], [0, H, 0], [0, W, 0]),
        "01": pol(R2, Rt, [0, 1, 0], [0, W - 1, 0]),
        "02": pol(R2, L, [H - 1, H, 0], [1, W, 0]),
        "03": pol(R2, U, [1, H, 0], [0, 1, 0]),
        "04": pol(R2, D, [0, H - 1, 0], [W - 1, W, 0]),
        "05": pol(R1, Rt, [r2, r2 + 1, 0], [a, b + 1, 0]),
        "06": pol(R1, L, [r1, r1 + 1, 0], [a + 1, b + 1, 0]),
        "07": pol(R1, U, [r1 + 1, r2 + 1, 0], [b, b + 1, 0]),
        "08": pol(R1, D, [r1, r2, 0], [a, a + 1, 0]),
        "09": pol(R2, Rt, [0, 1, 0], [0, 1, 0]),
        "10": pol(R2, L, [H - 1, H, 0], [W - 1, W, 0]),
        "11": pol(R2, U, [H - 1, H, 0], [0, 1, 0]),
        "12": pol(R2, D, [0, 1, 0], [W - 1, W, 0]),
    }
    mdrs = {
        "00": {"mdr": 0, "slicex": [0, H, 0], "slicey": [0, W, 0]},
        "01": {"mdr": 4, "slicex": [0, 1, 0], "slicey": [0, W - 1, 0]},
        "02": {"mdr": 3, "slicex": [H - 1, H, 0], "slicey": [1, W, 0]},
        "03": {"mdr": 1, "slicex": [1, H, 0], "slicey": [0, 1, 0]},
        "04": {"mdr": 2, "slicex": [0, H - 1, 0], "slicey": [W - 1, W, 0]},
    }
    apples = {"apple_0": [H - 1, 0], "apple_1": [H // 2, b]}
    for k in range(2, n_rl):  # extra RL agents: apples spread along the top road
        apples[f"apple_{k}"] = [0, (k * W) // (n_rl + 1)]
    return {
        "AgentLocations": [], "Map": {"Region": region.tolist(), "Walls": [], "OneWays": []},
        "MdRs": mdrs, "N_Agents": n_agents, "N_Intelligent": n_rl, "Policies": policies,
        "SpecificAction4Agents": [], "defaultAction": "random", "Apples": apples,
    }


BUILTIN = {
    # name: (H, W, N, K)
    "level3": (10, 16, 4, 2),       # Level 3 of custom/Scenarios.json (BASELINE config 1)
    "grid32": (32, 32, 4, 2),       # BASELINE configs 2, 3, 5
    "grid64_n8": (64, 64, 8, 2),    # BASELINE config 4
    "level3_single": (10, 16, 4, 1),  # single-agent CustomEnv: Level 3, apple_0 at (9, 15) (customenv.py:334)
}


def _builtin_dict(name: str) -> dict:
    H, W, N, K = BUILTIN[name]
    sc = level3_like(H, W, N, K)
    if name == "level3_single":
        sc["Apples"] = {"apple_0": [H - 1, W - 1]}
    return sc


def builtin(name: str) -> CompiledScenario:
    path = os.path.join(SCENARIO_DIR, f"{name}.json")
    if os.path.exists(path):
        with open(path) as f:
            sc = json.load(f)
    elif name in BUILTIN:
        sc = _builtin_dict(name)
    else:
        raise KeyError(f"unknown scenario {name!r}; builtins: {sorted(BUILTIN)}")
    return compile_scenario(sc, name=name)


def write_builtin_jsons() -> None:
    os.makedirs(SCENARIO_DIR, exist_ok=True)
    for name in BUILTIN:
        with open(os.path.join(SCENARIO_DIR, f"{name}.json"), "w") as f:
            json.dump(_builtin_dict(name), f)
