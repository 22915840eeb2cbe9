"""Drop-in single-agent ``CustomEnv`` (custom/customenv.py of the reference) backed by the HIP env.

Same constructor and gym-style ``reset()`` / ``step(action)`` as the reference
(custom/customenv.py:48-183, 186-348): one RL agent (agent 0) among Level 3's four world agents,
the apple at (9, 15), ``step(action)`` uses ``action[0]`` and returns
``(obs f64 [10, 16], [reward], [terminated], truncated, info)`` with ``info = {"episode": {"r",
"l"}, "restricted", "fear"}``.  The kernels run the variant 1 of ``gw_config`` (see
include/gridenv.h): float rewards (-10 crash, +20 apple when apples_caught has exactly one
entry, +0.1 closer to the apple), no truncation on a crash, raw WorldState ids in the obs.

Differences, deliberate: the RNG of spawns / scripted agents is the Philox stream keyed by
``seed`` (the reference uses an unseeded module-level default_rng, numpy's global MT19937 and
Python's ``random``); after the apple is eaten the reference raises StopIteration on a further
step (``next(iter({}))``, customenv.py:130) while this env keeps measuring the distance to the
apple's cell; ``render`` is out of scope.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from marlnav.scenario import CompiledScenario, builtin
from marlnav.vec_env import VecGridEnv

from .ma_customenv import Box, Discrete

N_DISCRETE_ACTIONS = 9


class CustomEnv:
    def __init__(self, render=False, fear=True, seed=None, scenario: str | CompiledScenario = "level3_single",
                 device=None):
        if render:
            raise NotImplementedError("render() is out of scope of the HIP build (pygame UI)")
        sc = builtin(scenario) if isinstance(scenario, str) else scenario
        if sc.K != 1:
            raise ValueError("the single-agent CustomEnv needs a scenario with one RL agent")
        self.scenario = sc
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")
        self.seed = int(seed)
        self.action_space = Discrete(N_DISCRETE_ACTIONS)                                   # :55
        self.observation_space = Box(low=-1.0, high=16.0, shape=(sc.H, sc.W), dtype=np.float64)  # :57-58
        self.num_agents = 1
        self.fear = fear
        self.rendering = False
        self._env = VecGridEnv(sc, num_envs=1, fear=fear, fear_weight=0.0, max_steps=0, auto_reset=False,
                               seed=self.seed, device=device, debug=True, variant=1)
        self._initialized = False
        self.episode_reward = 0
        self.episode_length = 0
        self.observation = None

    @property
    def AgentLocations(self):
        pos = self._env.positions()[0].cpu().numpy()
        return [self.scenario.rc(c) for c in pos]

    def render(self, mode="human"):
        raise NotImplementedError("render() is out of scope of the HIP build (pygame UI)")

    def close(self):
        pass

    def reset(self, seed=None, options=None):                                              # :186-348
        obs, _ = self._env.reset()
        torch.cuda.synchronize(self._env.device)
        self._initialized = True
        self.episode_reward = 0
        self.episode_length = 0
        self.observation = obs[0, 0].cpu().numpy().astype(np.float64)
        return self.observation, {}

    def step(self, action):                                                                # :78-183
        if not self._initialized:
            raise RuntimeError("step() before reset()")
        a = int(action[0])
        if not 0 <= a < N_DISCRETE_ACTIONS:
            raise ValueError(f"action must be in 0..8, got {action!r}")
        r = self._env.step(torch.tensor([[a]], dtype=torch.int32))
        torch.cuda.synchronize(self._env.device)
        reward = float(r.reward[0, 0].item())
        reward = int(reward) if reward == int(reward) else reward  # the reference's int unless +0.1
        self.episode_length += 1
        self.episode_reward += reward
        self.observation = r.obs[0, 0].cpu().numpy().astype(np.float64)
        info = {"episode": {"r": self.episode_reward, "l": self.episode_length},
                "restricted": bool(int(r.restr_bits[0].item()) & 1),
                "fear": np.float64(r.fear[0, 0].item())}
        return self.observation, [reward], [bool(r.term[0, 0].item())], bool(r.trunc[0, 0].item()), info


def manhattan_dist(loc_1, loc_2):                                                          # :404-405
    return sum(abs(a - b) for a, b in zip(loc_1, loc_2))
