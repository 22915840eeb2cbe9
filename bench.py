#!/usr/bin/env python3
"""Headline benchmark: agent-env-steps/s of the vectorised grid-world step (BASELINE.json).

A "step" = one batched CustomMAEnv.step (custom/ma_customenv.py:217-334) over every env of
this rank: scripted policy + random RL policy drawn on device, FeAR counterfactuals
(custom/Responsibility.py:135-210), world update, rewards, the rollout reward/score arithmetic
(maddpg/agent.py:124-173), auto-reset, float32 observations for every RL agent and the
per-block statistics, and the per-step all-gather of the completed-episode returns (RCCL over
xGMI with --gpus N > 1: a fixed-size packed slot per rank; the statistics are accumulated by the
step kernels and all-reduced once, after the timed region).  Inputs are resident in HBM before
the timed region.

Default workload = BASELINE config 3 (the north-star shape): 4-agent 32x32 grid, 65536 envs
per GPU, FeAR on with weight -5 (configs/custom_fear_5.yaml).  value = all ranks' envs x N
agents x steps / max-over-ranks wall time.

  python bench.py [--gpus N --steps K --warmup W] [--config c3|c2|c2env|c4|c1|c5|...] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "marl-responsible-nav_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "agent-env-steps/sec at 64k envs × 4 agents, 1/2/4/8 MI355X; HBM BW fraction"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

CONFIGS = {
    "c3": dict(scenario="grid32", envs=65536, fear=True, fear_weight=-5.0,
               workload="BASELINE config 3: 4-agent (2 RL) 32x32 Level-3-like grid, 65536 envs/GPU, "
                        "FeAR on (weight -5, configs/custom_fear_5.yaml), random RL policy"),
    "c2": dict(scenario="grid32", envs=4096, fear=False, fear_weight=-2.0, rollout=True,
               workload="BASELINE config 2: 4-agent 32x32 grid, 4096 envs, FeAR off (configs/custom.yaml), the "
                        "MLP actors of configs/mlp.yaml (128-128, GumbelSoftmax + mask + argmax; fused "
                        "gw_actor_act) acting on the full-grid obs every step, env step, zero-copy replay ring "
                        "of MEMORY_SIZE 200000 (maddpg/agent.py:89,109-127,190-197)"),
    "c2env": dict(scenario="grid32", envs=4096, fear=False, fear_weight=-2.0,
                  workload="BASELINE config 2's env alone: 4-agent 32x32 grid, 4096 envs, FeAR off, random RL "
                           "policy on device (no actor)"),
    "c4": dict(scenario="grid64_n8", envs=65536, fear=False, fear_weight=-5.0,
               workload="BASELINE config 4: 8-agent 64x64 grid, 65536 envs, FeAR off"),
    "c4f": dict(scenario="grid64_n8", envs=65536, fear=True, fear_weight=-5.0,
                workload="8-agent 64x64 grid, 65536 envs, FeAR on"),
    "c1": dict(scenario="level3", envs=1, fear=False, fear_weight=-2.0,
               workload="BASELINE config 1: Level 3 (10x16), 1 env, random policy"),
    "c5": dict(scenario="grid32", envs=65536, fear=True, fear_weight=-5.0, rollout=True,
               workload="BASELINE config 5 per GPU: 32x32, N=4, K=2, 65536 envs/GPU, FeAR on, full rollout "
                        "(stacked MLP actors + GumbelSoftmax + mask + argmax, env step, zero-copy replay ring of "
                        "MEMORY_SIZE 200000, per-step RCCL all-gather of the completed-episode returns; statistics "
                        "accumulated by the step kernels, all-reduced once when read)"),
    "c5patch": dict(scenario="grid32", envs=65536, fear=True, fear_weight=-5.0, rollout=True, patch=11,
                    workload="C5's rollout with egocentric 11x11 local observations (gw_obs_patch; not a "
                             "reference format, reported separately): no dense obs, the MADDPG MLP actors on "
                             "121 inputs (fused gw_patch_actor_act), patch replay ring, FeAR on"),
    "c4patch": dict(scenario="grid64_n8", envs=65536, fear=False, fear_weight=-5.0, rollout=True, arch="cnn", patch=16,
                    workload="BASELINE config 4's CNN head (configs/cnn.yaml: conv 32-64 k2 s2, 128-128; f32 weights, layer 2 "
                             "as bf16x3 MFMA products) on "
                             "egocentric 16x16 local windows (gw_obs_patch; not a reference format, reported "
                             "separately): 8-agent 64x64 grid, 65536 envs, no dense obs, the fused CNN head "
                             "(gw_patch_cnn_act: per-centre tables + recomputed positions), patch replay ring"),
    "c4cnn": dict(scenario="grid64_n8", envs=65536, fear=False, fear_weight=-5.0, rollout=True, arch="cnn",
                  workload="BASELINE config 4 as a rollout: 8-agent 64x64 grid, 65536 envs, the configs/cnn.yaml "
                           "actor head (conv 32-64, k2 s2, 128-128; f32 weights, layer 2 as bf16x3 MFMA products; fused "
                           "gw_cnn_act from the obs "
                           "descriptors), env step, replay ring"),
}


def algorithmic_bytes(N: int, K: int, HW: int, obs_bytes: int = 4):
    """Bytes per env-step each kernel must move at minimum:
    step_kernel: state read+write (pos 4N, flags 4, t 4, prev 4K, score 8, fear_score 8; x2)
                 + episode 4 read + outputs (reward/fear/shaped 24K, term/trunc 2K, mask 2K,
                 done 1, crashes 4, apples 4, ep_return 8, ep_fear 8, ep_len 4)
                 + obs descriptor 20 written;
    obs_kernel:  obs 4*K*HW written (2*K*HW with --obs-dtype bf16) + descriptor 20 read."""
    state = 2 * (4 * N + 4 + 4 + 4 * K + 8 + 8) + 4
    outputs = 24 * K + 2 * K + 2 * K + 1 + 4 + 4 + 8 + 8 + 4
    step_b = state + outputs + 20
    obs_b = obs_bytes * K * HW + 20
    return step_b, obs_b


# gw_profile span kinds (include/gridenv.h GW_SPAN_*) -> the kernel names of bench lines / rocprofv3
SPAN_KINDS = {0: "step_kernel", 1: "obs_kernel", 2: "fear_kernel", 3: "act_kernel", 4: "cnn_l1_kernel",
              5: "cnn_list_kernels", 6: "cnn_rare_kernel", 7: "window_kernel", 8: "learn_update"}
F32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA (v_mfma_f32_16x16x4_f32), no xf32 on gfx950
# VALU issue peak (MI355X_MICROARCH.md "Execution model": "A wave (64 lanes) is assigned to one SIMD
# and issues each VALU instruction over 2 cycles (32 lanes/cycle x 2)"): each of 256 CUs x 4 SIMD-32
# issues one wave64 vector instruction per 2 cycles at the 2.4 GHz max clock = 1.2288e12
# wave-instructions/s = 64 lanes x 4 SIMDs / 2 = 128 lane-ops per CU per clock.  Against the
# one-wave64-per-CU-per-clock figure sometimes quoted for CDNA (64 lane-ops per CU per clock) every
# VALU fraction would be 2x; the line states the basis (VALU_PEAK_BASIS)
VALU_PEAK_GIPS = 256 * 4 * 2.4e9 / 2 / 1e9
VALU_PEAK_BASIS = ("256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md "
                   "'Execution model'); at 1 wave64 per CU per clock the fractions would double")
HID, N_ACT = 128, 9        # the fused actors' hidden width and actions (configs/mlp.yaml, configs/cnn.yaml)
# what the fused actors compute in: f32 weights and activations, layer 2 as bf16x3 products
# (hi / mid / lo bf16 parts, the 6 largest of the 9 part products on v_mfma_f32_16x16x32_bf16, f32
# accumulation: ~2^-23 relative per product), layer 3 on f32 MFMA; their roofline counts the f32-equivalent
# flops against the f32 MFMA peak
ACT_PRECISION = "f32 weights; layer 2 as bf16x3 MFMA products (f32-equivalent flops vs the f32 MFMA peak); layer 3 f32 MFMA"


def kernel_work(kind: int, N: int, K: int, HW: int, E: int, obs_bytes: int = 4, patch: int = 0, valu=None):
    """(bound, algorithmic work per step of one GW_SPAN kind, unit) for the roofline:
    HBM bytes for the env / writer kernels, f32 MFMA flops for the fused
    actors' MLP kernel (layers 2-3, 2 * (128 * 128 + 128 * 9) per (env, agent);
    its layer 1 is a gather of table rows, not a GEMM).  None where the work is data-dependent
    (the CNN recompute: a few positions per step)."""
    step_b, obs_b = algorithmic_bytes(N, K, HW, obs_bytes)
    valu = valu or {}
    if kind in (0, 2) and valu.get(kind):
        # the world update and the FeAR counterfactuals are integer-VALU / latency chains (SURVEY
        # §8d): their work is the vector instructions per step, from the committed rocprofv3
        # SQ_INSTS_VALU pass of the same config (profiles/latest.json), against the VALU issue peak
        return "valu", valu[kind], "inst"
    if kind == 0:
        return "hbm", step_b * E, "B"
    if kind == 1:
        return "hbm", obs_b * E, "B"
    if kind == 2:  # FeAR: integer-VALU bound; without a VALU pass, its state / output bytes
        return "hbm", (16 + 32 + 16 * K + 16) * E, "B"
    if kind == 3:
        return "mfma", 2 * E * K * (HID * HID + HID * N_ACT), "flop"
    if kind in (4, 5):  # descriptors read + a per-(env, agent) word of positions / list entries
        return "hbm", (48 + 4 * K) * E, "B"
    if kind == 7:  # the windows written (f32) + the 48-byte descriptors read
        return "hbm", (4 * K * patch * patch + 48) * E, "B"
    if kind == 8:  # one descriptor-learner update: its 128 x 128 layers on f32 MFMA --
        # critic tail: K target actors + target critic + critic forward + critic backward, actor
        # tail: actor / critic forward, critic / actor backward, and the two W2 gradients, per agent
        # and row: (4 + 4 + 2) K B (2 * 128 * 128) flops with B = 128 (layer 1 is a table gather)
        return "mfma", 10 * K * 128 * 2 * HID * HID, "flop"
    return "mfma", None, "flop"


def host_cpus():
    """What the host offers this job: the machine's logical CPUs, the ones this process may run
    on (affinity), the cgroup CPU quota (cpu.max) and the CPU model (lscpu / /proc/cpuinfo)."""
    total = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                model = ln.split(":", 1)[1].strip()
                break
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    if model is None:
        try:
            with open("/proc/cpuinfo") as f:
                model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
        except OSError:
            pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota)))
    return {"nproc": total, "affinity": affinity, "cgroup_quota_cpus": quota, "usable": usable, "model": model}


def cpu_baseline(cfg, seconds: float = 12.0):
    """The C restatement (oracle/, test infrastructure) on the host cores: same scenario,
    same step semantics, native-RNG mode, OpenMP over envs (one thread per usable host core:
    the job's CPU affinity capped by its cgroup quota; MARLNAV_CPU_THREADS overrides).
    Bounded sample (~`seconds` of CPU work)."""
    import numpy as np
    from marlnav import scenario as S
    from oracle import oracle as O

    sc = S.builtin(cfg["scenario"])
    cpus = host_cpus()
    threads = int(os.environ.get("MARLNAV_CPU_THREADS", "0") or 0) or cpus["usable"]
    threads = max(1, threads)
    E = max(4096 if cfg["fear"] else 16384, 256 * threads)
    orc = O.OracleEnvs(sc, E, fear=cfg["fear"], fear_weight=cfg["fear_weight"], seed=42, reset=False)
    obs = np.zeros((sc.K, E, sc.HW), np.float32)
    orc.reset_all(obs=obs, nthreads=threads)
    orc.vec_step(None, obs=obs, nthreads=threads)  # warm
    steps, t0 = 0, time.perf_counter()
    while True:
        orc.vec_step(None, obs=obs, nthreads=threads)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 2000:
            break
    value = E * sc.N * steps / el
    return {"value": value, "unit": "agent-env-steps/s", "cores": threads, "kind": "port",
            "per_core": value / threads, "host": cpus,
            "sample": f"{E} envs x {steps} steps of {cfg['scenario']} (fear={'on' if cfg['fear'] else 'off'}, "
                      f"obs written) in {el:.1f}s by oracle/gw_oracle.c (bit-exact C restatement of the "
                      f"reference step), {threads} OpenMP threads = every core this job may use "
                      f"(affinity {cpus['affinity']} of nproc {cpus['nproc']}, cgroup quota "
                      f"{cpus['cgroup_quota_cpus']}; {cpus['model']})"}


def launch_plan(gpus: int, argv: list, base_env: dict, port: int):
    """The per-rank (argv, env) of ``bench.py --gpus N`` started without a launcher: N child
    processes of this script, one per GPU, with torchrun's variables (RANK = LOCAL_RANK = r,
    WORLD_SIZE = N, rendezvous on 127.0.0.1:port).  Pure function (tests/test_bench_cpu.py)."""
    plans = []
    for r in range(int(gpus)):
        env = dict(base_env)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plans.append(([sys.executable, os.path.abspath(__file__)] + list(argv), env))
    return plans


def launch_ranks(gpus: int, argv: list) -> int:
    """Run ``launch_plan`` and wait; a rank that fails ends the others.  Called before anything
    touches the GPU (the children initialise it, each on its own device)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen(cmd, env=env) for cmd, env in launch_plan(gpus, argv, os.environ, port)]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def busy_ms(spans, kind: int):
    """(union of the launch intervals of `kind`, launches): a kernel's busy time, with launches
    that overlap (obs writers of consecutive steps on two streams) counted once."""
    iv = sorted((float(b), float(e)) for k, b, e in spans if int(k) == kind)
    total, cur_b, cur_e = 0.0, None, None
    for b, e in iv:
        if cur_e is None or b > cur_e:
            if cur_e is not None:
                total += cur_e - cur_b
            cur_b, cur_e = b, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        total += cur_e - cur_b
    return total, len(iv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=0, help="override envs per GPU")
    ap.add_argument("--fear", type=int, default=-1, help="override FeAR on (1) / off (0)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--updates-per-step", type=int, default=0,
                    help="c5 only: MADDPG updates (batch 128, one HIP-graph replay each) per env step")
    ap.add_argument("--dense-learn", action="store_true",
                    help="with --updates-per-step: sample the dense obs slots (waiting for the obs writer) "
                         "instead of the descriptor ring (A/B)")
    ap.add_argument("--learn-launches", action="store_true",
                    help="with --updates-per-step: re-issue the update's recorded launches (MADDPG.capture("
                         "launches=True)); the default since late round 4")
    ap.add_argument("--learn-graph", action="store_true",
                    help="with --updates-per-step: replay the update as a HIP graph instead (A/B)")
    ap.add_argument("--eager-learn", action="store_true",
                    help="with --updates-per-step: issue the update eagerly instead of replaying its HIP graph (A/B)")
    ap.add_argument("--profile-steps", type=int, default=64,
                    help="after the timed region, time this many more steps' kernels with HIP events "
                         "carried by their launches (the live roofline; 0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cnn-torch", action="store_true",
                    help="c4cnn: the PyTorch CNN forward on the dense obs instead of gw_cnn_act (A/B)")
    ap.add_argument("--patch-torch", action="store_true",
                    help="c5patch / c4patch: the PyTorch actor forward on the written windows instead of "
                         "gw_patch_actor_act / gw_patch_cnn_act (A/B)")
    ap.add_argument("--high-prio", action="store_true",
                    help="run the step chain on a high-priority stream (its kernels' workgroups are "
                         "dispatched ahead of the concurrent obs writer's)")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the per-step all-gather of every env's completed-episode return (A/B)")
    ap.add_argument("--sync-obs", action="store_true",
                    help="write each step's obs before the next step starts (no step pipeline; A/B)")
    ap.add_argument("--fear-async", action="store_true",
                    help="c5: let the next actor overlap the FeAR kernel (gw_set_obs_async | 4; A/B, "
                         "measured slower: profiles/r1_async)")
    ap.add_argument("--obs-dtype", default="f32", choices=["f32", "bf16"],
                    help="bf16: the lossless compact obs format (gw_set_obs_dtype); reported separately, "
                         "the metric's definition is f32 obs")
    ap.add_argument("--obs-eager", action="store_true",
                    help="start each step's obs writer right after its world update (the default)")
    ap.add_argument("--obs-lazy", action="store_true",
                    help="launch each step's obs writer at the next step (gw_set_obs_async 2; A/B)")
    ap.add_argument("--obs-ring", type=int, default=-1,
                    help="env-only workloads: write each step's obs into the next of this many buffers "
                         "(a replay ring's slots), so consecutive pipelined writers need no order "
                         "between them (-1 = auto: 2 with async obs on the defer path, else 1)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="replay the timed steps as HIP graphs of this many captured steps (0 = eager "
                         "launches, -1 = auto: 16 for the launch-bound env-only workloads that run "
                         "synchronous obs on one rank, i.e. C1/C2, else eager)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start one rank per GPU ourselves, before any GPU call in this process
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    from marlnav.vec_env import VecGridEnv

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        # RCCL ("nccl") over xGMI; MARLNAV_DIST_BACKEND=gloo only rehearses the multi-rank path
        # with several ranks on one GPU (RCCL refuses duplicate devices)
        backend = os.environ.get("MARLNAV_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()
    if world != args.gpus:
        print(f"bench.py: the process group has {world} rank(s) but --gpus {args.gpus}", file=sys.stderr)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(2)

    if args.high_prio:
        torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    cfg = dict(CONFIGS[args.config])
    # obs writer pipelined with the next step (gw_set_obs_async), launched right after the world
    # update.  Measured A/B: profiles/r1_async/, profiles/r2_c5modes/
    obs_mode = False if args.sync_obs else ("lazy" if args.obs_lazy else True)
    if cfg.get("rollout") and not cfg.get("arch") and not cfg.get("patch") and not (args.obs_lazy or args.sync_obs):
        # the rollout's writer starts right after the world update, as 2 launches so that the next
        # actor's kernels are dispatched between them (150 vs 168 us per step lazily in one launch,
        # profiles/r2_c5modes); read by gw_create
        os.environ.setdefault("GW_OBS_CHUNKS", "2")
    if cfg.get("patch"):  # no dense obs: nothing to pipeline
        obs_mode = False
    if cfg.get("arch") == "cnn" and not cfg.get("patch") and not (args.cnn_torch or args.obs_lazy or args.sync_obs):
        # the 2.1 GB writer starts right after the world update, as 4 launches so that the next
        # actor's kernels are dispatched between them (profiles/r2_cnn: 0.715 ms per step lazy in
        # one launch -> 0.636); read by gw_create
        obs_mode = True
        os.environ.setdefault("GW_OBS_CHUNKS", "4")
        # one obs stream: overlapping writers take CUs from the CNN actor (614 vs 658 us per step)
        os.environ.setdefault("GW_OBS_STREAMS", "1")
    if args.envs:
        cfg["envs"] = args.envs
    if args.fear >= 0:
        cfg["fear"] = bool(args.fear)
        cfg["workload"] += f" [override: FeAR {'on' if cfg['fear'] else 'off'}]"
    E = cfg["envs"]
    env = VecGridEnv(cfg["scenario"], num_envs=E, fear=cfg["fear"], fear_weight=cfg["fear_weight"],
                     max_steps=150, auto_reset=True, seed=42, env_offset=rank * E, stats=True,
                     obs=not cfg.get("patch"),
                     obs_dtype=torch.bfloat16 if args.obs_dtype == "bf16" else torch.float32)
    N, K, HW = env.N, env.K, env.H * env.W
    # the defer path's small batches (below 128 MB of obs per step) run synchronous obs: its
    # pipeline's cross-queue waits cost more than the overlap saves there.  Batches of at most
    # 64 MiB run the merged path (gw_kernel_path), whose pipeline has no cross-queue waits.
    obs_bytes = E * K * HW * (2 if args.obs_dtype == "bf16" else 4)
    if obs_mode and env.kernel_path != "merged" and not cfg.get("rollout") and \
            not (args.obs_lazy or args.obs_eager) and obs_bytes < (128 << 20):
        obs_mode = False
    # a step of a few envs (C1) is bound by the host's launches: synchronous obs, HIP graphs
    if args.graph < 0 and not cfg.get("rollout") and world == 1 and obs_bytes <= (1 << 20) and \
            not (args.obs_lazy or args.obs_eager):
        obs_mode = False
    stream = torch.cuda.current_stream()

    from marlnav.parallel import ReturnGather
    # the step kernels add their statistics rows into a running total (gw_step_out.stats_acc):
    # no per-step reduction launch or collective; the per-step exchange is the return gather
    stats_acc = torch.zeros_like(env.out["stats"])
    # per-step RCCL all-gather of every env's completed-episode return + done flag (SURVEY §8e;
    # maddpg/agent.py:229-247): gw_step writes them straight into the send buffer
    graph_n = args.graph
    if graph_n < 0:  # auto: the host-bound regime (one rank; synchronous obs or merged path): the
        # env-only C1 / C2 lines, and the small-batch rollout (C2) with the fused MLP actor
        small_rollout = (cfg.get("rollout") and not cfg.get("patch") and not cfg.get("arch") and
                         env.kernel_path == "merged" and not args.updates_per_step)
        # the local-window rollouts (c5patch / c4patch): the fused window actors' host enqueue is
        # about as long as the step, so their steps replay as ring-phase graphs too
        window_rollout = (cfg.get("rollout") and cfg.get("patch") and not args.patch_torch and
                          not args.updates_per_step)
        graph_n = 16 if (world == 1 and (not obs_mode or env.kernel_path == "merged") and
                         (not cfg.get("rollout") or small_rollout or window_rollout)) else 0
    graph_n = min(graph_n, args.steps)
    if obs_mode and env.kernel_path == "merged":
        graph_n -= graph_n % 2  # merged async: an even number of captured steps
    gather = None if args.no_gather else ReturnGather(world * E, rank, world, env.device,
                                                      **({"window": graph_n} if graph_n else {}))

    n_ring = args.obs_ring if args.obs_ring >= 0 else \
        (2 if (obs_mode and env.kernel_path == "defer" and not cfg.get("rollout")) else 1)
    obs_ring = [env.out["obs"]] + [torch.empty_like(env.out["obs"]) for _ in range(n_ring - 1)] \
        if (n_ring > 1 and env.out["obs"] is not None) else None

    def one_step(i):
        into = gather.into() if gather is not None else {}
        into["stats_acc"] = stats_acc
        if obs_ring is not None:
            into["obs"] = obs_ring[i % len(obs_ring)]
        r = env.step(into=into)
        if gather is not None:
            gather.push()
        return r

    if cfg.get("rollout"):  # c5: actor -> env -> replay (+ optional MADDPG updates) per step
        from marlnav.maddpg import MADDPG
        from marlnav.rollout import Rollout
        from marlnav.parallel import broadcast_module
        # one set of actor weights for every rank: built from the same seed and broadcast from
        # rank 0 (MADDPG does it itself); every rank's sampling draws its own batches
        torch.cuda.manual_seed(1234 + rank)
        if cfg.get("patch") and cfg.get("arch") == "cnn":  # the CNN head on the P x P windows (fused
            # gw_patch_cnn_act from the obs descriptors; --patch-torch: the PyTorch forward, A/B)
            from marlnav.actor import MultiAgentActors
            learner = None
            actors = MultiAgentActors(K, cfg["patch"], cfg["patch"], arch="cnn", device=env.device, seed=0)
            broadcast_module(actors)
        elif cfg.get("patch"):  # local observations: the MADDPG actors on the P x P windows (fused
            # gw_patch_actor_act from the obs descriptors; --patch-torch: the PyTorch forward, A/B)
            learner = MADDPG(K, cfg["patch"], cfg["patch"], device=env.device, seed=0, capturable=True)
            actors = learner.actors
        elif cfg.get("arch") == "cnn":  # configs/cnn.yaml head: fused gw_cnn_act (or PyTorch, A/B)
            from marlnav.actor import MultiAgentActors
            learner = None
            actors = MultiAgentActors(K, env.H, env.W, arch="cnn", device=env.device, seed=0)
            broadcast_module(actors)
            if args.cnn_torch:  # the PyTorch forward reads the dense obs: synchronous obs
                obs_mode = False
        else:
            learner = MADDPG(K, env.H, env.W, device=env.device, seed=0, capturable=True)
            actors = learner.actors
        # the fused actor's Gumbel noise is Philox keyed by (seed; global env id, step, agent):
        # one seed for all ranks keeps every env's trajectory independent of the rank count
        # MEMORY_SIZE 200,000 transitions (configs/custom*.yaml); with graphs the ring's slots are
        # rounded up to a multiple of the graph length (one captured graph per ring phase)
        slots = -(-200_000 // E) + 1
        if graph_n:
            slots = -(-slots // graph_n) * graph_n
        ro = Rollout(env, actors, replay_slots=slots, training=True, seed=42,
                     fused=False if (args.cnn_torch or args.patch_torch) else None,
                     obs_async=obs_mode, fear_async=bool(obs_mode) and args.fear_async, gather=gather,
                     patch=cfg.get("patch", 0),
                     desc_ring=bool(args.updates_per_step) and not cfg.get("patch") and not args.dense_learn)
        ro.reset()

        def one_step(i):  # noqa: F811
            r = ro.step()  # the return gather inside is the per-step exchange across ranks
            if args.updates_per_step and learner is not None and ro.replay.t >= 2:
                ro.learn_fence()  # sampling reads the ring's descriptor (or obs) slots
                if args.eager_learn:  # A/B: the update's launches issued from the host each step
                    for _ in range(args.updates_per_step):
                        learner.learn_from(ro.replay)
                    return r
                if learner._graph is None:
                    learner.capture(ro.replay, actor_env=env if ro.fused and not cfg.get("patch") else None,
                                    launches=not args.learn_graph)
                for _ in range(args.updates_per_step):
                    learner.replay_learn()
            return r

    if not cfg.get("rollout"):
        env.set_obs_async(obs_mode)
        env.reset()
    # no Python garbage collection inside the timed region (as timeit does): the warmup's step
    # results would otherwise trigger a collection pause that idles the GPU (measured: +30 us per
    # step over 20 steps after 2,000 warmup steps).  The collection runs before the LAST warmup
    # step, which re-warms the host path: collecting right before the timed region left the first
    # timed step's host work (the return gather's views, gw_step's enqueue) 4-5x slower on cold
    # CPU caches, ~230 us of idle GPU in a 20-step run (tools/host_probe.py ... first)
    import gc
    for i in range(args.warmup):
        if i == args.warmup - 1:
            gc.collect()
            gc.disable()
        one_step(i)
    if args.warmup == 0:
        gc.collect()
        gc.disable()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # kernel spans come from --profile-steps eager steps AFTER the timed region (each profiled step
    # costs ~4-6 us of event bookkeeping in the pipeline, profiles/r2_events), so the timed steps
    # carry no profiling at all
    n_prof = max(0, args.profile_steps)
    graph = None
    if graph_n:
        # the timed steps as HIP graphs of graph_n steps (captured here, before the timed region:
        # nothing runs at capture), the remainder eagerly after them
        if env.obs_async and not env._obs_queued:  # merged async: capture after a queued writer
            graph_n = 0
    if graph_n:
        if gather is not None:
            gather.compact()  # the warmup's partial window
        # env only: VecGridEnv.capture_steps; the rollout: one graph per ring phase (Rollout.capture)
        graph = ro.capture(graph_n) if cfg.get("rollout") else env.capture_steps(graph_n, gather)
    n_graph = args.steps - args.steps % graph_n if graph_n else 0

    if n_prof:  # the profiling events exist before they are used (gw_profile creates them)
        env.profile(True, reserve=16 * (n_prof + 2))
        env.profile(False)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(0, n_graph, max(graph_n, 1)):
        graph.replay()
    t_first = []  # host time of the first eager timed steps (the pipeline fill is host-visible)
    for i in range(n_graph, args.steps):
        if len(t_first) < 4:
            th = time.perf_counter()
            one_step(i)
            t_first.append((time.perf_counter() - th) * 1e6)
        else:
            one_step(i)
    t_enq = time.perf_counter() - t0  # host time to enqueue the timed steps (host-bound if ~ wall)
    if cfg.get("rollout"):
        ro._flush()  # an unjoined FeAR step's statistics and return push (fear_async)
    if gather is not None:
        # the gathered returns of the last steps, compacted on the device (before the fences: the
        # compaction reads what the world updates wrote, so it overlaps the last obs writer)
        gather.compact()
    if cfg.get("rollout"):
        ro.fence()  # the last step's obs writes, FeAR outputs and statistics
    env.obs_fence()  # belong to the timed region
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gc.enable()
    gpu_ms = ev0.elapsed_time(ev1)
    spans = None
    sims = None
    if n_prof:
        # the kernel spans: n_prof eager steps right after the timed region (same env, same
        # kernels and pipeline, untimed; HIP timing events cannot be recorded inside a graph)
        sim_ctr = torch.zeros(1, dtype=torch.int64, device=env.device) if cfg["fear"] else None
        if sim_ctr is not None:
            env.count_sims(sim_ctr)  # the FeAR kernels' counterfactual world updates (gw_count_sims)
        env.profile(True)
        for i in range(n_prof):
            one_step(args.steps + i)
        if cfg.get("rollout"):
            ro.fence()
        env.obs_fence()  # the last profiled step's writer
        torch.cuda.synchronize()
        env.profile(False)
        if sim_ctr is not None:
            env.count_sims(None)
            sims = int(sim_ctr.item()) / n_prof  # de-duplicated sims per step (this rank)
        spans = env.profile_spans()
    (ms_step, ms_obs, ms_fear), nprof = env.profile_read()

    t_local = torch.tensor([wall], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t_local, op=dist.ReduceOp.MAX)
    t_max = float(t_local.item())
    stats = env.out["stats"].sum(0).cpu().tolist()
    gathered = None
    if gather is not None:
        drained = gather.drain()  # collective: the senders' backlogs (several ranks), untimed
        gathered = {"episodes": int(gather.n_completed.item()), "bytes_per_rank_per_step": gather.slot_bytes,
                    "drain_steps": drained,
                    "cap": getattr(gather, "cap", None),
                    "mean_return_last_100": float(gather.completed(last=100).mean()) if int(gather.n_completed) else None}

    if rank == 0:
        step_b, obs_b = algorithmic_bytes(N, K, cfg["patch"] ** 2 if cfg.get("patch") else HW,
                                          2 if args.obs_dtype == "bf16" else 4)
        avg_step_ms, avg_obs_ms = ms_step / max(nprof, 1), ms_obs / max(nprof, 1)
        avg_fear_ms = ms_fear / max(nprof, 1)
        # busy time per launch: the union of the launches' intervals / launches.  Equal to the
        # mean launch duration when launches do not overlap; with the obs writers of consecutive
        # steps overlapping on two streams a launch's own span covers part of its
        # neighbours' work, and the busy time is what a launch costs the timeline
        busy = {k: busy_ms(spans, k) if spans is not None and len(spans) else (0.0, 0) for k in SPAN_KINDS}
        busy_step_ms, busy_obs_ms = (busy[k][0] / max(busy[k][1], 1) for k in (0, 1))
        fused = env.fused
        merged = env.kernel_path == "merged" and bool(obs_mode)
        obs_bytes = 2 if args.obs_dtype == "bf16" else 4
        # the committed rocprofv3 evidence of this workload: profiles/latest.json["configs"][prof_key]
        # (C5 with n MADDPG updates per env step: "c5u<n>")
        prof_key = args.config + (f"u{args.updates_per_step}" if args.updates_per_step else "")
        # the VALU instructions per step of the integer-VALU kernels (world update, FeAR) from the
        # committed rocprofv3 SQ_INSTS_VALU pass of this config (tools/gpu_profile.sh)
        valu = {}
        try:
            with open(os.path.join(REPO, "profiles", "latest.json")) as f:
                pk = json.load(f).get("configs", {}).get(prof_key, {}).get("kernels", {})
            if not args.envs and args.fear < 0 and args.obs_dtype == "f32":
                for kd, nm in ((0, "step_kernel"), (2, "fear_kernel")):
                    v = pk.get(nm, {}).get("valu_insts_per_step")
                    if v:
                        valu[kd] = v
        except (OSError, ValueError, AttributeError):
            pass
        # every kernel kind's busy time per profiled step (the union of its launches' intervals /
        # steps: overlapping launches of one kind count once) and its roofline
        per_kind = {}
        for k, name in SPAN_KINDS.items():
            tot, n = busy[k]
            if not n:
                continue
            bound, work, unit = kernel_work(k, N, K, HW, E, obs_bytes, cfg.get("patch", 0), valu)
            ms = tot / max(nprof, 1)
            if k == 8:  # the learner's span is one update; a step may run several
                work = work * (n / max(nprof, 1)) if work else work
            peak = {"mfma": F32_MFMA_PEAK_TFS * 1e3, "valu": VALU_PEAK_GIPS}.get(bound, HBM_PEAK_GBS)
            rate = work / (ms * 1e-3) / 1e9 if (work and ms > 0) else None  # GB/s, GFLOP/s or G inst/s
            per_kind[name] = {"busy_ms_per_step": ms, "launches_per_step": n / max(nprof, 1), "bound": bound,
                              **({"precision": ACT_PRECISION} if k == 3 else {}),
                              "work_per_step": work, "work_unit": unit,
                              "achieved": rate / 1e3 if (rate and bound == "mfma") else rate,
                              "achieved_unit": {"mfma": "TFLOP/s", "valu": "G inst/s"}.get(bound, "GB/s"),
                              "frac": rate / peak if rate else None}
        if fused:  # one launch per step moves every byte of the step
            dom, bytes_per_launch, span, dur = "step_fused", (step_b + obs_b) * E, avg_step_ms, busy_step_ms
        elif merged:  # step_obs: step t + the obs writer of step t-1 in one launch (its spans: kind 1)
            dom, bytes_per_launch, span, dur = "step_obs", (step_b + obs_b) * E, avg_obs_ms, busy_obs_ms
        elif "learn_update" in per_kind:  # with updates the learner chain is the step's critical path
            # (the obs writer overlaps it on its own stream): the line names the update
            dom = "learn_update"
            _, bytes_per_launch, _ = kernel_work(8, N, K, HW, E, obs_bytes, cfg.get("patch", 0))
            launches = busy[8][1] / max(nprof, 1)
            dur = per_kind[dom]["busy_ms_per_step"] / max(launches, 1e-9)
            span = dur
        else:  # the kernel kind with the largest busy time per step
            dom = max(per_kind, key=lambda n: per_kind[n]["busy_ms_per_step"]) if per_kind else "obs_kernel"
            kd = next(k for k, n in SPAN_KINDS.items() if n == dom)
            _, bytes_per_launch, _ = kernel_work(kd, N, K, HW, E, obs_bytes, cfg.get("patch", 0))
            launches = busy[kd][1] / max(nprof, 1)  # launches (spans) of the kind per step
            dur = per_kind[dom]["busy_ms_per_step"] / max(launches, 1e-9) if per_kind else busy_obs_ms
            if bytes_per_launch is not None:
                bytes_per_launch = bytes_per_launch / max(launches, 1e-9)
            span = {0: avg_step_ms, 1: avg_obs_ms, 2: avg_fear_ms}.get(kd, dur)
        dom_bound = per_kind.get(dom, {}).get("bound", "hbm")
        mfma = dom_bound == "mfma"
        peak_u = F32_MFMA_PEAK_TFS if mfma else HBM_PEAK_GBS
        # the busy time comes from profiled steps after the timed region (their
        # events cost a few us per step), so it can exceed the timed step.  A kernel's busy time per
        # step cannot exceed the step it ran in: the time per launch used below is capped at the
        # timed ms_per_step / launches per step, and the uncapped profiled figure is kept beside it
        timed_ms = t_max * 1e3 / args.steps
        dom_lps = per_kind.get(dom, {}).get("launches_per_step") or 1.0
        dur_profiled = dur
        dur_cap = timed_ms / max(dom_lps, 1e-9)
        if dur > dur_cap:
            dur = dur_cap
        # achieved: GB/s (hbm) or TFLOP/s (mfma) of the dominant kernel's algorithmic work per launch
        # over its busy time per launch
        achieved = (bytes_per_launch / (dur * 1e-3) / (1e12 if mfma else 1e9)) if (dur > 0 and bytes_per_launch) else None
        traffic, traffic_src, prof_frac = None, None, None
        try:  # HBM bytes measured by the PMC passes committed under profiles/ for this workload
            with open(os.path.join(REPO, "profiles", "latest.json")) as f:
                prof = json.load(f)
            pc = prof.get("configs", {}).get(prof_key)
            if pc and not args.envs and args.fear < 0 and not fused and dom in pc["kernels"] \
                    and args.obs_dtype == "f32":
                pk = pc["kernels"][dom]
                traffic_src = pc["source"]
                # per step on both sides (the kernel trace may count a step's kernel as several
                # launches, e.g. the chunked obs writer): the trace's HBM bytes and busy time per
                # step, the live launches per step
                live_lps = per_kind.get(dom, {}).get("launches_per_step") or 1.0
                if pk.get("hbm_bytes_per_step") is not None:
                    traffic = pk["hbm_bytes_per_step"] / live_lps
                if bytes_per_launch and pk.get("busy_us_per_step"):
                    # the trace's busy time per step, capped at the timed step like `dur`
                    busy_us = min(pk["busy_us_per_step"], timed_ms * 1e3)
                    prof_frac = bytes_per_launch * live_lps / (busy_us * 1e-6) / \
                        (1e12 if mfma else 1e9) / peak_u
        except (OSError, KeyError, ValueError, TypeError):
            pass
        total_units = world * E * N * args.steps
        line = {
            "metric": METRIC,
            "value": total_units / t_max,
            "unit": "agent-env-steps/s",
            "n_gpus": world,
            # the process group the timed steps ran in (the driver's multi-GPU runs: RCCL over xGMI)
            "process_group": {"size": world, "backend": dist.get_backend() if world > 1 else None,
                              "packed_bytes_per_rank_per_step": gather.slot_bytes if (gather is not None and world > 1)
                              else None},
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (device Philox spawns / scripted policy / random RL policy)",
            "config": {"workload": cfg["workload"], "scenario": cfg["scenario"], "envs_per_gpu": E,
                       "global_envs": world * E, "agents": N, "rl_agents": K, "grid": [env.H, env.W],
                       "fear": cfg["fear"], "parallelism": f"env-sharded dp{world}", "obs_dtype": args.obs_dtype},
            "roofline": {"bound": dom_bound, "kernel": dom, "achieved": achieved, "peak": peak_u,
                         "unit": "TFLOP/s" if mfma else "GB/s", "frac": achieved / peak_u if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src, "frac_rocprof": prof_frac,
                         "bytes_per_launch": None if mfma else bytes_per_launch,
                         "flops_per_launch": bytes_per_launch if mfma else None,
                         # achieved = the algorithmic work per launch / avg_launch_ms, the kernel's busy
                         # time per launch (see busy_ms); avg_launch_span_ms = the launches' own mean
                         # duration, which overlapping writers stretch (the per-span figure beside it
                         # is the lower, per-launch view)
                         "avg_launch_ms": dur, "avg_launch_span_ms": span,
                         # the busy time per launch as profiled (uncapped) and the cap applied to it
                         "avg_launch_busy_profiled_ms": dur_profiled, "avg_launch_cap_timed_ms": dur_cap,
                         "busy_capped_by_timed_step": dur_profiled > dur_cap,
                         # the dominant kernel's work per step over the whole timed step: a lower
                         # bound of its rate (its busy time per step is at most the step)
                         "frac_timed_step_bound": (bytes_per_launch * dom_lps / (timed_ms * 1e-3) /
                                                   (1e12 if mfma else 1e9) / peak_u) if bytes_per_launch else None,
                         "frac_per_launch_span": (bytes_per_launch / (span * 1e-3) / (1e12 if mfma else 1e9) / peak_u
                                                  if (span and span > 0 and bytes_per_launch) else None),
                         "launches_profiled": busy[1 if dom in ("obs_kernel", "step_obs") else
                                                   next((k for k, n in SPAN_KINDS.items() if n == dom), 0)][1],
                         # every algorithmic byte of a whole step (state + obs) over the wall time
                         # per step: what the pipelined steps sustain end to end
                         "step_level_GBps": (step_b + obs_b) * E / (t_max / args.steps) / 1e9,
                         # with an obs ring the writers of consecutive steps overlap on two streams
                         # (DESIGN §5.4), so a launch's duration spans two writers' shared bandwidth:
                         # the dominant kernel's bytes per launch over the launch PERIOD (= the
                         # stream time per step) is its sustained rate
                         "writers_overlap": n_ring > 1 and bool(obs_mode) and env.kernel_path == "defer",
                         "achieved_per_period": (bytes_per_launch / (gpu_ms / args.steps * 1e-3) /
                                                 (1e12 if mfma else 1e9)) if bytes_per_launch else None,
                         "frac_per_period": (bytes_per_launch / (gpu_ms / args.steps * 1e-3) / (1e12 if mfma else 1e9) /
                                             peak_u) if bytes_per_launch else None,
                         # every profiled kernel kind: busy time per step and its own roofline
                         "kernels": per_kind},
            "kernels_ms": {"profiled_steps": nprof, "step_kernel": avg_step_ms, "obs_kernel": avg_obs_ms, "fear_kernel": avg_fear_ms,
                           "kernel_path": env.kernel_path,
                           "stream_ms_per_step": gpu_ms / args.steps,
                           "obs_async": obs_mode, "fear_async": env.fear_async,
                           "graph_steps": graph_n, "obs_ring": n_ring,
                           "host_enqueue_ms_per_step": t_enq * 1e3 / args.steps,
                           "host_first_steps_us": [round(x, 1) for x in t_first],
                           "spans_from": f"{n_prof} eager steps after the timed region"},
            "last_step_episodes": {"completed": stats[1], "mean_return": stats[0] / max(stats[1], 1.0),
                         "mean_len": stats[6] / max(stats[1], 1.0)},
            # completed-episode returns all-gathered every step (warmup + timed steps, all ranks)
            "return_gather": gathered,
            # FeAR's integer work: the counterfactual world updates the FeAR kernels ran
            # per step (gw_count_sims over the profiled steps, after the exact de-duplication of
            # DESIGN §5.2) and the reference's nominal K (N - 1) 18 per env-step, per second at the
            # timed step time, all ranks
            "fear_sims": None if sims is None else {
                "per_step": sims, "per_s": world * sims / (t_max / args.steps),
                "ref_equiv_per_step": E * K * (N - 1) * 18,
                "ref_equiv_per_s": world * E * K * (N - 1) * 18 / (t_max / args.steps),
                "dedup_factor": E * K * (N - 1) * 18 / sims if sims else None,
                "unit": "world updates (custom/Responsibility.py:16-54 UpdateGWorld counterfactuals)"},
        }
        rf = line["roofline"]
        if dom == "act_kernel":
            rf["precision"] = ACT_PRECISION
        if dom_bound == "valu" and dom in per_kind and per_kind[dom].get("achieved"):
            # an integer-VALU kernel leads (c5patch: FeAR with the windows in its launch): its
            # instruction rate against the VALU issue peak, as in roofline.kernels
            pk = per_kind[dom]
            rf.update(achieved=pk["achieved"], peak=VALU_PEAK_GIPS, unit="G inst/s", frac=pk["frac"],
                      peak_basis=VALU_PEAK_BASIS,
                      bytes_per_launch=None, frac_rocprof=None, frac_per_launch_span=None,
                      achieved_per_period=None, frac_per_period=None)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
