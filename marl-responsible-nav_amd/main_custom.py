"""MADDPG training on the HIP grid world: ``main_custom.py`` (custom-env branch) + ``MADDPGAgent.train``
(maddpg/agent.py:77-252), batched over ``--envs`` envs (in total, sharded over the ranks).

    python marl-responsible-nav_amd/main_custom.py --config marl-responsible-nav_amd/configs/custom_fear_5.yaml \
        --scenario level3 --envs 1024 --iters 50 --updates-per-step 4 --save run.safetensors
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        marl-responsible-nav_amd/main_custom.py --envs 524288 ...       (one rank per GPU, RCCL)

With several ranks every rank steps its contiguous shard of the global envs, acts with the same
(broadcast) weights and learns data-parallel (marlnav/maddpg.py: one gradient all-reduce per
backward); rank 0 prints and saves.

Each iteration advances every env by TRAIN_STEPS steps (episodes auto-reset in the kernel) and
prints the completed-episode statistics and the latest loss, as the reference's tqdm loop does
per episode.  Checkpoints are safetensors (``MADDPG.save``)."""
import argparse
import os
import sys

import yaml

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs",
                                                     "custom_fear_5.yaml"))
    ap.add_argument("--scenario", default="level3")
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--updates-per-step", type=int, default=None,
                    help="MADDPG updates per env step (default: the reference rule, E // LEARN_STEP)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--save", default=None)
    args = ap.parse_args(argv)
    with open(args.config) as f:
        hp = yaml.safe_load(f)

    import torch
    from marlnav.maddpg import MADDPG
    from marlnav.parallel import init_from_env, shard
    from marlnav.train import MADDPGTrainer
    from marlnav.vec_env import VecGridEnv

    rank, world, local = init_from_env()
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    torch.manual_seed(hp["SEED"])
    torch.cuda.manual_seed(hp["SEED"] + rank)  # each rank samples its own replay batches
    offset, count = shard(args.envs, rank, world)
    env = VecGridEnv(args.scenario, num_envs=count, fear=hp["WITH_FEAR"], fear_weight=hp["FeAR_weight"],
                     max_steps=hp["TRAIN_STEPS"], seed=hp["SEED"], env_offset=offset, stats=True, final_obs=True)
    m = MADDPG(env.K, env.H, env.W, arch=hp["ARCH"], lr_actor=hp["LR_ACTOR"], lr_critic=hp["LR_CRITIC"],
               gamma=hp["GAMMA"], tau=hp["TAU"], batch_size=hp["BATCH_SIZE"], learn_step=hp["LEARN_STEP"],
               device=env.device, seed=hp["SEED"], capturable=not args.no_graph)
    tr = MADDPGTrainer(env, m, memory_size=hp["MEMORY_SIZE"], updates_per_step=args.updates_per_step,
                       graph=False if args.no_graph else "launches", seed=hp["SEED"])
    tr.reset()
    for it in range(args.iters):
        s = tr.train(hp["TRAIN_STEPS"])  # the statistics are all-reduced over the ranks
        if rank == 0:
            print(f"iter {it}: env_steps {s['env_steps'] * world} updates {s['updates']} episodes {s['episodes']:.0f} "
                  f"return {s['mean_return']:.3f} len {s['mean_len']:.1f} fear {s['fear']:.3f} "
                  f"crashes {s['crashes']:.0f} apples {s['apples']:.0f} loss {tr.total_loss():.4f}", flush=True)
    if args.save and rank == 0:
        m.save(args.save)
    env.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
