"""Debug: merged async graph replay vs eager over several replays."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd")]
os.environ["GW_KERNEL"] = "merged"
import torch  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402

E, n = 64, 2
envs = []
for i in range(2):
    env = VecGridEnv("grid32", num_envs=E, fear=False, max_steps=12, seed=5, stats=True)
    if i == 1:
        env.set_obs_async(True)
    env.reset()
    envs.append(env)
a, b = envs
snaps = []
for _ in range(3):
    a.step(); b.step(); snaps.append(a.out["obs"].clone())
g = b.capture_steps(n)
for rep in range(3):
    for _ in range(n):
        a.step(); snaps.append(a.out["obs"].clone())
    g.replay()
    torch.cuda.synchronize()
    pre = [i + 1 for i, s in enumerate(snaps) if torch.equal(s, b.out["obs"])]
    b.obs_fence()
    torch.cuda.synchronize()
    post = [i + 1 for i, s in enumerate(snaps) if torch.equal(s, b.out["obs"])]
    sa, sb = a.state(), b.state()
    print("rep", rep, "steps", len(snaps), "pre", pre, "post", post,
          "t a/b", sa["t"][:4].tolist(), sb["t"][:4].tolist(), "pos eq", torch.equal(sa["pos"], sb["pos"]))
