"""Diagnostic: flat GPU learner vs the per-agent fp32 loop (tests/test_maddpg.py), per iteration,
with the HIP epilogue on/off (GW_LN_FUSED)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-responsible-nav_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from test_maddpg import PerAgentReference, _seq  # noqa: E402
from marlnav.maddpg import MADDPG  # noqa: E402

torch.manual_seed(0)
K, H, W, B, steps, lr = 2, 32, 32, 128, 4, 1e-3
m = MADDPG(K, H, W, lr_actor=lr, lr_critic=lr, gamma=0.98, tau=0.01, batch_size=B, device="cuda", seed=3)
with torch.no_grad():
    for net in (m.actor_targets.net, m.critic_targets):
        net.flat_params().add_(0.05 * torch.randn_like(net.flat_params()))
ref = PerAgentReference(m, lr, lr)
g = torch.Generator(device="cuda").manual_seed(1)
for it in range(steps):
    states = torch.randint(-1, 6, (K, B, H, W), generator=g, device="cuda").float()
    next_states = torch.randint(-1, 6, (K, B, H, W), generator=g, device="cuda").float()
    actions = torch.softmax(torch.randn((K, B, 9), generator=g, device="cuda"), -1)
    rewards = torch.randn((B, K), generator=g, dtype=torch.float64, device="cuda") * 10
    dones = (torch.rand((B, K), generator=g, device="cuda") < 0.2).to(torch.uint8)
    u_next = torch.rand((K, B, 9), generator=g, device="cuda")
    u_cur = torch.rand((K, B, 9), generator=g, device="cuda")
    a_loss, c_loss = m.learn(states, actions, rewards, next_states, dones, u_next, u_cur)
    want = ref.learn(states, actions, rewards, next_states, dones, u_next, u_cur)
    print(it, [(a_loss[k].item() - want[k][0], c_loss[k].item() - want[k][1], want[k][0], want[k][1]) for k in range(K)])
    for name, stacked, seqs in (("actor", m.actors.net, ref.actors), ("critic", m.critics, ref.critics)):
        rels = []
        for a, b in zip(_seq(stacked, 0).parameters(), seqs[0].parameters()):
            rels.append(float((a - b).norm() / b.norm().clamp_min(1e-12)))
        print("   ", name, ["%.1e" % r for r in rels])
