"""Golden fixture: the actor weights of the reference's shipped single-agent checkpoints
(/root/reference/models/custom/single/level3/**/*.pt, agilerl 1.0.15 MADDPG saves),
read WITHOUT unpickling by marlnav/checkpoint.py (pickletools opcodes replayed into inert
records, raw little-endian f32 storages from the zip), written to tests/golden/ckpt_actors.npz:

    <tag>/feature_net.<layer>.<weight|bias>   f32 arrays in the checkpoint's (out, in) layout
    <tag>/meta_steps                          the checkpoint's `steps` entry (training env steps)

so that the GPU box (where /root/reference does not exist) evaluates the trained policies.
Run here: python tests/golden/make_golden_checkpoint.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "marl-responsible-nav_amd"))

from marlnav import checkpoint as ck  # noqa: E402

REF = "/root/reference/models/custom/single/level3"
CKPTS = {"level3_fear_4k": "fear/Single_MADDPG_4k.pt", "level3_wofear": "wo_fear/Single_MADDPG.pt"}
NAMES = ["linear_layer_0", "layer_norm_0", "linear_layer_1", "layer_norm_1", "linear_layer_output"]


def main():
    out = {}
    for tag, rel in CKPTS.items():
        c = ck.read_checkpoint(os.path.join(REF, rel))
        sd = ck.state_dict_tensors(c["actors_state_dict"][0])
        for nm in NAMES:
            for p in ("weight", "bias"):
                key = f"feature_net.{nm}.{p}"
                out[f"{tag}/{key}"] = sd[key].astype(np.float32)
        out[f"{tag}/meta_steps"] = np.array(c.get("steps") or [0], dtype=np.int64)
        print(tag, {k.split('/')[1]: v.shape for k, v in out.items() if k.startswith(tag)})
    np.savez_compressed(os.path.join(HERE, "ckpt_actors.npz"), **out)


if __name__ == "__main__":
    main()
