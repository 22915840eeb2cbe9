"""Summarise GW_LEARN_STAMP block stamps of the descriptor learner (maddpg_ops.hip DSTAMP).

usage: python tools/learn_stamps.py <stamp file> [skip updates]
Per launch (critic tail, critic grads, actor tail, actor grads): the median over updates of the
launch's span and, per block type, of each stamp's offset from the launch's first block start
(wall_clock64 ticks, 100 MHz)."""
import struct
import sys
from collections import defaultdict

import numpy as np

NAMES = ["dcritic_tail", "dgrads_adam(critic)", "dactor_tail", "dgrads_adam(actor)"]
TICK_US = 0.01
NS = 16  # stamps per block (slot 15: the block type)
TAIL_ORDER = {0: [0, 11, 14, 12, 13, 1, 6, 7, 8, 2, 9, 10, 3, 4, 5], 2: [0, 1, 2, 6, 7, 8, 9, 3, 10, 11, 4, 5]}


def read(path):
    ups, cur = [], {}
    with open(path, "rb") as f:
        data = f.read()
    o = 0
    while o + 8 <= len(data):
        l, nb = struct.unpack_from("<ii", data, o)
        o += 8
        a = np.frombuffer(data, dtype=np.uint64, count=nb * NS, offset=o).reshape(nb, NS).astype(np.int64)
        o += nb * NS * 8
        cur[l] = a
        if l == 3:
            ups.append(cur)
            cur = {}
    return ups


def main():
    ups = read(sys.argv[1])
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ups = ups[skip:]
    print(f"{len(ups)} updates")
    gaps = []
    for u in ups:
        ends = [u[l][:, 5].max() if l in (0, 2) else u[l][:, 2].max() for l in range(4)]
        starts = [u[l][:, 0].min() for l in range(4)]
        gaps.append([(starts[l + 1] - ends[l]) * TICK_US for l in range(3)] + [(ends[3] - starts[0]) * TICK_US])
    g = np.median(np.array(gaps), axis=0)
    print(f"gaps between launches (us): {g[0]:.2f} {g[1]:.2f} {g[2]:.2f}; update span {g[3]:.2f} us")
    for l in range(4):
        tail = l in (0, 2)
        span, per = [], defaultdict(list)
        for u in ups:
            a = u[l]
            t0 = a[:, 0].min()
            end_slot = 5 if tail else 2
            span.append((a[:, end_slot].max() - t0) * TICK_US)
            types = np.zeros(len(a), dtype=np.int64) if tail else a[:, 15]
            for ty in np.unique(types):
                sel = a[types == ty]
                slots = TAIL_ORDER[l] if tail else ([0, 5, 6, 3, 1, 2] if ty == 0 else [0, 3, 4, 5, 2] if ty == 1 else [0, 2])
                per[int(ty)].append([np.median((sel[:, s] - t0)) * TICK_US for s in slots] +
                                    [np.max(sel[:, end_slot] - t0) * TICK_US, len(sel)])
        print(f"{NAMES[l]}: span {np.median(span):.2f} us")
        for ty, rows in sorted(per.items()):
            r = np.median(np.array(rows), axis=0)
            print(f"   type {ty} ({int(r[-1])} blocks): median stamps " + " ".join(f"{x:.2f}" for x in r[:-2]) +
                  f" | last end {r[-2]:.2f}")
        # the slowest block of the last update, all its stamps
        a = ups[-1][l]
        end_slot = 5 if tail else 2
        i = int(np.argmax(a[:, end_slot]))
        t0 = a[:, 0].min()
        order = TAIL_ORDER[l] if tail else [0, 5, 6, 3, 1, 2]
        print(f"   slowest block {i} (type {a[i, 15] if not tail else 0}): " +
              " ".join(f"{(a[i, s] - t0) * TICK_US:.2f}" for s in order))


if __name__ == "__main__":
    main()
