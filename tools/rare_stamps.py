"""Summarise GW_RARE_STAMP block stamps of the window CNN's rare kernel (actor_ops.hip RSTAMP):
per launch, median over blocks of each stamp's offset from the launch's first block start.
usage: python tools/rare_stamps.py <file> [blocks per launch (512)]"""
import sys

import numpy as np

nb = int(sys.argv[2]) if len(sys.argv) > 2 else 512
a = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64).reshape(-1, nb, 8)
a = a[2:]  # skip the first launches
names = ["start", "unit offsets", "staged", "inputs", "mfma", "end"]
rows = []
for L in a:
    t0 = L[:, 0].min()
    rows.append([np.median(L[:, i] - t0) * 0.01 for i in range(6)] + [(L[:, 5].max() - t0) * 0.01,
                                                                        np.mean(L[:, 6])])
r = np.median(np.array(rows), axis=0)
print(f"{len(a)} launches: " + "  ".join(f"{n} {v:.2f}" for n, v in zip(names, r[:6])) +
      f"  | span {r[6]:.2f} us, units per block {r[7]:.2f}")
st = np.array([np.sort((L[:, 0] - L[:, 0].min()) * 0.01) for L in a])
print("block start percentiles (us): " + " ".join(f"p{q}={np.median(np.percentile(st, q, axis=1)):.2f}" for q in (10, 25, 50, 75, 90, 100)))
