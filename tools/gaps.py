"""Gaps between the pipelined kernels of a C3-style step in a rocprofv3 kernel trace (us):
obs(t-1) end -> obs(t) start (same queue), obs(t-1) end -> step_v2(t+1) start (cross-queue
WAR wait), step_v2(t) end -> fear_v2(t) start, and the period per step.
    python tools/gaps.py run_kernel_trace.csv [last_n_steps]"""
import csv
import statistics as S
import sys


def main(path, n=300):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))

    def ks(sub):
        return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if sub in r["Kernel_Name"]]
    o, s, f = ks("obs_kernel")[-n:], ks("step_v2")[-n:], ks("fear_v2")[-n:]

    def q(v):
        v = sorted(v)
        return f"p10 {v[len(v) // 10]:.1f} p50 {S.median(v):.1f} p90 {v[9 * len(v) // 10]:.1f} mean {S.mean(v):.1f}"
    print("obs duration          ", q([(b - a) / 1e3 for a, b in o]))
    print("obs->obs gap          ", q([(o[i + 1][0] - o[i][1]) / 1e3 for i in range(len(o) - 1)]))
    if s and len(s) == len(o):
        print("obs(t-1)->step(t+1)   ", q([(s[i + 1][0] - o[i - 1][1]) / 1e3 for i in range(1, len(o) - 1)]))
    if f and len(f) == len(s):
        print("step(t)->fear(t)      ", q([(f[i][0] - s[i][1]) / 1e3 for i in range(len(f))]))
        print("fear(t)->step(t+1)    ", q([(s[i + 1][0] - f[i][1]) / 1e3 for i in range(len(f) - 1)]))
    print(f"period {(o[-1][1] - o[0][0]) / 1e3 / len(o):.1f} us/step over {len(o)} steps")


if __name__ == "__main__":
    main(sys.argv[1], *map(int, sys.argv[2:3]))
