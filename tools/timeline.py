"""Per-step kernel timeline from a rocprofv3 kernel trace CSV (start/end relative to the step's
first kernel, in us), to see which launches overlap and what sits on the critical path.
    python tools/timeline.py run_kernel_trace.csv [first_kernel_substring] [n_steps]"""
import csv
import sys


def main(path, anchor="step_v2", nsteps=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    mid = starts[len(starts) // 2: len(starts) // 2 + nsteps + 1]
    for a, b in zip(mid, mid[1:]):
        t0 = int(rows[a]["Start_Timestamp"])
        print(f"--- step (period {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us)")
        for r in rows[a:b]:
            s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
            print(f"  q{r['Queue_Id']:>2} {s:8.1f} -> {e:8.1f} ({e - s:7.1f})  {r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or ["step_v2"]), *(map(int, sys.argv[3:4]) if len(sys.argv) > 3 else []))
