"""Timeline of a short bench run from a rocprofv3 kernel trace (run_kernel_trace.csv): where the
driver-size run's time goes beyond the steady-state period (pipeline fill, drain, host gaps).

Usage: python tools/run_span.py <run_kernel_trace.csv> [timed_steps]
Splits the trace at its largest idle gap after the first 10% of kernels (the synchronize that
opens the timed region), then prints, for the kernels after it: the first start, the obs-writer
launches' starts / ends, the steady period (median writer start-to-start), and the excess of the
span over timed_steps x period, attributed to the head (first start -> first writer start) and the
tail (last writer start -> last end)."""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    lo = max(1, len(rows) // 10)
    gaps = [(rows[i][0] - max(e for _, e, _ in rows[:i]), i) for i in range(lo, len(rows))]
    gap, cut = max(gaps)
    tail = rows[cut:]
    t0 = tail[0][0]
    writers = [(s, e) for s, e, n in tail if "obs_kernel" in n or "step_obs" in n]
    print(f"split at kernel {cut} of {len(rows)} after an idle gap of {gap / 1e3:.1f} us")
    if not writers:
        print("no obs writer launches after the split")
        return
    starts = [s for s, _ in writers]
    period = statistics.median([b - a for a, b in zip(starts, starts[1:])]) if len(starts) > 1 else 0
    end = max(e for _, e, _ in tail)
    span = end - t0
    print(f"kernels after the split: {len(tail)}, writer launches: {len(writers)}")
    print(f"span first start -> last end: {span / 1e3:.1f} us; steady writer period {period / 1e3:.1f} us; "
          f"{steps} x period = {steps * period / 1e3:.1f} us; excess {(span - steps * period) / 1e3:.1f} us")
    print(f"head: first kernel -> first writer start {(starts[0] - t0) / 1e3:.1f} us")
    print(f"tail: last writer start -> last kernel end {(end - starts[-1]) / 1e3:.1f} us "
          f"(last writer lasts {(writers[-1][1] - writers[-1][0]) / 1e3:.1f} us)")
    print("first kernels after the split:")
    for s, e, n in tail[:8]:
        print(f"  {(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f} us  {n[:70]}")
    print("last kernels:")
    for s, e, n in tail[-6:]:
        print(f"  {(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f} us  {n[:70]}")


if __name__ == "__main__":
    main()
