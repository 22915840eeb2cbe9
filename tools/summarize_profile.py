"""Summarise a tools/gpu_profile.sh run (rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes +
a SQ_INSTS_VALU / SQ_WAVES / SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE pass)
into profiles/<tag>/SUMMARY.md and copy the raw CSVs next to it.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced stream -> x2; WRITE_SIZE is exact for 16-B/lane stores.  Both are in KiB."""
import csv
import json
import os
import shutil
import sys


STEP_KERNELS = ("gw::step_v2", "gw::step_obs", "gw::step_kernel_fear", "gw::step_kernel_nofear")


def busy_per_launch(trace_csv, last_steps=64):
    """kernel short name -> (launches, union of their [start, end] intervals / launches in us):
    the busy time per launch bench.py reports as avg_launch_ms (overlapping launches of one
    kernel, e.g. obs writers of consecutive steps on two streams, counted once).  Only the
    launches of the last `last_steps` steps count (bench.py's profiled steps, after its timed
    region: warmup and the pipeline's fill are outside the window bench.py measures too)."""
    iv = {}
    for r in csv.DictReader(open(trace_csv)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        iv.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    steps = sorted(b for n, v in iv.items() if n.split("<")[0].strip() in STEP_KERNELS for b, _ in v)
    t0 = steps[-last_steps] if last_steps and len(steps) >= last_steps else None
    out = {}
    for name, v in iv.items():
        if t0 is not None:
            v = [x for x in v if x[0] >= t0] or v

        v.sort()
        total, cb, ce = 0, None, None
        for b, e in v:
            if ce is None or b > ce:
                if ce is not None:
                    total += ce - cb
                cb, ce = b, e
            else:
                ce = max(ce, e)
        total += ce - cb
        out[name] = (len(v), total / len(v) / 1e3)
    return out


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    trace = os.path.join(src, "trace", "run_kernel_trace.csv")
    busy = busy_per_launch(trace) if os.path.exists(trace) else {}
    pmc = {}
    for which, ctrs in (("fetch", ("FETCH_SIZE",)), ("write", ("WRITE_SIZE",)),
                        ("valu", ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"))):
        path = os.path.join(src, which, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] not in ctrs:
                continue
            pmc.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    lines = [f"# rocprofv3 summary ({os.path.basename(dst)})", "",
             "| kernel | calls | avg us | busy us / launch | min us | max us | % time | FETCH MB/launch (x2 corr.) | WRITE MB/launch | HBM MB/launch |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    out = {}
    for r in stats:
        name = r["Name"]
        p = pmc.get(name, {})
        f = p.get("FETCH_SIZE")
        w = p.get("WRITE_SIZE")
        fmb = (sum(f) / len(f)) * 1024 * 2 / 1e6 if f else None
        wmb = (sum(w) / len(w)) * 1024 / 1e6 if w else None
        tot = (fmb or 0) + (wmb or 0) if (f or w) else None
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        bz = busy.get(short, (0, None))[1]
        lines.append(f"| `{short}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                     f"{'' if bz is None else f'{bz:.2f}'} | {float(r['MinNs'])/1e3:.2f} | "
                     f"{float(r['MaxNs'])/1e3:.2f} | {float(r['Percentage']):.1f} | "
                     f"{'' if fmb is None else f'{fmb:.2f}'} | {'' if wmb is None else f'{wmb:.2f}'} | "
                     f"{'' if tot is None else f'{tot:.2f}'} |")
        out[short] = dict(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3, busy_us=bz, fetch_mb=fmb,
                          write_mb=wmb, hbm_mb=tot)
        vi = p.get("SQ_INSTS_VALU")
        if vi:  # wave-level vector instructions per launch; GRBM_GUI_ACTIVE summed over the 8 XCDs
            avg = lambda c: sum(p[c]) / len(p[c]) if p.get(c) else None  # noqa: E731
            out[short].update(valu_insts=avg("SQ_INSTS_VALU"), waves=avg("SQ_WAVES"), wave_cycles=avg("SQ_WAVE_CYCLES"),
                              gui_active=avg("GRBM_GUI_ACTIVE"))
            dur = bz or float(r["AverageNs"]) / 1e3
            rate = out[short]["valu_insts"] / (dur * 1e-6) / 1e9
            out[short]["valu_gips"] = rate
            out[short]["valu_frac"] = rate / (256 * 4 * 2.4e9 / 2 / 1e9)
            lines.append(f"|   VALU | {out[short]['valu_insts']:.4g} wave-instructions per launch, {rate:.1f} G/s over "
                         f"{dur:.2f} us = {out[short]['valu_frac']:.3f} of the 1,228.8 G/s issue peak; "
                         f"{out[short]['waves']:.0f} waves |  |  |  |  |  |  |  |  |")
    for log in ("trace.log", "fetch.log", "write.log", "valu.log"):
        p = os.path.join(src, log)
        if os.path.exists(p):
            for l in open(p):
                if l.startswith("{"):
                    j = json.loads(l)
                    lines += ["", f"bench line under `{log}`: value {j['value']:.4g} {j['unit']}, "
                              f"{j['ms_per_step']:.4f} ms/step, kernels_ms {j.get('kernels_ms')}"]
    open(os.path.join(dst, "SUMMARY.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    for sub in ("trace", "fetch", "write", "valu"):
        for fn in ("run_kernel_stats.csv", "run_counter_collection.csv"):
            p = os.path.join(src, sub, fn)
            if os.path.exists(p):
                shutil.copy(p, os.path.join(dst, f"{sub}_{fn}"))
    for log in ("trace.log", "fetch.log", "write.log", "valu.log"):
        p = os.path.join(src, log)
        if os.path.exists(p):
            with open(p) as fi, open(os.path.join(dst, log), "w") as fo:
                fo.writelines(l for l in fi if l.startswith("{"))
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
