"""One-line summary of a bench.py JSON line (the last line of a log).
    python tools/bench_line.py bench.log [label]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k, r = d["kernels_ms"], d["roofline"]
lab = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
print(f"{lab:>14}: {d['value'] / 1e9:.3f} G  {d['ms_per_step'] * 1e3:.1f} us/step  stream "
      f"{k['stream_ms_per_step'] * 1e3:.1f}  obs {k['obs_kernel'] * 1e3:.1f} step {k['step_kernel'] * 1e3:.1f} "
      f"fear {k['fear_kernel'] * 1e3:.1f} (n={k['profiled_steps']}, graph {k.get('graph_steps')}) "
      f"{r['kernel']} frac {r['frac'] if r['frac'] is None else round(r['frac'], 3)} "
      f"(span {r.get('frac_per_launch_span') and round(r['frac_per_launch_span'], 3)}, "
      f"period {r.get('frac_per_period') and round(r['frac_per_period'], 3)}) "
      f"host {k.get('host_enqueue_ms_per_step', 0) * 1e3:.1f} us/step")
kk = k.get("kernels") or r.get("kernels") or {}
if kk:
    print(" " * 16 + "  ".join(f"{n} {v['busy_ms_per_step'] * 1e3:.1f}us" + (f" ({v['frac']:.3f} {v['bound']})" if v.get('frac') else "")
                                for n, v in sorted(kk.items(), key=lambda x: -x[1]['busy_ms_per_step'])))
