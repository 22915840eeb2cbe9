"""profiles/<tag>/summary.json -> profiles/latest.json["configs"][CONFIG]: per-launch HBM bytes and
rocprofv3 busy time per launch of each kernel kind, which bench.py reports as roofline.traffic /
frac_rocprof when it runs the same config.  Other configs' entries are kept."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# rocprofv3 kernel name (namespace stripped, before the template arguments) -> bench.py's SPAN_KINDS name
KIND = {"gw::obs_kernel": "obs_kernel", "gw::step_v2": "step_kernel", "gw::fear_v2": "fear_kernel", "gw::fear_rows_kernel": "fear_kernel",
        "gw::step_obs": "step_obs", "act_kernel": "act_kernel", "window_kernel": "window_kernel",
        "wcnn_rare_kernel": "cnn_rare_kernel", "cnn_rare_kernel": "cnn_rare_kernel",
        "wcnn_l1_kernel": "cnn_l1_kernel", "cnn_l1_kernel": "cnn_l1_kernel",
        "window_rows_kernel": "window_kernel", "rows_list_kernel": "window_kernel", "wcnn_list_kernel": "cnn_l1_kernel",
        # the descriptor learner: one update = dcritic_tail + dgrads_adam x 2 + dactor_tail
        "dcritic_tail": "learn_update", "dactor_tail": "learn_update", "dgrads_adam": "learn_update"}
# kinds made of several kernels: per launch of the first kernel (one per update), the kernels' time summed
MULTI = {"learn_update": "dcritic_tail"}


STEP_KERNELS = ("gw::step_v2", "gw::step_obs", "gw::step_kernel_fear", "gw::step_kernel_nofear")


def main(tag, config, cmd=None):
    s = json.load(open(os.path.join(ROOT, "profiles", tag, "summary.json")))
    # steps in the traced run: the world-update kernel runs once per step
    steps = max((v["calls"] for n, v in s.items() if n.split("<")[0].strip() in STEP_KERNELS), default=0) or None
    kernels = {}
    for kind, lead in MULTI.items():
        parts = {n: v for n, v in s.items() if KIND.get(n.split("<")[0].strip()) == kind}
        lv = next((v for n, v in parts.items() if lead in n), None)
        if lv and lv.get("calls"):
            tot_us = sum(v["avg_us"] * v["calls"] for v in parts.values())
            busy = sum((v.get("busy_us") or v["avg_us"]) * v["calls"] for v in parts.values())
            k = {"avg_us": tot_us / lv["calls"], "calls": lv["calls"], "busy_us": busy / lv["calls"],
                 "kernels": sorted(parts)}
            kernels[kind] = k
    for name, v in s.items():
        kind = KIND.get(name.split("<")[0].strip())
        if kind in MULTI:
            continue
        if kind in kernels and (kernels[kind].get("calls") or 0) >= (v.get("calls") or 0):
            continue  # a kind with several kernels (a few launches of another form): the most called
        if kind and (v.get("hbm_mb") is not None or v.get("busy_us") or v.get("valu_insts")):
            k = {"avg_us": v["avg_us"], "calls": v.get("calls")}
            if v.get("hbm_mb") is not None:
                k["hbm_bytes_per_launch"] = v["hbm_mb"] * 1e6
            if v.get("busy_us"):
                k["busy_us"] = v["busy_us"]  # union of the launches' intervals / launches
            if steps:  # per step (a kernel may run as several launches per step: the chunked writer)
                k["launches_per_step"] = v["calls"] / steps
                if v.get("busy_us"):
                    k["busy_us_per_step"] = v["busy_us"] * v["calls"] / steps
                if v.get("hbm_mb") is not None:
                    k["hbm_bytes_per_step"] = v["hbm_mb"] * 1e6 * v["calls"] / steps
            if v.get("valu_insts"):
                k["valu_insts_per_launch"] = v["valu_insts"]
                if steps:
                    k["valu_insts_per_step"] = v["valu_insts"] * v["calls"] / steps
            kernels[kind] = k
    cmd = cmd or f"python bench.py --config {config}"
    path = os.path.join(ROOT, "profiles", "latest.json")
    try:
        out = json.load(open(path))
    except (OSError, ValueError):
        out = {}
    if "configs" not in out:  # round-3 layout (one config at the top level)
        old = {k: out[k] for k in ("source", "config", "kernels") if k in out}
        out = {"configs": {old["config"]: {"source": old["source"], "kernels": old["kernels"]}} if old else {}}
    out["configs"][config] = {
        "source": f"profiles/{tag} (rocprofv3 --kernel-trace --stats, --pmc FETCH_SIZE / WRITE_SIZE and SQ_INSTS_VALU passes of "
                  f"`{cmd}`; FETCH_SIZE x2 per MI355X_MICROARCH.md; busy_us = the union of the launches' "
                  f"intervals in the kernel trace / launches)",
        "kernels": kernels}
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out["configs"][config], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "c3", sys.argv[3] if len(sys.argv) > 3 else None)
