"""profiles/<tag>/summary.json -> profiles/latest.json (per-launch HBM bytes that bench.py reports as
roofline.traffic when it runs the same config)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KIND = {"gw::obs_kernel": "obs_kernel", "gw::step_v2": "step_kernel", "gw::fear_v2": "fear_kernel"}


def main(tag, config, cmd=None):
    s = json.load(open(os.path.join(ROOT, "profiles", tag, "summary.json")))
    kernels = {}
    for name, v in s.items():
        kind = KIND.get(name.split("<")[0].strip())
        if kind and v.get("hbm_mb") is not None:
            kernels[kind] = {"hbm_bytes_per_launch": v["hbm_mb"] * 1e6, "avg_us": v["avg_us"]}
            if v.get("busy_us"):
                kernels[kind]["busy_us"] = v["busy_us"]  # union of the launches' intervals / launches
    cmd = cmd or f"python bench.py --config {config}"
    out = {"source": f"profiles/{tag} (rocprofv3 --kernel-trace --stats and --pmc FETCH_SIZE / WRITE_SIZE passes of "
                     f"`{cmd}`; FETCH_SIZE x2 per MI355X_MICROARCH.md; busy_us = the union of the launches' "
                     f"intervals in the kernel trace / launches)",
           "config": config, "kernels": kernels}
    json.dump(out, open(os.path.join(ROOT, "profiles", "latest.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "c3", sys.argv[3] if len(sys.argv) > 3 else None)
