"""bench.py contract pieces that need no GPU: the metric matches BASELINE.json, the byte
accounting behind roofline.achieved, the CLI parses."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_metric_is_baseline_metric():
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert bench.METRIC == json.load(f)["metric"]


def test_algorithmic_bytes():
    step_b, obs_b = bench.algorithmic_bytes(4, 2, 32 * 32)       # C3
    assert obs_b == 4 * 2 * 1024 + 20 and step_b == 205
    assert bench.algorithmic_bytes(4, 2, 1024, obs_bytes=2)[1] == 2 * 2 * 1024 + 20
    assert bench.algorithmic_bytes(8, 2, 64 * 64)[1] == 4 * 2 * 4096 + 20   # C4


def test_configs_name_the_baseline_workloads():
    assert {"c1", "c2", "c3", "c4", "c5"} <= set(bench.CONFIGS)
    c3 = bench.CONFIGS["c3"]
    assert c3["envs"] == 65536 and c3["scenario"] == "grid32" and c3["fear"]


def test_cli_help_without_gpu():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "--steps" in r.stdout and "--obs-dtype" in r.stdout


def test_launch_plan_one_rank_per_gpu():
    """`bench.py --gpus N` without a launcher starts N copies of itself with torchrun's variables
    (the plan only: nothing is started and no GPU is touched here)."""
    argv = ["--gpus", "4", "--steps", "20", "--warmup", "5"]
    plans = bench.launch_plan(4, argv, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29511)
    assert len(plans) == 4
    for r, (cmd, env) in enumerate(plans):
        assert cmd[0] == sys.executable and cmd[1] == os.path.join(REPO, "bench.py") and cmd[2:] == argv
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/bin"


def test_busy_time_merges_overlapping_launches():
    spans = [(1, 0.0, 1.4), (1, 1.0, 2.4), (0, 0.0, 0.2), (1, 2.0, 3.4), (1, 5.0, 6.0)]
    total, n = bench.busy_ms(spans, 1)
    assert n == 4 and abs(total - (3.4 + 1.0)) < 1e-12
    assert bench.busy_ms(spans, 0) == (0.2, 1)
    assert bench.busy_ms([], 1) == (0.0, 0)
