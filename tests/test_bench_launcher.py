"""bench.py's multi-GPU launcher on CPU: `--gpus 2` without torch.distributed.run spawns two rank processes
(fresh interpreters, gloo in --dry-run), which shard the frames, time with a barrier + max over ranks and
print ONE JSON line from rank 0 with n_gpus = 2; a failing rank makes the parent exit non-zero."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True,
                          timeout=300, env=env, cwd="/tmp")


def test_two_rank_spawn_prints_one_line():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--batch", "3", "--height", "32",
              "--width", "48"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["warmup"] == 1
    assert line["config"]["frames_per_step"] == 6 and line["config"]["parallelism"].startswith("frame-sharded dp2")
    assert len(line["per_rank_fps"]) == 2
    # the ranks really were distinct processes with distinct LOCAL_RANKs, joined in one process group
    assert line["rccl_world"] == 2
    assert sorted(r["local_rank"] for r in line["ranks"]) == [0, 1]
    assert sorted(r["rank"] for r in line["ranks"]) == [0, 1]
    # value = all ranks' frames over the max-over-ranks time
    assert abs(line["value"] - 2 * 2 * 3 / line["max_over_ranks_s"]) / line["value"] < 0.01
    assert min(line["per_rank_fps"]) * 2 >= line["value"] * 0.99


def test_failing_rank_fails_the_parent():
    # an invalid shape makes every rank raise inside the worker: the parent must exit non-zero
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0", "--height", "0", "--width", "48"])
    assert r.returncode != 0
