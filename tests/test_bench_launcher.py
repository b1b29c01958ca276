"""bench.py's launcher: `python bench.py --gpus N` starts N ranks itself
(torch.distributed.run, one process per GPU) when no launcher set WORLD_SIZE,
so the driver's N-GPU command measures N GPUs (VERDICT r02 missing item 1).
Runs on CPU with the gloo stub (`--stub`: the same rendezvous, barrier and
all-reduce path, no evaluation)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True, env=env,
                       timeout=240, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only prints
    return json.loads(lines[0])


def test_bench_launches_two_ranks_itself():
    out = _run(["--gpus", "2", "--stub", "--steps", "2", "--warmup", "1"])
    assert out["stub"] and out["n_gpus"] == 2
    assert out["rank_sum"] == 3.0  # ranks 0 and 1 both took part in the all-reduce


def test_bench_single_rank_does_not_launch():
    out = _run(["--gpus", "1", "--stub"])
    assert out["n_gpus"] == 1 and out["rank_sum"] == 1.0
