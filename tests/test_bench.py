"""bench.py's multi-rank launcher on CPU: `--gpus 2` without a torch.distributed environment starts
the two ranks itself (a child torch.distributed.run), the ranks exchange over gloo, and the one
relayed JSON line reports the world the driver asked for."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_launches_its_own_ranks_gloo():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                          "--n-gaussians", "20000", "--steps", "2", "--warmup", "1"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "view-dp2"
    ex = rec["exchange"]
    assert ex["world"] == 2 and ex["collectives_per_step"] > 0
    assert ex["grad_bytes_per_rank"] == 20000 * 59 * 4 and ex["algbw_GBps"] > 0
    bx = rec["exchange_bf16"]
    assert bx["wire_bytes_per_rank"] * 2 == bx["grad_bytes_per_rank"] and bx["collectives_per_step"] > 0
    assert rec["value"] is None  # the headline stays unmeasured
