"""bench.py's multi-rank launcher on CPU: `--gpus N` (2 and 8) without a torch.distributed environment
starts the ranks itself (a child torch.distributed.run), the ranks exchange over gloo, and the one
relayed JSON line reports the world the driver asked for, with every replica bit-identical (VERDICT r03
item 5, r04 item 4).  Also the line's self-description: the CPU-share evidence and the committed
profile the traffic figure is read from."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("gpus", [2, 8])
def test_bench_launches_its_own_ranks_gloo(gpus):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "gloo",
                          "--n-gaussians", "20000", "--steps", "2", "--warmup", "1"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == gpus
    assert rec["config"]["parallelism"] == f"view-dp{gpus}"
    ex = rec["exchange"]
    assert ex["world"] == gpus and ex["collectives_per_step"] > 0
    assert ex["grad_bytes_per_rank"] == 20000 * 59 * 4 and ex["algbw_GBps"] > 0
    assert ex["replicas_bit_identical"] is True
    bx = rec["exchange_bf16"]
    assert bx["wire_bytes_per_rank"] * 2 == bx["grad_bytes_per_rank"] and bx["collectives_per_step"] > 0
    assert bx["replicas_bit_identical"] is True
    assert rec["value"] is None  # the headline stays unmeasured


def test_cpu_share_reports_its_evidence():
    share = bench.cpu_share()
    assert share["cores"] >= 1 and share["sched_getaffinity"] >= share["cores"]
    assert share["cores_source"] and "cgroup_cpu_setting" in share and share["host_cpu_count"] == os.cpu_count()
    if share["cgroup_cpu_quota"] is not None:
        assert share["cores"] <= share["cgroup_cpu_quota"]


def test_traffic_profile_key_resolves():
    """The committed PMC summary holds the bench's dominant kernels at the bench's own grid (ADVICE r04:
    a scout-count change once left segment_sort's key unresolved), and it says where it was taken."""
    table = json.load(open(bench.TRAFFIC_FILE))
    K, T = 8586682, 8160  # the bench view (BENCH_r04)
    for dom in ("radix_scatter_u64", "segment_sort"):
        key, ent = bench.traffic_entry(dom, K, T, table)
        assert key == {"radix_scatter_u64": "radix_scatter_kernel@1073664",
                       "segment_sort": f"segment_sort_kernel@{(T + bench.SCOUTS) * 256}"}[dom]
        assert ent["hbm_bytes_per_launch"] > 0
    meta = json.load(open(bench.TRAFFIC_META))
    assert meta["commit"] and len(meta["sources_sha256"]) == 64
    src = open(os.path.join(ROOT, "hidegs_amd", "csrc", "primitives.hip")).read()
    assert f"#define HIDEGS_SCOUTS {bench.SCOUTS} " in src
