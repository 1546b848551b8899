"""The view-DP exchange on a one-rank RCCL group with the N-rank path forced (every collective real):
per-transport time, for rocprofv3 --kernel-trace --stats.  python tools/exchange_time.py [N_GAUSSIANS]"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from hidegs_amd.view_dp import GradArena, ViewDPExchange  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
s = socket.socket()
s.bind(("127.0.0.1", 0))
os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(s.getsockname()[1])
s.close()
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
g = torch.Generator(device="cuda").manual_seed(0)
visible = torch.rand(n, device="cuda", generator=g) < 0.9
arena = GradArena(n, device="cuda")
arena.flat.normal_(generator=g)
for transport in ("fp32", "bf16"):
    ex = ViewDPExchange(transport=transport, force_collectives=True)
    for _ in range(3):
        ex.exchange(arena, visible)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ex.exchange(arena, visible)
    torch.cuda.synchronize()
    print(f"{transport}: {(time.perf_counter() - t0) * 100:.3f} ms per exchange, {ex.last.collectives} collectives",
          flush=True)
dist.destroy_process_group()
