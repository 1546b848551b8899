"""Masked Adam step timing at the bench's shape (2M Gaussians x 59 floats, 90% visible) with the
library HIDEGS_LIB points at."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib  # noqa: E402
from hidegs_amd.optim import Adam  # noqa: E402

N = 2_000_000
widths = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
g = torch.Generator(device="cuda").manual_seed(100)
prm = {k: torch.nn.Parameter(torch.randn(N, w, device="cuda", generator=g)) for k, w in widths.items()}
for p in prm.values():
    p.grad = torch.randn(p.shape, device="cuda", generator=g)
vis = torch.rand(N, device="cuda", generator=g) < 0.9
opt = Adam([{"params": [prm[k]], "lr": 1e-3, "name": k} for k in widths], lr=0.0, eps=1e-15)
for _ in range(5):
    opt.step(vis)
torch.cuda.synchronize()
with _lib.kernel_timer() as kt:
    for _ in range(30):
        opt.step(vis)
    torch.cuda.synchronize()
    ms, n = kt.get("masked_adam")
nb = 28 * 59 * int(vis.sum()) + N
print(os.environ.get("HIDEGS_LIB", "default"), f"masked_adam {ms * 1e3 / n:.1f}us {nb / (ms / n * 1e-3) / 1e12:.2f} TB/s",
      flush=True)
