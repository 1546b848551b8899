"""Division of an fp32 tensor by a Python scalar in PyTorch ROCm: a * f32(1.0 / s) (double reciprocal).

Found while matching OurAdam bit for bit (hidegs_amd/csrc/adam.hip); see tools/probe_torch_contraction.py."""
import math, numpy as np, torch
torch.manual_seed(0)
c = torch.rand(1 << 20, device="cuda") + 0.5
res = {"f32(1/f32(s))": 0, "f32(1/s)": 0, "true_div_f32s": 0, "true_div_f64s": 0}
for k in range(200):
    s = 0.5 + k * 0.00731
    got = c / s
    cands = {"f32(1/f32(s))": (c.double() * float(np.float32(1.0) / np.float32(s))).float(),
             "f32(1/s)": (c.double() * float(np.float32(1.0 / s))).float(),
             "true_div_f32s": (c.double() / float(np.float32(s))).float(),
             "true_div_f64s": (c.double() / s).float()}
    for name, emu in cands.items():
        res[name] += int((got != emu).sum().item() > 0)
print("scalars (of 200) where torch's c / s differs from each candidate:", res)
b2s = math.sqrt(1 - 0.999 ** 6.0)
x = torch.tensor(np.array([1113496192] * 8, dtype=np.uint32).view(np.float32), device="cuda")
print("case x/b2s", (x / b2s).cpu().numpy().view(np.uint32)[0], "x*f32(1/b2s)", (x.double() * float(np.float32(1.0 / b2s))).float().cpu().numpy().view(np.uint32)[0])
