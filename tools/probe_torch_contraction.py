"""Which of PyTorch's ROCm pointwise kernels contract a*b+c into one fma?  (Fixes the op-by-op
arithmetic the fused masked-Adam kernel must reproduce to match OurAdam's torch ops bit for bit.)"""
import torch

torch.manual_seed(0)
n = 1 << 20
dev = "cuda"
a = torch.randn(n, device=dev)
b = torch.randn(n, device=dev) * 1e-3
c = torch.rand(n, device=dev) + 0.5
alpha = 0.09999999999999998  # python float like 1 - beta1
al32 = torch.tensor(alpha, dtype=torch.float32).item()


def f32(x):
    return x.to(torch.float32)


def report(name, got, fused, unfused):
    print(f"{name:10s} fused={torch.equal(got, fused)} unfused={torch.equal(got, unfused)} "
          f"fused_mismatch={(got != fused).sum().item()} unfused_mismatch={(got != unfused).sum().item()}")


# add_(b, alpha): a + alpha*b
got = a.clone().add_(b, alpha=alpha)
fused = f32(a.double() + al32 * b.double())
unfused = a + f32(al32 * b.double())
report("add_alpha", got, fused, unfused)
# addcmul_(b, b, value): a + value*b*b
got = a.clone().addcmul_(b, b, value=alpha)
vb = f32(al32 * b.double())  # (value*t1) rounded
fused = f32(a.double() + vb.double() * b.double())
unfused = a + f32(vb.double() * b.double())
report("addcmul", got, fused, unfused)
# addcdiv_(b, c, value): a + value*(b/c)
q = b / c
got = a.clone().addcdiv_(b, c, value=-alpha)
fused = f32(a.double() + (-al32) * q.double())
unfused = a + f32((-al32) * q.double())
report("addcdiv", got, fused, unfused)
# div by python scalar: reciprocal-multiply or true division?
s = 0.97234567891
got = c / s
recip = c * torch.tensor(1.0, dtype=torch.float32) / torch.tensor(s, dtype=torch.float32)
inv = f32(torch.tensor(1.0, dtype=torch.float64) / torch.tensor(float(torch.tensor(s, dtype=torch.float32)), dtype=torch.float64))
by_recip = f32(c.double() * inv.double())
by_div = f32(c.double() / torch.tensor(s, dtype=torch.float32).double())
print(f"div_scalar recip={torch.equal(got, by_recip)} true_div={torch.equal(got, by_div)} "
      f"recip_mismatch={(got != by_recip).sum().item()} div_mismatch={(got != by_div).sum().item()}")
# sqrt correctly rounded?
v = torch.rand(n, device=dev)
print("sqrt_cr", torch.equal(v.sqrt(), f32(v.double().sqrt())), (v.sqrt() != f32(v.double().sqrt())).sum().item())
# mul by scalar
print("mul_scalar", torch.equal(a * 0.9, f32(a.double() * float(torch.tensor(0.9, dtype=torch.float32)))))
# add scalar eps
e = 1e-15
print("add_eps", torch.equal(c + e, f32(c.double() + float(torch.tensor(e, dtype=torch.float32)))))
