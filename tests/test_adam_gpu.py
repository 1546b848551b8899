"""Fused masked Adam on the MI355X (hidegs_amd/csrc/adam.hip) -- bit-exact against
(a) the CPU oracle (oracle/adam_ref.c) and (b) the reference's op sequence, restated from
scene/OurAdam.py:249-337 and executed as the same torch ops on the same GPU.  Tolerance: none;
rows outside the mask must keep their bits."""
import math

import numpy as np
import pytest
import torch

import oracle
from hidegs_amd import _lib
from hidegs_amd.optim import Adam

pytestmark = pytest.mark.gpu

SHAPES = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}
LRS = {"xyz": 0.00016 * 4.2, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005,
       "rotation": 0.001}


def torch_reference_step(params, grads, state, relevant, lr, beta1=0.9, beta2=0.999, eps=1e-15, wd=0.0):
    """OurAdam's per-parameter step restated op for op from its text (masked and dense paths)."""
    for k, parami in params.items():
        st = state[k]
        st["step"] += 1
        step = st["step"].item()
        if relevant.size(0) == 0:
            grad, exp_avg, exp_avg_sq, param = grads[k], st["exp_avg"], st["exp_avg_sq"], parami
        else:
            grad, exp_avg = grads[k][relevant], st["exp_avg"][relevant]
            exp_avg_sq, param = st["exp_avg_sq"][relevant], parami[relevant]
        if wd != 0:
            grad = grad.add(param, alpha=wd)
        exp_avg.mul_(beta1).add_(grad, alpha=1 - beta1)
        exp_avg_sq.mul_(beta2).addcmul_(grad, grad.conj(), value=1 - beta2)
        bias_correction1 = 1 - beta1 ** step
        bias_correction2 = 1 - beta2 ** step
        step_size = lr[k] / bias_correction1
        bias_correction2_sqrt = math.sqrt(bias_correction2)
        denom = (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
        param.addcdiv_(exp_avg, denom, value=-step_size)
        if relevant.size(0) != 0:
            st["exp_avg"][relevant] = exp_avg
            st["exp_avg_sq"][relevant] = exp_avg_sq
            parami[relevant] = param


def make(n, seed):
    g = torch.Generator().manual_seed(seed)
    return {k: torch.randn((n, *s), generator=g) for k, s in SHAPES.items()}


@pytest.mark.parametrize("n,wd", [(1, 0.0), (5, 0.0), (1003, 0.0), (4096, 0.01), (100_001, 0.0)])
def test_against_torch_op_sequence_and_oracle(n, wd):
    init = make(n, n)
    g = torch.Generator().manual_seed(n + 1)
    dev = "cuda"
    ours = {k: torch.nn.Parameter(v.clone().to(dev)) for k, v in init.items()}
    opt = Adam([{"params": [ours[k]], "lr": LRS[k], "name": k} for k in SHAPES], lr=0.0, eps=1e-15, weight_decay=wd)
    ref = {k: v.clone().to(dev) for k, v in init.items()}
    ref_state = {k: {"step": torch.tensor(0.), "exp_avg": torch.zeros_like(v), "exp_avg_sq": torch.zeros_like(v)}
                 for k, v in ref.items()}
    orc = {k: v.clone().numpy() for k, v in init.items()}
    orc_state = {k: (np.zeros_like(v), np.zeros_like(v)) for k, v in orc.items()}
    for step in range(1, 7):
        if step == 4:
            rel = torch.zeros(0, dtype=torch.bool)
        elif step == 5:
            rel = torch.zeros(n, dtype=torch.bool)  # nothing visible: only the counters advance
        else:
            rel = torch.rand(n, generator=g) < 0.6
        grads = {k: torch.randn((n, *s), generator=g) * 10.0 ** (step - 3) for k, s in SHAPES.items()}
        for k in SHAPES:
            ours[k].grad = grads[k].to(dev)
        opt.step(rel.to(dev))
        torch_reference_step(ref, {k: v.to(dev) for k, v in grads.items()}, ref_state, rel.to(dev), LRS, wd=wd)
        for k in SHAPES:
            m, v = orc_state[k]
            oracle.masked_adam(orc[k], grads[k].numpy().copy(), m, v, None if rel.numel() == 0 else rel.numpy(),
                               LRS[k], 0.9, 0.999, 1e-15, wd, step)
    torch.cuda.synchronize()
    for k in SHAPES:
        st = opt.state[ours[k]]
        assert torch.equal(ours[k].detach(), ref[k]), k
        assert torch.equal(st["exp_avg"], ref_state[k]["exp_avg"]) and torch.equal(st["exp_avg_sq"], ref_state[k]["exp_avg_sq"]), k
        assert np.array_equal(ours[k].detach().cpu().numpy().view(np.uint32), orc[k].view(np.uint32)), k
        assert float(st["step"]) == 6.0


def same_bits_or_both_nan(a, b):
    """Bit-identical, except that NaN only has to be NaN on both sides (payloads are the hardware's)."""
    a, b = a.detach().cpu().reshape(-1), b.detach().cpu().reshape(-1)
    na, nb = torch.isnan(a), torch.isnan(b)
    return torch.equal(na, nb) and torch.equal(a[~na].view(torch.int32), b[~nb].view(torch.int32))


def test_non_finite_and_extreme_gradients():
    """Gradients a diverging step produces -- NaN, +-inf, squares that overflow (1e20, 1e30), denormals
    (1e-40), signed zeros -- through three steps: every element as OurAdam's torch ops leave it on this
    GPU (NaN positions equal, other bits equal), and as the C oracle leaves it."""
    n = 5003
    init = make(n, 17)
    g = torch.Generator().manual_seed(18)
    ours = {k: torch.nn.Parameter(v.clone().cuda()) for k, v in init.items()}
    opt = Adam([{"params": [ours[k]], "lr": LRS[k], "name": k} for k in SHAPES], lr=0.0, eps=1e-15)
    ref = {k: v.clone().cuda() for k, v in init.items()}
    ref_state = {k: {"step": torch.tensor(0.), "exp_avg": torch.zeros_like(v), "exp_avg_sq": torch.zeros_like(v)}
                 for k, v in ref.items()}
    orc = {k: v.clone().numpy() for k, v in init.items()}
    orc_state = {k: (np.zeros_like(v), np.zeros_like(v)) for k, v in orc.items()}
    specials = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e20, -1e30, 1e-40, -1e-40, 0.0, -0.0, 3e38])
    for step in range(1, 4):
        rel = torch.rand(n, generator=g) < 0.7
        grads = {}
        for k, s in SHAPES.items():
            t = torch.randn((n, *s), generator=g)
            pick = torch.rand(t.shape, generator=g) < 0.05
            t[pick] = specials[torch.randint(0, specials.numel(), (int(pick.sum()),), generator=g)]
            grads[k] = t
            ours[k].grad = t.cuda()
        opt.step(rel.cuda())
        torch_reference_step(ref, {k: v.cuda() for k, v in grads.items()}, ref_state, rel.cuda(), LRS)
        for k in SHAPES:
            m, v = orc_state[k]
            oracle.masked_adam(orc[k], grads[k].numpy().copy(), m, v, rel.numpy(), LRS[k], 0.9, 0.999, 1e-15, 0.0, step)
    torch.cuda.synchronize()
    for k in SHAPES:
        st = opt.state[ours[k]]
        assert same_bits_or_both_nan(ours[k], ref[k]), k
        assert same_bits_or_both_nan(st["exp_avg"], ref_state[k]["exp_avg"]), k
        assert same_bits_or_both_nan(st["exp_avg_sq"], ref_state[k]["exp_avg_sq"]), k
        assert same_bits_or_both_nan(ours[k], torch.from_numpy(orc[k])), k
        assert bool(torch.isnan(ours[k]).any()) and bool(torch.isfinite(ours[k]).any())


def test_index_relevant_equals_bool_mask():
    n = 5000
    init = make(n, 3)
    idx = torch.randperm(n)[:1234].cuda()
    mask = torch.zeros(n, dtype=torch.bool, device="cuda")
    mask[idx] = True
    outs = []
    for rel in (idx, mask):
        ps = {k: torch.nn.Parameter(v.clone().cuda()) for k, v in init.items()}
        opt = Adam(list(ps.values()), lr=0.01)
        for p in ps.values():
            p.grad = torch.ones_like(p)
        opt.step(rel)
        outs.append([p.detach().clone() for p in ps.values()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_2m_gaussians_one_step_bit_exact_and_masked_rows_kept(oracle_lib):
    n = 2_000_000
    g = torch.Generator().manual_seed(9)
    rel = torch.rand(n, generator=g) < 0.7
    for k, s in SHAPES.items():
        p0 = torch.randn((n, *s), generator=g)
        gr = torch.randn((n, *s), generator=g)
        p = torch.nn.Parameter(p0.cuda())
        p.grad = gr.cuda()
        opt = Adam([p], lr=LRS[k], eps=1e-15)
        opt.step(rel.cuda())
        pn = p0.numpy().copy()
        m, v = np.zeros_like(pn), np.zeros_like(pn)
        oracle.masked_adam(pn, gr.numpy().copy(), m, v, rel.numpy(), LRS[k], 0.9, 0.999, 1e-15, 0.0, 1)
        got = p.detach().cpu().numpy()
        assert np.array_equal(got.view(np.uint32), pn.view(np.uint32)), k
        assert np.array_equal(got[~rel.numpy()], p0.numpy()[~rel.numpy()]), k


def test_unaligned_views_take_the_scalar_path():
    base = torch.randn(10_001 * 3 + 1, device="cuda")
    p = torch.nn.Parameter(base[1:].view(10_001, 3))  # 4-byte offset: no 16-byte vectors
    p.grad = torch.randn(10_001, 3, device="cuda")
    ref = p.detach().clone()
    opt = Adam([p], lr=0.01)
    opt.step(torch.zeros(0, dtype=torch.bool))
    st = {"a": {"step": torch.tensor(0.), "exp_avg": torch.zeros_like(ref), "exp_avg_sq": torch.zeros_like(ref)}}
    torch_reference_step({"a": ref}, {"a": p.grad}, st, torch.zeros(0, dtype=torch.bool), {"a": 0.01}, eps=1e-8)
    assert torch.equal(p.detach(), ref)


def test_multi_tensor_launch_batches_widths_and_ragged_ends(oracle_lib):
    """hidegs_masked_adam_multi over 11 tensors (more than one launch's 8), widths 1..45, row counts
    that leave ragged 16-byte vectors, each with its own mask (or none), lr, weight decay and step
    count -- every tensor bit-exact against the oracle."""
    g = torch.Generator().manual_seed(21)
    specs = [(1, 1), (2, 5), (3, 7), (4, 4099), (5, 333), (6, 1), (7, 2048), (1, 65537), (3, 12345), (45, 1001),
             (2, 3)]
    dev = torch.device("cuda", 0)
    descs, keep, expect = [], [], []
    for i, (w, r) in enumerate(specs):
        p = torch.randn(r, w, generator=g)
        gr = torch.randn(r, w, generator=g)
        m = torch.randn(r, w, generator=g).abs() * 0.1
        v = torch.rand(r, w, generator=g) * 0.01
        rel = None if i % 3 == 0 else (torch.rand(r, generator=g) < 0.5)
        lr, wd, step = 0.001 * (i + 1), (0.01 if i % 4 == 1 else 0.0), 1 + i % 3
        pe, me, ve = p.numpy().copy(), m.numpy().copy(), v.numpy().copy()
        oracle.masked_adam(pe, gr.numpy().copy(), me, ve, None if rel is None else rel.numpy(), lr, 0.9, 0.999,
                           1e-15, wd, step)
        expect.append((pe, me, ve))
        t = [x.to(dev) for x in (p, gr, m, v)] + [None if rel is None else rel.to(dev)]
        keep.append(t)
        descs.append(_lib.AdamTensor(*[_lib.ptr(x) for x in t], r, w, lr, 0.9, 0.999, 1e-15, wd, step))
    arr = (_lib.AdamTensor * len(descs))(*descs)
    _lib.check(_lib.lib().hidegs_masked_adam_multi(arr, len(descs), _lib.stream_handle(dev)), "multi")
    torch.cuda.synchronize()
    for (pe, me, ve), t, spec in zip(expect, keep, specs):
        for got, exp in ((t[0], pe), (t[2], me), (t[3], ve)):
            assert np.array_equal(got.cpu().numpy().view(np.uint32), exp.view(np.uint32)), spec


def test_multi_tensor_rejects_bad_descriptor():
    dev = torch.device("cuda", 0)
    x = torch.zeros(4, 4, device=dev)
    bad = _lib.AdamTensor(_lib.ptr(x), _lib.ptr(x), _lib.ptr(x), _lib.ptr(x), None, 4, 4, 0.1, 0.9, 0.999, 1e-8, 0.0, 0)
    arr = (_lib.AdamTensor * 1)(bad)
    with pytest.raises(RuntimeError, match="step counts from 1"):
        _lib.check(_lib.lib().hidegs_masked_adam_multi(arr, 1, _lib.stream_handle(dev)), "multi")


def test_step_plan_row_ranges_equal_the_whole_step():
    """AdamStepPlan.run_rows over any split of the rows (4-row multiples and ragged cuts, which drop
    to the scalar path) gives bit-identical parameters and moments to one whole step."""
    n = 10_003
    init = make(n, 11)
    g = torch.Generator().manual_seed(12)
    a = {k: torch.nn.Parameter(v.clone().cuda()) for k, v in init.items()}
    b = {k: torch.nn.Parameter(v.clone().cuda()) for k, v in init.items()}
    opt_a = Adam([{"params": [a[k]], "lr": LRS[k]} for k in SHAPES], lr=0.0, eps=1e-15)
    opt_b = Adam([{"params": [b[k]], "lr": LRS[k]} for k in SHAPES], lr=0.0, eps=1e-15)
    cuts = [0, 4, 1000, 1001, 1004, 5003, 9996, n]
    for step in range(3):
        rel = (torch.rand(n, generator=g) < 0.6).cuda() if step != 1 else torch.zeros(0, dtype=torch.bool)
        for k, s in SHAPES.items():
            gr = torch.randn((n, *s), generator=g).cuda()
            a[k].grad, b[k].grad = gr, gr.clone()
        opt_a.step(rel)
        plan = opt_b.begin_step(rel)
        assert len(plan) == len(SHAPES)
        for k in SHAPES:
            for r0, r1 in zip(cuts, cuts[1:]):
                plan.run_rows(b[k], r0, r1)
    torch.cuda.synchronize()
    for k in SHAPES:
        assert torch.equal(a[k].detach(), b[k].detach()), k
        for m in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(opt_a.state[a[k]][m], opt_b.state[b[k]][m]), (k, m)
    with pytest.raises(ValueError):
        opt_b.begin_step(torch.zeros(0, dtype=torch.bool)).run_rows(b["xyz"], 5, n + 1)
