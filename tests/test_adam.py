"""Masked Adam: the CPU oracle and the optimizer's host-side behaviour.

The oracle (oracle/adam_ref.c) restates one OurAdam step from the reference text
(scene/OurAdam.py:249-337 masked, :340-420 dense).  It cannot be pinned against the reference's
own outputs (DESIGN.md, round-3 decision), so it is checked here against the textbook Adam
recursion in float64 and against the closed form of the first step.
"""
import numpy as np
import pytest
import torch

import oracle
from hidegs_amd.optim import Adam


def textbook(p, g, m, v, lr, b1, b2, eps, step):
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    mh, vh = m / (1 - b1 ** step), v / (1 - b2 ** step)
    return p - lr * mh / (np.sqrt(vh) + eps), m, v


def test_oracle_first_step_closed_form(oracle_lib):
    g = np.random.default_rng(0).normal(size=(100, 3)).astype(np.float32)
    p = np.zeros_like(g)
    m, v = np.zeros_like(g), np.zeros_like(g)
    oracle.masked_adam(p, g.copy(), m, v, None, lr=0.01, eps=1e-15, step=1)
    np.testing.assert_allclose(p, -0.01 * np.sign(g), rtol=1e-5)  # first Adam step moves by lr * sign(g)


def test_oracle_matches_float64_recursion_over_steps(oracle_lib):
    rng = np.random.default_rng(1)
    p = rng.normal(size=(500, 4)).astype(np.float32)
    m, v = np.zeros_like(p), np.zeros_like(p)
    p64, m64, v64 = p.astype(np.float64), m.astype(np.float64), v.astype(np.float64)
    for step in range(1, 8):
        g = (rng.normal(size=p.shape) * 10.0 ** (step - 4)).astype(np.float32)
        oracle.masked_adam(p, g.copy(), m, v, None, lr=1e-3, eps=1e-8, step=step)
        p64, m64, v64 = textbook(p64, g.astype(np.float64), m64, v64, 1e-3, 0.9, 0.999, 1e-8, step)
    np.testing.assert_allclose(p, p64, rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(m, m64, rtol=1e-5, atol=1e-12)


def test_oracle_masked_rows_untouched_and_dense_equals_all_true(oracle_lib):
    rng = np.random.default_rng(2)
    p0 = rng.normal(size=(300, 15, 3)).astype(np.float32)
    g = rng.normal(size=p0.shape).astype(np.float32)
    m0 = rng.normal(size=p0.shape).astype(np.float32) * 0.1
    v0 = np.abs(rng.normal(size=p0.shape)).astype(np.float32) * 0.01
    mask = rng.random(300) < 0.4
    p, m, v = p0.copy(), m0.copy(), v0.copy()
    oracle.masked_adam(p, g, m, v, mask, lr=0.0025, eps=1e-15, step=3)
    assert np.array_equal(p[~mask], p0[~mask]) and np.array_equal(m[~mask], m0[~mask])
    assert not np.array_equal(p[mask], p0[mask])
    pd, md, vd = p0.copy(), m0.copy(), v0.copy()
    oracle.masked_adam(pd, g, md, vd, None, lr=0.0025, eps=1e-15, step=3)
    pa, ma, va = p0.copy(), m0.copy(), v0.copy()
    oracle.masked_adam(pa, g, ma, va, np.ones(300, bool), lr=0.0025, eps=1e-15, step=3)
    assert np.array_equal(pd, pa) and np.array_equal(md, ma) and np.array_equal(vd, va)


def test_optimizer_arguments_like_reference():
    p = torch.nn.Parameter(torch.zeros(4, 3))
    for kw in (dict(lr=-1), dict(eps=-1), dict(betas=(1.0, 0.9)), dict(betas=(0.9, 1.0)), dict(weight_decay=-1)):
        with pytest.raises(ValueError):
            Adam([p], **kw)
    for kw in (dict(amsgrad=True), dict(maximize=True), dict(capturable=True)):
        with pytest.raises(NotImplementedError):
            Adam([p], **kw)


def test_optimizer_refuses_host_parameters(built_lib):
    p = torch.nn.Parameter(torch.zeros(4, 3))
    p.grad = torch.ones(4, 3)
    opt = Adam([p], lr=0.1)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        opt.step(torch.ones(4, dtype=torch.bool))
    assert float(opt.state[p]["step"]) == 1.0  # the counter advanced, as step_t += 1 does first
