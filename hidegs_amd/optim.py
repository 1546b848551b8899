"""Drop-in for the reference's row-masked Adam, `scene.OurAdam.Adam` (scene/OurAdam.py:7-175).

HiDeGS builds it with one parameter group per Gaussian attribute (gaussian_model.py:300-310:
xyz, f_dc, f_rest, opacity, scaling, rotation; eps 1e-15) and steps it with the visibility
mask: `optimizer.step(relevant)`.  Rows where `relevant` is set get an Adam update; the others
keep their parameter and moments unchanged; an empty `relevant` updates every row
(OurAdam.py:230-244).  Each parameter's step counter advances on every call, masked or not,
exactly as the reference's `step_t += 1`.

The whole step is one fused gfx950 launch over all parameters (hidegs_masked_adam_multi,
csrc/adam.hip) that reads and writes every relevant element once, instead of the reference's
per-parameter boolean-index gathers, eight elementwise ops and scatters.  Results equal the reference's torch ops on the
GPU bit for bit (tests/test_adam_gpu.py).  No CPU fallback: parameters must live on the GPU.

`begin_step(relevant)` splits the step in two: it advances the counters and describes every
parameter's update (an `AdamStepPlan`) without running it; the plan then runs whole or row range
by row range.  The view-DP exchange uses the row ranges to update each gradient bucket as soon as
its all-reduce has landed (hidegs_amd.view_dp.ViewDPExchange.exchange_and_step).

Not supported, as in the reference's masked path, which fails on them with a shape error:
amsgrad, maximize; capturable (a different op sequence) is not reproduced.
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import Optimizer

from hidegs_amd import _lib


class AdamStepPlan:
    """One prepared optimizer step: every parameter's step counter has advanced and its update is
    described (device pointers, mask, hyper-parameters), nothing has run yet.

    run()                  the whole step, one launch per device (what Adam.step does)
    run_rows(p, r0, r1)    the update of rows [r0, r1) of parameter p only
    Each row of each parameter is updated by exactly one of these per plan; how the rows are split
    does not change a bit of the result (the update is row-local).
    """

    def __init__(self):
        self._entries = []  # (param, device, descriptor, tensors the descriptor points into)
        self._index = {}

    def _add(self, p, dev, desc, keep) -> None:
        self._index[id(p)] = len(self._entries)
        self._entries.append((p, dev, desc, keep))

    def __len__(self) -> int:
        return len(self._entries)

    def run(self) -> None:
        batches = {}
        for _, dev, desc, _ in self._entries:
            batches.setdefault(dev, []).append(desc)
        L = _lib.lib()
        for dev, descs in batches.items():
            arr = (_lib.AdamTensor * len(descs))(*descs)
            with torch.cuda.device(dev):
                _lib.check(L.hidegs_masked_adam_multi(arr, len(descs), _lib.stream_handle(dev)), "masked Adam")

    def run_except(self, params) -> None:
        """The update of every parameter of the plan not in `params` (whole), as run() would."""
        skip = {id(p) for p in params}
        batches = {}
        for p, dev, desc, _ in self._entries:
            if id(p) not in skip:
                batches.setdefault(dev, []).append(desc)
        L = _lib.lib()
        for dev, descs in batches.items():
            arr = (_lib.AdamTensor * len(descs))(*descs)
            with torch.cuda.device(dev):
                _lib.check(L.hidegs_masked_adam_multi(arr, len(descs), _lib.stream_handle(dev)), "masked Adam")

    def run_rows(self, param, row_start: int, row_end: int) -> None:
        i = self._index.get(id(param))
        if i is None:
            raise KeyError("parameter is not part of this step (no gradient, or another optimizer's)")
        _, dev, d, _ = self._entries[i]
        r0, r1 = int(row_start), int(row_end)
        if not 0 <= r0 <= r1 <= d.rows:
            raise ValueError(f"rows [{r0}, {r1}) outside the parameter's {d.rows} rows")
        if r0 == r1:
            return
        off = 4 * r0 * d.width  # fp32 bytes
        sub = _lib.AdamTensor(d.param + off, d.grad + off, d.exp_avg + off, d.exp_avg_sq + off,
                              (d.relevant + r0) if d.relevant else None, r1 - r0, d.width, d.lr, d.beta1, d.beta2,
                              d.eps, d.weight_decay, d.step)
        arr = (_lib.AdamTensor * 1)(sub)
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().hidegs_masked_adam_multi(arr, 1, _lib.stream_handle(dev)), "masked Adam")


class Adam(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=False):
        if not 0.0 <= lr:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {}".format(eps))
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError("Invalid beta parameter at index 0: {}".format(betas[0]))
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameter at index 1: {}".format(betas[1]))
        if not 0.0 <= weight_decay:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        if amsgrad or maximize or capturable:
            raise NotImplementedError("amsgrad / maximize / capturable are not supported by the masked step")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable)
        super().__init__(params, defaults)

    @staticmethod
    def _row_mask(relevant: torch.Tensor, rows: int, device) -> torch.Tensor:
        if relevant.dtype == torch.bool:
            if relevant.dim() != 1 or relevant.numel() != rows:
                raise RuntimeError(f"relevant mask has {relevant.numel()} entries for {rows} parameter rows")
            return relevant.to(device).contiguous()
        mask = torch.zeros(rows, dtype=torch.bool, device=device)  # an index tensor selects rows
        mask[relevant.to(device).long()] = True
        return mask

    @torch.no_grad()
    def begin_step(self, relevant) -> AdamStepPlan:
        """Advance every parameter's step counter and describe its update; see AdamStepPlan."""
        dense = relevant.size(0) == 0
        masks = {}
        plan = AdamStepPlan()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients, please consider SparseAdam instead")
                state = self.state[p]
                if len(state) == 0:  # lazy state initialisation, as OurAdam.py:135-146
                    state["step"] = torch.tensor(0.)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["step"] += 1
                step = int(state["step"].item())
                rows = p.shape[0] if p.dim() > 0 else 1
                width = p.numel() // rows if rows else 0
                dev = _lib.device_of(p, p.grad, state["exp_avg"], state["exp_avg_sq"])
                mask = None
                if not dense:
                    key = (rows, dev)
                    if key not in masks:
                        masks[key] = self._row_mask(relevant, rows, dev)
                    mask = masks[key]
                for t in (p, p.grad, state["exp_avg"], state["exp_avg_sq"]):
                    if not t.is_contiguous() or t.dtype != torch.float32:
                        raise RuntimeError("masked Adam needs contiguous float32 parameters, grads and moments")
                desc = _lib.AdamTensor(
                    _lib.ptr(p), _lib.ptr(p.grad), _lib.ptr(state["exp_avg"]), _lib.ptr(state["exp_avg_sq"]),
                    _lib.ptr(mask), rows, width, float(group["lr"]), float(beta1), float(beta2),
                    float(group["eps"]), float(group["weight_decay"]), step)
                plan._add(p, dev, desc, (p, p.grad, state["exp_avg"], state["exp_avg_sq"], mask))
        return plan

    @torch.no_grad()
    def step(self, relevant, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.begin_step(relevant).run()
        return loss
