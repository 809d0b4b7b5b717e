"""Flat, NaN-guarded Adam (train.py:71 uses ``torch.optim.Adam(lr=5e-4)``).

``FlatAdam`` keeps every trainable fp32 parameter, its gradient and both Adam
moments in four flat device buffers; the module's parameters and ``.grad``
tensors are views into them.  That buys three things:

* the data-parallel gradient bucket IS the gradient buffer: the RCCL
  all-reduce runs on it in place (no pack / unpack copies), and the 1/world
  average is folded into the update;
* a step is three HIP launches (``csrc/optim.hip``) regardless of the
  parameter count: count non-finite gradient entries, masked Adam update,
  finalize the device step counter;
* the NaN/Inf guard is exact and asynchronous: when the loss (written into a
  trailing indicator slot of the gradient buffer before the all-reduce) or
  any gradient on any rank is non-finite, the parameters, both moments and
  the step counter are left untouched -- no host sync to decide.

The update is torch.optim.Adam's (L2 weight decay, bias correction, eps
outside the sqrt), and ``state_dict()`` / ``load_state_dict()`` use
torch.optim.Adam's layout, so checkpoints interchange with the reference's
``optimizer`` entry (train.py:197-205).  On CPU the same masked update runs
as torch ops (the oracle for tests/test_optim.py).
"""
from __future__ import annotations

import torch

from ..ops import _ext


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0):
        params = [p for p in params]
        if not params:
            raise ValueError("FlatAdam: no parameters")
        if any(p.dtype != torch.float32 for p in params):
            raise TypeError("FlatAdam: all parameters must be fp32")
        dev = params[0].device
        if any(p.device != dev for p in params):
            raise ValueError("FlatAdam: parameters must share one device")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdam: one parameter group only")
        self.params = params
        self.n = n = sum(p.numel() for p in params)
        self.flat_param = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n + 1, dtype=torch.float32, device=dev)   # + loss-indicator slot
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self._step = torch.zeros(1, dtype=torch.float32, device=dev)
        self._count = torch.zeros(1, dtype=torch.int32, device=dev)
        self._skipped = torch.zeros(1, dtype=torch.int32, device=dev)
        self.grad_scale = 1.0          # set to 1/world by a GradBucket that all-reduces flat_grad in place
        self.guard = True              # False (Trainer(nan_guard=False)): no non-finite skip
        self.spans = []
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.flat_param[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat_param[off:off + k].view_as(p)
                p.grad = self.flat_grad[off:off + k].view_as(p)
                self.spans.append((off, k))
                off += k
        self._hip = dev.type == "cuda" and _ext.use_hip(self.flat_param)

    # -- gradient buffer -------------------------------------------------
    def zero_grad(self, set_to_none: bool = True) -> None:  # noqa: ARG002 - views must survive
        """Zero the flat gradient buffer; the ``.grad`` views stay in place so
        autograd accumulates straight into the bucket."""
        for p, (off, k) in zip(self.params, self.spans):
            if p.grad is None or p.grad.data_ptr() != self.flat_grad[off:].data_ptr():
                p.grad = self.flat_grad[off:off + k].view_as(p)
        self.flat_grad.zero_()

    def mark_loss(self, loss: torch.Tensor) -> None:
        """Write 0 (finite loss) or NaN (non-finite loss) into the indicator
        slot; call before the gradient all-reduce so every rank sees it."""
        torch.mul(loss.detach().reshape(1).float(), 0.0, out=self.flat_grad[self.n:])

    # -- update ----------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.check_bindings()
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = float(g["lr"]), g["betas"], float(g["eps"]), float(g["weight_decay"])
        if self._hip:
            ext = _ext.ext()
            if self.guard:
                ext.nonfinite_count(self.flat_grad, self._count)   # else _count stays 0 (finalize resets it)
            ext.adam_masked(self.flat_param, self.flat_grad, self.exp_avg, self.exp_avg_sq, self._count, self._step,
                            lr, float(b1), float(b2), eps, wd, float(self.grad_scale))
            ext.adam_finalize(self._step, self._count, self._skipped)
            # the kernels wrote the parameters behind autograd's back: bump the
            # version counters so any version-keyed cache sees the update
            for p in self.params:
                torch.autograd.graph.increment_version(p)
        else:
            self._step_torch(lr, float(b1), float(b2), eps, wd)
        return loss

    def check_bindings(self) -> None:
        """Every parameter must still be a view of ``flat_param``: a later
        ``module._apply`` (``.to()``, ``.cuda()``, ``.half()``) or an assignment
        to ``p.data`` rebinds it to new storage, after which this optimizer would
        update buffers the model no longer reads.  make_adam must be the LAST
        placement step (train.py / bench.py build the model on its device first)."""
        base = self.flat_param.data_ptr()
        esz = self.flat_param.element_size()
        for i, (p, (off, _)) in enumerate(zip(self.params, self.spans)):
            if p.data_ptr() != base + off * esz:
                raise RuntimeError(f"FlatAdam: parameter {i} {tuple(p.shape)} is no longer a view of the flat "
                                   "buffer (the module was moved or p.data reassigned after make_adam); "
                                   "create the optimizer after the last .to()/.cuda()/load")

    def _step_torch(self, lr, b1, b2, eps, wd):
        bad = int((~torch.isfinite(self.flat_grad)).sum()) if self.guard else 0
        grad = self.flat_grad[: self.n]
        if bad:
            grad.zero_()
            self._skipped += 1
            return
        if self.grad_scale != 1.0:
            grad.mul_(self.grad_scale)
        t = float(self._step) + 1.0
        gi = grad + wd * self.flat_param if wd != 0.0 else grad
        self.exp_avg.lerp_(gi, 1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(gi, gi, value=1 - b2)
        step_size = lr / (1 - b1 ** t)
        denom = (self.exp_avg_sq.sqrt() / (1 - b2 ** t) ** 0.5).add_(eps)
        self.flat_param.addcdiv_(self.exp_avg, denom, value=-step_size)
        self._step += 1

    @property
    def skipped_steps(self) -> int:
        """Steps skipped by the NaN/Inf guard so far (host read: syncs)."""
        return int(self._skipped)

    @property
    def steps_taken(self) -> int:
        return int(self._step)

    # -- torch.optim.Adam-compatible state -------------------------------
    def _publish_state(self):
        self.state.clear()
        t = float(self._step)
        if t == 0.0:
            return
        for p, (off, k) in zip(self.params, self.spans):
            self.state[p] = {"step": torch.tensor(t, dtype=torch.float32),
                             "exp_avg": self.exp_avg[off:off + k].view_as(p),
                             "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p)}

    def state_dict(self):
        self._publish_state()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = set()
        with torch.no_grad():
            for p, (off, k) in zip(self.params, self.spans):
                st = self.state.get(p)
                if not st:
                    continue
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(float(st["step"]))
            if len(steps) > 1:
                raise ValueError(f"FlatAdam: parameters at different Adam steps {sorted(steps)}")
            self._step.fill_(steps.pop() if steps else 0.0)
        self._publish_state()
