"""fp32 master weights for a model that computes in bf16.

``model.to(torch.bfloat16)`` followed by Adam updates the bf16 weights directly: every step
rounds ``w - lr * u`` to 8 significant bits, so small updates vanish (the GraphCast trainer
and benchmark did this in round 1). :class:`MasterWeights` keeps an fp32 copy of every
parameter, builds the optimizer over the fp32 copies, and per step

    master.grad = bf16 grad (as fp32)  ->  optimizer.step() on fp32  ->  bf16 <- master

so the forward/backward stay bf16 (the MFMA/HBM rate) while the optimizer state and the
accumulated weights keep fp32 precision. ``state_dict()`` / ``load_state_dict()`` speak
fp32 under the model's own parameter names (checkpoints are precision-preserving and load
into an fp32 model as well).
"""
from __future__ import annotations

from typing import Callable, Dict

import torch


class MasterWeights:
    def __init__(self, model: torch.nn.Module,
                 make_optimizer: Callable[[list], torch.optim.Optimizer]):
        self.model = model
        self.names = [n for n, p in model.named_parameters() if p.requires_grad]
        self.low = [p for p in model.parameters() if p.requires_grad]
        self.master = [p.detach().float().clone().requires_grad_(True) for p in self.low]
        self.optimizer = make_optimizer(self.master)

    @torch.no_grad()
    def step(self) -> None:
        # multi-tensor copies (a handful of launches for all parameters, not two per
        # parameter: ~250 tiny kernels per GraphCast step before, profiles/)
        los, his = [], []
        for lo, hi in zip(self.low, self.master):
            if lo.grad is None:
                hi.grad = None
                continue
            if hi.grad is None or hi.grad.shape != hi.shape:
                hi.grad = torch.empty_like(hi)
            los.append(lo.grad)
            his.append(hi.grad)
        if his:
            torch._foreach_copy_(his, los)
        self.optimizer.step()
        torch._foreach_copy_(self.low, self.master)

    def zero_grad(self, set_to_none: bool = True) -> None:
        self.model.zero_grad(set_to_none=set_to_none)
        self.optimizer.zero_grad(set_to_none=set_to_none)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {k: v.detach() for k, v in self.model.state_dict().items()}
        for n, hi in zip(self.names, self.master):
            sd[n] = hi.detach()
        return sd

    @torch.no_grad()
    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        self.model.load_state_dict({k: v.to(self.model.state_dict()[k].dtype)
                                    for k, v in sd.items()})
        for n, hi, lo in zip(self.names, self.master, self.low):
            hi.copy_(sd[n].float())
            lo.copy_(hi)
