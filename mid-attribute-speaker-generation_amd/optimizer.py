"""``ScheduledOptim`` (``model/optimizer.py:5-51``) over the flat parameter arena.

Adam(betas, eps, weight_decay=0) + Noam warm-up / step-anneal schedule, with the
reference's ``clip_grad_norm_`` (``train.py:202``) fused in: ``clip_grad_norm_`` computes
the global norm on the device and the Adam kernel applies the clip coefficient while it
reads the gradients (one pass over 34.7 M gradients instead of three).  ``_optimizer``
exposes a torch.optim.Adam-compatible ``state_dict``/``load_state_dict``/``param_groups``
so checkpoints (``train.py:276-285``) round-trip with the reference's format.
"""
import math

import numpy as np
import torch

from . import kernels as K


class _AdamView:
    """torch.optim.Adam-shaped facade (state_dict format, param_groups[*]['lr'])."""

    def __init__(self, owner, params, betas, eps, weight_decay):
        self._o = owner
        self.param_groups = [{"params": params, "lr": 0.0, "betas": tuple(betas), "eps": eps,
                              "weight_decay": weight_decay, "amsgrad": False, "maximize": False,
                              "foreach": None, "capturable": False, "differentiable": False,
                              "fused": None, "decoupled_weight_decay": False}]

    def state_dict(self):
        o = self._o
        arena = o.arena
        index = {id(p): i for i, p in enumerate(self.param_groups[0]["params"])}
        state = {}
        if o.adam_steps > 0:
            for p, off in zip(arena.params, arena.offsets):
                n = p.numel()
                state[index[id(p)]] = {
                    "step": torch.tensor(float(o.adam_steps)),
                    "exp_avg": o.m[off:off + n].view(p.shape).clone(),
                    "exp_avg_sq": o.v[off:off + n].view(p.shape).clone()}
        g = dict(self.param_groups[0])
        g["params"] = list(range(len(g["params"])))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, sd):
        o = self._o
        arena = o.arena
        params = self.param_groups[0]["params"]
        steps = 0
        with torch.no_grad():
            for i, st in sd["state"].items():
                p = params[int(i)]
                off = arena.offsets[[id(q) for q in arena.params].index(id(p))]
                n = p.numel()
                o.m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                o.v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps = int(float(st["step"]))
        o.adam_steps = steps
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in sd["param_groups"][0]:
                self.param_groups[0][k] = sd["param_groups"][0][k]

    def zero_grad(self, set_to_none=False):
        self._o.zero_grad()


class ScheduledOptim:
    """``model/optimizer.py:5-51`` with the same constructor and methods."""

    def __init__(self, model, train_config, model_config, current_step):
        oc = train_config["optimizer"]
        self.arena = model.arena()
        self._join = getattr(model, "join_side", None)  # weight-gradient stream
        self.betas = tuple(float(b) for b in oc["betas"])
        self.eps = float(oc["eps"])
        wd = float(oc["weight_decay"])
        if wd != 0.0:
            raise NotImplementedError("weight_decay != 0 is not built (all configs use 0.0)")
        dev = self.arena.flat.device
        self.m = K.zeros(self.arena.numel, dev)
        self.v = K.zeros(self.arena.numel, dev)
        self.norm_coef = torch.empty(2, dtype=torch.float32, device=dev)
        self._clip_pending = False
        self.adam_steps = 0
        self.n_warmup_steps = oc["warm_up_step"]
        self.anneal_steps = oc["anneal_steps"]
        self.anneal_rate = oc["anneal_rate"]
        self.current_step = current_step
        self.init_lr = np.power(model_config["transformer"]["encoder_hidden"], -0.5)
        self._optimizer = _AdamView(self, list(model.parameters()), self.betas, self.eps, wd)

    # -- reference API ------------------------------------------------------------------
    def step_and_update_lr(self):
        self._update_learning_rate()
        self.step()

    def zero_grad(self):
        self.arena.zero_grad()

    def load_state_dict(self, sd):
        self._optimizer.load_state_dict(sd)

    def _get_lr_scale(self):
        lr = np.min([np.power(self.current_step, -0.5),
                     np.power(self.n_warmup_steps, -1.5) * self.current_step])
        for s in self.anneal_steps:
            if self.current_step > s:
                lr = lr * self.anneal_rate
        return lr

    def _update_learning_rate(self):
        self.current_step += 1
        lr = self.init_lr * self._get_lr_scale()
        for g in self._optimizer.param_groups:
            g["lr"] = lr

    # -- fused clip + Adam ----------------------------------------------------------------
    def clip_grad_norm_(self, max_norm):
        """Global L2 norm of all gradients; the clip is applied inside the next ``step``.
        Returns the (pre-clip) norm as a 0-dim device tensor, like torch's clip_grad_norm_."""
        if self._join is not None:
            self._join()
        K.grad_norm(self.arena.grad, float(max_norm), self.norm_coef)
        self._clip_pending = True
        return self.norm_coef[0]

    def step(self):
        if self._join is not None:
            self._join()
        self.adam_steps += 1
        b1, b2 = self.betas
        t = self.adam_steps
        lr = float(self._optimizer.param_groups[0]["lr"])
        K.adam_step(self.arena.flat, self.arena.grad, self.m, self.v,
                    self.norm_coef if self._clip_pending else None, lr, b1, b2, self.eps,
                    1.0 - b1 ** t, math.sqrt(1.0 - b2 ** t))
        self._clip_pending = False
        self.arena.version += 1
