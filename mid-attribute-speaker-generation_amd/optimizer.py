"""``ScheduledOptim`` (``model/optimizer.py:5-51``) over the flat parameter arena.

Adam(betas, eps, weight_decay=0) + Noam warm-up / step-anneal schedule, with the
reference's ``clip_grad_norm_`` (``train.py:202``) fused in: ``clip_grad_norm_`` computes
the global norm on the device and the Adam kernel applies the clip coefficient while it
reads the gradients (one pass over 34.7 M gradients instead of three).  ``_optimizer``
exposes a torch.optim.Adam-compatible ``state_dict``/``load_state_dict``/``param_groups``
so checkpoints (``train.py:276-285``) round-trip with the reference's format.
"""

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
        o._sync_counters()
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
        # device mirrors of the counters and the per-step hyper-parameters: the kernels read
        # these, so the step is a fixed launch sequence (HIP-graph capturable)
        self._dev_steps = torch.zeros(2, dtype=torch.int64, device=dev)
        self._hyper = torch.zeros(3, dtype=torch.float32, device=dev)
        self._sync_counters()

    def _sync_counters(self):
        """Host counters -> device mirrors (construction, checkpoint load)."""
        self._dev_steps.copy_(torch.tensor([int(self.current_step), int(self.adam_steps)],
                                           dtype=torch.int64))

    def host_advance(self, update_lr=True):
        """Advance the host-side counters exactly as one replayed (graph-captured) step did
        on the device."""
        if update_lr:
            self._update_learning_rate()
        self.adam_steps += 1

    # -- reference API ------------------------------------------------------------------
    def step_and_update_lr(self):
        self._update_learning_rate()  # host mirror (param_groups lr, checkpoints)
        self.step(_advance_lr=True)

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
        # a Python float (the reference's is np.float64): checkpoints then load with
        # torch.load(..., weights_only=True)
        lr = float(self.init_lr * self._get_lr_scale())
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

    def step(self, _advance_lr=False):
        if self._join is not None:
            self._join()
        self.adam_steps += 1
        b1, b2 = self.betas
        K.sched_step(self._dev_steps, self._hyper, self.init_lr, self.n_warmup_steps,
                     self.anneal_steps, self.anneal_rate, b1, b2, advance_lr=_advance_lr)
        K.adam_step(self.arena.flat, self.arena.grad, self.m, self.v,
                    self.norm_coef if self._clip_pending else None, 0.0, b1, b2, self.eps,
                    1.0, 1.0, hyper=self._hyper)
        self._clip_pending = False
        self.arena.version += 1
