"""FusedAdamW — the reference's ``AdamW(model.parameters(), lr, weight_decay)`` (train.py:578)
as one multi-tensor HIP kernel over the model's flat fp32 parameter buffer.

Numerics follow torch 2.10's single-tensor AdamW (decoupled weight decay, bias-corrected,
``exp_avg.lerp_``), see ``sd_adamw`` in csrc/misc.hip.  The step counter lives on the device
and only advances when the batch had valid pixels (train.py:331-332 skips the step).

``state_dict()`` / ``load_state_dict()`` use torch.optim.AdamW's format and numbering: state
index i is ``param_groups[0]["params"][i]`` (``model.parameters()`` registration order, enc1
first), mapped to its slice of the flat buffer (which is in backward order, heads first) through
the parameter's storage offset.  A checkpoint written here loads into the reference's AdamW and
vice versa (train.py:421-436 ``optimizer_state_dict``).

Parameters whose ``.grad`` is None at ``step()`` are skipped, as torch's AdamW skips them (no weight
decay, no moment update, no step count).  Once that happens the optimizer keeps one device step
counter per parameter and updates parameter by parameter; the common path (every parameter has a
gradient, the fused train step) is one launch over the whole buffer.
"""

from __future__ import annotations

import torch

from . import _lib as L


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdamW supports a single parameter group")
        owners = {getattr(p, "_sd_owner", lambda: None)() for p in params}
        self.model = None
        if len(owners) == 1 and None not in owners:
            self.model = owners.pop()
        self._m = self._v = None
        self._pstep = None  # per-parameter step counters (int32, param_groups order) once steps diverge

    def attach(self, model):
        """Bind to a stereo_depth_estimation_amd.StereoUNet (needed before its first forward)."""
        self.model = model
        return self

    def _state_buffers(self):
        flat_p, _ = self.model.flat_buffers()
        if self._m is None or self._m.device != flat_p.device or self._m.numel() != flat_p.numel():
            self._m = torch.zeros_like(flat_p)
            self._v = torch.zeros_like(flat_p)
        return self._m, self._v

    def _slots(self) -> list[tuple[torch.Tensor, int, int]]:
        """(param, flat offset, numel) in param_groups order (= torch AdamW's state numbering)."""
        flat_p, _ = self.model.flat_buffers()
        base, end = flat_p.data_ptr(), flat_p.data_ptr() + 4 * flat_p.numel()
        out = []
        for p in self.param_groups[0]["params"]:
            ptr = p.data_ptr()
            if not (base <= ptr < end):
                raise RuntimeError("FusedAdamW: a parameter is not a view of the model's flat buffer")
            out.append((p, (ptr - base) // 4, p.numel()))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise NotImplementedError("closure")
        self.fused_step(gather_grads=True, gate_on_count=False)

    @torch.no_grad()
    def fused_step(self, gather_grads: bool, gate_on_count: bool):
        """One AdamW step over the flat buffer.  gate_on_count: skip when the last fused
        loss saw zero valid pixels (train.py:331-332)."""
        if self.model is None:
            raise RuntimeError("FusedAdamW: call .attach(model) (params are not owned by a HIP StereoUNet)")
        eng = self.model._engine
        if eng is None:
            raise RuntimeError("FusedAdamW.step() before the model's first forward")
        flat_p, flat_g = self.model.flat_buffers()
        has_grad = None
        if gather_grads:  # autograd path: gradients were accumulated into p.grad
            gviews = {id(p): self.model._grad_views[k] for k, p in self.model._named_trainable()}
            has_grad = []
            for p in self.param_groups[0]["params"]:
                gv = gviews[id(p)]
                has_grad.append(p.grad is not None)
                if p.grad is not None and p.grad.data_ptr() != gv.data_ptr():
                    gv.copy_(p.grad)
        m, v = self._state_buffers()
        g = self.param_groups[0]
        if self._pstep is None and (has_grad is None or all(has_grad)):
            eng.adamw(flat_p, flat_g, m, v, g["lr"], g["weight_decay"], g["betas"], g["eps"], gate_on_count=gate_on_count)
            return
        if self._pstep is None:  # first skipped parameter: from here on every parameter counts its own steps
            self._pstep = eng.adam_step.repeat(len(g["params"]))
        eng.touch_state()
        es = 4
        for i, (p, off, n) in enumerate(self._slots()):
            if has_grad is not None and not has_grad[i]:
                continue
            L.call("sd_adamw", flat_p.data_ptr() + es * off, flat_g.data_ptr() + es * off, m.data_ptr() + es * off,
                   v.data_ptr() + es * off, n, float(g["lr"]), float(g["weight_decay"]), float(g["betas"][0]),
                   float(g["betas"][1]), float(g["eps"]), self._pstep.data_ptr() + 4 * i,
                   eng.count.data_ptr() if gate_on_count else None, eng.adam_scratch.data_ptr(), eng._s())

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none)

    def state_dict(self):
        """torch.optim.AdamW-format state (per-parameter exp_avg / exp_avg_sq, float step), numbered
        in param_groups order."""
        sd = {"state": {}, "param_groups": []}
        if self.model is not None and self._m is not None:
            steps = (self._pstep if self._pstep is not None else self.model._engine.adam_step).tolist()
            for i, (p, off, n) in enumerate(self._slots()):
                step = float(steps[i] if len(steps) > 1 else steps[0])
                if step == 0.0 and self._pstep is not None:
                    continue  # never stepped: torch AdamW holds no state for it
                sd["state"][i] = {
                    "step": torch.tensor(step),
                    "exp_avg": self._m[off:off + n].view_as(p).clone(),
                    "exp_avg_sq": self._v[off:off + n].view_as(p).clone(),
                }
        g = dict(self.param_groups[0])
        g["params"] = list(range(len(g.pop("params"))))
        g.update(amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                 decoupled_weight_decay=True)
        sd["param_groups"].append(g)
        return sd

    def load_state_dict(self, state_dict):
        st = state_dict.get("state", {})
        if not st:
            return
        if self.model is None:
            raise RuntimeError("FusedAdamW: call .attach(model) before load_state_dict")
        self.model.engine()  # flat buffers + device step counter exist before the first forward
        m, v = self._state_buffers()
        m.zero_()
        v.zero_()
        steps = []
        for i, (p, off, n) in enumerate(self._slots()):
            s = st.get(i, st.get(str(i)))
            if s is None:
                steps.append(0)
                continue
            if tuple(s["exp_avg"].shape) != tuple(p.shape):
                raise ValueError(f"optimizer state {i}: exp_avg shape {tuple(s['exp_avg'].shape)} does not match "
                                 f"parameter shape {tuple(p.shape)}")
            m[off:off + n].copy_(s["exp_avg"].reshape(-1))
            v[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
            steps.append(int(float(s["step"])))
        eng = self.model._engine
        eng.adam_step.fill_(max(steps))
        if len(set(steps)) == 1:
            self._pstep = None
        else:
            self._pstep = torch.tensor(steps, dtype=torch.int32, device=eng.adam_step.device)
        grp = state_dict["param_groups"][0]
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in grp:
                self.param_groups[0][k] = grp[k]
