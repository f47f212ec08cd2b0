"""Drop-in StereoUNet (reference ``src/foundation_stereo_depth/model.py:8-104``) on the HIP path.

Same constructor, same ``forward(x, return_uncertainty=False)`` contract, same module tree
and therefore the same 120 state_dict keys and the same default initialisation (the
parameter containers are ordinary nn.Conv2d / BatchNorm2d / ConvTranspose2d modules,
created in the reference's registration order).  The computation never goes through
those modules: ``forward`` runs the hand-written gfx950 kernels of libstereo_hip via
:class:`~stereo_depth_estimation_amd.engine.UNetEngine`.  There is no CPU path — a
non-HIP input raises.

Parameters live in ONE flat fp32 device buffer (and gradients in another), ordered by
the order backward produces them (heads, dec1, up1, dec2, …, enc1), so that gradient
all-reduce buckets are contiguous and AdamW is a single multi-tensor kernel.
"""

from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from . import _lib as L
from .engine import UNetEngine


def load_state_dict_compat(model: nn.Module, state_dict: dict[str, torch.Tensor]) -> tuple[list[str], list[str]]:
    """model.py:8-29: legacy ``output_head.*`` -> ``disparity_head.*``; missing logvar head
    filled from the fresh model; strict=False.  Returns (missing, unexpected)."""
    mapped = dict(state_dict)
    if "output_head.weight" in mapped and "disparity_head.weight" not in mapped:
        mapped["disparity_head.weight"] = mapped.pop("output_head.weight")
    if "output_head.bias" in mapped and "disparity_head.bias" not in mapped:
        mapped["disparity_head.bias"] = mapped.pop("output_head.bias")
    own = model.state_dict()
    for k in ("logvar_head.weight", "logvar_head.bias"):
        if k not in mapped:
            mapped[k] = own[k]
    res = model.load_state_dict(mapped, strict=False)
    return list(res.missing_keys), list(res.unexpected_keys)


class ConvBlock(nn.Module):
    """Parameter container with the reference's layout (model.py:32-45)."""

    def __init__(self, in_channels: int, out_channels: int) -> None:
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
        )


GRAD_ORDER = ("disparity_head", "logvar_head", "dec1", "up1", "dec2", "up2", "dec3", "up3", "dec4", "up4",
              "bottleneck", "enc4", "enc3", "enc2", "enc1")


class _UNetFunction(torch.autograd.Function):
    """Autograd bridge for ``loss.backward()`` driven by an arbitrary external loss."""

    @staticmethod
    def forward(ctx, model, x, *params):
        eng = model._engine
        B, _, H, W = x.shape
        eng.pack_weights(train=model.training)
        eng.forward(x, train=model.training, need_backward=True)
        disp = torch.empty(B, 1, H, W, dtype=torch.float32, device=x.device)
        logvar = torch.empty_like(disp)
        eng.heads(L.SD_HEADS_INFER, disp=disp, logvar=logvar)
        model._generation += 1
        ctx.model = model
        ctx.generation = model._generation
        # an output no loss uses arrives as None in backward (not zeros): its head then gets no gradient,
        # as in the reference, where that head is not in the autograd graph (model.py:98-104)
        ctx.set_materialize_grads(False)
        return disp, logvar

    @staticmethod
    def backward(ctx, gdisp, glogvar):
        model = ctx.model
        if model._generation != ctx.generation:
            raise RuntimeError(
                "StereoUNet (HIP) keeps the activations of the latest forward only: call backward before the next forward"
            )
        eng = model._engine
        if not eng.ws.train:
            raise RuntimeError("backward through an eval-mode/no-grad workspace")
        gd = None if gdisp is None else gdisp.contiguous().float()
        gl = None if glogvar is None else glogvar.contiguous().float()
        eng.heads(L.SD_HEADS_GRADS, gdisp=gd, glogvar=gl)
        eng.backward()
        unused = set()
        if gdisp is None:
            unused.add("disparity_head")
        if glogvar is None:
            unused.add("logvar_head")
        grads = [None if k.split(".")[0] in unused else model._grad_views[k].clone()
                 for k, _ in model._named_trainable()]
        return (None, None, *grads)


class StereoUNet(nn.Module):
    def __init__(self, in_channels: int = 6, out_channels: int = 1, base_channels: int = 32,
                 precision: str = "fp32") -> None:
        """precision: "fp32" (default: the reference's arithmetic, model.py:48-51, held to its outputs within 1e-3
        per pixel), "bf16" (opt-in fast training/inference: bf16 activations, fp32 accumulation and master weights;
        drifts from fp32 less than the reference itself does under torch.autocast(bf16)), or "fp8" (e4m3
        inference forward for the live app, BASELINE config 5)."""
        super().__init__()
        c1 = base_channels
        c2, c3, c4, c5 = c1 * 2, c1 * 4, c1 * 8, c1 * 16
        self.pool = nn.MaxPool2d(2)
        self.enc1 = ConvBlock(in_channels, c1)
        self.enc2 = ConvBlock(c1, c2)
        self.enc3 = ConvBlock(c2, c3)
        self.enc4 = ConvBlock(c3, c4)
        self.bottleneck = ConvBlock(c4, c5)
        self.up4 = nn.ConvTranspose2d(c5, c4, kernel_size=2, stride=2)
        self.dec4 = ConvBlock(c4 + c4, c4)
        self.up3 = nn.ConvTranspose2d(c4, c3, kernel_size=2, stride=2)
        self.dec3 = ConvBlock(c3 + c3, c3)
        self.up2 = nn.ConvTranspose2d(c3, c2, kernel_size=2, stride=2)
        self.dec2 = ConvBlock(c2 + c2, c2)
        self.up1 = nn.ConvTranspose2d(c2, c1, kernel_size=2, stride=2)
        self.dec1 = ConvBlock(c1 + c1, c1)
        self.disparity_head = nn.Conv2d(c1, out_channels, kernel_size=1)
        self.logvar_head = nn.Conv2d(c1, 1, kernel_size=1)
        self.in_channels, self.out_channels, self.base_channels = in_channels, out_channels, base_channels
        self.precision = precision
        self._engine: UNetEngine | None = None
        self._bound = None  # identity of what the engine was last bound to (engine, flat buffers, BN buffers)
        self._bn_modules = [m for m in self.modules() if isinstance(m, nn.BatchNorm2d)]
        self._flat_p: torch.Tensor | None = None
        self._flat_g: torch.Tensor | None = None
        self._grad_views: dict[str, torch.Tensor] = {}
        self._generation = 0
        for p in self.parameters():
            p._sd_owner = weakref.ref(self)

    # ------------------------------------------------------------------ flat storage
    def _named_trainable(self):
        """(state_dict key, Parameter) in backward-production order. The module tree is fixed after construction, so
        the list is built once (rebuilding it took ~0.4 ms of host time per forward, which B=1 inference felt)."""
        cache = self.__dict__.get("_trainable_cache")  # dropped by _apply and by _is_flat when a Parameter moved
        if cache is None:
            named = dict(self.named_parameters())
            cache = []
            for top in GRAD_ORDER:
                cache.extend((k, p) for k, p in named.items() if k.split(".")[0] == top)
            self.__dict__["_trainable_cache"] = cache
            # where each Parameter is registered: a replaced Parameter object (load_state_dict(assign=True), or
            # `module.weight = nn.Parameter(...)`) is noticed by _is_flat without rebuilding the list
            mods = dict(self.named_modules())
            self.__dict__["_trainable_slots"] = [(mods[k.rpartition(".")[0]]._parameters, k.rpartition(".")[2], p)
                                                 for k, p in cache]
        return cache

    def _is_flat(self, device) -> bool:
        named = self._named_trainable()
        if any(d.get(n) is not p for d, n, p in self.__dict__["_trainable_slots"]):
            self.__dict__.pop("_trainable_cache", None)  # a Parameter was replaced: new list, new flat buffer
            return False
        if self._flat_p is None or self._flat_p.device != device:
            return False
        base = self._flat_p.untyped_storage().data_ptr()
        return all(p.untyped_storage().data_ptr() == base for _, p in named)

    def _flatten(self, device):
        # ordinary tensors even when the first forward runs under torch.inference_mode(): inference
        # tensors could not be trained later and carry no version counters (eval-state tracking)
        with torch.inference_mode(False):
            self._flatten_impl(device)

    def _flatten_impl(self, device):
        named = self._named_trainable()
        n = sum(p.numel() for _, p in named)
        flat_p = torch.empty(n, dtype=torch.float32, device=device)
        flat_g = torch.zeros(n, dtype=torch.float32, device=device)
        views = {}
        off = 0
        with torch.no_grad():
            for k, p in named:
                k_n = p.numel()
                flat_p[off:off + k_n].copy_(p.detach().reshape(-1))
                p.data = flat_p[off:off + k_n].view_as(p)
                views[k] = flat_g[off:off + k_n].view_as(p)
                p._sd_owner = weakref.ref(self)
                off += k_n
        self._flat_p, self._flat_g, self._grad_views = flat_p, flat_g, views
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.running_mean.data = m.running_mean.data.to(device)
                m.running_var.data = m.running_var.data.to(device)
                m.num_batches_tracked.data = m.num_batches_tracked.data.to(device)

    def flat_buffers(self) -> tuple[torch.Tensor, torch.Tensor]:
        return self._flat_p, self._flat_g

    def bucket_ranges(self) -> list[tuple[str, int, int]]:
        """(top-level module, start, end) ranges of the flat buffers, in backward order."""
        out, off = [], 0
        for top in GRAD_ORDER:
            n = sum(p.numel() for k, p in self._named_trainable() if k.split(".")[0] == top)
            out.append((top, off, off + n))
            off += n
        return out

    def engine(self, device=None) -> UNetEngine:
        device = torch.device(device) if device is not None else next(self.parameters()).device
        if device.type != "cuda":
            raise RuntimeError(
                "stereo_depth_estimation_amd.StereoUNet runs only on a HIP device (MI355X); "
                f"got device {device}. There is no CPU fallback."
            )
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if not self._is_flat(device):
            self._flatten(device)
            self._engine = None
        if self._engine is None or self._engine.device != device:
            with torch.inference_mode(False):  # its state (step counter, metric sums) must stay trainable
                self._engine = UNetEngine(self.in_channels, self.out_channels, self.base_channels, self.precision,
                                          device)
            self._bound = None
        # (re)bind only when the storages may have moved: the flat parameter buffer and every buffer tensor are the
        # same objects as at the last bind (the dicts took ~0.5 ms of host time to rebuild per forward)
        bufs_now = tuple(self._buffers_list())
        key = (self._engine, self._flat_p, self._flat_g) + bufs_now
        if self._bound is None or len(self._bound) != len(key) or any(a is not b for a, b in zip(self._bound, key)):
            params = {k: p.data for k, p in self.named_parameters()}
            bufs = {k: b for k, b in self.named_buffers()}
            self._engine.bind(params, bufs, self._grad_views, watch=list(self.parameters()) + list(self.buffers()))
            self._bound = key
        return self._engine

    def _buffers_list(self):
        """The BatchNorm buffer tensors (their identity changes on .to() and on assignment)."""
        return [m._buffers[n] for m in self._bn_modules for n in ("running_mean", "running_var", "num_batches_tracked")]

    def _apply(self, fn, recurse=True):
        # .to()/.cuda()/.float() replace parameter storages: re-flatten lazily on next use
        out = super()._apply(fn, recurse)
        self._flat_p = None
        self.__dict__.pop("_trainable_cache", None)
        return out

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def calibrate(self, x: torch.Tensor):
        """precision="fp8": make this forward a calibration forward (its activations set the static e4m3 scales that
        the following forwards of this model state reuse). Returns the forward's (disparity, logvar). The engine also
        recalibrates by itself when a frame's input range outgrows the calibration frame's (UNetEngine._fp8_policy)."""
        if self.precision == "fp8":
            self.engine(x.device).request_calibration()
        return self.forward(x, return_uncertainty=True)

    def forward(self, x: torch.Tensor, return_uncertainty: bool = False):
        """model.py:79-104: returns softplus disparity [B,1,H,W] (and clamped logvar).
        precision="fp8" is the inference-only path (eval mode; outputs carry no autograd graph)."""
        eng = self.engine(x.device)
        if self.precision == "fp8" and self.training:
            raise RuntimeError("StereoUNet(precision='fp8') is inference-only (the live app's forward): call .eval()")
        # launches go to current_stream(eng.device); the guard keeps that device current (a model on cuda:1 while
        # cuda:0 is current, or engines of several devices in one process)
        with torch.cuda.device(eng.device):
            return self._forward(eng, x, return_uncertainty)

    def _forward(self, eng: UNetEngine, x: torch.Tensor, return_uncertainty: bool):
        if (self.precision != "fp8" and torch.is_grad_enabled()
                and any(p.requires_grad for p in self.parameters())):
            disp, logvar = _UNetFunction.apply(self, x, *[p for _, p in self._named_trainable()])
        else:
            B, _, H, W = x.shape
            eng.pack_weights(cached=not self.training, train=self.training)
            eng.forward(x, train=self.training)
            disp = torch.empty(B, 1, H, W, dtype=torch.float32, device=x.device)
            logvar = torch.empty_like(disp) if return_uncertainty else None
            eng.heads(L.SD_HEADS_INFER, disp=disp, logvar=logvar)
        if not return_uncertainty:
            return disp
        return disp, logvar
