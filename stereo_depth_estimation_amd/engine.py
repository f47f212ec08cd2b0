"""UNetEngine — drives the HIP kernels of libstereo_hip for one StereoUNet.

Replaces, for the reference's StereoUNet (model.py:48-104) and train step (train.py:320-343):
  forward   : 18 conv3x3 (+BN stats epilogue), 18 BN finalize, 4 ConvTranspose2d, heads
  backward  : heads+loss gradient, BN backward, ReLU/MaxPool backward, conv dgrad/wgrad,
              ConvTranspose2d dgrad/wgrad/bias-grad — hand-scheduled (no autograd graph)
All tensors are NHWC (``act_dtype`` = bf16 or fp32); parameters/grads/optimizer state are
fp32 in PyTorch layout.  precision="fp8" is the inference-only forward of the live app
(depth_live_dl.py:516-529): e4m3 3x3-conv weights and activations on the block-scaled
MFMA, dynamic per-layer activation scales computed on the device, bf16 activations in HBM.  Every launch goes on torch's current HIP stream, nothing syncs
the host, so a whole step can be captured into a HIP graph (torch.cuda.CUDAGraph).
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch

from . import _lib as L

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
BLOCKS_FWD = ("enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1")
LEVEL = {"enc1": 0, "enc2": 1, "enc3": 2, "enc4": 3, "bottleneck": 4, "dec4": 3, "dec3": 2, "dec2": 1, "dec1": 0}
UP_OF_DEC = {"dec4": "up4", "dec3": "up3", "dec2": "up2", "dec1": "up1"}
DEC_OF_UP = {u: d for d, u in UP_OF_DEC.items()}
SKIP_OF_DEC = {"dec4": "enc4", "dec3": "enc3", "dec2": "enc2", "dec1": "enc1"}
UP_SRC = {"up4": "bottleneck", "up3": "dec4", "up2": "dec3", "up1": "dec2"}
PREV_ENC = {"enc2": "enc1", "enc3": "enc2", "enc4": "enc3", "bottleneck": "enc4"}


def _r64(x: int) -> int:
    return (x + 63) // 64 * 64


def _r16(x: int) -> int:
    return (x + 15) // 16 * 16


@dataclass
class ConvL:
    name: str  # e.g. "enc1.0"
    blk: str
    idx: int  # 0 or 1 (conv within block)
    cin: int  # real input channels
    cin_pad: int
    cout: int
    level: int
    w_key: str
    bn_key: str
    kpad_f: int = 0
    kpad_d: int = 0
    off_f: int = 0
    off_d: int = -1
    kpad8: int = 0  # fp8 weights [cout][kpad8], k = tap*r16(cin_pad) + c
    off8: int = 0
    soff8: int = 0
    kpad_s: int = 0  # hi/lo split weights (wsplit layers): [cout][kpad_s] in UNetEngine.wsplit_pack, -1 offset: none
    off_s: int = -1


@dataclass
class UpL:
    name: str
    cin: int
    cout: int
    level: int  # level of the (low-res) input
    kpad_f: int = 0
    kpad_d: int = 0
    off_f: int = 0
    off_d: int = 0
    kpad_s: int = 0  # hi/lo split forward weights (wsplit layers), -1 offset: none
    off_s: int = -1


@dataclass
class Workspace:
    B: int
    H: int
    W: int
    train: bool  # backward buffers allocated
    t: dict = field(default_factory=dict)
    fwd_train: bool = True  # BN mode of the last forward (batch stats vs running stats)
    coeff_key: object = None  # state key the eval-mode BN coefficients in t were computed for
    slab_off: dict = field(default_factory=dict)  # deferred reduces: each weight gradient's slab region (floats)
    q8_ready: bool = False  # fp8: the activation scales of a calibration forward are in t
    graph: object = None  # HIP graph of the eval forward (after the input pack) for graph_key = (state key, path)
    graph_key: object = None
    graph_zs: frozenset = frozenset()  # the layers whose stored output the captured body BN-applied (engine._zs)


class UNetEngine:
    def __init__(self, in_channels=6, out_channels=1, base_channels=32, precision="bf16", device=None):
        if base_channels % 8 != 0:
            raise ValueError(f"base_channels={base_channels}: the HIP path needs a multiple of 8")
        if out_channels != 1:
            raise ValueError("out_channels must be 1 (disparity head)")
        if precision not in ("bf16", "fp32", "fp8"):
            raise ValueError(f"precision={precision!r}: expected 'bf16', 'fp32' or 'fp8' (inference only)")
        self.in_channels, self.base = in_channels, base_channels
        self.precision = precision
        # bumped by every device-side write to the parameters or BN buffers that PyTorch's version counters
        # cannot see (the AdamW kernel, train-mode running statistics): eval forwards reuse packed weights
        # and BN coefficients while (epoch, storages, versions) is unchanged
        self.state_epoch = 0
        self._packed_key = None
        self._split_pack_jobs = None
        self._eval_coeffs = True
        self.fp8 = precision == "fp8"  # bf16 activations, e4m3 3x3 convs (eval forward only)
        # fp8: static activation scales from a calibration forward per model state (SD_FP8_STATIC=0: dynamic always)
        self.fp8_static = os.environ.get("SD_FP8_STATIC", "1") != "0"
        # fp8 recalibration triggers (_fp8_policy): input amax above margin x the calibration frame's, and age
        self.fp8_range_margin = float(os.environ.get("SD_FP8_RANGE_MARGIN", "1.25"))
        self.fp8_recalib_every = int(os.environ.get("SD_FP8_RECALIB_EVERY", "0"))
        self.fp8_calibrations = self.fp8_range_recalibrations = self._fp8_age = self._fp8_frame = 0
        self._amax_dev: torch.Tensor | None = None  # [3] max |x| of the last frames' inputs (float bits), a ring
        self._amax_host: torch.Tensor | None = None  # pinned copies
        self._amax_ev: list = [None, None, None]
        self._amax_used: list = [False, False, False]
        self._amax_checked: list = [True, True, True]  # whether _fp8_policy has compared that word's read-back
        self._amax_packed = None
        self._amax_pending: int | None = None
        self._fp8_cal = None  # (slot, event) of the calibration frame's amax
        self._fp8_cal_amax: float | None = None
        # eval forwards of an unchanged state replay a captured HIP graph (SD_EVAL_GRAPH=0: eager launches)
        self.eval_graphs = os.environ.get("SD_EVAL_GRAPH", "1") != "0"
        self.sd_dtype = L.SD_F32 if precision == "fp32" else L.SD_BF16
        self.act_dtype = torch.float32 if precision == "fp32" else torch.bfloat16
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        L.load()
        c = [base_channels * (1 << i) for i in range(5)]
        self.cin_pad0 = (in_channels + 7) // 8 * 8
        bc = {
            "enc1": (in_channels, c[0]), "enc2": (c[0], c[1]), "enc3": (c[1], c[2]), "enc4": (c[2], c[3]),
            "bottleneck": (c[3], c[4]), "dec4": (2 * c[3], c[3]), "dec3": (2 * c[2], c[2]),
            "dec2": (2 * c[1], c[1]), "dec1": (2 * c[0], c[0]),
        }
        self.convs: dict[str, ConvL] = {}
        off = 0
        for blk in BLOCKS_FWD:
            cin, cout = bc[blk]
            for idx, (ci, wk, bk) in enumerate(((cin, 0, 1), (cout, 3, 4))):
                cp = self.cin_pad0 if (blk == "enc1" and idx == 0) else ci
                cl = ConvL(f"{blk}.{idx}", blk, idx, ci, cp, cout, LEVEL[blk], f"{blk}.block.{wk}.weight", f"{blk}.block.{bk}")
                cl.kpad_f = _r64(9 * cp)
                cl.off_f = off
                off += cout * cl.kpad_f
                if not (blk == "enc1" and idx == 0):
                    cl.kpad_d = _r64(9 * cout)
                    cl.off_d = off
                    off += ci * cl.kpad_d
                self.convs[cl.name] = cl
        self.ups: dict[str, UpL] = {}
        for k, lvl in (("up4", 4), ("up3", 3), ("up2", 2), ("up1", 1)):
            cin, cout = c[lvl], c[lvl - 1]
            u = UpL(k, cin, cout, lvl, _r64(cin), _r64(4 * cout))
            u.off_f = off
            off += 4 * cout * u.kpad_f
            u.off_d = off
            off += cin * u.kpad_d
            self.ups[k] = u
        self.wpack = torch.zeros(off, dtype=self.act_dtype, device=self.device)
        # hi/lo split weights for the bf16 (and fp8's bf16 layers') EVAL forwards: the bf16 rounding of the weights is
        # a systematic change of the function, and on reference-trained checkpoints it shifted the EPE by 2e-3..1e-2 px
        # (enc1.0 most: its raw-image input has |mean|/std ~ 4.6; on a better-trained model the deeper layers' share
        # grows); with every weight as a hi + lo pair the shift over 32 held-out pairs is ~2e-4 px, what remains is the
        # zero-mean noise of the bf16 activations (tools/precision_study.py). The training forward keeps
        # plain bf16 weights (the EPE is an eval-mode quantity). SD_WSPLIT=all (default) | fullres (the level-0 layers
        # only) | 0 (off); SD_WSPLIT_TRAIN=1: in the training forward too.
        # eval forwards of the bf16 path store z = scale*y + shift (the eval BatchNorm applied in the conv epilogue,
        # sd_conv3x3_ex out_scale/out_shift) instead of y, so bf16's relative precision sits on the normalised value
        # (tools/precision_study.py: the per-batch EPE noise of the bf16 activations 1.5e-3 -> 5.4e-4 px, what fp32
        # storage of y would give); consumers then apply only the ReLU. SD_ZSTORE=0: store y.
        self.zstore = precision == "bf16" and os.environ.get("SD_ZSTORE", "1") != "0"
        self._zs: set = set()
        # the current forward may be backpropagated (forward(need_backward=True): an eval-mode forward through
        # autograd, e.g. frozen-BatchNorm fine-tuning): no BN-applied stores then, since the backward reads the raw y
        self._zs_ok = True
        self._one = torch.ones(16 * base_channels, dtype=torch.float32, device=self.device)
        self._zero = torch.zeros(16 * base_channels, dtype=torch.float32, device=self.device)
        mode = os.environ.get("SD_WSPLIT", "all")
        self.wsplit = precision == "bf16" and mode != "0"  # fp8: e4m3 dominates its error (measured: no gain)
        self.wsplit_train = self.wsplit and os.environ.get("SD_WSPLIT_TRAIN", "0") == "1"
        self.wsplit_eval = True  # per-instance switch (bench.py times the bf16 eval forward both ways)
        offs = 0
        if self.wsplit:
            for cl in self.convs.values():
                if (cl.level == 0 or mode != "fullres") and (cl.cout == 32 or cl.cout % 64 == 0):  # halo shapes
                    cl.kpad_s, cl.off_s = _r64(18 * cl.cin_pad), offs
                    offs += cl.cout * cl.kpad_s
            for u in self.ups.values():
                if u.name == "up1" or mode != "fullres":
                    u.kpad_s, u.off_s = _r64(2 * u.cin), offs
                    offs += 4 * u.cout * u.kpad_s
        self.wsplit_pack = torch.zeros(max(offs, 1), dtype=torch.bfloat16, device=self.device)
        if self.fp8:
            off8 = soff = 0
            for cl in self.convs.values():
                cl.kpad8 = _r64(9 * _r16(cl.cin_pad))
                cl.off8, cl.soff8 = off8, soff
                off8 += cl.cout * cl.kpad8
                soff += cl.cout
            self.wq8 = torch.zeros(off8, dtype=torch.uint8, device=self.device)
            self.wscale8 = torch.zeros(soff, dtype=torch.float32, device=self.device)
        self.c1 = c[0]
        # sd_conv3x3_q8's shapes (N = 32 or a multiple of 64, <= 512 input channels): base_channels 32 and its multiples
        self._q8_shapes = all((cl.cout == 32 or cl.cout % 64 == 0) and cl.cin_pad <= 512 for cl in self.convs.values()) \
            and all(u.cout % 16 == 0 for u in self.ups.values())
        # persistent small device state
        dev = self.device
        # this rank's valid pixels (metric sums) and the loss normaliser, two ints of one buffer that sd_count_valid
        # fills together (ncount=2); DDP all-reduces `count` alone to the global count (ddp.DataParallel), so the two
        # never alias and nothing has to copy one into the other. Two slots of them, alternating per batch: the count
        # kernel fills one (zero) and zeroes the other for the next batch, so no memset launch precedes it
        self._counts = torch.zeros(2, 2, dtype=torch.int32, device=dev)
        self._cslot = 0
        self.count_local = self._counts[0, 0:1]
        self.count = self._counts[0, 1:2]
        self.metrics = torch.zeros(5, dtype=torch.float64, device=dev)
        self.adam_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.adam_scratch = torch.zeros(4, dtype=torch.float32, device=dev)
        self.ws: Workspace | None = None
        # bf16 training: BatchNorm-backward apply fused into the weight gradients (SD_BN_FUSE=0: separate pass)
        self.bn_fuse = os.environ.get("SD_BN_FUSE", "1") != "0"
        # bf16 training: ConvTranspose2d bias gradients from the decoder dgrad epilogue (SD_BIAS_FUSE=0: own pass)
        self.bias_fuse = os.environ.get("SD_BIAS_FUSE", "1") != "0"
        # bf16 training: the BatchNorm-backward sums of a block's conv0 from its conv1 dgrad epilogue
        # (sd_conv_gemm_bnsum; SD_BNSUM_FUSE=0: sd_bn_bwd_reduce pass)
        self.bnsum_fuse = os.environ.get("SD_BNSUM_FUSE", "1") != "0"
        # bf16 training: the whole backward of the full-resolution 32 -> 32 conv1 layers (enc1.1, dec1.1) in one pass
        # (sd_conv3x3_bwd_fused / _dec: dy stays in LDS; SD_BWD_FUSE=0: weight gradient + dgrad launches;
        # SD_BWD_FUSE=1: the conv1 layers only)
        self.bwd_fuse = {"0": 0, "1": 1}.get(os.environ.get("SD_BWD_FUSE", "2"), 2)
        # train step: the valid count, the weight packs and the input pack in one launch (step_prologue;
        # SD_PROLOGUE=0: three launches)
        self.prologue = os.environ.get("SD_PROLOGUE", "1") != "0"
        self._bnsum_rows: dict[str, int] = {}
        # training: the split-K slab reduce of every weight gradient on a second stream (SD_SIDE_REDUCE=1), so it
        # overlaps the next layer's kernels instead of adding a kernel boundary to the critical path; 2: the
        # weight-gradient GEMMs that nothing downstream reads (no fused dy) on that stream too. Two slabs
        # alternate; an event per slab orders its reuse. 0: everything on the current stream.
        self.side_mode = int(os.environ.get("SD_SIDE_REDUCE", "0"))
        # training: every weight gradient gets its own slab region and the split-K reduces are deferred and run as ONE
        # launch per gradient-ready group (sd_wgrad_reduce_batch: once per step single-process, once per top-level
        # module under DDP) instead of one launch per weight; bit-identical sums (SD_DEFER_REDUCE=0: per weight)
        self.defer_reduce = os.environ.get("SD_DEFER_REDUCE", "1") != "0" and not self.side_mode
        self._red_jobs: list = []
        self._side: torch.cuda.Stream | None = None
        self._slab_free: list = [None, None]
        self._slab_i = 0
        # SyncBatchNorm (ddp.DataParallel(sync_bn=True)): bn_sync(t) SUM-all-reduces an fp64 device tensor in stream
        # order (the per-channel sums and each rank's pixel count). None: per-rank BatchNorm statistics.
        self.bn_sync = None
        self._bn64: torch.Tensor | None = None
        self.params: dict[str, torch.Tensor] = {}
        self.grads: dict[str, torch.Tensor] = {}
        self.bufs: dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ binding
    def bind(self, params: dict, bufs: dict, grads: dict | None = None, watch: list | None = None):
        """params/bufs/grads: state_dict-keyed fp32 device tensors (PyTorch layouts). watch: the tensors
        whose version counters reveal in-place edits made through PyTorch (the module's Parameters and
        buffers; `.data` aliases carry counters of their own)."""
        self.params, self.bufs = params, bufs
        self.grads = grads or {}
        self._watch = watch if watch is not None else list(params.values()) + list(bufs.values())
        # fixed per bind: whether any watched tensor is an inference tensor (no version counter), and the storages
        # (a rebind means new storages; _state_key then only reads the version counters: ~15 us instead of ~70)
        self._watch_inference = any(t.is_inference() for t in self._watch)
        self._bind_id = getattr(self, "_bind_id", 0) + 1
        self._buf_list = list(bufs.values())

    def _s(self):
        return L.stream_handle(self.device)

    def touch_state(self):
        """Parameters or BN buffers were written outside PyTorch's view (kernels, collectives)."""
        self.state_epoch += 1

    def _state_key(self):
        """None when the state cannot be tracked (inference tensors carry no version counter)."""
        if self._watch_inference:
            return None
        # the BN buffers' storages too: a `.data` swap keeps the tensor object (and its version counter) but moves the
        # storage, which a bind() would not notice (the parameters live in the flat buffer, whose moves rebind)
        return (self.state_epoch, self._bind_id, tuple([t._version for t in self._watch]),
                tuple([b.data_ptr() for b in self._buf_list]))

    def pack_weights(self, cached: bool = False, train: bool = False):
        """Pack the weights into the kernels' layouts. cached=True (eval-mode inference): skip when the
        parameters are unchanged since the last pack (the live app's forward repeats on fixed weights).
        train=True: the next forward is a training forward, which reads no hi/lo split weights (unless
        SD_WSPLIT_TRAIN=1), so their pack (a second launch, ~28 us at B=64) is left for the next eval forward."""
        key = self._state_key() if cached else None
        if key is not None and key == self._packed_key:
            return
        self._packed_key = key
        dt, s = self.sd_dtype, self._s()
        base = self.wpack.data_ptr()
        es = self.wpack.element_size()
        if self.fp8:  # e4m3 3x3 weights with per-output-channel scales; ConvTranspose stays bf16
            for cl in self.convs.values():
                L.call("sd_pack_conv3_w_fp8", self.params[cl.w_key].data_ptr(), cl.cout, cl.cin, cl.cin_pad, cl.kpad8,
                       self.wq8.data_ptr() + cl.off8, self.wscale8.data_ptr() + 4 * cl.soff8, s)
                if self._q8_bf16(cl):  # the static forward's bf16 layers
                    L.call("sd_pack_conv3_w", dt, self.params[cl.w_key].data_ptr(), cl.cout, cl.cin, cl.cin_pad, 0,
                           cl.kpad_f, base + cl.off_f * es, s)
            for u in self.ups.values():
                L.call("sd_pack_convT_w", dt, self.params[u.name + ".weight"].data_ptr(), u.cin, u.cout, 0, u.kpad_f,
                       base + u.off_f * es, s)
            jobs = self._split_jobs()
            if jobs:
                arr = (L.SdPackJob * len(jobs))(*[L.SdPackJob(*j) for j in jobs])
                L.call("sd_pack_weights", L.SD_BF16, arr, len(jobs), self.wsplit_pack.data_ptr(), s)
            return
        # every bf16/fp32 pack of the step in one launch (job table rebuilt when the parameters move)
        jobs = self._pack_table()
        L.call("sd_pack_weights", dt, jobs, len(jobs), base, s)
        if self._split_pack_jobs is not None and (not train or self.wsplit_train):
            L.call("sd_pack_weights", L.SD_BF16, self._split_pack_jobs, len(self._split_pack_jobs),
                   self.wsplit_pack.data_ptr(), s)

    def _pack_table(self):
        """The bf16/fp32 sd_pack_weights job table of every layer (and the split-pack table), rebuilt when the
        parameters move."""
        key = tuple(t.data_ptr() for t in self.params.values())
        if getattr(self, "_pack_key", None) != key:
            jobs = []
            for cl in self.convs.values():
                w = self.params[cl.w_key].data_ptr()
                jobs.append((w, L.SD_PACK_CONV3_FWD, cl.cout, cl.cin, cl.cin_pad, cl.kpad_f, cl.off_f))
                if cl.off_d >= 0:
                    jobs.append((w, L.SD_PACK_CONV3_DGRAD, cl.cout, cl.cin, cl.cin, cl.kpad_d, cl.off_d))
            for u in self.ups.values():
                w = self.params[u.name + ".weight"].data_ptr()
                jobs.append((w, L.SD_PACK_CONVT_FWD, u.cout, u.cin, u.cin, u.kpad_f, u.off_f))
                jobs.append((w, L.SD_PACK_CONVT_DGRAD, u.cout, u.cin, u.cin, u.kpad_d, u.off_d))
            self._pack_jobs = (L.SdPackJob * len(jobs))(*[L.SdPackJob(*j) for j in jobs])
            sj = self._split_jobs()
            self._split_pack_jobs = (L.SdPackJob * len(sj))(*[L.SdPackJob(*j) for j in sj]) if sj else None
            self._pack_key = key
        return self._pack_jobs

    def step_prologue(self, x: torch.Tensor, target: torch.Tensor, valid: torch.Tensor, train: bool) -> bool:
        """count_valid(target, valid) + pack_weights(train=train) + the next forward(x)'s input pack as ONE launch
        (sd_step_prologue: three independent jobs that were three kernel boundaries). Returns False, having launched
        nothing, where it does not apply (the fp8 forward, SD_PROLOGUE=0, an input that is not a contiguous fp32 NCHW
        batch of this model, targets or mask not aligned for the vector count): the caller then makes the three
        calls."""
        if (self.fp8 or not self.prologue or x.dim() != 4 or x.shape[1] != self.in_channels or not x.is_contiguous()
                or x.dtype != torch.float32 or x.shape[2] % 16 or x.shape[3] % 16 or target.data_ptr() % 16
                or valid.data_ptr() % 4 or target.numel() != valid.numel()):
            return False
        B, C, H, W = x.shape
        ws = self.workspace(B, H, W, train)
        k = self._count_slot()
        jobs = self._pack_table()
        s = self._s()
        self._packed_key = None
        L.call("sd_step_prologue", self.sd_dtype, jobs, len(jobs), self.wpack.data_ptr(), x.data_ptr(), B, C, H, W,
               self.cin_pad0, ws.t["xin"].data_ptr(), target.data_ptr(), valid.data_ptr(), target.numel(),
               self._counts[k].data_ptr(), 2, self._counts[k ^ 1].data_ptr(), s)
        if self._split_pack_jobs is not None and (not train or self.wsplit_train):
            L.call("sd_pack_weights", L.SD_BF16, self._split_pack_jobs, len(self._split_pack_jobs),
                   self.wsplit_pack.data_ptr(), s)
        self._xin_ready = (x.data_ptr(), tuple(x.shape), ws.t["xin"].data_ptr())
        return True

    def _split_jobs(self) -> list:
        """sd_pack_weights jobs of the hi/lo split weights (wsplit layers)."""
        if not self.wsplit:
            return []
        jobs = []
        for cl in self.convs.values():
            if cl.off_s >= 0:
                jobs.append((self.params[cl.w_key].data_ptr(), L.SD_PACK_CONV3_FWD_SPLIT, cl.cout, cl.cin, cl.cin_pad,
                             cl.kpad_s, cl.off_s))
        for u in self.ups.values():
            if u.off_s >= 0:
                jobs.append((self.params[u.name + ".weight"].data_ptr(), L.SD_PACK_CONVT_FWD_SPLIT, u.cout, u.cin, u.cin,
                             u.kpad_s, u.off_s))
        return jobs

    def _ws_ptr(self, off: int) -> int:
        return self.wsplit_pack.data_ptr() + 2 * off

    def _use_wsplit(self, layer, train: bool) -> bool:
        return layer.off_s >= 0 and self.wsplit_eval and (not train or self.wsplit_train)

    def _wp(self, off: int) -> int:
        return self.wpack.data_ptr() + off * self.wpack.element_size()

    # ------------------------------------------------------------------ workspace
    def workspace(self, B: int, H: int, W: int, train: bool) -> Workspace:
        if H % 16 or W % 16:
            raise ValueError(f"H={H}, W={W}: StereoUNet needs H and W divisible by 16 (model.py:59,83-95)")
        ws = self.ws
        if ws is not None and (ws.B, ws.H, ws.W) == (B, H, W) and (ws.train or not train):
            return ws
        ws = Workspace(B, H, W, train)
        dev, adt, dt = self.device, self.act_dtype, self.sd_dtype
        f32 = torch.float32

        def act(level, ch):
            return torch.empty(B * (H >> level) * (W >> level), ch, dtype=adt, device=dev)

        t = ws.t
        t["xin"] = act(0, self.cin_pad0)
        max_stat = 0
        for cl in self.convs.values():
            P = B * (H >> cl.level) * (W >> cl.level)
            t["y:" + cl.name] = act(cl.level, cl.cout)
            for k in ("mean", "invstd", "scale", "shift"):
                t[f"{k}:{cl.name}"] = torch.empty(cl.cout, dtype=f32, device=dev)
            rows = L.call("sd_conv_gemm_stat_rows", dt, B, H >> cl.level, W >> cl.level, cl.cout)
            max_stat = max(max_stat, rows * cl.cout * 2)
            if train and cl.blk in UP_OF_DEC and cl.idx == 0:  # dgrad SPLIT_STATS rows (ConvTranspose bias grad)
                rows = L.call("sd_conv_gemm_stat_rows", dt, B, H >> cl.level, W >> cl.level, cl.cin)
                max_stat = max(max_stat, rows * cl.cin * 2)
                # or the fused dec1.0 backward's d(up) column-sum rows (sd_conv3x3_bwd_fused_dec)
                max_stat = max(max_stat, L.call("sd_conv3x3_bwd_fused_splits", B, H, W) * 32 * 2)
        t["stats"] = torch.empty(max_stat, dtype=f32, device=dev)
        for u in self.ups.values():
            t["u:" + u.name] = act(u.level - 1, u.cout)
        if self.sd_dtype == L.SD_BF16:
            for blk in ("enc1", "enc2", "enc3", "enc4"):
                cl = self.convs[blk + ".1"]
                t["pool:" + cl.name] = act(cl.level + 1, cl.cout)
            # split-K partials of the eval convs (sd_conv3x3_ex_ws: the batch-1 shapes of the deep layers)
            hws = 0
            for cl in self.convs.values():
                ch = self._fp8_src_chans(cl) + (0,)
                dummy = L.make_src(None, ch[0], H >> cl.level, W >> cl.level, taps=9, c1=ch[1])
                for flags in (0, L.SD_CONV_WSPLIT) if cl.off_s >= 0 else (0,):  # wsplit_eval may change later
                    hws = max(hws, L.call("sd_conv3x3_ex_ws_bytes", dummy, B, H >> cl.level, W >> cl.level, cl.cout,
                                          L.SD_EPI_STORE, flags))
            t["hws"] = torch.empty(max(hws // 4, 4), dtype=f32, device=dev)
        if self.fp8:
            if train:
                raise RuntimeError("precision='fp8' is the inference-only forward (BASELINE config 5): no training")
            for cl in self.convs.values():
                rows = L.call("sd_conv3x3_fp8_rows", B, H >> cl.level, W >> cl.level, cl.cout)
                t["mm:" + cl.name] = torch.empty(rows, cl.cout, 2, dtype=f32, device=dev)
                t["as:" + cl.name] = torch.empty(1, dtype=f32, device=dev)
                for k, ch in enumerate(self._fp8_src_chans(cl)):
                    t[f"qs{k}:{cl.name}"] = torch.empty(ch, dtype=f32, device=dev)
                    t[f"qh{k}:{cl.name}"] = torch.empty(ch, dtype=f32, device=dev)
            t["mm:xin"] = torch.empty(L.call("sd_chan_minmax_rows", B * H * W, self.cin_pad0), self.cin_pad0, 2,
                                      dtype=f32, device=dev)
            for u in self.ups.values():
                P = B * (H >> (u.level - 1)) * (W >> (u.level - 1))
                t["mm:" + u.name] = torch.empty(L.call("sd_chan_minmax_rows", P, u.cout), u.cout, 2, dtype=f32,
                                                device=dev)
        if train:
            max_chan = max_slab = 0
            for cl in self.convs.values():
                lv = cl.level
                P = B * (H >> lv) * (W >> lv)
                t["da:" + cl.name] = act(lv, cl.cout)
                t["dy:" + cl.name] = act(lv, cl.cout)
                t["coef:" + cl.name] = torch.empty(cl.cout, 3, dtype=f32, device=dev)
                max_chan = max(max_chan, L.call("sd_chan_reduce_rows", P, cl.cout) * cl.cout * 2)
                if self._bwd_fused(cl, H, W) == 1:  # sd_conv3x3_bwd_fused: splits x 32 (sum, sum*xhat) partials
                    max_chan = max(max_chan, L.call("sd_conv3x3_bwd_fused_splits", B, H >> lv, W >> lv) * 32 * 2)
                sp = self._conv_splits(cl, B, H, W)
                max_slab = max(max_slab, sp * cl.cout * 9 * cl.cin_pad)
            for u in self.ups.values():
                lv = u.level
                t["du:" + u.name] = act(lv - 1, u.cout)
                t["dskip:" + u.name] = act(lv - 1, u.cout)
                P = B * (H >> (lv - 1)) * (W >> (lv - 1))
                max_chan = max(max_chan, L.call("sd_chan_reduce_rows", P, u.cout) * u.cout * 2)
                sp = L.call("sd_wgrad_splits", dt, B, H >> lv, W >> lv, u.cin, 4 * u.cout)
                max_slab = max(max_slab, sp * u.cin * 4 * u.cout)
                # BatchNorm-backward rows of the ConvTranspose dgrad (sd_conv_gemm_bnsum)
                dsrc = L.make_src(t["du:" + u.name], u.cout, H >> (lv - 1), W >> (lv - 1), taps=4)
                if L.call("sd_conv_gemm_bnsum_ok", dt, dsrc, u.cin) == 1:
                    rows = L.call("sd_conv_gemm_bnsum_rows", dsrc, B, H >> lv, W >> lv, u.cin)
                    max_chan = max(max_chan, rows * u.cin * 2)
            for blk in ("enc2", "enc3", "enc4", "bottleneck"):
                prev = self.convs[PREV_ENC[blk] + ".1"]
                t["dpool:" + blk] = act(prev.level + 1, prev.cout)
                if self._pool_bn_fused(prev):
                    rows = L.call("sd_pool_bwd_rows", B, H >> prev.level, W >> prev.level, prev.cout)
                    max_chan = max(max_chan, rows * prev.cout * 2)
            max_chan = max(max_chan, L.call("sd_heads_rows", B * H * W) * self.convs["dec1.1"].cout * 2)
            t["chan"] = torch.empty(max_chan, dtype=f32, device=dev)
            if self.defer_reduce:  # one region per weight gradient (deferred reduces): ~0.7 GB at B=64, 320x240
                ws.slab_off = {}
                tot = 0
                for cl in self.convs.values():
                    sp = self._conv_splits(cl, B, H, W)
                    ws.slab_off[cl.name] = tot
                    tot += _r16(sp * cl.cout * 9 * cl.cin_pad)
                for u in self.ups.values():
                    lv = u.level
                    sp = L.call("sd_wgrad_splits", dt, B, H >> lv, W >> lv, u.cin, 4 * u.cout)
                    ws.slab_off[u.name] = tot
                    tot += _r16(sp * u.cin * 4 * u.cout)
                    # the statistics rows of d(up) the decoder dgrad leaves for this layer's bias gradient, summed in
                    # the deferred batch (an SD_W_ROWSUM job) instead of a launch of their own
                    dec0 = self.convs[DEC_OF_UP[u.name] + ".0"]
                    Hd, Wd = H >> dec0.level, W >> dec0.level
                    rows = L.call("sd_conv_gemm_stat_rows", dt, B, Hd, Wd, dec0.cin) * dec0.cin * 2
                    rows = max(rows, L.call("sd_conv3x3_bwd_fused_splits", B, Hd, Wd) * 32 * 2)
                    ws.slab_off["brows:" + u.name] = tot
                    tot += _r16(rows)
                max_slab = tot
            t["slab"] = torch.empty(max_slab, dtype=f32, device=dev)
            if self.side_mode:
                t["slab1"] = torch.empty(max_slab, dtype=f32, device=dev)
                self._slab_free = [None, None]
            P0 = B * H * W
            t["heads_part"] = torch.empty(L.call("sd_heads_rows", P0) * (2 * self.c1 + 7), dtype=f32, device=dev)
        self.ws = ws
        return ws

    def _bwd_fused(self, cl: ConvL, H: int, W: int) -> int:
        """Whether conv `cl`'s backward runs as one fused pass (bf16 training, at a tiling the kernels take):
        1: sd_conv3x3_bwd_fused, a 32 -> 32 conv1 whose input is its block's conv0 output (enc1.1, dec1.1);
        2: sd_conv3x3_bwd_fused_dec, a decoder conv0 on cat(32-channel up, 32-channel skip) -> 32 (dec1.0)."""
        if not self.bwd_fuse or self.sd_dtype != L.SD_BF16:
            return 0
        Hl, Wl = H >> cl.level, W >> cl.level
        if cl.idx == 1 and cl.cout == 32 and cl.cin == 32 and self.bnsum_fuse:
            return 1 if L.call("sd_conv3x3_bwd_fused_ok", cl.cout, cl.cin, Hl, Wl) == 1 else 0
        if cl.idx == 0 and cl.blk in UP_OF_DEC and self.bwd_fuse >= 2:
            up, sk = self.ups[UP_OF_DEC[cl.blk]], self.convs[SKIP_OF_DEC[cl.blk] + ".1"]
            if cl.cin == up.cout + sk.cout and L.call("sd_conv3x3_bwd_fused_dec_ok", cl.cout, up.cout, sk.cout, Hl,
                                                      Wl) == 1:
                return 2
        return 0

    def _conv_splits(self, cl: ConvL, B: int, H: int, W: int) -> int:
        """Split-K slabs of conv `cl`'s weight gradient (its slab region holds the larger of the two kernels')."""
        lv = cl.level
        sp = L.call("sd_wgrad_splits", self.sd_dtype, B, H >> lv, W >> lv, cl.cout, 9 * cl.cin_pad)
        if self._bwd_fused(cl, H, W):
            sp = max(sp, L.call("sd_conv3x3_bwd_fused_splits", B, H >> lv, W >> lv))
        return sp

    # ------------------------------------------------------------------ forward
    def _bn(self, cl: ConvL):
        """The affine its consumers apply (before the ReLU) to conv `cl`'s stored output: the BatchNorm's (scale,
        shift), or the identity when the eval forward stored z = scale*y + shift already (self._zs)."""
        t = self.ws.t
        if cl.name in self._zs:
            return (self._one[:cl.cout], self._zero[:cl.cout])
        return (t["scale:" + cl.name], t["shift:" + cl.name])

    def _src_fwd(self, cl: ConvL) -> L.SdSrc:
        """The gather feeding conv `cl` (model.py:79-95 dataflow)."""
        ws, t = self.ws, self.ws.t
        Hl, Wl = ws.H >> cl.level, ws.W >> cl.level
        if cl.name == "enc1.0":
            return L.make_src(t["xin"], self.cin_pad0, Hl, Wl, taps=9)
        if cl.idx == 1:
            prev = self.convs[cl.blk + ".0"]
            return L.make_src(t["y:" + prev.name], prev.cout, Hl, Wl, taps=9, bn0=self._bn(prev))
        if cl.blk in PREV_ENC:  # pooled encoder input
            prev = self.convs[PREV_ENC[cl.blk] + ".1"]
            if self.sd_dtype == L.SD_BF16:  # materialised by _pool_fwd (sd_bnrelu_pool)
                return L.make_src(t["pool:" + prev.name], prev.cout, Hl, Wl, taps=9)
            return L.make_src(t["y:" + prev.name], prev.cout, 2 * Hl, 2 * Wl, taps=9, pool=True, bn0=self._bn(prev))
        # decoder conv0: cat([up, skip]) (model.py:89-95)
        up = self.ups[UP_OF_DEC[cl.blk]]
        sk = self.convs[SKIP_OF_DEC[cl.blk] + ".1"]
        return L.make_src(
            t["u:" + up.name], up.cout, Hl, Wl, taps=9, src1=t["y:" + sk.name], c1=sk.cout, bn1=self._bn(sk)
        )

    def _conv_fwd(self, cl: ConvL, train: bool):
        ws, t, s, dt = self.ws, self.ws.t, self._s(), self.sd_dtype
        Hl, Wl = ws.H >> cl.level, ws.W >> cl.level
        src = self._src_fwd(cl)
        y = t["y:" + cl.name]
        g, b = self.params[cl.bn_key + ".weight"], self.params[cl.bn_key + ".bias"]
        mean, invstd = t["mean:" + cl.name], t["invstd:" + cl.name]
        scale, shift = t["scale:" + cl.name], t["shift:" + cl.name]
        split = self._use_wsplit(cl, train) and dt == L.SD_BF16
        if train:
            stats = t["stats"]
            if split:
                L.call("sd_conv3x3_ex", src, ws.B, Hl, Wl, self._ws_ptr(cl.off_s), cl.cout, cl.kpad_s,
                       L.SD_EPI_STATS, L.SD_CONV_WSPLIT, None, None, y.data_ptr(), stats.data_ptr(), s)
            else:
                L.call("sd_conv_gemm", dt, src, ws.B, Hl, Wl, self._wp(cl.off_f), cl.cout, cl.kpad_f, L.SD_EPI_STATS,
                       y.data_ptr(), None, 0, None, stats.data_ptr(), s)
            rows = L.call("sd_conv_gemm_stat_rows", dt, ws.B, Hl, Wl, cl.cout)
            rm, rv = self.bufs[cl.bn_key + ".running_mean"], self.bufs[cl.bn_key + ".running_var"]
            nbt = self.bufs.get(cl.bn_key + ".num_batches_tracked")
            if self.bn_sync is not None:  # global batch statistics (torch SyncBatchNorm) over the global count
                sums = self._sync_sums(stats, rows, cl.cout, ws.B * Hl * Wl)[0]
                L.call("sd_bn_fwd_finalize64", sums.data_ptr(), cl.cout, g.data_ptr(), b.data_ptr(), rm.data_ptr(),
                       rv.data_ptr(), L.ptr(nbt), BN_MOMENTUM, BN_EPS,
                       mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), s)
            else:
                L.call("sd_bn_fwd_finalize", stats.data_ptr(), rows, cl.cout, float(ws.B * Hl * Wl), g.data_ptr(),
                       b.data_ptr(), rm.data_ptr(), rv.data_ptr(), L.ptr(nbt), BN_MOMENTUM, BN_EPS, mean.data_ptr(),
                       invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), s)
        else:
            if self._eval_coeffs:  # before the conv: an affine epilogue (zstore) stores with them
                rm, rv = self.bufs[cl.bn_key + ".running_mean"], self.bufs[cl.bn_key + ".running_var"]
                L.call("sd_bn_eval_coeffs", rm.data_ptr(), rv.data_ptr(), g.data_ptr(), b.data_ptr(), cl.cout,
                       BN_EPS, mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), s)
            zs = self.zstore and self._zs_ok and dt == L.SD_BF16 and L.call("sd_conv3x3_ex_ok", src, cl.cout) == 1
            if split or zs:
                hws = t["hws"]
                L.call("sd_conv3x3_ex_ws", src, ws.B, Hl, Wl, self._ws_ptr(cl.off_s) if split else self._wp(cl.off_f),
                       cl.cout, cl.kpad_s if split else cl.kpad_f, L.SD_EPI_STORE, L.SD_CONV_WSPLIT if split else 0,
                       scale.data_ptr() if zs else None, shift.data_ptr() if zs else None, y.data_ptr(), None,
                       hws.data_ptr(), 4 * hws.numel(), s)
                if zs:
                    self._zs.add(cl.name)
            else:
                L.call("sd_conv_gemm", dt, src, ws.B, Hl, Wl, self._wp(cl.off_f), cl.cout, cl.kpad_f, L.SD_EPI_STORE,
                       y.data_ptr(), None, 0, None, None, s)

    def _up_fwd(self, u: UpL, train: bool = True):
        ws, t, s, dt = self.ws, self.ws.t, self._s(), self.sd_dtype
        src_cl = self.convs[UP_SRC[u.name] + ".1"]
        Hl, Wl = ws.H >> u.level, ws.W >> u.level
        if self._use_wsplit(u, train) and dt == L.SD_BF16:
            # hi/lo split weights: the source twice along K, against [hi | lo] (the generic 1x1 GEMM's two sources)
            y, bn = t["y:" + src_cl.name], self._bn(src_cl)
            src = L.make_src(y, src_cl.cout, Hl, Wl, taps=1, bn0=bn, src1=y, c1=src_cl.cout, bn1=bn)
            L.call("sd_conv_gemm", dt, src, ws.B, Hl, Wl, self._ws_ptr(u.off_s), 4 * u.cout, u.kpad_s,
                   L.SD_EPI_PIXSHUF, t["u:" + u.name].data_ptr(), None, 0, self.params[u.name + ".bias"].data_ptr(),
                   None, s)
            return
        src = L.make_src(t["y:" + src_cl.name], src_cl.cout, Hl, Wl, taps=1, bn0=self._bn(src_cl))
        L.call("sd_conv_gemm", dt, src, ws.B, Hl, Wl, self._wp(u.off_f), 4 * u.cout, u.kpad_f, L.SD_EPI_PIXSHUF,
               t["u:" + u.name].data_ptr(), None, 0, self.params[u.name + ".bias"].data_ptr(), None, s)

    # ------------------------------------------------------------------ fp8 inference forward
    def _fp8_src_chans(self, cl: ConvL) -> tuple[int, ...]:
        if cl.name == "enc1.0":
            return (self.cin_pad0,)
        if cl.idx == 1 or cl.blk in PREV_ENC:
            return (cl.cin,)
        up = self.ups[UP_OF_DEC[cl.blk]]
        return (up.cout, self.convs[SKIP_OF_DEC[cl.blk] + ".1"].cout)

    def _rows(self, key: str) -> int:
        return self.ws.t[key].shape[0]

    def _fp8_src(self, cl: ConvL):
        """(qsrc list for sd_fp8_qparams, sd_src with the folded quantisation affines) of conv `cl`'s input."""
        ws, t = self.ws, self.ws.t
        Hl, Wl = ws.H >> cl.level, ws.W >> cl.level
        qs = [t[f"qs{k}:{cl.name}"] for k in range(len(self._fp8_src_chans(cl)))]
        qh = [t[f"qh{k}:{cl.name}"] for k in range(len(qs))]
        if cl.name == "enc1.0":  # packed input (dataset.py:184-193: RGB/255, zero channel padding)
            q = [L.make_qsrc(t["mm:xin"], self._rows("mm:xin"), self.cin_pad0, qs[0], qh[0])]
            src = L.make_src(t["xin"], self.cin_pad0, Hl, Wl, taps=9, bn0=(qs[0], qh[0]), xform0=L.SD_AFFINE)
        elif cl.idx == 1:
            prev = self.convs[cl.blk + ".0"]
            q = [L.make_qsrc(t["mm:" + prev.name], self._rows("mm:" + prev.name), prev.cout, qs[0], qh[0],
                             bn=self._bn(prev), relu=True)]
            src = L.make_src(t["y:" + prev.name], prev.cout, Hl, Wl, taps=9, bn0=(qs[0], qh[0]))
        elif cl.blk in PREV_ENC:  # materialised MaxPool2d(relu(bn(y))) of the previous encoder block
            prev = self.convs[PREV_ENC[cl.blk] + ".1"]
            q = [L.make_qsrc(t["mm:" + prev.name], self._rows("mm:" + prev.name), prev.cout, qs[0], qh[0],
                             bn=self._bn(prev), relu=True, ident=True)]
            src = L.make_src(t["pool:" + prev.name], prev.cout, Hl, Wl, taps=9, bn0=(qs[0], qh[0]),
                             xform0=L.SD_AFFINE)
        else:  # decoder conv0: cat([up, skip]) (model.py:89-95)
            up = self.ups[UP_OF_DEC[cl.blk]]
            sk = self.convs[SKIP_OF_DEC[cl.blk] + ".1"]
            q = [L.make_qsrc(t["mm:" + up.name], self._rows("mm:" + up.name), up.cout, qs[0], qh[0]),
                 L.make_qsrc(t["mm:" + sk.name], self._rows("mm:" + sk.name), sk.cout, qs[1], qh[1],
                             bn=self._bn(sk), relu=True)]
            src = L.make_src(t["u:" + up.name], up.cout, Hl, Wl, taps=9, bn0=(qs[0], qh[0]), xform0=L.SD_AFFINE,
                             src1=t["y:" + sk.name], c1=sk.cout, bn1=(qs[1], qh[1]))
        return q, src

    def _conv_fwd_fp8(self, cl: ConvL):
        """One eval-mode conv3x3 + BN coefficients on the fp8 path (model.py:36-41): the input's dynamic
        scale from its producers' (min, max) rows, then the e4m3 halo conv."""
        ws, t, s = self.ws, self.ws.t, self._s()
        Hl, Wl = ws.H >> cl.level, ws.W >> cl.level
        q, src = self._fp8_src(cl)
        arr = (L.SdQSrc * len(q))(*q)
        act_scale = t["as:" + cl.name]
        L.call("sd_fp8_qparams", arr, len(q), act_scale.data_ptr(), s)
        L.call("sd_conv3x3_fp8", src, ws.B, Hl, Wl, self.wq8.data_ptr() + cl.off8,
               self.wscale8.data_ptr() + 4 * cl.soff8, act_scale.data_ptr(), cl.cout, cl.kpad8,
               t["y:" + cl.name].data_ptr(), t["mm:" + cl.name].data_ptr(), s)
        if self._eval_coeffs:
            g, b = self.params[cl.bn_key + ".weight"], self.params[cl.bn_key + ".bias"]
            rm, rv = self.bufs[cl.bn_key + ".running_mean"], self.bufs[cl.bn_key + ".running_var"]
            L.call("sd_bn_eval_coeffs", rm.data_ptr(), rv.data_ptr(), g.data_ptr(), b.data_ptr(), cl.cout, BN_EPS,
                   t["mean:" + cl.name].data_ptr(), t["invstd:" + cl.name].data_ptr(),
                   t["scale:" + cl.name].data_ptr(), t["shift:" + cl.name].data_ptr(), s)

    def _q8_bf16(self, cl: ConvL) -> bool:
        """Static fp8 forward: the full-resolution 32-channel convs stay bf16 (k_halo_conv). Their 8/32-channel inputs
        fill a 64-channel e4m3 chunk (one k-step of v_mfma_scale_f32_32x32x64_f8f6f4) an eighth to a half, so e4m3 was
        slower there (960x720: enc1.0 35 vs 22 us, dec1.0 57 vs 45 us); they hold 20 % of the forward's FLOPs."""
        return cl.cout == 32 and cl.level == 0

    def _conv_fwd_q8(self, cl: ConvL):
        """The same conv with the static scales its calibration forward left (sd_conv3x3_q8): one launch."""
        ws, t = self.ws, self.ws.t
        if self._q8_bf16(cl):
            if self._use_wsplit(cl, False):
                L.call("sd_conv3x3_ex", self._src_fwd(cl), ws.B, ws.H >> cl.level, ws.W >> cl.level,
                       self._ws_ptr(cl.off_s), cl.cout, cl.kpad_s, L.SD_EPI_STORE, L.SD_CONV_WSPLIT, None, None,
                       t["y:" + cl.name].data_ptr(), None, self._s())
                return
            L.call("sd_conv_gemm", L.SD_BF16, self._src_fwd(cl), ws.B, ws.H >> cl.level, ws.W >> cl.level,
                   self._wp(cl.off_f), cl.cout, cl.kpad_f, L.SD_EPI_STORE, t["y:" + cl.name].data_ptr(), None, 0, None,
                   None, self._s())
            return
        _, src = self._fp8_src(cl)
        L.call("sd_conv3x3_q8", src, ws.B, ws.H >> cl.level, ws.W >> cl.level, self.wq8.data_ptr() + cl.off8,
               self.wscale8.data_ptr() + 4 * cl.soff8, t["as:" + cl.name].data_ptr(), cl.cout, cl.kpad8,
               t["y:" + cl.name].data_ptr(), self._s())

    def _forward_q8(self, ws: Workspace):
        """Static-scale fp8 forward: model state unchanged since the calibration forward (the live app's loop)."""
        t, s, B, H, W = ws.t, self._s(), ws.B, ws.H, ws.W
        for blk in BLOCKS_FWD:
            if blk in UP_OF_DEC:
                self._up_fwd(self.ups[UP_OF_DEC[blk]], train=False)
            if blk in PREV_ENC:
                prev = self.convs[PREV_ENC[blk] + ".1"]
                lv = prev.level
                L.call("sd_bnrelu_pool", L.SD_BF16, t["y:" + prev.name].data_ptr(), t["scale:" + prev.name].data_ptr(),
                       t["shift:" + prev.name].data_ptr(), B, H >> lv, W >> lv, prev.cout,
                       t["pool:" + prev.name].data_ptr(), s)
            self._conv_fwd_q8(self.convs[blk + ".0"])
            self._conv_fwd_q8(self.convs[blk + ".1"])
        return ws

    def _forward_fp8(self, ws: Workspace):
        # calibration: the first forward of a model state (and every one with SD_FP8_STATIC=0) computes each conv
        # input's scale from the activations (dynamic); the next forwards of that state reuse the scales
        if self.fp8_static and self._q8_shapes and ws.q8_ready and not self._eval_coeffs:
            return self._forward_q8(ws)
        ws.q8_ready = True
        t, s, B, H, W = ws.t, self._s(), ws.B, ws.H, ws.W
        L.call("sd_chan_minmax", t["xin"].data_ptr(), B * H * W, self.cin_pad0, t["mm:xin"].data_ptr(), s)
        for blk in BLOCKS_FWD:
            if blk in UP_OF_DEC:
                u = self.ups[UP_OF_DEC[blk]]
                self._up_fwd(u, train=False)  # bf16 ConvTranspose2d (model.py:88-94)
                Pu = B * (H >> (u.level - 1)) * (W >> (u.level - 1))
                L.call("sd_chan_minmax", t["u:" + u.name].data_ptr(), Pu, u.cout, t["mm:" + u.name].data_ptr(), s)
            if blk in PREV_ENC:
                prev = self.convs[PREV_ENC[blk] + ".1"]
                lv = prev.level
                L.call("sd_bnrelu_pool", L.SD_BF16, t["y:" + prev.name].data_ptr(), t["scale:" + prev.name].data_ptr(),
                       t["shift:" + prev.name].data_ptr(), B, H >> lv, W >> lv, prev.cout,
                       t["pool:" + prev.name].data_ptr(), s)
            self._conv_fwd_fp8(self.convs[blk + ".0"])
            self._conv_fwd_fp8(self.convs[blk + ".1"])
        return ws

    def forward(self, x: torch.Tensor, train: bool, need_backward: bool | None = None):
        """x: [B, in_channels, H, W] fp32 NCHW on device. Fills the workspace; heads not run.
        need_backward (default: train): backward() may follow. An eval-mode forward with need_backward=True (autograd
        through a model in eval mode) gets the backward buffers and stores the raw conv outputs the backward reads
        (no BN-applied stores, no graph replay)."""
        B, C, H, W = x.shape
        if C != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {C}")
        if self.fp8 and train:
            raise RuntimeError("precision='fp8' is the inference-only forward (BASELINE config 5): call model.eval()")
        if need_backward is None:
            need_backward = train
        if self.fp8 and need_backward:
            raise RuntimeError("precision='fp8' is the inference-only forward: no backward")
        self._zs_ok = not need_backward
        ws = self.workspace(B, H, W, train or need_backward)
        ws.fwd_train = train
        if train:  # batch statistics overwrite the BN coefficients; running statistics move
            self.touch_state()
            ws.coeff_key = None
            self._eval_coeffs = True
        else:  # running-statistics coefficients: recomputed only when the state moved since the last eval forward
            key = self._state_key()
            self._eval_coeffs = key is None or ws.coeff_key != key
            ws.coeff_key = key
        self.phase = "fwd"  # read by measurement hooks (bench.py) to tell forward from backward launches
        x = x.contiguous().float()
        ready, self._xin_ready = getattr(self, "_xin_ready", None), None
        if ready is not None and ready == (x.data_ptr(), tuple(x.shape), ws.t["xin"].data_ptr()):
            pass  # packed by step_prologue
        elif self.fp8 and self.fp8_static and self._q8_shapes:
            self._pack_input_fp8(ws, x)
        else:
            L.call("sd_pack_input", self.sd_dtype, x.data_ptr(), B, C, H, W, self.cin_pad0, ws.t["xin"].data_ptr(),
                   self._s())
        # eval forwards of an unchanged model state (the live app's loop): the launches after the input pack are
        # captured into a HIP graph on the second such forward and replayed from the third on (one host call instead
        # of 27-45 ctypes launches; B=1 960x720 forwards were host-bound at ~20 us of GPU time per kernel)
        gkey = None
        if not need_backward and self.eval_graphs and not self._eval_coeffs and ws.coeff_key is not None:
            gkey = (ws.coeff_key, self._fwd_path(ws))
            if ws.graph is not None and ws.graph_key == gkey:
                with torch.cuda.device(self.device):  # replays on the current stream of the engine's device
                    ws.graph.replay()
                # the replayed body stored what the captured one did: its BN-applied (z) layers, not whatever the
                # last eager forward on this workspace (e.g. a grad-enabled eval forward, raw y stores) left
                self._zs = set(ws.graph_zs)
                self._amax_readback()
                return ws
        self._forward_body(ws, train)
        self._amax_readback()
        if gkey is not None and gkey[1] == self._fwd_path(ws):
            self._capture(ws, gkey, train)
        return ws

    # ------------------------------------------------------------------ fp8 static-scale recalibration
    def request_calibration(self):
        """The next eval forward recomputes the fp8 activation scales from its own input (a calibration forward)."""
        if self.ws is not None:
            self.ws.q8_ready = False

    def _fp8_policy(self, ws: Workspace, slot: int):
        """Static fp8 scales come from one calibration frame; a later frame with a wider range would saturate at
        +-448. Two triggers make this forward a calibration forward again:
          * range: the input pack of every static forward also takes max |x| (sd_pack_input_amax, no extra pass),
            read back to pinned memory without a sync; when a frame's amax exceeds `fp8_range_margin` x the calibration
            frame's, the next forward recalibrates (one frame late, no host stall);
          * age: every `fp8_recalib_every` static forwards (0: never).
        `fp8_calibrations` counts calibration forwards. Returns whether this forward calibrates."""
        if not ws.q8_ready or self._eval_coeffs:  # new state, new workspace, or requested
            return True
        # The host copy of ring word s is overwritten by the read-back of the next frame that takes word s, i.e. this
        # frame's for word `slot` (frame f - 3's). A word is checked once its read-back has landed (query, no host
        # block); only frame f - 3's word, on its last chance, is waited for — which happens only when the caller
        # queues frames three deep. The side stream completes in order, so a landed frame implies the calibration
        # frame before it landed too.
        if self._fp8_cal_amax is None and self._fp8_cal is not None:  # the calibration frame's amax, once it landed
            s, ev = self._fp8_cal
            if s == slot:
                ev.synchronize()
            if ev.query():
                self._fp8_cal_amax = float(self._amax_host[s])
        hit = False
        for s in (slot, (slot + 1) % 3, (slot + 2) % 3):  # frames f - 3, f - 2, f - 1
            if not self._amax_used[s] or self._amax_checked[s]:
                continue
            ev = self._amax_ev[s]
            if s == slot:
                ev.synchronize()
            elif not ev.query():
                continue
            if self._fp8_cal_amax is None and self._fp8_cal is not None:  # landed: the calibration frame has too
                self._fp8_cal_amax = float(self._amax_host[self._fp8_cal[0]])
            self._amax_checked[s] = True
            if (self.fp8_range_margin > 0 and self._fp8_cal_amax is not None
                    and float(self._amax_host[s]) > self.fp8_range_margin * self._fp8_cal_amax):
                hit = True
        if hit:
            self.fp8_range_recalibrations += 1
            return True
        if self.fp8_recalib_every and self._fp8_age >= self.fp8_recalib_every:
            return True
        self._fp8_age += 1
        return False

    def _pack_input_fp8(self, ws: Workspace, x: torch.Tensor):
        """The static-scale fp8 path's input pack: sd_pack_input + the input amax for _fp8_policy. A ring of three
        device words: frame f takes word f % 3 and zeroes word (f + 1) % 3, after the launch stream has waited for the
        side-stream read-back of that word (frame f - 2's, long complete: a barrier packet, no stall)."""
        B, C, H, W = x.shape
        slot = self._fp8_frame % 3
        clear = (slot + 1) % 3
        self._fp8_frame += 1
        if self._amax_dev is None:
            with torch.inference_mode(False):  # written in place by later forwards, in or out of inference mode
                self._amax_dev = torch.zeros(3, dtype=torch.float32, device=self.device)
                self._amax_host = torch.zeros(3, dtype=torch.float32, pin_memory=True)
            self._amax_ev = [torch.cuda.Event() for _ in range(3)]
            self._amax_used = [False] * 3
            self._amax_checked = [True] * 3
            self._amax_packed = torch.cuda.Event()
        if self._fp8_policy(ws, slot):
            ws.q8_ready = False
            self.fp8_calibrations += 1
            self._fp8_age = 0
            self._fp8_cal_amax = None
            self._amax_checked = [True] * 3  # earlier frames are not held against the new calibration frame's range
        main = torch.cuda.current_stream(self.device)
        if self._amax_used[clear]:
            main.wait_event(self._amax_ev[clear])
        L.call("sd_pack_input_amax", self.sd_dtype, x.data_ptr(), B, C, H, W, self.cin_pad0, ws.t["xin"].data_ptr(),
               self._amax_dev.data_ptr(), slot, clear, self._s())
        self._amax_packed.record(main)
        self._amax_pending = slot  # read back by _amax_readback once the forward's launches are queued
        if not ws.q8_ready:
            self._fp8_cal = (slot, self._amax_ev[slot])

    def _amax_readback(self):
        """The input amax of this frame -> pinned host memory on a side stream, queued after the forward's launches
        (the 4-byte copy on the launch stream, and its host calls before the graph replay, cost ~25 us per frame)."""
        slot = self._amax_pending
        if slot is None:
            return
        self._amax_pending = None
        side = self._side_stream()
        side.wait_event(self._amax_packed)
        with torch.cuda.stream(side):
            self._amax_host[slot:slot + 1].copy_(self._amax_dev[slot:slot + 1], non_blocking=True)
            self._amax_ev[slot].record(side)
        self._amax_used[slot] = True
        self._amax_checked[slot] = False

    def _capture(self, ws: Workspace, gkey, train: bool):
        """Capture the forward body into a HIP graph on the engine's OWN capture stream on its device (torch's shared
        default capture stream lives on whichever device was current at the first capture anywhere in the process;
        launches on another device's stream would leave the graph empty). Inside the capture, current_stream(device)
        is that stream, so every launch of the body (L.stream_handle) is recorded."""
        if getattr(self, "_capture_stream", None) is None:
            self._capture_stream = torch.cuda.Stream(self.device)
        g = torch.cuda.CUDAGraph()
        # outside inference mode: capture_begin advances the CUDA generator's graph-safe state in place, and a state
        # created by a capture under inference_mode would be an inference tensor that a later capture outside it (a
        # validation epoch after the live loop) could not update
        with torch.inference_mode(False), torch.cuda.device(self.device):
            cur = torch.cuda.current_stream(self.device)
            self._capture_stream.wait_stream(cur)
            # thread_local: loader threads may use the device while this thread captures
            with torch.cuda.graph(g, stream=self._capture_stream, capture_error_mode="thread_local"):
                if L.stream_handle(self.device) != self._capture_stream.cuda_stream:
                    raise RuntimeError("eval graph capture: launches would not go to the capture stream")
                self._forward_body(ws, train)
            cur.wait_stream(self._capture_stream)
        ws.graph, ws.graph_key, ws.graph_zs = g, gkey, frozenset(self._zs)

    def _fwd_path(self, ws: Workspace) -> str:
        if not self.fp8:
            return "bf16" if self.sd_dtype == L.SD_BF16 else "fp32"
        return "q8" if self.fp8_static and self._q8_shapes and ws.q8_ready and not self._eval_coeffs else "fp8"

    def _forward_body(self, ws: Workspace, train: bool):
        B, H, W = ws.B, ws.H, ws.W
        self._zs = set()  # layers whose stored output is the BN-applied z (eval, zstore)
        if self.fp8:
            return self._forward_fp8(ws)
        for blk in BLOCKS_FWD:
            if blk in UP_OF_DEC:
                self._up_fwd(self.ups[UP_OF_DEC[blk]], train)
            if blk in PREV_ENC and self.sd_dtype == L.SD_BF16:
                prev = self.convs[PREV_ENC[blk] + ".1"]
                lv = prev.level
                sc, sh = self._bn(prev)
                L.call("sd_bnrelu_pool", self.sd_dtype, ws.t["y:" + prev.name].data_ptr(), sc.data_ptr(),
                       sh.data_ptr(), B, H >> lv, W >> lv, prev.cout, ws.t["pool:" + prev.name].data_ptr(), self._s())
            self._conv_fwd(self.convs[blk + ".0"], train)
            self._conv_fwd(self.convs[blk + ".1"], train)
        return ws

    def heads(self, mode: int, disp=None, logvar=None, target=None, valid=None, gdisp=None, glogvar=None,
              no_grad: bool = False):
        """model.py:76-77,98,103 heads (+ train.py:329-352 loss/metrics for SD_HEADS_LOSS).
        no_grad: LOSS mode for evaluation (metrics only, no gradient written)."""
        ws, t, s = self.ws, self.ws.t, self._s()
        cl = self.convs["dec1.1"]
        P = ws.B * ws.H * ws.W
        p = self.params
        da = None if no_grad else t.get("da:dec1.1")
        if mode != L.SD_HEADS_INFER and "heads_part" not in t:
            t["heads_part"] = torch.empty(L.call("sd_heads_rows", P) * (2 * self.c1 + 7), dtype=torch.float32,
                                          device=self.device)
        part = t.get("heads_part")
        hsc, hsh = self._bn(cl)  # identity after a zstore eval forward (y:dec1.1 holds z)
        args = (self.sd_dtype, mode, t["y:dec1.1"].data_ptr(), hsc.data_ptr(), hsh.data_ptr(), P, cl.cout, p["disparity_head.weight"].data_ptr(),
                p["disparity_head.bias"].data_ptr(), p["logvar_head.weight"].data_ptr(),
                p["logvar_head.bias"].data_ptr(), L.ptr(disp), L.ptr(logvar), L.ptr(target), L.ptr(valid),
                self.count.data_ptr() if mode == L.SD_HEADS_LOSS else None, L.ptr(gdisp), L.ptr(glogvar),
                L.ptr(da) if mode != L.SD_HEADS_INFER else None, L.ptr(part) if mode != L.SD_HEADS_INFER else None)
        self._heads_bn_rows = 0
        if mode != L.SD_HEADS_INFER and da is not None and "chan" in t:
            # da:dec1.1 and that layer's BN-backward sums in one pass (backward() skips its reduce)
            L.call("sd_heads_bnsum", *args, t["mean:dec1.1"].data_ptr(), t["invstd:dec1.1"].data_ptr(),
                   t["chan"].data_ptr(), s)
            self._heads_bn_rows = L.call("sd_heads_rows", P)
        else:
            L.call("sd_heads", *args, s)
        if mode != L.SD_HEADS_INFER:
            g = {} if no_grad else self.grads
            L.call("sd_heads_finalize", part.data_ptr(), L.call("sd_heads_rows", P), cl.cout,
                   L.ptr(g.get("disparity_head.weight")), L.ptr(g.get("disparity_head.bias")),
                   L.ptr(g.get("logvar_head.weight")), L.ptr(g.get("logvar_head.bias")),
                   self.metrics.data_ptr() if mode == L.SD_HEADS_LOSS else None,
                   self.count_local.data_ptr() if mode == L.SD_HEADS_LOSS else None, s)

    def count_valid(self, target: torch.Tensor, valid: torch.Tensor):
        """train.py:329-330 valid count, on device: count_local (this rank's pixels, for the
        metric sums) and count (the loss normaliser; DDP all-reduces it to the global count)."""
        k = self._count_slot()
        L.call("sd_count_valid", target.data_ptr(), valid.data_ptr(), target.numel(), self._counts[k].data_ptr(), 2,
               self._counts[k ^ 1].data_ptr(), self._s())

    def _count_slot(self) -> int:
        """The double-buffered counter pair this batch counts into (count_local / count point at it)."""
        k = self._cslot
        self._cslot ^= 1
        self.count_local = self._counts[k, 0:1]
        self.count = self._counts[k, 1:2]
        return k

    # ------------------------------------------------------------------ backward
    @staticmethod
    def _pool_bn_fused(cl: ConvL) -> bool:
        """sd_pool_bwd_add can produce this layer's BN-backward sums (C/8 must divide 256)."""
        return 256 % (cl.cout // 8) == 0

    def _bn_bwd(self, cl: ConvL, fused_rows: int = 0, apply: bool = True):
        """da:<cl> -> dy:<cl>, dgamma/dbeta (model.py:37,40 BatchNorm2d backward, ReLU mask fused).
        fused_rows > 0: the producer of da already wrote that many partial-sum rows into t["chan"].
        apply=False: only the sums and coefficients; the weight gradient forms dy while staging it."""
        ws, t, s, dt = self.ws, self.ws.t, self._s(), self.sd_dtype
        P = ws.B * (ws.H >> cl.level) * (ws.W >> cl.level)
        args = (t["scale:" + cl.name].data_ptr(), t["shift:" + cl.name].data_ptr(), t["mean:" + cl.name].data_ptr(),
                t["invstd:" + cl.name].data_ptr())
        chan = t["chan"]
        if fused_rows:
            rows = fused_rows
        else:
            L.call("sd_bn_bwd_reduce", dt, t["da:" + cl.name].data_ptr(), t["y:" + cl.name].data_ptr(), *args, P,
                   cl.cout, chan.data_ptr(), s)
            rows = L.call("sd_chan_reduce_rows", P, cl.cout)
        coef = t["coef:" + cl.name]
        if self.bn_sync is not None and ws.fwd_train:
            loc, glob = self._sync_sums(chan, rows, cl.cout, P, keep_local=True)
            L.call("sd_bn_bwd_finalize64", loc.data_ptr(), glob.data_ptr(), cl.cout,
                   self.params[cl.bn_key + ".weight"].data_ptr(), t["invstd:" + cl.name].data_ptr(), 1,
                   self.grads[cl.bn_key + ".weight"].data_ptr(), self.grads[cl.bn_key + ".bias"].data_ptr(),
                   coef.data_ptr(), s)
        else:
            L.call("sd_bn_bwd_finalize", chan.data_ptr(), rows, cl.cout, float(P),
                   self.params[cl.bn_key + ".weight"].data_ptr(), t["invstd:" + cl.name].data_ptr(),
                   int(ws.fwd_train), self.grads[cl.bn_key + ".weight"].data_ptr(),
                   self.grads[cl.bn_key + ".bias"].data_ptr(), coef.data_ptr(), s)
        if apply:
            L.call("sd_bn_bwd_apply", dt, t["da:" + cl.name].data_ptr(), t["y:" + cl.name].data_ptr(), *args,
                   coef.data_ptr(), P, cl.cout, t["dy:" + cl.name].data_ptr(), s)

    def _sync_sums(self, rows_t: torch.Tensor, rows: int, C: int, pixels: int, keep_local: bool = False):
        """SyncBatchNorm: this rank's float2 partial rows -> fp64 per-channel sums plus its pixel count, SUM-all-reduced
        over the ranks (stream-ordered), so the finalizes divide by the global count even when the ranks' batches
        differ. Returns (global, _) or, with keep_local, (local, global)."""
        if C > 2048:
            raise ValueError(f"SyncBatchNorm: {C} channels > 2048")
        if self._bn64 is None or self._bn64.device != self.device:
            self._bn64 = torch.empty(2, 2 * 2048 + 1, dtype=torch.float64, device=self.device)
        loc, glob = self._bn64[0, :2 * C + 1], self._bn64[1, :2 * C + 1]
        L.call("sd_bn_rows_sum64", rows_t.data_ptr(), rows, C, float(pixels), loc.data_ptr(), self._s())
        if not keep_local:
            self.bn_sync(loc)
            return loc, None
        glob.copy_(loc)
        self.bn_sync(glob)
        return loc, glob

    def _wgrad(self, a: L.SdSrc, b: L.SdSrc, lvl: int, M: int, N: int, layout: int, ci_real: int, dw: torch.Tensor,
               key: str):
        ws, dt = self.ws, self.sd_dtype
        Hl, Wl = ws.H >> lvl, ws.W >> lvl
        sp = L.call("sd_wgrad_splits", dt, ws.B, Hl, Wl, M, N)
        self._wgrad_slabs(lambda slab, st: L.call("sd_wgrad_gemm", dt, a, b, ws.B, Hl, Wl, M, N, slab, sp, st),
                          sp, M, N, layout, ci_real, dw, gemm_may_side=True, key=key)

    def _side_stream(self) -> torch.cuda.Stream:
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def _wgrad_slabs(self, gemm, sp: int, M: int, N: int, layout: int, ci_real: int, dw: torch.Tensor,
                     gemm_may_side: bool, key: str):
        """gemm(slab_ptr, stream) writes sp split-K slabs of an M x N weight gradient; sd_wgrad_reduce sums them
        into dw. defer_reduce: the slabs go to the weight's own region and the reduce joins the next batch
        (_flush_reduces). With side_mode the reduce runs on the side stream (and with side_mode 2 a gemm_may_side GEMM
        too)."""
        s = self._s()
        if self.defer_reduce:
            slab = self.ws.t["slab"].data_ptr() + 4 * self.ws.slab_off[key]
            gemm(slab, s)
            self._red_jobs.append(L.SdWredJob(slab, sp, M, N, layout, ci_real, dw.data_ptr()))
            return
        if not self.side_mode:
            slab = self.ws.t["slab"].data_ptr()
            gemm(slab, s)
            L.call("sd_wgrad_reduce", slab, sp, M, N, layout, ci_real, dw.data_ptr(), s)
            return
        main, side = torch.cuda.current_stream(self.device), self._side_stream()
        i = self._slab_i
        self._slab_i ^= 1
        slab = self.ws.t["slab1" if i else "slab"].data_ptr()
        if gemm_may_side and self.side_mode >= 2:
            side.wait_stream(main)  # its operands (dy, x) come from the current stream; the slab's last reduce
            gemm(slab, side.cuda_stream)  # precedes it on the side stream
        else:
            if self._slab_free[i] is not None:
                main.wait_event(self._slab_free[i])  # the reduce that last read this slab
            gemm(slab, s)
            side.wait_stream(main)
        L.call("sd_wgrad_reduce", slab, sp, M, N, layout, ci_real, dw.data_ptr(), side.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(side)
        self._slab_free[i] = ev

    def _bias_rows_ptr(self, up_name: str) -> int:
        """Where the decoder dgrad writes the d(up) statistics rows of up_name's bias gradient: its own region of the
        slab buffer when the reduces are deferred (they are summed at the flush), else the shared t["stats"]."""
        if self.defer_reduce:
            return self.ws.t["slab"].data_ptr() + 4 * self.ws.slab_off["brows:" + up_name]
        return self.ws.t["stats"].data_ptr()

    def _flush_reduces(self):
        """Every deferred slab reduce in one launch (the gradients they write are final after it, in stream order)."""
        if self._red_jobs:
            jobs = (L.SdWredJob * len(self._red_jobs))(*self._red_jobs)
            L.call("sd_wgrad_reduce_batch", jobs, len(self._red_jobs), self._s())
            self._red_jobs = []

    def _side_join(self):
        """The current stream waits for everything queued on the side stream (gradients final)."""
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    def _conv_bwd(self, cl: ConvL, need_dgrad: bool, fused_rows: int = 0):
        ws, t, s, dt = self.ws, self.ws.t, self._s(), self.sd_dtype
        Hl, Wl = ws.H >> cl.level, ws.W >> cl.level
        kind = self._bwd_fused(cl, ws.H, ws.W) if need_dgrad else 0
        if kind == 2:
            # one pass: dy = BatchNorm-backward(da, y) staged in LDS, the weight gradient's split-K slabs over
            # x = cat(u, relu(bn(y_skip))), the dgrad split into d(u) and d(skip), and d(u)'s column sums (the
            # ConvTranspose2d bias gradient, for _up_bwd): da, y, u, y_skip read once, no dy round trip
            self._bn_bwd(cl, fused_rows, apply=False)
            up, sk = self.ups[UP_OF_DEC[cl.blk]], self.convs[SKIP_OF_DEC[cl.blk] + ".1"]
            ssc, ssh = self._bn(sk)
            sp = L.call("sd_conv3x3_bwd_fused_splits", ws.B, Hl, Wl)
            args = (t["da:" + cl.name].data_ptr(), t["y:" + cl.name].data_ptr(), t["scale:" + cl.name].data_ptr(),
                    t["shift:" + cl.name].data_ptr(), t["mean:" + cl.name].data_ptr(),
                    t["invstd:" + cl.name].data_ptr(), t["coef:" + cl.name].data_ptr(), t["u:" + up.name].data_ptr(),
                    t["y:" + sk.name].data_ptr(), ssc.data_ptr(), ssh.data_ptr(), self._wp(cl.off_d), cl.kpad_d,
                    ws.B, Hl, Wl, t["du:" + up.name].data_ptr(), t["dskip:" + up.name].data_ptr())
            brows = self._bias_rows_ptr(up.name)
            self._wgrad_slabs(lambda slab, st: L.call("sd_conv3x3_bwd_fused_dec", *args, slab, brows, st),
                              sp, cl.cout, 9 * cl.cin_pad, L.SD_W_CONV3, cl.cin, self.grads[cl.w_key],
                              gemm_may_side=False, key=cl.name)
            self._up_bias_rows = (sp, 32, brows)
            return
        if kind == 1:
            # one pass: dy = BatchNorm-backward(da, y) staged in LDS, the weight gradient's split-K slabs, the dgrad
            # into da of conv0 and conv0's BatchNorm-backward sums (4 full-resolution tensor passes instead of 7)
            self._bn_bwd(cl, fused_rows, apply=False)
            c0 = self.convs[cl.blk + ".0"]
            sp = L.call("sd_conv3x3_bwd_fused_splits", ws.B, Hl, Wl)
            args = (t["da:" + cl.name].data_ptr(), t["y:" + cl.name].data_ptr(), t["scale:" + cl.name].data_ptr(),
                    t["shift:" + cl.name].data_ptr(), t["mean:" + cl.name].data_ptr(),
                    t["invstd:" + cl.name].data_ptr(), t["coef:" + cl.name].data_ptr(), t["y:" + c0.name].data_ptr(),
                    t["scale:" + c0.name].data_ptr(), t["shift:" + c0.name].data_ptr(),
                    t["mean:" + c0.name].data_ptr(), t["invstd:" + c0.name].data_ptr(), self._wp(cl.off_d),
                    cl.kpad_d, ws.B, Hl, Wl, t["da:" + c0.name].data_ptr())
            self._wgrad_slabs(lambda slab, st: L.call("sd_conv3x3_bwd_fused", *args, slab, t["chan"].data_ptr(), st),
                              sp, cl.cout, 9 * cl.cin_pad, L.SD_W_CONV3, cl.cin, self.grads[cl.w_key],
                              gemm_may_side=False, key=cl.name)
            self._bnsum_rows[c0.name] = sp
            return
        dy = t["dy:" + cl.name]
        a = L.make_src(dy, cl.cout, Hl, Wl, taps=1)
        b = self._src_fwd(cl)
        M, N = cl.cout, 9 * cl.cin_pad
        if not need_dgrad and dt == L.SD_BF16:  # enc1.0: nothing reads dy after the weight gradient
            a_nody = L.make_src(None, cl.cout, Hl, Wl, taps=1)
            if self.bn_fuse and L.call("sd_wgrad_bnbwd_ok", dt, a_nody, b, M, N) == 1:
                a = a_nody
        # bf16: the weight gradient applies the BatchNorm backward while staging dy (and writes dy for the
        # dgrad), so the apply pass over (da, y) -> dy is gone; it runs first, the dgrad reads its dy. Each
        # x-channel block of the kernel repeats the transform of the same dy tile on its loader waves, whose VALU
        # then paces the kernel: fused where one block covers x (two at full resolution, where the separate pass
        # costs most). Measured per layer (tools/bench_variants.sh): enc1-enc3.0, dec2.1, dec1 gain; deeper lose.
        nblk = L.call("sd_wgrad_bnbwd_ok", dt, a, b, M, N) if self.bn_fuse and dt == L.SD_BF16 else 0
        fuse = nblk == 1 or (nblk == 2 and cl.level == 0)
        self._bn_bwd(cl, fused_rows, apply=not fuse)
        if fuse:
            sp = L.call("sd_wgrad_splits", dt, ws.B, Hl, Wl, M, N)
            args = (t["da:" + cl.name].data_ptr(), t["y:" + cl.name].data_ptr(), t["scale:" + cl.name].data_ptr(),
                    t["shift:" + cl.name].data_ptr(), t["mean:" + cl.name].data_ptr(),
                    t["invstd:" + cl.name].data_ptr(), t["coef:" + cl.name].data_ptr())
            # writes dy, which the dgrad below reads: stays on the current stream
            self._wgrad_slabs(lambda slab, st: L.call("sd_wgrad_gemm_bnbwd", dt, a, b, ws.B, Hl, Wl, M, N, *args,
                                                      slab, sp, st),
                              sp, M, N, L.SD_W_CONV3, cl.cin, self.grads[cl.w_key], gemm_may_side=False, key=cl.name)
        if need_dgrad:
            dsrc = L.make_src(dy, cl.cout, Hl, Wl, taps=9)
            if cl.idx == 1:
                out = t["da:" + cl.blk + ".0"]
                c0 = self.convs[cl.blk + ".0"]
                if (self.bnsum_fuse and dt == L.SD_BF16 and cl.cin <= 64
                        and L.call("sd_conv_gemm_bnsum_ok", dt, dsrc, cl.cin) == 1):
                    # da of conv0 and its BatchNorm-backward sums (for _bn_bwd(conv0)) from one launch. At 32/64
                    # channels (240x320, 120x160) the epilogue's sums cost less than the reduce pass they replace;
                    # deeper, the two measured equal (the epilogue is MFMA-wave time, the pass was HBM time)
                    L.call("sd_conv_gemm_bnsum", dt, dsrc, ws.B, Hl, Wl, self._wp(cl.off_d), cl.cin, cl.kpad_d,
                           out.data_ptr(), t["y:" + c0.name].data_ptr(), t["scale:" + c0.name].data_ptr(),
                           t["shift:" + c0.name].data_ptr(), t["mean:" + c0.name].data_ptr(),
                           t["invstd:" + c0.name].data_ptr(), t["chan"].data_ptr(), s)
                    self._bnsum_rows[c0.name] = L.call("sd_conv_gemm_bnsum_rows", dsrc, ws.B, Hl, Wl, cl.cin)
                else:
                    L.call("sd_conv_gemm", dt, dsrc, ws.B, Hl, Wl, self._wp(cl.off_d), cl.cin, cl.kpad_d,
                           L.SD_EPI_STORE, out.data_ptr(), None, 0, None, None, s)
            elif cl.blk in PREV_ENC:
                out = t["dpool:" + cl.blk]
                L.call("sd_conv_gemm", dt, dsrc, ws.B, Hl, Wl, self._wp(cl.off_d), cl.cin, cl.kpad_d, L.SD_EPI_STORE,
                       out.data_ptr(), None, 0, None, None, s)
            else:  # decoder: split into d(up) and d(skip) (cat backward, model.py:89-95)
                up = self.ups[UP_OF_DEC[cl.blk]]
                # bf16: the same epilogue sums d(up) per channel = the ConvTranspose2d bias gradient (_up_bwd)
                sums = self.bias_fuse and dt == L.SD_BF16 and (cl.cin == 32 or cl.cin % 64 == 0)
                brows = self._bias_rows_ptr(up.name) if sums else None
                L.call("sd_conv_gemm", dt, dsrc, ws.B, Hl, Wl, self._wp(cl.off_d), cl.cin, cl.kpad_d,
                       L.SD_EPI_SPLIT_STATS if sums else L.SD_EPI_SPLIT, t["du:" + up.name].data_ptr(),
                       t["dskip:" + up.name].data_ptr(), up.cout, None, brows, s)
                self._up_bias_rows = ((L.call("sd_conv_gemm_stat_rows", dt, ws.B, Hl, Wl, cl.cin), cl.cin, brows)
                                      if sums else None)
        if not fuse:
            self._wgrad(a, b, cl.level, M, N, L.SD_W_CONV3, cl.cin, self.grads[cl.w_key], cl.name)

    def _up_bwd(self, u: UpL):
        ws, t, s, dt = self.ws, self.ws.t, self._s(), self.sd_dtype
        du = t["du:" + u.name]
        Hh, Wh = ws.H >> (u.level - 1), ws.W >> (u.level - 1)
        Hl, Wl = ws.H >> u.level, ws.W >> u.level
        P = ws.B * Hh * Wh
        rows_ld = getattr(self, "_up_bias_rows", None)
        if rows_ld is not None:  # left by the decoder dgrad that produced du (_conv_bwd, _bias_rows_ptr)
            rows, ld, ptr = rows_ld
            bias = self.grads[u.name + ".bias"].data_ptr()
            if self.defer_reduce:
                self._red_jobs.append(L.SdWredJob(ptr, rows, 1, ld, L.SD_W_ROWSUM, u.cout, bias))
            else:
                L.call("sd_stat_rows_sum", ptr, rows, ld, u.cout, bias, s)
            self._up_bias_rows = None
        else:
            L.call("sd_chan_sum", dt, du.data_ptr(), P, u.cout, t["chan"].data_ptr(),
                   self.grads[u.name + ".bias"].data_ptr(), s)
        src_cl = self.convs[UP_SRC[u.name] + ".1"]
        a = L.make_src(t["y:" + src_cl.name], src_cl.cout, Hl, Wl, taps=1, bn0=self._bn(src_cl))
        b = L.make_src(du, u.cout, Hh, Wh, taps=4)
        self._wgrad(a, b, u.level, u.cin, 4 * u.cout, L.SD_W_CONVT, u.cin, self.grads[u.name + ".weight"], u.name)
        if self.bnsum_fuse and L.call("sd_conv_gemm_bnsum_ok", dt, b, u.cin) == 1:
            # da of the source conv and its BatchNorm-backward sums (for _bn_bwd(src_cl)) from one launch:
            # the reduce pass over (da, y) that followed every ConvTranspose dgrad is gone
            L.call("sd_conv_gemm_bnsum", dt, b, ws.B, Hl, Wl, self._wp(u.off_d), u.cin, u.kpad_d,
                   t["da:" + src_cl.name].data_ptr(), t["y:" + src_cl.name].data_ptr(),
                   t["scale:" + src_cl.name].data_ptr(), t["shift:" + src_cl.name].data_ptr(),
                   t["mean:" + src_cl.name].data_ptr(), t["invstd:" + src_cl.name].data_ptr(), t["chan"].data_ptr(), s)
            self._bnsum_rows[src_cl.name] = L.call("sd_conv_gemm_bnsum_rows", b, ws.B, Hl, Wl, u.cin)
        else:
            L.call("sd_conv_gemm", dt, b, ws.B, Hl, Wl, self._wp(u.off_d), u.cin, u.kpad_d, L.SD_EPI_STORE,
                   t["da:" + src_cl.name].data_ptr(), None, 0, None, None, s)

    def backward(self, grad_hook=None):
        """Full backward after heads() wrote da:dec1.1 (model.py:79-104 in reverse).
        grad_hook(name) fires when the gradients of top-level module `name` are final."""
        self.phase = "bwd"
        if self._zs:
            raise RuntimeError("backward after a forward that stored BN-applied outputs (an eval forward without "
                               "need_backward=True): its activations are not the ones the backward reads")
        ws, t, s, dt = self.ws, self.ws.t, self._s(), self.sd_dtype
        for blk in reversed(BLOCKS_FWD):
            if blk in ("enc1", "enc2", "enc3", "enc4"):
                # encoder output gradient = skip grad + MaxPool2d backward of the pooled path
                cl = self.convs[blk + ".1"]
                nxt = {"enc1": "enc2", "enc2": "enc3", "enc3": "enc4", "enc4": "bottleneck"}[blk]
                up = self.ups[{"enc1": "up1", "enc2": "up2", "enc3": "up3", "enc4": "up4"}[blk]]
                # the pool backward also produces this BN layer's backward sums (no sd_bn_bwd_reduce pass)
                fused = self._pool_bn_fused(cl)
                Hl, Wl = ws.H >> cl.level, ws.W >> cl.level
                fused_rows = L.call("sd_pool_bwd_rows", ws.B, Hl, Wl, cl.cout) if fused else 0
                L.call("sd_pool_bwd_add", dt, t["y:" + cl.name].data_ptr(), t["scale:" + cl.name].data_ptr(),
                       t["shift:" + cl.name].data_ptr(), t["dskip:" + up.name].data_ptr(),
                       t["dpool:" + nxt].data_ptr(), ws.B, Hl, Wl, cl.cout, t["da:" + cl.name].data_ptr(),
                       t["mean:" + cl.name].data_ptr() if fused else None,
                       t["invstd:" + cl.name].data_ptr() if fused else None,
                       t["chan"].data_ptr() if fused else None, s)
                self._conv_bwd(cl, need_dgrad=True, fused_rows=fused_rows)
            else:
                # dec1.1: heads() left its BN-backward sums in t["chan"]; deeper layers: the ConvTranspose dgrad
                # that wrote their da may have (sd_conv_gemm_bnsum in _up_bwd)
                fused_rows = getattr(self, "_heads_bn_rows", 0) if blk == "dec1" else self._bnsum_rows.pop(blk + ".1", 0)
                self._conv_bwd(self.convs[blk + ".1"], need_dgrad=True, fused_rows=fused_rows)
            self._conv_bwd(self.convs[blk + ".0"], need_dgrad=(blk != "enc1"),
                           fused_rows=self._bnsum_rows.pop(blk + ".0", 0))
            if grad_hook is not None:
                self._grads_ready(grad_hook, blk)
            if blk in UP_OF_DEC:
                self._up_bwd(self.ups[UP_OF_DEC[blk]])
                if grad_hook is not None:
                    self._grads_ready(grad_hook, UP_OF_DEC[blk])
        self._flush_reduces()
        self._side_join()

    def _grads_ready(self, grad_hook, name: str):
        """grad_hook(name) with the current stream at a point where `name`'s gradients are final. With side-stream
        reduces that is the side stream once it has caught up with this one: a collective the hook launches then
        waits for the reduces without the current stream waiting for them."""
        self._flush_reduces()
        if self._side is None:
            grad_hook(name)
            return
        side = self._side
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            grad_hook(name)

    def adamw(self, flat_p, flat_g, m, v, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8, gate_on_count=True):
        self.touch_state()
        L.call("sd_adamw", flat_p.data_ptr(), flat_g.data_ptr(), m.data_ptr(), v.data_ptr(), flat_p.numel(),
               float(lr), float(weight_decay), float(betas[0]), float(betas[1]), float(eps),
               self.adam_step.data_ptr(), self.count.data_ptr() if gate_on_count else None,
               self.adam_scratch.data_ptr(), self._s())
