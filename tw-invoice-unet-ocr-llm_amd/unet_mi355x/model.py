"""Drop-in ``UNet`` for the reference ``unet_model.UNet`` (unet_model.py:23-86).

Same constructor, same sub-module tree and therefore the same 136 ``state_dict`` keys
and shapes, so ``load_state_dict(torch.load("checkpoints/best_unet_model.pth"))``
works unchanged (inference.py:20-21).  ``forward`` runs the MI355X native path
(libunet_mi355x.so): the parameters held by the torch sub-modules are only the
weight *container*; they are BN-folded and pre-packed into the native handle the
first time a forward runs on a device, and again whenever a parameter changes.

There is no CPU / eager fallback: a CPU input raises.
"""
from __future__ import annotations

import os
import threading

import torch
import torch.nn as nn

from . import native

DEFAULT_DTYPE = os.environ.get("UNET_MI355X_DTYPE", "fp32")

# Bumped whenever a module of a UNet's tree (the _Tracked classes below) changes its parameters, buffers or
# children -- attribute assignment, register_parameter / register_buffer / add_module, deletion -- or converts
# its tensors (_apply: .to / .cuda / .half): the cached list of tensors whose (data_ptr, _version) signature
# decides re-packing is then rebuilt.  Between such events the per-forward check reads 136 cached tensors
# instead of rebuilding state_dict().  Scoped to these classes: no process-global torch hooks, so other
# modules of the app process (EasyOCR's) are never touched.
_TREE_EPOCH = [0]


def _bump_epoch(*_args):
    _TREE_EPOCH[0] += 1


class _Tracked:
    """Mixin of every module class in the UNet tree: any change to this module's own tensors or children
    bumps _TREE_EPOCH.  A tree holding a module without it (a user-assigned plain nn.Module) makes
    UNet._signature walk the live tree on every call instead of trusting the cached list."""

    def __setattr__(self, name, value):
        super().__setattr__(name, value)
        _bump_epoch()

    def __delattr__(self, name):
        super().__delattr__(name)
        _bump_epoch()

    def register_parameter(self, name, param):
        super().register_parameter(name, param)
        _bump_epoch()

    def register_buffer(self, name, tensor, persistent=True):
        super().register_buffer(name, tensor, persistent)
        _bump_epoch()

    def add_module(self, name, module):
        super().add_module(name, module)
        _bump_epoch()

    def register_module(self, name, module):
        self.add_module(name, module)

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        _bump_epoch()
        return out


# the reference's layer classes (same constructor, parameters, state_dict keys and repr), tracked
class Conv2d(_Tracked, nn.Conv2d):
    pass


class BatchNorm2d(_Tracked, nn.BatchNorm2d):
    pass


class ReLU(_Tracked, nn.ReLU):
    pass


class Sequential(_Tracked, nn.Sequential):
    pass


class MaxPool2d(_Tracked, nn.MaxPool2d):
    pass


class ConvTranspose2d(_Tracked, nn.ConvTranspose2d):
    pass


class DoubleConv(_Tracked, nn.Module):
    """unet_model.py:6-20: (conv3x3, BN, ReLU) x 2 -- the same parameters (and state_dict keys).

    Inside UNet.forward the blocks run fused with pooling / concat / head (the whole-network native
    path).  Called on its own, forward runs the block on the native library too (unet_block_*: the
    first-conv kernel or the MFMA rings, BN folded, eval semantics), for every block shape of the
    reference network; ``compute_dtype`` as UNet's (None: the UNET_MI355X_DTYPE default, fp32).
    """

    def __init__(self, in_ch: int, out_ch: int, compute_dtype: str | None = None):
        super().__init__()
        self.net = Sequential(
            Conv2d(in_ch, out_ch, kernel_size=3, padding=1),
            BatchNorm2d(out_ch),
            ReLU(inplace=True),
            Conv2d(out_ch, out_ch, kernel_size=3, padding=1),
            BatchNorm2d(out_ch),
            ReLU(inplace=True),
        )
        self.in_ch, self.out_ch = in_ch, out_ch
        self.compute_dtype = compute_dtype
        self._blocks: dict = {}
        self._packed_sig: dict = {}
        self._lock = threading.Lock()

    def forward(self, x):
        """unet_model.py:19-20 on the native path: NCHW in -> NCHW fp32 out [N, out_ch, H, W]."""
        if not isinstance(x, torch.Tensor) or x.dim() != 4:
            raise RuntimeError("DoubleConv.forward expects a 4-D NCHW tensor")
        if x.shape[1] != self.in_ch:
            raise RuntimeError(f"expected input with {self.in_ch} channels, got {x.shape[1]}")
        if x.device.type != "cuda":
            raise RuntimeError("unet_mi355x: DoubleConv runs only on a ROCm GPU tensor "
                               f"(got device {x.device}); there is no CPU fallback")
        if self.training and torch.is_grad_enabled():
            raise RuntimeError("unet_mi355x.DoubleConv is inference-only (eval BatchNorm folded, no autograd); "
                               "call .eval() or run under torch.no_grad()")
        dtype = self.compute_dtype or DEFAULT_DTYPE
        idx = x.device.index if x.device.index is not None else torch.cuda.current_device()
        with self._lock:
            blk = self._blocks.get((idx, dtype))
            if blk is None:
                blk = self._blocks[(idx, dtype)] = native.Block(self.in_ch, self.out_ch, dtype, idx)
            sd = self.state_dict(keep_vars=True)
            sig = tuple((t.data_ptr(), t._version) for t in sd.values())
            if self._packed_sig.get((idx, dtype)) != sig:
                blk.load_weights(sd)
                self._packed_sig[(idx, dtype)] = sig
        x = x.detach()
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.to(torch.float32).contiguous()
        n, _, h, w = x.shape
        y = torch.empty((n, self.out_ch, h, w), device=x.device, dtype=torch.float32)
        with torch.cuda.device(x.device):
            blk.forward(x, y, torch.cuda.current_stream(x.device).cuda_stream)
        return y

    def close(self):
        for b in self._blocks.values():
            b.close()
        self._blocks.clear()
        self._packed_sig.clear()


class UNet(_Tracked, nn.Module):
    """unet_model.UNet(n_channels=3, n_classes=3) with an MI355X forward.

    compute_dtype: "fp32" (default; exact fp32 MFMA, reference semantics), "bf16" or
    "fp16" (16-bit activations/weights, fp32 accumulation, fp32 head), or "mixed" (bf16 at
    resolution levels 2-4, fp16 at the full-resolution levels 0-1; the benchmark's plan, chosen
    so the masks meet IoU >= 0.999 against fp32).  Default from the UNET_MI355X_DTYPE
    environment variable.

    Inference only: the native forward folds eval-mode BatchNorm and builds no autograd graph, so
    calling it in training mode with grad enabled raises (use the reference module to train).
    """

    def __init__(self, n_channels: int = 3, n_classes: int = 3, compute_dtype: str | None = None,
                 thresholds=(0.25, 0.40, 0.30)):
        super().__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.compute_dtype = compute_dtype or DEFAULT_DTYPE
        if self.compute_dtype not in native.DTYPES:
            raise ValueError(f"compute_dtype must be one of {sorted(native.DTYPES)}")
        self.thresholds = tuple(float(t) for t in thresholds)

        cd = self.compute_dtype   # the blocks' own forward (called stand-alone) uses the model's precision plan
        self.down1 = DoubleConv(n_channels, 64, cd)
        self.down2 = DoubleConv(64, 128, cd)
        self.down3 = DoubleConv(128, 256, cd)
        self.down4 = DoubleConv(256, 512, cd)
        self.pool = MaxPool2d(2)
        self.bottleneck = DoubleConv(512, 1024, cd)
        self.up4 = ConvTranspose2d(1024, 512, 2, stride=2)
        self.conv4 = DoubleConv(1024, 512, cd)
        self.up3 = ConvTranspose2d(512, 256, 2, stride=2)
        self.conv3 = DoubleConv(512, 256, cd)
        self.up2 = ConvTranspose2d(256, 128, 2, stride=2)
        self.conv2 = DoubleConv(256, 128, cd)
        self.up1 = ConvTranspose2d(128, 64, 2, stride=2)
        self.conv1 = DoubleConv(128, 64, cd)
        self.out_conv = Conv2d(64, n_classes, kernel_size=1)
        nn.init.constant_(self.out_conv.bias, -4)  # unet_model.py:52-53

        self._handles: dict[int, native.Handle] = {}
        self._packed_sig: dict[int, tuple] = {}
        self._lock = threading.Lock()
        self._sig_tensors = None
        self._sig_epoch = -1
        self._sig_tracked = False
        # set by the drop-in's private model cache (inference._cached_model), whose model nobody can
        # reach to modify: once packed, its handle skips the per-call weight signature (136 tensors,
        # ~40-50 us of host time on the batch-1 call path)
        self._frozen = False

    # ------------------------------------------------------------------ native plumbing
    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """nn.Module.load_state_dict; every packed handle re-packs at its next use (also when frozen)."""
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        with self._lock:
            self._packed_sig.clear()
        _bump_epoch()
        return out

    def _signature(self):
        """(data_ptr, _version) of every state_dict tensor: changes on any in-place update
        (load_state_dict, optimizer steps, ``with no_grad(): p.add_``), on .to() / .data
        replacement and on re-registration (the cached tensor list is rebuilt then)."""
        if self._sig_epoch != _TREE_EPOCH[0] or self._sig_tensors is None or not self._sig_tracked:
            self._sig_tracked = all(isinstance(m, _Tracked) for m in self.modules())
            self._sig_tensors = list(self.state_dict(keep_vars=True).values())
            self._sig_epoch = _TREE_EPOCH[0]
        return tuple((t.data_ptr(), t._version) for t in self._sig_tensors)

    def native_handle(self, device: torch.device) -> native.Handle:
        """The packed native handle for ``device`` (re-packs if any parameter changed)."""
        if device.type != "cuda":
            raise RuntimeError("unet_mi355x: UNet.forward runs only on a ROCm GPU tensor "
                               f"(got device {device}); there is no CPU fallback")
        idx = device.index if device.index is not None else torch.cuda.current_device()
        with self._lock:
            h = self._handles.get(idx)
            # frozen (the drop-in's private cache): skip the 136-tensor signature while nothing was
            # re-registered or converted anywhere (_TREE_EPOCH) and no load_state_dict ran (it clears
            # _packed_sig); otherwise check it as usual
            if (h is not None and self._frozen and idx in self._packed_sig and self._sig_epoch == _TREE_EPOCH[0]
                    and self._sig_tracked):
                return h
            if h is None:
                h = native.Handle(self.n_channels, self.n_classes, self.compute_dtype, idx,
                                  self.thresholds)
                self._handles[idx] = h
            sig = self._signature()
            if self._packed_sig.get(idx) != sig:
                h.load_weights(self.state_dict())
                self._packed_sig[idx] = sig
        return h

    def _prepack(self, device: torch.device, host_state) -> None:
        """Pack the native handle for ``device`` from ``host_state``: host copies of exactly the module's
        current weights (inference.load_model passes the checkpoint it just assigned), so the pack reads
        no weight back from the device.  The handle then counts as packed for the current weights."""
        idx = device.index if device.index is not None else torch.cuda.current_device()
        with self._lock:
            h = self._handles.get(idx)
            if h is None:
                h = native.Handle(self.n_channels, self.n_classes, self.compute_dtype, idx, self.thresholds)
                self._handles[idx] = h
            h.load_weights(host_state)
            self._packed_sig[idx] = self._signature()

    def _check_input(self, x: torch.Tensor):
        if not isinstance(x, torch.Tensor) or x.dim() != 4:
            raise RuntimeError("UNet.forward expects a 4-D NCHW tensor")
        if x.shape[1] != self.n_channels:
            raise RuntimeError(f"expected input with {self.n_channels} channels, got {x.shape[1]}")
        if x.shape[2] % 16 or x.shape[3] % 16:
            # the reference fails inside torch.cat for such sizes
            raise RuntimeError(f"UNet input H and W must be divisible by 16, got {tuple(x.shape[2:])}")

    def _run(self, x: torch.Tensor, want_logits: bool, mask_kind: int, want_boxes: bool = False,
             out_masks: torch.Tensor | None = None, out_boxes: torch.Tensor | None = None):
        self._check_input(x)
        if self.training and torch.is_grad_enabled():
            raise RuntimeError("unet_mi355x.UNet is inference-only (eval BatchNorm folded, no autograd); "
                               "call .eval() or run under torch.no_grad()")
        h = self.native_handle(x.device)
        x = x.detach()
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.to(torch.float32).contiguous()
        n, _, hh, ww = x.shape
        logits = masks = None
        if want_logits:
            logits = torch.empty((n, self.n_classes, hh, ww), device=x.device, dtype=torch.float32)
        if mask_kind != native.MASK_NONE:
            shape = (n, self.n_classes, hh, ww if mask_kind == native.MASK_U8 else ww // 8)
            if out_masks is not None:   # a caller-owned buffer reused across calls (run_unet)
                if (out_masks.dtype != torch.uint8 or tuple(out_masks.shape) != shape or
                        not out_masks.is_contiguous() or out_masks.device != x.device):
                    raise ValueError(f"out masks must be a contiguous uint8 {shape} tensor on {x.device}")
                masks = out_masks
            else:
                masks = torch.empty(shape, device=x.device, dtype=torch.uint8)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        boxes = None
        h.reserve(n, hh, ww)   # grows the workspace if needed (a no-op otherwise); forwards never allocate
        with torch.cuda.device(x.device):
            if want_boxes:
                boxes = out_boxes if out_boxes is not None else \
                    torch.empty((n, self.n_classes, 4), device=x.device, dtype=torch.int32)
                h.forward_boxes(x, logits, masks, mask_kind, boxes, stream)
            else:
                h.forward(x, logits, masks, mask_kind, stream)
        if want_boxes:
            return logits, masks, boxes
        return logits, masks

    # ------------------------------------------------------------------ public API
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """unet_model.py:55-86: NCHW fp32 in -> NCHW fp32 logits [N, n_classes, H, W]."""
        logits, _ = self._run(x, True, native.MASK_NONE)
        return logits

    def forward_masks(self, x: torch.Tensor, packed: bool = False, with_logits: bool = False):
        """Fused sigmoid + per-class threshold (inference.py:72-79) on the device.

        Returns uint8 masks [N, n_classes, H, W] (0/1), or bit-packed [N, n_classes, H, W/8]
        (bit b of byte j = pixel 8j+b) when ``packed``; with ``with_logits`` also the logits.
        """
        logits, masks = self._run(x, with_logits, native.MASK_BITS if packed else native.MASK_U8)
        return (masks, logits) if with_logits else masks

    def forward_boxes(self, x: torch.Tensor, masks: str | None = None, out=None):
        """Fused masks + per-(image, field) bounding boxes on the device (inference.py:72-90).

        Returns int32 boxes [N, n_classes, 4] = (x_min, y_min, x_max, y_max) in mask pixels,
        inclusive, (-1, -1, -1, -1) for an empty mask -- the np.where -> min/max of run_unet.
        ``masks`` = None (boxes only), "u8" or "bits": also return that mask tensor first.
        ``out`` = (masks tensor or None, boxes tensor): caller-owned device buffers to fill.
        """
        kind = {None: native.MASK_NONE, "u8": native.MASK_U8, "bits": native.MASK_BITS}[masks]
        om, ob = out if out is not None else (None, None)
        _, m, boxes = self._run(x, False, kind, want_boxes=True, out_masks=om, out_boxes=ob)
        return boxes if masks is None else (m, boxes)

    def preprocess(self, img: torch.Tensor, size: int = 512, out: torch.Tensor | None = None) -> torch.Tensor:
        """inference.py:62-64 + :30-44 on the device: a photo as uint8 [H, W, 3] (RGB) or
        [H, W] / [H, W, 1] (L) device tensor -> fp32 [1, 3, size, size] network input, with
        Pillow's default BICUBIC resize reproduced bit-exactly (csrc/unet_preprocess.hip).
        ``out`` (optional, fp32 [3, size, size] contiguous, e.g. a slot of a batch) is filled
        in place."""
        if img.dim() == 2:
            img = img.unsqueeze(-1)
        if img.device.type != "cuda":
            raise RuntimeError("unet_mi355x: preprocess runs on a ROCm GPU tensor; there is no CPU fallback")
        img = img.contiguous()
        h = self.native_handle(img.device)
        dst = out if out is not None else torch.empty((3, size, size), device=img.device, dtype=torch.float32)
        with torch.cuda.device(img.device):
            h.preprocess(img, dst, torch.cuda.current_stream(img.device).cuda_stream)
        return dst.unsqueeze(0) if out is None else out

    def reserve(self, n: int, h: int, w: int, device=None) -> None:
        """Pre-allocate the native workspace (so forwards do not allocate)."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        self.native_handle(dev).reserve(n, h, w)

    def intermediate(self, name: str, device=None) -> torch.Tensor:
        """Intermediate activation of the last forward as fp32 NCHW (debug / per-layer parity)."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        h = self.native_handle(dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        numel = h.debug_fetch(name, stream)
        out = torch.empty(numel, device=dev, dtype=torch.float32)
        with torch.cuda.device(dev):
            h.debug_fetch_into(name, out, stream)
        return out

    def close(self):
        for h in self._handles.values():
            h.close()
        self._handles.clear()
        self._packed_sig.clear()
        for m in self.modules():
            if isinstance(m, DoubleConv):
                m.close()
