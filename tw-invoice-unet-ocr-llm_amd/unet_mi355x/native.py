"""ctypes binding of libunet_mi355x.so (the C-ABI declared in include/unet_mi355x.h).

torch is imported first on purpose: the library's NEEDED ``libamdhip64.so.7`` then
resolves to the HIP runtime torch already loaded, so torch device pointers and
``torch.cuda`` streams are valid inside the library.  There is no fallback: if the
library is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import numpy as np
import torch  # noqa: F401  (must precede the library load, see module docstring)

LIB_NAME = "libunet_mi355x.so"
LIB_PATH = os.environ.get("UNET_MI355X_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

UNET_OK, UNET_EINVAL, UNET_ESHAPE, UNET_ENOMEM, UNET_EHIP, UNET_ESTATE, UNET_EKEY = 0, -1, -2, -3, -4, -5, -6
# "mixed": bf16 storage at resolution levels 2-4, fp16 at levels 0-1 (include/unet_mi355x.h)
# "fp32": fp32 storage, every product as three bf16 terms per operand (fp32 accuracy on the bf16 MFMA pipe);
# "fp32_exact": the same plan on the exact-fp32 MFMA
DTYPES = {"fp32": 0, "float32": 0, "bf16": 1, "bfloat16": 1, "fp16": 2, "float16": 2, "mixed": 3, "fp32_exact": 4}
MASK_NONE, MASK_U8, MASK_BITS = 0, 1, 2
LAYOUT_NCHW, LAYOUT_NHWC = 0, 1
COMM_ID_BYTES = 128
ABI_VERSION = 5   # include/unet_mi355x.h UNET_ABI_VERSION
IN_F32, IN_U8 = 0, 1

# every function include/unet_mi355x.h declares: name -> (restype, argtypes)
_vp, _i, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t


class UnetConfig(ctypes.Structure):
    _fields_ = [("n_channels", ctypes.c_int), ("n_classes", ctypes.c_int), ("dtype", ctypes.c_int),
                ("device", ctypes.c_int), ("thresholds", ctypes.c_float * 4)]


class TensorView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("dtype", ctypes.c_int),
                ("ndim", ctypes.c_int), ("shape", ctypes.c_int64 * 4)]


class BlockConfig(ctypes.Structure):
    _fields_ = [("in_ch", ctypes.c_int), ("out_ch", ctypes.c_int), ("dtype", ctypes.c_int), ("device", ctypes.c_int)]


def tensor_views(state_dict):
    """state_dict (name -> torch.Tensor / np.ndarray, any device) -> (TensorView array, arrays to keep alive):
    floating tensors as contiguous host fp32 (numpy has no bfloat16: a model cast with .to(torch.bfloat16)
    loads like the reference UNet does, its parameters simply read back in fp32), integers as int64."""
    keep, views = [], []
    for k, v in state_dict.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu()
            arr = (v.to(torch.float32) if v.is_floating_point() else v).numpy()
        else:
            arr = np.asarray(v)
        if arr.dtype.kind == "f":
            arr = np.ascontiguousarray(arr, dtype=np.float32)
            code = 0
        else:
            arr = np.ascontiguousarray(arr, dtype=np.int64)
            code = 1
        keep.append(arr)
        shape = list(arr.shape) + [0] * (4 - arr.ndim)
        views.append(TensorView(k.encode(), arr.ctypes.data, code, arr.ndim, (ctypes.c_int64 * 4)(*shape)))
    return (TensorView * len(views))(*views), keep


SIGNATURES = {
    "unet_create": (_i, [ctypes.POINTER(UnetConfig), ctypes.POINTER(_vp)]),
    "unet_load_weights": (_i, [_vp, ctypes.POINTER(TensorView), _i]),
    "unet_workspace_bytes": (_sz, [_vp, _i, _i, _i]),
    "unet_reserve": (_i, [_vp, _i, _i, _i]),
    "unet_forward": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp]),
    "unet_forward_boxes": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _i, _i, _i, _vp]),
    "unet_preprocess": (_i, [_vp, _vp, _i, _i, _i, _vp, _i, _i, _vp]),
    "unet_crop_stats": (_i, [_vp, _i, _i, _i, _vp, _i, _i, _i, ctypes.c_double, _vp, _vp, _vp]),
    "unet_num_launches": (_i, []),
    "unet_launch_label": (ctypes.c_char_p, [_vp, _i]),
    "unet_launch_label_at": (ctypes.c_char_p, [_vp, _i, _i, _i, _i]),
    "unet_small_batch_limit": (_i, [_vp]),
    "unet_photo_graph_create": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _i, _vp, _i, _vp, ctypes.c_double, _vp, _vp,
                                     _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "unet_photo_graph_set_masks": (_i, [_vp, _vp]),
    "unet_forward_timed": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp, ctypes.POINTER(ctypes.c_float)]),
    "unet_debug_fetch": (_i, [_vp, ctypes.c_char_p, _vp, ctypes.POINTER(_sz), _vp]),
    "unet_graph_create": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _i, _i, _i, ctypes.POINTER(_vp)]),
    "unet_graph_launch": (_i, [_vp, _vp]),
    "unet_graph_destroy": (_i, [_vp]),
    "unet_comm_get_unique_id": (_i, [_vp]),
    "unet_comm_init": (_i, [_vp, _i, _i, _vp]),
    "unet_allgather": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "unet_comm_destroy": (_i, [_vp]),
    "unet_destroy": (_i, [_vp]),
    "unet_block_create": (_i, [ctypes.POINTER(BlockConfig), ctypes.POINTER(_vp)]),
    "unet_block_load_weights": (_i, [_vp, ctypes.POINTER(TensorView), _i]),
    "unet_block_reserve": (_i, [_vp, _i, _i, _i]),
    "unet_block_forward": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp]),
    "unet_block_destroy": (_i, [_vp]),
    "unet_last_error": (ctypes.c_char_p, []),
    "unet_abi_version": (_i, []),
    "unet_logit_cut": (ctypes.c_float, [ctypes.c_float]),
}

_lib = None
_lib_lock = threading.Lock()
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def kernel_sources_sha256() -> str:
    """sha256 over the library's sources (csrc/*.hip, *.cpp, *.h, in name order): stamped into
    the PMC summaries (tools/pmc_summary.py) so bench.py can tell whether a traffic figure was
    collected on the kernels it is timing."""
    import hashlib
    h = hashlib.sha256()
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".cpp", ".h")):
            h.update(name.encode())
            with open(os.path.join(CSRC, name), "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def load_library(path: str = LIB_PATH):
    """Load (once) and type the native library; raises RuntimeError if it is absent."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"unet_mi355x: native library {path} not built; run "
                "`make -C tw-invoice-unet-ocr-llm_amd/csrc` (or __graft_entry__.build()). "
                "There is no CPU/PyTorch fallback.")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.unet_abi_version() != ABI_VERSION:
            raise RuntimeError("unet_mi355x: ABI version mismatch")
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc == UNET_OK:
        return
    msg = f"{what}: {load_library().unet_last_error().decode(errors='replace')}"
    if rc == UNET_EINVAL:
        raise ValueError(msg)
    if rc == UNET_ENOMEM:
        raise torch.cuda.OutOfMemoryError(msg) if hasattr(torch.cuda, "OutOfMemoryError") else MemoryError(msg)
    raise RuntimeError(msg)


def crop_stats(img: torch.Tensor, boxes: torch.Tensor, box_h: int, box_w: int, pad: float,
               rects: torch.Tensor, sums: torch.Tensor, stream: int) -> None:
    """unet_crop_stats: crop rectangles (int32 [n, 4]) and crop pixel sums (int64 [n]) of the mask
    boxes (int32 [n, 4]) on the uint8 HWC device photo ``img``, with run_unet's arithmetic."""
    if img.dtype != torch.uint8 or img.dim() != 3 or not img.is_contiguous():
        raise ValueError("img must be a contiguous uint8 [H, W, C] device tensor")
    n = boxes.numel() // 4
    for t, dt, shape in ((boxes, torch.int32, (n, 4)), (rects, torch.int32, (n, 4)), (sums, torch.int64, (n,))):
        if t.dtype != dt or t.numel() != int(np.prod(shape)) or not t.is_contiguous() or t.device != img.device:
            raise ValueError(f"crop_stats: expected a contiguous {dt} tensor of {shape} on {img.device}")
    ih, iw, c = img.shape
    check(load_library().unet_crop_stats(img.data_ptr(), ih, iw, c, boxes.data_ptr(), n, box_h, box_w, float(pad),
                                         rects.data_ptr(), sums.data_ptr(), stream), "unet_crop_stats")


class Handle:
    """One native handle = one device, one packed weight set, one workspace.  Calls are serialised
    on the host by ``lock``; on the device the library orders a call issued on another stream
    after the previous one (include/unet_mi355x.h)."""

    def __init__(self, n_channels: int, n_classes: int, dtype: str, device: int,
                 thresholds=(0.25, 0.40, 0.30, 0.5)):
        self.lib = load_library()
        self.n_channels, self.n_classes, self.device = n_channels, n_classes, device
        self.dtype = dtype
        cfg = UnetConfig(n_channels, n_classes, DTYPES[dtype], device,
                         (ctypes.c_float * 4)(*[float(t) for t in list(thresholds)[:4]] +
                                              [0.5] * (4 - len(list(thresholds)[:4]))))
        h = ctypes.c_void_p()
        check(self.lib.unet_create(ctypes.byref(cfg), ctypes.byref(h)), "unet_create")
        self._h = h
        # re-entrant: a Graph's close (unet_graph_destroy drains the handle's pending work and clears its
        # stream-order state) takes it too, and may run from a garbage collection inside a locked call
        self.lock = threading.RLock()
        self._graphs = weakref.WeakSet()   # captured graphs die before the handle

    def load_weights(self, state_dict) -> None:
        """state_dict: mapping name -> torch.Tensor / np.ndarray (any device); strict."""
        arr_t, _keep = tensor_views(state_dict)
        with self.lock:
            check(self.lib.unet_load_weights(self._h, arr_t, len(arr_t)), "unet_load_weights")

    def workspace_bytes(self, n: int, h: int, w: int) -> int:
        return int(self.lib.unet_workspace_bytes(self._h, n, h, w))

    def reserve(self, n: int, h: int, w: int) -> None:
        with self.lock:
            check(self.lib.unet_reserve(self._h, n, h, w), "unet_reserve")

    @staticmethod
    def _geometry(x: torch.Tensor, layout: int):
        if x.dtype not in (torch.float32, torch.uint8) or not x.is_contiguous():
            raise ValueError("x must be a contiguous float32 or uint8 tensor")
        if layout == LAYOUT_NCHW:
            n, c, h, w = x.shape
        else:
            n, h, w, c = x.shape
        return n, h, w, IN_F32 if x.dtype == torch.float32 else IN_U8

    def forward(self, x: torch.Tensor, logits: torch.Tensor | None, masks: torch.Tensor | None,
                mask_kind: int, stream: int, layout: int = LAYOUT_NCHW) -> None:
        """x: device [N, C, H, W] (layout NCHW) or [N, H, W, C] (NHWC), float32 or uint8 (/255).
        The workspace must have been reserved for (N, H, W) (``reserve``)."""
        n, h, w, xdt = self._geometry(x, layout)
        with self.lock:
            check(self.lib.unet_forward(self._h, x.data_ptr(), layout, xdt,
                                        None if logits is None else logits.data_ptr(),
                                        None if masks is None else masks.data_ptr(),
                                        mask_kind, n, h, w, stream), "unet_forward")

    def forward_boxes(self, x: torch.Tensor, logits: torch.Tensor | None, masks: torch.Tensor | None,
                      mask_kind: int, boxes: torch.Tensor, stream: int, layout: int = LAYOUT_NCHW) -> None:
        """forward + per-(image, field) mask boxes: int32 [N][n_classes][4] = x0, y0, x1, y1 (-1s if empty)."""
        n, h, w, xdt = self._geometry(x, layout)
        if boxes.dtype != torch.int32 or tuple(boxes.shape) != (n, self.n_classes, 4) or not boxes.is_contiguous():
            raise ValueError(f"boxes must be a contiguous int32 tensor of shape {(n, self.n_classes, 4)}")
        with self.lock:
            check(self.lib.unet_forward_boxes(self._h, x.data_ptr(), layout, xdt,
                                              None if logits is None else logits.data_ptr(),
                                              None if masks is None else masks.data_ptr(),
                                              mask_kind, boxes.data_ptr(), n, h, w, stream), "unet_forward_boxes")

    def preprocess(self, img: torch.Tensor, out: torch.Tensor, stream: int) -> None:
        """uint8 HWC image (device) -> fp32 [3, oh, ow] (device, ``out``): Pillow-exact resize + /255."""
        if img.dtype != torch.uint8 or img.dim() != 3 or not img.is_contiguous():
            raise ValueError("img must be a contiguous uint8 [H, W, C] device tensor")
        if out.dtype != torch.float32 or out.dim() != 3 or out.shape[0] != 3 or not out.is_contiguous():
            raise ValueError("out must be a contiguous float32 [3, oh, ow] device tensor")
        ih, iw, c = img.shape
        with self.lock:
            check(self.lib.unet_preprocess(self._h, img.data_ptr(), ih, iw, c, out.data_ptr(),
                                           out.shape[1], out.shape[2], stream), "unet_preprocess")

    def forward_timed(self, x: torch.Tensor, logits: torch.Tensor | None, masks: torch.Tensor | None,
                      mask_kind: int, stream: int, layout: int = LAYOUT_NCHW) -> list:
        """forward + HIP-event time (ms) of every launch, in include/unet_mi355x.h order."""
        n, h, w, xdt = self._geometry(x, layout)
        nl = self.lib.unet_num_launches()
        ms = (ctypes.c_float * nl)()
        with self.lock:
            check(self.lib.unet_forward_timed(self._h, x.data_ptr(), layout, xdt,
                                              None if logits is None else logits.data_ptr(),
                                              None if masks is None else masks.data_ptr(),
                                              mask_kind, n, h, w, stream, ms), "unet_forward_timed")
        return list(ms)

    def graph(self, x: torch.Tensor, logits: torch.Tensor | None, masks: torch.Tensor | None, mask_kind: int,
              boxes: torch.Tensor | None = None, layout: int = LAYOUT_NCHW) -> "Graph":
        """Capture one forward over these fixed buffers into a hipGraph (unet_graph_create)."""
        n, h, w, xdt = self._geometry(x, layout)
        g = ctypes.c_void_p()
        with self.lock:
            check(self.lib.unet_graph_create(self._h, x.data_ptr(), layout, xdt,
                                             None if logits is None else logits.data_ptr(),
                                             None if masks is None else masks.data_ptr(), mask_kind,
                                             None if boxes is None else boxes.data_ptr(), n, h, w,
                                             ctypes.byref(g)), "unet_graph_create")
        gr = Graph(self, g, (x, logits, masks, boxes))
        self._graphs.add(gr)
        return gr

    def photo_graph(self, h_img: torch.Tensor | None, img: torch.Tensor, x: torch.Tensor, masks: torch.Tensor | None,
                    mask_kind: int, boxes: torch.Tensor, pad: float, rects: torch.Tensor, sums: torch.Tensor,
                    h_masks=None, h_boxes=None, h_rects=None, h_sums=None) -> "Graph":
        """unet_photo_graph_create: upload (pinned ``h_img`` -> ``img``) + preprocess into ``x`` + forward with
        masks and boxes at N = 1 + crop statistics + copies into the pinned host tensors given, as one
        graph (run_unet's device work for one photo geometry)."""
        if img.dtype != torch.uint8 or img.dim() != 3 or not img.is_contiguous():
            raise ValueError("img must be a contiguous uint8 [H, W, C] device tensor")
        size = x.shape[-1]
        if x.dtype != torch.float32 or x.numel() != 3 * size * size or not x.is_contiguous():
            raise ValueError("x must be a contiguous float32 [1, 3, S, S] device tensor")
        for t in (h_img, h_masks, h_boxes, h_rects, h_sums):
            if t is not None and (t.device.type != "cpu" or not t.is_pinned() or not t.is_contiguous()):
                raise ValueError("host buffers of a photo graph must be contiguous pinned CPU tensors")
        if h_img is not None and h_img.numel() < img.numel():
            raise ValueError("h_img is smaller than img")
        ih, iw, c = img.shape
        ptr = lambda t: None if t is None else t.data_ptr()   # noqa: E731
        g = ctypes.c_void_p()
        with self.lock:
            check(self.lib.unet_photo_graph_create(self._h, ptr(h_img), img.data_ptr(), ih, iw, c, x.data_ptr(), size,
                                                   ptr(masks), mask_kind, boxes.data_ptr(), float(pad),
                                                   rects.data_ptr(), sums.data_ptr(), ptr(h_masks), ptr(h_boxes),
                                                   ptr(h_rects), ptr(h_sums), ctypes.byref(g)),
                  "unet_photo_graph_create")
        gr = Graph(self, g, (h_img, img, x, masks, boxes, rects, sums, h_masks, h_boxes, h_rects, h_sums),
                   masks_ptr=0 if h_masks is None else h_masks.data_ptr())
        self._graphs.add(gr)
        return gr

    def small_batch_limit(self) -> int:
        """Largest N of the small-batch (split-K) plan; 0 when it is off (include/unet_mi355x.h)."""
        return int(self.lib.unet_small_batch_limit(self._h))

    def launch_labels_at(self, n: int, h: int, w: int) -> list:
        """launch_labels for a forward of n x h x w (the small-batch plan's kernels at n <= its limit)."""
        return [self.lib.unet_launch_label_at(self._h, i, n, h, w).decode() for i in range(self.lib.unet_num_launches())]

    # ---- multi-GPU extras (include/unet_mi355x.h): RCCL all-gather for a host without torch.distributed
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        check(load_library().unet_comm_get_unique_id(buf), "unet_comm_get_unique_id")
        return buf.raw

    def comm_init(self, rank: int, nranks: int, uid: bytes) -> None:
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        with self.lock:
            check(self.lib.unet_comm_init(self._h, rank, nranks, buf), "unet_comm_init")
        self.nranks = nranks

    def allgather(self, send: torch.Tensor, recv: torch.Tensor, stream: int) -> None:
        """recv[r] = rank r's ``send`` (contiguous device tensors, recv = nranks x send bytes)."""
        if not (send.is_contiguous() and recv.is_contiguous()):
            raise ValueError("send and recv must be contiguous")
        nranks = getattr(self, "nranks", None)
        if nranks is None:
            raise RuntimeError("unet_allgather: no communicator, call comm_init first")
        sb = send.numel() * send.element_size()
        if recv.numel() * recv.element_size() != nranks * sb:   # RCCL would write past a short recv
            raise ValueError(f"recv holds {recv.numel() * recv.element_size()} bytes, expected nranks x send = "
                             f"{nranks} x {sb}")
        with self.lock:
            check(self.lib.unet_allgather(self._h, send.data_ptr(), recv.data_ptr(),
                                          sb, stream), "unet_allgather")

    def comm_destroy(self) -> None:
        with self.lock:
            check(self.lib.unet_comm_destroy(self._h), "unet_comm_destroy")
        self.nranks = None

    def launch_labels(self) -> list:
        """Kernel instantiation of every launch of a forward (include/unet_mi355x.h order)."""
        return [self.lib.unet_launch_label(self._h, i).decode() for i in range(self.lib.unet_num_launches())]

    def debug_fetch(self, name: str, stream: int) -> int:
        cnt = ctypes.c_size_t(0)
        check(self.lib.unet_debug_fetch(self._h, name.encode(), None, ctypes.byref(cnt), stream), "unet_debug_fetch")
        return int(cnt.value)

    def debug_fetch_into(self, name: str, dst: torch.Tensor, stream: int) -> None:
        cnt = ctypes.c_size_t(0)
        check(self.lib.unet_debug_fetch(self._h, name.encode(), dst.data_ptr(), ctypes.byref(cnt), stream),
              "unet_debug_fetch")

    def close(self) -> None:
        for gr in list(getattr(self, "_graphs", ())):
            gr.close()
        if getattr(self, "_h", None):
            with self.lock:
                if self._h:
                    self.lib.unet_destroy(self._h)
                    self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Block:
    """A stand-alone DoubleConv (unet_block_*): conv3x3 + BN + ReLU twice on the network's kernels."""

    def __init__(self, in_ch: int, out_ch: int, dtype: str, device: int):
        self.lib = load_library()
        self.in_ch, self.out_ch, self.dtype, self.device = in_ch, out_ch, dtype, device
        b = ctypes.c_void_p()
        check(self.lib.unet_block_create(ctypes.byref(BlockConfig(in_ch, out_ch, DTYPES[dtype], device)), ctypes.byref(b)),
              "unet_block_create")
        self._b = b
        self.lock = threading.Lock()

    def load_weights(self, state_dict) -> None:
        arr_t, _keep = tensor_views(state_dict)
        with self.lock:
            check(self.lib.unet_block_load_weights(self._b, arr_t, len(arr_t)), "unet_block_load_weights")

    def forward(self, x: torch.Tensor, y: torch.Tensor, stream: int) -> None:
        """x: device fp32 NCHW [N, in_ch, H, W] -> y: device fp32 NCHW [N, out_ch, H, W] (contiguous)."""
        n, c, h, w = x.shape
        if x.dtype != torch.float32 or not x.is_contiguous() or c != self.in_ch:
            raise ValueError(f"x must be a contiguous float32 [N, {self.in_ch}, H, W] tensor")
        if y.dtype != torch.float32 or not y.is_contiguous() or tuple(y.shape) != (n, self.out_ch, h, w):
            raise ValueError(f"y must be a contiguous float32 {(n, self.out_ch, h, w)} tensor")
        with self.lock:
            check(self.lib.unet_block_reserve(self._b, n, h, w), "unet_block_reserve")
            check(self.lib.unet_block_forward(self._b, x.data_ptr(), y.data_ptr(), n, h, w, stream), "unet_block_forward")

    def close(self) -> None:
        if getattr(self, "_b", None):
            self.lib.unet_block_destroy(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Graph:
    """A captured forward (unet_graph_*); keeps its buffers alive; replay with ``launch``."""

    def __init__(self, handle: Handle, g: ctypes.c_void_p, buffers, masks_ptr: int = 0):
        self.handle, self._g, self._buffers = handle, g, buffers
        self.masks_ptr = masks_ptr   # a photo graph's current masks copy destination (host pointer)

    def launch(self, stream: int) -> None:
        with self.handle.lock:
            check(self.handle.lib.unet_graph_launch(self._g, stream), "unet_graph_launch")

    def set_masks(self, h_masks: torch.Tensor) -> None:
        """unet_photo_graph_set_masks: the next replays copy the masks into ``h_masks`` (pinned, contiguous,
        the size of the masks the graph was captured with)."""
        if h_masks.device.type != "cpu" or not h_masks.is_pinned() or not h_masks.is_contiguous():
            raise ValueError("h_masks must be a contiguous pinned CPU tensor")
        cur = self._buffers[7]
        if cur is None or h_masks.numel() * h_masks.element_size() != cur.numel() * cur.element_size():
            raise ValueError("h_masks must have the size of the graph's masks buffer")
        with self.handle.lock:
            check(self.handle.lib.unet_photo_graph_set_masks(self._g, h_masks.data_ptr()), "unet_photo_graph_set_masks")
        self._masks_target = h_masks   # kept alive while the graph may copy into it
        self.masks_ptr = h_masks.data_ptr()

    def close(self) -> None:
        """unet_graph_destroy under the handle's lock: it drains the handle (reads and clears the stream-order
        state a forward on another thread and stream sets), so it must not run beside a call of the handle."""
        if getattr(self, "_g", None):
            with self.handle.lock:
                if self._g:
                    self.handle.lib.unet_graph_destroy(self._g)
                    self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
