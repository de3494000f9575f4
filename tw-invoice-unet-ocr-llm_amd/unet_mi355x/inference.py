"""Drop-in for the reference ``inference.py`` (inference.py:1-129) on the MI355X path.

Same module constants (DEVICE, IMG_SIZE, FIELDS) and functions (load_model,
preprocess, run_unet) with the same arguments, return values and error classes.
Differences are internal only:
  * the model is cached per (checkpoint, mtime, device) instead of re-loaded on every
    call (the reference re-reads the 124 MB checkpoint per call, inference.py:58);
  * sigmoid + thresholds run fused in the native head kernel (masks come back as
    uint8), so the 3x512x512 fp32 probability map never leaves the GPU;
  * the per-field bounding boxes (np.where -> min/max, inference.py:84-90) are computed
    on the GPU too (unet_forward_boxes); the scale / 15 % pad / crop stays on the host;
  * RGB / L photos are resized on the GPU (unet_preprocess, bit-exact with Pillow's
    BICUBIC resize), so only the original uint8 photo crosses PCIe (an RGB photo as Pillow's own
    RGBX pixels, copied out without repacking);
  * for RGB / L photos the call's device work -- photo upload, resize, forward with masks and
    boxes, crop statistics and the copies back -- is one hipGraph per photo geometry
    (unet_photo_graph_create), replayed with one host call and one synchronisation.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from collections import OrderedDict

import numpy as np
import torch
from PIL import Image

from . import native
from .model import UNet

DEVICE = "cuda" if torch.cuda.is_available() else "cpu"   # inference.py:9
IMG_SIZE = 512                                            # inference.py:10
FIELDS = ["invoice_no", "date", "total_amount"]           # inference.py:12
THRESHOLDS = (0.25, 0.40, 0.30)                           # inference.py:76-78
CROP_PAD = 0.15                                           # inference.py:106-107

_cache: dict = {}
_cache_lock = threading.Lock()


def load_model(checkpoint_path: str, compute_dtype: str | None = None):
    """inference.py:17-24: UNet(3,3) on DEVICE, strict state_dict load, eval().  The module is built on
    DEVICE (its random initialisation runs there, not as 31 M host draws; the meta device would cost
    ~0.7 s of one-time setup in a fresh process) and takes the checkpoint's tensors (strict,
    assign=True), and the native handle is packed from the host copies the checkpoint was read into (no
    read-back of the weights from the device): the cold start of the first run_unet."""
    state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    with torch.device(DEVICE):
        model = UNet(n_channels=3, n_classes=3, compute_dtype=compute_dtype, thresholds=THRESHOLDS)
    model.load_state_dict({k: v.to(DEVICE) for k, v in state.items()}, assign=True)
    model.eval()
    if str(DEVICE).startswith("cuda"):
        model._prepack(torch.device(DEVICE), state)
    return model


def _cached_model(checkpoint_path: str, compute_dtype: str | None = None):
    key = (os.path.abspath(checkpoint_path), os.path.getmtime(checkpoint_path), DEVICE, compute_dtype)
    with _cache_lock:
        m = _cache.get(key)
        if m is None:
            m = load_model(checkpoint_path, compute_dtype)
            m._frozen = True   # private to the cache: its weights never change after the load
            _cache.clear()
            _cache[key] = m
        return m


def preprocess_array(pil_img: Image.Image) -> np.ndarray:
    """Host half of inference.py:30-44: RGB, resize to 512 (PIL default filter), /255, CHW."""
    img = pil_img.convert("RGB").resize((IMG_SIZE, IMG_SIZE))
    arr = np.array(img).astype(np.float32) / 255.0
    if arr.ndim != 3 or arr.shape[2] != 3:
        raise ValueError(f"Invalid image shape: {arr.shape}")
    return arr.transpose(2, 0, 1)


def preprocess(pil_img: Image.Image) -> torch.Tensor:
    """inference.py:30-44: PIL -> Tensor [1, 3, 512, 512] fp32 on DEVICE."""
    return torch.from_numpy(preprocess_array(pil_img)).unsqueeze(0).to(DEVICE)


def crop_rect(box, ow: int, oh: int):
    """inference.py:96-112: mask-space box (x_min, y_min, x_max, y_max) -> crop rectangle in
    photo pixels (float64 scale, int() truncation, 15 % pad, clamp).  The device twin is
    unet_crop_stats (csrc/unet_preprocess.hip, crop_rect)."""
    mx1, my1, mx2, my2 = (int(v) for v in box)
    scale_x, scale_y = ow / IMG_SIZE, oh / IMG_SIZE
    x1, x2 = int(mx1 * scale_x), int(mx2 * scale_x)
    y1, y2 = int(my1 * scale_y), int(my2 * scale_y)
    pad_x, pad_y = int((x2 - x1) * CROP_PAD), int((y2 - y1) * CROP_PAD)
    return max(0, x1 - pad_x), max(0, y1 - pad_y), min(ow, x2 + pad_x), min(oh, y2 + pad_y)


def crop_from_box(pil_img: Image.Image, box):
    """inference.py:92-127 for one field: mask-space box (x_min, y_min, x_max, y_max), or None
    for an empty mask -> original scale -> 15% pad -> clamp -> crop, rejecting degenerate and
    near-black crops (None)."""
    if box is None:
        return None
    x1, y1, x2, y2 = crop_rect(box, *pil_img.size)
    if x2 <= x1 or y2 <= y1:
        return None
    crop = pil_img.crop((x1, y1, x2, y2))
    arr = np.array(crop)
    if arr.size == 0 or arr.mean() < 3:
        return None
    return crop


def crop_from_stats(pil_img: Image.Image, rect, pixel_sum: int, channels: int):
    """crop_from_box from device crop statistics (unet_crop_stats): the rectangle and the sum of
    the crop's uint8 values.  np.array(crop).mean() < 3 is pixel_sum < 3 * count exactly (numpy
    sums the integers in float64 without rounding below 2^53), so no crop pixel is read here."""
    x1, y1, x2, y2 = (int(v) for v in rect)
    if x2 <= x1 or y2 <= y1:   # also the -1s of an empty mask
        return None
    if int(pixel_sum) < 3 * (x2 - x1) * (y2 - y1) * channels:
        return None
    return pil_img.crop((x1, y1, x2, y2))


def boxes_to_crops(pil_img: Image.Image, boxes) -> dict:
    """Crops from device-computed mask boxes (int32 [n_fields, 4], -1s = empty mask)."""
    b = np.asarray(boxes)
    return {k: crop_from_box(pil_img, None if b[i, 2] < 0 else b[i]) for i, k in enumerate(FIELDS)}


def photo_array(pil_img: Image.Image) -> np.ndarray:
    """np.asarray(pil_img) of an RGB / L photo ([H, W, 3] / [H, W] uint8), packed by ONE raw-encoder
    pass into one buffer: Image.tobytes (behind np.asarray) packs in 64 KB pieces and joins them,
    about half again the time of the pack itself (40 us of a 600x400 photo on the GPU box's host).
    Any other outcome of the encoder falls back to np.asarray."""
    w, h = pil_img.size
    c = 3 if pil_img.mode == "RGB" else 1
    shape = (h, w, 3) if c == 3 else (h, w)
    if pil_img.mode not in ("RGB", "L") or w == 0 or h == 0:
        return np.asarray(pil_img)
    try:
        pil_img.load()
        enc = Image._getencoder(pil_img.mode, "raw", pil_img.mode)
        enc.setimage(pil_img.im, (0, 0, w, h))
        _, err, data = enc.encode(w * h * c + 65536)
    except Exception:   # an encoder API this Pillow does not have
        return np.asarray(pil_img)
    if err != 1 or len(data) != w * h * c:
        return np.asarray(pil_img)
    return np.frombuffer(data, np.uint8).reshape(shape)


class _ArrowArray(ctypes.Structure):
    """The Arrow C data interface's ArrowArray (a stable ABI)."""


_ArrowArray._fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                        ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64),
                        ("buffers", ctypes.POINTER(ctypes.c_void_p)),
                        ("children", ctypes.POINTER(ctypes.POINTER(_ArrowArray))),
                        ("dictionary", ctypes.POINTER(_ArrowArray)), ("release", ctypes.c_void_p),
                        ("private_data", ctypes.c_void_p)]
_capsule_pointer = ctypes.pythonapi.PyCapsule_GetPointer
_capsule_pointer.restype = ctypes.c_void_p
_capsule_pointer.argtypes = [ctypes.py_object, ctypes.c_char_p]


def copy_rgbx(pil_img: Image.Image, dst_ptr: int, capacity: int):
    """Copy an "RGB" photo's pixels as Pillow holds them -- RGBX, 4 bytes per pixel -- to dst_ptr, without
    the 3-byte repacking np.asarray does (about 60 us of a 600x400 photo on the GPU box's host): through
    Pillow's zero-copy Arrow export of the image (a fixed-size list of 4 uint8 per pixel, one memory block).
    Returns (H, W, 4), or None when the export is not available -- another mode (Pillow's export of "L"
    images is not used: it crashes in Pillow 12), an image split over several memory blocks, an older
    Pillow -- and the caller packs the photo instead."""
    if pil_img.mode != "RGB":
        return None
    w, h = pil_img.size
    n = w * h * 4
    if n == 0 or n > capacity:
        return None
    try:
        pil_img.load()
        cap = pil_img.im.__arrow_c_array__()
    except (AttributeError, ValueError, TypeError):
        return None
    try:
        a = ctypes.cast(_capsule_pointer(cap, b"arrow_array"), ctypes.POINTER(_ArrowArray)).contents
        if a.length != w * h or a.n_children != 1 or a.offset != 0:
            return None
        c = a.children[0].contents
        if c.length != n or c.offset != 0 or c.n_buffers < 2 or not c.buffers[1]:
            return None
        ctypes.memmove(dst_ptr, c.buffers[1], n)
    except (ValueError, TypeError):
        return None
    finally:
        del cap   # the capsule's destructor releases the export (Pillow keeps the image alive until then)
    return (h, w, 4)


class _MaskPool:
    """Pinned [n_fields, 512, 512] blocks that run_unet returns its masks in (the photo graph DMAs the masks
    straight into one, and run_unet hands out bool views of it instead of copying 768 KB out of a shared
    pinned buffer: about 27 us per call on the GPU box's host, the data being cold after the DMA).

    A block is lent with an owner object (a ctypes array over the pinned memory) that the returned bool
    array is built on: every mask view keeps it alive, and a weakref.finalize on it hands the block back
    when the last view dies -- however the caller drops them, and also when run_unet fails after taking
    the block.  At most ``size`` blocks; when all are lent, ``take`` returns None (run_unet then copies)."""

    def __init__(self, shape, size: int = 4):
        self.shape, self.size = tuple(shape), size
        self.blocks: list = []    # pinned uint8 tensors
        self.idle: list = []      # per block: not lent

    def take(self):
        """(pinned block tensor, bool array over it whose views hand it back when they are all gone), or None."""
        for i, ok in enumerate(self.idle):
            if ok:
                break
        else:
            if len(self.blocks) >= self.size:
                return None
            self.blocks.append(torch.empty(self.shape, dtype=torch.uint8, pin_memory=True))
            self.idle.append(True)
            i = len(self.blocks) - 1
        self.idle[i] = False
        t = self.blocks[i]
        owner = (ctypes.c_ubyte * t.numel()).from_address(t.data_ptr())
        arr = np.frombuffer(owner, dtype=np.bool_).reshape(self.shape)
        weakref.finalize(owner, self._give_back, i)
        return t, arr

    def _give_back(self, i: int):
        self.idle[i] = True   # one list item store: safe from the finaliser's thread


class _Staging:
    """Buffers of one device's run_unet calls, reused across calls: the photo (pinned host + device),
    the network input, the u8 masks and boxes, the crop statistics (device + pinned host), so a call
    allocates nothing and makes ONE stream synchronisation; the pinned mask blocks run_unet returns its
    masks in (_MaskPool); and the photo graphs captured over them -- one per photo geometry of one model,
    LRU-bounded, its masks copy retargeted per call to the block lent (unet_photo_graph_set_masks) --,
    which stay valid while these buffers do."""

    MASK_POOL = 4     # pinned mask blocks lent as run_unet's masks (no host copy), see _MaskPool
    MAX_GRAPHS = 8    # photo geometries with a captured graph (LRU)

    def __init__(self, device):
        self.device = torch.device(device)
        self.lock = threading.Lock()
        self.h_img = self.d_img = None
        self.x = torch.empty((1, 3, IMG_SIZE, IMG_SIZE), dtype=torch.float32, device=self.device)
        # the outputs, u8 masks | boxes | crop rectangles | crop pixel sums, carved from one device and
        # one pinned host block in the same order: the photo graph copies boxes | rects | sums back as one
        self.m, self.b, self.r, self.s = self._outputs(torch.empty(self._out_bytes(), dtype=torch.uint8,
                                                                   device=self.device))
        self.hm, self.hb, self.hr, self.hs = self._outputs(torch.empty(self._out_bytes(), dtype=torch.uint8, pin_memory=True))
        self.graphs: OrderedDict = OrderedDict()   # key -> (model, native.Graph); key = (ih, iw, c)
        self.masks = _MaskPool(self.m.shape[1:], self.MASK_POOL)
        self.retarget_error = None   # the runtime's last refusal to retarget a masks copy (then: re-capture)

    @staticmethod
    def _out_bytes():
        n = len(FIELDS)
        return n * IMG_SIZE * IMG_SIZE + n * 16 + n * 16 + n * 8

    @staticmethod
    def _outputs(block: torch.Tensor):
        n = len(FIELDS)
        o1 = n * IMG_SIZE * IMG_SIZE   # a multiple of 8: the int64 sums stay aligned
        o2, o3 = o1 + n * 16, o1 + n * 32
        m = block[:o1].view(1, n, IMG_SIZE, IMG_SIZE)
        b = block[o1:o2].view(torch.int32).view(1, n, 4)
        r = block[o2:o3].view(torch.int32).view(n, 4)
        s = block[o3:o3 + n * 8].view(torch.int64)
        return m, b, r, s

    def stage(self, arr: np.ndarray) -> torch.Tensor:
        """uint8 [H, W(, C)] host photo -> the pinned host buffer (grown when needed: the photo graphs
        captured over the old buffers are dropped then).  Returns the device view it is uploaded to."""
        n = arr.size
        if self.h_img is None or self.h_img.numel() < n:
            self.drop_graphs()
            self.h_img = torch.empty(max(n, 1 << 20), dtype=torch.uint8, pin_memory=True)
            self.d_img = torch.empty(self.h_img.numel(), dtype=torch.uint8, device=self.device)
        self.h_img[:n].numpy()[:] = arr.reshape(-1)
        return self.d_img[:n].view(arr.shape)

    def stage_photo(self, pil_img: Image.Image):
        """The photo into the pinned host buffer: "RGB" as Pillow's RGBX pixels (copy_rgbx), else (and when
        that export is unavailable) packed by photo_array.  Returns (device view it is uploaded to, channel
        count of the crop statistics: 3 or 1)."""
        w, h = pil_img.size
        if pil_img.mode == "RGB":
            if self.h_img is None or self.h_img.numel() < w * h * 4:
                self.drop_graphs()
                self.h_img = torch.empty(max(w * h * 4, 1 << 20), dtype=torch.uint8, pin_memory=True)
                self.d_img = torch.empty(self.h_img.numel(), dtype=torch.uint8, device=self.device)
            shape = copy_rgbx(pil_img, self.h_img.data_ptr(), self.h_img.numel())
            if shape is not None:
                return self.d_img[:w * h * 4].view(shape), 3
        arr = photo_array(pil_img)
        return self.stage(arr), (3 if arr.ndim == 3 else 1)

    def upload(self, arr: np.ndarray) -> torch.Tensor:
        """uint8 [H, W(, C)] host photo -> device tensor of the same shape (pinned, async)."""
        dst = self.stage(arr)
        dst.view(-1).copy_(self.h_img[:arr.size], non_blocking=True)
        return dst

    def drop_graphs(self):
        for _, g in self.graphs.values():
            g.close()
        self.graphs.clear()

    def drop_graph(self, key):
        e = self.graphs.pop(key, None)
        if e is not None:
            e[1].close()

    def graph_key(self, img: torch.Tensor, target: torch.Tensor = None):
        return tuple(img.shape)

    def photo_graph(self, model, img: torch.Tensor, target: torch.Tensor):
        """The photo graph of (model, photo geometry): upload + resize + forward (masks, boxes) + crop
        statistics + copies back (unet_photo_graph_create), captured at the first call of the geometry, its
        masks copy pointed at ``target`` (a lent mask block, or the shared pinned buffer).  A cached graph is
        retargeted (unet_photo_graph_set_masks); should the runtime refuse that, the geometry's graph is
        captured again over the new target (the refusal is kept in ``retarget_error``)."""
        key = self.graph_key(img)
        e = self.graphs.get(key)
        if e is not None and e[0] is model:
            g = e[1]
            if g.masks_ptr != target.data_ptr():
                try:
                    g.set_masks(target.view(self.hm.shape))
                except RuntimeError as exc:
                    self.retarget_error = str(exc)
                    self.drop_graph(key)
                    e = None
            if e is not None:
                self.graphs.move_to_end(key)
                return g
        if any(m is not model for m, _ in self.graphs.values()):
            # another model (a re-loaded checkpoint or another precision plan): the model cache holds one
            # model, so drop its graphs -- they keep its handle (workspace, weights) alive
            self.drop_graphs()
        h = model.native_handle(self.device)
        h.reserve(1, IMG_SIZE, IMG_SIZE)
        img3 = img if img.dim() == 3 else img.unsqueeze(-1)
        g = h.photo_graph(self.h_img, img3, self.x, self.m, native.MASK_U8, self.b, CROP_PAD, self.r, self.s,
                          target.view(self.hm.shape), self.hb, self.hr, self.hs)
        self.graphs[key] = (model, g)
        while len(self.graphs) > self.MAX_GRAPHS:
            self.graphs.popitem(last=False)[1][1].close()
        return g


_staging: dict = {}


def run_unet(pil_img: Image.Image, checkpoint_path: str, compute_dtype: str | None = None):
    """inference.py:50-129 -> (masks: {field: bool[512,512]}, crops: {field: PIL.Image | None})."""
    model = _cached_model(checkpoint_path, compute_dtype)
    if not str(DEVICE).startswith("cuda"):
        raise RuntimeError("unet_mi355x: run_unet runs on a ROCm GPU; there is no CPU fallback")
    with _cache_lock:
        st = _staging.get(str(DEVICE))
        if st is None:
            st = _staging[str(DEVICE)] = _Staging(DEVICE)
    with st.lock:
        stream = torch.cuda.current_stream(st.device)
        if pil_img.mode in ("RGB", "L"):
            # inference.py:63-64 (Pillow-exact BICUBIC resize + convert("RGB") + /255), the forward with the
            # fused sigmoid + threshold + per-field boxes, and the crop statistics, all on the device as
            # one graph per photo geometry: one launch, one synchronisation
            img, ch = st.stage_photo(pil_img)
            lent = st.masks.take()   # (pinned block, bool array over it) or None: all blocks are held
            target = lent[0] if lent is not None else st.hm[0]
            g = st.photo_graph(model, img, target)
            try:
                g.launch(stream.cuda_stream)
            except RuntimeError:   # stale (the cached model's workspace grew, e.g. run_unet_batch): capture again
                st.drop_graph(st.graph_key(img))
                st.photo_graph(model, img, target).launch(stream.cuda_stream)
            stream.synchronize()
            # the kernel writes 0 / 1 bytes: bool views of the lent block, or a copy out of the shared buffer
            m = lent[1] if lent is not None else st.hm.numpy()[0].view(np.bool_).copy()
            del lent
            rects, sums = st.hr.numpy().copy(), st.hs.numpy().copy()
            masks = {k: m[i] for i, k in enumerate(FIELDS)}
            return masks, {k: crop_from_stats(pil_img, rects[i], sums[i], ch) for i, k in enumerate(FIELDS)}
        # other PIL modes (RGBA premultiplied resize, P nearest, ...): the reference's host path
        x = preprocess(pil_img.resize((IMG_SIZE, IMG_SIZE)))      # inference.py:63-64
        with torch.no_grad():
            model.forward_boxes(x, masks="u8", out=(st.m, st.b))
        st.hm.copy_(st.m, non_blocking=True)
        st.hb.copy_(st.b, non_blocking=True)
        stream.synchronize()
        m = st.hm.numpy()[0].view(np.bool_).copy()
        boxes = st.hb.numpy()[0].copy()
    masks = {k: m[i] for i, k in enumerate(FIELDS)}
    return masks, boxes_to_crops(pil_img, boxes)


def run_unet_batch(pil_imgs, checkpoint_path: str, compute_dtype: str | None = None, exact: bool = True):
    """Batched run_unet for serving: N photos -> [(masks, crops)] in order, with run_unet's
    preprocessing, forward, masks, boxes and crop rules.  RGB / L photos are resized on the GPU
    straight into their slot of the batch input; other PIL modes take the reference's host resize.

    exact=True (default): the forward runs in chunks of at most the library's small-batch limit
    (unet_small_batch_limit, 4), the batches whose outputs are bitwise the same as at N = 1, so every
    photo's masks and crops are exactly run_unet's.  exact=False: one forward over the whole batch
    (the large-batch kernels: higher throughput; above the limit the logits agree with run_unet's
    within the fp32-accumulation tolerance only, so a mask pixel within rounding of its threshold
    may differ); it runs as chunks of 8 or more photos (each above the limit, so the outputs are those
    of one forward over all of them).

    The chunks form a pipeline on the caller's stream: while the GPU runs chunk k (upload, resize,
    forward, crop statistics, copies back), the host packs chunk k + 1's photos and then builds chunk
    k - 1's crops."""
    model = _cached_model(checkpoint_path, compute_dtype)
    pil_imgs = list(pil_imgs)
    if not pil_imgs:
        return []
    n = len(pil_imgs)
    on_dev = str(DEVICE).startswith("cuda")
    if not on_dev:
        raise RuntimeError("unet_mi355x: run_unet_batch runs on a ROCm GPU; there is no CPU fallback")
    nf = len(FIELDS)
    x = torch.empty((n, 3, IMG_SIZE, IMG_SIZE), dtype=torch.float32, device=DEVICE)
    m = torch.empty((n, nf, IMG_SIZE, IMG_SIZE), dtype=torch.uint8, device=x.device)
    boxes = torch.empty((n, nf, 4), dtype=torch.int32, device=x.device)
    rects = torch.empty((n, nf, 4), dtype=torch.int32, device=x.device)
    sums = torch.empty((n, nf), dtype=torch.int64, device=x.device)
    # the masks come back into one pinned block from torch's host allocator; the returned masks are views
    # of it (it goes back to the allocator's cache once none is referenced): no pageable staging copy
    # (pageable past 256 MB of masks -- 341 photos --: pinned memory is a scarcer resource; the copies
    # are then synchronous)
    hm = torch.empty(m.shape, dtype=torch.uint8, pin_memory=m.numel() <= 256 << 20)
    hsmall = torch.empty((n, 2 * nf * 4 + 2 * nf), dtype=torch.int32, pin_memory=True)   # boxes | rects | sums
    limit = model.native_handle(x.device).small_batch_limit()
    if exact:   # chunks of at most the limit: bitwise the batch-1 outputs
        bounds = list(range(0, n, limit if limit > 0 else n)) + [n]
    else:       # chunks of 8 or more photos, all above the limit: the same outputs as one large forward
        k = max(1, n // 8) if n >= 16 else 1
        bounds = [i * n // k for i in range(k + 1)]
    stream = torch.cuda.current_stream(x.device)
    out = [None] * n
    keep = []   # the chunks' pinned photo blocks, alive until their uploads are done

    def launch(lo, hi):
        """Upload + resize + forward + crop statistics + copies back of photos lo .. hi-1 (asynchronous)."""
        arrs = [photo_array(p) if p.mode in ("RGB", "L") else None for p in pil_imgs[lo:hi]]
        offs, total = [], 0
        for a_ in arrs:
            offs.append(total)
            total += 0 if a_ is None else -(-a_.size // 256) * 256
        imgs = [None] * (hi - lo)
        if total:   # the RGB / L photos packed into one pinned block, one copy
            hbuf = torch.empty(total, dtype=torch.uint8, pin_memory=True)   # (allocated pinned: no copy)
            hnp = hbuf.numpy()
            for a_, o in zip(arrs, offs):
                if a_ is not None:
                    hnp[o:o + a_.size] = a_.reshape(-1)
            dbuf = torch.empty(total, dtype=torch.uint8, device=x.device)
            dbuf.copy_(hbuf, non_blocking=True)
            keep.append(hbuf)
            for j, (a_, o) in enumerate(zip(arrs, offs)):
                if a_ is not None:
                    imgs[j] = dbuf[o:o + a_.size].view(a_.shape)
        for j in range(hi - lo):
            if imgs[j] is not None:
                model.preprocess(imgs[j], IMG_SIZE, out=x[lo + j])
            else:   # other PIL modes (RGBA premultiplied resize, P nearest, ...): the reference's host resize
                x[lo + j] = preprocess(pil_imgs[lo + j].resize((IMG_SIZE, IMG_SIZE)))[0]
        with torch.no_grad():
            model.forward_boxes(x[lo:hi], masks="u8", out=(m[lo:hi], boxes[lo:hi]))
        for j, img in enumerate(imgs):
            if img is not None:
                img3 = img if img.dim() == 3 else img.unsqueeze(-1)
                native.crop_stats(img3, boxes[lo + j], IMG_SIZE, IMG_SIZE, CROP_PAD, rects[lo + j], sums[lo + j],
                                  stream.cuda_stream)
        hm[lo:hi].copy_(m[lo:hi], non_blocking=True)
        small = torch.cat([boxes[lo:hi].view(hi - lo, -1), rects[lo:hi].view(hi - lo, -1),
                           sums[lo:hi].view(torch.int32).view(hi - lo, -1)], 1)
        hsmall[lo:hi].copy_(small, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev, [img is not None for img in imgs], [None if img is None else img.dim() for img in imgs]

    def finish(lo, hi, ev, dev_photo, dims):
        """Masks (views of the pinned block) and crops of photos lo .. hi-1, once their copies landed."""
        ev.synchronize()
        mb = hm.numpy().view(np.bool_)   # the kernel writes 0 / 1 bytes
        sm = hsmall.numpy()
        k4 = nf * 4
        for j in range(hi - lo):
            i = lo + j
            masks = {k: mb[i, f] for f, k in enumerate(FIELDS)}
            bx = sm[i, :k4].reshape(nf, 4)
            if dev_photo[j]:   # the reference's crop rules on device statistics: no crop pixel read here
                rc = sm[i, k4:2 * k4].reshape(nf, 4)
                sv = np.ascontiguousarray(sm[i, 2 * k4:]).view(np.int64)
                ch = 3 if dims[j] == 3 else 1
                crops = {k: crop_from_stats(pil_imgs[i], rc[f], sv[f], ch) for f, k in enumerate(FIELDS)}
            else:
                crops = boxes_to_crops(pil_imgs[i], bx)
            out[i] = (masks, crops)

    pending = None
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        cur = (lo, hi) + launch(lo, hi)
        if pending is not None:
            finish(*pending)
        pending = cur
    finish(*pending)
    del keep
    return out
