/* unet_mi355x.h -- C-ABI of the MI355X-native UNet forward path.
 *
 * Drop-in for the reference segmentation call surface (tingyu-c/TW-invoice-unet-ocr-llm):
 *   unet_model.UNet(n_channels, n_classes)      unet_model.py:23-53   -> unet_create
 *   model.load_state_dict(torch.load(ckpt))     inference.py:17-24     -> unet_load_weights
 *   model(x)  (UNet.forward)                    unet_model.py:55-86    -> unet_forward (logits)
 *   sigmoid + per-field thresholds              inference.py:72-79     -> unet_forward (masks)
 *
 * The reference has no FFI (it is pure Python on torch); this header is the boundary a
 * ctypes/cffi binding loads.  Plain C types only; no torch or C++ types cross it.
 *
 * Conventions
 *   - return value: 0 = OK, negative = error (UNET_E*); unet_last_error() gives the
 *     message for the calling thread.  C++ exceptions never cross the ABI.
 *   - device pointers are caller-owned (e.g. torch data_ptr()); work is enqueued on the
 *     caller's HIP stream (hipStream_t passed as void*), with no hidden synchronisation
 *     except inside unet_load_weights / unet_reserve (allocation + upload) and the first
 *     unet_preprocess of a new photo geometry (coefficient upload).  unet_forward never
 *     allocates: size the workspace with unet_reserve first.
 *   - a handle owns one workspace.  Calls on it must not overlap on the host (serialise them;
 *     the Python wrapper holds a lock).  On the device, a call issued on a different stream than
 *     the previous one waits for that previous call (hipStreamWaitEvent), so the workspace is
 *     never shared by two forwards in flight.
 */
#ifndef UNET_MI355X_H
#define UNET_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UNET_ABI_VERSION 5   /* 2: unet_forward requires unet_reserve; Cfg renumbered; fp16 range check. 3: unet_crop_stats.
                                 4: unet_launch_label_at, unet_small_batch_limit, unet_photo_graph_create, unet_block_*
                                 5: unet_photo_graph_set_masks (the masks copy is its own node); UNET_DTYPE_F32 as
                                    three bf16 terms, UNET_DTYPE_F32_EXACT the exact-fp32 MFMA */

/* error codes */
#define UNET_OK 0
#define UNET_EINVAL (-1)     /* bad argument (maps to ValueError)                    */
#define UNET_ESHAPE (-2)     /* unsupported shape, e.g. H or W not divisible by 16     */
#define UNET_ENOMEM (-3)     /* device allocation failed                               */
#define UNET_EHIP (-4)       /* HIP runtime error                                      */
#define UNET_ESTATE (-5)     /* call out of order (e.g. forward before weights)       */
#define UNET_EKEY (-6)       /* state_dict key missing / unexpected / wrong shape      */

/* compute / storage dtype of the activations and packed weights (accumulation is fp32).
 * UNET_DTYPE_F32: fp32 storage and weights; every product of the 3x3 and ConvTranspose layers computed as
 * three bf16 terms per operand (x = hi + mid + lo, 6 bf16 MFMA products per K block, fp32 accumulation):
 * fp32 accuracy (the reference's fp32 forward within 2e-5 of the logit scale, tests/test_forward_gpu.py)
 * on the 2.5 PFLOP/s bf16 pipe.  UNET_DTYPE_F32_EXACT: the same plan on the exact-fp32 MFMA
 * (v_mfma_f32_16x16x4_f32, 157 TFLOP/s). */
#define UNET_DTYPE_F32 0
#define UNET_DTYPE_BF16 1
#define UNET_DTYPE_F16 2
/* bf16 at resolution levels 2-4, fp16 at the two full-resolution levels 0-1 (where the mask
 * boundaries are decided): the precision plan of the headline benchmark, see DESIGN.md §2.
 * fp16 storage (UNET_DTYPE_F16, and levels 0-1 of MIXED) holds |v| <= 65504: unet_load_weights
 * refuses (UNET_EINVAL) a checkpoint whose BN-folded weights or biases exceed that at an fp16
 * level; activations beyond it would become inf -- use BF16 (fp32's range) or F32 for such nets. */
#define UNET_DTYPE_MIXED 3
#define UNET_DTYPE_F32_EXACT 4

/* input layouts / dtypes accepted by unet_forward */
#define UNET_LAYOUT_NCHW 0   /* [N][n_channels][H][W] (the reference's torch layout)             */
#define UNET_LAYOUT_NHWC 1   /* [N][H][W][n_channels] (decoded photos)                           */
#define UNET_IN_F32 0        /* float32 values                                                   */
#define UNET_IN_U8 1         /* uint8 values v, read as v / 255.0f (inference.py:40's scaling)   */

/* mask outputs of unet_forward */
#define UNET_MASK_NONE 0
#define UNET_MASK_U8 1    /* uint8 [N][n_classes][H][W], 1 where sigmoid(logit) > thr      */
#define UNET_MASK_BITS 2  /* uint8 [N][n_classes][H][W/8], bit b of byte x/8 = pixel x      */

typedef struct unet_handle unet_handle;

typedef struct unet_config {
  int n_channels;     /* input channels: 1 or 3 (UNet(n_channels=...), unet_model.py:24) */
  int n_classes;      /* 1..4 (UNet(n_classes=...); the app uses 3)                       */
  int dtype;          /* UNET_DTYPE_*                                                     */
  int device;         /* HIP device ordinal                                               */
  float thresholds[4];/* per-class probability thresholds (inference.py:76-78)           */
} unet_config;

typedef struct unet_tensor_view {
  const char* name;   /* state_dict key, e.g. "down1.net.0.weight"                       */
  const void* data;   /* host pointer, contiguous                                         */
  int dtype;          /* 0 = float32, 1 = int64 (num_batches_tracked; ignored)            */
  int ndim;
  int64_t shape[4];
} unet_tensor_view;

/* Create a handle for UNet(n_channels, n_classes) on cfg->device.
 * Replaces: unet_model.UNet.__init__ (unet_model.py:24-53). */
int unet_create(const unet_config* cfg, unet_handle** out);

/* Strictly load the 136-key reference state_dict (host fp32), fold eval BatchNorm
 * (eps 1e-5) into the convs, pre-pack NHWC/MFMA panels and upload them.
 * Replaces: load_state_dict(strict=True) + eval() (inference.py:20-23). */
int unet_load_weights(unet_handle* h, const unet_tensor_view* tensors, int n);

/* Bytes of device workspace unet_forward needs for (N, H, W). */
size_t unet_workspace_bytes(const unet_handle* h, int N, int H, int W);

/* Allocate (grow) the workspace for up to (N, H, W): unet_forward requires it (UNET_ESTATE
 * otherwise; ABI 1 allocated inside the forward) and then neither allocates nor synchronises
 * (graph-capturable).  Growing waits for the handle's queued work.
 * A forward issued on a stream under capture (unet_graph_create, or the caller's own capture, e.g.
 * torch.cuda.graph on its side stream) neither waits for nor records the handle's stream-order
 * event; ordering the replay after other work on the handle is then the caller's. */
int unet_reserve(unet_handle* h, int N, int H, int W);

/* Forward pass.  x: device tensor [N][n_channels][H][W] (x_layout UNET_LAYOUT_NCHW) or
 * [N][H][W][n_channels] (UNET_LAYOUT_NHWC) of fp32 (x_dtype UNET_IN_F32) or uint8 (UNET_IN_U8,
 * value / 255).
 * logits: device fp32 NCHW [N][n_classes][H][W] or NULL.
 * masks:  device uint8 per mask_kind or NULL (mask_kind UNET_MASK_NONE).
 * H, W must be divisible by 16 (the reference raises inside torch.cat otherwise).
 * Replaces: UNet.forward (unet_model.py:55-86) and inference.py:72-79. */
int unet_forward(unet_handle* h, const void* x, int x_layout, int x_dtype,
                 void* logits, void* masks, int mask_kind,
                 int N, int H, int W, void* hip_stream);

/* unet_forward, plus the bounding box of every (image, field) mask -- the np.where ->
 * min/max step of run_unet (inference.py:84-90) on the device, so a caller that only needs
 * the crop rectangles copies 16 bytes per field instead of the mask (and a multi-GPU caller
 * all-gathers 48 bytes per image).
 * boxes: device int32 [N][n_classes][4] = x_min, y_min, x_max, y_max in mask pixels
 *        (inclusive), all four -1 for an empty mask.
 * masks / mask_kind as for unet_forward; when masks is NULL (or mask_kind is
 * UNET_MASK_NONE) the masks go to the workspace and only the boxes are returned.
 * Replaces: UNet.forward + inference.py:72-90. */
int unet_forward_boxes(unet_handle* h, const void* x, int x_layout, int x_dtype,
                       void* logits, void* masks, int mask_kind, int32_t* boxes,
                       int N, int H, int W, void* hip_stream);

/* GPU preprocessing of one photo (inference.py:62-64 + preprocess, :30-44):
 * PIL Image.resize((ow, oh)) with Pillow's default BICUBIC filter -- bit-exact with Pillow's
 * fixed-point separable resampler --, convert("RGB") (gray replicated), /255 as float32, CHW.
 * img: device uint8 HWC [ih][iw][channels], channels 3 (mode "RGB"), 1 (mode "L") or 4 (RGBX: Pillow's own
 *      in-memory layout of an "RGB" image, 4 bytes per pixel, the 4th ignored -- uploaded without repacking);
 * x:   device fp32 [3][oh][ow] (e.g. one image's slot of the unet_forward input batch).
 * Coefficient tables are cached per (ih, iw, oh, ow) in the handle (first call per geometry
 * uploads them synchronously).  Stream-ordered on hip_stream. */
int unet_preprocess(unet_handle* h, const void* img, int ih, int iw, int channels,
                    float* x, int oh, int ow, void* hip_stream);

/* The crop step of run_unet (inference.py:92-127) on the device photo, so the host never reads
 * crop pixels: for every mask box (unet_forward_boxes' output, in a box_h x box_w mask), the crop
 * rectangle in photo pixels -- the reference's float64 arithmetic: scale = iw / box_w, x1 =
 * int(x_min * scale), x2 = int(x_max * scale), pad_x = int((x2 - x1) * pad) (pad = 0.15), clamp
 * to [0, iw] (y likewise) -- and the sum of the crop's uint8 values over every channel.  The
 * reference's rejections are then host tests: x2 <= x1 or y2 <= y1 (empty crop), and
 * np.array(crop).mean() < 3  <=>  sum < 3 * (x2 - x1) * (y2 - y1) * channels (numpy's float64 sum
 * of the integers is exact).  img: device uint8 HWC [ih][iw][channels] (unet_preprocess's input);
 * boxes: device int32 [n_boxes][4]; rects: device int32 [n_boxes][4] (x1, y1, x2, y2; -1s for an
 * empty box); sums: device uint64 [n_boxes] (channels 4 = RGBX: the sum over R, G, B).  Needs no handle;
 * stream-ordered on hip_stream. */
int unet_crop_stats(const void* img, int ih, int iw, int channels, const int32_t* boxes, int n_boxes,
                    int box_h, int box_w, double pad, int32_t* rects, uint64_t* sums, void* hip_stream);

/* Number of launch slots in one forward (first conv, 17 implicit-GEMM 3x3 convs with
 * the fused pool / head epilogues, 4 ConvTranspose2d), in execution order:
 * down1.0 down1.3 down2.0 down2.3 down3.0 down3.3 down4.0 down4.3 bottleneck.0
 * bottleneck.3 up4 conv4.0 conv4.3 up3 conv3.0 conv3.3 up2 conv2.0 conv2.3 up1 conv1.0
 * conv1.3+out_conv.  On the 16-bit plans up1 runs inside the conv2.3 launch (its slot issues no
 * kernel: empty label, ~0 ms); the environment variable UNET_MI355X_FUSE_UP1=0, read by
 * unet_create, keeps it a launch of its own. */
#define UNET_NUM_LAUNCHES 22
int unet_num_launches(void);

/* Kernel instantiation run by launch i of a forward (e.g.
 * "conv3x3_ring_kernel<__bf16, 1, 4, 8, 3, 0, 1, 0, __bf16, __bf16, 16, 16>"), spelled like the demangled
 * symbol that rocprofv3 reports; "" for a bad index or a slot fused into the previous launch. */
const char* unet_launch_label(const unet_handle* h, int i);

/* The same for a forward of N x H x W: batches N <= unet_small_batch_limit(h) run the small-batch
 * plan, whose split layers launch two kernels -- "partial kernel + splitk_reduce_kernel<...>" -- and
 * whose under-filled layers may run finer row tiles; N = 0 (or N above the limit) gives the
 * large-batch labels of unet_launch_label.  The string lives until the calling thread's next call. */
const char* unet_launch_label_at(const unet_handle* h, int i, int N, int H, int W);

/* Largest batch of the small-batch (split-K) plan, 0 when it is off (UNET_MI355X_KSPLIT=0 at
 * unet_create).  An image's outputs are bitwise the same for every N <= the limit, and for every N
 * above it; the two regimes agree within the fp32-accumulation tolerance, not bit for bit, so a
 * caller that must reproduce batch-1 results exactly runs its batches in chunks of at most the limit
 * (inference.run_unet_batch does). */
int unet_small_batch_limit(const unet_handle* h);

/* unet_forward, plus HIP-event timing of every launch on the given stream (ms, in the
 * order above, launch_ms[UNET_NUM_LAUNCHES]).  Synchronises on the stream; for
 * measurement only. */
int unet_forward_timed(unet_handle* h, const void* x, int x_layout, int x_dtype,
                       void* logits, void* masks, int mask_kind,
                       int N, int H, int W, void* hip_stream, float* launch_ms);

/* Copy an intermediate activation of the last forward (debug / per-layer parity):
 * name in {"c1","p1","c2","p2","c3","p3","c4","p4","bn","c7","u1","u2","u3","u4","c8a"}
 * (c_k: encoder skips, p_k: pooled maps, u_k: ConvTranspose outputs, c7: conv2 output,
 * c8a: conv1.net.0 output).  "c7" is UNET_ESTATE after a forward with up1 fused into conv2.3
 * (conv2's output then never leaves the registers; UNET_MI355X_FUSE_UP1=0 keeps it).
 * dst: device buffer receiving fp32 NCHW [N][C][h][w]; *numel receives the element count
 * when dst is NULL. */
int unet_debug_fetch(unet_handle* h, const char* name, float* dst, size_t* numel, void* hip_stream);

/* hipGraph of one forward (unet_forward, or unet_forward_boxes when boxes != NULL) over fixed
 * device buffers and a fixed (N, H, W): the 22-launch sequence is captured once and replayed by
 * unet_graph_launch with one host call -- the launch-bound small-batch case (run_unet's batch
 * of 1, inference.py:42).  A graph is stale (UNET_ESTATE at launch) once unet_load_weights or a
 * growing unet_reserve re-allocates the handle's device memory; capture again then.  Destroy
 * graphs before their handle. */
typedef struct unet_graph unet_graph;
int unet_graph_create(unet_handle* h, const void* x, int x_layout, int x_dtype,
                      void* logits, void* masks, int mask_kind, int32_t* boxes,
                      int N, int H, int W, unet_graph** out);
int unet_graph_launch(unet_graph* g, void* hip_stream);
int unet_graph_destroy(unet_graph* g);

/* One graph per photo geometry: the whole device part of run_unet (inference.py:58-129) -- the
 * upload of the pinned host photo (h_img; NULL: the caller fills img), unet_preprocess to size x size
 * into x (on the 16-bit plans, when the photo's height differs from size, the resize writes the first
 * conv's pre-cast input into the workspace instead and x is not written; the graph owns its resize
 * tables and row buffer, so the handle's geometry cache may evict its own copy), unet_forward_boxes at N = 1 (masks / mask_kind / boxes as there), unet_crop_stats (pad,
 * rects, sums as there) and the copies of masks, boxes, rects and sums into the pinned host buffers
 * given (each may be NULL; the masks copy is a node of its own; of the others, copies whose device and
 * host buffers both follow the previous one's in memory, e.g. boxes | rects | sums carved from one
 * device and one host block, are made as one) -- captured once and replayed by unet_graph_launch: one
 * host call and one stream synchronisation per photo.  Needs unet_reserve(h, 1, size, size) first;
 * stale (UNET_ESTATE at launch) under the same rules as unet_graph_create's graphs.  Destroy with
 * unet_graph_destroy. */
int unet_photo_graph_create(unet_handle* h, const void* h_img, void* img, int ih, int iw, int channels, float* x,
                            int size, void* masks, int mask_kind, int32_t* boxes, double pad, int32_t* rects,
                            uint64_t* sums, void* h_masks, void* h_boxes, void* h_rects, void* h_sums,
                            unet_graph** out);
/* Retarget a photo graph's masks copy (created with h_masks != NULL) to another pinned host buffer of the
 * same size, for its next replays (hipGraphExecMemcpyNodeSetParams1D): one graph per photo geometry serves
 * any number of caller-held mask buffers.  Host-side only; replays already enqueued keep their target.
 * Call it under the same serialisation as unet_graph_launch. */
int unet_photo_graph_set_masks(unet_graph* g, void* h_masks);

/* Multi-GPU data parallelism: one process per GPU, each rank runs
 * unet_forward / unet_forward_boxes on its contiguous shard of the batch, and the one exchange
 * step is an all-gather of the per-rank bit-packed masks (or boxes) over RCCL/xGMI.  These
 * entry points give a C host that collective without torch.distributed; RCCL is loaded at run
 * time (dlopen), so a host that never calls them never loads it.
 *   rank 0: unet_comm_get_unique_id(id) -> send the UNET_COMM_ID_BYTES bytes to every rank
 *   every rank: unet_comm_init(h, rank, nranks, id); ... unet_allgather(h, my_masks,
 *     all_masks, bytes_per_rank, stream) (recv = nranks x bytes_per_rank, rank order);
 *     unet_comm_destroy(h) (also done by unet_destroy).
 * unet_allgather is stream-ordered like unet_forward (it follows the handle's previous call). */
#define UNET_COMM_ID_BYTES 128
int unet_comm_get_unique_id(void* id);
int unet_comm_init(unet_handle* h, int rank, int nranks, const void* id);
int unet_allgather(unet_handle* h, const void* send, void* recv, size_t bytes_per_rank, void* hip_stream);
int unet_comm_destroy(unet_handle* h);

int unet_destroy(unet_handle* h);

/* Stand-alone DoubleConv block: unet_model.DoubleConv(in_ch, out_ch).forward (unet_model.py:6-20,
 * conv3x3 + BN + ReLU twice, padding 1) on its own, on the network's kernels: the first-conv kernel
 * for in_ch 1 or 3 (out_ch 64), the 8-wave MFMA rings (16-bit plans; MIXED = fp16 up to 128 output
 * channels, bf16 beyond, as the network's levels) or the fp32 LDS-halo kernels.  Supported: in_ch in
 * {1, 3} with out_ch 64, or in_ch a multiple of 32 with out_ch a multiple of 64 (on the 16-bit plans:
 * out_ch 64 or a multiple of 128, the ring tiles) -- every block of the reference UNet (UNET_ESHAPE
 * otherwise, at unet_block_create).  Any H, W >= 1.
 * unet_block_load_weights takes the block's own 14 state_dict keys (net.0.weight, net.0.bias,
 * net.1.weight / bias / running_mean / running_var / num_batches_tracked, and net.3 / net.4 alike;
 * BN folded, eps 1e-5).  x / y: device fp32 NCHW [N][in_ch][H][W] / [N][out_ch][H][W]; the workspace
 * is sized by unet_block_reserve (unet_block_forward never allocates). */
typedef struct unet_block unet_block;
typedef struct unet_block_config {
  int in_ch, out_ch;   /* DoubleConv(in_ch, out_ch) */
  int dtype;           /* UNET_DTYPE_* */
  int device;          /* HIP device ordinal */
} unet_block_config;
int unet_block_create(const unet_block_config* cfg, unet_block** out);
int unet_block_load_weights(unet_block* b, const unet_tensor_view* tensors, int n);
int unet_block_reserve(unet_block* b, int N, int H, int W);
int unet_block_forward(unet_block* b, const float* x, float* y, int N, int H, int W, void* hip_stream);
int unet_block_destroy(unet_block* b);

/* Message of the last error on this thread ("" if none). */
const char* unet_last_error(void);

int unet_abi_version(void);

/* Logit cut of a probability threshold: for every fp32 logit x,
 *   (1 / (1 + expf(-x)) > thr)  ==  (x > unet_logit_cut(thr)).
 * The masks epilogue thresholds logits with it (inference.py:72-78 thresholds
 * torch.sigmoid(logits)); host-only, no device call. */
float unet_logit_cut(float thr);

#ifdef __cplusplus
}
#endif
#endif /* UNET_MI355X_H */
