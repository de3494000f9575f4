// Internal (non-ABI) declarations shared by the HIP kernels and the C-ABI host layer.
// Nothing here crosses the library boundary; see include/unet_mi355x.h for that.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

namespace unet {

enum class DType : int { F32 = 0, BF16 = 1, F16 = 2 };

inline size_t dtype_size(DType t) { return t == DType::F32 ? 4 : 2; }

// Epilogue kinds of the implicit-GEMM kernel.
enum Epi : int {
  EPI_STORE = 0,    // bias + ReLU -> NHWC store (conv3x3 + folded BN + ReLU)
  EPI_POOL = 1,     // EPI_STORE + fused 2x2/2 max-pool into a second NHWC tensor
  EPI_HEAD = 2,     // bias + ReLU kept in fp32 -> fused 1x1 out_conv -> logits / masks
  EPI_UPSCATTER = 3,// ConvTranspose2d(k2,s2): bias, no ReLU, pixel-shuffle store
  EPI_UPFUSE = 4,   // conv2.3 + up1 in one launch: bias + ReLU kept in registers as the B operand of
                    // the ConvTranspose2d GEMM (no store), whose output is scattered like EPI_UPSCATTER
  EPI_PARTIAL = 5   // split-K (small batches): one K slice's fp32 accumulators, no bias, into
                    // part[slice][pixel][Ctot]; launch_splitk_reduce applies the layer's own epilogue
};

// Mask output formats for EPI_HEAD.
enum MaskKind : int { MASK_NONE = 0, MASK_U8 = 1, MASK_BITS = 2 };

constexpr int kMaxClasses = 4;

// One implicit-GEMM launch.  GEMM view: rows = output channels (A = packed
// weights [Ctot][K]), columns = pixels (B = gathered NHWC activations),
// K = TAPS * Cin ordered (tap, cin).
struct IgemmArgs {
  const void* in;      // NHWC activations (element type T), pixel stride ldi
  const void* wgt;     // packed weights [Ctot][TAPS*Cin], rows permuted in 64-row groups
  const float* bias;   // [Ctot] natural row order (BN folded)
  const void* zero;    // 4096 zero bytes (source of the conv zero padding; ring halos add 64 B per chunk)
  void* out;           // NHWC output, pixel stride ldo, channel offset out_off
  void* out2;          // EPI_POOL: pooled NHWC output (pixel stride ldo2)
  const float* head_w; // EPI_HEAD: [ncls][64] fp32
  const float* head_b; // EPI_HEAD: [ncls]
  float* logits;       // EPI_HEAD: NCHW fp32 logits or nullptr
  uint8_t* masks;      // EPI_HEAD: masks or nullptr
  int N, H, W;         // input spatial dims (3x3: == output dims; convT: output is 2H x 2W)
  int Cin, ldi;
  int Ctot;            // GEMM rows (Cout, or 4*Cout for convT)
  int Cout;            // convT: channels per (a,b) group
  int ldo, out_off, ldo2;
  int ncls, mask_kind;
  float thr_logit[kMaxClasses];   // logit cut per class: sigmoid(x) > thr  <=>  x > thr_logit
  int tiles_x, tiles_y, n_ct;
  // fused first conv (halo computed from the raw input instead of loaded): down1.0 + down1.3
  const void* x0;      // network input: NCHW fp32 [N][c0][H][W] (halo kernel), or T [N][H][W][4]
                       // (CFG_RING_FUSED_IN, see launch_x_to_px4)
  const void* w0p;     // first conv packed [2][2][3][16][16] (unet_capi.cpp, CFG_RING_FUSED_IN)
  const float* b0;     // first conv folded bias [64]
  int c0;              // network input channels (1 or 3)
  // EPI_UPFUSE: the ConvTranspose2d's bias [4 * Cout / 2] in natural (a, b, o) row order; its
  // output goes to out2 (pixel stride ldo2, channels [0, Cout / 2)) at 2H x 2W
  const float* bias2;
  // EPI_PARTIAL: K (= Cin chunks) split into ksplit equal slices; slice k of pixel p, row r at
  // part[(k * N*H*W + p) * Ctot + r] (natural row order, fp32)
  float* part;
  int ksplit;
  int src_br;   // EPI_PARTIAL on the 8-wave ring: row tile of the weight packing when finer than BR (0 = BR)
  int x3;       // fp32 LDS-halo family: 0 = exact-fp32 MFMA (v_mfma_f32_16x16x4_f32); fp32 operands as three
                // bf16 terms (6 bf16 MFMAs per 32 K): 1 = both split on the fly (the ConvTranspose), 2 = weights
                // pre-split by the packing, activations on the fly (3x3 layers, CFG_HALO_R64_W4), 3 = weights
                // pre-split, activations split once per chunk into LDS planes (conv3x3_x3s_kernel,
                // CFG_HALO_R128: the 3x3 layers with Cout >= 128), 4 = the same on 64 rows x 16x32 pixels
                // from a register-prefetched halo (conv3x3_x3w_kernel, CFG_HALO_X3W: the 64-channel layers)
};

struct FirstConvArgs {
  const float* x;      // NCHW fp32 input [N][C][H][W]
  const float* w;      // [64][C][3][3] folded (fp32 VALU path)
  const void* wp;      // [4][3][16][16] packed element type: row tile t, MFMA m, packed row, k = 4q + c
                       // (tap 4m + q, channel c; rows permuted like the implicit-GEMM weights)
  const float* b;      // [64] folded
  void* out;           // NHWC [N][H][W][64] element type T
  int N, C, H, W;
};

// First conv on MFMA (K = 9 taps x 4 channels): K slot 4q + c of MFMA m (m = 0..2, lane group q)
// holds (tap first_tap(4m + q), channel c); 15 = a zero slot.  The two 32-lane halves of a
// ds_read_b64 are the lane groups {0, 1} and {2, 3}: each half reads two horizontally adjacent
// taps (their 16-pixel runs overlap in all but one pixel, which the LDS broadcasts) or one tap and
// a zero slot that reads the same address (first_tap_addr), so the window reads are conflict-free.
__host__ __device__ constexpr int first_tap(int s) { return (int)((0xF8F5F2764310ull >> (4 * s)) & 15); }
__host__ __device__ constexpr int first_tap_addr(int s) { return (int)((0x885522764310ull >> (4 * s)) & 15); }

// Kernel configurations.  The LDS-halo family (128-byte K chunks, one tile per block) is the
// fp32 path; the 64-byte-row ring family (persistent walkers, double-buffered halo, weight ring;
// K order chunk32-major / tap-minor) is the 16-bit path; the ConvTranspose ring runs the 2x
// upsamplers.  Selection per layer: unet_capi.cpp (defaults tuned on MI355X, profiles/tune_r1*).
enum Cfg : int {
  CFG_HALO_R64_W4 = 0,    // 64 rows x 16x16 pixels, 4 waves, 3 weight slots
  CFG_HALO_R64_W8 = 1,    // 64 rows, 8 waves
  CFG_HALO_R128 = 2,      // 128-row x 64-pixel wave tiles, 4 waves, 2 weight slots (also the fp32 ConvTranspose)
  CFG_RING_R128 = 3,      // ring: 128-row x 64-pixel wave tiles, 3 weight slots, one tap per step
  CFG_RING_R64_T3 = 4,    // ring: 64-row wave tiles, one kernel row (3 taps) per step
  CFG_RING_FUSED_IN = 5,  // RING_R64_T3 for down1.3 with down1.0 fused (halo chunks computed from the input)
  CFG_TRING_R128 = 6,     // ConvTranspose ring: 128-row x 256-pixel block tiles, 3 slots
  CFG_TRING_R256 = 7,     // ConvTranspose ring: 8 waves, 256-row x 256-pixel block tiles, 4 slots
  // 8-wave ring over 16x32 pixel tiles, one block per CU (half the weight bytes per MFMA)
  CFG_RING8_R128 = 8,     // 128 rows, 3 taps per step (pipelined A-fragment stream), 3 slots
  CFG_RING8_R64_T9 = 9,   // 64 rows, one 32-channel chunk (9 pipelined taps) per step, 2 slots of 36 KB
  CFG_RING8_R64_WS = 10,  // 64 rows, 3 taps per step, weight-stationary (Cin = 64)
  CFG_RING8_FUSED_IN = 11,// RING8_R64_WS for down1.3 with down1.0 fused
  // 4-wave ring over 12x32 pixel tiles, two blocks per CU: 384 pixels per weight step (1.5x the
  // 16x16 tile's MFMAs per weight byte), one tap per step, 4 weight slots (64-row layers).
  // Rejected on A/B (3x the barriers of the T3 ring): built only in `make abl`
  CFG_RING_R64_W12 = 12,
  // the three-term fp32 plan's 64-channel layers: 64 rows x 16x32 pixels, 8 waves, activations split once
  // per chunk from a register-prefetched halo (conv3x3_x3w_kernel; set by the plan only, not an override)
  CFG_HALO_X3W = 13,
  CFG_COUNT = 14
};
int cfg_rows(int cfg);
bool cfg_is_halo(int cfg);
bool cfg_is_ring(int cfg);   // 64-byte-row ring kernel: step-major packed weights
int ring_ns(int cfg);       // ring kernel: weight-ring slots
int ring_tps(int cfg);      // ring kernel: taps per step
int cfg_tile_w(int cfg);    // pixel-tile width (16, or 32 for the 8-wave ring, CFG_RING_R64_W12 and CFG_HALO_X3W)
int cfg_tile_h(int cfg);    // pixel-tile height (16, or 12 for CFG_RING_R64_W12)
bool cfg_is_ring8(int cfg); // the 8-wave ring kernel (conv3x3_ring8_kernel)
bool cfg_fused_in(int cfg); // down1.0 fused into down1.3 (the network input feeds the kernel)
bool cfg_is_tring(int cfg); // ConvTranspose ring kernel: step-major packed weights
int cfg_limit();            // valid Cfg values of this build (ablation builds: + 16 * ablation)

// t: operand (activation + weight) type; to / tq: types of the output / pooled map (t unless
// the layer sits at a seam of the mixed bf16/fp16 plan)
hipError_t launch_igemm(DType t, DType to, DType tq, int cfg, int taps, int epi, const IgemmArgs& a,
                        hipStream_t s);
hipError_t launch_first_conv(DType t, const FirstConvArgs& a, hipStream_t s);
// Split-K reduction of an EPI_PARTIAL launch: out = epilogue(bias + part[0] + part[1] + ...) in
// slice order, with the layer's epilogue epi (EPI_STORE / EPI_POOL / EPI_UPSCATTER) and its output
// arguments (out, ldo, out_off, out2, ldo2, Cout) taken from `a`
hipError_t launch_splitk_reduce(DType to, DType tq, int epi, const IgemmArgs& a, hipStream_t s);
// Network input (fp32 or uint8 = value/255, NCHW or NHWC; include/unet_mi355x.h) -> element type
// t, 4 channels per pixel [N][H][W][4] (input of the fused first conv of CFG_RING_FUSED_IN)
hipError_t launch_x_to_px4(DType t, const void* x, int layout, int xdt, int N, int C, int H, int W, void* out,
                           hipStream_t s);
// the same input -> fp32 NCHW (the fp32 path's first conv reads fp32 NCHW)
hipError_t launch_x_to_nchw_f32(const void* x, int layout, int xdt, int N, int C, int H, int W, float* out,
                                hipStream_t s);
// NHWC (pixel stride ld, channel offset choff, C channels) element type t -> NCHW fp32
// stand-alone DoubleConv (unet_block_*): fp32 NCHW [N][C][H][W] <-> NHWC T [N][H][W][C] (dense)
hipError_t launch_nchw_to_nhwc(DType t, const float* x, int N, int C, int H, int W, void* out, hipStream_t s);
hipError_t launch_nhwc_to_nchw(DType t, const void* src, int N, int C, int H, int W, float* y, hipStream_t s);
hipError_t launch_nhwc_to_nchw_f32(DType t, const void* src, int N, int H, int W, int C, int ld,
                                   int choff, float* dst, hipStream_t s);
// Pillow-exact separable resize (unet_preprocess.hip): device coefficient tables of one
// (ih, iw) -> (oh, ow) geometry.  bounds: [out][2] = (first input index, taps); kk: [out][ksize]
// int32 fixed-point weights (22 fractional bits).  The vertical bounds are relative to h_y0
// when the horizontal pass runs (it produces only rows h_y0 .. h_y0 + h_rows - 1).
struct ResamplePlan {
  int ih, iw, oh, ow;
  bool need_h, need_v;
  int h_y0, h_rows, h_ksize, v_ksize;
  const int* h_bounds; const int* h_kk;
  const int* v_bounds; const int* v_kk;
};
// out: fp32 planes [3][oh][ow]; px4 = F16 / BF16 (with a vertical pass only): the fused first
// conv's pre-cast input [oh][ow][4] of that type instead (launch_x_to_px4's format and values)
hipError_t launch_resample(const ResamplePlan& p, const uint8_t* img, int C, uint8_t* tmp, void* out,
                           hipStream_t s, DType px4 = DType::F32);

// Cross-block reductions (mask boxes, crop sums) meet in "sync entries" of kSyncInts ints: the
// blocks' atomics plus a block counter; the last block writes the result and restores the idle
// state, so an entry is initialised once (init_box_sync / zeroed) and then reused by every launch.
constexpr int kSyncInts = 8;
// Idle state: mask-box entry {INT_MAX, INT_MAX, -1, -1, 0, 0, 0, 0}; crop-sum entry all zero.

// per-(image, field) mask bounding boxes [N*ncls][4] = x_min, y_min, x_max, y_max (-1s if empty);
// sync: N*ncls idle mask-box entries
constexpr int kMaxBoxW = 16384;
hipError_t launch_mask_boxes(const uint8_t* masks, int kind, int N, int ncls, int H, int W, int* boxes, int* sync,
                             hipStream_t s);
// crop rectangles + crop pixel sums of mask boxes on the device photo (unet_preprocess.hip);
// sync: n_boxes zeroed entries, or NULL (sums are then cleared by a memset node and accumulated in place)
hipError_t launch_crop_stats(const uint8_t* img, int ih, int iw, int C, const int* boxes, int n_boxes, int bh, int bw,
                             double pad, int* rects, unsigned long long* sums, int* sync, hipStream_t s);

}  // namespace unet
