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
  EPI_UPSCATTER = 3 // ConvTranspose2d(k2,s2): bias, no ReLU, pixel-shuffle store
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
  const void* zero;    // >= 256 zero bytes (source of the conv zero padding)
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
  int tiles_x, tiles_y, n_ct, n_blocks;
  // fused first conv (halo computed from the raw input instead of loaded): down1.0 + down1.3
  const void* x0;      // network input: NCHW fp32 [N][c0][H][W] (halo kernel), or T [N][H][W][4]
                       // (CFG_RING_FUSED_IN, see launch_x_to_px4)
  const void* w0p;     // first conv packed [64][32] element type (rows permuted)
  const float* b0;     // first conv folded bias [64]
  int c0;              // network input channels (1 or 3)
  unsigned long long* dbg;   // diagnostic (ablation build) per-wave cycle stamps, or nullptr
};

struct FirstConvArgs {
  const float* x;      // NCHW fp32 input [N][C][H][W]
  const float* w;      // [64][C][3][3] folded (fp32 VALU path)
  const void* wp;      // [64][32] packed element type, k = c*9 + ky*3 + kx, zero-padded,
                       // rows permuted like the implicit-GEMM weights (MFMA path)
  const float* b;      // [64] folded
  void* out;           // NHWC [N][H][W][64] element type T
  int N, C, H, W;
};

// Kernel configurations (rows tile x pixel tile).
// CFG_R*_P*: per-tap gathered B tile (rows x pixels, tile 16 px wide); CFG_HALO_*: 16x16
// pixel tile with an LDS halo (3x3 only), R = rows per block, W = waves per block.
enum Cfg : int {
  CFG_R128_P128 = 0, CFG_R64_P128 = 1, CFG_R64_P256 = 2, CFG_R128_P256 = 3,
  CFG_HALO_R128_W4 = 4, CFG_HALO_R128_W8 = 5, CFG_HALO_R64_W4 = 6, CFG_HALO_R64_W8 = 7,
  CFG_HALO1_R64_W4 = 8, CFG_HALO1_R64_W8 = 9,   // single halo buffer, two blocks per CU
  CFG_HALO1_R128_W4 = 10,                       // single halo buffer, 2-slot weight ring
  // software-pipelined fragment reads (next kk / next step read behind the MFMAs)
  CFG_PHALO_R128_W8 = 11, CFG_PHALO1_R64_W4 = 12, CFG_PHALO1_R64_W8 = 13,
  // 128-row x 64-pixel wave tiles (4 waves, 128 x 256 block), single halo buffer
  CFG_HALO1_R128T8_NS2 = 14, CFG_HALO1_R128T8_NS3 = 15,
  // down1.3 with down1.0 fused: the 18x18x64 halo is computed from the raw input (16-bit)
  CFG_FUSED_IN_W4 = 16, CFG_FUSED_IN_W8 = 17,
  // 8x16 pixel tiles (10x18 halo, 23 KB): HB=1 -> 3 blocks per CU; HB=2 persistent -> 2 per CU
  CFG_T8_HALO1_R64_W4 = 18, CFG_T8_HALO_R64_W4 = 19, CFG_T8_HALO_R64_W2 = 20,
  // persistent, 3-deep halo ring (two chunks / tiles of HBM loads in flight per CU)
  CFG_HALO3_R64_W8 = 21, CFG_HALO3_R64_W4 = 22,
  // single halo buffer with the fixed read/MFMA interleave (PIPE 7, sched_group_barrier)
  CFG_SG_R128T8_NS2 = 23, CFG_SG_R128T8_NS3 = 24, CFG_SG_R64_W4 = 25, CFG_SG_R64_W8 = 26,
  // 32-channel (64-byte-row) K chunks: double-buffered halo + NS-slot weight ring, persistent,
  // weights pre-packed in step order per row tile (a different K order: chunk32-major, tap-minor)
  CFG_RING_R128 = 27, CFG_RING_R64 = 28, CFG_RING_R128_NS3 = 29, CFG_RING_R64_NS5 = 30,
  // 64-row ring stepping one kernel row (3 taps, 48 MFMAs per wave) per barrier, 3 slots of 3 taps
  CFG_RING_R64_T3 = 31,
  // ConvTranspose only: persistent ring GEMM, A and B through one 3-slot LDS-DMA ring (64-byte K steps)
  CFG_TRING_R128 = 32,
  // down1.0 fused into down1.3 on the 3-taps-per-step ring (halo chunks computed from the input)
  CFG_RING_FUSED_IN = 33,
  // ConvTranspose ring with the row tiles of one pixel tile taken back to back by one walker
  CFG_TRING_R128_CTI = 34,
  // ConvTranspose ring with 8-wave 256-row x 256-pixel block tiles (one block per CU)
  CFG_TRING_R256 = 35, CFG_TRING_R256_NS4 = 36,
  CFG_COUNT = 37
};
bool cfg_single_chunk(int cfg);
int cfg_rows(int cfg);
int cfg_pixels(int cfg);
bool cfg_is_halo(int cfg);
bool cfg_is_ring(int cfg);   // 64-byte-row ring kernel: step-major packed weights
int ring_ns(int cfg);       // ring kernel: weight-ring slots
int ring_tps(int cfg);      // ring kernel: taps per step
bool cfg_is_tring(int cfg); // ConvTranspose ring kernel: step-major packed weights
int cfg_limit();   // number of valid Cfg values in this build

hipError_t launch_igemm(DType t, int cfg, int taps, int epi, const IgemmArgs& a, hipStream_t s);
hipError_t launch_first_conv(DType t, const FirstConvArgs& a, hipStream_t s);
// fp32 NCHW input -> T [N][H][W][4] (input of the fused first conv of CFG_RING_FUSED_IN)
hipError_t launch_x_to_px4(DType t, const float* x, int N, int C, int H, int W, void* out, hipStream_t s);
// NHWC (pixel stride ld, channel offset choff, C channels) element type t -> NCHW fp32
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
hipError_t launch_resample(const ResamplePlan& p, const uint8_t* img, int C, uint8_t* tmp, float* out,
                           hipStream_t s);

// per-(image, field) mask bounding boxes [N*ncls][4] = x_min, y_min, x_max, y_max (-1s if empty)
constexpr int kMaxBoxW = 16384;
hipError_t launch_mask_boxes(const uint8_t* masks, int kind, int N, int ncls, int H, int W, int* boxes,
                             hipStream_t s);

}  // namespace unet
