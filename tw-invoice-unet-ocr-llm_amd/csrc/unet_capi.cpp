// C-ABI host layer of the MI355X UNet forward path (include/unet_mi355x.h).
//
// Owns: strict state_dict ingestion (unet_model.py:24-53 key set), eval-BatchNorm folding
// (unet_model.py:11,15; eps 1e-5), the per-layer storage-precision plan, weight pre-packing for
// the implicit-GEMM kernels, the activation workspace, and the per-forward launch sequence that
// mirrors UNet.forward (unet_model.py:55-86).
#include "unet_internal.h"
#include "../../include/unet_mi355x.h"

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

using namespace unet;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(UNET_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

uint16_t f32_to_f16(float f) {
  _Float16 h = (_Float16)f;
  uint16_t r;
  std::memcpy(&r, &h, 2);
  return r;
}

// Packed-weight row permutation inside each 64-row group (see unet_kernels.hip
// epilogue): packed row rho = t*16 + r holds natural row (r>>2)*16 + t*4 + (r&3).
inline int natural_of_packed(int rho) {
  const int g = rho & ~63, w = rho & 63, t = w >> 4, r = w & 15;
  return g + (r >> 2) * 16 + t * 4 + (r & 3);
}

struct Layer {
  int cin = 0, cout = 0, ctot = 0, taps = 9, cfg = CFG_RING_R128;
  DType dt = DType::BF16;    // operand type (activations read + packed weights)
  DType dto = DType::BF16;   // output type (type of the consumer's operand)
  DType dtq = DType::BF16;   // pooled-map type (EPI_POOL layers)
  void* w = nullptr;         // packed weights
  float* b = nullptr;        // [ctot] natural order
  int x3 = 0;                // fp32 plan: operands as three bf16 terms (IgemmArgs::x3; 2 = pre-split packing)
};

// Device coefficient tables of one resize geometry (unet_preprocess), owned by the handle.
struct ResampleStore {
  ResamplePlan plan{};
  std::vector<void*> bufs;
};
constexpr size_t kResampleCacheMax = 16;   // geometries kept (LRU)

struct Buffers {
  size_t tA, cat1, cat2, cat3, cat4, p1, p2, p3, p4, bnb, tB, mbits, xpx, part, total;  // byte offsets
};

}  // namespace

struct unet_handle {
  unet_config cfg{};
  DType dt = DType::BF16;   // storage element type of the workspace (bf16 / f16 plans: 2 bytes)
  float* w0 = nullptr;  // first conv folded fp32 [64][C][3][3]
  void* w0p = nullptr;  // first conv packed [64][32] (16-bit MFMA path, down1.3's operand type)
  void* w0r = nullptr;  // the ring kernel's fused first conv: [cb][t][m][16 rows][16 k] (unet_load_weights)
  float* b0 = nullptr;
  Layer L[17];          // d1b d2a d2b d3a d3b d4a d4b bna bnb c4a c4b c3a c3b c2a c2b c1a c1b
  Layer U[4];           // up4 up3 up2 up1
  // the three-term plan's small-batch ConvTranspose (N <= kSmallBatch with the split-K plan on; w == nullptr
  // otherwise): pre-split weights on 64-row tiles, where the large-batch plan's 128-row tiles split both
  // operands on the fly -- the same products in the same order per accumulator (unsplit: bitwise the same)
  Layer Us[4];
  // up1 fused into conv2.3 (EPI_UPFUSE, 16-bit plans): conv2.3's ring weights followed by 8
  // ConvTranspose steps (pack_fused_up); the forward then has no up1 launch and conv2.3's output
  // is never stored (unet_debug_fetch "c7" is unavailable).  UNET_MI355X_FUSE_UP1=0 disables it.
  bool fuse_up1 = false;
  void* wf_c2b = nullptr;
  bool last_fused = false;
  float* head_w = nullptr;
  float* head_b = nullptr;
  void* zero = nullptr;
  bool loaded = false;
  char* ws = nullptr;
  size_t ws_bytes = 0;
  int lastN = 0, lastH = 0, lastW = 0;
  std::vector<void*> allocs;
  // (ih, iw, oh, ow) -> tables, most recently used first
  std::list<std::pair<std::tuple<int, int, int, int>, ResampleStore>> resample;
  uint8_t* pp_tmp = nullptr;              // horizontal-pass rows of unet_preprocess
  size_t pp_tmp_bytes = 0;
  std::string labels[UNET_NUM_LAUNCHES];   // kernel instantiation of every launch
  float thr_logit[kMaxClasses];           // per-class logit cut, see unet_logit_cut
  // stream ordering of the shared workspace: the last call's completion event and stream
  hipEvent_t done = nullptr;
  hipStream_t last_stream = nullptr;
  bool pending = false;
  bool capturing = false;        // inside unet_graph_create: no event record / wait in the stream
  void* comm = nullptr;          // RCCL communicator (unet_comm_init), ncclComm_t
  unsigned long long generation = 1;   // bumped whenever device pointers a graph captured change
  // split-K of under-filled layers (small batches, layer_split): the largest slice count
  // (UNET_MI355X_KSPLIT; 0 or 1 = never split) and per-launch forced counts for A/B runs
  // (UNET_MI355X_KSPLIT_FORCE="i:ks,...", i = 3x3 layer 0..16 or 17 + ConvTranspose 0..3; 0 = auto;
  // ks + 100 = ks slices on 64-row tiles of the 8-wave ring)
  int ksplit_max = 32;
  int f32x3 = 0;   // fp32 plan: operands as three bf16 terms on the bf16 MFMA pipe (IgemmArgs::x3): 2 = split-once
                   // 128-row tiles on the Cout >= 128 layers, 1 = 64-row tiles everywhere
  int ksplit_force[21] = {};
  void* part = nullptr;   // the current forward's partial buffer (workspace region Buffers::part)
  // mask-box sync entries (launch_mask_boxes: kSyncInts ints per (image, field), idle between
  // launches), grown by unet_reserve
  int* box_sync = nullptr;
  int box_sync_n = 0;
};

struct unet_graph {
  unet_handle* h = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  unsigned long long generation = 0;
  // unet_photo_graph_create: the resize tables and row buffer the captured preprocess reads, owned by
  // the graph (the handle's geometry cache may evict its own copy without staling the graph)
  ResampleStore rs;
  uint8_t* pp_tmp = nullptr;
  int* crop_sync = nullptr;   // the crop sums' sync entries (n_classes, zeroed at capture)
  // the photo graph's masks copy node (unet_photo_graph_set_masks retargets its host destination)
  hipGraphNode_t masks_node = nullptr;
  void* masks_dst = nullptr;
  const void* masks_src = nullptr;
  size_t masks_bytes = 0;
};

namespace {

enum LayerId { D1B, D2A, D2B, D3A, D3B, D4A, D4B, BNA, BNB, C4A, C4B, C3A, C3B, C2A, C2B, C1A, C1B };
const char* kLayerKey[17][2] = {  // (block, conv index) of each implicit-GEMM 3x3 conv
    {"down1", "3"}, {"down2", "0"}, {"down2", "3"}, {"down3", "0"}, {"down3", "3"},
    {"down4", "0"}, {"down4", "3"}, {"bottleneck", "0"}, {"bottleneck", "3"},
    {"conv4", "0"}, {"conv4", "3"}, {"conv3", "0"}, {"conv3", "3"},
    {"conv2", "0"}, {"conv2", "3"}, {"conv1", "0"}, {"conv1", "3"}};
const int kLayerCh[17][2] = {{64, 64},    {64, 128},   {128, 128}, {128, 256}, {256, 256},
                             {256, 512},  {512, 512},  {512, 1024}, {1024, 1024},
                             {1024, 512}, {512, 512},  {512, 256}, {256, 256},
                             {256, 128},  {128, 128},  {128, 64},  {64, 64}};
// Resolution level (0 = full resolution) of each 3x3 layer's input and output; EPI_POOL layers
// also write a pooled map one level down.  ConvTranspose up_k reads level k and writes k-1.
const int kLayerLevel[17] = {0, 1, 1, 2, 2, 3, 3, 4, 4, 3, 3, 2, 2, 1, 1, 0, 0};
const int kUpLevel[4] = {4, 3, 2, 1};   // input level of up4..up1
// Default kernel configuration per 3x3 layer, from in-process A/B timing on MI355X at bs256
// 512x512 (tools/tune.py; profiles/tune_r1*.txt).
//   16-bit: the 64-byte-row ring kernel; 128-row wave tiles on every layer with Cout >= 128
//   (profiles/tune_r1_ring.txt), 3 taps per step on the 64-channel layers (tune_r1_ring_t3.txt),
//   down1.0 fused into down1.3 (tune_r1_ring_fused_in.txt).
//   fp32: the 128-byte LDS-halo kernel (tune_r1.txt).
//   round 2: the 8-wave 16x32-tile weight-stationary ring on the two Cin = 64 layers at 512^2
//   (conv1.3 + head -14 %, down1.3 with the fused first conv -4 %: profiles/tune_r2_ring8*.txt);
//   session 2: the 8-wave 16x32-tile ring with 3 pipelined taps per step on every 128-row layer
//   (-4..-11 % per layer, profiles/tune_r2j_ring8_r128_t3.txt), conv2.3 with the fused up1
//   (EPI_UPFUSE) included (-5.5 %, tune_r2j_fused_up1.txt); conv1.0 on the 8-wave 64-row ring with
//   a whole 32-channel chunk (9 pipelined taps) per step (-11 %, tune_r2j_ring8_r64_t9.txt).
const int kRingCfg[17] = {
    CFG_RING8_FUSED_IN,                                 // down1.0 + down1.3 (+pool), fused
    CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128,
    CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128, CFG_RING8_R128,
    CFG_RING8_R128, CFG_RING8_R128,                     // down2.0 .. conv2.3 (+ up1 fused)
    CFG_RING8_R64_T9, CFG_RING8_R64_WS};                // conv1.0 (one chunk per step), conv1.3 (+head)
const int kHaloCfg[17] = {
    CFG_HALO_R64_W8,                                    // down1.3 (+pool)
    CFG_HALO_R128, CFG_HALO_R128, CFG_HALO_R128, CFG_HALO_R64_W4, CFG_HALO_R128, CFG_HALO_R64_W4,
    CFG_HALO_R128, CFG_HALO_R128, CFG_HALO_R128, CFG_HALO_R128, CFG_HALO_R128, CFG_HALO_R128,
    CFG_HALO_R128, CFG_HALO_R128,                       // down2.0 .. conv2.3
    CFG_HALO_R64_W4, CFG_HALO_R64_W8};                  // conv1.0, conv1.3 (+head)
const char* kUpKey[4] = {"up4", "up3", "up2", "up1"};
const int kUpCh[4][2] = {{1024, 512}, {512, 256}, {256, 128}, {128, 64}};

// Storage precision of a level under the handle's dtype.  UNET_DTYPE_MIXED: fp16 at the two
// full-resolution levels 0-1 (where the mask boundaries are decided), bf16 at levels 2-4.
// Chosen by tools/numerics_emulate.py: bf16 everywhere gives a worst field IoU of 0.9983 against
// the fp32 reference masks on the bench pages, fp16 at levels 0-1 0.9994, fp16 at level 0 only
// 0.9990.  fp16 and bf16 run the same MFMA rate on gfx950.
DType level_dtype(int dtype, int level) {
  switch (dtype) {
    case UNET_DTYPE_F32: case UNET_DTYPE_F32_EXACT: return DType::F32;
    case UNET_DTYPE_F16: return DType::F16;
    case UNET_DTYPE_MIXED: return level <= 1 ? DType::F16 : DType::BF16;
    default: return DType::BF16;
  }
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Split-K over Cin for a layer whose grid of (pixel tile, row tile) blocks under-fills the chip --
// the small-batch plan of the production call (inference.py: one photo per run_unet; at batch 1 the
// 32^2 bottleneck has 16 ring blocks for 256 CUs).  KS slices run as independent blocks writing fp32
// partials (EPI_PARTIAL) that launch_splitk_reduce adds to the bias in slice order (deterministic,
// bitwise repeatable).  The plan applies to batches N <= kSmallBatch with KS chosen from the layer's
// batch-1 geometry, so an image's outputs are bitwise the same for every N <= kSmallBatch (and, with
// the unsplit kernels, for every N > kSmallBatch); the two regimes accumulate in different orders and
// agree within the fp32-accumulation tolerance, not bit for bit.  KS is the power of two minimising a
// two-term model: compute on min(blocks x KS, 256) CUs at the family's per-CU rate, plus the partials'
// HBM round trip and one more launch.  Eligible: the 8-wave 128-row ring (16-bit plans) and the
// LDS-halo family (fp32 plan, 3x3 and ConvTranspose) with a plain store, pool or scatter epilogue;
// never the fused first conv, the head or the fused up1.
constexpr int kSmallBatch = 4;
// ConvTranspose j's layer at batch N: the small-batch variant Us[j] where the plan has one
const Layer& up_layer(const unet_handle* h, int j, int N) {
  return (h->Us[j].w && h->ksplit_max > 1 && N >= 1 && N <= kSmallBatch) ? h->Us[j] : h->U[j];
}
struct Split {
  int ks = 1;     // K slices (1 = the layer runs unsplit)
  int rows = 0;   // 8-wave ring: row tile of the slices (64 = halves of the 128-row packing), 0 = the layer's own
};
Split layer_split(const unet_handle* h, int id, const Layer& L, int epi, int N, int Hl, int Wl) {
  Split best;
  if (h->ksplit_max <= 1 || N <= 0 || N > kSmallBatch || Hl <= 0 || Wl <= 0) return best;
  const bool ring8 = L.cfg == CFG_RING8_R128 && L.dt != DType::F32 && L.taps == 9;
  const bool halo = cfg_is_halo(L.cfg) && L.dt == DType::F32;
  if (L.cfg == CFG_TRING_R256 && L.dt != DType::F32 && epi == EPI_UPSCATTER) {
    // the 16-bit ConvTranspose ring: no K split (its partials' bytes per FLOP are 4-8x a 3x3 layer's),
    // but 128-row tiles over the 256-row packing (4-wave blocks, two per CU) when its 256-row grid
    // fills less than half the CUs (batch 1: up4 32 blocks, up3 64, up2 128)
    const long long blocks = (long long)(L.ctot / 256) * ((Hl + 15) / 16) * ((Wl + 15) / 16);
    if (blocks < 128 && L.ctot % 256 == 0) best.rows = 128;
    return best;
  }
  if (!(ring8 || halo)) return best;
  if (!(epi == EPI_STORE || epi == EPI_POOL || epi == EPI_UPSCATTER)) return best;
  const int chunk = 32;   // K slice granule: one 32-channel chunk (ring8 16-bit, halo fp32)
  const int nch = L.cin / chunk;
  if (L.cin % chunk) return best;
  const int tw = cfg_tile_w(L.cfg), th = cfg_tile_h(L.cfg);
  // resident blocks: one 512-thread block per CU (the 8-wave ring, the split-once three-term tiles) / two halo blocks
  const int cap = ring8 || L.x3 >= 3 ? 256 : 512;
  // per-CU FLOP/s of the family and the partials' effective write + read rate, fitted to the batch-1
  // per-layer times with and without the split (profiles/tune_r4b_bs1_ksplit_*.txt: 134 MB of fp32
  // partials cost ~42 us = 3.2 TB/s including the reduction's launch)
  const double bw = 3.2e12, t_launch = 4e-6;
  const double P = (double)Hl * Wl;
  const double flops = 2.0 * L.ctot * L.cin * L.taps * P;
  // blocks of ONE image (the plan depends on the layer and resolution only, not on N)
  const long long tiles = (long long)((Hl + th - 1) / th) * ((Wl + tw - 1) / tw);
  const int forced = h->ksplit_force[id];
  // candidate row tiles: the layer's own; on the ring also 64-row halves (twice the blocks per slice, so
  // half the slices for the same CU count; 0.8x the per-CU rate: half the MFMAs per halo byte)
  const int own = cfg_rows(L.cfg);
  // the LDS-halo family's per-CU rate: exact-fp32 MFMA ~0.5 TF/s, the three-term plan ~0.85 TF/s (fp32 FLOPs) on
  // 64-row tiles, ~1.1 on the split-once 128-row tiles (a first estimate: to be fitted on the batch-1 sweep)
  const double halo_rate = L.x3 >= 3 ? 1.1e12 : L.x3 ? 0.85e12 : 0.5e12;
  // CUs' worth of throughput from `blocks` resident blocks.  The three-term 64-row tiles run two blocks per CU,
  // and a CU holding only one runs at ~0.6 of its two-block rate (the second block covers the first one's
  // split and halo waits): count the first 256 blocks at 0.6 and the next 256 at 0.4 (fitted to the batch-1
  // sweep of forced slice counts, gpurun_out/bs1_sweep_r6i_fp32.txt: every deep layer fastest at 512 blocks)
  const bool two_tier = !ring8 && L.x3 == 2 && cap == 512;
  auto cu_eq = [&](long long blocks) -> double {
    if (!two_tier) return (double)std::min<long long>(blocks, 256);
    return 0.6 * (double)std::min<long long>(blocks, 256) +
           0.4 * (double)std::max<long long>(0, std::min<long long>(blocks, 512) - 256);
  };
  double tbest = flops / (cu_eq(tiles * (L.ctot / own)) * (ring8 ? 6e12 : halo_rate));
  for (int rows : {own, ring8 ? 64 : 0}) {
    if (rows == 0) break;
    const double rate = ring8 ? (rows == 128 ? 6e12 : 4.8e12) : halo_rate;
    const long long blocks = tiles * (L.ctot / rows);
    if (forced > 0) {   // A/B runs: ks on the layer's own row tile, ks + 100 on 64-row tiles (the ring)
      const int fks = forced % 100, frows = forced >= 100 ? 64 : own;
      if (rows == frows && fks <= nch && nch % fks == 0 && blocks * fks <= 8LL * cap)
        best = {fks, rows == own ? 0 : rows};
      continue;
    }
    if (rows != own && epi != EPI_UPSCATTER) {   // finer row tiles alone, no K split (no partials)
      const double t = flops / (cu_eq(blocks) * rate);
      if (t < 0.9 * tbest) { tbest = t; best = {1, rows}; }
    }
    for (int ks = 2; ks <= h->ksplit_max && nch % ks == 0 && nch / ks >= (ring8 ? 2 : 1) && blocks * ks <= cap; ks *= 2) {
      const double t = flops / (cu_eq(blocks * ks) * rate) + ks * P * L.ctot * 8.0 / bw + t_launch;
      if (t < 0.9 * tbest) { tbest = t; best = {ks, rows == own ? 0 : rows}; }   // a split must win by 10 %
    }
  }
  return best;
}

// Launch order of forward_impl with each launch's layer, epilogue and input level, for the split-K
// plan's workspace bound (the largest partial buffer of one launch).
size_t split_bytes(const unet_handle* h, int N, int H, int W) {
  size_t m = 0;
  auto one = [&](int id, const Layer& L, int epi, int lvl) {
    const int Hl = H >> lvl, Wl = W >> lvl;
    const int ks = layer_split(h, id, L, epi, N, Hl, Wl).ks;
    if (ks > 1) m = std::max(m, (size_t)ks * N * Hl * Wl * L.ctot * 4);
  };
  for (int i = 0; i < 17; ++i) {
    const bool pool = i == D1B || i == D2B || i == D3B || i == D4B;
    int epi = pool ? EPI_POOL : i == C1B ? EPI_HEAD : EPI_STORE;
    if (i == C2B && h->fuse_up1) epi = EPI_UPFUSE;
    if (i == D1B && cfg_fused_in(h->L[D1B].cfg)) continue;
    one(i, h->L[i], epi, kLayerLevel[i]);
  }
  for (int j = 0; j < 4; ++j)
    if (!(j == 3 && h->fuse_up1)) one(17 + j, up_layer(h, j, N), EPI_UPSCATTER, kUpLevel[j]);
  return m;
}

Buffers plan(const unet_handle* h, int N, int H, int W) {
  const DType dt = h->dt;
  const size_t e = dtype_size(dt);
  const size_t P = (size_t)N * H * W;  // full-resolution pixels
  Buffers b{};
  size_t o = 0;
  auto take = [&](size_t elems) { size_t r = o; o = align256(o + elems * e); return r; };
  b.tA = take(P * 64);
  b.cat1 = take(P * 128);
  b.cat2 = take(P / 4 * 256);
  b.cat3 = take(P / 16 * 512);
  b.cat4 = take(P / 64 * 1024);
  b.p1 = take(P / 4 * 64);
  b.p2 = take(P / 16 * 128);
  b.p3 = take(P / 64 * 256);
  b.p4 = take(P / 256 * 512);
  b.bnb = take(P / 256 * 1024);
  b.tB = take(P / 4 * 128);
  b.mbits = o;   // bit-packed masks for unet_forward_boxes without caller masks (<= kMaxClasses fields)
  o = align256(o + (size_t)kMaxClasses * P / 8);
  // network input in the first layer's format: T [N][H][W][4] (16-bit ring kernel's fused first
  // conv) or fp32 NCHW (fp32 path, when the caller's input is not fp32 NCHW already)
  // (either buffer of the two: 8 B per pixel for T [N][H][W][4], up to 12 B for fp32 NCHW with C = 3
  // -- the latter also on a 16-bit plan whose down1.3 is overridden to a non-fused configuration)
  b.xpx = o;
  o = align256(o + P * 3 * 4);
  b.part = o;   // split-K partials (small batches; 0 bytes when no launch splits)
  o = align256(o + split_bytes(h, N, H, W));
  b.total = o;
  return b;
}

int dev_alloc(unet_handle* h, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return fail(UNET_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  h->allocs.push_back(*p);
  return UNET_OK;
}

int upload(unet_handle* h, void** dst, const void* src, size_t bytes) {
  int rc = dev_alloc(h, dst, bytes);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return UNET_OK;
}

struct SD {
  std::map<std::string, const unet_tensor_view*> m;
  const float* get(const std::string& k, std::initializer_list<int64_t> shape, std::string& err) const {
    auto it = m.find(k);
    if (it == m.end()) { err = "missing key " + k; return nullptr; }
    const unet_tensor_view* v = it->second;
    if (v->dtype != 0) { err = "key " + k + " must be float32"; return nullptr; }
    if ((size_t)v->ndim != shape.size()) { err = "key " + k + ": wrong rank"; return nullptr; }
    int i = 0;
    for (int64_t s : shape) {
      if (v->shape[i++] != s) { err = "key " + k + ": wrong shape"; return nullptr; }
    }
    return static_cast<const float*>(v->data);
  }
};

// Fold eval BatchNorm into conv (double precision): W' = W*g/sqrt(v+eps), b' = (b-m)*g/sqrt(v+eps)+beta
int fold(const SD& sd, const std::string& blk, const std::string& ci, int cin, int cout,
         std::vector<double>& w, std::vector<double>& b) {
  std::string err;
  const std::string bn = std::to_string(std::stoi(ci) + 1);
  const float* W = sd.get(blk + ".net." + ci + ".weight", {cout, cin, 3, 3}, err);
  const float* B = W ? sd.get(blk + ".net." + ci + ".bias", {cout}, err) : nullptr;
  const float* g = B ? sd.get(blk + ".net." + bn + ".weight", {cout}, err) : nullptr;
  const float* be = g ? sd.get(blk + ".net." + bn + ".bias", {cout}, err) : nullptr;
  const float* mu = be ? sd.get(blk + ".net." + bn + ".running_mean", {cout}, err) : nullptr;
  const float* var = mu ? sd.get(blk + ".net." + bn + ".running_var", {cout}, err) : nullptr;
  if (!var) return fail(UNET_EKEY, err);
  if (!sd.m.count(blk + ".net." + bn + ".num_batches_tracked"))
    return fail(UNET_EKEY, "missing key " + blk + ".net." + bn + ".num_batches_tracked");
  w.assign((size_t)cout * cin * 9, 0.0);
  b.assign(cout, 0.0);
  for (int o = 0; o < cout; ++o) {
    const double s = (double)g[o] / std::sqrt((double)var[o] + 1e-5);
    for (int k = 0; k < cin * 9; ++k) w[(size_t)o * cin * 9 + k] = (double)W[(size_t)o * cin * 9 + k] * s;
    b[o] = ((double)B[o] - (double)mu[o]) * s + (double)be[o];
  }
  return UNET_OK;
}

void put_elem(DType dt, std::vector<uint8_t>& buf, size_t idx, double v) {
  if (dt == DType::F32) {
    float f = (float)v;
    std::memcpy(&buf[idx * 4], &f, 4);
  } else {
    uint16_t u = dt == DType::BF16 ? f32_to_bf16((float)v) : f32_to_f16((float)v);
    std::memcpy(&buf[idx * 2], &u, 2);
  }
}

// fp16 storage (the fp16 and mixed plans) holds |v| <= 65504: a folded weight or bias beyond that
// (e.g. a BatchNorm with a tiny running_var: scale gamma / sqrt(var + 1e-5) up to ~316 gamma) would
// silently become inf.  Refused at load time; bf16 keeps fp32's range.
int check_f16_range(DType dt, const std::vector<double>& w, const std::vector<double>& b, const std::string& what) {
  if (dt != DType::F16) return UNET_OK;
  double m = 0.0;
  for (double v : w) m = std::max(m, std::fabs(v));
  for (double v : b) m = std::max(m, std::fabs(v));
  if (!(m <= 65504.0))
    return fail(UNET_EINVAL, what + ": folded weights reach " + std::to_string(m) +
                                 ", beyond the fp16 range (65504) of this precision plan; use dtype bf16 or fp32");
  return UNET_OK;
}

// The first conv's MFMA operand (first_conv_mfma_kernel): [t][m][16 rows][16 k], packed row
// rho = 16t + r = natural channel natural_of_packed(rho), k = 4q + c <-> tap first_tap(4m + q) (< 9), channel c
// (< C); w = the folded [64][C][3][3] weights.
void pack_first_mfma(DType t0, const std::vector<double>& w, int C, std::vector<uint8_t>& pk) {
  pk.assign((size_t)4 * 3 * 16 * 16 * 2, 0);
  for (int rho = 0; rho < 64; ++rho) {
    const int o = natural_of_packed(rho), tt = rho >> 4, r = rho & 15;
    for (int m = 0; m < 3; ++m)
      for (int q = 0; q < 4; ++q) {
        const int tap = first_tap(4 * m + q);
        if (tap >= 9) continue;
        for (int c = 0; c < C; ++c)
          put_elem(t0, pk, (((size_t)(tt * 3 + m) * 16 + r) * 16 + 4 * q + c), w[(size_t)o * 9 * C + c * 9 + tap]);
      }
  }
}

// 3x3 layer: packed[rho][tap*cin + c] = W'[nat(rho)][c][ky][kx], tap = ky*3+kx
// Ring kernels (cfg_is_ring) take the same rows in step order instead: per row tile of BR rows,
// step s = (c / BKE) * 9 + tap holds a contiguous [BR][BKE] block (BKE = 64 bytes of K), so
// packed[((ct * S + s) * BR + rho % BR) * BKE + c % BKE], S = 9 * cin / BKE.
// fp32 as three bf16 terms (round to nearest even, each difference exact in fp32): the device's split3_bf16
void split3_host(float v, uint16_t (&t)[3]) {
  t[0] = f32_to_bf16(v);
  float hi;
  uint32_t u = (uint32_t)t[0] << 16;
  std::memcpy(&hi, &u, 4);
  const float r = v - hi;
  t[1] = f32_to_bf16(r);
  u = (uint32_t)t[1] << 16;
  float mid;
  std::memcpy(&mid, &u, 4);
  t[2] = f32_to_bf16(r - mid);
}

// The three-term fp32 plan's 3x3 weights (L.x3 == 2, conv3x3_halo_kernel X3 = 2): per 64-row tile ct and K
// step g = (32-channel chunk, tap) -- the halo kernel's step order -- three bf16 planes (hi, mid, lo) of
// 64 rows x 64 B; in row r, 16-byte chunk q holds channels 4q..4q+3 and 16+4q..16+4q+3 of the chunk (the
// K values lane group q of the activation fragments holds) at position q ^ ((r >> 1) & 3).
// One row of a pre-split step block (blk = the block's byte offset, r = row in the tile): value(c) for the
// chunk's 32 channels c = 32 * ch + ...
template <typename F>
void put_split_row(std::vector<uint8_t>& buf, size_t blk, int BR, int r, int ch, F value) {
  for (int j = 0; j < 32; ++j) {   // bf16 slot j of the row: chunk q = j / 8, element e = j % 8
    const int q = j >> 3, e = j & 7;
    const int c = 32 * ch + (e < 4 ? 4 * q + e : 16 + 4 * q + e - 4);
    uint16_t t[3];
    split3_host((float)value(c), t);
    const size_t off = (size_t)r * 64 + (size_t)((q ^ ((r >> 1) & 3)) * 16) + (size_t)e * 2;
    for (int p = 0; p < 3; ++p) std::memcpy(&buf[blk + (size_t)p * BR * 64 + off], &t[p], 2);
  }
}
int pack3x3_split(const Layer& L, const std::vector<double>& w, std::vector<uint8_t>& buf) {
  const int BR = cfg_rows(L.cfg), NCH = L.cin / 32, S = 9 * NCH;
  if (L.cout % BR || L.cin % 32) return fail(UNET_EINVAL, "pre-split weight tiling does not divide the layer");
  buf.assign((size_t)L.cout * 9 * L.cin * 6, 0);
  for (int rho = 0; rho < L.cout; ++rho) {
    const int o = natural_of_packed(rho), ct = rho / BR, r = rho % BR;
    for (int ch = 0; ch < NCH; ++ch)
      for (int tap = 0; tap < 9; ++tap)
        put_split_row(buf, ((size_t)ct * S + (size_t)ch * 9 + tap) * 3 * BR * 64, BR, r, ch,
                      [&](int c) { return w[((size_t)o * L.cin + c) * 9 + tap]; });
  }
  return UNET_OK;
}

int pack3x3_host(const Layer& L, const std::vector<double>& w, std::vector<uint8_t>& buf) {
  if (L.x3 >= 2) return pack3x3_split(L, w, buf);
  const int K = 9 * L.cin;
  buf.assign((size_t)L.cout * K * dtype_size(L.dt), 0);
  const bool ring = cfg_is_ring(L.cfg);
  const int BR = cfg_rows(L.cfg), BKE = 64 / (int)dtype_size(L.dt), S = K / BKE;
  if (ring && (L.cout % BR || L.cin % BKE)) return fail(UNET_EINVAL, "ring kernel tiling does not divide the layer");
  for (int rho = 0; rho < L.cout; ++rho) {
    const int o = natural_of_packed(rho);
    for (int tap = 0; tap < 9; ++tap)
      for (int c = 0; c < L.cin; ++c) {
        const size_t idx = ring ? (((size_t)(rho / BR) * S + (size_t)(c / BKE) * 9 + tap) * BR + rho % BR) * BKE + c % BKE
                                : (size_t)rho * K + (size_t)tap * L.cin + c;
        put_elem(L.dt, buf, idx, w[((size_t)o * L.cin + c) * 9 + tap]);
      }
  }
  return UNET_OK;
}
int pack3x3(unet_handle* h, Layer& L, const std::vector<double>& w, const std::vector<double>& b) {
  std::vector<uint8_t> buf;
  int rc = pack3x3_host(L, w, buf);
  const std::vector<float> bf(b.begin(), b.end());
  if (!rc) rc = upload(h, &L.w, buf.data(), buf.size());
  if (!rc) rc = upload(h, (void**)&L.b, bf.data(), bf.size() * 4);
  return rc;
}

// conv2.3 + up1 (EPI_UPFUSE): conv2.3's ring stream (one 128-row tile, S = 9 * cin / BKE steps,
// as pack3x3) followed by 8 ConvTranspose steps u = (quadrant u >> 1, K blocks 2 (u & 1) + kbl):
// slot row 64 kbl + rr = packed row rho = 64 * quadrant + rr (natural row natural_of_packed(rho) =
// quadrant x 64 + o) of K block kb, K slot 8q + j <-> input channel 64 * (kb >> 1) + 16q + 8 * (kb & 1)
// + j (the channels each lane of the conv's accumulators holds, ring_body EPI_UPFUSE).
// The 8-wave ring (CFG_RING8_R128, 24 KB slots of 3 taps) takes the same conv bytes and 4
// ConvTranspose slots instead, one quadrant each: slot row 64 kb + rr (kb = 0..3), rows 256..383 zero.
int pack_fused_up(unet_handle* h, const Layer& L, const Layer& U, const std::vector<double>& w, const float* Wt) {
  const int BR = 128, BKE = 64 / (int)dtype_size(L.dt), S = 9 * L.cin / BKE;
  const bool ring8 = L.cfg == CFG_RING8_R128;
  if (L.cout != BR || U.cin != BR || U.cout != 64 || BKE != 32) return fail(UNET_EINVAL, "fused up1: layer shapes");
  std::vector<uint8_t> buf((size_t)(S + 8 + (ring8 ? 4 : 0)) * BR * BKE * dtype_size(L.dt));
  for (int rho = 0; rho < BR; ++rho) {
    const int o = natural_of_packed(rho);
    for (int tap = 0; tap < 9; ++tap)
      for (int c = 0; c < L.cin; ++c)
        put_elem(L.dt, buf, ((size_t)((c / BKE) * 9 + tap) * BR + rho) * BKE + c % BKE, w[((size_t)o * L.cin + c) * 9 + tap]);
  }
  for (int u = 0; u < 8; ++u) {
    // 4-wave ring: step u = (quadrant u >> 1, K blocks 2 (u & 1) + kbl), slot row 64 kbl + rr;
    // 8-wave ring: 128-row block u of the 4 x 384-row quadrant slots (rows 64 kb + rr, zero past 256)
    const int quad = u >> 1, khalf = u & 1;
    for (int r = 0; r < BR; ++r) {
      const int kb = 2 * khalf + (r >> 6);
      const int nat = natural_of_packed(64 * quad + (r & 63)), ab = nat / 64, o = nat % 64;
      const size_t row = ring8 ? (size_t)S * BR + (size_t)quad * 3 * BR + 64 * kb + (r & 63) : (size_t)(S + u) * BR + r;
      for (int sl = 0; sl < 32; ++sl) {
        const int c = 64 * (kb >> 1) + 16 * (sl >> 3) + 8 * (kb & 1) + (sl & 7);
        put_elem(L.dt, buf, row * BKE + sl, Wt[(((size_t)c * U.cout + o) * 2 + (ab >> 1)) * 2 + (ab & 1)]);
      }
    }
  }
  return upload(h, &h->wf_c2b, buf.data(), buf.size());
}

// ConvTranspose2d (Cin, Cout, 2, 2) as GEMM rows (a, b, o): packed[rho][c] = W[c][o][a][b]; the
// ring kernel (cfg_is_tring) takes them in step order per BR-row tile: [ct][c / BKE][BR][BKE].
int packT(unet_handle* h, Layer& L, const float* W, const float* B) {
  const int R = 4 * L.cout;
  std::vector<uint8_t> buf((size_t)R * L.cin * (L.x3 == 2 ? 6 : dtype_size(L.dt)));
  if (L.x3 == 2) {   // the three-term plan: pre-split planes per (row tile, chunk), as pack3x3_split with one tap
    const int BR = cfg_rows(L.cfg), NCH = L.cin / 32;
    if (R % BR || L.cin % 32) return fail(UNET_EINVAL, "pre-split ConvTranspose tiling does not divide the layer");
    for (int rho = 0; rho < R; ++rho) {
      const int nat = natural_of_packed(rho), ab = nat / L.cout, o = nat % L.cout;
      for (int ch = 0; ch < NCH; ++ch)
        put_split_row(buf, ((size_t)(rho / BR) * NCH + ch) * 3 * BR * 64, BR, rho % BR, ch,
                      [&](int c) { return W[(((size_t)c * L.cout + o) * 2 + (ab >> 1)) * 2 + (ab & 1)]; });
    }
  } else {
    const bool ring = cfg_is_tring(L.cfg);
    const int BR = cfg_rows(L.cfg), BKE = 64 / (int)dtype_size(L.dt), S = L.cin / BKE;
    if (ring && (R % BR || L.cin % BKE)) return fail(UNET_EINVAL, "ring ConvTranspose tiling does not divide the layer");
    for (int rho = 0; rho < R; ++rho) {
      const int nat = natural_of_packed(rho);
      const int ab = nat / L.cout, o = nat % L.cout;
      for (int c = 0; c < L.cin; ++c) {
        const size_t idx = ring ? (((size_t)(rho / BR) * S + c / BKE) * BR + rho % BR) * BKE + c % BKE
                                : (size_t)rho * L.cin + c;
        put_elem(L.dt, buf, idx, W[(((size_t)c * L.cout + o) * 2 + (ab >> 1)) * 2 + (ab & 1)]);
      }
    }
  }
  std::vector<float> bias(R);
  for (int r = 0; r < R; ++r) bias[r] = B[r % L.cout];
  int rc = upload(h, &L.w, buf.data(), buf.size());
  if (!rc) rc = upload(h, (void**)&L.b, bias.data(), bias.size() * 4);
  return rc;
}

// Make the next use of the shared workspace (and of the preprocess buffers) on `s` wait for the
// previous call if that ran on another stream; unet_forward / unet_preprocess calls on different
// streams are thus serialised on the device, not only on the host (the handle has ONE workspace).
// A stream under capture (unet_graph_create's own, or a caller's: torch.cuda.graph captures on a
// side stream) records nothing and waits for nothing: an event recorded outside the capture must not
// enter it, and the captured work runs only when the graph is launched (the caller orders that).
bool stream_capturing(unet_handle* h, hipStream_t s) {
  if (h->capturing) return true;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}
void order_after_last(unet_handle* h, hipStream_t s) {
  if (h->pending && h->last_stream != s && !stream_capturing(h, s)) (void)hipStreamWaitEvent(s, h->done, 0);
}
void mark_done(unet_handle* h, hipStream_t s) {
  if (!stream_capturing(h, s) && hipEventRecord(h->done, s) == hipSuccess) {
    h->last_stream = s;
    h->pending = true;
  }
}

// Every device buffer that queued work may still read is freed only after that work.
void drain(unet_handle* h) {
  if (h->pending) (void)hipEventSynchronize(h->done);
  h->pending = false;
}

void free_resample(ResampleStore& st) {
  for (void* p : st.bufs) (void)hipFree(p);
  st.bufs.clear();
}

void free_all(unet_handle* h) {
  drain(h);
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  for (auto& kv : h->resample) free_resample(kv.second);
  h->resample.clear();
  if (h->pp_tmp) (void)hipFree(h->pp_tmp);
  h->pp_tmp = nullptr;
  h->pp_tmp_bytes = 0;
  if (h->ws) (void)hipFree(h->ws);
  h->ws = nullptr;
  h->ws_bytes = 0;
  if (h->box_sync) (void)hipFree(h->box_sync);
  h->box_sync = nullptr;
  h->box_sync_n = 0;
}

// At least n idle mask-box sync entries (at least 1024: N * n_classes up to 1024 never reallocates).
int ensure_box_sync(unet_handle* h, int n) {
  if (n <= h->box_sync_n) return UNET_OK;
  n = std::max(n, 1024);
  std::vector<int> idle((size_t)n * kSyncInts, 0);
  for (int i = 0; i < n; ++i) {
    int* e = idle.data() + (size_t)i * kSyncInts;
    e[0] = e[1] = 0x7FFFFFFF;
    e[2] = e[3] = -1;
  }
  ++h->generation;   // graphs captured the old entries
  drain(h);
  if (h->box_sync) (void)hipFree(h->box_sync);
  h->box_sync = nullptr;
  h->box_sync_n = 0;
  hipError_t e = hipMalloc((void**)&h->box_sync, idle.size() * sizeof(int));
  if (e != hipSuccess) {
    h->box_sync = nullptr;
    return fail(UNET_ENOMEM, std::string("mask-box sync hipMalloc: ") + hipGetErrorString(e));
  }
  e = hipMemcpy(h->box_sync, idle.data(), idle.size() * sizeof(int), hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("mask-box sync init: ") + hipGetErrorString(e));
  h->box_sync_n = n;
  return UNET_OK;
}

// ---- Pillow's resize coefficients (libImaging/Resample.c: precompute_coeffs +
// normalize_coeffs_8bpc, BICUBIC a = -0.5, support 2), same double-precision operation order
#pragma clang fp contract(off)
double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

int resample_coeffs(int in_size, int out_size, std::vector<int>& bounds, std::vector<int>& kk) {
  const float in0 = 0.f, in1 = (float)in_size;   // Pillow's box edges are floats
  const double scale = (double)(in1 - in0) / out_size;
  double filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 2.0 * filterscale;      // antialiasing: widen by the downscale factor
  const int ksize = (int)std::ceil(support) * 2 + 1;
  bounds.assign((size_t)2 * out_size, 0);
  kk.assign((size_t)out_size * ksize, 0);
  std::vector<double> k(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
      const double w = bicubic_filter((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x) {
      double v = k[x];
      if (ww != 0.0) v /= ww;
      kk[(size_t)xx * ksize + x] = v < 0 ? (int)(-0.5 + v * (1 << 22)) : (int)(0.5 + v * (1 << 22));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}
#pragma clang fp contract(on)

// Pillow's separable BICUBIC tables of one (ih, iw) -> (oh, ow) resize, uploaded (synchronously) into
// device buffers owned by st (unet_preprocess's geometry cache, or a photo graph).
int build_resample(int ih, int iw, int oh, int ow, ResampleStore& st) {
  ResamplePlan& p = st.plan;
  p.ih = ih; p.iw = iw; p.oh = oh; p.ow = ow;
  p.need_h = ow != iw;
  p.need_v = oh != ih;
  std::vector<int> hb, hk, vb, vk;
  p.h_ksize = resample_coeffs(iw, ow, hb, hk);
  p.v_ksize = resample_coeffs(ih, oh, vb, vk);
  p.h_y0 = 0;
  p.h_rows = ih;
  if (p.need_h && p.need_v) {   // the horizontal pass covers only the rows the vertical pass reads
    p.h_y0 = vb[0];
    p.h_rows = vb[2 * (oh - 1)] + vb[2 * (oh - 1) + 1] - p.h_y0;
    for (int i = 0; i < oh; ++i) vb[2 * i] -= p.h_y0;
  }
  const std::vector<int>* src[4] = {&hb, &hk, &vb, &vk};
  const int** dst[4] = {&p.h_bounds, &p.h_kk, &p.v_bounds, &p.v_kk};
  for (int i = 0; i < 4; ++i) {
    void* d = nullptr;
    const size_t bytes = src[i]->size() * sizeof(int);
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) {
      free_resample(st);
      return fail(UNET_ENOMEM, std::string("resample tables: ") + hipGetErrorString(e));
    }
    st.bufs.push_back(d);
    e = hipMemcpy(d, src[i]->data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      free_resample(st);
      return fail(UNET_EHIP, std::string("resample tables upload: ") + hipGetErrorString(e));
    }
    *dst[i] = static_cast<const int*>(d);
  }
  return UNET_OK;
}

int check_geometry(const unet_handle* h, int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return fail(UNET_EINVAL, "N, H, W must be positive");
  if (H % 16 || W % 16)
    return fail(UNET_ESHAPE, "H and W must be divisible by 16 (4 pooling levels; the reference "
                             "fails in torch.cat otherwise, unet_model.py:71)");
  if ((long long)N * H * W > (1LL << 31) / 2) return fail(UNET_ESHAPE, "N*H*W too large for one call");
  (void)h;
  return UNET_OK;
}

const char* tname(DType t) { return t == DType::F32 ? "float" : t == DType::BF16 ? "__bf16" : "_Float16"; }

// "kernel<template args>" of a layer, in the same spelling as the demangled symbol.  sp: the
// small-batch plan's choice for the launch (layer_split): a split layer runs its EPI_PARTIAL kernel and
// the reduction ("A + B"), finer row tiles the 64-row 8-wave ring / the 128-row ConvTranspose ring.
std::string layer_label(const unet_handle* h, const Layer& L, int epi, Split sp = Split{}) {
  char buf[160];
  int cfg = L.cfg;
  (void)h;
  if (sp.ks == 1 && sp.rows && cfg == CFG_TRING_R256) cfg = CFG_TRING_R128;   // run_igemm's batch-1 halves
  if (sp.ks > 1) {   // launch_igemm(..., EPI_PARTIAL) + launch_splitk_reduce
    Layer P = L;
    P.dto = P.dtq = L.dt;
    std::string part = layer_label(h, P, EPI_PARTIAL, Split{1, sp.rows});
    std::snprintf(buf, sizeof buf, " + splitk_reduce_kernel<%s, %s, %d>", tname(L.dto),
                  tname(epi == EPI_POOL ? L.dtq : L.dto), epi);
    return part + buf;
  }
  if (cfg_is_tring(cfg)) {
    std::snprintf(buf, sizeof buf, "convT_ring_kernel<%s, 8, %d, %d, %s>", tname(L.dt), cfg == CFG_TRING_R256 ? 4 : 3,
                  cfg == CFG_TRING_R256 ? 2 : 1, tname(L.dto));
  } else if (cfg_is_ring8(cfg)) {
    const int wst = cfg == CFG_RING8_R64_WS || cfg == CFG_RING8_FUSED_IN;   // weight-stationary
    const int rows = (sp.rows && cfg == CFG_RING8_R128) ? sp.rows : cfg_rows(cfg);
    std::snprintf(buf, sizeof buf, "conv3x3_ring8_kernel<%s, %d, %d, %d, %d, %d, %s, %s, %d, 0>", tname(L.dt),
                  rows / 16, ring_ns(cfg), epi, ring_tps(cfg), wst, tname(L.dto),
                  tname(epi == EPI_POOL ? L.dtq : L.dto), cfg == CFG_RING8_FUSED_IN ? 1 : 0);
  } else if (cfg_is_ring(cfg)) {
    std::snprintf(buf, sizeof buf, "conv3x3_ring_kernel<%s, 1, 4, %d, %d, %d, %d, %d, %s, %s, %d, %d>", tname(L.dt),
                  cfg_rows(cfg) / 16, ring_ns(cfg), epi, ring_tps(cfg), cfg == CFG_RING_FUSED_IN ? 1 : 0,
                  tname(L.dto), tname(epi == EPI_POOL ? L.dtq : L.dto), cfg_tile_h(cfg), cfg_tile_w(cfg));
  } else if (L.x3 == 3 || L.x3 == 4) {
    std::snprintf(buf, sizeof buf, L.x3 == 3 ? "conv3x3_x3s_kernel<%d>" : "conv3x3_x3w_kernel<%d>", epi);
  } else {
    const int wpx = cfg == CFG_HALO_R64_W8 ? 8 : 4, tc = cfg == CFG_HALO_R128 ? 8 : 4,
              ns = L.x3 == 2 ? 2 : cfg == CFG_HALO_R128 ? 2 : 3;
    std::snprintf(buf, sizeof buf, "conv3x3_halo_kernel<%s, 1, %d, %d, %d, %d, %d, %d>", tname(L.dt), wpx, tc, ns,
                  L.taps == 9 ? 3 : 1, epi, L.x3);
  }
  return buf;
}

// Labels of every launch slot for a forward of N x H x W (N = 0: the large-batch plan, N > kSmallBatch,
// whatever the size; otherwise the small-batch plan's choices at that shape, layer_split).
void build_labels_at(const unet_handle* h, int N, int H, int W, std::string (&out)[UNET_NUM_LAUNCHES]) {
  const int C = h->cfg.n_channels;
  char buf[96];
  const DType t0 = h->L[D1B].dt;
  std::snprintf(buf, sizeof buf, t0 == DType::F32 ? "first_conv_kernel<%s, %d>" : "first_conv_mfma_kernel<%s, %d>",
                tname(t0), C);
  // launch order (include/unet_mi355x.h): first, d1b .. bnb, up4, c4a, c4b, up3, c3a, c3b, up2, c2a, c2b, up1, c1a, c1b
  const int order[UNET_NUM_LAUNCHES] = {-1, D1B, D2A, D2B, D3A, D3B, D4A, D4B, BNA, BNB, 100, C4A, C4B,
                                        101, C3A, C3B, 102, C2A, C2B, 103, C1A, C1B};
  for (int i = 0; i < UNET_NUM_LAUNCHES; ++i) {
    const int id = order[i];
    if (id < 0) {
      out[i] = cfg_fused_in(h->L[D1B].cfg) ? std::string("x_to_px4_kernel<") + tname(t0) + ">" : buf;
      continue;
    }
    if (id >= 100) {   // a fused up1 launches nothing: empty label (tools: its time and work go to conv2.3)
      const int j = id - 100;
      out[i] = (j == 3 && h->fuse_up1) ? std::string()
                                       : layer_label(h, up_layer(h, j, N), EPI_UPSCATTER,
                                                     layer_split(h, 17 + j, up_layer(h, j, N), EPI_UPSCATTER, N,
                                                                 H >> kUpLevel[j], W >> kUpLevel[j]));
      continue;
    }
    int epi = id == C1B ? EPI_HEAD : (id == D1B || id == D2B || id == D3B || id == D4B) ? EPI_POOL : EPI_STORE;
    if (id == C2B && h->fuse_up1) epi = EPI_UPFUSE;
    out[i] = layer_label(h, h->L[id], epi,
                         layer_split(h, id, h->L[id], epi, N, H >> kLayerLevel[id], W >> kLayerLevel[id]));
  }
}
void build_labels(unet_handle* h) { build_labels_at(h, 0, 0, 0, h->labels); }

// "layer:cfg,..." override list (tools/tune.py A/B runs)
void parse_overrides(const char* ov, int n, int* cfg_out, bool (*ok)(int, int)) {
  if (!ov) return;
  std::string o(ov);
  size_t pos = 0;
  while (pos < o.size()) {
    size_t end = o.find(',', pos);
    if (end == std::string::npos) end = o.size();
    const std::string item = o.substr(pos, end - pos);
    const size_t colon = item.find(':');
    if (colon != std::string::npos) {
      const int li = std::atoi(item.substr(0, colon).c_str()), c = std::atoi(item.substr(colon + 1).c_str());
      if (li >= 0 && li < n && c >= 0 && c < cfg_limit() && ok(li, c)) cfg_out[li] = c;
      else std::fprintf(stderr, "unet_mi355x: ignoring configuration override '%s'\n", item.c_str());
    }
    pos = end + 1;
  }
}

// RCCL, resolved at run time (dlopen) so the library has no link-time dependency on it and a
// host that never calls unet_comm_* never loads it.  ncclUniqueId is 128 opaque bytes.
struct NcclId { char internal[UNET_COMM_ID_BYTES]; };
struct Rccl {
  void* lib = nullptr;
  int (*get_unique_id)(NcclId*) = nullptr;
  int (*comm_init_rank)(void**, int, NcclId, int) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*comm_destroy)(void*) = nullptr;
  const char* (*error_string)(int) = nullptr;
};
const Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r.lib ? &r : nullptr;
  tried = true;
  for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
    r.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    if (r.lib) break;
  }
  if (!r.lib) return nullptr;
  r.get_unique_id = reinterpret_cast<int (*)(NcclId*)>(dlsym(r.lib, "ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<int (*)(void**, int, NcclId, int)>(dlsym(r.lib, "ncclCommInitRank"));
  r.all_gather = reinterpret_cast<int (*)(const void*, void*, size_t, int, void*, hipStream_t)>(dlsym(r.lib, "ncclAllGather"));
  r.comm_destroy = reinterpret_cast<int (*)(void*)>(dlsym(r.lib, "ncclCommDestroy"));
  r.error_string = reinterpret_cast<const char* (*)(int)>(dlsym(r.lib, "ncclGetErrorString"));
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.error_string) {
    dlclose(r.lib);
    r.lib = nullptr;
    return nullptr;
  }
  return &r;
}
int rccl_fail(const Rccl* r, int rc, const char* what) {
  return fail(UNET_EHIP, std::string(what) + ": " + (r ? r->error_string(rc) : "RCCL unavailable"));
}

}  // namespace

extern "C" {

const char* unet_last_error(void) { return g_err.c_str(); }

namespace {
// fp32 values in a total order as integers (-0 and +0 share a key), so bisection over keys
// walks every float between -inf and +inf.
long long float_key(float f) {
  int32_t i;
  std::memcpy(&i, &f, 4);
  return i >= 0 ? (long long)i : (long long)INT32_MIN - (long long)i;
}
float key_float(long long k) {
  const int32_t i = k >= 0 ? (int32_t)k : (int32_t)((long long)INT32_MIN - k);
  float f;
  std::memcpy(&f, &i, 4);
  return f;
}
bool sigmoid_above(float x, float thr) { return 1.0f / (1.0f + std::exp(-x)) > thr; }
}  // namespace

float unet_logit_cut(float thr) {
  // The reference thresholds probabilities: torch.sigmoid(logits) > thr (inference.py:72-78).
  // The fp32 sigmoid is monotone non-decreasing in x, so that predicate is exactly
  // "x > cut" for the largest float cut at which it is still false; the masks kernel
  // compares logits against the cut and never evaluates exp.  The cut is bisected with the
  // host libm expf; torch's sigmoid (Sleef on CPU, ocml on ROCm) may round a logit within an
  // ulp or two of the cut differently (tests/test_forward_gpu.py::test_logit_cut_matches_torch_sigmoid).
  const float inf = INFINITY;
  long long lo = float_key(-inf), hi = float_key(inf);
  if (sigmoid_above(-inf, thr)) return -inf;        // every logit passes
  if (!sigmoid_above(inf, thr)) return inf;         // none passes (thr >= 1, or NaN)
  while (hi - lo > 1) {                              // pred(lo) false, pred(hi) true
    const long long mid = lo + (hi - lo) / 2;
    if (sigmoid_above(key_float(mid), thr)) hi = mid; else lo = mid;
  }
  return key_float(lo);
}
int unet_abi_version(void) { return UNET_ABI_VERSION; }

int unet_create(const unet_config* cfg, unet_handle** out) {
  if (!cfg || !out) return fail(UNET_EINVAL, "null argument");
  if (cfg->n_channels != 1 && cfg->n_channels != 3) return fail(UNET_EINVAL, "n_channels must be 1 or 3");
  if (cfg->n_classes < 1 || cfg->n_classes > kMaxClasses) return fail(UNET_EINVAL, "n_classes must be 1..4");
  if (cfg->dtype < 0 || cfg->dtype > UNET_DTYPE_F32_EXACT) return fail(UNET_EINVAL, "bad dtype");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) return fail(UNET_EINVAL, "bad device ordinal");
  unet_handle* h = new unet_handle();
  h->cfg = *cfg;
  const bool f32 = cfg->dtype == UNET_DTYPE_F32 || cfg->dtype == UNET_DTYPE_F32_EXACT;
  // the three-term plan: 2 = the split-once 128-row tiles on the Cout >= 128 layers (x3 = 3), 64-row tiles
  // splitting per tap elsewhere (x3 = 2); 1 = x3 = 2 everywhere; 0 = exact fp32 (UNET_MI355X_F32X3: A/B runs)
  h->f32x3 = cfg->dtype == UNET_DTYPE_F32 ? 2 : 0;
  if (const char* x3 = std::getenv("UNET_MI355X_F32X3")) h->f32x3 = f32 ? std::atoi(x3) : 0;
  h->dt = f32 ? DType::F32 : DType::BF16;   // workspace element size (all 16-bit plans: 2 bytes)
  for (int i = 0; i < kMaxClasses; ++i) h->thr_logit[i] = unet_logit_cut(cfg->thresholds[i]);
  // Kernel configuration per layer (tuned on MI355X).  A/B override for tuning:
  // UNET_MI355X_CFG="layer:cfg,..." (layer = index into L[], cfg = Cfg) and
  // UNET_MI355X_UPCFG="i:cfg,..." (i = 0..3 = up4..up1).
  int cfgs[17], ucfgs[4];
  // the three-term fp32 plan: every 3x3 layer on 64-row 4-wave tiles with pre-split weights (the only halo
  // tile whose two weight slots of three bf16 planes leave two blocks per CU)
  for (int i = 0; i < 17; ++i) cfgs[i] = h->f32x3 ? (int)CFG_HALO_R64_W4 : f32 ? kHaloCfg[i] : kRingCfg[i];
  for (int i = 0; i < 4; ++i) ucfgs[i] = f32 ? (int)CFG_HALO_R128 : (int)CFG_TRING_R256;
  parse_overrides(std::getenv("UNET_MI355X_CFG"), 17, cfgs, [](int, int c) { return cfg_is_halo(c) || cfg_is_ring(c); });
  parse_overrides(std::getenv("UNET_MI355X_UPCFG"), 4, ucfgs, [](int, int c) { return cfg_is_tring(c) || c == CFG_HALO_R128; });
  for (int i = 0; i < 17; ++i) {
    Layer& L = h->L[i];
    L.cin = kLayerCh[i][0];
    L.cout = L.ctot = kLayerCh[i][1];
    L.taps = 9;
    L.dt = L.dto = level_dtype(cfg->dtype, kLayerLevel[i]);
    L.dtq = level_dtype(cfg->dtype, kLayerLevel[i] + 1);
    int c = cfgs[i];
    // keep every layer on a configuration it supports, within the same kernel family (the
    // configurations of a family accumulate in the same K order, so they agree bitwise)
    const bool ring = cfg_is_ring(c);
    if (cfg_fused_in(c) && (i != D1B || f32))   // the same ring family on the other layers
      c = cfg_is_ring8(c) ? (L.cout == 64 ? CFG_RING8_R64_T9 : CFG_RING8_R128)
                          : (L.cout == 64 ? CFG_RING_R64_T3 : CFG_RING_R128);
    if (c == CFG_RING8_R64_WS && (L.cin != 64 || f32)) c = L.cout == 64 ? CFG_RING8_R64_T9 : CFG_RING8_R128;   // 72 KB of weights max
    if (c == CFG_RING8_R128 && (L.cout == 64 || f32)) c = CFG_RING8_R64_T9;   // fp32 128-row 8-wave tiles spill
    if (c == CFG_RING_R64_W12 && f32) c = CFG_RING_R64_T3;   // 16-bit only
    if (cfg_rows(c) > L.cout || (i == C1B && cfg_rows(c) != 64))
      c = ring ? CFG_RING_R64_T3 : CFG_HALO_R64_W8;
    // the LDS-halo family stores its own operand type only: keep it off the mixed plan's seams
    const bool pool = i == D1B || i == D2B || i == D3B || i == D4B;
    if (cfg_is_halo(c) && (L.dto != L.dt || (pool && L.dtq != L.dt))) c = L.cout == 64 || pool ? CFG_RING_R64_T3 : CFG_RING_R128;
    if (c == CFG_RING_R128 && pool) c = CFG_RING_R64_T3;   // pooled 128-row 4-wave tiles spill: same family, 64 rows
    if (h->f32x3 && f32) {   // the three-term plan: pre-split weights; split-once tiles (f32x3 = 2) of 128 rows
                             // x 16x16 pixels where Cout >= 128 and Cin >= 128, 64 rows x 16x32 on conv1.3 (its
                             // head epilogue on whole 32-pixel rows), split per tap on 64-row tiles elsewhere (a
                             // one-block-per-CU tile exposes its prologue and epilogue: short-K layers lose)
#ifndef UNET_X3_ONCE_MIN_CIN
#define UNET_X3_ONCE_MIN_CIN 128
#endif
      const bool once = h->f32x3 == 2 && L.cout % 128 == 0 && L.cin >= UNET_X3_ONCE_MIN_CIN && i != C1B;
      const bool wide = h->f32x3 == 2 && i == C1B;
      c = once ? CFG_HALO_R128 : wide ? CFG_HALO_X3W : CFG_HALO_R64_W4;
      L.x3 = once ? 3 : wide ? 4 : 2;
    }
    L.cfg = c;
  }
  for (int i = 0; i < 4; ++i) {
    Layer& U = h->U[i];
    U.cin = kUpCh[i][0];
    U.cout = kUpCh[i][1];
    U.ctot = 4 * kUpCh[i][1];
    U.taps = 1;
    U.dt = level_dtype(cfg->dtype, kUpLevel[i]);
    U.dto = U.dtq = level_dtype(cfg->dtype, kUpLevel[i] - 1);
    U.cfg = (ucfgs[i] == CFG_HALO_R128 && U.dto != U.dt) ? (int)CFG_TRING_R256 : ucfgs[i];
    if (h->f32x3 && f32) {   // both operands split on the fly on 128-row tiles
      U.cfg = CFG_HALO_R128;
      U.x3 = 1;
      if (h->f32x3 == 2) {   // + the small-batch variant: pre-split weights on 64-row tiles (two blocks per CU)
        h->Us[i] = U;
        h->Us[i].cfg = CFG_HALO_R64_W4;
        h->Us[i].x3 = 2;
      }
    }
  }
  {
    const char* fz = std::getenv("UNET_MI355X_FUSE_UP1");
    const Layer &c2b = h->L[C2B], &u1 = h->U[3];
    h->fuse_up1 = !(fz && fz[0] == '0') && !f32 && (c2b.cfg == CFG_RING_R128 || c2b.cfg == CFG_RING8_R128) &&
                  u1.dt == c2b.dt && u1.dto == c2b.dto;
  }
  if (const char* ks = std::getenv("UNET_MI355X_KSPLIT")) h->ksplit_max = std::atoi(ks);
  if (const char* kf = std::getenv("UNET_MI355X_KSPLIT_FORCE")) {   // "i:ks,..." (A/B runs)
    std::string o(kf);
    size_t pos = 0;
    while (pos < o.size()) {
      size_t end = o.find(',', pos);
      if (end == std::string::npos) end = o.size();
      const std::string item = o.substr(pos, end - pos);
      const size_t colon = item.find(':');
      const int li = colon == std::string::npos ? -1 : std::atoi(item.substr(0, colon).c_str());
      if (li >= 0 && li < 21) h->ksplit_force[li] = std::atoi(item.substr(colon + 1).c_str());
      pos = end + 1;
    }
  }
  build_labels(h);   // after every layer's configuration (3x3 and ConvTranspose) is final
  DeviceGuard g(cfg->device);
  hipError_t e = hipEventCreateWithFlags(&h->done, hipEventDisableTiming);
  if (e != hipSuccess) { delete h; return fail(UNET_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(e)); }
  std::vector<uint8_t> z(4096, 0);   // zero page: conv padding source, + 64 B per K chunk (ring halo cursors)
  int rc = upload(h, &h->zero, z.data(), z.size());
  if (rc) { free_all(h); (void)hipEventDestroy(h->done); delete h; return rc; }
  *out = h;
  return UNET_OK;
}

int unet_load_weights(unet_handle* h, const unet_tensor_view* t, int n) {
  if (!h || (!t && n)) return fail(UNET_EINVAL, "null argument");
  SD sd;
  for (int i = 0; i < n; ++i) {
    if (!t[i].name) return fail(UNET_EINVAL, "tensor without a name");
    sd.m[t[i].name] = &t[i];
  }
  // strict: exactly the reference key set (136 keys for the reference widths)
  const int expected = 9 * 14 + 4 * 2 + 2;
  if ((int)sd.m.size() != expected)
    return fail(UNET_EKEY, "state_dict has " + std::to_string(sd.m.size()) + " keys, expected " +
                               std::to_string(expected));
  DeviceGuard g(h->cfg.device);
  drain(h);   // in-flight forwards may still read the weights about to be freed
  ++h->generation;
  for (void* p : h->allocs)
    if (p != h->zero) (void)hipFree(p);
  h->allocs.assign(1, h->zero);
  h->loaded = false;

  std::vector<double> w, b;
  const int C = h->cfg.n_channels;
  int rc = fold(sd, "down1", "0", C, 64, w, b);
  if (!rc) rc = check_f16_range(h->L[D1B].dt, w, b, "down1.net.0");
  if (rc) return rc;
  {
    std::vector<float> wf(w.begin(), w.end()), bf(b.begin(), b.end());
    rc = upload(h, (void**)&h->w0, wf.data(), wf.size() * 4);
    if (!rc) rc = upload(h, (void**)&h->b0, bf.data(), bf.size() * 4);
    if (rc) return rc;
    h->w0p = nullptr;
    h->w0r = nullptr;
    const DType t0 = h->L[D1B].dt;
    if (t0 != DType::F32) {   // MFMA operand [t][m][16 rows][16 k] (first_conv_mfma_kernel), packed row
      // rho = 16t + r = natural channel natural_of_packed(rho), k = 4q + c <-> tap first_tap(4m + q) (< 9), channel c (< C)
      std::vector<uint8_t> pk;
      pack_first_mfma(t0, w, C, pk);
      rc = upload(h, &h->w0p, pk.data(), pk.size());
      if (rc) return rc;
      // the ring kernel's fused first conv: [cb][t][m][16 rows][16 k], row (cb, t, r) = channel
      // 32cb + 8(r>>2) + 4t + (r&3), k = 4q + c <-> tap first_tap(4m + q) (15 = zero), channel c (< C)
      std::vector<uint8_t> pr((size_t)2 * 2 * 3 * 16 * 16 * 2, 0);
      for (int cb = 0; cb < 2; ++cb)
        for (int tt = 0; tt < 2; ++tt)
          for (int m = 0; m < 3; ++m)
            for (int r = 0; r < 16; ++r) {
              const int o = 32 * cb + 8 * (r >> 2) + 4 * tt + (r & 3);
              for (int q = 0; q < 4; ++q) {
                const int tap = first_tap(4 * m + q);
                if (tap >= 9) continue;
                for (int c = 0; c < C; ++c)
                  put_elem(t0, pr, ((((size_t)(cb * 2 + tt) * 3 + m) * 16 + r) * 16 + 4 * q + c),
                           w[(size_t)o * 9 * C + c * 9 + tap]);
              }
            }
      rc = upload(h, &h->w0r, pr.data(), pr.size());
      if (rc) return rc;
    }
  }
  {   // the 17 3x3 layers (29 M of the 31 M weights): BN fold + range check + packing on host threads,
      // largest layers first; then the uploads in order on this thread (a cold start's ~0.1 s)
    struct Packed { std::vector<uint8_t> w; std::vector<float> b; int rc = UNET_OK; std::string err; };
    std::vector<Packed> pk(17);
    std::vector<int> order(17);
    for (int i = 0; i < 17; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int a, int c) {
      return (long long)h->L[a].cin * h->L[a].cout > (long long)h->L[c].cin * h->L[c].cout;
    });
    auto job = [&](int i) {
      std::vector<double> wl, bl;
      Packed& P = pk[i];
      P.rc = fold(sd, kLayerKey[i][0], kLayerKey[i][1], h->L[i].cin, h->L[i].cout, wl, bl);
      if (!P.rc) P.rc = check_f16_range(h->L[i].dt, wl, bl, std::string(kLayerKey[i][0]) + ".net." + kLayerKey[i][1]);
      if (!P.rc) P.rc = pack3x3_host(h->L[i], wl, P.w);
      if (P.rc) P.err = g_err;   // the worker's own thread-local message
      P.b.assign(bl.begin(), bl.end());
    };
    const int nt = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t)
      pool.emplace_back([&, t]() { for (int k = t; k < 17; k += nt) job(order[k]); });
    for (int k = 0; k < 17; k += nt) job(order[k]);
    for (auto& th : pool) th.join();
    for (int i = 0; i < 17; ++i) {
      if (pk[i].rc) return fail(pk[i].rc, pk[i].err);
      rc = upload(h, &h->L[i].w, pk[i].w.data(), pk[i].w.size());
      if (!rc) rc = upload(h, (void**)&h->L[i].b, pk[i].b.data(), pk[i].b.size() * 4);
      if (rc) return rc;
      std::vector<uint8_t>().swap(pk[i].w);
    }
  }
  std::string err;
  for (int i = 0; i < 4; ++i) {
    const Layer& L = h->U[i];
    const float* W = sd.get(std::string(kUpKey[i]) + ".weight", {L.cin, L.cout, 2, 2}, err);
    const float* B = W ? sd.get(std::string(kUpKey[i]) + ".bias", {L.cout}, err) : nullptr;
    if (!B) return fail(UNET_EKEY, err);
    rc = check_f16_range(L.dt, std::vector<double>(W, W + (size_t)L.cin * L.cout * 4), std::vector<double>(B, B + L.cout),
                         kUpKey[i]);
    if (!rc) rc = packT(h, h->U[i], W, B);
    if (!rc && h->Us[i].x3) rc = packT(h, h->Us[i], W, B);
    if (rc) return rc;
    if (i == 3 && h->fuse_up1) {   // conv2.3 + up1 in one launch
      rc = fold(sd, kLayerKey[C2B][0], kLayerKey[C2B][1], h->L[C2B].cin, h->L[C2B].cout, w, b);
      if (!rc) rc = pack_fused_up(h, h->L[C2B], h->U[3], w, W);
      if (rc) return rc;
    }
  }
  const int ncls = h->cfg.n_classes;
  const float* HW = sd.get("out_conv.weight", {ncls, 64, 1, 1}, err);
  const float* HB = HW ? sd.get("out_conv.bias", {ncls}, err) : nullptr;
  if (!HB) return fail(UNET_EKEY, err);
  // the 16-bit plans' 1x1 head runs on MFMA operands of conv1.3's type (weights rounded in the
  // kernel; the bias stays fp32), so its weights must fit fp16 there too
  rc = check_f16_range(h->L[C1B].dt, std::vector<double>(HW, HW + (size_t)ncls * 64), {}, "out_conv");
  if (!rc) rc = upload(h, (void**)&h->head_w, HW, (size_t)ncls * 64 * 4);
  if (!rc) rc = upload(h, (void**)&h->head_b, HB, (size_t)ncls * 4);
  if (rc) return rc;
  h->loaded = true;
  return UNET_OK;
}

size_t unet_workspace_bytes(const unet_handle* h, int N, int H, int W) {
  if (!h || N <= 0 || H <= 0 || W <= 0) return 0;
  return plan(h, N, H, W).total;
}

int unet_reserve(unet_handle* h, int N, int H, int W) {
  if (!h) return fail(UNET_EINVAL, "null handle");
  int rc = check_geometry(h, N, H, W);
  if (rc) return rc;
  const size_t need = plan(h, N, H, W).total;
  DeviceGuard g(h->cfg.device);
  rc = ensure_box_sync(h, N * h->cfg.n_classes);
  if (rc) return rc;
  if (need <= h->ws_bytes) return UNET_OK;
  ++h->generation;
  if (h->ws) {
    drain(h);   // the old workspace may still be in use by queued forwards
    (void)hipFree(h->ws);
    h->ws = nullptr;
    h->ws_bytes = 0;
  }
  hipError_t e = hipMalloc((void**)&h->ws, need);
  if (e != hipSuccess) {
    h->ws = nullptr;
    return fail(UNET_ENOMEM, std::string("workspace hipMalloc: ") + hipGetErrorString(e));
  }
  h->ws_bytes = need;
  return UNET_OK;
}

namespace {

int run_igemm(unet_handle* h, const Layer& L, int epi, const void* in, int N, int H, int W, int ldi,
              void* out, int ldo, int out_off, void* out2, int ldo2, hipStream_t s,
              float* logits = nullptr, void* masks = nullptr, int mask_kind = MASK_NONE,
              const void* x0 = nullptr) {
  IgemmArgs a{};
  a.in = in;
  a.wgt = L.w;
  a.bias = L.b;
  a.zero = h->zero;
  a.out = out;
  a.out2 = out2;
  a.head_w = h->head_w;
  a.head_b = h->head_b;
  a.logits = logits;
  a.masks = static_cast<uint8_t*>(masks);
  a.N = N; a.H = H; a.W = W;
  a.Cin = L.cin; a.ldi = ldi;
  a.Ctot = L.ctot; a.Cout = L.cout;
  a.ldo = ldo; a.out_off = out_off; a.ldo2 = ldo2;
  a.ncls = h->cfg.n_classes;
  a.mask_kind = mask_kind;
  a.x3 = L.x3;
  if (epi == EPI_UPFUSE) {   // the fused up1's weights, bias and output (the concat buffer's lower half)
    a.wgt = h->wf_c2b;
    a.bias2 = h->U[3].b;
  }
  if (cfg_fused_in(L.cfg)) {
    a.x0 = x0;
    a.w0p = h->w0r;
    a.b0 = h->b0;
    a.c0 = h->cfg.n_channels;
  }
  for (int i = 0; i < kMaxClasses; ++i) a.thr_logit[i] = h->thr_logit[i];
  a.tiles_x = (W + cfg_tile_w(L.cfg) - 1) / cfg_tile_w(L.cfg);
  a.tiles_y = (H + cfg_tile_h(L.cfg) - 1) / cfg_tile_h(L.cfg);
  a.n_ct = L.ctot / cfg_rows(L.cfg);
  const int id = (&L >= h->L && &L < h->L + 17) ? (int)(&L - h->L)
                 : (&L >= h->Us && &L < h->Us + 4) ? 17 + (int)(&L - h->Us) : 17 + (int)(&L - h->U);
  const Split sp = layer_split(h, id, L, epi, N, H, W);
  int cfg = L.cfg;
  if (sp.ks == 1 && sp.rows) {   // small-batch plan, unsplit: finer row tiles over the layer's packing
    a.src_br = cfg_rows(L.cfg);
    a.n_ct = L.ctot / sp.rows;
    if (L.cfg == CFG_TRING_R256) cfg = CFG_TRING_R128;   // the 4-wave 128-row ConvTranspose ring
  }
  if (sp.ks > 1) {   // small-batch plan: K slices into fp32 partials, then the layer's epilogue over their sum
    a.part = static_cast<float*>(h->part);
    a.ksplit = sp.ks;
    if (sp.rows) {   // finer row tiles over the layer's own packing (8-wave ring)
      a.src_br = cfg_rows(L.cfg);
      a.n_ct = L.ctot / sp.rows;
    }
    hipError_t e = launch_igemm(L.dt, L.dt, L.dt, L.cfg, L.taps, EPI_PARTIAL, a, s);
    if (e == hipSuccess) e = launch_splitk_reduce(L.dto, epi == EPI_POOL ? L.dtq : L.dto, epi, a, s);
    if (e != hipSuccess) return fail(UNET_EHIP, std::string("split-K igemm launch: ") + hipGetErrorString(e));
    return UNET_OK;
  }
  hipError_t e = launch_igemm(L.dt, L.dto, epi == EPI_POOL ? L.dtq : L.dto, cfg, L.taps, epi, a, s);
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("igemm launch: ") + hipGetErrorString(e));
  return UNET_OK;
}

// The launch sequence of UNet.forward (unet_model.py:55-86).  ev (optional, kLaunches+1
// events) brackets every launch for per-layer timing.
// x_px4 (the photo graph): x is already the fused first conv's pre-cast input (launch_resample's
// px4 output), so the pre-cast launch is skipped.
int forward_impl(unet_handle* h, const void* x, int x_layout, int x_dtype, void* logits, void* masks,
                 int mask_kind, int32_t* boxes, int N, int H, int W, void* stream, hipEvent_t* ev,
                 bool x_px4 = false) {
  if (!h || !x) return fail(UNET_EINVAL, "null argument");
  if (!h->loaded) return fail(UNET_ESTATE, "weights not loaded");
  if ((x_layout != UNET_LAYOUT_NCHW && x_layout != UNET_LAYOUT_NHWC) || (x_dtype != UNET_IN_F32 && x_dtype != UNET_IN_U8))
    return fail(UNET_EINVAL, "x_layout must be UNET_LAYOUT_NCHW / NHWC and x_dtype UNET_IN_F32 / U8");
  if (mask_kind < 0 || mask_kind > 2) return fail(UNET_EINVAL, "bad mask_kind");
  if (mask_kind != UNET_MASK_NONE && !masks) return fail(UNET_EINVAL, "mask_kind set but masks is NULL");
  int rc = check_geometry(h, N, H, W);
  if (rc) return rc;
  // no allocation (and so no hidden device synchronisation) here: unet_reserve sizes the workspace
  if (plan(h, N, H, W).total > h->ws_bytes)
    return fail(UNET_ESTATE, "workspace too small for this (N, H, W): call unet_reserve first");
  if (boxes && N * h->cfg.n_classes > h->box_sync_n)
    return fail(UNET_ESTATE, "mask-box sync entries too few for this N: call unet_reserve first");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  order_after_last(h, s);
  const Buffers B = plan(h, N, H, W);
  char* ws = h->ws;
  auto buf = [&](size_t off) { return static_cast<void*>(ws + off); };
  if (boxes && (!masks || mask_kind == UNET_MASK_NONE)) {   // boxes only: bit masks into the workspace
    masks = buf(B.mbits);
    mask_kind = UNET_MASK_BITS;
  }
  const int H2 = H / 2, W2 = W / 2, H4 = H / 4, W4 = W / 4, H8 = H / 8, W8 = W / 8, H16 = H / 16, W16 = W / 16;
  const int C = h->cfg.n_channels;

  int li = 0;
  auto mark = [&]() { if (ev) (void)hipEventRecord(ev[li], s); ++li; };
  h->part = buf(B.part);   // split-K partials of the small-batch plan (run_igemm, layer_split)
  mark();
  // down1.net.0 (C -> 64): fused into down1.3 on the 16-bit ring path (fed by the pre-cast input),
  // a direct conv otherwise
  const void* x0 = x;
  if (x_px4 && !cfg_fused_in(h->L[D1B].cfg)) return fail(UNET_EINVAL, "pre-cast input on a plan without the fused first conv");
  if (cfg_fused_in(h->L[D1B].cfg) && !x_px4) {
    hipError_t e = launch_x_to_px4(h->L[D1B].dt, x, x_layout, x_dtype, N, C, H, W, buf(B.xpx), s);
    if (e != hipSuccess) return fail(UNET_EHIP, std::string("input pre-cast launch: ") + hipGetErrorString(e));
    x0 = buf(B.xpx);
  } else if (!x_px4) {
    const float* xf = static_cast<const float*>(x);
    if (x_layout != UNET_LAYOUT_NCHW || x_dtype != UNET_IN_F32) {
      hipError_t e = launch_x_to_nchw_f32(x, x_layout, x_dtype, N, C, H, W, static_cast<float*>(buf(B.xpx)), s);
      if (e != hipSuccess) return fail(UNET_EHIP, std::string("input conversion launch: ") + hipGetErrorString(e));
      xf = static_cast<const float*>(buf(B.xpx));
    }
    FirstConvArgs f{};
    f.x = xf;
    f.w = h->w0;
    f.wp = h->w0p;
    f.b = h->b0;
    f.out = buf(B.tA);
    f.N = N; f.C = C; f.H = H; f.W = W;
    hipError_t e = launch_first_conv(h->L[D1B].dt, f, s);
    if (e != hipSuccess) return fail(UNET_EHIP, std::string("first conv launch: ") + hipGetErrorString(e));
  }

#define RUN(...) do { mark(); rc = run_igemm(__VA_ARGS__); if (rc) return rc; } while (0)
  // encoder: conv b of each level writes the skip into the upper half of the concat
  // buffer (torch.cat([up, skip]) puts skip second, unet_model.py:71) and the pooled map.
  RUN(h, h->L[D1B], EPI_POOL, buf(B.tA), N, H, W, 64, buf(B.cat1), 128, 64, buf(B.p1), 64, s,
      nullptr, nullptr, MASK_NONE, x0);
  RUN(h, h->L[D2A], EPI_STORE, buf(B.p1), N, H2, W2, 64, buf(B.tA), 128, 0, nullptr, 0, s);
  RUN(h, h->L[D2B], EPI_POOL, buf(B.tA), N, H2, W2, 128, buf(B.cat2), 256, 128, buf(B.p2), 128, s);
  RUN(h, h->L[D3A], EPI_STORE, buf(B.p2), N, H4, W4, 128, buf(B.tA), 256, 0, nullptr, 0, s);
  RUN(h, h->L[D3B], EPI_POOL, buf(B.tA), N, H4, W4, 256, buf(B.cat3), 512, 256, buf(B.p3), 256, s);
  RUN(h, h->L[D4A], EPI_STORE, buf(B.p3), N, H8, W8, 256, buf(B.tA), 512, 0, nullptr, 0, s);
  RUN(h, h->L[D4B], EPI_POOL, buf(B.tA), N, H8, W8, 512, buf(B.cat4), 1024, 512, buf(B.p4), 512, s);
  RUN(h, h->L[BNA], EPI_STORE, buf(B.p4), N, H16, W16, 512, buf(B.tA), 1024, 0, nullptr, 0, s);
  RUN(h, h->L[BNB], EPI_STORE, buf(B.tA), N, H16, W16, 1024, buf(B.bnb), 1024, 0, nullptr, 0, s);
  // decoder: up_k writes the lower half of the concat buffer, conv_k reads all of it
  RUN(h, up_layer(h, 0, N), EPI_UPSCATTER, buf(B.bnb), N, H16, W16, 1024, buf(B.cat4), 1024, 0, nullptr, 0, s);
  RUN(h, h->L[C4A], EPI_STORE, buf(B.cat4), N, H8, W8, 1024, buf(B.tA), 512, 0, nullptr, 0, s);
  RUN(h, h->L[C4B], EPI_STORE, buf(B.tA), N, H8, W8, 512, buf(B.tB), 512, 0, nullptr, 0, s);
  RUN(h, up_layer(h, 1, N), EPI_UPSCATTER, buf(B.tB), N, H8, W8, 512, buf(B.cat3), 512, 0, nullptr, 0, s);
  RUN(h, h->L[C3A], EPI_STORE, buf(B.cat3), N, H4, W4, 512, buf(B.tA), 256, 0, nullptr, 0, s);
  RUN(h, h->L[C3B], EPI_STORE, buf(B.tA), N, H4, W4, 256, buf(B.tB), 256, 0, nullptr, 0, s);
  RUN(h, up_layer(h, 2, N), EPI_UPSCATTER, buf(B.tB), N, H4, W4, 256, buf(B.cat2), 256, 0, nullptr, 0, s);
  RUN(h, h->L[C2A], EPI_STORE, buf(B.cat2), N, H2, W2, 256, buf(B.tA), 128, 0, nullptr, 0, s);
  if (h->fuse_up1) {   // conv2.3 + up1 in one launch (EPI_UPFUSE): up1's slot launches nothing
    RUN(h, h->L[C2B], EPI_UPFUSE, buf(B.tA), N, H2, W2, 128, nullptr, 0, 0, buf(B.cat1), 128, s);
    mark();
  } else {
    RUN(h, h->L[C2B], EPI_STORE, buf(B.tA), N, H2, W2, 128, buf(B.tB), 128, 0, nullptr, 0, s);
    RUN(h, up_layer(h, 3, N), EPI_UPSCATTER, buf(B.tB), N, H2, W2, 128, buf(B.cat1), 128, 0, nullptr, 0, s);
  }
  RUN(h, h->L[C1A], EPI_STORE, buf(B.cat1), N, H, W, 128, buf(B.tA), 64, 0, nullptr, 0, s);
  // conv1.net.3 + BN + ReLU + out_conv (1x1) + sigmoid/threshold, one launch
  RUN(h, h->L[C1B], EPI_HEAD, buf(B.tA), N, H, W, 64, nullptr, 0, 0, nullptr, 0, s,
      static_cast<float*>(logits), masks, mask_kind);
#undef RUN
  if (boxes) {   // per-(image, field) mask bounding boxes (inference.py:84-90)
    hipError_t e = launch_mask_boxes(static_cast<const uint8_t*>(masks), mask_kind, N, h->cfg.n_classes, H, W,
                                     boxes, h->box_sync, s);
    if (e != hipSuccess) return fail(UNET_EHIP, std::string("mask boxes launch: ") + hipGetErrorString(e));
  }
  mark();
  mark_done(h, s);
  h->lastN = N; h->lastH = H; h->lastW = W;
  h->last_fused = h->fuse_up1;
  return UNET_OK;
}
}  // namespace

int unet_forward(unet_handle* h, const void* x, int x_layout, int x_dtype, void* logits, void* masks,
                 int mask_kind, int N, int H, int W, void* stream) {
  return forward_impl(h, x, x_layout, x_dtype, logits, masks, mask_kind, nullptr, N, H, W, stream, nullptr);
}

int unet_forward_boxes(unet_handle* h, const void* x, int x_layout, int x_dtype, void* logits, void* masks,
                       int mask_kind, int32_t* boxes, int N, int H, int W, void* stream) {
  if (!boxes) return fail(UNET_EINVAL, "boxes is NULL");
  return forward_impl(h, x, x_layout, x_dtype, logits, masks, mask_kind, boxes, N, H, W, stream, nullptr);
}

int unet_preprocess(unet_handle* h, const void* img, int ih, int iw, int channels, float* x, int oh, int ow,
                    void* stream) {
  if (!h || !img || !x) return fail(UNET_EINVAL, "null argument");
  if (channels != 1 && channels != 3 && channels != 4)
    return fail(UNET_EINVAL, "channels must be 1 (L), 3 (RGB) or 4 (RGBX: Pillow's in-memory RGB, the 4th byte ignored)");
  if (ih <= 0 || iw <= 0 || oh <= 0 || ow <= 0 || (long long)ih * iw > (1LL << 30) || oh > 16384 || ow > 16384)
    return fail(UNET_EINVAL, "bad image or output size");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const auto key = std::make_tuple(ih, iw, oh, ow);
  auto it = h->resample.begin();
  while (it != h->resample.end() && it->first != key) ++it;
  if (it != h->resample.end()) {
    h->resample.splice(h->resample.begin(), h->resample, it);   // most recently used first
  } else {
    if (h->resample.size() >= kResampleCacheMax) {   // evict the least recently used geometry
      drain(h);
      free_resample(h->resample.back().second);
      h->resample.pop_back();
    }
    ResampleStore st;
    const int rc = build_resample(ih, iw, oh, ow, st);
    if (rc) return rc;
    h->resample.emplace_front(key, std::move(st));
    it = h->resample.begin();
  }
  const ResamplePlan& p = it->second.plan;
  const size_t tmp = p.need_h ? (size_t)p.h_rows * ow * channels : 0;
  if (tmp > h->pp_tmp_bytes) {
    if (h->pp_tmp) {
      drain(h);
      (void)hipFree(h->pp_tmp);
      h->pp_tmp = nullptr;
      h->pp_tmp_bytes = 0;
    }
    hipError_t e = hipMalloc((void**)&h->pp_tmp, tmp);
    if (e != hipSuccess) return fail(UNET_ENOMEM, std::string("preprocess buffer: ") + hipGetErrorString(e));
    h->pp_tmp_bytes = tmp;
  }
  order_after_last(h, s);
  hipError_t e = launch_resample(p, static_cast<const uint8_t*>(img), channels, h->pp_tmp, x, s);
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("resample launch: ") + hipGetErrorString(e));
  mark_done(h, s);
  return UNET_OK;
}

int unet_crop_stats(const void* img, int ih, int iw, int channels, const int32_t* boxes, int n_boxes, int box_h,
                    int box_w, double pad, int32_t* rects, uint64_t* sums, void* stream) {
  if (!img || !boxes || !rects || !sums) return fail(UNET_EINVAL, "null argument");
  if (channels != 1 && channels != 3 && channels != 4)
    return fail(UNET_EINVAL, "channels must be 1 (L), 3 (RGB) or 4 (RGBX: Pillow's in-memory RGB, the 4th byte ignored)");
  if (ih <= 0 || iw <= 0 || (long long)ih * iw > (1LL << 30) || box_h <= 0 || box_w <= 0 || n_boxes <= 0 ||
      n_boxes > 65535 || !(pad >= 0.0 && pad < 1.0))
    return fail(UNET_EINVAL, "bad image size, box geometry, box count or pad");
  hipError_t e = launch_crop_stats(static_cast<const uint8_t*>(img), ih, iw, channels, boxes, n_boxes, box_h, box_w,
                                   pad, rects, reinterpret_cast<unsigned long long*>(sums), nullptr,
                                   static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("crop stats launch: ") + hipGetErrorString(e));
  return UNET_OK;
}

int unet_num_launches(void) { return UNET_NUM_LAUNCHES; }

const char* unet_launch_label(const unet_handle* h, int i) {
  if (!h || i < 0 || i >= UNET_NUM_LAUNCHES) return "";
  return h->labels[i].c_str();
}

const char* unet_launch_label_at(const unet_handle* h, int i, int N, int H, int W) {
  thread_local std::string labels[UNET_NUM_LAUNCHES];
  if (!h || i < 0 || i >= UNET_NUM_LAUNCHES || N < 0 || H < 0 || W < 0) return "";
  build_labels_at(h, N, H, W, labels);
  return labels[i].c_str();
}

int unet_small_batch_limit(const unet_handle* h) {
  if (!h) return fail(UNET_EINVAL, "null handle");
  return h->ksplit_max > 1 ? kSmallBatch : 0;
}

int unet_forward_timed(unet_handle* h, const void* x, int x_layout, int x_dtype, void* logits, void* masks,
                       int mask_kind, int N, int H, int W, void* stream, float* launch_ms) {
  if (!h || !launch_ms) return fail(UNET_EINVAL, "null argument");
  DeviceGuard g(h->cfg.device);
  hipEvent_t ev[UNET_NUM_LAUNCHES + 1];
  for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  int rc = forward_impl(h, x, x_layout, x_dtype, logits, masks, mask_kind, nullptr, N, H, W, stream, ev);
  if (!rc) {
    HIP_TRY(hipEventSynchronize(ev[UNET_NUM_LAUNCHES]));
    for (int i = 0; i < UNET_NUM_LAUNCHES; ++i) HIP_TRY(hipEventElapsedTime(&launch_ms[i], ev[i], ev[i + 1]));
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return rc;
}

int unet_debug_fetch(unet_handle* h, const char* name, float* dst, size_t* numel, void* stream) {
  if (!h || !name) return fail(UNET_EINVAL, "null argument");
  if (!h->lastN) return fail(UNET_ESTATE, "no forward has run");
  const int N = h->lastN, H = h->lastH, W = h->lastW;
  const Buffers B = plan(h, N, H, W);
  struct Src { size_t off; int level, C, ld, choff; };
  static const std::map<std::string, int> idx = {
      {"c1", 0}, {"p1", 1}, {"c2", 2}, {"p2", 3}, {"c3", 4}, {"p3", 5}, {"c4", 6}, {"p4", 7},
      {"bn", 8}, {"c7", 9}, {"u1", 10}, {"u2", 11}, {"u3", 12}, {"u4", 13}, {"c8a", 14}};
  auto it = idx.find(name);
  if (it == idx.end()) return fail(UNET_EINVAL, std::string("unknown intermediate ") + name);
  if (it->second == 9 && h->last_fused)
    return fail(UNET_ESTATE, "c7 (conv2.3's output) is not stored when up1 is fused into conv2.3 "
                             "(set UNET_MI355X_FUSE_UP1=0 before creating the handle to keep it)");
  const Src table[] = {{B.cat1, 0, 64, 128, 64},   {B.p1, 1, 64, 64, 0},     {B.cat2, 1, 128, 256, 128},
                       {B.p2, 2, 128, 128, 0},     {B.cat3, 2, 256, 512, 256}, {B.p3, 3, 256, 256, 0},
                       {B.cat4, 3, 512, 1024, 512}, {B.p4, 4, 512, 512, 0},  {B.bnb, 4, 1024, 1024, 0},
                       {B.tB, 1, 128, 128, 0},     {B.cat1, 0, 64, 128, 0},  {B.cat2, 1, 128, 256, 0},
                       {B.cat3, 2, 256, 512, 0},   {B.cat4, 3, 512, 1024, 0}, {B.tA, 0, 64, 64, 0}};
  const Src& t = table[it->second];
  const int h_ = H >> t.level, w_ = W >> t.level;
  const size_t cnt = (size_t)N * t.C * h_ * w_;
  if (numel) *numel = cnt;
  if (!dst) return UNET_OK;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  order_after_last(h, s);
  // each buffer holds its consumer's operand type (the mixed plan: fp16 at levels 0-1)
  hipError_t e = launch_nhwc_to_nchw_f32(level_dtype(h->cfg.dtype, t.level), h->ws + t.off, N, h_, w_, t.C, t.ld,
                                         t.choff, dst, s);
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("debug fetch: ") + hipGetErrorString(e));
  mark_done(h, s);
  return UNET_OK;
}

int unet_graph_create(unet_handle* h, const void* x, int x_layout, int x_dtype, void* logits, void* masks,
                      int mask_kind, int32_t* boxes, int N, int H, int W, unet_graph** out) {
  if (!h || !out) return fail(UNET_EINVAL, "null argument");
  DeviceGuard g(h->cfg.device);
  hipStream_t cs = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  unet_graph* gr = new unet_graph();
  gr->h = h;
  hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
  int rc = UNET_OK;
  if (e != hipSuccess) {
    rc = fail(UNET_EHIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
  } else {
    h->capturing = true;
    rc = boxes ? forward_impl(h, x, x_layout, x_dtype, logits, masks, mask_kind, boxes, N, H, W, cs, nullptr)
               : forward_impl(h, x, x_layout, x_dtype, logits, masks, mask_kind, nullptr, N, H, W, cs, nullptr);
    h->capturing = false;
    e = hipStreamEndCapture(cs, &gr->graph);
    if (!rc && e != hipSuccess) rc = fail(UNET_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    if (!rc) {
      e = hipGraphInstantiate(&gr->exec, gr->graph, nullptr, nullptr, 0);
      if (e != hipSuccess) rc = fail(UNET_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    }
  }
  (void)hipStreamDestroy(cs);
  if (rc) {
    if (gr->exec) (void)hipGraphExecDestroy(gr->exec);
    if (gr->graph) (void)hipGraphDestroy(gr->graph);
    delete gr;
    return rc;
  }
  gr->generation = h->generation;
  *out = gr;
  return UNET_OK;
}

int unet_photo_graph_create(unet_handle* h, const void* h_img, void* img, int ih, int iw, int channels, float* x,
                            int size, void* masks, int mask_kind, int32_t* boxes, double pad, int32_t* rects,
                            uint64_t* sums, void* h_masks, void* h_boxes, void* h_rects, void* h_sums,
                            unet_graph** out) {
  if (!h || !img || !x || !boxes || !rects || !sums || !out) return fail(UNET_EINVAL, "null argument");
  if (channels != 1 && channels != 3 && channels != 4)
    return fail(UNET_EINVAL, "channels must be 1 (L), 3 (RGB) or 4 (RGBX: Pillow's in-memory RGB, the 4th byte ignored)");
  if (ih <= 0 || iw <= 0 || (long long)ih * iw > (1LL << 30) || size <= 0 || size > 16384)
    return fail(UNET_EINVAL, "bad image or network size");
  if (!(pad >= 0.0 && pad < 1.0)) return fail(UNET_EINVAL, "bad pad");
  if (mask_kind < 0 || mask_kind > 2 || (mask_kind != UNET_MASK_NONE && !masks) || (h_masks && mask_kind == UNET_MASK_NONE))
    return fail(UNET_EINVAL, "bad masks / mask_kind");
  int rc = check_geometry(h, 1, size, size);
  if (rc) return rc;
  if (!h->loaded) return fail(UNET_ESTATE, "weights not loaded");
  if (plan(h, 1, size, size).total > h->ws_bytes)
    return fail(UNET_ESTATE, "workspace too small for (1, size, size): call unet_reserve first");
  DeviceGuard g(h->cfg.device);
  unet_graph* gr = new unet_graph();
  gr->h = h;
  // the graph's own resize tables and row buffer (allocated and uploaded before the capture)
  rc = build_resample(ih, iw, size, size, gr->rs);
  const ResamplePlan& p = gr->rs.plan;
  const size_t tmp = p.need_h ? (size_t)p.h_rows * size * channels : 0;
  if (!rc && tmp) {
    hipError_t e = hipMalloc((void**)&gr->pp_tmp, tmp);
    if (e != hipSuccess) rc = fail(UNET_ENOMEM, std::string("preprocess buffer: ") + hipGetErrorString(e));
  }
  const size_t sync_bytes = (size_t)h->cfg.n_classes * kSyncInts * sizeof(int);
  if (!rc) {   // the crop sums' sync entries
    hipError_t e = hipMalloc((void**)&gr->crop_sync, sync_bytes);
    if (e != hipSuccess) rc = fail(UNET_ENOMEM, std::string("crop sync entries: ") + hipGetErrorString(e));
  }
  hipStream_t cs = nullptr;
  if (!rc) {
    hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    if (e != hipSuccess) rc = fail(UNET_EHIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  if (!rc) {   // idle (zero) before the capture: set on the capture stream and waited for, so no replay on any
               // caller stream can start before it (a null-stream memset is asynchronous to the host)
    hipError_t e = hipMemsetAsync(gr->crop_sync, 0, sync_bytes, cs);
    if (e == hipSuccess) e = hipStreamSynchronize(cs);
    if (e != hipSuccess) rc = fail(UNET_EHIP, std::string("crop sync entries: ") + hipGetErrorString(e));
  }
  if (!rc) {
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
      rc = fail(UNET_EHIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
    } else {
      h->capturing = true;
      const size_t img_bytes = (size_t)ih * iw * channels;
      const int ncls = h->cfg.n_classes;
      // on the 16-bit plans with a vertical pass, the resize writes the fused first conv's pre-cast
      // input straight into the workspace (one launch less; x is not written then)
      const bool px4 = cfg_fused_in(h->L[D1B].cfg) && p.need_v;
      void* xin = px4 ? static_cast<void*>(h->ws + plan(h, 1, size, size).xpx) : static_cast<void*>(x);
      if (h_img) e = hipMemcpyAsync(img, h_img, img_bytes, hipMemcpyHostToDevice, cs);   // the photo upload
      if (e == hipSuccess)
        e = launch_resample(p, static_cast<const uint8_t*>(img), channels, gr->pp_tmp, xin, cs,
                            px4 ? h->L[D1B].dt : DType::F32);
      if (e != hipSuccess) rc = fail(UNET_EHIP, std::string("photo graph upload / resize: ") + hipGetErrorString(e));
      if (!rc)
        rc = forward_impl(h, xin, UNET_LAYOUT_NCHW, UNET_IN_F32, nullptr, masks, mask_kind, boxes, 1, size, size, cs,
                          nullptr, px4);
      if (!rc) {
        e = launch_crop_stats(static_cast<const uint8_t*>(img), ih, iw, channels, boxes, ncls, size, size, pad, rects,
                              reinterpret_cast<unsigned long long*>(sums), gr->crop_sync, cs);
        // the copies back, adjacent ones (device and host both contiguous) merged: each copy node
        // costs about 4.5 us, whatever its size
        const size_t mbytes = (size_t)ncls * size * (mask_kind == UNET_MASK_BITS ? size / 8 : size);
        struct Copy { char* dst; const char* src; size_t bytes; };
        std::vector<Copy> copies;
        auto add = [&](void* dst, const void* src, size_t bytes) {
          if (!dst) return;
          char* d = static_cast<char*>(dst);
          const char* sp = static_cast<const char*>(src);
          if (!copies.empty() && copies.back().dst + copies.back().bytes == d && copies.back().src + copies.back().bytes == sp)
            copies.back().bytes += bytes;
          else
            copies.push_back({d, sp, bytes});
        };
        // the masks copy stays a node of its own (never merged): unet_photo_graph_set_masks retargets it
        if (h_masks && e == hipSuccess) {
          e = hipMemcpyAsync(h_masks, masks, mbytes, hipMemcpyDeviceToHost, cs);
          hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
          const hipGraphNode_t* deps = nullptr;
          size_t ndeps = 0;
          if (e == hipSuccess) e = hipStreamGetCaptureInfo_v2(cs, &st, nullptr, nullptr, &deps, &ndeps);
          if (e == hipSuccess && ndeps == 1) {   // the node just captured
            gr->masks_node = deps[0];
            gr->masks_dst = h_masks;
            gr->masks_src = masks;
            gr->masks_bytes = mbytes;
          }
        }
        add(h_boxes, boxes, (size_t)ncls * 16);
        add(h_rects, rects, (size_t)ncls * 16);
        add(h_sums, sums, (size_t)ncls * 8);
        for (const Copy& c : copies)
          if (e == hipSuccess) e = hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost, cs);
        if (e != hipSuccess) rc = fail(UNET_EHIP, std::string("photo graph crop stats / copies: ") + hipGetErrorString(e));
      }
      h->capturing = false;
      e = hipStreamEndCapture(cs, &gr->graph);
      if (!rc && e != hipSuccess) rc = fail(UNET_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
      if (!rc) {
        e = hipGraphInstantiate(&gr->exec, gr->graph, nullptr, nullptr, 0);
        if (e != hipSuccess) rc = fail(UNET_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
      }
    }
  }
  if (cs) (void)hipStreamDestroy(cs);
  if (rc) {
    (void)unet_graph_destroy(gr);
    return rc;
  }
  gr->generation = h->generation;
  *out = gr;
  return UNET_OK;
}

int unet_photo_graph_set_masks(unet_graph* gr, void* h_masks) {
  if (!gr || !gr->exec || !h_masks) return fail(UNET_EINVAL, "null argument");
  if (!gr->masks_node) return fail(UNET_ESTATE, "graph has no retargetable masks copy (not a photo graph with h_masks)");
  if (h_masks == gr->masks_dst) return UNET_OK;
  DeviceGuard g(gr->h->cfg.device);
  // the next replay copies into h_masks; launches already enqueued keep their destination
  hipError_t e = hipGraphExecMemcpyNodeSetParams1D(gr->exec, gr->masks_node, h_masks, gr->masks_src, gr->masks_bytes,
                                                   hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("hipGraphExecMemcpyNodeSetParams1D: ") + hipGetErrorString(e));
  gr->masks_dst = h_masks;
  return UNET_OK;
}

int unet_graph_launch(unet_graph* gr, void* stream) {
  if (!gr || !gr->exec) return fail(UNET_EINVAL, "null graph");
  unet_handle* h = gr->h;
  if (gr->generation != h->generation)
    return fail(UNET_ESTATE, "graph is stale: the handle's weights or workspace were re-allocated after capture");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  order_after_last(h, s);
  HIP_TRY(hipGraphLaunch(gr->exec, s));
  mark_done(h, s);
  return UNET_OK;
}

int unet_graph_destroy(unet_graph* gr) {
  if (!gr) return UNET_OK;
  DeviceGuard g(gr->h->cfg.device);
  drain(gr->h);
  if (gr->exec) (void)hipGraphExecDestroy(gr->exec);
  if (gr->graph) (void)hipGraphDestroy(gr->graph);
  free_resample(gr->rs);
  if (gr->pp_tmp) (void)hipFree(gr->pp_tmp);
  if (gr->crop_sync) (void)hipFree(gr->crop_sync);
  delete gr;
  return UNET_OK;
}

int unet_comm_get_unique_id(void* id) {
  if (!id) return fail(UNET_EINVAL, "null argument");
  const Rccl* r = rccl();
  if (!r) return fail(UNET_EHIP, "RCCL (librccl.so) could not be loaded");
  NcclId nid;
  const int rc = r->get_unique_id(&nid);
  if (rc) return rccl_fail(r, rc, "ncclGetUniqueId");
  std::memcpy(id, &nid, sizeof nid);
  return UNET_OK;
}

int unet_comm_init(unet_handle* h, int rank, int nranks, const void* id) {
  if (!h || !id) return fail(UNET_EINVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(UNET_EINVAL, "bad rank / nranks");
  if (h->comm) return fail(UNET_ESTATE, "communicator already initialised");
  const Rccl* r = rccl();
  if (!r) return fail(UNET_EHIP, "RCCL (librccl.so) could not be loaded");
  DeviceGuard g(h->cfg.device);
  NcclId nid;
  std::memcpy(&nid, id, sizeof nid);
  const int rc = r->comm_init_rank(&h->comm, nranks, nid, rank);
  if (rc) { h->comm = nullptr; return rccl_fail(r, rc, "ncclCommInitRank"); }
  return UNET_OK;
}

int unet_allgather(unet_handle* h, const void* send, void* recv, size_t bytes_per_rank, void* stream) {
  if (!h || !send || !recv) return fail(UNET_EINVAL, "null argument");
  if (!h->comm) return fail(UNET_ESTATE, "no communicator: call unet_comm_init first");
  const Rccl* r = rccl();
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  order_after_last(h, s);   // e.g. after this rank's forward on another stream
  const int rc = r->all_gather(send, recv, bytes_per_rank, /*ncclUint8*/ 1, h->comm, s);
  if (rc) return rccl_fail(r, rc, "ncclAllGather");
  mark_done(h, s);
  return UNET_OK;
}

int unet_comm_destroy(unet_handle* h) {
  if (!h || !h->comm) return UNET_OK;
  DeviceGuard g(h->cfg.device);
  drain(h);
  const Rccl* r = rccl();
  const int rc = r ? r->comm_destroy(h->comm) : 0;
  h->comm = nullptr;
  return rc ? rccl_fail(r, rc, "ncclCommDestroy") : UNET_OK;
}

int unet_destroy(unet_handle* h) {
  if (!h) return UNET_OK;
  {
    DeviceGuard g(h->cfg.device);
    if (h->comm) (void)unet_comm_destroy(h);
    free_all(h);
    if (h->done) (void)hipEventDestroy(h->done);
  }
  delete h;
  return UNET_OK;
}

// ---------------------------------------------------------------------------------
// Stand-alone DoubleConv (unet_model.py:6-20): conv3x3 + BN + ReLU twice on an NCHW fp32 tensor,
// on the network's own kernels (the first-conv kernel for 1 / 3 input channels, the 8-wave rings on
// the 16-bit plans, the LDS-halo kernels on fp32), no split-K.
// ---------------------------------------------------------------------------------
}  // extern "C"

struct unet_block {
  unet_handle core;     // allocations, zero page, stream order; the two convs in core.L[0], core.L[1]
  int cin = 0, cout = 0;
  bool first = false;   // cin in {1, 3}: conv a is the first-conv kernel (64 outputs)
};

namespace {
struct BlockBuffers { size_t in, mid, out, total; };
BlockBuffers block_plan(const unet_block* b, int N, int H, int W) {
  const size_t e = dtype_size(b->core.L[1].dt), P = (size_t)N * H * W;
  BlockBuffers r{};
  size_t o = 0;
  r.in = o;
  if (!b->first) o = align256(o + P * b->cin * e);
  r.mid = o;
  o = align256(o + P * b->cout * e);
  r.out = o;
  o = align256(o + P * b->cout * e);
  r.total = o;
  return r;
}
int block_geometry(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return fail(UNET_EINVAL, "N, H, W must be positive");
  if ((long long)N * H * W > (1LL << 30)) return fail(UNET_ESHAPE, "N*H*W too large for one call");
  return UNET_OK;
}
}  // namespace

extern "C" {

int unet_block_create(const unet_block_config* cfg, unet_block** out) {
  if (!cfg || !out) return fail(UNET_EINVAL, "null argument");
  const int cin = cfg->in_ch, cout = cfg->out_ch;
  if (cfg->dtype < 0 || cfg->dtype > UNET_DTYPE_F32_EXACT) return fail(UNET_EINVAL, "bad dtype");
  const bool first = cin == 1 || cin == 3;
  if (cout <= 0 || cout % 64 || (first && cout != 64) || (!first && (cin <= 0 || cin % 32)))
    return fail(UNET_ESHAPE, "DoubleConv(in_ch, out_ch) runs natively for in_ch in {1, 3} with out_ch = 64, or in_ch "
                             "a multiple of 32 and out_ch a multiple of 64 (every block of the reference UNet)");
  const bool f32 = cfg->dtype == UNET_DTYPE_F32 || cfg->dtype == UNET_DTYPE_F32_EXACT;
  if (!f32 && cout != 64 && cout % 128)   // the 16-bit rings tile 64 or 128-row groups
    return fail(UNET_ESHAPE, "DoubleConv(in_ch, out_ch) on the 16-bit plans needs out_ch = 64 or a multiple of 128 "
                             "(the 128-row MFMA ring tiles); fp32 takes any multiple of 64");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) return fail(UNET_EINVAL, "bad device ordinal");
  unet_block* b = new unet_block();
  b->cin = cin;
  b->cout = cout;
  b->first = first;
  unet_handle& h = b->core;
  h.cfg.n_channels = first ? cin : 3;
  h.cfg.n_classes = 1;
  h.cfg.dtype = cfg->dtype;
  h.cfg.device = cfg->device;
  h.ksplit_max = 0;
  h.f32x3 = cfg->dtype == UNET_DTYPE_F32;
  if (const char* x3 = std::getenv("UNET_MI355X_F32X3")) h.f32x3 = f32 && std::atoi(x3) != 0;   // A/B runs
  // the mixed plan's storage type at this block's resolution level in the reference network: fp16 up to
  // 128 channels (levels 0-1), bf16 beyond (levels 2-4)
  const DType t = f32 ? DType::F32 : cfg->dtype == UNET_DTYPE_F16 ? DType::F16 : cfg->dtype == UNET_DTYPE_BF16 ? DType::BF16
                : (cout <= 128 ? DType::F16 : DType::BF16);
  h.dt = f32 ? DType::F32 : DType::BF16;
  for (int i = 0; i < 2; ++i) {
    Layer& L = h.L[i];
    L.cin = i == 0 ? cin : cout;
    L.cout = L.ctot = cout;
    L.taps = 9;
    L.dt = L.dto = L.dtq = t;
    if (f32 && h.f32x3) {   // the three-term fp32 plan (as the network's layers)
      L.cfg = CFG_HALO_R64_W4;
      L.x3 = 2;
    } else if (f32) L.cfg = cout == 64 ? CFG_HALO_R64_W8 : CFG_HALO_R128;
    else L.cfg = cout == 64 ? (L.cin == 64 ? CFG_RING8_R64_WS : CFG_RING8_R64_T9) : CFG_RING8_R128;
  }
  DeviceGuard g(cfg->device);
  hipError_t e = hipEventCreateWithFlags(&h.done, hipEventDisableTiming);
  if (e != hipSuccess) { delete b; return fail(UNET_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(e)); }
  std::vector<uint8_t> z(4096, 0);
  int rc = upload(&h, &h.zero, z.data(), z.size());
  if (rc) { free_all(&h); (void)hipEventDestroy(h.done); delete b; return rc; }
  *out = b;
  return UNET_OK;
}

int unet_block_load_weights(unet_block* b, const unet_tensor_view* t, int n) {
  if (!b || (!t && n)) return fail(UNET_EINVAL, "null argument");
  SD sd;
  std::vector<std::string> names(n);
  for (int i = 0; i < n; ++i) {
    if (!t[i].name) return fail(UNET_EINVAL, "tensor without a name");
    names[i] = std::string("b.") + t[i].name;   // fold() reads <block>.net.<i>.*
  }
  for (int i = 0; i < n; ++i) sd.m[names[i]] = &t[i];
  if ((int)sd.m.size() != 14)   // net.{0,3}.{weight,bias} + net.{1,4}.{weight,bias,running_mean,running_var,num_batches_tracked}
    return fail(UNET_EKEY, "DoubleConv state_dict has " + std::to_string(sd.m.size()) + " keys, expected 14");
  unet_handle& h = b->core;
  DeviceGuard g(h.cfg.device);
  drain(&h);
  ++h.generation;
  for (void* p : h.allocs)
    if (p != h.zero) (void)hipFree(p);
  h.allocs.assign(1, h.zero);
  h.loaded = false;
  std::vector<double> w, bb;
  int rc = fold(sd, "b", "0", b->cin, b->cout, w, bb);
  if (!rc) rc = check_f16_range(h.L[0].dt, w, bb, "net.0");
  if (rc) return rc;
  if (b->first) {
    std::vector<float> wf(w.begin(), w.end()), bf(bb.begin(), bb.end());
    rc = upload(&h, (void**)&h.w0, wf.data(), wf.size() * 4);
    if (!rc) rc = upload(&h, (void**)&h.b0, bf.data(), bf.size() * 4);
    h.w0p = nullptr;
    if (!rc && h.L[0].dt != DType::F32) {
      std::vector<uint8_t> pk;
      pack_first_mfma(h.L[0].dt, w, b->cin, pk);
      rc = upload(&h, &h.w0p, pk.data(), pk.size());
    }
  } else {
    rc = pack3x3(&h, h.L[0], w, bb);
  }
  if (rc) return rc;
  rc = fold(sd, "b", "3", b->cout, b->cout, w, bb);
  if (!rc) rc = check_f16_range(h.L[1].dt, w, bb, "net.3");
  if (!rc) rc = pack3x3(&h, h.L[1], w, bb);
  if (rc) return rc;
  h.loaded = true;
  return UNET_OK;
}

int unet_block_reserve(unet_block* b, int N, int H, int W) {
  if (!b) return fail(UNET_EINVAL, "null block");
  int rc = block_geometry(N, H, W);
  if (rc) return rc;
  unet_handle& h = b->core;
  const size_t need = block_plan(b, N, H, W).total;
  if (need <= h.ws_bytes) return UNET_OK;
  DeviceGuard g(h.cfg.device);
  ++h.generation;
  if (h.ws) {
    drain(&h);
    (void)hipFree(h.ws);
    h.ws = nullptr;
    h.ws_bytes = 0;
  }
  hipError_t e = hipMalloc((void**)&h.ws, need);
  if (e != hipSuccess) {
    h.ws = nullptr;
    return fail(UNET_ENOMEM, std::string("block workspace hipMalloc: ") + hipGetErrorString(e));
  }
  h.ws_bytes = need;
  return UNET_OK;
}

int unet_block_forward(unet_block* b, const float* x, float* y, int N, int H, int W, void* stream) {
  if (!b || !x || !y) return fail(UNET_EINVAL, "null argument");
  unet_handle& h = b->core;
  if (!h.loaded) return fail(UNET_ESTATE, "weights not loaded");
  int rc = block_geometry(N, H, W);
  if (rc) return rc;
  const BlockBuffers B = block_plan(b, N, H, W);
  if (B.total > h.ws_bytes) return fail(UNET_ESTATE, "workspace too small for this (N, H, W): call unet_block_reserve first");
  DeviceGuard g(h.cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  order_after_last(&h, s);
  const DType t = h.L[1].dt;
  void* mid = h.ws + B.mid;
  void* outb = h.ws + B.out;
  hipError_t e = hipSuccess;
  if (b->first) {
    FirstConvArgs f{};
    f.x = x;
    f.w = h.w0;
    f.wp = h.w0p;
    f.b = h.b0;
    f.out = mid;
    f.N = N; f.C = b->cin; f.H = H; f.W = W;
    e = launch_first_conv(t, f, s);
    if (e != hipSuccess) return fail(UNET_EHIP, std::string("block first conv launch: ") + hipGetErrorString(e));
  } else {
    e = launch_nchw_to_nhwc(t, x, N, b->cin, H, W, h.ws + B.in, s);
    if (e != hipSuccess) return fail(UNET_EHIP, std::string("block input transpose: ") + hipGetErrorString(e));
    rc = run_igemm(&h, h.L[0], EPI_STORE, h.ws + B.in, N, H, W, b->cin, mid, b->cout, 0, nullptr, 0, s);
    if (rc) return rc;
  }
  rc = run_igemm(&h, h.L[1], EPI_STORE, mid, N, H, W, b->cout, outb, b->cout, 0, nullptr, 0, s);
  if (rc) return rc;
  e = launch_nhwc_to_nchw(t, outb, N, b->cout, H, W, y, s);
  if (e != hipSuccess) return fail(UNET_EHIP, std::string("block output transpose: ") + hipGetErrorString(e));
  mark_done(&h, s);
  return UNET_OK;
}

int unet_block_destroy(unet_block* b) {
  if (!b) return UNET_OK;
  {
    DeviceGuard g(b->core.cfg.device);
    free_all(&b->core);
    if (b->core.done) (void)hipEventDestroy(b->core.done);
  }
  delete b;
  return UNET_OK;
}

}  // extern "C"

