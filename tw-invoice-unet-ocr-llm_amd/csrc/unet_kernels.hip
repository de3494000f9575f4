// HIP kernels for the UNet forward path on MI355X (gfx950 / CDNA4).
//
// Reference semantics: unet_model.py:6-86 (DoubleConv = conv3x3 -> BN(eval) -> ReLU
// twice; MaxPool2d(2); ConvTranspose2d(k2, s2); torch.cat([up, skip], 1); 1x1 out_conv).
//
// Design:
//  * activations are NHWC in HBM (bf16 / f16 / f32), so one pixel's channel run is a
//    contiguous 128-byte row of a GEMM operand;
//  * every 3x3 conv, the ConvTranspose2d and the fused 1x1 head run through ONE
//    implicit-GEMM kernel: rows = output channels (A = pre-packed, BN-folded weights),
//    columns = output pixels (B = the shifted NHWC input gathered per tap),
//    K = (tap, cin).  Tiles are staged global -> LDS with global_load_lds_dwordx4
//    (LDS-DMA, no VGPR round trip); conv zero padding comes from a zero page so the
//    DMA never needs a mask; the LDS image is XOR-swizzled through the per-lane
//    source address (lane-linear destination) so the ds_read_b128 fragment reads are
//    bank-conflict free;
//  * MFMA v_mfma_f32_16x16x32_{bf16,f16} (f32: v_mfma_f32_16x16x4_f32, exact fp32);
//  * epilogues: bias (BN folded) + ReLU; fused 2x2 max-pool (the skip tensor and
//    the pooled tensor are written by the same launch); fused 64->ncls 1x1 head with
//    sigmoid/threshold masks; ConvTranspose pixel-shuffle scatter.  torch.cat is
//    zero-copy: producers write straight into channel halves of one NHWC buffer.
#include "unet_internal.h"

#include <algorithm>
#include <type_traits>

namespace unet {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef int frag_t __attribute__((ext_vector_type(4)));   // one 16-byte MFMA operand fragment

// (ablation builds encode cfg = base + 16 * ablation; the helpers describe the base)
int cfg_rows(int cfg) {
  switch (cfg % 16) {
    case CFG_HALO_R128: case CFG_RING_R128: case CFG_TRING_R128: case CFG_RING8_R128: return 128;
    case CFG_TRING_R256: return 256;
    default: return 64;
  }
}
bool cfg_is_halo(int cfg) {
  return cfg == CFG_HALO_R64_W4 || cfg == CFG_HALO_R64_W8 || cfg == CFG_HALO_R128 || cfg == CFG_HALO_X3W;
}
bool cfg_is_ring(int cfg) {
  cfg %= 16;
  return cfg == CFG_RING_R128 || cfg == CFG_RING_R64_T3 || cfg == CFG_RING_FUSED_IN || cfg == CFG_RING8_R128 ||
         cfg == CFG_RING8_R64_T9 || cfg == CFG_RING8_R64_WS || cfg == CFG_RING8_FUSED_IN || cfg == CFG_RING_R64_W12;
}
bool cfg_is_ring8(int cfg) {
  cfg %= 16;
  return cfg == CFG_RING8_R128 || cfg == CFG_RING8_R64_T9 || cfg == CFG_RING8_R64_WS || cfg == CFG_RING8_FUSED_IN;
}
int cfg_tile_w(int cfg) {
  return (cfg_is_ring8(cfg) || cfg % 16 == CFG_RING_R64_W12 || cfg == CFG_HALO_X3W) ? 32 : 16;
}
int cfg_tile_h(int cfg) { return cfg % 16 == CFG_RING_R64_W12 ? 12 : 16; }
bool cfg_fused_in(int cfg) { return cfg % 16 == CFG_RING_FUSED_IN || cfg % 16 == CFG_RING8_FUSED_IN; }
int ring_ns(int cfg) { return cfg % 16 == CFG_RING_R64_W12 ? 4 : (cfg % 16 == CFG_RING8_R64_T9 ? 2 : 3); }
int ring_tps(int cfg) {
  cfg %= 16;
  if (cfg == CFG_RING8_R64_T9) return 9;
  return (cfg == CFG_RING_R64_T3 || cfg == CFG_RING_FUSED_IN || cfg == CFG_RING8_R128 || cfg == CFG_RING8_R64_WS ||
          cfg == CFG_RING8_FUSED_IN) ? 3 : 1;
}
int cfg_limit() {
#ifdef UNET_ABLATION
  return CFG_COUNT + 16 * 10;
#else
  return CFG_RING_R64_W12;   // the configurations after it are ablation-build only
#endif
}
bool cfg_is_tring(int cfg) { return cfg == CFG_TRING_R128 || cfg == CFG_TRING_R256; }

// ---------------------------------------------------------------------------------
// element traits
// ---------------------------------------------------------------------------------
template <typename T> struct Elem;
template <> struct Elem<float> { static constexpr int BKE = 32; };   // 32 f32 = 128 B
template <> struct Elem<__bf16> { static constexpr int BKE = 64; };  // 64 bf16 = 128 B
template <> struct Elem<_Float16> { static constexpr int BKE = 64; };

template <typename T>
__device__ __forceinline__ void mfma_frag(f32x4& acc, const uint4& a, const uint4& b);

template <>
__device__ __forceinline__ void mfma_frag<__bf16>(f32x4& acc, const uint4& a, const uint4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma_frag<_Float16>(f32x4& acc, const uint4& a, const uint4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                               __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
}
// f32: the 16-byte fragment holds 4 consecutive k of one row; four 16x16x4 MFMAs, the
// e-th one taking element e of every lane.  A and B read the same (row, chunk) map, so
// this is the same dot product in a permuted (exact fp32 fma-chain) order.
template <>
__device__ __forceinline__ void mfma_frag<float>(f32x4& acc, const uint4& a, const uint4& b) {
  const f32x4 av = __builtin_bit_cast(f32x4, a);
  const f32x4 bv = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], acc, 0, 0, 0);
}

// 16x16x16 MFMA (K = 16: 4 values of 2 bytes per lane), the fused first conv's shape
template <typename T>
__device__ __forceinline__ f32x4 mfma16(const uint2& a, const uint2& b, const f32x4& c);
template <>
__device__ __forceinline__ f32x4 mfma16<__bf16>(const uint2& a, const uint2& b, const f32x4& c) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4, a), __builtin_bit_cast(s4, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16<_Float16>(const uint2& a, const uint2& b, const f32x4& c) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4, a), __builtin_bit_cast(h4, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16<float>(const uint2&, const uint2&, const f32x4& c) { return c; }   // unused

// fp32 as three bf16 terms (the fp32 plan's arithmetic on the bf16 MFMA pipe): x = hi + mid + lo with
// hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (round to nearest even; each difference is
// exact in fp32), so hi + mid + lo carries x's 24-bit significand.  A product of two split values is
// sum_{i+j<=2} a_i b_j (6 bf16 products, exact in the fp32 MFMA accumulator) up to terms below 2^-24 of
// |a b|: fp32 accuracy (unet_model.py:10,14 in fp32) at 6 MFMAs of 16x16x32 (6 x 16 cycles) where the
// exact-fp32 path needs 8 of 16x16x4 f32 (8 x 32 cycles) for the same 32 K.  x0, x1: the 8 fp32 K values of
// this lane (two 16-byte fragments); A and B are split with the same K order.
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {   // v_cvt_pk_bf16_f32 (RNE), lo in bits 0..15
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}
__device__ __forceinline__ void split3_bf16(const frag_t& x0, const frag_t& x1, frag_t& h, frag_t& m, frag_t& l) {
#ifdef UNET_ABL_X3_NOSPLIT   // timing-only ablation build: no split arithmetic (operand bits reused as terms)
  h = x0;
  m = x1;
  l = x0;
  return;
#endif
  // per pair of values: one v_cvt_pk_bf16_f32 per term and the two halves widened back with a shift / a
  // mask (11 VALU per pair; the element-wise form compiled to ~14 with single-value conversions)
  const f32x4 a = __builtin_bit_cast(f32x4, x0), b = __builtin_bit_cast(f32x4, x1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float v0 = i < 2 ? a[2 * i] : b[2 * i - 4], v1 = i < 2 ? a[2 * i + 1] : b[2 * i - 3];
    const uint32_t hp = cvt_pk_bf16(v0, v1);
    const float r0 = v0 - __uint_as_float(hp << 16), r1 = v1 - __uint_as_float(hp & 0xffff0000u);
    const uint32_t mp = cvt_pk_bf16(r0, r1);
    const float s0 = r0 - __uint_as_float(mp << 16), s1 = r1 - __uint_as_float(mp & 0xffff0000u);
    h[i] = (int)hp;
    m[i] = (int)mp;
    l[i] = (int)cvt_pk_bf16(s0, s1);
  }
}
__device__ __forceinline__ void mfma_bf16(f32x4& acc, const frag_t& a, const frag_t& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}

// torch semantics of ReLU / MaxPool2d: a NaN propagates (unet_model.py:12,16,34).  One
// v_maximum3_f32 (IEEE-754-2019 maximum) each; fmaxf would turn a NaN into the other operand.
__device__ __forceinline__ float relu_nan(float x) { return __builtin_elementwise_maximum(x, 0.f); }
__device__ __forceinline__ float max_nan(float a, float b) { return __builtin_elementwise_maximum(a, b); }

// store 16 consecutive channels (fp32 values) as element type T (16-byte vector stores)
template <typename T>
__device__ __forceinline__ void store16(T* dst, const float (&v)[16]);
template <>
__device__ __forceinline__ void store16<float>(float* dst, const float (&v)[16]) {
  f32x4* d = reinterpret_cast<f32x4*>(dst);
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
}
template <>
__device__ __forceinline__ void store16<__bf16>(__bf16* dst, const float (&v)[16]) {
  bf16x8 lo, hi;
#pragma unroll
  for (int i = 0; i < 8; ++i) { lo[i] = (__bf16)v[i]; hi[i] = (__bf16)v[8 + i]; }
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = __builtin_bit_cast(uint4, lo);
  d[1] = __builtin_bit_cast(uint4, hi);
}
template <>
__device__ __forceinline__ void store16<_Float16>(_Float16* dst, const float (&v)[16]) {
  f16x8 lo, hi;
#pragma unroll
  for (int i = 0; i < 8; ++i) { lo[i] = (_Float16)v[i]; hi[i] = (_Float16)v[8 + i]; }
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = __builtin_bit_cast(uint4, lo);
  d[1] = __builtin_bit_cast(uint4, hi);
}

// A 64-channel group of one pixel (128 B in NHWC) leaves the MFMA layout spread over the four
// lane rows q (16 channels each), so two plain 16-byte stores per lane write 64 scattered
// 16-byte pieces per instruction.  One v_permlane32_swap per dword pair regroups them: after
// it, lane row q holds channels 8*perm(q) .. +7 and 32 + 8*perm(q) .. +7 (perm = 0, 16, 8, 24 /
// 8), so each of the two store instructions writes one contiguous, 64-byte aligned 64-byte run
// per pixel: 16 full segments per instruction instead of 64 partial ones.  (Time-neutral on
// MI355X, profiles/tune_r2_stores.txt: the no-store ablation's apparent gain was the higher
// clock of MFMAs on all-zero operands, not store cost.)  `grp` = channel 0 of the 64-row group.
__device__ __forceinline__ int swz_store_off(int q) { return 8 * ((q & 1) * 2 + (q >> 1)); }
template <typename T>
__device__ __forceinline__ void store64_grouped(T* grp, const float (&v)[16]) {
  if constexpr (sizeof(T) == 4) {
    store16<T>(grp + 16 * ((threadIdx.x & 63) >> 4), v);
  } else {
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 lo, hi;
#pragma unroll
    for (int i = 0; i < 8; ++i) { lo[i] = (T)v[i]; hi[i] = (T)v[8 + i]; }
    uint4 x = __builtin_bit_cast(uint4, lo), y = __builtin_bit_cast(uint4, hi);
    uint4 xs, ys;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane32_swap(x[i], y[i], false, false);
      xs[i] = r[0];
      ys[i] = r[1];
    }
    T* dst = grp + swz_store_off((threadIdx.x & 63) >> 4);
    *reinterpret_cast<uint4*>(dst) = xs;
    *reinterpret_cast<uint4*>(dst + 32) = ys;
  }
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4): lane l's bytes land at
// lds_dst + 16*l.  Issued from inline asm on purpose: hipcc would otherwise treat every
// later ds_read as aliasing the in-flight DMA and drain vmcnt(0) in front of it, which
// serialises the load of step s+2 behind the compute of step s.  The waits are ours
// (counted vmcnt before each barrier); M0 is saved/restored inside the statement.  No
// "memory" clobber: the DMA never targets an LDS slot read in the same step, and the
// barriers (volatile asm + memory clobber) keep it inside its step.
__device__ __forceinline__ void glds16(const void* src, char* lds_dst) {
  const uint32_t lds_addr = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)lds_dst)));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_addr));
}

// The same with the LDS destination given as a wave-uniform 32-bit LDS address (an SGPR value:
// the LDS array's base + offsets built from scalars).  glds16 derives it from a generic pointer
// per call -- a 64-bit VALU add, two v_readfirstlane and the generic -> LDS null check in front of
// every DMA; the 8-wave and ConvTranspose rings issue 4-6 DMAs per wave and step (round 3).
__device__ __forceinline__ void glds16_s(const void* src, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_addr)));
}
// The saddr form: lane l's 16 bytes come from sbase + voff, a wave-uniform 64-bit base in SGPRs plus a
// 32-bit per-lane offset.  A stream whose per-lane pattern is fixed (the packed weight pieces) then
// advances by scalar adds only, instead of a 64-bit VALU add per piece (round 4).
__device__ __forceinline__ void glds16_sv(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(sbase);
  // (readfirstlane returns int: each half goes through uint32_t, so the low half is not sign-extended)
  const unsigned long long ub =
      ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32)) << 32) |
      (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(ub), "s"(__builtin_amdgcn_readfirstlane(lds_addr)));
}
// LDS address of a __shared__ object (a constant for the kernel's one LDS array)
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)p));
}

// Pixel p (0..BP-1) of a block tile -> (row, col) inside the TH x 16 tile.  Pixels come
// in groups of 16 = 2 rows x 8 columns, so an MFMA column group (lane & 15) covers whole
// 2x2 pooling windows: partners are lanes ^1 and ^8.
__device__ __forceinline__ void pix_of(int p, int& py, int& px) {
  const int g = p >> 4, j = p & 15;
  py = 2 * (g >> 1) + (j >> 3);
  px = 8 * (g & 1) + (j & 7);
}
// the same for a 16 x TW tile (TW / 8 column groups per row pair)
template <int TW>
__device__ __forceinline__ void pix_of_w(int p, int& py, int& px) {
  const int g = p >> 4, j = p & 15;
  py = 2 * (g / (TW / 8)) + (j >> 3);
  px = 8 * (g % (TW / 8)) + (j & 7);
}

// ---------------------------------------------------------------------------------
// shared epilogue
// ---------------------------------------------------------------------------------
// Lane holds, for pixel column (lane & 15) of each p tile, the 16 consecutive natural
// rows rbase .. rbase+15 (the weight packing permutes rows so that MFMA row
// 4*(lane>>4)+e of row-tile t is natural row 16*(lane>>4) + 4*t + e).
// Pixel p of the wave = group (g0 + p) of the block tile whose origin is (oy0, ox0).
// Cross-lane helpers on the VALU (gfx950): DPP for intra-row moves, permlane swaps for
// the lane^16 / lane^32 exchanges.  Both avoid the LDS crossbar that __shfl_xor uses.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float xsum_lane16(float x) {   // x[l] + x[l ^ 16]
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum_lane32(float x) {   // x[l] + x[l ^ 32]
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// TO: element type of the NHWC output (and of the ConvTranspose scatter), TQ: of the pooled map
// (the two differ where a layer feeds consumers of different storage type, see unet_capi.cpp).
// up_out (EPI_UPSCATTER only): scatter into up_out (pixel stride up_ldo, channel offset 0, up_cout
// channels per (a, b) group) instead of a.out / a.ldo / a.out_off / a.Cout (EPI_UPFUSE).
// EPI_HEAD: conv1.3 + BN + ReLU kept in fp32, the 64 -> ncls 1x1 out_conv as per-lane FMA chains
// summed over the wave's four row quads with permlane16/32 swaps (VALU, no LDS round trip), then
// the logits and / or masks (sigmoid > thr as logit > the host-bisected cut).  Round 3 (the
// per-layer no-epilogue ablation put this epilogue at 29 % of conv1.3, profiles/
// tune_r3g_epilogue_ablation.txt): the 1x1 weights are read once per tile instead of per pixel
// group and class (each read was waited for right before its dot), every class is computed
// without a branch (classes >= ncls have zero weights here), the mask kind is resolved once per
// tile (one straight-line loop per kind), and bit-packed masks of a full 16 x 32 tile leave as one
// dword per (class, row): the wave's TP = 4 pixel groups are one row pair x 32 columns, so each
// class's ballots assemble into two 32-bit row words in scalar registers.  Same arithmetic per
// logit (fmaf order, swaps, + bias), so bitwise the same logits and masks.
//
// HT = _Float16 / __bf16 (the 16-bit plans, round 3): the 1x1 dot runs on two v_mfma_f32_16x16x32
// per 16-pixel group instead of 48 FMAs + 6 swaps per lane: A = the head weights (16 rows = classes,
// rows >= ncls zero), B = the ReLU outputs rounded to HT, fp32 accumulation, the bias added in fp32.
// A lane's 16 channels (16q + 4t + e) are B's K slots 8q + j of MFMA h = t / 2 (v[8h + j]), so A's
// K slot 8kq + j of MFMA h is channel 16kq + 8h + j; the logit of class c < 4 lands in lane (pixel,
// q = 0) element c -- the lanes the stores and ballots below read.  Rounding the head's operands to
// fp16 leaves the bench pages' masks unchanged (tools/numerics_emulate.py --head fp16: IoU min
// 0.99945 either way); HT = float (the fp32 plan) keeps the exact fp32 FMA chains.
template <int TP, int TW, int BACC, typename HT = float>
__device__ __forceinline__ void head_epilogue(const IgemmArgs& a, const f32x4 (&acc)[4][TP], int n, int oy0, int ox0,
                                              int g0, const float (&bv)[16], const float* head_w,
                                              const float* head_b) {
  constexpr bool MH = sizeof(HT) == 2;
  static_assert(!MH || kMaxClasses <= 4, "MFMA head: the classes are the 4 rows of lane group q = 0");
  const int H = a.H, W = a.W;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4;
  const int col = lane & 15;
  const int ncls = a.ncls;
  float hw[MH ? 1 : kMaxClasses][16], hb[kMaxClasses], cut[kMaxClasses];
  uint4 haf[2];   // MH: the A fragments (row = class col, K group q) of the two MFMAs
#pragma unroll
  for (int c = 0; c < kMaxClasses; ++c) {
    const bool live = c < ncls;   // wave-uniform
    hb[c] = live ? head_b[c] : 0.f;
    cut[c] = a.thr_logit[c];
    if constexpr (!MH) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 w4 = live ? *reinterpret_cast<const f32x4*>(head_w + c * 64 + q * 16 + 4 * i)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
        hw[c][4 * i] = w4[0]; hw[c][4 * i + 1] = w4[1]; hw[c][4 * i + 2] = w4[2]; hw[c][4 * i + 3] = w4[3];
      }
    }
  }
  if constexpr (MH) {
    typedef HT h8 __attribute__((ext_vector_type(8)));
    const bool live = col < ncls;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      h8 w;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 w4 = live ? *reinterpret_cast<const f32x4*>(head_w + col * 64 + 16 * q + 8 * h + 4 * i)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) w[4 * i + e] = (HT)w4[e];
      }
      haf[h] = __builtin_bit_cast(uint4, w);
    }
  }
  auto logits_of = [&](int p, float (&logit)[kMaxClasses]) {
    float v[16];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[t * 4 + e] = relu_nan(BACC ? acc[t][p][e] : acc[t][p][e] + bv[t * 4 + e]);
    if constexpr (MH) {
      typedef HT h8 __attribute__((ext_vector_type(8)));
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        h8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = (HT)v[8 * h + j];
        mfma_frag<HT>(d, haf[h], __builtin_bit_cast(uint4, b));
      }
#pragma unroll
      for (int c = 0; c < kMaxClasses; ++c) logit[c] = d[c] + hb[c];   // valid in lanes q = 0
    } else {
#pragma unroll
      for (int c = 0; c < kMaxClasses; ++c) {
        float sum = 0.f;
        if (c < ncls) {   // wave-uniform: a dead class costs a scalar branch, not 16 FMAs + 2 swaps
#pragma unroll
          for (int e = 0; e < 16; ++e) sum = fmaf(hw[c][e], v[e], sum);
          sum = xsum_lane16(sum);
          sum = xsum_lane32(sum);
        }
        logit[c] = sum + hb[c];
      }
    }
  };
  auto pixel = [&](int p, int& oy, int& ox) {
    int py, px;
    pix_of_w<TW>((g0 + p) * 16 + col, py, px);
    oy = oy0 + py;
    ox = ox0 + px;
  };
  const long long plane = (long long)H * W;
  float* const lg = a.logits;
  if (a.mask_kind == MASK_BITS && TW == 32 && TP == 4 && (W & 31) == 0 && ox0 + 32 <= W && (g0 & 3) == 0) {
    unsigned w0[kMaxClasses], w1[kMaxClasses];
#pragma unroll
    for (int c = 0; c < kMaxClasses; ++c) w0[c] = w1[c] = 0u;
#pragma unroll
    for (int p = 0; p < TP; ++p) {
      float logit[kMaxClasses];
      logits_of(p, logit);
      int oy, ox;
      pixel(p, oy, ox);
#pragma unroll
      for (int c = 0; c < kMaxClasses; ++c) {
        // group p = bits 8p .. 8p+7 of the pair's row words (lanes q = 0: row col >> 3, column col & 7)
        const unsigned long long bal = __ballot(logit[c] > cut[c]);
        w0[c] |= ((unsigned)bal & 0xFFu) << (8 * p);
        w1[c] |= ((unsigned)(bal >> 8) & 0xFFu) << (8 * p);
        if (lg && c < ncls && q == 0 && oy < H) lg[(long long)(n * ncls + c) * plane + (long long)oy * W + ox] = logit[c];
      }
    }
    const int oy = oy0 + 2 * (g0 / (TW / 8)) + lane;   // lane r < 2 stores row r of the wave's row pair
    if (lane < 2 && oy < H) {
#pragma unroll
      for (int c = 0; c < kMaxClasses; ++c)
        if (c < ncls)
          *reinterpret_cast<unsigned*>(a.masks + ((long long)(n * ncls + c) * H + oy) * (W >> 3) + (ox0 >> 3)) =
              lane ? w1[c] : w0[c];
    }
    return;
  }
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    float logit[kMaxClasses];
    logits_of(p, logit);
    int oy, ox;
    pixel(p, oy, ox);
    const bool inside = oy < H && ox < W;
#pragma unroll
    for (int c = 0; c < kMaxClasses; ++c) {
      if (c >= ncls) break;
      const long long pix = (long long)(n * ncls + c) * plane + (long long)oy * W + ox;
      if (lg && q == 0 && inside) lg[pix] = logit[c];
      const bool on = logit[c] > cut[c];
      if (a.mask_kind == MASK_U8) {
        if (q == 0 && inside) a.masks[pix] = on ? 1 : 0;
      } else if (a.mask_kind == MASK_BITS) {
        const unsigned long long bal = __ballot(on);
        if (q == 0 && (col & 7) == 0 && inside)
          a.masks[((long long)(n * ncls + c) * H + oy) * (W >> 3) + (ox >> 3)] = (uint8_t)((bal >> (col & 8)) & 0xFFu);
      }
    }
  }
}

// BACC = 1: the accumulators already hold the bias (the 8-wave ring starts every tile's
// accumulators at the bias instead of zero, init_acc_bias), so no bias add here.
template <typename TO, typename TQ, int TP, int EPI, int TW = 16, int NOSTORE = 0, int BACC = 0>
__device__ __forceinline__ void conv_epilogue(const IgemmArgs& a, const f32x4 (&acc)[4][TP], int n, int oy0,
                                              int ox0, int g0, int row0, const float* bias_w,
                                              const float* head_w, const float* head_b,
                                              void* up_out = nullptr, int up_ldo = 0, int up_cout = 0) {
  // bias_w: bias of this wave's 64 rows (global or LDS); head_w: [ncls][64] with the
  // wave's 64 rows at +0 (EPI_HEAD only, single 64-row tile); head_b: [ncls]
  constexpr int TC = 4;
  const int H = a.H, W = a.W;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4;
  const int col = lane & 15;
  float bv[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 b4 = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!BACC) b4 = *reinterpret_cast<const f32x4*>(bias_w + q * 16 + 4 * i);
    bv[4 * i] = b4[0]; bv[4 * i + 1] = b4[1]; bv[4 * i + 2] = b4[2]; bv[4 * i + 3] = b4[3];
  }
  if constexpr (EPI == EPI_HEAD && !NOSTORE) {
    head_epilogue<TP, TW, BACC, TO>(a, acc, n, oy0, ox0, g0, bv, head_w, head_b);
    return;
  }

#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of_w<TW>((g0 + p) * 16 + col, py, px);
    const int oy = oy0 + py, ox = ox0 + px;
    const bool inside = oy < H && ox < W;
    float v[16];
#pragma unroll
    for (int t = 0; t < TC; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = BACC ? acc[t][p][e] : acc[t][p][e] + bv[t * 4 + e];
        if (EPI != EPI_UPSCATTER) x = relu_nan(x);
        v[t * 4 + e] = x;
      }
    if constexpr (NOSTORE == 2 && sizeof(TO) == 2 && (EPI == EPI_STORE || EPI == EPI_POOL)) {
      // ablation builds: the stores alone (zeros to the same addresses, no arithmetic)
      if (inside) {
        TO* d = reinterpret_cast<TO*>(a.out) + ((long long)(n * H + oy) * W + ox) * a.ldo + a.out_off + row0 +
                swz_store_off(q);
        *reinterpret_cast<uint4*>(d) = uint4{0u, 0u, 0u, 0u};
        *reinterpret_cast<uint4*>(d + 32) = uint4{0u, 0u, 0u, 0u};
      }
      if constexpr (EPI == EPI_POOL) {
        if ((col & 9) == 0 && oy + 1 < H && ox + 1 < W) {
          TQ* d = reinterpret_cast<TQ*>(a.out2) + ((long long)(n * (H >> 1) + (oy >> 1)) * (W >> 1) + (ox >> 1)) * a.ldo2 +
                  row0 + swz_store_off(q);
          *reinterpret_cast<uint4*>(d) = uint4{0u, 0u, 0u, 0u};
          *reinterpret_cast<uint4*>(d + 32) = uint4{0u, 0u, 0u, 0u};
        }
      }
    } else if constexpr (NOSTORE) {   // ablation builds: the epilogue arithmetic without its stores
#pragma unroll
      for (int e = 0; e < 16; ++e) asm volatile("" ::"v"(v[e]));
      if constexpr (EPI == EPI_POOL) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float o = max_nan(v[e], dpp_f32<0xB1>(v[e]));
          asm volatile("" ::"v"(max_nan(o, dpp_f32<0x128>(o))));
        }
      }
    } else if constexpr (EPI == EPI_STORE || EPI == EPI_POOL) {
      if (inside) {
        TO* grp = reinterpret_cast<TO*>(a.out) + ((long long)(n * H + oy) * W + ox) * a.ldo + a.out_off + row0;
        store64_grouped<TO>(grp, v);
      }
      if constexpr (EPI == EPI_POOL) {
        float m[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          // 2x2 window partners are lanes ^1 (quad_perm [1,0,3,2]) and ^8 (row_ror:8).  The values
          // are ReLU outputs (+0 .. +inf or NaN), whose fp32 order is their unsigned bit-pattern
          // order, NaN (either sign) above all: an unsigned max with the DPP move folded into it
          // (one v_max_u32_dpp per partner) is MaxPool2d's max with its NaN propagation.
          const unsigned u = __float_as_uint(v[e]);
          const unsigned o = max(u, (unsigned)__builtin_amdgcn_update_dpp(0, (int)u, 0x128, 0xF, 0xF, true));
          m[e] = __uint_as_float(max(o, (unsigned)__builtin_amdgcn_update_dpp(0, (int)o, 0xB1, 0xF, 0xF, true)));
        }
        if ((col & 9) == 0 && oy + 1 < H && ox + 1 < W) {
          const int Ho = H >> 1, Wo = W >> 1;
          TQ* grp = reinterpret_cast<TQ*>(a.out2) + ((long long)(n * Ho + (oy >> 1)) * Wo + (ox >> 1)) * a.ldo2 + row0;
          store64_grouped<TQ>(grp, m);   // (lane rows q of one column are all anchors or none)
        }
      }
    } else if constexpr (EPI == EPI_UPSCATTER) {
      if (inside) {
        const int cout = up_out ? up_cout : a.Cout;
        const int ab = row0 / cout;   // a 64-row group lies in one (a, b) quadrant (Cout % 64 == 0)
        const int o0 = row0 - ab * cout;
        const int Y = 2 * oy + (ab >> 1), X = 2 * ox + (ab & 1);
        TO* grp = up_out ? reinterpret_cast<TO*>(up_out) + ((long long)(n * 2 * H + Y) * (2 * W) + X) * up_ldo + o0
                         : reinterpret_cast<TO*>(a.out) + ((long long)(n * 2 * H + Y) * (2 * W) + X) * a.ldo + a.out_off + o0;
        store64_grouped<TO>(grp, v);
      }
    }   // EPI_HEAD: head_epilogue above
  }
}

// EPI_PARTIAL (split-K, small batches): the lane's 16 natural rows row0 + 16q .. + 15 of each of its
// TP pixels (acc[t][p][e] = row 16q + 4t + e) as fp32 into slice `slice` of a.part: four 16-byte
// stores per pixel, 256 contiguous bytes per pixel and 64-row group across the four lane rows.
template <int TP, int TW>
__device__ __forceinline__ void partial_store(const IgemmArgs& a, const f32x4 (&acc)[4][TP], int n, int oy0, int ox0,
                                              int g0, int row0, int slice) {
  const int lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  const long long P = (long long)a.N * a.H * a.W;
  float* base = a.part + (long long)slice * P * a.Ctot + row0 + 16 * q;
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of_w<TW>((g0 + p) * 16 + col, py, px);
    const int oy = oy0 + py, ox = ox0 + px;
    if (oy < a.H && ox < a.W) {
      f32x4* d = reinterpret_cast<f32x4*>(base + ((long long)(n * a.H + oy) * a.W + ox) * a.Ctot);
#pragma unroll
      for (int t = 0; t < 4; ++t) d[t] = acc[t][p];
    }
  }
}


// ---------------------------------------------------------------------------------
// 3x3 conv with an LDS halo tile (the fp32 path; 128-byte K chunks)
// ---------------------------------------------------------------------------------
// Block = BR output channels x a 16x16 output-pixel tile.  Per 128-byte input chunk (32 f32 /
// 64 bf16 channels) the block stages the 18x18 input halo ONCE into LDS; the nine taps then
// read shifted windows of it, so the activation operand is fetched from L2 once per chunk
// instead of nine times.  Weights stream through an NS-slot ring, NS-1 K-steps ahead.  All
// staging is LDS-DMA (global_load_lds_dwordx4) with counted vmcnt waits, so loads stay in
// flight across the per-step barrier.  One halo buffer, two blocks per CU: the other block
// covers this one's exposed halo load and epilogue.
//
// LDS: [halo][w slot 0 .. NS-1][bias/head params]; halo pixel (hy,hx) -> row hy*18+hx
// (128 B), 16-byte chunk c stored at c ^ (hx & 7): conflict-free ds_read_b128 for every tap
// (the 18-pixel row stride breaks the usual row&7 swizzle).  Weight rows: c ^ (row & 7).
// KT = 3: 3x3 conv (18x18 halo, 9 taps); KT = 1: the same pipeline as a plain GEMM over a
// 16x16 pixel tile (ConvTranspose2d k2 s2 on the fp32 path: K = Cin, rows = (a, b, cout),
// EPI_UPSCATTER).
constexpr int kNumCUs = 256;          // MI355X: 8 XCDs x 32 CUs

// s_waitcnt vmcnt(N) lgkmcnt(0) + s_barrier.  The wait goes through the builtin (not asm) so
// hipcc's waitcnt tracker knows every LDS read is retired here and does not re-wait for
// them after the barrier; the empty asm statements keep memory operations from moving across.
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));   // vmcnt(N) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// NT consecutive taps of one ring step (no barrier between them) with the fragment reads of tap
// k+1 issued under the MFMAs of tap k (register double buffering): only the first tap's LDS read
// latency is exposed.  Without it every tap opened with a full read -> wait -> MFMA bubble,
// which the partner wave of a SIMD covers only when it is not in the same phase -- never true
// right after a barrier of the 8-wave ring, whose two waves per SIMD belong to ONE block.
// hs[k]: halo fragment base of tap k (+ prow[p] per pixel group), ws[k]: weight row base of tap
// k (+ t * 1 KB per 16-row group).  Same MFMA sequence per accumulator as one tap at a time.
// mid (optional): work issued after the first tap's MFMAs -- the step's LDS-DMA issue, which then
// runs while those MFMAs execute instead of in front of the step's first fragment reads (round 3).
struct NoMid { __device__ void operator()() const {} };
template <typename T, int TC, int TP, int NT, typename Mid = NoMid>
__device__ __forceinline__ void mfma_taps(f32x4 (&acc)[TC][TP], const char* const (&hs)[NT],
                                          const char* const (&ws)[NT], const int (&prow)[TP], Mid mid = Mid{}) {
  constexpr int NR = TC + TP, NM = TC * TP;
  static_assert(NM % NR == 0, "read / MFMA interleave");
  frag_t fa[2][TC], fb[2][TP];
  auto load = [&](int k, int b) {
#pragma unroll
    for (int p = 0; p < TP; ++p) fb[b][p] = *reinterpret_cast<const frag_t*>(hs[k] + prow[p]);
#pragma unroll
    for (int t = 0; t < TC; ++t) fa[b][t] = *reinterpret_cast<const frag_t*>(ws[k] + t * 16 * 64);
  };
  load(0, 0);
  __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const int b = k & 1;
    if (k + 1 < NT) load(k + 1, b ^ 1);
#pragma unroll
    for (int t = 0; t < TC; ++t)
#pragma unroll
      for (int p = 0; p < TP; ++p)
        mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, fa[b][t]), __builtin_bit_cast(uint4, fb[b][p]));
    if (k + 1 < NT) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, NM / NR, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    } else {
      __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
    }
    if (k == 0) mid();   // after the first tap's MFMAs (and the next tap's reads) are issued
  }
}

// The same for wide row tiles (TC = 8: 8 A + 4 B fragments per tap would need 96 registers
// double-buffered): the A fragments of all NT taps form ONE stream through a 3-register ring two
// row groups ahead (crossing tap boundaries), and only the TP B fragments are double-buffered --
// tap k+1's are read under the first TP row groups of tap k.
// ABL (ablation builds only, timing): 2 = the fragment reads without the MFMAs, 3 = the MFMAs on
// register fragments without the LDS reads.
template <typename T, int TC, int TP, int NT, int ABL = 0, typename Mid = NoMid>
__device__ __forceinline__ void mfma_taps_astream(f32x4 (&acc)[TC][TP], const char* const (&hs)[NT],
                                                  const char* const (&ws)[NT], const int (&prow)[TP], Mid mid = Mid{}) {
  static_assert(TC >= TP && TC >= 3, "B prefetch spread over the row groups");
  frag_t ar[3], fb[2][TP];
  frag_t rf = {};   // ABL 3: one real fragment per call (MFMAs on zeros would run at a higher clock)
  if constexpr (ABL == 3) rf = *reinterpret_cast<const frag_t*>(hs[0] + prow[0]);
  auto ldsread = [&](const char* p) {
    if constexpr (ABL == 3) {
      frag_t v = rf;
      asm volatile("" : "+v"(v));
      return v;
    } else {
      return *reinterpret_cast<const frag_t*>(p);
    }
  };
  auto lda = [&](int j) { return ldsread(ws[j / TC] + (j % TC) * 16 * 64); };
#pragma unroll
  for (int p = 0; p < TP; ++p) fb[0][p] = ldsread(hs[0] + prow[p]);
  ar[0] = lda(0);
  ar[1] = lda(1);
  __builtin_amdgcn_sched_group_barrier(0x100, TP + 2, 0);
#pragma unroll
  for (int k = 0; k < NT; ++k) {
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      const int j = k * TC + t;
      if (j + 2 < NT * TC) ar[(j + 2) % 3] = lda(j + 2);
      if (k + 1 < NT && t < TP) fb[(k + 1) & 1][t] = ldsread(hs[k + 1] + prow[t]);
      const frag_t af = ar[j % 3];
#pragma unroll
      for (int p = 0; p < TP; ++p) {
        if constexpr (ABL == 2) asm volatile("" ::"v"(af), "v"(fb[k & 1][p]));
        else mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, fb[k & 1][p]));
      }
      if (j + 2 < NT * TC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (k + 1 < NT && t < TP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TP, 0);
      if (j == 1) mid();   // after the first two row groups' MFMAs
    }
  }
}

// Derived geometry / LDS budget of a halo-kernel instantiation (shared with the launcher).
template <typename T, int WR, int WPX, int TCW, int NS, int KT, int X3 = 0>
struct HaloGeom {
  static constexpr int NW = WR * WPX;
  static constexpr int TC = TCW;
  static constexpr int TP = 16 / WPX;               // 16-pixel groups per wave (16 per tile)
  static constexpr int BR = WR * 16 * TC;
  static constexpr int BKE = Elem<T>::BKE;
  static constexpr int PAD = KT == 3 ? 1 : 0;
  static constexpr int HWD = 16 + 2 * PAD;          // halo width = height
  static constexpr int NPIX = HWD * HWD;
  static constexpr int NTAP = KT * KT;
  static constexpr int HI = (NPIX + 8 * NW - 1) / (8 * NW);   // halo DMA instructions per wave (at most)
  // X3 = 2: a step's weights as three bf16 planes (hi, mid, lo) of BR rows x 64 B (unet_capi.cpp pack3x3_split);
  // the halo's 1 KB DMA pieces are dealt over the waves round-robin, only as many as the halo needs (NI),
  // so that three weight slots fit beside it at two blocks per CU
  static constexpr int WSLOT = X3 == 2 ? 3 * BR * 64 : BR * 128;
  static constexpr int WI = X3 == 2 ? WSLOT / (1024 * NW) : BR / (8 * NW);   // weight DMA instructions per wave
  static constexpr int NI = (NPIX + 7) / 8;                    // halo DMA pieces (X3 = 2)
  static constexpr int HALO_BYTES = X3 == 2 ? NI * 1024 : HI * NW * 8 * 128;
  static constexpr int WOFF = HALO_BYTES;
  static constexpr int PARAM_OFF = WOFF + NS * WSLOT;
  static constexpr int LDS_BYTES = PARAM_OFF + (BR + kMaxClasses * 64 + kMaxClasses) * 4;
};

// X3 (fp32 only): the fp32 operands as three bf16 terms (split3_bf16), 6 bf16 MFMAs per 32-K block instead of
// 8 exact-fp32 ones, same epilogues.  X3 = 1: both operands split on the fly (same LDS images and weight
// packing as the fp32 kernel; the ConvTranspose at larger batches).  X3 = 2: the weights come pre-split from
// the packing as three bf16 planes per step (no VALU for A, which the block's waves share), the activations
// are split on the fly per fragment (the short-K 3x3 layers, the batch-1 ConvTranspose).
template <typename T, int WR, int WPX, int TCW, int NS, int KT, int EPI, int X3 = 0>
__global__ __launch_bounds__(64 * WR * WPX, 2 * WR * WPX / 4) void conv3x3_halo_kernel(const IgemmArgs a) {
  using G = HaloGeom<T, WR, WPX, TCW, NS, KT, X3>;
  constexpr int NW = G::NW, TC = G::TC, TP = G::TP, BR = G::BR, BKE = G::BKE;
  constexpr int HWD = G::HWD, NPIX = G::NPIX, NTAP = G::NTAP, PAD = G::PAD;
  constexpr int HI = G::HI, WI = G::WI, WSLOT = G::WSLOT, WOFF = G::WOFF;
  static_assert(NS == 2 || NS == 3, "weight ring depth");
  static_assert(WI >= 1 && BR % (8 * NW) == 0, "weight tile split");
  static_assert(G::LDS_BYTES <= 160 * 1024 / 2, "two blocks per CU");
  __shared__ __attribute__((aligned(16))) char lds[G::LDS_BYTES];
  float* bias_s = reinterpret_cast<float*>(lds + G::PARAM_OFF);
  float* headw_s = bias_s + BR;
  float* headb_s = headw_s + kMaxClasses * 64;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wr = wave / WPX;
  const int wp = wave % WPX;

  int bid;
  {  // XCD-contiguous remap; consecutive ids = the n_ct row tiles of one pixel tile
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7;
    const int b = blockIdx.x, x = b & 7, k = b >> 3;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  // EPI_PARTIAL: block = (row tile, K slice, pixel tile); the slice covers Cin chunks c_lo .. c_lo + nch
  constexpr bool PART = EPI == EPI_PARTIAL;
  const int KS = PART ? a.ksplit : 1;
  const int ct = bid % a.n_ct;
  int mt = bid / a.n_ct;
  const int kslice = PART ? mt % KS : 0;
  if (PART) mt /= KS;
  const int tx = mt % a.tiles_x;
  mt /= a.tiles_x;
  const int ty = mt % a.tiles_y;
  const int n = mt / a.tiles_y;
  if (n >= a.N) return;

  const int H = a.H, W = a.W;
  const int K = NTAP * a.Cin;
  const int nch = a.Cin / BKE / KS;
  const int c_lo = kslice * nch;
  const int S = NTAP * nch;

  const int w_chk = ((lane & 7) ^ ((lane >> 3) & 7)) * 16;
  const char* wbase = reinterpret_cast<const char*>(a.wgt) +
                      (size_t)(ct * BR + wave * WI * 8 + (lane >> 3)) * K * sizeof(T) + w_chk;
  const size_t wstep = (size_t)8 * K * sizeof(T);   // 8 rows per DMA instruction
  const char* in = reinterpret_cast<const char*>(a.in);
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const long long pix0 = (long long)(n * H + ty * 16) * W + tx * 16;

  auto issue_halo = [&](int c) {
    constexpr bool RR = X3 == 2;   // round-robin pieces, NI in all
    char* dst = lds + wave * HI * 8 * 128;
    const long long c0 = (long long)c * BKE;
#pragma unroll
    for (int j = 0; j < HI; ++j) {
      const int piece = RR ? j * NW + wave : wave * HI + j;
      if (RR && piece >= G::NI) break;
      if constexpr (RR) dst = lds + (piece - j) * 1024;       // + j KB below
      const int row = piece * 8 + (lane >> 3);
      const int hy = row / HWD, hx = row - hy * HWD;
      const int iy = ty * 16 + hy - PAD, ix = tx * 16 + hx - PAD;
      const bool ok = row < NPIX && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const int chk = ((lane & 7) ^ (hx & 7)) * 16;
      const long long pix = pix0 + (long long)(hy - PAD) * W + (hx - PAD);
      const char* src = ok ? in + (pix * a.ldi + c0) * (long long)sizeof(T) + chk : zero + chk;
      glds16(src, dst + j * 8 * 128);
    }
  };
  auto issue_w = [&](int g) {   // K step g = (chunk, tap) of the slice, weights [row][tap*Cin + c]
    if constexpr (X3 == 2) {   // [ct][step][3][BR][64 B]: one contiguous block per step, 1 KB per DMA instruction
      constexpr int WJ = WI;
      static_assert(WSLOT % (1024 * NW) == 0, "pre-split weight slot split");
      const long long step = (long long)ct * (NTAP * (a.Cin / BKE)) + (long long)c_lo * NTAP + g;
      const char* src = reinterpret_cast<const char*>(a.wgt) + step * WSLOT + (wave * WJ) * 1024 + lane * 16;
      char* dst = lds + WOFF + (g % NS) * WSLOT + wave * WJ * 1024;
#pragma unroll
      for (int j = 0; j < WJ; ++j) glds16(src + j * 1024, dst + j * 1024);
    } else {
      const int c = c_lo + g / NTAP, tap = g - (g / NTAP) * NTAP;
      const size_t koff = ((size_t)tap * a.Cin + (size_t)c * BKE) * sizeof(T);
      char* dst = lds + WOFF + (g % NS) * WSLOT + wave * WI * 8 * 128;
#pragma unroll
      for (int j = 0; j < WI; ++j) glds16(wbase + koff + j * wstep, dst + j * 8 * 128);
    }
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int t = 0; t < TC; ++t)
#pragma unroll
    for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int col = lane & 15, q = lane >> 4;
  int prow[TP];
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of((wp * TP + p) * 16 + col, py, px);
    prow[p] = py * HWD + px;
  }
  const int px_lane = col & 7;

  issue_halo(c_lo);
  issue_w(0);
  if (NS == 3 && S > 1) issue_w(1);
  // epilogue parameters into LDS with plain loads, issued after the first DMAs so the two
  // latencies overlap (their vmcnt(0) also covers the DMAs; the barrier publishes them)
  for (int i = tid; i < BR; i += 64 * NW) bias_s[i] = a.bias[ct * BR + i];
  if (EPI == EPI_HEAD) {
    for (int i = tid; i < a.ncls * 64; i += 64 * NW) headw_s[i] = a.head_w[i];
    if (tid < a.ncls) headb_s[tid] = a.head_b[tid];
  }
  if (NS == 3 && S > 1) wait_vm_barrier<WI>(); else wait_vm_barrier<0>();

  auto read_frags = [&](int g, int tp, int kk, frag_t (&af)[TC], frag_t (&bf)[TP]) {
    const int dy = tp / KT, dx = tp - (tp / KT) * KT;
    const char* Ws = lds + WOFF + (g % NS) * WSLOT + (wr * 16 * TC + col) * 128;
    const int toff = dy * HWD + dx;
    const int hx7 = (px_lane + dx) & 7;
    const int chunk = kk * 4 + q;
#pragma unroll
    for (int t = 0; t < TC; ++t)
      af[t] = *reinterpret_cast<const frag_t*>(Ws + t * 16 * 128 + ((chunk ^ (lane & 7)) << 4));
#pragma unroll
    for (int p = 0; p < TP; ++p)
      bf[p] = *reinterpret_cast<const frag_t*>(lds + (prow[p] + toff) * 128 + ((chunk ^ hx7) << 4));
  };
  auto mfmas = [&](const frag_t (&af)[TC], const frag_t (&bf)[TP]) {
#pragma unroll
    for (int t = 0; t < TC; ++t)
#pragma unroll
      for (int p = 0; p < TP; ++p)
        mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, af[t]), __builtin_bit_cast(uint4, bf[p]));
  };

  // X3: the step's 32 K as one 16x16x32 block per fragment pair -- lane (col, q) holds K chunks q and
  // 4 + q (the kk = 0 and 1 fragments of read_frags), for A and B alike
  auto x3_step = [&](int g, int tp) {
    static_assert(X3 == 0 || sizeof(T) == 4, "X3 splits fp32 operands");
    const char* hal = lds;
    const int dy = tp / KT, dx = tp - (tp / KT) * KT;
    const char* Ws = lds + WOFF + (g % NS) * WSLOT + (wr * 16 * TC + col) * 128;
    const int toff = dy * HWD + dx;
    const int hx7 = (px_lane + dx) & 7;
    if constexpr (X3 == 2) {
      // pixel-group-major: the step's A terms (3 x TC fragments, pre-split) stay in registers, and the split
      // of group p + 1's activations (VALU) is interleaved with group p's 6 x TC MFMAs, so the VALU runs
      // under the matrix pipe instead of in a block in front of it (-6.5 % against the row-group-major order
      // below on the same box; carrying the next step's group-0 split under the last group's MFMAs measured
      // +1.5 %).  Same products, same per-accumulator order (small terms first) as the row-group-major order.
      const char* Wp = lds + WOFF + (g % NS) * WSLOT + (wr * 16 * TC + col) * 64 + ((q ^ ((col >> 1) & 3)) << 4);
      frag_t ah[TC], am[TC], al[TC];
#pragma unroll
      for (int t = 0; t < TC; ++t) {
        ah[t] = *reinterpret_cast<const frag_t*>(Wp + t * 16 * 64);
        am[t] = *reinterpret_cast<const frag_t*>(Wp + BR * 64 + t * 16 * 64);
        al[t] = *reinterpret_cast<const frag_t*>(Wp + 2 * BR * 64 + t * 16 * 64);
      }
      auto braw = [&](int p, int to, int h7, frag_t& v0, frag_t& v1) {
        const char* hp = hal + (prow[p] + to) * 128;
        v0 = *reinterpret_cast<const frag_t*>(hp + ((q ^ h7) << 4));
        v1 = *reinterpret_cast<const frag_t*>(hp + (((4 + q) ^ h7) << 4));
      };
      frag_t bh, bm, bl, x0, x1;
      braw(0, toff, hx7, x0, x1);
      split3_bf16(x0, x1, bh, bm, bl);
      __builtin_amdgcn_sched_barrier(0);
      auto group = [&](int p, bool split_next) {
        frag_t nh, nm, nl;
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], am[t], bm);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], al[t], bh);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bl);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], am[t], bh);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bm);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bh);
        if (split_next) {
          split3_bf16(x0, x1, nh, nm, nl);
          // 6 TC MFMAs with the next group's split spread between them (2 VALU per MFMA)
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
          for (int i = 0; i < 6 * TC; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
          bh = nh;
          bm = nm;
          bl = nl;
        }
        __builtin_amdgcn_sched_barrier(0);
      };
#pragma unroll
      for (int p = 0; p + 1 < TP; ++p) {
        braw(p + 1, toff, hx7, x0, x1);
        group(p, true);
      }
      group(TP - 1, false);
      return;
    }
    frag_t bh[TP], bm[TP], bl[TP];
#pragma unroll
    for (int p = 0; p < TP; ++p) {
      const char* hb = lds + (prow[p] + toff) * 128;
      const frag_t x0 = *reinterpret_cast<const frag_t*>(hb + ((q ^ hx7) << 4));
      const frag_t x1 = *reinterpret_cast<const frag_t*>(hb + (((4 + q) ^ hx7) << 4));
      split3_bf16(x0, x1, bh[p], bm[p], bl[p]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // X3 = 2: plane row r's 16-byte chunk q (K values 4q..4q+3, 16+4q..16+4q+3) sits at position
    // q ^ ((r >> 1) & 3): each ds_read_b128 lane group's 16 pieces cover the 64 banks once (MI355X_MICROARCH.md
    // §LDS lane groups; checked in tests/test_lds_layout_cpu.py)
    const char* Wp = lds + WOFF + (g % NS) * WSLOT + (wr * 16 * TC + col) * 64 + ((q ^ ((col >> 1) & 3)) << 4);
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      frag_t ah, am, al;
      if constexpr (X3 == 2) {
        ah = *reinterpret_cast<const frag_t*>(Wp + t * 16 * 64);
        am = *reinterpret_cast<const frag_t*>(Wp + BR * 64 + t * 16 * 64);
        al = *reinterpret_cast<const frag_t*>(Wp + 2 * BR * 64 + t * 16 * 64);
      } else {
        const char* wr_ = Ws + t * 16 * 128;
        const frag_t w0 = *reinterpret_cast<const frag_t*>(wr_ + ((q ^ (lane & 7)) << 4));
        const frag_t w1 = *reinterpret_cast<const frag_t*>(wr_ + (((4 + q) ^ (lane & 7)) << 4));
        split3_bf16(w0, w1, ah, am, al);
      }
      // term-major: TP independent accumulators between two MFMAs of one chain; small terms first
#pragma unroll
      for (int p = 0; p < TP; ++p) mfma_bf16(acc[t][p], am, bm[p]);
#pragma unroll
      for (int p = 0; p < TP; ++p) mfma_bf16(acc[t][p], al, bh[p]);
#pragma unroll
      for (int p = 0; p < TP; ++p) mfma_bf16(acc[t][p], ah, bl[p]);
#pragma unroll
      for (int p = 0; p < TP; ++p) mfma_bf16(acc[t][p], am, bh[p]);
#pragma unroll
      for (int p = 0; p < TP; ++p) mfma_bf16(acc[t][p], ah, bm[p]);
#pragma unroll
      for (int p = 0; p < TP; ++p) mfma_bf16(acc[t][p], ah, bh[p]);
      // one row group's A fragments live at a time (register budget: 128 accumulators + 48 B terms)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  frag_t a0[TC], b0[TP], a1[TC], b1[TP];
  int c = 0, tap = 0;
  for (int g = 0; g < S; ++g) {
    const bool wnext = g + NS - 1 < S;
    if (wnext) issue_w(g + NS - 1);
    if constexpr (X3 != 0) {
      x3_step(g, tap);
    } else {
      read_frags(g, tap, 0, a0, b0);
      mfmas(a0, b0);
      // 128-row wave tiles: keep one kk's fragments live at a time (register budget)
      if constexpr (TC == 8) __builtin_amdgcn_sched_barrier(0);
      read_frags(g, tap, 1, a1, b1);
      mfmas(a1, b1);
    }
    // the next step needs W(g+1); the barrier's lgkmcnt(0) also retires this step's reads (WAR)
    if (NS == 2) {
      wait_vm_barrier<0>();
    } else {
      if (wnext) wait_vm_barrier<WI>(); else wait_vm_barrier<0>();
    }
    if (tap == NTAP - 1 && c + 1 < nch) {   // every wave has finished reading the halo (barrier above)
#ifdef UNET_ABL_X3_NOHALO   // timing-only ablation build: the chunk's halo is never reloaded
      if constexpr (X3 == 0)
#endif
      {
        issue_halo(c_lo + c + 1);
        wait_vm_barrier<0>();
      }
    }
    if (++tap == NTAP) { tap = 0; ++c; }
  }
#pragma unroll
  for (int h = 0; h < TC / 4; ++h) {
    if constexpr (PART)
      partial_store<TP, 16>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n, ty * 16, tx * 16, wp * TP,
                            ct * BR + wr * 16 * TC + 64 * h, kslice);
    else
      conv_epilogue<T, T, TP, EPI>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n, ty * 16, tx * 16,
                                   wp * TP, ct * BR + wr * 16 * TC + 64 * h, bias_s + wr * 16 * TC + 64 * h, headw_s,
                                   headb_s);
  }
}

// ---------------------------------------------------------------------------------
// three-term fp32 with the activations split once per chunk (IgemmArgs::x3 = 3)
// ---------------------------------------------------------------------------------
// The X3 = 2 halo kernel above splits an activation fragment at every tap that reads it (nine splits of
// each halo value per row tile): ~176 VALU per wave and K step beside its 96 MFMAs, and a 16x16x32 MFMA
// leaves the SIMD's vector issue free for only 8 of its 16 cycles (MI355X_MICROARCH.md, constants table),
// so that step is vector-issue bound.  Here the block splits each 32-channel chunk's halo ONCE, into three
// bf16 planes in LDS, from an fp32 staging copy the LDS DMA filled during the previous chunk; the nine
// taps then read the planes (per wave and step: 96 MFMAs, 24 ds_read_b128, no conversion).  Staging
// (41 KB) + planes (62 KB) + two 24 KB weight slots take 151 KB: one 8-wave block per CU, 128 rows x
// 16x16 pixels (a 64-row x 64-pixel tile per wave, two waves per SIMD), for the layers with Cout >= 128.
// The same products in the same order per accumulator as X3 = 2 (bitwise the same sums per K slice).
// Planes: halo pixel r = hy * 18 + hx is a 64-byte row per plane; its 16-byte piece q (K values 4q..4q+3,
// 16+4q..16+4q+3, the weight planes' order) sits at q ^ ((hy & 1) << 1), so each ds_read_b128 lane group
// (4 pixels of row y and 4 of row y + 1, two pieces) covers the 64 banks once at every tap
// (tests/test_lds_layout_cpu.py).
template <int EPI>
__global__ __launch_bounds__(512, 1) void conv3x3_x3s_kernel(const IgemmArgs a) {
  constexpr int NW = 8, WPX = 4, TC = 4, TP = 4, BR = 128, HWD = 18, NPIX = HWD * HWD, NTAP = 9;
  constexpr int NI = (NPIX + 7) / 8;        // staging DMA pieces (8 halo pixels x 128 B)
  constexpr int HJ = (NI + NW - 1) / NW;    // per wave (the last round's surplus repeats piece NI - 1)
  constexpr int PLANE = NPIX * 64;
  constexpr int SPL = NI * 1024;            // the planes follow the staging buffer
  constexpr int WSLOT = 3 * BR * 64;
  constexpr int WJ = WSLOT / (1024 * NW);   // weight DMA pieces per wave and step
  constexpr int WOFF = SPL + 3 * PLANE;
  constexpr int PARAM_OFF = WOFF + 2 * WSLOT;
  constexpr int LDS_BYTES = PARAM_OFF + BR * 4;
  static_assert(LDS_BYTES <= 160 * 1024 && WSLOT % (1024 * NW) == 0, "one 8-wave block per CU");
  static_assert(SPL % 256 == 0 && PLANE % 256 == 0 && WOFF % 256 == 0, "bank-aligned regions");
  static_assert(EPI == EPI_STORE || EPI == EPI_POOL || EPI == EPI_PARTIAL, "x3s epilogues");
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float* bias_s = reinterpret_cast<float*>(lds + PARAM_OFF);

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wr = wave / WPX;
  const int wp = wave % WPX;
  int bid;
  {  // XCD-contiguous remap (as conv3x3_halo_kernel)
    const int nb = gridDim.x, qq = nb >> 3, rr = nb & 7;
    const int b = blockIdx.x, x = b & 7, k = b >> 3;
    bid = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + k;
  }
  constexpr bool PART = EPI == EPI_PARTIAL;
  const int KS = PART ? a.ksplit : 1;
  const int ct = bid % a.n_ct;
  int mt = bid / a.n_ct;
  const int kslice = PART ? mt % KS : 0;
  if (PART) mt /= KS;
  const int tx = mt % a.tiles_x;
  mt /= a.tiles_x;
  const int ty = mt % a.tiles_y;
  const int n = mt / a.tiles_y;
  if (n >= a.N) return;

  const int H = a.H, W = a.W;
  const int nch = a.Cin / 32 / KS;
  const int c_lo = kslice * nch;
  const int S = NTAP * nch;
  const char* in = reinterpret_cast<const char*>(a.in);
  const char* zero = reinterpret_cast<const char*>(a.zero);
  const long long pix0 = (long long)(n * H + ty * 16) * W + tx * 16;

  auto issue_halo = [&](int c) {   // chunk c's fp32 halo -> staging row r at r * 128, piece k at k ^ (hx & 7)
    const long long c0 = (long long)c * 32;
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int piece = min(j * NW + wave, NI - 1);
      const int row = piece * 8 + (lane >> 3);
      const int hy = row / HWD, hx = row - hy * HWD;
      const int iy = ty * 16 + hy - 1, ix = tx * 16 + hx - 1;
      const bool ok = row < NPIX && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const int chk = ((lane & 7) ^ (hx & 7)) * 16;
      const long long pix = pix0 + (long long)(hy - 1) * W + (hx - 1);
      const char* src = ok ? in + (pix * a.ldi + c0) * 4LL + chk : zero + chk;
      glds16(src, lds + piece * 1024);
    }
  };
  auto issue_w = [&](int g) {   // step g's pre-split weights [3][BR][64 B] (unet_capi.cpp pack3x3_split)
    const long long step = (long long)ct * (NTAP * (a.Cin / 32)) + (long long)c_lo * NTAP + g;
    const char* src = reinterpret_cast<const char*>(a.wgt) + step * WSLOT + (wave * WJ) * 1024 + lane * 16;
    char* dst = lds + WOFF + (g & 1) * WSLOT + wave * WJ * 1024;
#pragma unroll
    for (int j = 0; j < WJ; ++j) glds16(src + j * 1024, dst + j * 1024);
  };
  auto split_halo = [&]() {   // staging -> planes, one (pixel, piece) per thread and round
#pragma unroll
    for (int k = 0; k < (NPIX * 4 + 64 * NW - 1) / (64 * NW); ++k) {
      const int u = tid + k * 64 * NW;
      if (u < NPIX * 4) {
        const int r = u >> 2, pq = u & 3;
        const int hy = r / HWD, hx7 = (r - hy * HWD) & 7;
        const char* sp = lds + r * 128;
        const frag_t x0 = *reinterpret_cast<const frag_t*>(sp + ((pq ^ hx7) << 4));
        const frag_t x1 = *reinterpret_cast<const frag_t*>(sp + (((4 + pq) ^ hx7) << 4));
        frag_t h, m, l;
        split3_bf16(x0, x1, h, m, l);
        char* dp = lds + SPL + r * 64 + ((pq ^ ((hy & 1) << 1)) << 4);
        *reinterpret_cast<frag_t*>(dp) = h;
        *reinterpret_cast<frag_t*>(dp + PLANE) = m;
        *reinterpret_cast<frag_t*>(dp + 2 * PLANE) = l;
      }
    }
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int t = 0; t < TC; ++t)
#pragma unroll
    for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int col = lane & 15, q = lane >> 4;
  int prow[TP];
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of((wp * TP + p) * 16 + col, py, px);
    prow[p] = py * HWD + px;
  }
  const int ylo = (col >> 3) & 1;   // hy & 1 of this lane's pixels at dy = 0 (pix_of: row pairs)
  const char* Wl = lds + WOFF + (wr * 16 * TC + col) * 64 + ((q ^ ((col >> 1) & 3)) << 4);

  issue_halo(c_lo);
  issue_w(0);
  for (int i = tid; i < BR; i += 64 * NW) bias_s[i] = a.bias[ct * BR + i];
  wait_vm_barrier<0>();
  split_halo();
  wait_vm_barrier<0>();

  // one K step (chunk c, tap); LAST (the chunk's last tap, peeled so that it is its own code): the next
  // chunk's staged halo (landed at tap 1's wait) is split into registers between this tap's MFMAs, and
  // after the barrier only the plane stores remain exposed
  constexpr int SR = (NPIX * 4 + 64 * NW - 1) / (64 * NW);   // split units per thread
  auto step = [&](int c, int tap, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    const int g = c * NTAP + tap;
    if (g + 1 < S) issue_w(g + 1);
    // the next chunk's halo into the (free) staging buffer, behind W(g + 1): in flight for two steps
    const bool hnext = !LAST && tap == 0 && c + 1 < nch;
    if (hnext) issue_halo(c_lo + c + 1);
    frag_t sh[SR], sm[SR], sl[SR];
    if constexpr (LAST) {
#pragma unroll
      for (int k = 0; k < SR; ++k) {   // (past the last unit: a valid row, split and dropped)
        const int u = min(tid + k * 64 * NW, NPIX * 4 - 1);
        const int r = u >> 2, pq = u & 3, hx7 = (r - (r / HWD) * HWD) & 7;
        const char* sp = lds + r * 128;
        split3_bf16(*reinterpret_cast<const frag_t*>(sp + ((pq ^ hx7) << 4)),
                    *reinterpret_cast<const frag_t*>(sp + (((4 + pq) ^ hx7) << 4)), sh[k], sm[k], sl[k]);
      }
    }
    {
      const int dy = tap / 3, dx = tap - dy * 3;
      const char* Wp = Wl + (g & 1) * WSLOT;
      const char* Bl = lds + SPL + (dy * HWD + dx) * 64 + ((q ^ (((ylo ^ dy) & 1) << 1)) << 4);
      frag_t ah[TC], am[TC], al[TC];
#pragma unroll
      for (int t = 0; t < TC; ++t) {
        ah[t] = *reinterpret_cast<const frag_t*>(Wp + t * 16 * 64);
        am[t] = *reinterpret_cast<const frag_t*>(Wp + BR * 64 + t * 16 * 64);
        al[t] = *reinterpret_cast<const frag_t*>(Wp + 2 * BR * 64 + t * 16 * 64);
      }
#pragma unroll
      for (int p = 0; p < TP; ++p) {
        const char* bp = Bl + prow[p] * 64;
        const frag_t bh = *reinterpret_cast<const frag_t*>(bp);
        const frag_t bm = *reinterpret_cast<const frag_t*>(bp + PLANE);
        const frag_t bl = *reinterpret_cast<const frag_t*>(bp + 2 * PLANE);
        // the X3 = 2 order per accumulator: small terms first
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], am[t], bm);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], al[t], bh);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bl);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], am[t], bh);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bm);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bh);
      }
    }
    if constexpr (LAST) {   // the split is done before the barrier (else the compiler sinks it into the stores)
#pragma unroll
      for (int k = 0; k < SR; ++k) asm volatile("" ::"v"(sh[k]), "v"(sm[k]), "v"(sl[k]));
    }
    // W(g + 1) landed (and the halo, one step later); the barrier's lgkmcnt(0) retires this step's reads
    if (hnext) wait_vm_barrier<HJ>(); else wait_vm_barrier<0>();
    if constexpr (LAST) {
      if (c + 1 < nch) {   // every wave is past the chunk's last tap: the planes take the next chunk
#pragma unroll
        for (int k = 0; k < SR; ++k) {
          const int u = tid + k * 64 * NW;
          if (u < NPIX * 4) {
            const int r = u >> 2, pq = u & 3, hy = r / HWD;
            char* dp = lds + SPL + r * 64 + ((pq ^ ((hy & 1) << 1)) << 4);
            *reinterpret_cast<frag_t*>(dp) = sh[k];
            *reinterpret_cast<frag_t*>(dp + PLANE) = sm[k];
            *reinterpret_cast<frag_t*>(dp + 2 * PLANE) = sl[k];
          }
        }
        wait_vm_barrier<0>();
      }
    }
  };
  for (int c = 0; c < nch; ++c) {
    for (int tap = 0; tap < NTAP - 1; ++tap) step(c, tap, std::false_type{});
    step(c, NTAP - 1, std::true_type{});
  }
  const int row0 = ct * BR + wr * 16 * TC;
  if constexpr (PART)
    partial_store<TP, 16>(a, acc, n, ty * 16, tx * 16, wp * TP, row0, kslice);
  else
    conv_epilogue<float, float, TP, EPI>(a, acc, n, ty * 16, tx * 16, wp * TP, row0, bias_s + wr * 16 * TC, nullptr,
                                         nullptr);
}

// The 64-channel layers of the three-term plan (down1.3 + pool, conv1.0, conv1.3 + head; IgemmArgs::x3 = 4):
// the split-once scheme above on 64 rows x 16x32 pixels, 8 waves of one row pair x 32 columns (the 16-bit
// ring's tile and head epilogue), one block per CU.  The 18x34 halo's three planes take 115 KB, which
// leaves no room for an fp32 staging copy: each thread prefetches its five (pixel, piece) units of the next
// chunk into registers (40 VGPRs, issued behind the step's weights at the chunk's first tap) and splits them
// into the planes at the chunk's end.  Planes as conv3x3_x3s_kernel (pixel
// r = hy * 34 + hx, 34 = 2 mod 4 like 18: the same bank argument, tests/test_lds_layout_cpu.py).
template <int EPI>
__global__ __launch_bounds__(512, 1) void conv3x3_x3w_kernel(const IgemmArgs a) {
  constexpr int NW = 8, TC = 4, TP = 4, BR = 64, TW = 32, HWX = TW + 2, NPIX = 18 * HWX, NTAP = 9;
  constexpr int NU = NPIX * 4;                          // (pixel, piece) units of a chunk
  constexpr int UPT = (NU + 64 * NW - 1) / (64 * NW);   // per thread (past NU: loads of the zero page)
  constexpr int PLANE = NPIX * 64;
  constexpr int WSLOT = 3 * BR * 64;                    // 12 DMA pieces: waves 0..3 issue two
  constexpr int WOFF = 3 * PLANE;
  constexpr int PARAM_OFF = WOFF + 2 * WSLOT;
  constexpr int LDS_BYTES = PARAM_OFF + (BR + kMaxClasses * 64 + kMaxClasses) * 4;
  static_assert(LDS_BYTES <= 160 * 1024 && WSLOT == 12 * 1024, "one 8-wave block per CU");
  static_assert(PLANE % 256 == 0 && WOFF % 256 == 0, "bank-aligned regions");
  static_assert(EPI == EPI_STORE || EPI == EPI_POOL || EPI == EPI_HEAD || EPI == EPI_PARTIAL, "x3w epilogues");
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float* bias_s = reinterpret_cast<float*>(lds + PARAM_OFF);
  float* headw_s = bias_s + BR;
  float* headb_s = headw_s + kMaxClasses * 64;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  int bid;
  {  // XCD-contiguous remap (as conv3x3_halo_kernel)
    const int nb = gridDim.x, qq = nb >> 3, rr = nb & 7;
    const int b = blockIdx.x, x = b & 7, k = b >> 3;
    bid = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + k;
  }
  constexpr bool PART = EPI == EPI_PARTIAL;
  const int KS = PART ? a.ksplit : 1;
  const int ct = bid % a.n_ct;
  int mt = bid / a.n_ct;
  const int kslice = PART ? mt % KS : 0;
  if (PART) mt /= KS;
  const int tx = mt % a.tiles_x;
  mt /= a.tiles_x;
  const int ty = mt % a.tiles_y;
  const int n = mt / a.tiles_y;
  if (n >= a.N) return;

  const int H = a.H, W = a.W;
  const int nch = a.Cin / 32 / KS;
  const int c_lo = kslice * nch;
  const int S = NTAP * nch;
  const float* in = reinterpret_cast<const float*>(a.in);
  const float* zero = reinterpret_cast<const float*>(a.zero);
  const long long pix0 = (long long)(n * H + ty * 16) * W + tx * TW;

  frag_t hv[UPT][2];   // the next chunk's units: fp32 K values 4q..4q+3 and 16+4q..16+4q+3 of one pixel
  auto load_halo = [&](int c) {
    const long long c0 = (long long)c * 32;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = tid + k * 64 * NW;
      const int r = u >> 2, pq = u & 3;
      const int hy = r / HWX, hx = r - hy * HWX;
      const int iy = ty * 16 + hy - 1, ix = tx * TW + hx - 1;
      const bool ok = u < NU && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const float* src = ok ? in + (pix0 + (long long)(hy - 1) * W + (hx - 1)) * a.ldi + c0 : zero;
      hv[k][0] = *reinterpret_cast<const frag_t*>(src + 4 * pq);
      hv[k][1] = *reinterpret_cast<const frag_t*>(src + 16 + 4 * pq);
    }
  };
  auto split_halo = [&]() {
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = tid + k * 64 * NW;
      if (u < NU) {
        const int r = u >> 2, pq = u & 3, hy = r / HWX;
        frag_t h, m, l;
        split3_bf16(hv[k][0], hv[k][1], h, m, l);
        char* dp = lds + r * 64 + ((pq ^ ((hy & 1) << 1)) << 4);
        *reinterpret_cast<frag_t*>(dp) = h;
        *reinterpret_cast<frag_t*>(dp + PLANE) = m;
        *reinterpret_cast<frag_t*>(dp + 2 * PLANE) = l;
      }
    }
  };
  auto issue_w = [&](int g) {   // step g's pre-split weights [3][64][64 B] (unet_capi.cpp pack3x3_split)
    const long long step = (long long)ct * (NTAP * (a.Cin / 32)) + (long long)c_lo * NTAP + g;
    const char* src = reinterpret_cast<const char*>(a.wgt) + step * WSLOT + lane * 16;
    char* dst = lds + WOFF + (g & 1) * WSLOT;
    glds16(src + wave * 1024, dst + wave * 1024);
    if (wave < 4) glds16(src + (wave + 8) * 1024, dst + (wave + 8) * 1024);
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int t = 0; t < TC; ++t)
#pragma unroll
    for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int col = lane & 15, q = lane >> 4;
  int prow[TP];
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of_w<TW>((wave * TP + p) * 16 + col, py, px);
    prow[p] = py * HWX + px;
  }
  const int ylo = (col >> 3) & 1;   // hy & 1 of this lane's pixels at dy = 0
  const char* Wl = lds + WOFF + col * 64 + ((q ^ ((col >> 1) & 3)) << 4);

  load_halo(c_lo);
  issue_w(0);
  for (int i = tid; i < BR; i += 64 * NW) bias_s[i] = a.bias[ct * BR + i];
  if (EPI == EPI_HEAD) {
    for (int i = tid; i < a.ncls * 64; i += 64 * NW) headw_s[i] = a.head_w[i];
    if (tid < a.ncls) headb_s[tid] = a.head_b[tid];
  }
  split_halo();
  wait_vm_barrier<0>();

  // The next chunk's halo loads go out at the chunk's first tap, behind W(g + 1), and retire with it at
  // that step's vmcnt(0): a step of MFMAs covers both.  (Left in flight for a second step, the compiler's
  // own wait tracking -- blind to the asm weight DMAs, path-insensitive over the loop -- put a vmcnt(0)
  // in front of the next chunk's loads that also waited for the weights.)
  int c = 0, tap = 0;
  for (int g = 0; g < S; ++g) {
    if (g + 1 < S) issue_w(g + 1);
    if (tap == 0 && c + 1 < nch) load_halo(c_lo + c + 1);
    {
      const int dy = tap / 3, dx = tap - dy * 3;
      const char* Wp = Wl + (g & 1) * WSLOT;
      frag_t ah[TC], am[TC], al[TC];
#pragma unroll
      for (int t = 0; t < TC; ++t) {
        ah[t] = *reinterpret_cast<const frag_t*>(Wp + t * 16 * 64);
        am[t] = *reinterpret_cast<const frag_t*>(Wp + BR * 64 + t * 16 * 64);
        al[t] = *reinterpret_cast<const frag_t*>(Wp + 2 * BR * 64 + t * 16 * 64);
      }
      const char* Bl = lds + (dy * HWX + dx) * 64 + ((q ^ (((ylo ^ dy) & 1) << 1)) << 4);
#pragma unroll
      for (int p = 0; p < TP; ++p) {
        const char* bp = Bl + prow[p] * 64;
        const frag_t bh = *reinterpret_cast<const frag_t*>(bp);
        const frag_t bm = *reinterpret_cast<const frag_t*>(bp + PLANE);
        const frag_t bl = *reinterpret_cast<const frag_t*>(bp + 2 * PLANE);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], am[t], bm);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], al[t], bh);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bl);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], am[t], bh);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bm);
#pragma unroll
        for (int t = 0; t < TC; ++t) mfma_bf16(acc[t][p], ah[t], bh);
      }
    }
    wait_vm_barrier<0>();
    if (tap == NTAP - 1 && c + 1 < nch) {   // every wave is past the chunk's last tap: refill the planes
      split_halo();
      wait_vm_barrier<0>();
    }
    if (++tap == NTAP) { tap = 0; ++c; }
  }
  if constexpr (PART)
    partial_store<TP, TW>(a, acc, n, ty * 16, tx * TW, wave * TP, ct * BR, kslice);
  else
    conv_epilogue<float, float, TP, EPI, TW>(a, acc, n, ty * 16, tx * TW, wave * TP, ct * BR, bias_s, headw_s, headb_s);
}


// ---------------------------------------------------------------------------------
// 3x3 conv, ring pipeline over 32-channel (64-byte) K chunks (the main kernel for 3x3 layers)
// ---------------------------------------------------------------------------------
// The 128-byte-row halo kernel above keeps one 64-channel halo (41.5 KB) and two weight slots
// in LDS, so two blocks fit per CU but the next chunk's halo load is exposed and the weights
// are fetched only one step ahead -- ablations (profiles/tune_r1_ring.txt) put ~25 % of the
// time of the MFMA-bound layers in those waits.  Halving the row to 64 bytes (32 bf16/f16
// channels, 16 f32) halves every LDS image, which buys, at the same two blocks per CU:
//   * a double-buffered halo: the next chunk's 18x18 halo streams in during the current
//     chunk's nine taps (issued at tap 0, needed 9 steps later);
//   * an NS-slot weight ring: each step's weights are fetched NS-1 steps ahead.
// LDS: [halo 0][halo 1][w slot 0..NS-1][bias/head params] = 2*21 KB + NS*BR*64 B (+2 KB).
// A step = (chunk c32, tap): one MFMA K-block (16x16x32 bf16/f16; 4 x 16x16x4 f32) for each of
// the TC x TP fragment pairs of the wave.  The weights are pre-packed per row tile in step
// order ([ct][step][BR][64 B], unet_capi.cpp pack3x3) so every weight DMA instruction reads
// 1 KB contiguous.  Bank-conflict-free 64-byte-row images: halo pixel (hy,hx) chunk q at
// position q ^ (hx & 3); weight row r chunk q at position q ^ ((r >> 1) & 3) (exhaustive check
// over all ds_read_b128 lane groups, taps and pixel groups: the bank model of tools/halo_swizzle_search.py, tests/test_lds_layout_cpu.py).
// Blocks are persistent (n_ct row tiles x n_slots walkers, each walking pixel tiles slot,
// slot + n_slots, ...) so the rings run across tile boundaries and the epilogue of one tile
// overlaps the loads of the next.
// TH x TW: the pixel tile (16 x 16; or 12 x 32 for the 64-channel layers at full resolution:
// 384 pixels per block at two blocks per CU, see CFG_RING_R64_W12).  The halo is (TH+2) x (TW+2)
// pixels; its row stride (TW+2) * 16 dwords is 32 mod 64 banks for both widths, so the swizzle
// below stays conflict-free.
template <typename T, int WR, int WPX, int TCW, int NS, int TPS = 1, int HS = 0, int TH = 16, int TW = 16>
struct RingGeom {
  static constexpr int NW = WR * WPX;
  static constexpr int TC = TCW;
  static constexpr int HWD = TW + 2;                // halo width
  static constexpr int HP = (TH + 2) * HWD;         // halo pixels
  static constexpr int TP = TH * TW / 16 / WPX;     // 16-pixel groups per wave
  static constexpr int BR = WR * 16 * TC;
  static constexpr int BKE = 64 / (int)sizeof(T);   // K elements per step (64 bytes)
  static constexpr int RPI = 16;                    // 64-byte rows per LDS-DMA instruction
  static constexpr int HLW = NW >= 7 ? 7 : (NW >= 3 ? 3 : NW);   // halo loader waves (21 instr. at 16 x 16)
  static constexpr int HI = (HP + RPI * HLW - 1) / (RPI * HLW);
  // HS = 1: the halo is computed (fused first conv), not DMA'd: exactly 18x18 rows
  static constexpr int HALO_BYTES = HS ? HP * 64 : HI * HLW * RPI * 64;
  static constexpr int WI = BR / (RPI * NW);
  static constexpr int WSLOT = BR * 64;              // one tap's weights
  static constexpr int SLOT = TPS * WSLOT;           // one ring slot = one step = TPS taps
  static constexpr int WOFF = 2 * HALO_BYTES;
  static constexpr int PARAM_OFF = WOFF + NS * SLOT;
  static constexpr int XS_OFF = PARAM_OFF + (HS ? BR : BR + kMaxClasses * 64 + kMaxClasses) * 4;
  static constexpr int XS_BYTES = HS ? 20 * 20 * 4 * (int)sizeof(T) : 0;   // 20x20 input window, 4 ch
  static constexpr int LDS_BYTES = XS_OFF + XS_BYTES;
  static constexpr int BLOCKS_PER_CU = (160 * 1024) / LDS_BYTES;
};

// vmcnt(N) + barrier with N = nw * WI + (halo ? HI : 0), nw in [0, NS-2], as compile-time counts
template <int WI, int HI, int NSM2>
__device__ __forceinline__ void ring_wait(int nw, bool halo) {
  if constexpr (NSM2 >= 3) { if (nw == 3) { if (halo) wait_vm_barrier<3 * WI + HI>(); else wait_vm_barrier<3 * WI>(); return; } }
  if constexpr (NSM2 >= 2) { if (nw == 2) { if (halo) wait_vm_barrier<2 * WI + HI>(); else wait_vm_barrier<2 * WI>(); return; } }
  if constexpr (NSM2 >= 1) { if (nw == 1) { if (halo) wait_vm_barrier<WI + HI>(); else wait_vm_barrier<WI>(); return; } }
  if (halo) wait_vm_barrier<HI>(); else wait_vm_barrier<0>();
}

// TPS = taps per step (1, or 3 = one kernel row): a step then runs TPS x TC x TP MFMAs per wave
// between barriers and its ring slot holds TPS taps of weights (contiguous in the step-order
// packing, so the pack is the same).
// HS = 1 (down1.3 only): down1.0 is fused in -- every 32-channel halo chunk is COMPUTED from a
// 20x20 window of the network input (pre-cast to T, 4 channels per pixel, x_to_px4_kernel) on
// MFMA (K = 9*C <= 27 padded to 32) and written to the halo buffer with ds_write, one chunk
// ahead like the DMA halo; the window of the next tile is LDS-DMA'd (16-byte pieces, 2 pixels
// per lane) into a single buffer after the current window's last use.
// TO / TQ: element types of the output / pooled map (default T), see conv_epilogue.
// ABL (timing-only ablation builds, `make abl`; never in the product library): 1 = no barrier
// in the loop, 2 = no MFMA, 3 = no fragment reads in the loop, 4 = no DMA in the loop, 5 = no
// epilogue, 6 = epilogue arithmetic without the stores -- each gives wrong outputs by
// construction.  Variant with correct outputs, for A/B timing (launch_3x3): 8 = NS = 4 on the
// 128-row ring.
template <typename T, int WR, int WPX, int TCW, int NS, int EPI, int TPS, int HS, typename TO, typename TQ, int ABL,
          int TH = 16, int TW = 16>
__device__ __forceinline__ void ring_body(const IgemmArgs& a) {
  using G = RingGeom<T, WR, WPX, TCW, NS, TPS, HS, TH, TW>;
  constexpr int NW = G::NW, TC = G::TC, TP = G::TP, BR = G::BR, BKE = G::BKE;
  constexpr int HI = G::HI, WI = G::WI, HLW = G::HLW, HALO_BYTES = G::HALO_BYTES, WSLOT = G::WSLOT;
  constexpr int WOFF = G::WOFF, SLOT = G::SLOT;
  constexpr int HWD = G::HWD, kRingPix = G::HP;
  constexpr int SPC = 9 / TPS;   // steps per 32-channel chunk
  static_assert(TPS == 1 || TPS == 3, "taps per step");
  static_assert(NS >= 3 && NS <= 5, "weight ring depth");
  static_assert(WI >= 1 && BR % (G::RPI * NW) == 0, "weight tile split");
  static_assert(TP >= 1 && (TH * TW / 16) % WPX == 0 && TH % 2 == 0 && TW % 8 == 0, "pixel groups per wave");
  static_assert(EPI != EPI_HEAD || BR == 64, "fused head needs the 64 channels in one block");
  static_assert(HS == 0 || (sizeof(T) == 2 && BR == 64 && NW == 4 && TPS == 3 && EPI != EPI_HEAD && TH == 16 && TW == 16),
                "fused first conv: 16-bit, 64 rows, 3 taps per step, 16 x 16 tiles");
  static_assert(WR * WPX >= 8 || G::LDS_BYTES <= 160 * 1024 / 2, "two blocks per CU");
  // EPI_UPFUSE (conv2.3 + up1): after a tile's S conv steps, SU = 8 more ring steps run the
  // ConvTranspose2d (K = the 128 conv outputs, rows = 4 quadrants x 64) on the tile's pixels.
  constexpr bool UPF = EPI == EPI_UPFUSE;
  static_assert(!UPF || (sizeof(T) == 2 && WR == 1 && WPX == 4 && TC == 8 && TPS == 1 && HS == 0 && TH == 16 && TW == 16),
                "fused ConvTranspose: the 16-bit 128-row ring (all 128 channels of a pixel in one block)");
  constexpr int SU = UPF ? 8 : 0;
  __shared__ __attribute__((aligned(16))) char lds[G::LDS_BYTES];
  float* bias_s = reinterpret_cast<float*>(lds + G::PARAM_OFF);
  float* headw_s = bias_s + BR;
  float* headb_s = headw_s + kMaxClasses * 64;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wr = wave / WPX;
  const int wp = wave % WPX;

  int bid;
  {  // XCD-contiguous remap; consecutive ids = the n_ct row tiles of one pixel-tile walker
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7;
    const int b = blockIdx.x, x = b & 7, k = b >> 3;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  const int ct = bid % a.n_ct;
  const int slot = bid / a.n_ct;
  const int n_slots = gridDim.x / a.n_ct;
  const int n_mt = a.N * a.tiles_y * a.tiles_x;
  if (slot >= n_mt) return;
  const int items = (n_mt - slot + n_slots - 1) / n_slots;

  const int H = a.H, W = a.W;
  const int nch = a.Cin / BKE;
  const int S = SPC * nch;       // conv steps per tile
  const int ST = S + SU;         // ring steps per tile
  const int total = items * ST;
  const int hseq_end = items * nch;

  // weights of row tile ct in step order: step s at wblk + s * WSLOT; per lane one 16-byte
  // chunk of row (wave*WI + j)*16 + lane/4, stored at position lane&3 = chunk ^ ((row>>1)&3)
  const char* wblk = reinterpret_cast<const char*>(a.wgt) + (size_t)ct * ST * SLOT +
                     (wave * WI * 16 + (lane >> 2)) * 64 + (((lane & 3) ^ ((lane >> 3) & 3)) << 4);
  const char* in = reinterpret_cast<const char*>(a.in);
  const char* zero = reinterpret_cast<const char*>(a.zero);

  auto tile_of = [&](int i, int& n, int& ty, int& tx) {
    int mt = slot + i * n_slots;
    tx = mt % a.tiles_x;
    mt /= a.tiles_x;
    ty = mt % a.tiles_y;
    n = mt / a.tiles_y;
  };
  // Halo and weight DMAs are issued strictly in sequence (chunk after chunk, step after step), so
  // both sources advance by cursors: the per-lane halo piece pointers are computed once per
  // pixel tile (chunk c then adds 64c bytes; the zero page covers the invalid pieces of every
  // chunk) and the weight source by one step -- no divisions or 64-bit address math per piece.
  // OFF32 (the 12 x 32 tile, 10 pieces per loader lane; EPI_UPFUSE): 32-bit per-lane offsets from the
  // (wave-uniform) image base instead of 64-bit pointers, -1 - chk for a zero-page piece -- 10
  // VGPRs fewer in a kernel at the 256-register limit (launch_ring: one image < 2 GiB)
  constexpr bool OFF32 = TH != 16 || TW != 16 || UPF;
  const char* hsrc[OFF32 ? 1 : HI];
  int hoff[OFF32 ? HI : 1];
  const char* hbase = in;
  int hq_i = 0, hq_c = 0, hq_seq = 0;   // (tile, chunk, sequence number) of the next halo issue
  auto halo_tile = [&](int i) {
    int n, ty, tx;
    tile_of(i, n, ty, tx);
    const long long pix0 = (long long)(n * H + ty * TH) * W + tx * TW;
    if constexpr (OFF32) hbase = in + (long long)n * H * W * a.ldi * (long long)sizeof(T);
#pragma unroll
    for (int j = 0; j < HI; ++j) {
      const int row = (wave * HI + j) * 16 + (lane >> 2);
      const int hy = row / HWD, hx = row - (row / HWD) * HWD;
      const int iy = ty * TH + hy - 1, ix = tx * TW + hx - 1;
      const bool ok = row < kRingPix && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const int chk = ((lane & 3) ^ (hx & 3)) << 4;
      if constexpr (OFF32) {
        hoff[j] = ok ? (iy * W + ix) * a.ldi * (int)sizeof(T) + chk : -1 - chk;
      } else {
        const long long pix = pix0 + (long long)(hy - 1) * W + (hx - 1);
        hsrc[j] = ok ? in + pix * a.ldi * (long long)sizeof(T) + chk : zero + chk;
      }
    }
  };
  auto issue_halo = [&]() {   // the next chunk in sequence
    if (wave < HLW) {   // (wave-uniform) halo loader
      if (hq_c == 0) halo_tile(hq_i);
      char* dst = lds + (hq_seq & 1) * HALO_BYTES + wave * HI * 1024;
#pragma unroll
      for (int j = 0; j < HI; ++j) {
        if constexpr (OFF32) {
          const char* src = hoff[j] >= 0 ? hbase + hoff[j] : zero + (-1 - hoff[j]);
          glds16(src + hq_c * 64, dst + j * 1024);
        } else {
          glds16(hsrc[j] + hq_c * 64, dst + j * 1024);
        }
      }
    }
    ++hq_seq;
    if (++hq_c == nch) { hq_c = 0; ++hq_i; }
  };
  int wq_s = 0, wq_slot = 0;   // (step within the tile, ring slot) of the next weight issue
  auto issue_w = [&]() {
    const char* src = wblk + (size_t)wq_s * SLOT;
    char* dst = lds + WOFF + wq_slot * SLOT + wave * WI * 1024;
#pragma unroll
    for (int t = 0; t < TPS; ++t)
#pragma unroll
      for (int j = 0; j < WI; ++j) glds16(src + t * WSLOT + j * 1024, dst + t * WSLOT + j * 1024);
    if (++wq_s == ST) wq_s = 0;
    if (++wq_slot == NS) wq_slot = 0;
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int t = 0; t < TC; ++t)
#pragma unroll
    for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int col = lane & 15, q = lane >> 4;
  int prow[TP];
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of_w<TW>((wp * TP + p) * 16 + col, py, px);
    prow[p] = (py * HWD + px) * 64;
  }
  const int px_lane = col & 7;
  const int wpos = (q ^ ((col >> 1) & 3)) << 4;
  const char* wrow = lds + WOFF + (wr * 16 * TC + col) * 64 + wpos;

  // ---- HS: fused first conv (down1.0) -> halo chunks ----
  // window DMA of tile i: lane L < 200 of the block's 4 pieces copies input pixels
  // (2*(L%10), 2*(L%10)+1) of window row L/10 (8 B each) -> xs[(yy*20 + xx)*4 + c]
  auto issue_xs = [&](int i) {
    if constexpr (HS != 0) {
      int n, ty, tx;
      tile_of(i, n, ty, tx);
      const int L = wave * 64 + lane;
      if (L < 200) {
        const int yy = L / 10, seg = L - (L / 10) * 10;
        const int iy = ty * 16 + yy - 2, ix = tx * 16 + 2 * seg - 2;
        const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const char* src = ok ? reinterpret_cast<const char*>(a.x0) + ((long long)(n * H + iy) * W + ix) * 4 * sizeof(T)
                             : zero;
        glds16(src, lds + G::XS_OFF + wave * 1024);
      }
    }
  };
  // halo chunk cb (channels 32cb .. 32cb+31 of down1.0's output) of tile i -> halo buffer hb.
  // The first conv runs as three 16x16x16 MFMAs per 16 pixels x 16 channels: K slot 4q + c of
  // MFMA m is (tap first_tap(4m + q), channel c) (unet_internal.h: three slots are zero), so lane
  // group q's B operand is ONE 8-byte ds_read_b64 of the 4-channel window pixel under its tap,
  // conflict-free by the choice of the tap order: 3 reads per lane and pixel
  // group instead of 8 scattered 2-byte gathers.  Weights: a.w0p = [cb][t][m][16 rows][16 k].
  uint2 w0f[2][2][3];
  float b0v[2][8];
  int toff[3];   // byte offset of this lane's tap in the window, per MFMA (-1: zero tap)
  if constexpr (HS != 0) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int m = 0; m < 3; ++m)
          w0f[cb][t][m] = *reinterpret_cast<const uint2*>(
              reinterpret_cast<const char*>(a.w0p) + ((((cb * 2 + t) * 3 + m) * 16 + (lane & 15)) * 16 + 4 * (lane >> 4)) * sizeof(T));
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int j = 0; j < 8; ++j) b0v[cb][j] = a.b0[32 * cb + 8 * (lane >> 4) + j];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int ta = first_tap_addr(4 * m + (lane >> 4));   // bit 0: a zero slot
      toff[m] = ((ta / 3) * 20 + ta % 3) * 4 * (int)sizeof(T) + (first_tap(4 * m + (lane >> 4)) > 8 ? 1 : 0);
    }
  }
  // part = 0 / 1: the even / odd pixel groups of this wave (the chunk is computed over two
  // steps, so that no single step carries all of it); at most 3 groups per part, unrolled so
  // that the reads of all of them are in flight together
  constexpr int HGR = (kRingPix + 15) / 16;               // 16-pixel groups of the halo
  constexpr int HIT = (HGR + 2 * NW - 1) / (2 * NW);      // groups per wave and part
  auto compute_halo = [&](int i, int cb, int hb, int part) {
    if constexpr (HS != 0) {
      int n, ty, tx;
      tile_of(i, n, ty, tx);
      const char* xs = lds + G::XS_OFF;
      char* dst = lds + hb * HALO_BYTES;
      const int qq = lane >> 4;
#pragma unroll
      for (int it = 0; it < HIT; ++it) {
        const int grp = wave + part * NW + it * 2 * NW;
        if (grp >= HGR) break;   // wave-uniform
        const int p = grp * 16 + (lane & 15);
        const bool real = p < kRingPix;
        const int hy = real ? p / 18 : 0, hx = real ? p - (p / 18) * 18 : 0;
        const char* px = xs + (hy * 20 + hx) * 4 * (int)sizeof(T);
        f32x4 acc0[2];   // start at the first conv's bias (first_conv_mfma_kernel: bitwise the same)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc0[t] = f32x4{b0v[cb][4 * t], b0v[cb][4 * t + 1], b0v[cb][4 * t + 2], b0v[cb][4 * t + 3]};
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          uint2 bv = *reinterpret_cast<const uint2*>(px + (toff[m] & ~1));
          if (toff[m] & 1) bv = uint2{0u, 0u};   // 0 x (a NaN input) must stay 0
#pragma unroll
          for (int t = 0; t < 2; ++t) acc0[t] = mfma16<T>(w0f[cb][t][m], bv, acc0[t]);
        }
        // lane holds channels 32cb + 8q + 4t + e: 8 consecutive channels = one 16-byte piece
        const int iy = ty * 16 + hy - 1, ix = tx * 16 + hx - 1;
        const bool inimg = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        typedef T t8 __attribute__((ext_vector_type(8)));
        t8 o;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) o[4 * t + e] = (T)(inimg ? relu_nan(acc0[t][e]) : 0.f);
        if (real) *reinterpret_cast<uint4*>(dst + p * 64 + ((qq ^ (hx & 3)) << 4)) = __builtin_bit_cast(uint4, o);
      }
    }
  };

  // prologue: halo of chunk 0 and weights of steps 0 .. NS-2
  if constexpr (HS != 0) {
    issue_xs(0);
    wait_vm_barrier<0>();
    compute_halo(0, 0, 0, 0);
    compute_halo(0, 0, 0, 1);
  } else {
    issue_halo();
  }
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (k < total) issue_w();
  for (int i = tid; i < BR; i += 64 * NW) bias_s[i] = a.bias[ct * BR + i];
  if (EPI == EPI_HEAD) {
    for (int i = tid; i < a.ncls * 64; i += 64 * NW) headw_s[i] = a.head_w[i];
    if (tid < a.ncls) headb_s[tid] = a.head_b[tid];
  }
  {
    const int young = total - 1 < NS - 2 ? total - 1 : NS - 2;   // W(1..NS-2) may stay in flight
    ring_wait<TPS * WI, HI, NS - 2>(young, false);
  }

  // one step: A (weight) fragments stream through a 3-register ring two MFMA groups ahead;
  // sched_group_barrier pins the read/MFMA interleave (see step_sg above)
  frag_t abl_fr[2];   // ablation 3: the fragments every MFMA reads
  if constexpr (ABL == 3) {
    abl_fr[0] = *reinterpret_cast<const frag_t*>(lds + WOFF + lane * 16);
    abl_fr[1] = *reinterpret_cast<const frag_t*>(lds + lane * 16);
  }
  auto step = [&](int g, int hs, int tp, int tsub) {
    const int dy = tp / 3, dx = tp - (tp / 3) * 3;
    const char* Hs = lds + (hs & 1) * HALO_BYTES + (dy * HWD + dx) * 64 + ((q ^ ((px_lane + dx) & 3)) << 4);
    const char* Ws = wrow + (g % NS) * SLOT + tsub * WSLOT;
    frag_t bq[TP], ar[3];
    if constexpr (ABL == 3) {   // ablation: fragments from registers only
#pragma unroll
      for (int p = 0; p < TP; ++p) { bq[p] = abl_fr[p & 1]; asm volatile("" : "+v"(bq[p])); }
#pragma unroll
      for (int t = 0; t < TC; ++t) {
        frag_t af = abl_fr[t & 1];
        asm volatile("" : "+v"(af));
#pragma unroll
        for (int p = 0; p < TP; ++p)
          mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, bq[p]));
      }
      return;
    }
#pragma unroll
    for (int p = 0; p < TP; ++p) bq[p] = *reinterpret_cast<const frag_t*>(Hs + prow[p]);
    ar[0] = *reinterpret_cast<const frag_t*>(Ws);
    if (TC > 1) ar[1] = *reinterpret_cast<const frag_t*>(Ws + 16 * 64);
    __builtin_amdgcn_sched_group_barrier(0x100, TP + (TC > 1 ? 2 : 1), 0);
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      if (t + 2 < TC) ar[(t + 2) % 3] = *reinterpret_cast<const frag_t*>(Ws + (t + 2) * 16 * 64);
      const frag_t af = ar[t % 3];
#pragma unroll
      for (int p = 0; p < TP; ++p) {
        if constexpr (ABL == 2) asm volatile("" ::"v"(af), "v"(bq[p]));   // ablation: no MFMA
        else mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, bq[p]));
      }
      if (t + 2 < TC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TP, 0);
    }
  };

  // EPI_UPFUSE: the tile's conv outputs relu(acc + bias) as 16-bit B fragments of the
  // ConvTranspose GEMM.  Lane (pixel col, q) holds natural channels 64h + 16q + 0..15 of its pixels
  // (the row permutation of the packed weights), so K block kb = 2h + half takes channels
  // 64h + 16q + 8half + 0..7 in K slots 8q .. 8q+7: every lane's fragment is its own 8 values (the
  // ConvTranspose weights are packed in this K order, unet_capi.cpp pack_fused_up).  A ConvTranspose
  // step u = (quadrant u >> 1, K blocks 2 (u & 1) and 2 (u & 1) + 1) streams 64 rows x 64 K of
  // weights through the ring (slot row 64 kbl + r); a quadrant's 64 x 64-pixel accumulators reuse
  // acc[0..3], so only the tile's 64 output registers are live beside xb.
  frag_t xb[UPF ? TP : 1][UPF ? 4 : 1];
  auto stepT = [&](int g, int khalf) {   // one quadrant x K blocks 2 khalf, 2 khalf + 1: slot row 64 kbl + r
    if constexpr (UPF) {
      const char* Ws = wrow + (g % NS) * SLOT;
      frag_t ar[3];
      ar[0] = *reinterpret_cast<const frag_t*>(Ws);
      ar[1] = *reinterpret_cast<const frag_t*>(Ws + 16 * 64);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int t = 0; t < TC; ++t) {   // t = 4 kbl + row group
        if (t + 2 < TC) ar[(t + 2) % 3] = *reinterpret_cast<const frag_t*>(Ws + (t + 2) * 16 * 64);
        const frag_t af = ar[t % 3];
#pragma unroll
        for (int p = 0; p < TP; ++p)
          mfma_frag<T>(acc[t & 3][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, xb[p][2 * khalf + (t >> 2)]));
        if (t + 2 < TC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, TP, 0);
      }
    }
  };
  auto conv_to_xb = [&]() {   // bias + ReLU + cast (what EPI_STORE would store), then acc = 0
    if constexpr (UPF) {
      typedef T t8 __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          float bv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) bv[j] = bias_s[64 * h + 16 * q + 8 * half + j];
#pragma unroll
          for (int p = 0; p < TP; ++p) {
            t8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (T)relu_nan(acc[4 * h + 2 * half + (j >> 2)][p][j & 3] + bv[j]);
            xb[p][2 * h + half] = __builtin_bit_cast(frag_t, v);
          }
        }
#pragma unroll
      for (int t = 0; t < 4; ++t)   // acc[0..3]: the ConvTranspose accumulators (acc[4..7] stay dead)
#pragma unroll
        for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  static_assert(SPC >= NS - 1, "a halo issued after an epilogue is first needed after the barrier-only waits");
  int c = 0, tap = 0, hseq = 0, item = 0;   // tap = step index within the chunk (0 .. SPC-1)
  int wskip = 0;                            // barrier-only waits left after the last epilogue
  for (int g = 0; g < total; ++g) {
    const bool hnext = tap == 0 && hseq + 1 < hseq_end;
    if constexpr (HS == 0 && ABL != 4) {
      if (hnext) issue_halo();
    }
    if (ABL != 4 && g + NS - 1 < total) issue_w();
    if constexpr (HS != 0 && ABL != 4) {
      // the next tile's window, once this tile's last halo chunk has been computed from it (at
      // chunk 0, steps 0 and 1; the barrier after step 1 retired every read of xs).  Issued
      // after this step's weights, so the wait at the end of the NEXT step (for those weights)
      // is the one that retires it: chunk 1 computes the next tile's halo at its steps 1 and 2.
      if (c == 0 && tap == 2 && item + 1 < items) issue_xs(item + 1);
    }
    if constexpr (TPS == 3 && ABL == 0 && TC * TP % (TC + TP) == 0) {
      const char* hs3[3];
      const char* ws3[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {   // taps (dy = tap, dx = t): one kernel row
        hs3[t] = lds + (hseq & 1) * HALO_BYTES + (tap * HWD + t) * 64 + ((q ^ ((px_lane + t) & 3)) << 4);
        ws3[t] = wrow + (g % NS) * SLOT + t * WSLOT;
      }
      mfma_taps<T, TC, TP, 3>(acc, hs3, ws3, prow);
    } else {
#pragma unroll
      for (int t = 0; t < TPS; ++t) step(g, hseq, tap * TPS + t, t);
    }
    if constexpr (HS != 0) {   // next chunk's halo into the other buffer (last read a chunk ago),
      // in two halves: chunk 1 of this tile at steps 0, 1 of chunk 0; chunk 0 of the next tile
      // at steps 1, 2 of chunk 1 (down1.3: Cin = 64, so nch = 2 and SPC = 3)
      if (c == 0 && tap < 2) compute_halo(item, 1, (hseq + 1) & 1, tap);
      else if (c == 1 && tap >= 1 && item + 1 < items) compute_halo(item + 1, 0, (hseq + 1) & 1, tap - 1);
    }
    // W(g+1) must have landed (and, at a chunk end, the next halo -- issued 8 steps earlier,
    // so older than W(g+1)).  Younger loads may stay in flight: W(g+2 .. g+NS-1) and a halo
    // issued within the last NS-2 steps (this chunk's tap < NS-2).
    // Right after a tile's epilogue (wskip > 0) everything the next NS-2 steps need was issued
    // before it and waited for there, so the wait is the barrier alone: a vmcnt wait would also
    // wait for the epilogue's global stores (vmcnt counts loads and stores in issue order).
    {
      int young = total - 2 - g;
      young = young < 0 ? 0 : (young > NS - 2 ? NS - 2 : young);
      const bool hyoung = HS == 0 && wave < HLW && tap < NS - 2 && hseq + 1 < hseq_end;
      if constexpr (ABL == 1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // ablation: no barrier
      else if constexpr (ABL == 4) wait_vm_barrier<0>();
      else if (wskip > 0) { --wskip; wait_vm_barrier<63>(); }
      else ring_wait<TPS * WI, HI, NS - 2>(young, hyoung);
    }
    bool tile_end = false;
    if (++tap == SPC) {
      tap = 0;
      ++hseq;
      if (++c == nch) {
        c = 0;
        tile_end = true;
      }
    }
    if (UPF && tile_end) {
      // the conv part of the tile is done: its outputs become the B operand of the tile's SU
      // ConvTranspose ring steps, run right here (so xb lives only inside this block); after each
      // quadrant pair (4 steps) the pair's outputs are scattered into the concat buffer
      conv_to_xb();
      int n, ty, tx;
      tile_of(item, n, ty, tx);
#pragma nounroll
      for (int quad = 0; quad < 4; ++quad) {   // (a, b) quadrant of the ConvTranspose: 64 output rows
#pragma unroll
        for (int khalf = 0; khalf < 2; ++khalf) {   // unrolled: xb[p][kb] must index registers
          ++g;
          if (g + NS - 1 < total) issue_w();
          stepT(g, khalf);
          int young = total - 2 - g;
          young = young < 0 ? 0 : (young > NS - 2 ? NS - 2 : young);
          if (wskip > 0) { --wskip; wait_vm_barrier<63>(); }
          else ring_wait<TPS * WI, HI, NS - 2>(young, false);   // the last halo issue is older than W(g+1)
        }
        // no vmcnt(0) drain before the stores (unlike a tile end): the next step's wait (vmcnt of the
        // loads issued after them) retires them, so they drain under that step's MFMAs
        conv_epilogue<TO, TO, TP, EPI_UPSCATTER>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[0]), n, ty * 16,
                                                 tx * 16, wp * TP, 64 * quad, a.bias2 + 64 * quad, nullptr, nullptr,
                                                 a.out2, a.ldo2, a.Cout / 2);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int t = 4; t < TC; ++t)
#pragma unroll
        for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};
      ++item;
      continue;
    }
    if (tile_end) {
      int n, ty, tx;
      tile_of(item, n, ty, tx);
      if constexpr (ABL == 6 && EPI != EPI_HEAD) {   // ablation: epilogue arithmetic, no stores
#pragma unroll
        for (int h = 0; h < TC / 4; ++h)
          conv_epilogue<TO, TQ, TP, EPI, TW, 1>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n, ty * TH,
                                                tx * TW, wp * TP, ct * BR + wr * 16 * TC + 64 * h,
                                                bias_s + wr * 16 * TC + 64 * h, headw_s, headb_s);
      } else if constexpr (ABL == 5) {   // ablation: no epilogue (keep the accumulators alive)
#pragma unroll
        for (int t = 0; t < TC; ++t)
#pragma unroll
          for (int p = 0; p < TP; ++p) asm volatile("" ::"v"(acc[t][p]));
      } else {
        // every load issued so far (the weights of the next NS-2 steps, the next halo) has landed
        // before the stores go out; the next NS-2 waits are then barriers only (wskip)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int h = 0; h < TC / 4; ++h)
          conv_epilogue<TO, TQ, TP, EPI, TW>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n, ty * TH,
                                             tx * TW, wp * TP, ct * BR + wr * 16 * TC + 64 * h,
                                             bias_s + wr * 16 * TC + 64 * h, headw_s, headb_s);
        wskip = NS - 2;
      }
#pragma unroll
      for (int t = 0; t < TC; ++t)
#pragma unroll
        for (int p = 0; p < TP; ++p) acc[t][p] = f32x4{0.f, 0.f, 0.f, 0.f};
      ++item;
    }
  }
}

template <typename T, int WR, int WPX, int TCW, int NS, int EPI, int TPS = 1, int HS = 0, typename TO = T,
          typename TQ = TO, int TH = 16, int TW = 16>
__global__ __launch_bounds__(64 * WR * WPX, WR * WPX >= 8 ? 1 : 2) void conv3x3_ring_kernel(const IgemmArgs a) {
  ring_body<T, WR, WPX, TCW, NS, EPI, TPS, HS, TO, TQ, 0, TH, TW>(a);
}
#ifdef UNET_ABLATION
template <typename T, int WR, int WPX, int TCW, int NS, int EPI, int TPS, int HS, typename TO, typename TQ, int ABL>
__global__ __launch_bounds__(64 * WR * WPX, WR * WPX >= 8 ? 1 : 2) void conv3x3_ring_abl_kernel(const IgemmArgs a) {
  ring_body<T, WR, WPX, TCW, NS, EPI, TPS, HS, TO, TQ, ABL>(a);
}
#endif

// ---------------------------------------------------------------------------------
// 3x3 conv, 8-wave ring over 16 x 32 pixel tiles (one block per CU)
// ---------------------------------------------------------------------------------
// Ablations of the 4-wave ring (profiles/tune_r2_ablation.txt) point at the L2 -> LDS stream of
// the layers with few output channels: without the in-loop LDS-DMA conv1.0 runs 40 % faster,
// conv1.3 33 %, the 128-row layers 14-29 %, while dropping the LDS fragment reads or the barriers
// changes almost nothing (the no-epilogue ablations are confounded: their layers then compute on
// all-zero inputs, which the chip runs at a higher clock).  Per MFMA a 64-row x 256-pixel block
// tile streams ~100 B of weights + halo into LDS (mostly weights, re-fetched per pixel tile).
// This variant doubles the pixel tile (16 x 32, 512 pixels, 8 waves = 2 per SIMD of ONE block per
// CU, 64 pixels per wave as before), so every weight byte feeds twice the MFMAs and the halo
// overlap shrinks (18x34 / 512 = 1.20 vs 1.27).  WST = 1 (weight-stationary, Cin = 64 layers):
// all of the row tile's weights (6 steps x 12 KB = 72 KB) are DMA'd once per block and stay in
// LDS; the loop then streams only the halo, and needs a barrier only at chunk ends.
// LDS: [halo 0][halo 1][weights: NS slots, or all S steps (WST)][bias/head params].
// Same K order (chunk32-major, tap-minor), fragment layouts and swizzles as the 4-wave ring (the
// 34-pixel halo row stride is 544 dwords = 32 mod 64 banks, like the 18-pixel one), so the two
// agree bitwise.
template <typename T, int TCW, int NS, int TPS, int WST, int HS = 0>
struct Ring8Geom {
  static constexpr int NW = 8, TW = 32, TP = 4;
  static constexpr int TC = TCW;
  static constexpr int BR = 16 * TC;
  static constexpr int BKE = 64 / (int)sizeof(T);
  static constexpr int HWD = TW + 2;                  // halo width (34)
  static constexpr int HP = 18 * HWD;                 // halo pixels (612)
  static constexpr int HI = (HP + 16 * NW - 1) / (16 * NW);   // halo DMA instructions per wave (5)
  static constexpr int HALO_BYTES = HS ? HP * 64 : HI * NW * 16 * 64;   // HS: computed, exactly HP rows
  static constexpr int WSLOT = BR * 64;               // one tap's weights
  static constexpr int SLOT = TPS * WSLOT;            // one step
  static constexpr int PIECES = SLOT / 1024;          // weight DMA instructions per step (all waves)
  static constexpr int WST_STEPS = 6;                 // weight-stationary capacity: Cin = 64, 3 taps/step
  static constexpr int WBYTES = WST ? WST_STEPS * SLOT : NS * SLOT;
  static constexpr int WOFF = 2 * HALO_BYTES;
  static constexpr int PARAM_OFF = WOFF + WBYTES;
  static constexpr int XW = TW + 4;                   // fused first conv: input window 20 x XW, 4 channels
  static constexpr int XS_OFF = PARAM_OFF + (HS ? BR : BR + kMaxClasses * 64 + kMaxClasses) * 4;
  static constexpr int XS1 = 20 * XW * 4 * (int)sizeof(T);   // one input window
  static constexpr int XS_BYTES = HS ? 2 * XS1 : 0;            // double-buffered (tile i: buffer i & 1)
  static constexpr int LDS_BYTES = XS_OFF + XS_BYTES;          // HS: exactly 160 KiB
};

// ablation builds only (ABL = 1, no barrier): the counted wait alone
template <int N>
__device__ __forceinline__ void wait_vm_only() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
  asm volatile("" ::: "memory");
}

// vmcnt(n) + barrier for a runtime (wave-uniform) n in [0, 15]
__device__ __forceinline__ void wait_vm_barrier_rt(int n) {
  switch (n) {
    case 0: wait_vm_barrier<0>(); break;   case 1: wait_vm_barrier<1>(); break;
    case 2: wait_vm_barrier<2>(); break;   case 3: wait_vm_barrier<3>(); break;
    case 4: wait_vm_barrier<4>(); break;   case 5: wait_vm_barrier<5>(); break;
    case 6: wait_vm_barrier<6>(); break;   case 7: wait_vm_barrier<7>(); break;
    case 8: wait_vm_barrier<8>(); break;   case 9: wait_vm_barrier<9>(); break;
    case 10: wait_vm_barrier<10>(); break; case 11: wait_vm_barrier<11>(); break;
    case 12: wait_vm_barrier<12>(); break; case 13: wait_vm_barrier<13>(); break;
    case 14: wait_vm_barrier<14>(); break; default: wait_vm_barrier<15>(); break;
  }
}

// HS = 1 (down1.3): down1.0 fused in, as in the 4-wave ring (its halo chunks are computed from a
// 20 x 36 window of the pre-cast input on 16x16x16 MFMAs); needs WST (the loop then has a barrier
// after every step: the window is re-filled while the halo of the next tile is computed from it).
// ABL (timing-only ablation builds, `make abl`; 3-tap 128-row ring): 1 = the counted waits without
// the barriers, 2 = no MFMAs, 3 = no LDS fragment reads, 4 = no LDS-DMA in the loop (the slots keep
// the prologue's bytes); 5 = no tile epilogue (the accumulators are kept
// alive, nothing is stored) -- the per-tile epilogue's share of a layer, wrong outputs by construction;
// 6 = the epilogue's arithmetic without its stores; 7 = its stores (zeros) without the arithmetic;
// 8 = every 32-channel chunk's halo from the first 64 bytes of its 128-byte line (issue_halo); 9 = no
// halo DMA for odd chunks (issue_halo).
template <typename T, int TCW, int NS, int EPI, int TPS, int WST, typename TO, typename TQ, int HS = 0, int ABL = 0>
__global__ __launch_bounds__(512, 2) void conv3x3_ring8_kernel(const IgemmArgs a) {
  using G = Ring8Geom<T, TCW, NS, TPS, WST, HS>;
  constexpr int NW = G::NW, TW = G::TW, TC = G::TC, TP = G::TP, BR = G::BR, BKE = G::BKE;
  constexpr int HWD = G::HWD, HP = G::HP, HI = G::HI, HALO_BYTES = G::HALO_BYTES;
  constexpr int WSLOT = G::WSLOT, SLOT = G::SLOT, PIECES = G::PIECES, WOFF = G::WOFF;
  constexpr int SPC = 9 / TPS;   // steps per 32-channel chunk
  static_assert(TPS == 1 || TPS == 3 || (TPS == 9 && !WST && HS == 0), "taps per step");
  static_assert(WST || (NS >= 3 && NS <= 4) || (TPS == 9 && NS == 2), "weight ring depth");
  static_assert(EPI != EPI_HEAD || BR == 64, "fused head needs the 64 channels in one block");
  static_assert(G::LDS_BYTES <= 160 * 1024, "LDS");
  static_assert(HS == 0 || (WST && sizeof(T) == 2 && BR == 64 && TPS == 3 && EPI != EPI_HEAD),
                "fused first conv: weight-stationary 16-bit 64-row ring, 3 taps per step");
  // EPI_UPFUSE (conv2.3 + up1, see ring_body): after a tile's conv steps, SU = 4 more ring steps,
  // one (a, b) quadrant each: 64 rows x 128 K of ConvTranspose weights (16 KB of the 24 KB slot,
  // pseudo-row 64 kb + r), 64 MFMAs per wave; B = the tile's conv outputs in registers.
  constexpr bool UPF = EPI == EPI_UPFUSE;
  static_assert(!UPF || (sizeof(T) == 2 && TC == 8 && TPS == 3 && WST == 0 && HS == 0), "fused ConvTranspose");
  constexpr int SU = UPF ? 4 : 0;
  // EPI_PARTIAL (split-K, small batches): the walkers' items are (pixel tile, K slice) pairs, item
  // m = tile m / KS, slice m % KS; the launcher makes n_slots a multiple of KS, so a walker keeps ONE
  // slice (its weight ring cycles over that slice's steps) and its halo cursor starts at the slice's
  // first chunk.  Accumulators start at zero (the reduction adds the bias).
  constexpr bool PART = EPI == EPI_PARTIAL;
  static_assert(!PART || (HS == 0 && WST == 0 && !UPF), "split-K: the streamed-weight ring");
  __shared__ __attribute__((aligned(16))) char lds[G::LDS_BYTES];
  float* bias_s = reinterpret_cast<float*>(lds + G::PARAM_OFF);
  float* headw_s = bias_s + BR;
  float* headb_s = headw_s + kMaxClasses * 64;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar: the DMA addresses stay in SGPRs
  const uint32_t lds0 = lds_addr_of(lds);
  const int lane = tid & 63;
  const int wp = wave;   // all 8 waves split the pixels; each covers all BR rows

  int ct, slot;
  {  // XCD-contiguous remap; consecutive ids = the n_ct row tiles of one pixel-tile walker
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7;
    const int b = blockIdx.x, x = b & 7, k = b >> 3;
    const int bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
    ct = bid % a.n_ct;
    slot = bid / a.n_ct;
  }
  const int n_slots = gridDim.x / a.n_ct;
  const int KS = PART ? a.ksplit : 1;
  const int n_mt = a.N * a.tiles_y * a.tiles_x * KS;
  if (slot >= n_mt) return;
  const int items = (n_mt - slot + n_slots - 1) / n_slots;
  const int kslice = PART ? slot % KS : 0;

  const int H = a.H, W = a.W;
  const int nch = a.Cin / BKE / KS;   // 32-channel chunks per tile (of this walker's K slice)
  const int c_lo = kslice * nch;
  const int S = SPC * nch;       // conv steps per tile
  const int ST = S + SU;         // ring steps per tile
  const int total = items * ST;
  const int hseq_end = items * nch;
  // weight DMA pieces of this wave per step: pieces wave, wave + 8, ... of the step's PIECES
  const int wcnt = (PIECES - wave + NW - 1) / NW;
  // The loop's counted wait: young * wcnt (+ HI when a halo issued after W(g+1) may stay in flight).
  // young = NS - 2 on every step but the last ones, and wcnt is the same on every wave when PIECES
  // % NW == 0, so the common waits are two immediates; the runtime switch (a compare chain with a
  // barrier copy per case, ~40 scalar instructions and several branches per step) stays for the
  // ring's last steps only (round 3).
  constexpr int WCC = PIECES % NW == 0 ? PIECES / NW : -1;
  auto loop_wait = [&](int young, bool hy) {
    if constexpr (ABL == 1) {   // ablation: the counted wait without the barrier
      if (young == NS - 2 && WCC >= 0) {
        constexpr int base = (NS - 2) * (WCC < 0 ? 0 : WCC);
        if (hy) wait_vm_only<base + HI>();
        else wait_vm_only<base>();
      } else {
        wait_vm_only<0>();
      }
      return;
    }
    if constexpr (ABL == 4) {   // ablation: no DMA in the loop, so nothing to wait for
      wait_vm_barrier<63>();
      return;
    }
    if constexpr (NS == 2 || WCC >= 0) {
      if (young == NS - 2) {
        constexpr int base = NS == 2 ? 0 : (NS - 2) * WCC;
        if (hy) wait_vm_barrier<base + HI>();
        else wait_vm_barrier<base>();
        return;
      }
    }
    wait_vm_barrier_rt(young * wcnt + (hy ? HI : 0));
  };

  // weights of row tile ct in step order (the 4-wave ring's packing): piece j of a step = rows
  // 16j .. 16j+15; per lane one 16-byte chunk of row 16j + lane/4 at position chunk ^ ((row>>1)&3)
  // (the row tile's base is wave-uniform: the DMA takes it in SGPRs and the lane's 16-byte chunk as a
  // 32-bit offset, glds16_sv)
  // EPI_PARTIAL on a finer row tile than the packing's (a.src_br = 128 with BR = 64: the batch-1 split
  // gets twice the blocks per K slice, so half the slices -- and half the fp32 partials -- for the same
  // CU count): row tile ct is part ct % R of packed row tile ct / R, whose steps are R times longer
  // (also unsplit: the batch-1 plan runs under-filled 128-row layers on 64-row tiles, FINE instantiations)
  constexpr bool FINE = TCW == 4 && NS == 3 && TPS == 3 && WST == 0 && HS == 0 && !UPF;
  const int R = ((PART || FINE) && a.src_br > BR) ? a.src_br / BR : 1;
  const char* wblk = reinterpret_cast<const char*>(a.wgt) + ((size_t)(ct / R) * ST * KS + (size_t)kslice * S) * SLOT * R +
                     (size_t)(ct % R) * WSLOT;
  const uint32_t wlane = (lane >> 2) * 64 + (((lane & 3) ^ ((lane >> 3) & 3)) << 4);
  const char* in = reinterpret_cast<const char*>(a.in);
  const char* zero = reinterpret_cast<const char*>(a.zero);

  auto tile_of = [&](int i, int& n, int& ty, int& tx) {
    int mt = slot + i * n_slots;
    if (PART) mt /= KS;
    tx = mt % a.tiles_x;
    mt /= a.tiles_x;
    ty = mt % a.tiles_y;
    n = mt / a.tiles_y;
  };
  // sequential cursors, as in the 4-wave ring (per-lane halo pointers computed once per tile)
  const char* hsrc[HI];
  int hq_i = 0, hq_c = 0, hq_seq = 0;
  auto issue_halo = [&]() {
    if (hq_c == 0) {
      int n, ty, tx;
      tile_of(hq_i, n, ty, tx);
      const long long pix0 = (long long)(n * H + ty * 16) * W + tx * TW;
#pragma unroll
      for (int j = 0; j < HI; ++j) {
        const int row = (wave * HI + j) * 16 + (lane >> 2);
        const int hy = row / HWD, hx = row - (row / HWD) * HWD;
        const int iy = ty * 16 + hy - 1, ix = tx * TW + hx - 1;
        const bool ok = row < HP && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const int chk = ((lane & 3) ^ (hx & 3)) << 4;
        const long long pix = pix0 + (long long)(hy - 1) * W + (hx - 1);
        // (+ the K slice's first chunk; the zero page covers all 32 chunks of a 1024-channel input)
        hsrc[j] = (ok ? in + pix * a.ldi * (long long)sizeof(T) + chk : zero + chk) + c_lo * 64;
      }
    }
    const uint32_t dst = lds0 + (hq_seq & 1) * HALO_BYTES + wave * HI * 1024;
    // (ablation 8, timing only: every chunk of a 128-byte line loads the line's first 64 bytes, so each
    // line of the halo is fetched once -- wrong values, the cost of the sibling-chunk re-fetch)
    // (ablation 9: odd chunks issue no halo DMA at all -- their taps read the stale buffer; the counted
    // waits then wait for younger loads only, which is safe: timing only)
    const int hoff = ABL == 8 ? (hq_c & ~1) * 64 : hq_c * 64;
    if (ABL != 9 || (hq_c & 1) == 0) {
#pragma unroll
      for (int j = 0; j < HI; ++j) glds16_s(hsrc[j] + hoff, dst + j * 1024);
    }
    ++hq_seq;
    if (++hq_c == nch) { hq_c = 0; ++hq_i; }
  };
  // weights of step s into LDS slot `dst_slot` (this wave's pieces)
  auto issue_w_step = [&](int s, int dst_slot) {
    const char* src = wblk + (size_t)s * SLOT * R;
    const uint32_t dst = lds0 + WOFF + dst_slot * SLOT;
#pragma unroll
    for (int k = 0; k < (PIECES + NW - 1) / NW; ++k) {
      const int j = wave + k * NW;
      // piece j = 16 rows of tap j / PPT (PPT = pieces per tap); with R > 1 the packed taps are R times apart
      constexpr int PPT = WSLOT / 1024;
      const int off = (PART || FINE) ? (j / PPT) * WSLOT * R + (j % PPT) * 1024 : j * 1024;
      // wave-uniform; no test at all when every wave has the same count (straight-line issue: the
      // compiler had moved the tested pieces out of line, a taken branch each)
      if (PIECES % NW == 0 || j < PIECES) glds16_sv(src + off, wlane, dst + j * 1024);
    }
  };
  int wq_s = 0, wq_slot = 0;
  auto issue_w = [&]() {
    issue_w_step(wq_s, wq_slot);
    if (++wq_s == ST) wq_s = 0;
    if (++wq_slot == NS) wq_slot = 0;
  };

  f32x4 acc[TC][TP];
  const int col = lane & 15, q = lane >> 4;
  // Every tile's accumulators start at the layer bias (rows 64h + 16q + 4t + e of the lane, the packed
  // row permutation) instead of zero: the same number of register moves as the zeroing, and the
  // epilogue loses its bias add (one VALU op per output value).  bias_s must be visible (written in
  // the prologue, before its barrier).
  auto init_acc_bias = [&](int t0, int t1) {
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      if (t < t0 || t >= t1) continue;
      const f32x4 b4 = PART ? f32x4{0.f, 0.f, 0.f, 0.f}
                            : *reinterpret_cast<const f32x4*>(bias_s + 64 * (t / 4) + 16 * q + 4 * (t % 4));
#pragma unroll
      for (int p = 0; p < TP; ++p) acc[t][p] = b4;
    }
  };
  int prow[TP];
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of_w<TW>((wp * TP + p) * 16 + col, py, px);
    prow[p] = (py * HWD + px) * 64;
  }
  const int px_lane = col & 7;
  const int wpos = (q ^ ((col >> 1) & 3)) << 4;
  const char* wrow = lds + WOFF + col * 64 + wpos;

  // ---- HS: fused first conv (down1.0) -> halo chunks (see ring_body) ----
  // window DMA of tile i: thread L < 360 copies input pixels (2*(L%18), +1) of window row L/18
  // (HS) the tile coordinates of the current and the next tile are derived once per tile (tile_of
  // is two scalar divisions) and handed to the window DMA and the halo computation
  struct TileXY { int n, ty, tx; };
  auto tile_xy = [&](int i) { TileXY t; tile_of(i, t.n, t.ty, t.tx); return t; };
  auto issue_xs = [&](int i, const TileXY& tc) {   // -> window buffer i & 1
    if constexpr (HS != 0) {
      const int n = tc.n, ty = tc.ty, tx = tc.tx;
      const int L = tid;
      if (L < 20 * (G::XW / 2)) {   // lanes past the window stay inactive (no LDS write)
        const int yy = L / (G::XW / 2), seg = L - (L / (G::XW / 2)) * (G::XW / 2);
        const int iy = ty * 16 + yy - 2, ix = tx * TW + 2 * seg - 2;
        const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const char* src = ok ? reinterpret_cast<const char*>(a.x0) + ((long long)(n * H + iy) * W + ix) * 4 * sizeof(T)
                             : zero;
        glds16_s(src, lds0 + G::XS_OFF + (i & 1) * G::XS1 + wave * 1024);
      }
    }
  };
  uint2 w0f[2][2][3];
  float b0v[2][8];
  int toff[3];   // byte offset of this lane's tap in the window, per MFMA (-1: zero tap)
  if constexpr (HS != 0) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int m = 0; m < 3; ++m)
          w0f[cb][t][m] = *reinterpret_cast<const uint2*>(
              reinterpret_cast<const char*>(a.w0p) + ((((cb * 2 + t) * 3 + m) * 16 + (lane & 15)) * 16 + 4 * (lane >> 4)) * sizeof(T));
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int j = 0; j < 8; ++j) b0v[cb][j] = a.b0[32 * cb + 8 * (lane >> 4) + j];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int ta = first_tap_addr(4 * m + (lane >> 4));   // bit 0: a zero slot
      toff[m] = ((ta / 3) * G::XW + ta % 3) * 4 * (int)sizeof(T) + (first_tap(4 * m + (lane >> 4)) > 8 ? 1 : 0);
    }
  }
  // The computed halo's LDS image: quarter q of halo pixel (hy, hx) at q ^ (hx & 3) ^ (hy & 1) (the
  // DMA'd halo of the other layers has no hy term).  A 16-pixel group of the halo computation is
  // 2 rows x 8 pixels, rows (hy, hy + 3) -- lanes 0-3 / 4-7 at hx 0-3, 8-11 / 12-15 at hx 4-7 --
  // so that every 8-lane group of its ds_write_b128 covers 8 distinct 16-byte slots of a 128-byte
  // bank row (consecutive pixels of one row cover 4: 2-way conflicted, 10.5 % of the layer's LDS
  // cycles in r2p), while the taps' ds_read_b128 and the window's ds_read_b64 (the two rows
  // 3 x 288 B apart) stay conflict-free; the last two halo columns (36 pixels) follow in 3 groups
  // of row-consecutive pairs.  Rows paired: (0,3) (1,4) (2,5) (6,9) ... (14,17).
  // tools/halo_swizzle_search.py: no XOR table makes row-consecutive writes conflict-free as well.
  constexpr int HGR = (HP + 15) / 16;                     // 16-pixel groups of the halo
  constexpr int HIT = (HGR + 2 * NW - 1) / (2 * NW);      // groups per wave and part
  static_assert(HS == 0 || (HWD == 34 && HGR == 39), "computed halo groups: 9 row pairs x 4 + 3");
  // cb (the 32-channel chunk: selects w0f / b0v) and part are compile-time (std::integral_constant):
  // with runtime values the two register arrays are indexed dynamically and go to scratch.
  auto compute_halo = [&](int i, const TileXY& tc, auto cbc, int hb, auto partc) {
    constexpr int cb = decltype(cbc)::value, part = decltype(partc)::value;
    if constexpr (HS != 0) {
      const int ty = tc.ty, tx = tc.tx;
      const char* xs = lds + G::XS_OFF + (i & 1) * G::XS1;
      char* dst = lds + hb * HALO_BYTES;
      const int qq = lane >> 4, c = lane & 15;
      // The first conv's accumulators start at its bias (as first_conv_mfma_kernel's, so the fused
      // and unfused first convs agree bitwise), and a tile whose whole halo lies inside the image
      // (most of them) takes a path without the zero-padding select: 16 fewer VALU ops per group.
      auto groups = [&](auto borderc) {
        constexpr bool border = decltype(borderc)::value;
#pragma unroll
        for (int it = 0; it < HIT; ++it) {
          const int grp = wave + part * NW + it * 2 * NW;
          if (grp >= HGR) break;   // wave-uniform
          bool real = true;
          int hy, hx;
          if (grp < 36) {          // wave-uniform
            const int rp = grp >> 2;
            hy = 6 * (rp / 3) + rp % 3 + 3 * ((c >> 2) & 1);
            hx = 8 * (grp & 3) + (c & 3) + 4 * (c >> 3);
          } else {
            const int k = (grp - 36) * 16 + c;
            real = k < 36;
            hy = real ? k >> 1 : 0;
            hx = 32 + (k & 1);
          }
          const char* px = xs + (hy * G::XW + hx) * 4 * (int)sizeof(T);
          f32x4 acc0[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) acc0[t] = f32x4{b0v[cb][4 * t], b0v[cb][4 * t + 1], b0v[cb][4 * t + 2], b0v[cb][4 * t + 3]};
#pragma unroll
          for (int m = 0; m < 3; ++m) {
            uint2 bv = *reinterpret_cast<const uint2*>(px + (toff[m] & ~1));
            if (toff[m] & 1) bv = uint2{0u, 0u};   // 0 x (a NaN input) must stay 0
#pragma unroll
            for (int t = 0; t < 2; ++t) acc0[t] = mfma16<T>(w0f[cb][t][m], bv, acc0[t]);
          }
          bool inimg = true;
          if constexpr (border) {
            const int iy = ty * 16 + hy - 1, ix = tx * TW + hx - 1;
            inimg = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
          }
          typedef T t8 __attribute__((ext_vector_type(8)));
          t8 o;
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) o[4 * t + e] = (T)(inimg ? relu_nan(acc0[t][e]) : 0.f);
          if (real)
            *reinterpret_cast<uint4*>(dst + (hy * HWD + hx) * 64 + ((qq ^ (hx & 3) ^ (hy & 1)) << 4)) =
                __builtin_bit_cast(uint4, o);
        }
      };
      const bool interior = ty > 0 && tx > 0 && ty * 16 + 17 <= H && tx * TW + TW + 1 <= W;
      if (interior) groups(std::false_type{});
      else groups(std::true_type{});
    }
  };

  // prologue: halo of chunk 0; weights (all steps, or steps 0 .. NS-2); epilogue parameters
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  if constexpr (HS != 0) {
    const TileXY t0 = tile_xy(0);
    issue_xs(0, t0);
    wait_vm_barrier<0>();
    compute_halo(0, t0, C0{}, 0, C0{});
    compute_halo(0, t0, C0{}, 0, C1{});
  } else {
    issue_halo();
  }
  if constexpr (WST) {
    for (int s = 0; s < S; ++s) issue_w_step(s, s);
  } else {
#pragma unroll
    for (int k = 0; k < NS - 1; ++k)
      if (k < total) issue_w();
  }
  for (int i = tid; i < BR; i += 64 * NW) bias_s[i] = a.bias[ct * BR + i];
  if (EPI == EPI_HEAD) {
    for (int i = tid; i < a.ncls * 64; i += 64 * NW) headw_s[i] = a.head_w[i];
    if (tid < a.ncls) headb_s[tid] = a.head_b[tid];
  }
  // EPI_UPFUSE: the ConvTranspose bias (4 quadrants x 64 rows) in the head's LDS space.  Read
  // from global inside the quadrant loop it cost a vmcnt wait there -- in-order, so a drain of
  // every DMA in flight and of the previous quadrants' scatter stores, four times per tile.
  static_assert(kMaxClasses * 64 >= 4 * 64, "up1 bias in the head parameter space");
  if (UPF)
    for (int i = tid; i < 4 * 64; i += 64 * NW) headw_s[i] = a.bias2[i];
  if constexpr (WST) {
    wait_vm_barrier<0>();
  } else {
    const int young = total - 1 < NS - 2 ? total - 1 : NS - 2;   // W(1..NS-2) may stay in flight
    wait_vm_barrier_rt(young * wcnt);
  }
  init_acc_bias(0, TC);

  auto step = [&](int g, int hs, int tp, int tsub) {
    const int dy = tp / 3, dx = tp - (tp / 3) * 3;
    const char* Hs = lds + (hs & 1) * HALO_BYTES + (dy * HWD + dx) * 64 + ((q ^ ((px_lane + dx) & 3)) << 4);
    const int ws = WST ? g - (g / S) * S : g % NS;
    const char* Ws = wrow + ws * SLOT + tsub * WSLOT;
    frag_t bq[TP], ar[3];
#pragma unroll
    for (int p = 0; p < TP; ++p) bq[p] = *reinterpret_cast<const frag_t*>(Hs + prow[p]);
    ar[0] = *reinterpret_cast<const frag_t*>(Ws);
    if (TC > 1) ar[1] = *reinterpret_cast<const frag_t*>(Ws + 16 * 64);
    __builtin_amdgcn_sched_group_barrier(0x100, TP + (TC > 1 ? 2 : 1), 0);
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      if (t + 2 < TC) ar[(t + 2) % 3] = *reinterpret_cast<const frag_t*>(Ws + (t + 2) * 16 * 64);
      const frag_t af = ar[t % 3];
#pragma unroll
      for (int p = 0; p < TP; ++p)
        mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, bq[p]));
      if (t + 2 < TC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TP, 0);
    }
  };

  if constexpr (HS != 0) {
    // Fused first conv (down1.3, Cin = 64: two halo chunks, buffer c for chunk c; weights
    // stationary; the input window double-buffered, tile i in window i & 1).  A tile's 18 taps
    // run as two pipelined 9-tap phases (one per chunk) with ONE barrier each (instead of one per
    // 3-tap step):
    //   1: the next tile's window DMA'd | chunk 1's halo computed from this tile's window | the
    //      nine taps of chunk 0  -> vmcnt(0) + barrier (window landed; chunk 1's halo visible;
    //      every read of halo buffer 0 done)
    //   2: the next tile's chunk-0 halo computed into buffer 0 | the nine taps of chunk 1
    //      -> barrier (visible to the next tile's phase 1; every read of buffer 1 done)
    // A window buffer is re-filled one tile after its last read (two barriers later).  Each wave
    // computes its share of a halo after the phase's MFMAs (profiles/tune_r2j_fused_phases.txt:
    // computing it before them on waves 0-3, so that the two waves of a SIMD overlap halo work
    // with MFMAs, and three 6-tap phases per tile instead of two, were no faster).
    auto taps9 = [&](int ch) {   // the nine taps of chunk ch (halo buffer ch, weight steps 3ch .. 3ch+2)
      const char* hs9[9];
      const char* ws9[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {   // halo row of the lane's pixel: (col >> 3) + row (mod 2)
        const int row = k / 3, dx = k % 3;
        hs9[k] = lds + ch * HALO_BYTES + (row * HWD + dx) * 64 +
                 ((q ^ ((px_lane + dx) & 3) ^ (((col >> 3) + row) & 1)) << 4);
        ws9[k] = wrow + (ch * 3 + row) * SLOT + dx * WSLOT;
      }
      mfma_taps<T, TC, TP, 9>(acc, hs9, ws9, prow);
    };
    auto halo_all = [&](int i, const TileXY& tc, auto cbc) {   // both halves of chunk cb of tile i -> buffer cb
      compute_halo(i, tc, cbc, decltype(cbc)::value, C0{});
      compute_halo(i, tc, cbc, decltype(cbc)::value, C1{});
    };
    TileXY cur = tile_xy(0);
    for (int item = 0; item < items; ++item) {
      const bool more = item + 1 < items;
      const TileXY nxt = more ? tile_xy(item + 1) : cur;
      if (more) issue_xs(item + 1, nxt);
      taps9(0);
      halo_all(item, cur, C1{});
      wait_vm_barrier<0>();
      taps9(1);
      if (more) halo_all(item + 1, nxt, C0{});
      wait_vm_barrier<63>();   // barrier only: no load is waited for here
#pragma unroll
      for (int h = 0; h < TC / 4; ++h)
        conv_epilogue<TO, TQ, TP, EPI, TW, 0, 1>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), cur.n,
                                                 cur.ty * 16, cur.tx * TW, wp * TP, ct * BR + 64 * h, bias_s + 64 * h,
                                                 headw_s, headb_s);
      init_acc_bias(0, TC);
      cur = nxt;
    }
    return;
  }
  frag_t xb[UPF ? TP : 1][UPF ? 4 : 1];   // EPI_UPFUSE: see ring_body
  // EPI_UPFUSE: quadrant quad's accumulators (acc[0..3]) start at the ConvTranspose bias of its 64
  // rows (headw_s + 64 quad, rows 16q + 4t + e of the lane), so its scatter epilogue adds none
  auto init_up_bias = [&](int quad) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(headw_s + 64 * quad + 16 * q + 4 * t);
#pragma unroll
      for (int p = 0; p < TP; ++p) acc[t][p] = b4;
    }
  };
  auto conv_to_xb = [&]() {
    if constexpr (UPF) {
      typedef T t8 __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int p = 0; p < TP; ++p) {   // the accumulators hold the bias (init_acc_bias)
            t8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (T)relu_nan(acc[4 * h + 2 * half + (j >> 2)][p][j & 3]);
            xb[p][2 * h + half] = __builtin_bit_cast(frag_t, v);
          }
        }
      init_up_bias(0);
    }
  };
  auto stepT = [&](int g, bool dma) {   // one quadrant: acc[t] += A(kb, t) x xb[kb], kb = 0..3 (the ring's K order)
    if constexpr (UPF) {
      const char* Ws = wrow + (g % NS) * SLOT;
      frag_t ar[3];
      ar[0] = *reinterpret_cast<const frag_t*>(Ws);
      ar[1] = *reinterpret_cast<const frag_t*>(Ws + 16 * 64);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int j = 0; j < 16; ++j) {   // j = 4 kb + t
        if (j + 2 < 16) ar[(j + 2) % 3] = *reinterpret_cast<const frag_t*>(Ws + (j + 2) * 16 * 64);
        const frag_t af = ar[j % 3];
#pragma unroll
        for (int p = 0; p < TP; ++p)
          mfma_frag<T>(acc[j & 3][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, xb[p][j >> 2]));
        if (j + 2 < 16) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, TP, 0);
        if (j == 1 && dma) issue_w();   // the step's weight DMA under the first MFMAs (as the conv steps)
      }
    }
  };
  static_assert(WST || SPC >= NS - 1, "see ring_body");
  int wskip = 0;
  int c = 0, tap = 0, hseq = 0, item = 0;   // tap = step index within the chunk (0 .. SPC-1)
  for (int g = 0; g < total; ++g) {
    const bool hnext = tap == 0 && hseq + 1 < hseq_end;
    // the next chunk's halo is issued AFTER this step's weights: vmcnt retires in issue order, so
    // the halo then stays in flight through the wait for W(g+2) too (NS - 1 steps of latency
    // instead of NS - 2; it is needed only at the chunk end)
    // this step's LDS-DMA (W(g+NS-1), then the next chunk's halo): issued from inside the tap
    // sequence, after its first MFMAs (mfma_taps* `mid`); the step paths without a hook issue it here
    const bool dma_w = ABL != 4 && !WST && g + NS - 1 < total, dma_h = ABL != 4 && HS == 0 && hnext;
    auto dma = [&]() {
      if (dma_w) issue_w();
      if (dma_h) issue_halo();
    };
    // (TPS = 9, conv1.0's two-slot ring: the next step's DMA has one step of cover only, so it is
    // issued first, as before: from inside the taps it measured +0.8 %, profiles/tune_r3z_*)
    if constexpr (!((WST && HS == 0 && TPS == 3 && TC * TP % (TC + TP) == 0) || TPS == 3)) dma();
    if constexpr (WST && HS == 0 && TPS == 3 && TC * TP % (TC + TP) == 0) {
      // weight-stationary, DMA'd halo: no barrier inside a chunk, so its nine taps (three steps)
      // run as one pipelined sequence at the chunk's first step; the other two only keep count
      if (tap == 0) {
        const int ws0 = g - (g / S) * S;   // first step of the chunk within the tile
        const char* hs9[9];
        const char* ws9[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) {   // tap (dy, dx) = (k / 3, k % 3)
          const int dy = k / 3, dx = k % 3;
          hs9[k] = lds + (hseq & 1) * HALO_BYTES + (dy * HWD + dx) * 64 + ((q ^ ((px_lane + dx) & 3)) << 4);
          ws9[k] = wrow + (ws0 + dy) * SLOT + dx * WSLOT;
        }
        mfma_taps<T, TC, TP, 9>(acc, hs9, ws9, prow, dma);
      } else {
        dma();
      }
    } else if constexpr (TPS == 9) {
      // one step = a whole 32-channel chunk (nine taps, one barrier): the weights of the next chunk
      // (36 KB) and its halo load during this one (2-slot ring), and all nine taps are pipelined
      const char* hs9[9];
      const char* ws9[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {   // tap (dy, dx) = (k / 3, k % 3)
        const int dy = k / 3, dx = k % 3;
        hs9[k] = lds + (hseq & 1) * HALO_BYTES + (dy * HWD + dx) * 64 + ((q ^ ((px_lane + dx) & 3)) << 4);
        ws9[k] = wrow + (g % NS) * SLOT + k * WSLOT;
      }
      mfma_taps<T, TC, TP, 9>(acc, hs9, ws9, prow);
    } else if constexpr (TPS == 3) {
      const int wslot = WST ? g - (g / S) * S : g % NS;
      const char* hs3[3];
      const char* ws3[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {   // taps (dy = tap, dx = t): one kernel row
        hs3[t] = lds + (hseq & 1) * HALO_BYTES + (tap * HWD + t) * 64 + ((q ^ ((px_lane + t) & 3)) << 4);
        ws3[t] = wrow + wslot * SLOT + t * WSLOT;
      }
      if constexpr (TC * TP % (TC + TP) == 0) mfma_taps<T, TC, TP, 3>(acc, hs3, ws3, prow, dma);
      else mfma_taps_astream<T, TC, TP, 3, (ABL == 2 || ABL == 3) ? ABL : 0>(acc, hs3, ws3, prow, dma);
    } else {
#pragma unroll
      for (int t = 0; t < TPS; ++t) step(g, hseq, tap * TPS + t, t);
    }
    const bool chunk_end = tap == SPC - 1;
    if constexpr (WST) {
      // only the halo streams: the next chunk's halo (issued at this chunk's first step) must
      // have landed, and every wave must be done with this chunk's halo before the next issue
      if (chunk_end) wait_vm_barrier<0>();
    } else {
      // W(g+1) must have landed (and, at a chunk end, the next halo -- issued SPC-1 steps
      // earlier, older than W(g+1)).  Younger loads may stay in flight: W(g+2 .. g+NS-1) and a
      // halo issued within the last NS-1 steps (after W(g+1) -- issued NS-2 steps ago).
      int young = total - 2 - g;
      young = young < 0 ? 0 : (young > NS - 2 ? NS - 2 : young);
      const bool hyoung = tap < NS - 1 && tap < SPC - 1 && hseq + 1 < hseq_end;
      if (wskip > 0 && ABL != 1) { --wskip; wait_vm_barrier<63>(); }   // see ring_body
      else loop_wait(young, hyoung);
    }
    bool tile_end = false;
    if (++tap == SPC) {
      tap = 0;
      ++hseq;
      if (++c == nch) {
        c = 0;
        tile_end = true;
      }
    }
    if (UPF && tile_end) {   // the tile's SU ConvTranspose steps, right here (see ring_body)
      conv_to_xb();
      int n, ty, tx;
      tile_of(item, n, ty, tx);
#pragma nounroll
      for (int quad = 0; quad < SU; ++quad) {
        ++g;
        stepT(g, g + NS - 1 < total);
        int young = total - 2 - g;
        young = young < 0 ? 0 : (young > NS - 2 ? NS - 2 : young);
        if (wskip > 0) { --wskip; wait_vm_barrier<63>(); }
        else loop_wait(young, false);   // the last halo issue is older than W(g+1)
        // no vmcnt(0) drain: the stores retire under the next step's wait (see ring_body)
        conv_epilogue<TO, TO, TP, EPI_UPSCATTER, TW, 0, 1>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[0]), n,
                                                           ty * 16, tx * TW, wp * TP, 64 * quad, nullptr, nullptr,
                                                           nullptr, a.out2, a.ldo2, a.Cout / 2);
        init_up_bias((quad + 1) & 3);   // (after the last quadrant: overwritten by init_acc_bias below)
      }
      init_acc_bias(0, TC);   // the next tile's conv accumulators (acc[0..3] held the ConvTranspose quadrants)
      ++item;
      continue;
    }
    if (tile_end) {
      int n, ty, tx;
      tile_of(item, n, ty, tx);
      // No vmcnt(0) drain before the stores (the 4-wave ring's habit): with one block per CU that
      // drain (the next steps' weights and halo, issued up to NS-1 steps ahead) is exposed once per
      // tile.  The stores are issued after those loads, so the next step's counted wait (for loads
      // issued after them) retires them under that step's MFMAs.
#pragma unroll
      for (int h = 0; h < TC / 4; ++h) {
        if constexpr (PART) {
          partial_store<TP, TW>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n, ty * 16, tx * TW, wp * TP,
                                ct * BR + 64 * h, kslice);
        } else if constexpr (ABL == 5) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int p = 0; p < TP; ++p) asm volatile("" ::"v"(acc[4 * h + t][p]));
        } else if constexpr (ABL == 6 || ABL == 7) {   // 6: arithmetic without stores; 7: stores without arithmetic
          if constexpr (ABL == 7)   // the accumulators stay alive (else the MFMAs are dead code)
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
              for (int p = 0; p < TP; ++p) asm volatile("" ::"v"(acc[4 * h + t][p]));
          conv_epilogue<TO, TQ, TP, EPI, TW, ABL == 6 ? 1 : 2, 1>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n,
                                                               ty * 16, tx * TW, wp * TP, ct * BR + 64 * h, bias_s + 64 * h,
                                                               headw_s, headb_s);
        } else {
          conv_epilogue<TO, TQ, TP, EPI, TW, 0, 1>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n, ty * 16,
                                                   tx * TW, wp * TP, ct * BR + 64 * h, bias_s + 64 * h, headw_s,
                                                   headb_s);
        }
      }
      init_acc_bias(0, TC);
      ++item;
    }
  }
}

template <typename T, int TCW, int NS, int EPI, int TPS, int WST, typename TO, typename TQ, int HS = 0, int ABL = 0>
static hipError_t launch_ring8(const IgemmArgs& a, hipStream_t s) {
  using G = Ring8Geom<T, TCW, NS, TPS, WST, HS>;
  if constexpr (HS != 0) {
    if (a.Cin != 2 * G::BKE || a.c0 < 1 || a.c0 > 3 || !a.x0 || !a.w0p || !a.b0) return hipErrorInvalidValue;
  }
  if (a.tiles_y != (a.H + 15) / 16 || a.tiles_x != (a.W + G::TW - 1) / G::TW) return hipErrorInvalidValue;
  if (a.Cin % G::BKE || a.Ctot % G::BR || a.n_ct != a.Ctot / G::BR) return hipErrorInvalidValue;
  if (WST && (9 / TPS) * (a.Cin / G::BKE) > G::WST_STEPS) return hipErrorInvalidValue;
  const int KS = EPI == EPI_PARTIAL ? a.ksplit : 1;
  if (KS < 1 || a.Cin % (G::BKE * KS) || (EPI == EPI_PARTIAL && !a.part)) return hipErrorInvalidValue;
  constexpr bool fine = TCW == 4 && NS == 3 && TPS == 3 && WST == 0 && HS == 0 && EPI != EPI_UPFUSE;
  if (a.src_br && (!(EPI == EPI_PARTIAL || fine) || a.src_br % G::BR || a.Ctot % a.src_br)) return hipErrorInvalidValue;
  const int n_mt = a.N * a.tiles_y * a.tiles_x * KS;   // items: (pixel tile, K slice)
  int n_slots = kNumCUs / a.n_ct;   // one 512-thread block per CU
  n_slots -= n_slots % KS;          // every walker keeps one K slice (n_mt is a multiple of KS)
  if (n_slots < KS) n_slots = KS;
  if (n_slots > n_mt) n_slots = n_mt;
  hipLaunchKernelGGL((conv3x3_ring8_kernel<T, TCW, NS, EPI, TPS, WST, TO, TQ, HS, ABL>), dim3(a.n_ct * n_slots), dim3(512),
                     0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// ConvTranspose2d(k2, s2) as a persistent ring GEMM (up4 .. up1)
// ---------------------------------------------------------------------------------
// GEMM rows = (a, b, cout) (4 * Cout, packed per 128-row tile in step order like the 3x3 ring),
// K = Cin in 64-byte steps, columns = a 16x16 input-pixel tile; the pixel-shuffle store of the
// shared epilogue writes output pixels (2y+a, 2x+b) into the concat buffer.  K is short (2..32
// steps per tile at 64 B), so instead of the halo kernel's one-tile-per-block prologue both
// operands stream through ONE NS-slot LDS-DMA ring that runs across tile boundaries of a
// persistent walker: the next tile's first steps load during this tile's last MFMAs and its
// scatter epilogue.  LDS per slot: A [BR][64 B] (chunk q of row r at q ^ ((r >> 1) & 3)) +
// B [256 px][64 B] (pixel row py*16+px, chunk q at q ^ ((py & 1) << 1): conflict-free for all
// ds_read_b128 lane groups and pixel groups, checked exhaustively).
// WRW = 2: 8 waves as 2 (rows) x 4 (pixels), a 256-row x 256-pixel block tile (one block per
// CU): half the A + B LDS-DMA bytes per MFMA of the 128-row tile (the large-Cin layers up4/up3
// stream both operands from L2 at every step).  TO: element type of the scattered output.
template <typename T, int TCW, int NS, int WRW = 1, typename TO = T>
__global__ __launch_bounds__(256 * WRW, WRW == 1 ? 2 : 1) void convT_ring_kernel(const IgemmArgs a) {
  constexpr int NW = 4 * WRW, TC = TCW, TP = 4, BR = 16 * TC * WRW, BKE = 64 / (int)sizeof(T);
  constexpr int WI = BR / (16 * NW);          // A DMA instructions per wave and step
  constexpr int BI = 256 / (16 * NW);         // B DMA instructions per wave and step
  constexpr int ASLOT = BR * 64, BSLOT = 256 * 64, SLOT = ASLOT + BSLOT;
  static_assert((NS == 3 || NS == 4) && TC % 4 == 0, "ring depth / row tile");
  static_assert(NS * SLOT + BR * 4 <= 160 * 1024 / (WRW == 1 ? 2 : 1), "blocks per CU");
  __shared__ __attribute__((aligned(16))) char lds[NS * SLOT];
  // the walker's row-tile bias, for the epilogue: read from global there, its vmcnt wait (in
  // order) drained every DMA in flight and the previous pixel groups' scatter stores per tile
  __shared__ __attribute__((aligned(16))) float bias_s[BR];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const uint32_t lds0 = lds_addr_of(lds);
  const int wr = wave >> 2, wp = wave & 3;   // row group (WRW = 2), pixel group
  int bid;
  {  // XCD-contiguous remap; consecutive ids = the n_ct row tiles of one walker
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7;
    const int b = blockIdx.x, x = b & 7, k = b >> 3;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  const int ct = bid % a.n_ct;                      // row tile of this walker
  const int slot = bid / a.n_ct;
  const int n_slots = gridDim.x / a.n_ct;
  const int n_mt = a.N * a.tiles_y * a.tiles_x;
  if (slot >= n_mt) return;
  const int items = (n_mt - slot + n_slots - 1) / n_slots;
  const int H = a.H, W = a.W;
  const int S = a.Cin / BKE;
  const int total = items * S;

  const char* wblk = reinterpret_cast<const char*>(a.wgt) + wave * WI * 16 * 64;   // wave-uniform (glds16_sv)
  const uint32_t wlane = (lane >> 2) * 64 + (((lane & 3) ^ ((lane >> 3) & 3)) << 4);
  const char* in = reinterpret_cast<const char*>(a.in);
  const char* zero = reinterpret_cast<const char*>(a.zero);
  auto tile_of = [&](int i, int& n, int& ty, int& tx) {
    int mt = slot + i * n_slots;
    tx = mt % a.tiles_x;
    mt /= a.tiles_x;
    ty = mt % a.tiles_y;
    n = mt / a.tiles_y;
  };
  // Steps are issued strictly in order, so the issue side keeps cursors instead of dividing g by S
  // and re-deriving the tile per step (two scalar divisions and 64-bit VALU address math per piece,
  // round 3): at a tile's first step the B pieces' per-lane pointers are set once (the zero page for
  // pixels outside the image -- 4 KB, so + c * 64 stays inside it), every step adds c * 64.
  int iss_c = 0, iss_i = 0, iss_slot = 0;
  const char* bsrc[BI];
  // (batch-1 plan: 128-row tiles over the 256-row packing, a.src_br = 256 -- row tile ct is half ct % R of
  // packed row tile ct / R, whose steps are R times longer)
  const int R = (WRW == 1 && a.src_br > BR) ? a.src_br / BR : 1;
  const char* wct = wblk + (size_t)(ct / R) * S * ASLOT * R + (size_t)(ct % R) * ASLOT;
  auto issue = [&]() {
    const uint32_t As = lds0 + iss_slot * SLOT;
#pragma unroll
    for (int j = 0; j < WI; ++j)
      glds16_sv(wct + (size_t)iss_c * ASLOT * R + j * 1024, wlane, As + (wave * WI + j) * 1024);
    if (iss_c == 0) {
      int n, ty, tx;
      tile_of(iss_i, n, ty, tx);
#pragma unroll
      for (int j = 0; j < BI; ++j) {
        const int r = (wave * BI + j) * 16 + (lane >> 2), py = r >> 4, px = r & 15;
        const int iy = ty * 16 + py, ix = tx * 16 + px;
        const int chk = ((lane & 3) ^ ((py & 1) << 1)) << 4;
        const bool ok = iy < H && ix < W;
        bsrc[j] = ok ? in + ((long long)(n * H + iy) * W + ix) * a.ldi * (long long)sizeof(T) + chk : zero + chk;
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) glds16_s(bsrc[j] + iss_c * BKE * (int)sizeof(T), As + ASLOT + (wave * BI + j) * 1024);
    if (++iss_slot == NS) iss_slot = 0;
    if (++iss_c == S) { iss_c = 0; ++iss_i; }
  };

  // Every tile's accumulators start at the ConvTranspose bias (rows wr*16*TC + 64h + 16q + 4t + e of
  // the lane, the packed row permutation) instead of zero, as in the 8-wave ring: the epilogue
  // loses its bias add.  bias_s is visible after the prologue's barrier.
  f32x4 acc[TC][TP];
  const int col = lane & 15, q = lane >> 4;
  auto init_acc_bias = [&]() {
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias_s + wr * 16 * TC + 64 * (t / 4) + 16 * q + 4 * (t % 4));
#pragma unroll
      for (int p = 0; p < TP; ++p) acc[t][p] = b4;
    }
  };
  int prow[TP];
#pragma unroll
  for (int p = 0; p < TP; ++p) {
    int py, px;
    pix_of((wp * TP + p) * 16 + col, py, px);
    prow[p] = (py * 16 + px) * 64 + ((q ^ ((py & 1) << 1)) << 4);
  }
  const int wrow = (wr * 16 * TC + col) * 64 + ((q ^ ((col >> 1) & 3)) << 4);

#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (k < total) issue();
  for (int i = tid; i < BR; i += 64 * NW) bias_s[i] = a.bias[ct * BR + i];   // (the wait below covers it)
  {   // step 0 landed; steps 1 .. NS-2 may stay in flight
    const int young = total - 1 < NS - 2 ? total - 1 : NS - 2;
    if (young == 2) wait_vm_barrier<2 * (WI + BI)>(); else if (young == 1) wait_vm_barrier<WI + BI>(); else wait_vm_barrier<0>();
  }
  init_acc_bias();

  int c = 0, item = 0, wskip = 0;
  for (int g = 0; g < total; ++g) {
    // this step's LDS-DMA (step g+NS-1, into the slot step g-1 released) is issued after the first two
    // row groups' MFMAs, so it runs while they execute (as in the 8-wave ring, round 3)
    const bool dma = g + NS - 1 < total;
    const char* As = lds + (g % NS) * SLOT + wrow;
    const char* Bs = lds + (g % NS) * SLOT + ASLOT;
    frag_t bq[TP], ar[3];
#pragma unroll
    for (int p = 0; p < TP; ++p) bq[p] = *reinterpret_cast<const frag_t*>(Bs + prow[p]);
    ar[0] = *reinterpret_cast<const frag_t*>(As);
    ar[1] = *reinterpret_cast<const frag_t*>(As + 16 * 64);
    __builtin_amdgcn_sched_group_barrier(0x100, TP + 2, 0);
#pragma unroll
    for (int t = 0; t < TC; ++t) {
      if (t + 2 < TC) ar[(t + 2) % 3] = *reinterpret_cast<const frag_t*>(As + (t + 2) * 16 * 64);
      const frag_t af = ar[t % 3];
#pragma unroll
      for (int p = 0; p < TP; ++p)
        mfma_frag<T>(acc[t][p], __builtin_bit_cast(uint4, af), __builtin_bit_cast(uint4, bq[p]));
      if (t + 2 < TC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TP, 0);
      if (t == 1 && dma) issue();
    }
    // step g+1 must have landed; step g+2 (issued above) may stay in flight
    {   // step g+1 landed; steps g+2 .. g+NS-1 (issued) may stay in flight
      int young = total - 2 - g;
      young = young < 0 ? 0 : (young > NS - 2 ? NS - 2 : young);
      if (wskip > 0) { --wskip; wait_vm_barrier<63>(); }   // after an epilogue: see ring_body
      else if (young == 2) wait_vm_barrier<2 * (WI + BI)>(); else if (young == 1) wait_vm_barrier<WI + BI>(); else wait_vm_barrier<0>();
    }
    if (++c == S) {
      c = 0;
      int n, ty, tx;
      tile_of(item, n, ty, tx);
      // no vmcnt(0) drain before the stores with one block per CU (exposed): the next steps' counted
      // waits retire them (see conv3x3_ring8_kernel); the two-block configuration keeps the drain
      if (WRW == 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // steps g+2 .. g+NS-1 landed before the stores
        wskip = NS - 2;
      }
#pragma unroll
      for (int h = 0; h < TC / 4; ++h)
        conv_epilogue<TO, TO, TP, EPI_UPSCATTER, 16, 0, 1>(a, *reinterpret_cast<const f32x4(*)[4][TP]>(&acc[4 * h]), n,
                                                         ty * 16, tx * 16, wp * TP, ct * BR + wr * 16 * TC + 64 * h,
                                                         nullptr, nullptr, nullptr);
      init_acc_bias();
      ++item;
    }
  }
}

// ---------------------------------------------------------------------------------
// first conv: C in {1,3} input channels, fp32 NCHW in, 64 channels NHWC out.
// K = 9*C is far too short for MFMA; it is a VALU direct conv, bound by HBM
// (read 4*C B + write 64*sizeof(T) B per pixel).
// ---------------------------------------------------------------------------------
template <typename T, int C>
__global__ __launch_bounds__(256) void first_conv_kernel(const FirstConvArgs a) {
  constexpr int KW = 9 * C;
  __shared__ float ws[64 * KW];
  __shared__ float bs[64];
  __shared__ float xs_out[sizeof(T) == 4 ? 256 * 33 : 1];   // fp32: one 32-channel half of the block's outputs
  for (int i = threadIdx.x; i < 64 * KW; i += 256) ws[i] = a.w[i];
  if (threadIdx.x < 64) bs[threadIdx.x] = a.b[threadIdx.x];
  __syncthreads();
  const int total = a.N * a.H * a.W;   // <= 2^30 (unet_capi's shape check): 32-bit index math
  int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= total) {
    if constexpr (sizeof(T) != 4) return;
    pix = total - 1;   // (fp32: every thread reaches the block's barriers; its stores are masked)
  }
  const int x = pix % a.W;
  const int t = pix / a.W;
  const int y = t % a.H;
  const int n = t / a.H;
  float xin[KW];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = y + ky - 1, ix = x + kx - 1;
        const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        xin[(c * 3 + ky) * 3 + kx] = ok ? a.x[(((long long)n * C + c) * a.H + iy) * a.W + ix] : 0.f;
      }
  if constexpr (sizeof(T) == 4) {
    // fp32 out: 256 B per pixel.  A lane's own 64-byte stores would leave each store instruction scattered
    // over 64 pixels (16 KB); instead each 32-channel half goes through LDS and leaves as whole 128-byte
    // pixel runs, 8 lanes per pixel (round 6: the per-lane form moved 2.1 GB at ~2.6 TB/s)
    float* tile = xs_out;
    const int p0 = blockIdx.x * 256;
    const int npx = min(256, total - p0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const int co = h * 32 + e;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < KW; ++k) s = fmaf(ws[co * KW + k], xin[k], s);
        tile[threadIdx.x * 33 + e] = relu_nan(s + bs[co]);
      }
      __syncthreads();
      float* out = reinterpret_cast<float*>(a.out) + (long long)p0 * 64 + h * 32;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int u = it * 256 + threadIdx.x, px = u >> 3, c4 = (u & 7) * 4;
        if (px < npx) {
          const float* sp = tile + px * 33 + c4;
          *reinterpret_cast<f32x4*>(out + (long long)px * 64 + c4) = f32x4{sp[0], sp[1], sp[2], sp[3]};
        }
      }
      __syncthreads();
    }
  } else {
    T* dst = reinterpret_cast<T*>(a.out) + (long long)pix * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = g * 16 + e;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < KW; ++k) s = fmaf(ws[co * KW + k], xin[k], s);
        v[e] = relu_nan(s + bs[co]);
      }
      store16<T>(dst + g * 16, v);
    }
  }
}

// First conv on MFMA (16-bit types): K = 9*C <= 27 padded to 32 = ONE 16x16x32 MFMA per
// 16 pixels x 16 channels.  The fp32 input halo (18x18xC) is staged in LDS, B fragments are
// built per lane from it, and the 64 output channels go through the shared epilogue
// (bias + ReLU, 16-byte NHWC stores): the kernel is bound by the output write.
template <typename T, int C>
__global__ __launch_bounds__(256) void first_conv_mfma_kernel(const FirstConvArgs a, const IgemmArgs e) {
  __shared__ float xs[C * 18 * 18];
  __shared__ float bias_s[64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int H = a.H, W = a.W;
  int mt = blockIdx.x;
  const int tx = mt % e.tiles_x;
  mt /= e.tiles_x;
  const int ty = mt % e.tiles_y;
  const int n = mt / e.tiles_y;
  for (int i = tid; i < C * 324; i += 256) {
    const int c = i / 324, r = i - c * 324, hy = r / 18, hx = r - (r / 18) * 18;
    const int iy = ty * 16 + hy - 1, ix = tx * 16 + hx - 1;
    const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    xs[i] = ok ? a.x[(((long long)n * C + c) * H + iy) * W + ix] : 0.f;
  }
  if (tid < 64) bias_s[tid] = a.b[tid];
  // Three 16x16x16 MFMAs per 16 pixels x 16 channels with K slot 4q + c of MFMA m = (tap
  // first_tap(4m + q), channel c): the K order of the ring kernel's fused first conv, so both paths
  // agree bitwise.
  // A fragments (weights, a.wp = [t][m][16 rows][16 k]): row t*16 + (lane&15), k = 4q .. 4q+3
  const int q = lane >> 4, col = lane & 15;
  uint2 af[4][3];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 3; ++m)
      af[t][m] = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(a.wp) +
                                                 (((t * 3 + m) * 16 + col) * 16 + 4 * q) * sizeof(T));
  int toff[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int tp = first_tap(4 * m + q);
    toff[m] = tp < 9 ? (tp / 3) * 18 + tp % 3 : -1;
  }
  __syncthreads();
  f32x4 acc[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    int py, px;
    pix_of((wave * 4 + p) * 16 + col, py, px);
    const int base = py * 18 + px;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t][p] = *reinterpret_cast<const f32x4*>(bias_s + 16 * q + 4 * t);   // bias first
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      uint2 bv = uint2{0u, 0u};
      if constexpr (sizeof(T) == 2) {
        typedef T t4 __attribute__((ext_vector_type(4)));
        t4 h;
#pragma unroll
        for (int c = 0; c < 4; ++c) h[c] = (T)(c < C && toff[m] >= 0 ? xs[c * 324 + base + toff[m]] : 0.f);
        bv = __builtin_bit_cast(uint2, h);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t][p] = mfma16<T>(af[t][m], bv, acc[t][p]);
    }
  }
  conv_epilogue<T, T, 4, EPI_STORE, 16, 0, 1>(e, acc, n, ty * 16, tx * 16, wave * 4, 0, nullptr, nullptr, nullptr);
}

// ---------------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------------
template <typename T, int WR, int WPX, int TCW, int NS, int EPI, int KT>
static hipError_t launch_halo(const IgemmArgs& a, hipStream_t s) {
  using G = HaloGeom<T, WR, WPX, TCW, NS, KT>;
  if (a.tiles_y != (a.H + 15) / 16 || a.tiles_x != (a.W + 15) / 16) return hipErrorInvalidValue;
  if (a.Cin % G::BKE || a.Ctot % G::BR || a.n_ct != a.Ctot / G::BR) return hipErrorInvalidValue;
  const int KS = EPI == EPI_PARTIAL ? a.ksplit : 1;
  if (KS < 1 || a.Cin % (G::BKE * KS) || (EPI == EPI_PARTIAL && !a.part)) return hipErrorInvalidValue;
  // one block per (row tile, K slice, pixel tile)
  const long long nb = (long long)a.n_ct * KS * a.N * a.tiles_y * a.tiles_x;
  if (nb <= 0 || nb > 0x7FFFFFFFLL) return hipErrorInvalidValue;
  if (a.x3) {   // fp32 operands as three bf16 terms (split3_bf16): x3 = 3, the split-once 128-row tiles
                // (conv3x3_x3s_kernel); x3 = 2, pre-split weights on 64-row 4-wave tiles, the activations split
                // per tap (the short-K 3x3 layers; the batch-1 ConvTranspose, KT = 1) -- two weight slots: a
                // third fits beside the exactly sized halo, 78 KB, but measured 2 % slower; x3 = 1, both
                // operands split on the fly (the ConvTranspose at larger batches)
    if constexpr (sizeof(T) == 4 && WPX == 4 && TCW == 8 && KT == 3 &&
                  (EPI == EPI_STORE || EPI == EPI_POOL || EPI == EPI_PARTIAL)) {
      if (a.x3 == 3) {   // 128-row tiles, the activations split once per chunk (conv3x3_x3s_kernel)
        hipLaunchKernelGGL((conv3x3_x3s_kernel<EPI>), dim3((unsigned)nb), dim3(512), 0, s, a);
        return hipGetLastError();
      }
    }
    if constexpr (sizeof(T) == 4 && WPX == 4 && TCW == 4) {   // (KT = 1: the ConvTranspose, one tap)
      if (a.x3 == 2) {
        hipLaunchKernelGGL((conv3x3_halo_kernel<T, WR, WPX, TCW, 2, KT, EPI, 2>), dim3((unsigned)nb),
                           dim3(64 * WR * WPX), 0, s, a);
        return hipGetLastError();
      }
    }
    if constexpr (sizeof(T) == 4 && KT == 1) {
      if (a.x3 == 1) {
        hipLaunchKernelGGL((conv3x3_halo_kernel<T, WR, WPX, TCW, NS, KT, EPI, 1>), dim3((unsigned)nb),
                           dim3(64 * WR * WPX), 0, s, a);
        return hipGetLastError();
      }
    }
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL((conv3x3_halo_kernel<T, WR, WPX, TCW, NS, KT, EPI>), dim3((unsigned)nb), dim3(64 * WR * WPX), 0,
                     s, a);
  return hipGetLastError();
}

// the three-term plan's 64-channel layers (x3 = 4): 64 rows x 16x32 pixels per block
template <int EPI>
static hipError_t launch_x3w(const IgemmArgs& a, hipStream_t s) {
  if (a.x3 != 4 || a.tiles_y != (a.H + 15) / 16 || a.tiles_x != (a.W + 31) / 32) return hipErrorInvalidValue;
  if (a.Cin % 32 || a.Ctot % 64 || a.n_ct != a.Ctot / 64 || (EPI == EPI_HEAD && a.n_ct != 1)) return hipErrorInvalidValue;
  const int KS = EPI == EPI_PARTIAL ? a.ksplit : 1;
  if (KS < 1 || a.Cin % (32 * KS) || (EPI == EPI_PARTIAL && !a.part)) return hipErrorInvalidValue;
  const long long nb = (long long)a.n_ct * KS * a.N * a.tiles_y * a.tiles_x;
  if (nb <= 0 || nb > 0x7FFFFFFFLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv3x3_x3w_kernel<EPI>), dim3((unsigned)nb), dim3(512), 0, s, a);
  return hipGetLastError();
}

template <typename T, int WR, int WPX, int TCW, int NS, int EPI, int TPS, int HS, typename TO, typename TQ, int ABL = 0,
          int TH = 16, int TW = 16>
static hipError_t launch_ring(const IgemmArgs& a, hipStream_t s) {
  using G = RingGeom<T, WR, WPX, TCW, NS, TPS, HS, TH, TW>;
  if constexpr (HS != 0) {
    if (a.Cin != 2 * G::BKE || a.c0 < 1 || a.c0 > 3 || !a.x0 || !a.w0p || !a.b0) return hipErrorInvalidValue;
  }
  if (a.tiles_y != (a.H + TH - 1) / TH || a.tiles_x != (a.W + TW - 1) / TW) return hipErrorInvalidValue;
  if ((TH != 16 || TW != 16 || EPI == EPI_UPFUSE) && (long long)a.H * a.W * a.ldi * (long long)sizeof(T) >= (1LL << 31))
    return hipErrorInvalidValue;   // 32-bit halo offsets (ring_body OFF32)
  if (a.Cin % G::BKE || a.Ctot % G::BR || a.n_ct != a.Ctot / G::BR) return hipErrorInvalidValue;
  const int n_mt = a.N * a.tiles_y * a.tiles_x;
  constexpr int per_cu = G::NW >= 8 ? 1 : G::BLOCKS_PER_CU;   // 8-wave blocks: registers allow one per CU
  int n_slots = (kNumCUs * per_cu) / a.n_ct;
  if (n_slots < 1) n_slots = 1;
  if (n_slots > n_mt) n_slots = n_mt;
#ifdef UNET_ABLATION
  if constexpr (ABL != 0) {
    hipLaunchKernelGGL((conv3x3_ring_abl_kernel<T, WR, WPX, TCW, NS, EPI, TPS, HS, TO, TQ, ABL>), dim3(a.n_ct * n_slots),
                       dim3(64 * WR * WPX), 0, s, a);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((conv3x3_ring_kernel<T, WR, WPX, TCW, NS, EPI, TPS, HS, TO, TQ, TH, TW>), dim3(a.n_ct * n_slots),
                     dim3(64 * WR * WPX), 0, s, a);
  return hipGetLastError();
}

template <typename T, int TCW, int NS, int WRW, typename TO>
static hipError_t launch_tring(const IgemmArgs& a, hipStream_t s) {
  constexpr int BR = 16 * TCW * WRW, LDS = NS * (BR * 64 + 256 * 64);
  if (a.tiles_y != (a.H + 15) / 16 || a.tiles_x != (a.W + 15) / 16) return hipErrorInvalidValue;
  if (a.src_br && (WRW != 1 || a.src_br % BR || a.Ctot % a.src_br)) return hipErrorInvalidValue;
  if (a.Cin % (64 / (int)sizeof(T)) || a.Ctot % BR || a.n_ct != a.Ctot / BR) return hipErrorInvalidValue;
  const int n_mt = a.N * a.tiles_y * a.tiles_x;
  int n_slots = (kNumCUs * ((160 * 1024) / LDS)) / a.n_ct;
  if (n_slots < 1) n_slots = 1;
  if (n_slots > n_mt) n_slots = n_mt;
  hipLaunchKernelGGL((convT_ring_kernel<T, TCW, NS, WRW, TO>), dim3(a.n_ct * n_slots), dim3(256 * WRW), 0, s, a);
  return hipGetLastError();
}

// 3x3 layers.  T = operand type, TO / TQ = output / pooled-map types (the LDS-halo family runs
// only with TO = TQ = T: it is the fp32 path).
template <typename T, typename TO, typename TQ, int EPI, int ABL = 0>
static hipError_t launch_3x3(int cfg, const IgemmArgs& a, hipStream_t s) {
  constexpr bool same = std::is_same<T, TO>::value && std::is_same<TO, TQ>::value;
  if constexpr (EPI == EPI_UPFUSE) {   // conv2.3 + up1: the 16-bit 128-row ring only (one row tile)
    if constexpr (sizeof(T) == 2 && ABL == 0) {
      if (cfg == CFG_RING_R128 && a.n_ct == 1 && a.Cout == 128 && a.out2 && a.bias2)
        return launch_ring<T, 1, 4, 8, 3, EPI_UPFUSE, 1, 0, TO, TQ>(a, s);
      if (cfg == CFG_RING8_R128 && a.n_ct == 1 && a.Cout == 128 && a.out2 && a.bias2)
        return launch_ring8<T, 8, 3, EPI_UPFUSE, 3, 0, TO, TQ>(a, s);
    }
    return hipErrorInvalidValue;
  } else if constexpr (EPI == EPI_PARTIAL) {   // split-K slices: the LDS-halo family and the 8-wave 128-row ring
    if constexpr (ABL == 0) {
      switch (cfg) {
        case CFG_HALO_R64_W4: if constexpr (sizeof(T) == 4) return launch_halo<T, 1, 4, 4, 3, EPI, 3>(a, s); break;
        case CFG_HALO_R64_W8: if constexpr (sizeof(T) == 4) return launch_halo<T, 1, 8, 4, 3, EPI, 3>(a, s); break;
        case CFG_HALO_R128: if constexpr (sizeof(T) == 4) return launch_halo<T, 1, 4, 8, 2, EPI, 3>(a, s); break;
        case CFG_HALO_X3W: if constexpr (sizeof(T) == 4) return launch_x3w<EPI>(a, s); break;
        case CFG_RING8_R128:   // 128-row tiles, or 64-row tiles over the 128-row packing (a.src_br)
          if constexpr (sizeof(T) == 2) {
            if (a.src_br == 128) return launch_ring8<T, 4, 3, EPI, 3, 0, T, T>(a, s);
            return launch_ring8<T, 8, 3, EPI, 3, 0, T, T>(a, s);
          }
          break;
        default: break;
      }
    }
    return hipErrorInvalidValue;
  } else {
  if (EPI == EPI_HEAD && cfg_rows(cfg) != 64) return hipErrorInvalidValue;   // the head needs all 64 channels
  if constexpr (ABL != 0) {   // ablation builds: the ring configurations only
    switch (cfg) {
      case CFG_RING_R128:
        if constexpr (EPI != EPI_HEAD) {
          if constexpr (ABL == 8) return launch_ring<T, 1, 4, 8, 4, EPI, 1, 0, TO, TQ, 0>(a, s);   // variant: NS = 4
          else return launch_ring<T, 1, 4, 8, 3, EPI, 1, 0, TO, TQ, ABL>(a, s);
        }
        break;
      case CFG_RING_R64_T3: if constexpr (ABL < 7) return launch_ring<T, 1, 4, 4, 3, EPI, 3, 0, TO, TQ, ABL>(a, s); break;
      case CFG_RING_FUSED_IN:
        if constexpr (sizeof(T) == 2 && EPI == EPI_POOL) return launch_ring<T, 1, 4, 4, 3, EPI, 3, 1, TO, TQ, ABL>(a, s);
        break;
      case CFG_RING8_R128:   // (8: the halo-line ablation, issue_halo)
        if constexpr (ABL >= 1 && ABL <= 9 && EPI != EPI_HEAD && sizeof(T) == 2)
          return launch_ring8<T, 8, 3, EPI, 3, 0, TO, TQ, 0, ABL>(a, s);
        break;
      case CFG_RING8_R64_T9:
        if constexpr (ABL >= 5 && ABL <= 7 && EPI != EPI_HEAD) return launch_ring8<T, 4, 2, EPI, 9, 0, TO, TQ, 0, ABL>(a, s);
        break;
      case CFG_RING8_R64_WS: if constexpr (ABL == 5) return launch_ring8<T, 4, 3, EPI, 3, 1, TO, TQ, 0, 5>(a, s); break;
      default: break;
    }
    return hipErrorInvalidValue;
  }
  switch (cfg) {
    case CFG_HALO_R64_W4: if constexpr (same) return launch_halo<T, 1, 4, 4, 3, EPI, 3>(a, s); break;
    case CFG_HALO_R64_W8: if constexpr (same) return launch_halo<T, 1, 8, 4, 3, EPI, 3>(a, s); break;
    case CFG_HALO_R128: if constexpr (same && EPI != EPI_HEAD) return launch_halo<T, 1, 4, 8, 2, EPI, 3>(a, s); break;
    case CFG_HALO_X3W:
      if constexpr (same && sizeof(T) == 4 && (EPI == EPI_STORE || EPI == EPI_POOL || EPI == EPI_HEAD))
        return launch_x3w<EPI>(a, s);
      break;
    // (pooled 128-row 4-wave tiles spill two VGPRs: not built; unet_capi runs those layers on 64-row tiles)
    case CFG_RING_R128: if constexpr (EPI != EPI_HEAD && EPI != EPI_POOL) return launch_ring<T, 1, 4, 8, 3, EPI, 1, 0, TO, TQ>(a, s); break;
    case CFG_RING_R64_T3: return launch_ring<T, 1, 4, 4, 3, EPI, 3, 0, TO, TQ>(a, s);
#ifdef UNET_ABLATION   // rejected on A/B (profiles/tune_r2j_ring_w12_rejected.txt): ablation builds only
    case CFG_RING_R64_W12:
      if constexpr (sizeof(T) == 2) return launch_ring<T, 1, 4, 4, 4, EPI, 1, 0, TO, TQ, 0, 12, 32>(a, s);
      break;
#endif
    case CFG_RING_FUSED_IN:
      if constexpr (sizeof(T) == 2 && EPI == EPI_POOL) return launch_ring<T, 1, 4, 4, 3, EPI, 3, 1, TO, TQ>(a, s);
      break;
    case CFG_RING8_R128:   // (a.src_br = 128: the batch-1 plan's 64-row tiles over the 128-row packing)
      // 16-bit only: the fp32 128-row 8-wave ring spills (unet_capi runs fp32 on the 64-row ring8 instead)
      if constexpr (EPI != EPI_HEAD && sizeof(T) == 2) {
        if (a.src_br == 128) return launch_ring8<T, 4, 3, EPI, 3, 0, TO, TQ>(a, s);
        return launch_ring8<T, 8, 3, EPI, 3, 0, TO, TQ>(a, s);
      }
      break;
    case CFG_RING8_R64_T9: if constexpr (EPI != EPI_PARTIAL) return launch_ring8<T, 4, 2, EPI, 9, 0, TO, TQ>(a, s); break;
    case CFG_RING8_R64_WS: return launch_ring8<T, 4, 3, EPI, 3, 1, TO, TQ>(a, s);
    case CFG_RING8_FUSED_IN:
      if constexpr (sizeof(T) == 2 && EPI == EPI_POOL) return launch_ring8<T, 4, 3, EPI, 3, 1, TO, TQ, 1>(a, s);
      break;
    default: break;
  }
  return hipErrorInvalidValue;
  }
}

// ConvTranspose2d(k2, s2) layers (1-tap GEMM + pixel-shuffle scatter).  TO = output type.
template <typename T, typename TO, int EPI = EPI_UPSCATTER>
static hipError_t launch_up(int cfg, const IgemmArgs& a, hipStream_t s) {
  if constexpr (EPI == EPI_PARTIAL) {   // split-K slices of the LDS-halo ConvTranspose (the fp32 path)
    if (cfg == CFG_HALO_R128) return launch_halo<T, 1, 4, 8, 2, EPI_PARTIAL, 1>(a, s);
    if constexpr (sizeof(T) == 4)
      if (cfg == CFG_HALO_R64_W4 && a.x3 == 2) return launch_halo<T, 1, 4, 4, 2, EPI_PARTIAL, 1>(a, s);
    return hipErrorInvalidValue;
  }
  switch (cfg) {
    case CFG_HALO_R128:
      if constexpr (std::is_same<T, TO>::value) return launch_halo<T, 1, 4, 8, 2, EPI_UPSCATTER, 1>(a, s);
      break;
    case CFG_HALO_R64_W4:   // the three-term plan's pre-split 64-row tiles only
      if constexpr (std::is_same<T, TO>::value && sizeof(T) == 4)
        if (a.x3 == 2) return launch_halo<T, 1, 4, 4, 2, EPI_UPSCATTER, 1>(a, s);
      break;
    case CFG_TRING_R128: return launch_tring<T, 8, 3, 1, TO>(a, s);
    case CFG_TRING_R256: return launch_tring<T, 8, 4, 2, TO>(a, s);
    default: break;
  }
  return hipErrorInvalidValue;
}

template <typename T, typename TO, typename TQ>
static hipError_t launch_typed(int cfg, int taps, int epi, const IgemmArgs& a, hipStream_t s) {
#ifdef UNET_ABLATION
  if (taps == 9 && cfg >= CFG_COUNT) {   // cfg = base + 16 * ablation (csrc/unet_kernels.hip ring_body)
    const int base = cfg % 16;
#define UNET_ABL_CASE(k)                                                             \
  case k:                                                                            \
    switch (epi) {                                                                   \
      case EPI_STORE: return launch_3x3<T, TO, TQ, EPI_STORE, k>(base, a, s);       \
      case EPI_POOL: return launch_3x3<T, TO, TQ, EPI_POOL, k>(base, a, s);         \
      case EPI_HEAD: return launch_3x3<T, TO, TQ, EPI_HEAD, k>(base, a, s);         \
      default: return hipErrorInvalidValue;                                          \
    }
    switch (cfg / 16) {
      UNET_ABL_CASE(1) UNET_ABL_CASE(2) UNET_ABL_CASE(3) UNET_ABL_CASE(4) UNET_ABL_CASE(5) UNET_ABL_CASE(6)
      UNET_ABL_CASE(7) UNET_ABL_CASE(8) UNET_ABL_CASE(9)
      default: return hipErrorInvalidValue;
    }
#undef UNET_ABL_CASE
  }
#endif
  if (taps == 9) {
    switch (epi) {
      case EPI_STORE: return launch_3x3<T, TO, TQ, EPI_STORE>(cfg, a, s);
      case EPI_POOL: return launch_3x3<T, TO, TQ, EPI_POOL>(cfg, a, s);
      case EPI_HEAD: return launch_3x3<T, TO, TQ, EPI_HEAD>(cfg, a, s);
      case EPI_UPFUSE: return launch_3x3<T, TO, TQ, EPI_UPFUSE>(cfg, a, s);
      case EPI_PARTIAL:
        if constexpr (std::is_same<T, TO>::value && std::is_same<T, TQ>::value) return launch_3x3<T, T, T, EPI_PARTIAL>(cfg, a, s);
        return hipErrorInvalidValue;
      default: return hipErrorInvalidValue;
    }
  }
  if (taps == 1 && epi == EPI_UPSCATTER) return launch_up<T, TO>(cfg, a, s);
  if (taps == 1 && epi == EPI_PARTIAL) {
    if constexpr (std::is_same<T, float>::value && std::is_same<T, TO>::value) return launch_up<T, T, EPI_PARTIAL>(cfg, a, s);
    return hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

hipError_t launch_igemm(DType t, DType to, DType tq, int cfg, int taps, int epi, const IgemmArgs& a, hipStream_t s) {
  if (t == to && to == tq) {
    switch (t) {
      case DType::F32: return launch_typed<float, float, float>(cfg, taps, epi, a, s);
      case DType::BF16: return launch_typed<__bf16, __bf16, __bf16>(cfg, taps, epi, a, s);
      case DType::F16: return launch_typed<_Float16, _Float16, _Float16>(cfg, taps, epi, a, s);
    }
    return hipErrorInvalidValue;
  }
  // the mixed bf16 / fp16 plan's two seams (unet_capi.cpp): an fp16 pooled layer whose pooled map
  // feeds a bf16 layer, and a bf16 ConvTranspose whose output feeds an fp16 layer
  if (t == DType::F16 && to == DType::F16 && tq == DType::BF16 && taps == 9 && epi == EPI_POOL)
    return launch_typed<_Float16, _Float16, __bf16>(cfg, taps, epi, a, s);
  if (t == DType::BF16 && to == DType::F16 && tq == DType::F16 && taps == 1 && epi == EPI_UPSCATTER)
    return launch_up<__bf16, _Float16>(cfg, a, s);
  return hipErrorInvalidValue;
}

template <typename T>
static hipError_t first_t(const FirstConvArgs& a, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    if (a.wp) {
      IgemmArgs e{};
      e.out = a.out;
      e.N = a.N; e.H = a.H; e.W = a.W;
      e.ldo = 64; e.out_off = 0;
      e.tiles_x = (a.W + 15) / 16;
      e.tiles_y = (a.H + 15) / 16;
      const dim3 grid((unsigned)((long long)a.N * e.tiles_x * e.tiles_y));
      if (a.C == 1) hipLaunchKernelGGL((first_conv_mfma_kernel<T, 1>), grid, dim3(256), 0, s, a, e);
      else if (a.C == 3) hipLaunchKernelGGL((first_conv_mfma_kernel<T, 3>), grid, dim3(256), 0, s, a, e);
      else return hipErrorInvalidValue;
      return hipGetLastError();
    }
  }
  const long long total = (long long)a.N * a.H * a.W;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (a.C == 1) hipLaunchKernelGGL((first_conv_kernel<T, 1>), grid, dim3(256), 0, s, a);
  else if (a.C == 3) hipLaunchKernelGGL((first_conv_kernel<T, 3>), grid, dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_first_conv(DType t, const FirstConvArgs& a, hipStream_t s) {
  switch (t) {
    case DType::F32: return first_t<float>(a, s);
    case DType::BF16: return first_t<__bf16>(a, s);
    case DType::F16: return first_t<_Float16>(a, s);
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------
// split-K reduction (small batches: layers whose tile grid under-fills the 256 CUs run as KS
// independent K slices writing fp32 partials, EPI_PARTIAL)
// ---------------------------------------------------------------------------------
// One thread = 8 rows of one output pixel (EPI_STORE, EPI_UPSCATTER: input pixel) or of one 2x2
// pooling window (EPI_POOL).  The slices are added to the bias in slice order (deterministic), then
// the epilogue the layer's own kernel applies (conv_epilogue): NaN-propagating ReLU and TO stores;
// for EPI_POOL also the window max of the ReLU outputs as TQ; for EPI_UPSCATTER the pixel-shuffle
// store without ReLU.  Reads 32 contiguous bytes per thread and slice (coalesced across threads).
template <typename T>
__device__ __forceinline__ void store8(T* dst, const float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    f32x4* d = reinterpret_cast<f32x4*>(dst);
    d[0] = f32x4{v[0], v[1], v[2], v[3]};
    d[1] = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (T)v[i];
    *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, o);
  }
}

template <typename TO, typename TQ, int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const IgemmArgs a) {
  const int R8 = a.Ctot / 8;
  const int H = a.H, W = a.W;
  const int Hs = EPI == EPI_POOL ? H / 2 : H, Ws = EPI == EPI_POOL ? W / 2 : W;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n_idx = (long long)a.N * Hs * Ws * R8;
  if (idx >= n_idx) return;
  int r0, x, y, n;
  if (n_idx < (1LL << 31)) {   // 32-bit index math (64-bit divisions cost microseconds per launch here)
    const int id = (int)idx;
    r0 = 8 * (id % R8);
    int p = id / R8;
    x = p % Ws;
    p /= Ws;
    y = p % Hs;
    n = p / Hs;
  } else {
    r0 = 8 * (int)(idx % R8);
    long long pix = idx / R8;
    x = (int)(pix % Ws);
    pix /= Ws;
    y = (int)(pix % Hs);
    n = (int)(pix / Hs);
  }
  const long long slice = (long long)a.N * H * W * a.Ctot;
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.bias + r0), b1 = *reinterpret_cast<const f32x4*>(a.bias + r0 + 4);
  auto reduce = [&](int yy, int xx, float (&v)[8]) {
    const float* src = a.part + ((long long)(n * H + yy) * W + xx) * a.Ctot + r0;
    f32x4 s0 = b0, s1 = b1;
    for (int k = 0; k < a.ksplit; ++k) {
      s0 += *reinterpret_cast<const f32x4*>(src + k * slice);
      s1 += *reinterpret_cast<const f32x4*>(src + k * slice + 4);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = s0[e]; v[4 + e] = s1[e]; }
  };
  if constexpr (EPI == EPI_UPSCATTER) {
    const int ab = r0 / a.Cout, o0 = r0 - ab * a.Cout;   // 8 rows of one (a, b) quadrant (Cout % 8 == 0)
    const int Y = 2 * y + (ab >> 1), X = 2 * x + (ab & 1);
    float v[8];
    reduce(y, x, v);
    store8<TO>(reinterpret_cast<TO*>(a.out) + ((long long)(n * 2 * H + Y) * (2 * W) + X) * a.ldo + a.out_off + o0, v);
  } else if constexpr (EPI == EPI_POOL) {
    float m[8];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int yy = 2 * y + (d >> 1), xx = 2 * x + (d & 1);
      float v[8];
      reduce(yy, xx, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = relu_nan(v[e]);
        m[e] = d == 0 ? v[e] : max_nan(m[e], v[e]);
      }
      store8<TO>(reinterpret_cast<TO*>(a.out) + ((long long)(n * H + yy) * W + xx) * a.ldo + a.out_off + r0, v);
    }
    store8<TQ>(reinterpret_cast<TQ*>(a.out2) + ((long long)(n * Hs + y) * Ws + x) * a.ldo2 + r0, m);
  } else {
    float v[8];
    reduce(y, x, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = relu_nan(v[e]);
    store8<TO>(reinterpret_cast<TO*>(a.out) + ((long long)(n * H + y) * W + x) * a.ldo + a.out_off + r0, v);
  }
}

template <typename TO, typename TQ, int EPI>
static hipError_t splitk_reduce_t(const IgemmArgs& a, hipStream_t s) {
  if (a.Ctot % 8 || (EPI == EPI_UPSCATTER && a.Cout % 8) || a.ksplit < 1 || !a.part) return hipErrorInvalidValue;
  const long long threads = (long long)a.N * (EPI == EPI_POOL ? (a.H / 2) * (a.W / 2) : a.H * a.W) * (a.Ctot / 8);
  if (threads <= 0 || (threads + 255) / 256 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL((splitk_reduce_kernel<TO, TQ, EPI>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_splitk_reduce(DType to, DType tq, int epi, const IgemmArgs& a, hipStream_t s) {
  if (epi == EPI_POOL) {
    if (to == DType::F32 && tq == DType::F32) return splitk_reduce_t<float, float, EPI_POOL>(a, s);
    if (to == DType::BF16 && tq == DType::BF16) return splitk_reduce_t<__bf16, __bf16, EPI_POOL>(a, s);
    if (to == DType::F16 && tq == DType::F16) return splitk_reduce_t<_Float16, _Float16, EPI_POOL>(a, s);
    if (to == DType::F16 && tq == DType::BF16) return splitk_reduce_t<_Float16, __bf16, EPI_POOL>(a, s);
    return hipErrorInvalidValue;
  }
  if (epi != EPI_STORE && epi != EPI_UPSCATTER) return hipErrorInvalidValue;
  switch (to) {
    case DType::F32:
      return epi == EPI_STORE ? splitk_reduce_t<float, float, EPI_STORE>(a, s) : splitk_reduce_t<float, float, EPI_UPSCATTER>(a, s);
    case DType::BF16:
      return epi == EPI_STORE ? splitk_reduce_t<__bf16, __bf16, EPI_STORE>(a, s)
                              : splitk_reduce_t<__bf16, __bf16, EPI_UPSCATTER>(a, s);
    case DType::F16:
      return epi == EPI_STORE ? splitk_reduce_t<_Float16, _Float16, EPI_STORE>(a, s)
                              : splitk_reduce_t<_Float16, _Float16, EPI_UPSCATTER>(a, s);
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------
// per-(image, field) bounding box of a mask: inference.py:84-90 (np.where(mask) ->
// xs.min(), xs.max(), ys.min(), ys.max()) on the GPU, 4 ints instead of H*W host bytes.
// Blocks (n, c) x strips: each 256-thread block walks strips of 1024 16-pixel column words (bit j of
// word w = pixel 16*w + j: a little-endian 16-bit word of a bit-packed mask, or 16 bytes of a uint8
// mask reduced to their nonzero bits), four loads in flight per thread; with W / 16 dividing 256 a
// thread always sees the same column word and ORs it in a register (one LDS atomic per thread
// instead of one per set pixel), and keeps the first / last row with a set bit.  The strips' boxes
// meet in the handle's sync entry of (n, c) (device-scope atomics); the block that counts last
// writes the box and resets the entry to its idle state {INT_MAX, INT_MAX, -1, -1, 0}, so the next
// launch (or graph replay) needs no clearing pass.  One block per mask was 18.6 us per batch-1
// call: a single CU cannot keep enough loads in flight to pull a 256 KB plane faster.
// Empty mask -> (-1,-1,-1,-1).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ unsigned nz_bits4(unsigned d) {   // bit j = byte j of d nonzero
  d |= d >> 4;
  d |= d >> 2;
  d |= d >> 1;
  return (d & 1u) | ((d >> 7) & 2u) | ((d >> 14) & 4u) | ((d >> 21) & 8u);
}

constexpr int kBoxThreads = 256, kBoxLoads = 4, kBoxChunk = kBoxThreads * kBoxLoads, kBoxMaxStrips = 64;

template <int KIND, bool VEC>
__global__ __launch_bounds__(kBoxThreads) void mask_boxes_kernel(const uint8_t* __restrict__ masks, int H, int W,
                                                        int* __restrict__ boxes, int* __restrict__ sync) {
  __shared__ unsigned col_or[kMaxBoxW / 16];
  __shared__ int ymin_s, ymax_s, xmin_s, xmax_s;
  const int tid = threadIdx.x;
  const int words = W / 16;
  for (int i = tid; i < words; i += kBoxThreads) col_or[i] = 0u;
  if (tid == 0) { ymin_s = 0x7FFFFFFF; ymax_s = -1; xmin_s = 0x7FFFFFFF; xmax_s = -1; }
  __syncthreads();
  const int total = H * words;
  const int chunks = (total + kBoxChunk - 1) / kBoxChunk;
  const size_t plane = KIND == MASK_BITS ? (size_t)H * (W / 8) : (size_t)H * W;
  const uint8_t* base = masks + (size_t)blockIdx.x * plane;
  auto word_at = [&](int i) -> unsigned {   // 16-pixel column word i of the plane
    if constexpr (KIND == MASK_BITS) {
      return reinterpret_cast<const uint16_t*>(base)[i];
    } else if constexpr (VEC) {
      const uint4 v = reinterpret_cast<const uint4*>(base)[i];
      return nz_bits4(v.x) | (nz_bits4(v.y) << 4) | (nz_bits4(v.z) << 8) | (nz_bits4(v.w) << 12);
    } else {
      unsigned b = 0;
      for (int j = 0; j < 16; ++j) b |= (base[16 * i + j] ? 1u : 0u) << j;
      return b;
    }
  };
  int ymin = 0x7FFFFFFF, ymax = -1, cw = -1;
  unsigned cacc = 0;
  for (int c = blockIdx.y; c < chunks; c += gridDim.y) {
    const int i0 = c * kBoxChunk + tid;
    unsigned v[kBoxLoads];
#pragma unroll
    for (int k = 0; k < kBoxLoads; ++k) v[k] = i0 + k * kBoxThreads < total ? word_at(i0 + k * kBoxThreads) : 0u;
#pragma unroll
    for (int k = 0; k < kBoxLoads; ++k) {
      const int i = i0 + k * kBoxThreads;
      if (i >= total) break;
      const int y = i / words, w = i - y * words;
      if (w != cw) {
        if (cacc) atomicOr(&col_or[cw], cacc);
        cacc = 0;
        cw = w;
      }
      if (v[k]) {
        ymin = min(ymin, y);
        ymax = max(ymax, y);
        cacc |= v[k];
      }
    }
  }
  if (cacc) atomicOr(&col_or[cw], cacc);
  if (ymax >= 0) { atomicMin(&ymin_s, ymin); atomicMax(&ymax_s, ymax); }
  __syncthreads();
  for (int i = tid; i < words; i += kBoxThreads) {
    const unsigned v = col_or[i];
    if (v) {
      atomicMin(&xmin_s, 16 * i + __builtin_ctz(v));
      atomicMax(&xmax_s, 16 * i + 31 - __builtin_clz(v));
    }
  }
  __syncthreads();
  if (tid == 0) {
    int* e = sync + (size_t)blockIdx.x * kSyncInts;   // x_min, y_min, x_max, y_max, strips counted
    if (ymax_s >= 0) {
      atomicMin(e, xmin_s);
      atomicMin(e + 1, ymin_s);
      atomicMax(e + 2, xmax_s);
      atomicMax(e + 3, ymax_s);
    }
    __threadfence();
    if (atomicAdd(reinterpret_cast<unsigned*>(e + 4), 1u) == gridDim.y - 1) {   // the last strip of (n, c)
      __threadfence();
      const int x0 = atomicExch(e, 0x7FFFFFFF), y0 = atomicExch(e + 1, 0x7FFFFFFF);
      const int x1 = atomicExch(e + 2, -1), y1 = atomicExch(e + 3, -1);
      atomicExch(e + 4, 0);
      int* b = boxes + (size_t)blockIdx.x * 4;
      const bool any = y1 >= 0;
      b[0] = any ? x0 : -1;
      b[1] = any ? y0 : -1;
      b[2] = any ? x1 : -1;
      b[3] = any ? y1 : -1;
    }
  }
}

hipError_t launch_mask_boxes(const uint8_t* masks, int kind, int N, int ncls, int H, int W, int* boxes, int* sync,
                             hipStream_t s) {
  if (W % 16 || W > kMaxBoxW || (kind != MASK_BITS && kind != MASK_U8) || !sync) return hipErrorInvalidValue;
  const long long chunks = ((long long)H * (W / 16) + kBoxChunk - 1) / kBoxChunk;
  const dim3 grid((unsigned)(N * ncls), (unsigned)std::max(1LL, std::min<long long>(chunks, kBoxMaxStrips)));
  const dim3 block(kBoxThreads);
  if (kind == MASK_BITS) {
    hipLaunchKernelGGL((mask_boxes_kernel<MASK_BITS, false>), grid, block, 0, s, masks, H, W, boxes, sync);
  } else if (reinterpret_cast<uintptr_t>(masks) % 16 == 0) {
    hipLaunchKernelGGL((mask_boxes_kernel<MASK_U8, true>), grid, block, 0, s, masks, H, W, boxes, sync);
  } else {
    hipLaunchKernelGGL((mask_boxes_kernel<MASK_U8, false>), grid, block, 0, s, masks, H, W, boxes, sync);
  }
  return hipGetLastError();
}

// Network input element (n, c, y, x) of the caller's tensor: fp32 or uint8 (value / 255, the
// reference's np.float32 division, inference.py:40), NCHW or NHWC (include/unet_mi355x.h).
__device__ __forceinline__ float input_at(const void* x, int layout, int xdt, long long n, int c, long long hw,
                                          int C, long long HW) {
  const long long i = layout == 0 ? (n * C + c) * HW + hw : (n * HW + hw) * C + c;
  return xdt == 0 ? static_cast<const float*>(x)[i] : (float)static_cast<const uint8_t*>(x)[i] / 255.0f;
}

// Network input pre-cast for the fused first conv of the ring kernel (HS = 1): -> element type
// T, 4 channels per pixel [N][H][W][4] (zero-padded), so a 20-pixel window row is 160 contiguous
// bytes (10 LDS-DMA pieces).  The values are the (T) casts the first conv's MFMA operand needs.
template <typename T>
__global__ __launch_bounds__(256) void x_to_px4_kernel(const void* __restrict__ x, int layout, int xdt, int N, int C,
                                                      int H, int W, T* __restrict__ out) {
  const long long HW = (long long)H * W, P = (long long)N * HW;
  typedef T t4 __attribute__((ext_vector_type(4)));
  typedef T t8 __attribute__((ext_vector_type(8)));
  if (layout == 0 && xdt == 0 && C <= 3 && HW % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0) {
    // the common case (fp32 NCHW: bench.py, run_unet's preprocess output): four pixels per thread,
    // one 16-byte load per channel plane and two 16-byte stores (4-byte loads and 8-byte stores ran
    // at 3.9 TB/s); the same casts, so bitwise equal to the generic loop below
    // 32-bit index math: N*H*W <= 2^30 (unet_capi's shape check); with the named loads below, the
    // batch-1 launch 30 -> ~6 us in isolation (tools/calib/precast_bs1.hip)
    const float* xf = static_cast<const float*>(x);
    const int quads = (int)(P / 4), hw32 = (int)HW;
    if (C == 3) {   // the network's input (RGB): three unconditional plane loads per quad
      for (int qd = blockIdx.x * 256 + threadIdx.x; qd < quads; qd += gridDim.x * 256) {
        const int i = 4 * qd, n = i / hw32, hw = i - n * hw32;   // HW % 4 == 0: one image per quad
        const float* px0 = xf + (long long)n * 3 * HW + hw;
        const float4 v0 = *reinterpret_cast<const float4*>(px0);
        const float4 v1 = *reinterpret_cast<const float4*>(px0 + HW);
        const float4 v2 = *reinterpret_cast<const float4*>(px0 + 2 * HW);
        t8 o0 = {(T)v0.x, (T)v1.x, (T)v2.x, (T)0.f, (T)v0.y, (T)v1.y, (T)v2.y, (T)0.f};
        t8 o1 = {(T)v0.z, (T)v1.z, (T)v2.z, (T)0.f, (T)v0.w, (T)v1.w, (T)v2.w, (T)0.f};
        reinterpret_cast<t8*>(out)[2 * qd] = o0;
        reinterpret_cast<t8*>(out)[2 * qd + 1] = o1;
      }
      return;
    }
    for (int qd = blockIdx.x * 256 + threadIdx.x; qd < quads; qd += gridDim.x * 256) {
      const int i = 4 * qd, n = i / hw32, hw = i - n * hw32;   // HW % 4 == 0: one image per quad
      // the planes as named loads (a runtime-C loop into a float4[3] was promoted to LDS and,
      // with the 64-bit division, held the batch-1 launch at 30 us)
      const float* px0 = xf + (long long)n * C * HW + hw;
      const float4 z4 = {0.f, 0.f, 0.f, 0.f};
      float4 v[3];
      v[0] = *reinterpret_cast<const float4*>(px0);
      v[1] = C > 1 ? *reinterpret_cast<const float4*>(px0 + HW) : z4;
      v[2] = C > 2 ? *reinterpret_cast<const float4*>(px0 + 2 * HW) : z4;
      t8 o0, o1;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 vc = v[c < 3 ? c : 0];
        const bool live = c < C;
        o0[c] = (T)(live ? vc.x : 0.f);
        o0[4 + c] = (T)(live ? vc.y : 0.f);
        o1[c] = (T)(live ? vc.z : 0.f);
        o1[4 + c] = (T)(live ? vc.w : 0.f);
      }
      reinterpret_cast<t8*>(out)[2 * qd] = o0;
      reinterpret_cast<t8*>(out)[2 * qd + 1] = o1;
    }
    return;
  }
  const int P32 = (int)P, hw32 = (int)HW;   // <= 2^30 (see above)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < P32; i += gridDim.x * 256) {
    const int n = i / hw32, hw = i - n * hw32;
    t4 v;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (T)(c < C ? input_at(x, layout, xdt, n, c, hw, C, HW) : 0.f);
    reinterpret_cast<t4*>(out)[i] = v;
  }
}

// Grid-stride element kernels: at most 4096 blocks, and no more than one block per 1024 pixels (a
// batch-1 512^2 input is 256 blocks: the fixed 4096-block grid took 33 us there, mostly dispatching
// blocks with nothing to do).
static dim3 elem_grid(long long pixels) {
  const long long b = (pixels + 1023) / 1024;
  return dim3((unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b)));
}

hipError_t launch_x_to_px4(DType t, const void* x, int layout, int xdt, int N, int C, int H, int W, void* out,
                           hipStream_t s) {
  const dim3 grid = elem_grid((long long)N * H * W), block(256);
  if (t == DType::BF16)
    hipLaunchKernelGGL(x_to_px4_kernel<__bf16>, grid, block, 0, s, x, layout, xdt, N, C, H, W, static_cast<__bf16*>(out));
  else if (t == DType::F16)
    hipLaunchKernelGGL(x_to_px4_kernel<_Float16>, grid, block, 0, s, x, layout, xdt, N, C, H, W,
                       static_cast<_Float16*>(out));
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void x_to_nchw_f32_kernel(const void* __restrict__ x, int layout, int xdt, int N,
                                                           int C, int H, int W, float* __restrict__ out) {
  const long long HW = (long long)H * W, total = (long long)N * C * HW;
  const int hw32 = (int)HW;   // the pixel index stays 32-bit; (n, c) from the plane index
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int nc = (int)(i / hw32), hw = (int)(i - (long long)nc * hw32);
    out[i] = input_at(x, layout, xdt, nc / C, nc % C, hw, C, HW);
  }
}

hipError_t launch_x_to_nchw_f32(const void* x, int layout, int xdt, int N, int C, int H, int W, float* out,
                                hipStream_t s) {
  hipLaunchKernelGGL(x_to_nchw_f32_kernel, elem_grid((long long)N * H * W), dim3(256), 0, s, x, layout, xdt, N, C, H, W, out);
  return hipGetLastError();
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ src, int N, int H, int W, int C, int ld, int choff,
                                    float* __restrict__ dst) {
  const long long total = (long long)N * C * H * W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    long long r = i / W;
    const int y = (int)(r % H);
    r /= H;
    const int c = (int)(r % C);
    const int n = (int)(r / C);
    dst[i] = (float)src[((long long)(n * H + y) * W + x) * ld + choff + c];
  }
}

hipError_t launch_nhwc_to_nchw_f32(DType t, const void* src, int N, int H, int W, int C, int ld,
                                   int choff, float* dst, hipStream_t s) {
  const dim3 grid(2048), block(256);
  switch (t) {
    case DType::F32:
      hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, grid, block, 0, s, (const float*)src, N, H, W, C, ld, choff, dst);
      break;
    case DType::BF16:
      hipLaunchKernelGGL(nhwc_to_nchw_kernel<__bf16>, grid, block, 0, s, (const __bf16*)src, N, H, W, C, ld, choff, dst);
      break;
    case DType::F16:
      hipLaunchKernelGGL(nhwc_to_nchw_kernel<_Float16>, grid, block, 0, s, (const _Float16*)src, N, H, W, C, ld, choff, dst);
      break;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// layout transposes of the stand-alone DoubleConv (unet_block_*): fp32 NCHW <-> NHWC T through a
// 32-channel x 64-pixel LDS tile, both sides coalesced (pixels along the NCHW rows, 16-byte channel
// runs along the NHWC pixels).  HBM-bound.
// ---------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x, int C, int HW, T* __restrict__ out) {
  __shared__ float tile[32][65];
  const int n = blockIdx.z, c0 = blockIdx.y * 32, p0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  const float* src = x + (long long)n * C * HW;
#pragma unroll
  for (int k = 0; k < 8; ++k) {   // rows c0 + 4k + tid / 64, pixel p0 + tid % 64
    const int c = c0 + 4 * k + (tid >> 6), p = p0 + (tid & 63);
    tile[4 * k + (tid >> 6)][tid & 63] = (c < C && p < HW) ? src[(long long)c * HW + p] : 0.f;
  }
  __syncthreads();
  const int p = p0 + (tid >> 2), cg = (tid & 3) * 8;   // pixel, 8-channel group
  if (p >= HW || c0 + cg >= C) return;
  typedef T t8 __attribute__((ext_vector_type(8)));
  t8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (T)tile[cg + j][tid >> 2];
  T* dst = out + ((long long)n * HW + p) * C + c0 + cg;
  if (c0 + cg + 8 <= C) {
    *reinterpret_cast<t8*>(dst) = v;
  } else {
    for (int j = 0; c0 + cg + j < C; ++j) dst[j] = v[j];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void nhwc_to_nchw_tiled_kernel(const T* __restrict__ src, int C, int HW, float* __restrict__ y) {
  __shared__ float tile[32][65];
  const int n = blockIdx.z, c0 = blockIdx.y * 32, p0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  {
    const int p = p0 + (tid >> 2), cg = (tid & 3) * 8;
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 v = {};
    if (p < HW && c0 + cg + 8 <= C) {
      v = *reinterpret_cast<const t8*>(src + ((long long)n * HW + p) * C + c0 + cg);
    } else if (p < HW) {
      for (int j = 0; c0 + cg + j < C && j < 8; ++j) v[j] = src[((long long)n * HW + p) * C + c0 + cg + j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[cg + j][tid >> 2] = (float)v[j];
  }
  __syncthreads();
  float* dst = y + (long long)n * C * HW;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + 4 * k + (tid >> 6), p = p0 + (tid & 63);
    if (c < C && p < HW) dst[(long long)c * HW + p] = tile[4 * k + (tid >> 6)][tid & 63];
  }
}

hipError_t launch_nchw_to_nhwc(DType t, const float* x, int N, int C, int H, int W, void* out, hipStream_t s) {
  const int HW = H * W;
  const dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((C + 31) / 32), (unsigned)N), block(256);
  switch (t) {
    case DType::F32: hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, grid, block, 0, s, x, C, HW, (float*)out); break;
    case DType::BF16: hipLaunchKernelGGL(nchw_to_nhwc_kernel<__bf16>, grid, block, 0, s, x, C, HW, (__bf16*)out); break;
    case DType::F16: hipLaunchKernelGGL(nchw_to_nhwc_kernel<_Float16>, grid, block, 0, s, x, C, HW, (_Float16*)out); break;
  }
  return hipGetLastError();
}

hipError_t launch_nhwc_to_nchw(DType t, const void* src, int N, int C, int H, int W, float* y, hipStream_t s) {
  const int HW = H * W;
  const dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((C + 31) / 32), (unsigned)N), block(256);
  switch (t) {
    case DType::F32: hipLaunchKernelGGL(nhwc_to_nchw_tiled_kernel<float>, grid, block, 0, s, (const float*)src, C, HW, y); break;
    case DType::BF16: hipLaunchKernelGGL(nhwc_to_nchw_tiled_kernel<__bf16>, grid, block, 0, s, (const __bf16*)src, C, HW, y); break;
    case DType::F16: hipLaunchKernelGGL(nhwc_to_nchw_tiled_kernel<_Float16>, grid, block, 0, s, (const _Float16*)src, C, HW, y); break;
  }
  return hipGetLastError();
}

}  // namespace unet
