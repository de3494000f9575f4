// GPU preprocessing: the resize + convert("RGB") + /255 + CHW of
// inference.py:30-44 and :62-64, bit-exact with Pillow's Image.resize default filter.
//
// Pillow resizes 8-bit images with a separable two-pass fixed-point resampler (horizontal pass
// into an 8-bit intermediate over the rows the vertical pass needs, then the vertical pass):
// per output sample  clip8((1 << 21) + sum_k in[k] * coeff[k]) with 22 fractional bits, the
// coefficients being the normalised bicubic (a = -0.5) weights over a support widened by the
// downscale factor (antialiasing), rounded half away from zero.  The coefficient tables are
// computed on the host in double precision with the same operation order (unet_capi.cpp,
// resample_coeffs) and the kernels here do the integer arithmetic, so every output byte equals
// Pillow's.  The oracle (oracle/pil_resample.py) restates the same algorithm in numpy and is
// itself checked against Pillow (tests/test_preprocess_cpu.py).
#include "unet_internal.h"

#include <algorithm>
#include <type_traits>

namespace unet {

namespace {
constexpr int kResamplePrec = 22;   // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8_fixed(int v) {
  const int s = v >> kResamplePrec;   // arithmetic shift, as Pillow's clip8 lookup
  return s < 0 ? 0 : (s > 255 ? 255 : s);
}
}  // namespace

// The tap loops below take the taps eight at a time with all of a group's coefficient and pixel
// loads issued before the first multiply (the loads are independent; a loop of one tap per
// iteration waits out a memory latency per tap, 18 us per pass on a 600x400 photo), and the
// channel count is a template argument so the accumulators stay in registers.  Integer sums are
// exact, so the grouping does not change a byte.
constexpr int kTapGroup = 8;

// Source pixels: C channels of S bytes per pixel -- RGB (3, 3), L (1, 1), or Pillow's own in-memory
// RGB layout RGBX (3, 4: the fourth byte is padding, never read), which the drop-in uploads as is.
// Horizontal pass: tmp[r][xx][c] = clip8(sum_x src[y0 + r][xmin(xx) + x][c] * kh[xx][x]) (C bytes per
// pixel).  One thread per (row, output column), all channels.
template <int C, int S>
__global__ __launch_bounds__(256) void resample_h_kernel(const uint8_t* __restrict__ src, int src_stride, int y0,
                                                        int rows, const int* __restrict__ bounds,
                                                        const int* __restrict__ kk, int ksize, int ow,
                                                        uint8_t* __restrict__ tmp) {
  const int xx = blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y;
  if (xx >= ow || r >= rows) return;
  const int xmin = bounds[2 * xx], n = bounds[2 * xx + 1];
  const int* k = kk + (size_t)xx * ksize;
  const uint8_t* row = src + (size_t)(y0 + r) * src_stride + (size_t)xmin * S;
  int acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 1 << (kResamplePrec - 1);
  for (int x0 = 0; x0 < n; x0 += kTapGroup) {
    int w[kTapGroup], px[kTapGroup][C];
#pragma unroll
    for (int j = 0; j < kTapGroup; ++j) {
      const int t = min(x0 + j, n - 1);   // past the last tap: a valid address, weight 0
      const int wt = k[t];
      w[j] = x0 + j < n ? wt : 0;
#pragma unroll
      for (int c = 0; c < C; ++c) px[j][c] = (int)row[t * S + c];
    }
#pragma unroll
    for (int j = 0; j < kTapGroup; ++j)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += px[j][c] * w[j];
  }
  uint8_t* dst = tmp + ((size_t)r * ow + xx) * C;
#pragma unroll
  for (int c = 0; c < C; ++c) dst[c] = (uint8_t)clip8_fixed(acc[c]);
}

// Vertical pass fused with the final conversion: out[c][yy][xx] = clip8(...) / 255 (fp32, the
// reference's np.float32 division), gray (C = 1) replicated to 3 planes as convert("RGB").
// TO = _Float16 / __bf16 (the photo graph on the 16-bit plans): the same fp32 values cast to TO as
// the fused first conv's pre-cast input [oh][ow][4] (x_to_px4_kernel's format and casts), so the
// forward skips that launch and the fp32 planes are never written.
template <int C, int S, typename TO = float>
__global__ __launch_bounds__(256) void resample_v_kernel(const uint8_t* __restrict__ src, int src_stride,
                                                        const int* __restrict__ bounds, const int* __restrict__ kk,
                                                        int ksize, int oh, int ow, TO* __restrict__ out) {
  const int xx = blockIdx.x * 256 + threadIdx.x;
  const int yy = blockIdx.y;
  if (xx >= ow || yy >= oh) return;
  const int ymin = bounds[2 * yy], n = bounds[2 * yy + 1];
  const int* k = kk + (size_t)yy * ksize;
  const uint8_t* col = src + (size_t)ymin * src_stride + (size_t)xx * S;
  int acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 1 << (kResamplePrec - 1);
  for (int y0 = 0; y0 < n; y0 += kTapGroup) {
    int w[kTapGroup], px[kTapGroup][C];
#pragma unroll
    for (int j = 0; j < kTapGroup; ++j) {
      const int t = min(y0 + j, n - 1);
      const int wt = k[t];
      w[j] = y0 + j < n ? wt : 0;
#pragma unroll
      for (int c = 0; c < C; ++c) px[j][c] = (int)col[(size_t)t * src_stride + c];
    }
#pragma unroll
    for (int j = 0; j < kTapGroup; ++j)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += px[j][c] * w[j];
  }
  const size_t plane = (size_t)oh * ow, o = (size_t)yy * ow + xx;
  if constexpr (sizeof(TO) == 2) {
    typedef TO t4 __attribute__((ext_vector_type(4)));
    t4 v;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (TO)((float)clip8_fixed(acc[C == 3 ? c : 0]) / 255.0f);
    v[3] = (TO)0.f;
    reinterpret_cast<t4*>(out)[o] = v;
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c * plane + o] = (float)clip8_fixed(acc[C == 3 ? c : 0]) / 255.0f;
  }
}

// No vertical resampling (ih == oh): convert the (horizontally resampled or original) rows.
__global__ __launch_bounds__(256) void to_planar_f32_kernel(const uint8_t* __restrict__ src, int src_stride, int C,
                                                           int S, int oh, int ow, float* __restrict__ out) {
  const int xx = blockIdx.x * 256 + threadIdx.x;
  const int yy = blockIdx.y;
  if (xx >= ow || yy >= oh) return;
  const uint8_t* p = src + (size_t)yy * src_stride + (size_t)xx * S;
  const size_t plane = (size_t)oh * ow, o = (size_t)yy * ow + xx;
  for (int c = 0; c < 3; ++c) out[c * plane + o] = (float)p[C == 3 ? c : 0] / 255.0f;
}

// channels: 1 (L), 3 (RGB) or 4 (RGBX: 3 channels, 4 bytes per pixel).  px4 != F32 (only with a
// vertical pass): out is the pre-cast [oh][ow][4] input of that element type instead of fp32 planes.
hipError_t launch_resample(const ResamplePlan& p, const uint8_t* img, int channels, uint8_t* tmp, void* out,
                           hipStream_t s, DType px4) {
  if ((channels != 1 && channels != 3 && channels != 4) || p.oh <= 0 || p.ow <= 0) return hipErrorInvalidValue;
  if (px4 != DType::F32 && (!p.need_v || (px4 != DType::F16 && px4 != DType::BF16))) return hipErrorInvalidValue;
  const int C = channels == 1 ? 1 : 3, S = channels;
  const uint8_t* src = img;
  int stride = p.iw * S, sstep = S;
  if (p.need_h) {
    const dim3 grid((unsigned)((p.ow + 255) / 256), (unsigned)p.h_rows);
    if (S == 4)
      hipLaunchKernelGGL((resample_h_kernel<3, 4>), grid, dim3(256), 0, s, img, stride, p.h_y0, p.h_rows, p.h_bounds,
                         p.h_kk, p.h_ksize, p.ow, tmp);
    else if (S == 3)
      hipLaunchKernelGGL((resample_h_kernel<3, 3>), grid, dim3(256), 0, s, img, stride, p.h_y0, p.h_rows, p.h_bounds,
                         p.h_kk, p.h_ksize, p.ow, tmp);
    else
      hipLaunchKernelGGL((resample_h_kernel<1, 1>), grid, dim3(256), 0, s, img, stride, p.h_y0, p.h_rows, p.h_bounds,
                         p.h_kk, p.h_ksize, p.ow, tmp);
    src = tmp;   // C bytes per pixel
    stride = p.ow * C;
    sstep = C;
  }
  const dim3 grid((unsigned)((p.ow + 255) / 256), (unsigned)p.oh);
  auto vpass = [&](auto* o) {
    using TO = std::remove_pointer_t<decltype(o)>;
    if (sstep == 4)
      hipLaunchKernelGGL((resample_v_kernel<3, 4, TO>), grid, dim3(256), 0, s, src, stride, p.v_bounds, p.v_kk,
                         p.v_ksize, p.oh, p.ow, o);
    else if (sstep == 3)
      hipLaunchKernelGGL((resample_v_kernel<3, 3, TO>), grid, dim3(256), 0, s, src, stride, p.v_bounds, p.v_kk,
                         p.v_ksize, p.oh, p.ow, o);
    else
      hipLaunchKernelGGL((resample_v_kernel<1, 1, TO>), grid, dim3(256), 0, s, src, stride, p.v_bounds, p.v_kk,
                         p.v_ksize, p.oh, p.ow, o);
  };
  if (px4 == DType::F16)
    vpass(static_cast<_Float16*>(out));
  else if (px4 == DType::BF16)
    vpass(static_cast<__bf16*>(out));
  else if (p.need_v)
    vpass(static_cast<float*>(out));
  else
    hipLaunchKernelGGL(to_planar_f32_kernel, grid, dim3(256), 0, s, src, stride, C, sstep, p.oh, p.ow,
                       static_cast<float*>(out));
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Crop statistics (inference.py:92-127) on the device photo: per (image, field) mask box, the
// crop rectangle in photo pixels and the sum of the crop's uint8 values, so the host applies the
// reference's rejection rules without reading pixels.  The rectangle arithmetic is the
// reference's, in float64 as Python evaluates it: scale = ow / IMG_SIZE (true division),
// x1 = int(mx1 * scale) (truncation), pad = int((x2 - x1) * 0.15), clamp to [0, ow] / [0, oh].
// "arr.mean() < 3" over the crop's uint8 values (numpy's float64 pairwise sum of integers is
// exact below 2^53) is "sum < 3 * count" -- the host tests that.  Grid (blocks, boxes): the crop's
// rows are walked 8 at a time as 4-byte photo words (each row's byte range masked at its ends,
// RGBX's X byte masked out), 8 loads in flight per thread; each block's 64-bit sum meets the
// others' in the box's sync entry and the last block writes sums[box] (in a graph: no clearing
// node), or, without sync entries, is added into sums[box] cleared by the launcher.  One-byte loads
// over 8-row blocks were 35.6 us per batch-1 call, latency-bound.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void crop_rect(const int* b, int ih, int iw, int bh, int bw, double pad, int& x1, int& y1,
                                          int& x2, int& y2) {
  const double sx = (double)iw / (double)bw, sy = (double)ih / (double)bh;
  x1 = (int)((double)b[0] * sx);
  x2 = (int)((double)b[2] * sx);
  y1 = (int)((double)b[1] * sy);
  y2 = (int)((double)b[3] * sy);
  const int px = (int)((double)(x2 - x1) * pad), py = (int)((double)(y2 - y1) * pad);
  x1 = max(0, x1 - px);
  y1 = max(0, y1 - py);
  x2 = min(iw, x2 + px);
  y2 = min(ih, y2 + py);
}

__device__ __forceinline__ unsigned byte_sum(unsigned v) {
  return (v & 0xFFu) + ((v >> 8) & 0xFFu) + ((v >> 16) & 0xFFu) + (v >> 24);
}

constexpr int kCropThreads = 256, kCropRows = 8, kCropMaxBlocks = 128;
// A box's sync entry is one 64-bit word: blocks counted in the top 16 bits, the sum in the low 48
// (a crop sums at most 2^30 pixels x 3 bytes x 255 < 2^40), so one returning atomic add both
// merges a block's sum and tells the last block the total.
constexpr int kCropSumBits = 48;

__global__ __launch_bounds__(kCropThreads) void crop_stats_kernel(const uint8_t* __restrict__ img, int ih, int iw,
                                                                 int S, const int* __restrict__ boxes, int bh,
                                                                 int bw, double pad, int* __restrict__ rects,
                                                                 unsigned long long* __restrict__ sums,
                                                                 int* __restrict__ sync) {
  __shared__ unsigned long long part[kCropThreads / 64];
  const int i = blockIdx.y, tid = threadIdx.x;
  const int* b = boxes + 4 * i;
  const bool any = b[2] >= 0;   // else: empty mask
  int x1 = 0, y1 = 0, x2 = 0, y2 = 0;
  if (any) crop_rect(b, ih, iw, bh, bw, pad, x1, y1, x2, y2);
  if (blockIdx.x == 0 && tid < 4) {
    const int r[4] = {x1, y1, x2, y2};
    rects[4 * i + tid] = any ? r[tid] : -1;
  }
  const bool work = any && x2 > x1 && y2 > y1;
  const int groups = work ? (y2 - y1 + kCropRows - 1) / kCropRows : 0;   // groups of kCropRows crop rows
  const int nblk = min(groups, (int)gridDim.x);                          // blocks that take part
  if ((int)blockIdx.x >= nblk) {
    if (blockIdx.x == 0 && tid == 0) sums[i] = 0ull;   // nothing to sum (no block takes part)
    return;
  }
  // Each crop row is the byte range [lo, lo + len) of the photo, walked as 4-byte words from the
  // one containing lo (relative to the word below img: img itself need not be aligned), the ends
  // masked; thread j takes words j, j + 256, ... of kCropRows rows at once (8 loads in flight).
  const unsigned off = (unsigned)(reinterpret_cast<uintptr_t>(img) & 3u);
  const unsigned* words = reinterpret_cast<const unsigned*>(img - off);
  const unsigned xmask = S == 4 ? ~(0xFFu << (8u * ((3u + off) & 3u))) : 0xFFFFFFFFu;   // RGBX: not X
  const long long len = (long long)(x2 - x1) * S;
  const int wpr = (int)((len + 3) / 4) + 1;   // words a row can touch
  unsigned long long acc = 0;
  for (int g = blockIdx.x; g < groups; g += nblk) {
    for (int j = tid; j < wpr; j += kCropThreads) {
      unsigned v[kCropRows], m[kCropRows];
#pragma unroll
      for (int k = 0; k < kCropRows; ++k) {
        const int y = y1 + g * kCropRows + k;
        v[k] = 0u;
        m[k] = 0u;
        if (y < y2) {
          const long long lo = (long long)off + ((long long)y * iw + x1) * S;
          const long long w = (lo >> 2) + j;
          const long long blo = max(lo - 4 * w, 0LL), bhi = min(lo + len - 4 * w, 4LL);
          if (bhi > blo) {
            m[k] = (bhi >= 4 ? 0xFFFFFFFFu : (1u << (8 * bhi)) - 1u) & ~((1u << (8 * blo)) - 1u) & xmask;
            v[k] = words[w];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < kCropRows; ++k) acc += byte_sum(v[k] & m[k]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((tid & 63) == 0) part[tid >> 6] = acc;
  __syncthreads();
  if (tid != 0) return;
  unsigned long long t = 0;
  for (int k = 0; k < kCropThreads / 64; ++k) t += part[k];
  if (!sync) {   // standalone launch: sums were cleared by the launcher's memset
    if (t) atomicAdd(sums + i, t);
    return;
  }
  unsigned long long* e = reinterpret_cast<unsigned long long*>(sync + (size_t)i * kSyncInts);
  const unsigned long long one = 1ull << kCropSumBits;
  const unsigned long long old = atomicAdd(e, one + t);
  if ((old >> kCropSumBits) == (unsigned long long)nblk - 1) {   // the last block of box i
    sums[i] = (old + t) & (one - 1);
    atomicExch(e, 0ull);   // idle for the next launch
  }
}

hipError_t launch_crop_stats(const uint8_t* img, int ih, int iw, int C, const int* boxes, int n_boxes, int bh, int bw,
                             double pad, int* rects, unsigned long long* sums, int* sync, hipStream_t s) {
  if ((C != 1 && C != 3 && C != 4) || ih <= 0 || iw <= 0 || bh <= 0 || bw <= 0 || n_boxes <= 0) return hipErrorInvalidValue;
  if (!sync) {
    hipError_t e = hipMemsetAsync(sums, 0, (size_t)n_boxes * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
  }
  // a block per kCropRows rows of the largest crop (the whole photo), at most kCropMaxBlocks per box
  const unsigned gx = (unsigned)std::min(kCropMaxBlocks, (ih + kCropRows - 1) / kCropRows);
  hipLaunchKernelGGL(crop_stats_kernel, dim3(gx, (unsigned)n_boxes), dim3(kCropThreads), 0, s, img, ih, iw, C, boxes,
                     bh, bw, pad, rects, sums, sync);
  return hipGetLastError();
}

}  // namespace unet
