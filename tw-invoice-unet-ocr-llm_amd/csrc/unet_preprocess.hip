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

namespace unet {

namespace {
constexpr int kResamplePrec = 22;   // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8_fixed(int v) {
  const int s = v >> kResamplePrec;   // arithmetic shift, as Pillow's clip8 lookup
  return s < 0 ? 0 : (s > 255 ? 255 : s);
}
}  // namespace

// Horizontal pass: tmp[r][xx][c] = clip8(sum_x src[y0 + r][xmin(xx) + x][c] * kh[xx][x]).
// One thread per (row, output column), all channels.
__global__ __launch_bounds__(256) void resample_h_kernel(const uint8_t* __restrict__ src, int src_stride, int y0,
                                                        int rows, int C, const int* __restrict__ bounds,
                                                        const int* __restrict__ kk, int ksize, int ow,
                                                        uint8_t* __restrict__ tmp) {
  const int xx = blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y;
  if (xx >= ow || r >= rows) return;
  const int xmin = bounds[2 * xx], n = bounds[2 * xx + 1];
  const int* k = kk + (size_t)xx * ksize;
  const uint8_t* row = src + (size_t)(y0 + r) * src_stride + (size_t)xmin * C;
  int acc[3] = {1 << (kResamplePrec - 1), 1 << (kResamplePrec - 1), 1 << (kResamplePrec - 1)};
  for (int x = 0; x < n; ++x) {
    const int w = k[x];
    for (int c = 0; c < C; ++c) acc[c] += (int)row[x * C + c] * w;
  }
  uint8_t* dst = tmp + ((size_t)r * ow + xx) * C;
  for (int c = 0; c < C; ++c) dst[c] = (uint8_t)clip8_fixed(acc[c]);
}

// Vertical pass fused with the final conversion: out[c][yy][xx] = clip8(...) / 255 (fp32, the
// reference's np.float32 division), gray (C = 1) replicated to 3 planes as convert("RGB").
__global__ __launch_bounds__(256) void resample_v_kernel(const uint8_t* __restrict__ src, int src_stride, int C,
                                                        const int* __restrict__ bounds, const int* __restrict__ kk,
                                                        int ksize, int oh, int ow, float* __restrict__ out) {
  const int xx = blockIdx.x * 256 + threadIdx.x;
  const int yy = blockIdx.y;
  if (xx >= ow || yy >= oh) return;
  const int ymin = bounds[2 * yy], n = bounds[2 * yy + 1];
  const int* k = kk + (size_t)yy * ksize;
  const uint8_t* col = src + (size_t)ymin * src_stride + (size_t)xx * C;
  int acc[3] = {1 << (kResamplePrec - 1), 1 << (kResamplePrec - 1), 1 << (kResamplePrec - 1)};
  for (int y = 0; y < n; ++y) {
    const int w = k[y];
    for (int c = 0; c < C; ++c) acc[c] += (int)col[(size_t)y * src_stride + c] * w;
  }
  const size_t plane = (size_t)oh * ow, o = (size_t)yy * ow + xx;
  for (int c = 0; c < 3; ++c) out[c * plane + o] = (float)clip8_fixed(acc[C == 3 ? c : 0]) / 255.0f;
}

// No vertical resampling (ih == oh): convert the (horizontally resampled or original) rows.
__global__ __launch_bounds__(256) void to_planar_f32_kernel(const uint8_t* __restrict__ src, int src_stride, int C,
                                                           int oh, int ow, float* __restrict__ out) {
  const int xx = blockIdx.x * 256 + threadIdx.x;
  const int yy = blockIdx.y;
  if (xx >= ow || yy >= oh) return;
  const uint8_t* p = src + (size_t)yy * src_stride + (size_t)xx * C;
  const size_t plane = (size_t)oh * ow, o = (size_t)yy * ow + xx;
  for (int c = 0; c < 3; ++c) out[c * plane + o] = (float)p[C == 3 ? c : 0] / 255.0f;
}

hipError_t launch_resample(const ResamplePlan& p, const uint8_t* img, int C, uint8_t* tmp, float* out,
                           hipStream_t s) {
  if ((C != 1 && C != 3) || p.oh <= 0 || p.ow <= 0) return hipErrorInvalidValue;
  const uint8_t* src = img;
  int stride = p.iw * C;
  if (p.need_h) {
    const dim3 grid((unsigned)((p.ow + 255) / 256), (unsigned)p.h_rows);
    hipLaunchKernelGGL(resample_h_kernel, grid, dim3(256), 0, s, img, p.iw * C, p.h_y0, p.h_rows, C, p.h_bounds,
                       p.h_kk, p.h_ksize, p.ow, tmp);
    src = tmp;
    stride = p.ow * C;
  }
  const dim3 grid((unsigned)((p.ow + 255) / 256), (unsigned)p.oh);
  if (p.need_v)
    hipLaunchKernelGGL(resample_v_kernel, grid, dim3(256), 0, s, src, stride, C, p.v_bounds, p.v_kk, p.v_ksize, p.oh,
                       p.ow, out);
  else
    hipLaunchKernelGGL(to_planar_f32_kernel, grid, dim3(256), 0, s, src, stride, C, p.oh, p.ow, out);
  return hipGetLastError();
}

}  // namespace unet
