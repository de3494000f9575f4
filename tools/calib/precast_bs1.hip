// Batch-1 input pre-cast (x_to_px4_kernel's common path: fp32 NCHW, 3 channels -> 16-bit [H][W][4])
// at 512^2: why does it take ~30 us in the batch-1 forward (profiles/rocprof_r4v_bs1_mixed_*)?  Times,
// with HIP events over 200 back-to-back launches, (0) the product's shape: 4 pixels per thread, 64-bit
// index math, 256 blocks; (1) the same with 32-bit index math; (2) 4 pixels per thread, 1024 blocks of
// 64 threads; (3) 1 pixel per thread, 1024 blocks -- each after the same 2 MB "previous kernel" writing
// a different buffer, as in the forward.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

__global__ void k0(const float* xf, long long HW, long long quads, int C, h8* out) {   // product shape
  for (long long qd = (long long)blockIdx.x * blockDim.x + threadIdx.x; qd < quads; qd += (long long)gridDim.x * blockDim.x) {
    const long long i = 4 * qd, n = i / HW, hw = i - n * HW;
    float4 v[3] = {};
    for (int c = 0; c < C; ++c) v[c] = *reinterpret_cast<const float4*>(xf + (n * C + c) * HW + hw);
    h8 o0, o1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 vc = v[c < 3 ? c : 0];
      const bool live = c < C;
      o0[c] = (_Float16)(live ? vc.x : 0.f); o0[4 + c] = (_Float16)(live ? vc.y : 0.f);
      o1[c] = (_Float16)(live ? vc.z : 0.f); o1[4 + c] = (_Float16)(live ? vc.w : 0.f);
    }
    out[2 * qd] = o0;
    out[2 * qd + 1] = o1;
  }
}
__global__ void k1(const float* xf, int HW, int quads, h8* out) {   // 32-bit index math, C = 3
  for (int qd = blockIdx.x * blockDim.x + threadIdx.x; qd < quads; qd += gridDim.x * blockDim.x) {
    const int i = 4 * qd, n = i / HW, hw = i - n * HW;
    float4 v0 = *reinterpret_cast<const float4*>(xf + (n * 3 + 0) * HW + hw);
    float4 v1 = *reinterpret_cast<const float4*>(xf + (n * 3 + 1) * HW + hw);
    float4 v2 = *reinterpret_cast<const float4*>(xf + (n * 3 + 2) * HW + hw);
    h8 o0 = {(_Float16)v0.x, (_Float16)v1.x, (_Float16)v2.x, 0, (_Float16)v0.y, (_Float16)v1.y, (_Float16)v2.y, 0};
    h8 o1 = {(_Float16)v0.z, (_Float16)v1.z, (_Float16)v2.z, 0, (_Float16)v0.w, (_Float16)v1.w, (_Float16)v2.w, 0};
    out[2 * qd] = o0;
    out[2 * qd + 1] = o1;
  }
}
__global__ void k3(const float* xf, int HW, int P, h4* out) {   // one pixel per thread
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const int n = i / HW, hw = i - n * HW;
  out[i] = h4{(_Float16)xf[(n * 3) * HW + hw], (_Float16)xf[(n * 3 + 1) * HW + hw], (_Float16)xf[(n * 3 + 2) * HW + hw], 0};
}
__global__ void prev(float* buf, int n) {   // a "previous kernel": 2 MB of writes
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] = (float)i;
}

int main() {
  const int H = 512, W = 512, C = 3, N = 1, HW = H * W, P = N * HW, quads = P / 4;
  float *x, *junk; h8* out; h4* out4;
  hipMalloc(&x, (size_t)N * C * HW * 4); hipMalloc(&junk, 1 << 21); hipMalloc(&out, (size_t)P * 8); hipMalloc(&out4, (size_t)P * 8);
  hipMemset(x, 0, (size_t)N * C * HW * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const char* names[4] = {"product: 4 px/thread, 64-bit math, 256 x 256", "32-bit math, 256 x 256",
                          "32-bit math, 1024 x 64", "1 px/thread, 1024 x 256"};
  for (int mode = 0; mode < 4; ++mode) {
    float best = 1e9f, sum = 0.f;
    for (int it = 0; it < 220; ++it) {
      hipLaunchKernelGGL(prev, dim3(256), dim3(256), 0, 0, junk, (1 << 21) / 4);
      hipEventRecord(a, 0);
      if (mode == 0) hipLaunchKernelGGL(k0, dim3(256), dim3(256), 0, 0, x, (long long)HW, (long long)quads, C, out);
      if (mode == 1) hipLaunchKernelGGL(k1, dim3(256), dim3(256), 0, 0, x, HW, quads, out);
      if (mode == 2) hipLaunchKernelGGL(k1, dim3(1024), dim3(64), 0, 0, x, HW, quads, out);
      if (mode == 3) hipLaunchKernelGGL(k3, dim3(1024), dim3(256), 0, 0, x, HW, P, out4);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (it >= 20) { best = ms < best ? ms : best; sum += ms; }
    }
    printf("%-48s best %7.2f us  mean %7.2f us\n", names[mode], best * 1e3, sum / 200 * 1e3);
  }
  return 0;
}
