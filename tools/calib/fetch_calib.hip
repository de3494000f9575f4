// FETCH_SIZE calibration for the ring kernels' halo access shape.
//
// The rings LDS-DMA a halo chunk as 64-byte pieces (32 16-bit channels of one pixel, 4 lanes x 16 B),
// one piece per pixel at the pixel stride Cin * 2 B -- half (Cin = 64) or a quarter (Cin = 128) of a
// 128-byte line per piece, the rest of the line fetched by the next chunks' pieces a few us later.
// The guide calibrates FETCH_SIZE only for wide coalesced streams (it reports half the bytes).  This
// program reads KNOWN byte counts with global_load_lds_dwordx4 in four shapes, one kernel each, over
// 1 GiB regions (4x the Infinity Cache, so the lines come from DRAM):
//   mode 0: contiguous, 1 KB per wave instruction                    (the guide's calibrated case)
//   mode 1: 64-B pieces, pixel stride 128 B, both halves of each line by consecutive instructions
//   mode 2: 64-B pieces, pixel stride 128 B, only half 0 of every line (the other half never read)
//   mode 3: 64-B pieces, pixel stride 256 B, all four quarters by consecutive instructions
// and prints the requested and the unique-line bytes of each launch; rocprofv3 --pmc FETCH_SIZE (and
// TCC_EA0_RDREQ_*) over this program gives the counter side.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

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

// Each wave instruction covers 16 pixels (4 lanes x 16 B = one 64-B piece each) or, in mode 0,
// 1 KB contiguous.  A block walks its own slice; vmcnt is drained every 8 instructions.
template <int MODE>
__global__ __launch_bounds__(256) void calib_kernel(const char* __restrict__ base, long long region_bytes) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long nwaves = (long long)gridDim.x * 4;
  const long long gw = (long long)blockIdx.x * 4 + wave;
  char* dst = lds + wave * 1024;
  int issued = 0;
  if (MODE == 0) {
    const long long per = region_bytes / 1024 / nwaves;   // 1 KB blocks per wave
    for (long long k = 0; k < per; ++k) {
      glds16(base + (gw * per + k) * 1024 + lane * 16, dst);
      if (++issued % 8 == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    const int stride = MODE == 3 ? 256 : 128;
    const int pieces = MODE == 1 ? 2 : (MODE == 2 ? 1 : 4);
    const long long npix = region_bytes / stride;
    const long long groups = npix / 16 / nwaves;          // 16-pixel groups per wave
    const int p = lane >> 2, q = lane & 3;
    for (long long k = 0; k < groups; ++k) {
      const char* pix = base + ((gw * groups + k) * 16 + p) * stride + q * 16;
      for (int c = 0; c < pieces; ++c) {
        glds16(pix + c * 64, dst);
        if (++issued % 8 == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
  const long long R = 1LL << 30;
  char* buf = nullptr;
  if (hipMalloc(&buf, 4 * R) != hipSuccess) { std::printf("hipMalloc failed\n"); return 1; }
  (void)hipMemset(buf, 1, 4 * R);
  (void)hipDeviceSynchronize();
  const int blocks = 2048;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[4] = {"contiguous 1KB/instr", "64B pieces, stride 128, both halves", "64B pieces, stride 128, half 0 only",
                          "64B pieces, stride 256, all quarters"};
  for (int m = 0; m < 4; ++m) {
    hipEventRecord(e0);
    switch (m) {
      case 0: hipLaunchKernelGGL(calib_kernel<0>, dim3(blocks), dim3(256), 0, 0, buf + 0 * R, R); break;
      case 1: hipLaunchKernelGGL(calib_kernel<1>, dim3(blocks), dim3(256), 0, 0, buf + 1 * R, R); break;
      case 2: hipLaunchKernelGGL(calib_kernel<2>, dim3(blocks), dim3(256), 0, 0, buf + 2 * R, R); break;
      case 3: hipLaunchKernelGGL(calib_kernel<3>, dim3(blocks), dim3(256), 0, 0, buf + 3 * R, R); break;
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double requested = m == 2 ? R / 2.0 : (double)R;   // bytes the instructions ask for
    std::printf("mode %d (%s): requested %.3f GB, unique 128-B lines %.3f GB, %.3f ms, %.0f GB/s requested\n", m,
                names[m], requested / 1e9, (double)R / 1e9, ms, requested / ms / 1e6);
  }
  hipFree(buf);
  return 0;
}
