// FETCH_SIZE / WRITE_SIZE calibration on gfx950 (MI355X_MICROARCH.md: "Other
// access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern").  Each kernel streams a 1 GiB buffer (4x the Infinity
// Cache, so every line comes from HBM once) with one access width per lane,
// coalesced across the wavefront like the level-0 smoother's arrays:
//   k_read<4>   u8x4 / dword per lane   (row lengths: uchar4 per 4 rows)
//   k_read<8>   dwordx2 per lane        (16-bit column deltas: short4 per 4 rows)
//   k_read<16>  dwordx4 per lane        (values, b, x, diagonal: float4 per 4 rows)
//   k_write<16> dwordx4 stores          (x_out)
// rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) over `fetch_calib` gives the
// counter value per dispatch against the known 1 GiB: the factor to apply
// per width.  Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/bin/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

template <int W>
__global__ void __launch_bounds__(256) k_read(const unsigned char* __restrict__ p, size_t bytes, float* out) {
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.0f;
  for (size_t o = t * W; o + W <= bytes; o += lanes * W) {
    if constexpr (W == 4) {
      acc += (float)*reinterpret_cast<const unsigned int*>(p + o);
    } else if constexpr (W == 8) {
      const uint2 v = *reinterpret_cast<const uint2*>(p + o);
      acc += (float)(v.x ^ v.y);
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(p + o);
      acc += (float)(v.x ^ v.y ^ v.z ^ v.w);
    }
  }
  if (acc == 12345.678f) out[t & 1023] = acc;  // keeps the loads; never true for the zero buffer
}

__global__ void __launch_bounds__(256) k_write16(unsigned char* __restrict__ p, size_t bytes) {
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t o = t * 16; o + 16 <= bytes; o += lanes * 16)
    *reinterpret_cast<uint4*>(p + o) = make_uint4((unsigned)o, 1u, 2u, 3u);
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  unsigned char* buf;
  float* out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 1024 * sizeof(float)));
  CHECK(hipMemset(buf, 0, bytes));
  const dim3 grid(256 * 32), block(256);
  for (int rep = 0; rep < 2; ++rep) {  // second round: the one to read (first warms the TLB)
    hipLaunchKernelGGL(k_read<4>, grid, block, 0, 0, buf, bytes, out);
    hipLaunchKernelGGL(k_read<8>, grid, block, 0, 0, buf, bytes, out);
    hipLaunchKernelGGL(k_read<16>, grid, block, 0, 0, buf, bytes, out);
    hipLaunchKernelGGL(k_write16, grid, block, 0, 0, buf, bytes);
  }
  CHECK(hipDeviceSynchronize());
  std::printf("fetch_calib: 4 kernels x 2 rounds over %zu bytes each\n", bytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
