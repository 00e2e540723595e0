// Stream-count probe (round 3): does reading K separate arrays (one 16-byte
// load per thread from each, the AMG row kernels' access shape) run slower
// than reading the same bytes from ONE array laid out wave-block by
// wave-block (AoSoA: [wave][k][64 lanes x 16 B])?  Each variant moves the
// same bytes: K loads of 16 B per thread in, one 16-B store out.
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/bin/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

struct Arrs {
  const float4* p[16];
};

template <int K>
__global__ void __launch_bounds__(256) k_soa(Arrs a, float4* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = a.p[k][i];
  float4 s = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    s.x += v[k].x;
    s.y += v[k].y;
    s.z += v[k].z;
    s.w += v[k].w;
  }
  out[i] = s;
}

// the same K loads issued in batches of B, each batch waited for before the
// next issues (s_waitcnt vmcnt(0)): at most B loads in flight per wave
template <int K, int B>
__global__ void __launch_bounds__(256) k_batched(Arrs a, float4* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    v[k] = a.p[k][i];
    if ((k + 1) % B == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float4 s = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    s.x += v[k].x;
    s.y += v[k].y;
    s.z += v[k].z;
    s.w += v[k].w;
  }
  out[i] = s;
}

template <int K>
__global__ void __launch_bounds__(256) k_aosoa(const float4* __restrict__ a, float4* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const size_t w = i / 64, l = i % 64;
  const float4* base = a + w * (64 * K) + l;
  float4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = base[64 * k];
  float4 s = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    s.x += v[k].x;
    s.y += v[k].y;
    s.z += v[k].z;
    s.w += v[k].w;
  }
  out[i] = s;
}

// the same kernels with nontemporal loads (global_load ... nt; round 4)
__device__ __forceinline__ float4 ldnt(const float4* p) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
template <int K>
__global__ void __launch_bounds__(256) k_soa_nt(Arrs a, float4* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ldnt(a.p[k] + i);
  float4 s = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    s.x += v[k].x;
    s.y += v[k].y;
    s.z += v[k].z;
    s.w += v[k].w;
  }
  out[i] = s;
}
template <int K>
__global__ void __launch_bounds__(256) k_aosoa_nt(const float4* __restrict__ a, float4* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const size_t w = i / 64, l = i % 64;
  const float4* base = a + w * (64 * K) + l;
  float4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ldnt(base + 64 * k);
  float4 s = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    s.x += v[k].x;
    s.y += v[k].y;
    s.z += v[k].z;
    s.w += v[k].w;
  }
  out[i] = s;
}

template <int K>
void run(size_t n, int reps) {
  std::vector<float4*> bufs(K);
  for (int k = 0; k < K; ++k) {
    CK(hipMalloc(&bufs[k], n * sizeof(float4)));
    CK(hipMemset(bufs[k], 0, n * sizeof(float4)));
  }
  float4 *one, *out;
  // 512 MB written between launches: every launch starts with the Infinity
  // Cache holding none of its data (as in the solver, where other kernels'
  // data sit between two launches of one kernel); COLD=0 replays back to back
  static char* flush = nullptr;
  const bool cold = !getenv("COLD") || getenv("COLD")[0] != '0';
  if (cold && !flush) CK(hipMalloc(&flush, (size_t)512 << 20));
  CK(hipMalloc(&one, (size_t)K * n * sizeof(float4)));
  CK(hipMemset(one, 0, (size_t)K * n * sizeof(float4)));
  CK(hipMalloc(&out, n * sizeof(float4)));
  Arrs a{};
  for (int k = 0; k < K; ++k) a.p[k] = bufs[k];
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned nb = (unsigned)((n + 255) / 256);
  const double bytes = (double)(K + 1) * n * 16.0;
  for (int variant = 0; variant < 7; ++variant) {
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      if (cold) CK(hipMemsetAsync(flush, r & 0xff, (size_t)512 << 20, 0));
      CK(hipEventRecord(e0));
      if (variant == 0)
        hipLaunchKernelGGL(k_soa<K>, dim3(nb), dim3(256), 0, 0, a, out, n);
      else if (variant == 1)
        hipLaunchKernelGGL(k_aosoa<K>, dim3(nb), dim3(256), 0, 0, one, out, n);
      else if (variant == 2)
        hipLaunchKernelGGL((k_batched<K, 4>), dim3(nb), dim3(256), 0, 0, a, out, n);
      else if (variant == 3)
        hipLaunchKernelGGL((k_batched<K, 2>), dim3(nb), dim3(256), 0, 0, a, out, n);
      else if (variant == 4)
        hipLaunchKernelGGL((k_batched<K, 1>), dim3(nb), dim3(256), 0, 0, a, out, n);
      else if (variant == 5)
        hipLaunchKernelGGL(k_soa_nt<K>, dim3(nb), dim3(256), 0, 0, a, out, n);
      else
        hipLaunchKernelGGL(k_aosoa_nt<K>, dim3(nb), dim3(256), 0, 0, one, out, n);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    static const char* names[] = {"soa", "aosoa", "bat4", "bat2", "bat1", "soa-nt", "aosoa-nt"};
    std::printf("K=%2d %-6s n=%zu  %.1f us  %.2f TB/s\n", K, names[variant], n, best * 1e3,
                bytes / (best * 1e-3) / 1e12);
  }
  for (auto b : bufs) CK(hipFree(b));
  CK(hipFree(one));
  CK(hipFree(out));
}

int main(int argc, char** argv) {
  // 4-row groups of a 10 M-row level; argv[1] = multiplier (working sets past the 256 MB Infinity Cache)
  const size_t n = (size_t)10 * 1000 * 1000 / 4 * (argc > 1 ? std::atoi(argv[1]) : 1);
  run<1>(n, 12);
  run<2>(n, 12);
  run<4>(n, 12);
  run<6>(n, 12);
  run<8>(n, 12);
  run<11>(n, 12);
  run<16>(n, 12);
  return 0;
}
