// Stream-shape probe (round 4, after stream_probe.hip): at a fixed stream
// count K and cold Infinity Cache, does the rate depend on
//   R  the consecutive 16-byte pieces one thread reads per stream (R = 1: the
//      AMG row kernels' 4-row quad, 1 KiB per stream per wave; R = 3: the CGS
//      kernels' 4-cell unit, 3 KiB per stream per wave), and
//   B  the loads a wave keeps in flight (B = 0: all K*R issued at once; B = 1:
//      each waited for before the next issues, as k_cgs_dots<SER = true>)?
// Every variant reads K arrays of n float4 with nontemporal loads and writes
// one array of n float4 (the sum).  512 MB are written before every timed
// launch so that none of its data sits in the Infinity Cache.
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe2.hip -o tools/bin/stream_probe2
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

__device__ __forceinline__ float4 ldnt(const float4* p) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void acc(float4& s, const float4& v) {
  s.x += v.x;
  s.y += v.y;
  s.z += v.z;
  s.w += v.w;
}

// thread t reads pieces [R t, R t + R) of every stream (per wave: R KiB
// contiguous per stream), writes the same pieces of out
template <int K, int R, int B>
__global__ void __launch_bounds__(256) k_run(Arrs a, float4* out, size_t n) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  // lanes interleaved so that each wave-instruction reads 1 KiB contiguous:
  // piece q of thread (wave w, lane l) = w*64*R + q*64 + l
  const size_t w = t / 64, l = t % 64;
  const size_t base = w * 64 * R + l;
  if (base + 64 * (R - 1) >= n) return;
  float4 s[R];
#pragma unroll
  for (int q = 0; q < R; ++q) s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 v[K][R];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int q = 0; q < R; ++q) {
      v[k][q] = ldnt(a.p[k] + base + 64 * q);
      if (B > 0 && ((k * R + q + 1) % B) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int q = 0; q < R; ++q) acc(s[q], v[k][q]);
#pragma unroll
  for (int q = 0; q < R; ++q) out[base + 64 * q] = s[q];
}

template <int K, int R, int B>
float time_one(const Arrs& a, float4* out, size_t n, char* flush, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t threads = n / R;
  const unsigned nb = (unsigned)((threads + 255) / 256);
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipMemsetAsync(flush, r & 0xff, (size_t)512 << 20, 0));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_run<K, R, B>), dim3(nb), dim3(256), 0, 0, a, out, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0 && ms < best) best = ms;
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return best;
}

template <int K>
void run(size_t n, char* flush, int reps) {
  std::vector<float4*> bufs(K);
  for (int k = 0; k < K; ++k) {
    CK(hipMalloc(&bufs[k], n * sizeof(float4)));
    CK(hipMemset(bufs[k], 0, n * sizeof(float4)));
  }
  float4* out;
  CK(hipMalloc(&out, n * sizeof(float4)));
  Arrs a{};
  for (int k = 0; k < K; ++k) a.p[k] = bufs[k];
  const double bytes = (double)(K + 1) * n * 16.0;
  auto line = [&](const char* name, float ms) {
    std::printf("K=%2d %-10s n=%zu  %.1f us  %.2f TB/s\n", K, name, n, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
  };
  line("R1-all", time_one<K, 1, 0>(a, out, n, flush, reps));
  line("R1-ser", time_one<K, 1, 1>(a, out, n, flush, reps));
  line("R2-all", time_one<K, 2, 0>(a, out, n, flush, reps));
  line("R3-all", time_one<K, 3, 0>(a, out, n, flush, reps));
  line("R3-ser", time_one<K, 3, 1>(a, out, n, flush, reps));
  line("R3-b3", time_one<K, 3, 3>(a, out, n, flush, reps));
  for (auto b : bufs) CK(hipFree(b));
  CK(hipFree(out));
}

int main(int argc, char** argv) {
  // 4-row groups of a 10 M-row level, a multiple of 64 * 2 * 3 pieces
  const size_t n = (size_t)10 * 1000 * 1000 / 4 / 384 * 384 * (argc > 1 ? std::atoi(argv[1]) : 1);
  char* flush;
  CK(hipMalloc(&flush, (size_t)512 << 20));
  run<1>(n, flush, 12);
  run<4>(n, flush, 12);
  run<8>(n, flush, 12);
  run<11>(n, flush, 12);
  run<16>(n, flush, 12);
  return 0;
}
